#!/usr/bin/env python3
"""Exactness of a library variant (build_variants/*.so) before its A/B counts: wavefront images of
several scenes, ray-queue modes and a render-ahead run against the CPU oracle, bit for bit.
Usage: variant_parity.py LIB [LIB ...]; prints one line per library, exit 1 on any mismatch."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import os, sys
import numpy as np
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "oracle")); sys.path.insert(0, os.path.join(ROOT, "tests"))
import mafrixraytracing_amd.abi as abi
abi._lib = abi.load_library(LIB)
import pyoracle
pyoracle.build()
from conftest import scene, SEED
from mafrixraytracing_amd.native import NativeContext
bad = []
n = 0
for name, w, h, spp in [("spot", 64, 36, 6), ("cube_cornell", 48, 27, 5), ("renault", 40, 24, 4),
                        ("two_spheres_plane", 32, 32, 4), ("spot16_instanced@2l", 40, 24, 3)]:
    a = scene(name, w, h)
    ref = pyoracle.OracleScene(a).sample(spp, SEED, sample_base=0)
    for qf in ("-2", "-1", "0", "1"):
        os.environ["MFX_QUEUE_FROM"] = qf
        with NativeContext(a, seed=SEED) as ctx:
            img = ctx.sample(spp)
        n += 1
        if not np.array_equal(img, ref):
            bad.append((name, qf, float(np.abs(img - ref).max())))
    os.environ.pop("MFX_QUEUE_FROM")
a = scene("spot", 40, 24)
with NativeContext(a, seed=SEED) as c1, NativeContext(a, seed=SEED, render_ahead=4) as c2:
    for k in range(9):
        n += 1
        if not np.array_equal(c1.render_rgba8(1), c2.render_rgba8(1)):
            bad.append(("render_ahead", k))
print("OK" if not bad else "MISMATCH", n, "checks", bad)
'''


def main():
    rc = 0
    for lib in sys.argv[1:]:
        code = CHILD.replace("ROOT", repr(ROOT)).replace("LIB", repr(os.path.abspath(lib)))
        p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=600)
        line = p.stdout.strip().splitlines()[-1] if p.stdout.strip() else p.stderr[-1500:]
        print(os.path.basename(lib), line, flush=True)
        if p.returncode != 0 or not line.startswith("OK"):
            rc = 1
    return rc


if __name__ == "__main__":
    sys.exit(main())
