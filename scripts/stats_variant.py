#!/usr/bin/env python3
"""Traversal counters (MFX_F_COUNT_STATS) of libmafrix_rt variants on a scene, per ray:
stats_variant.py SCENE SPP LIB.so [LIB.so ...]. Each variant runs in its own process."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys, json
sys.path.insert(0, ROOT)
import mafrixraytracing_amd.abi as abi
abi._lib = abi.load_library(LIB)
from mafrixraytracing_amd.abi import MFX_F_COUNT_STATS
from mafrixraytracing_amd.native import NativeContext, DEFAULT_SEED
from mafrixraytracing_amd.scene_io import load_scene_file
ctx = NativeContext(load_scene_file(SCENE), seed=DEFAULT_SEED, flags=MFX_F_COUNT_STATS)
ctx.accum_clear(); ctx.trace_accumulate(SPP, 0); ctx.sync()
c = ctx.ray_counts()
print(json.dumps([float(x) for x in c]))
'''

if __name__ == "__main__":
    scene, spp = sys.argv[1], sys.argv[2]
    for lib in sys.argv[3:]:
        code = CHILD.replace("ROOT", repr(ROOT)).replace("LIB", repr(lib)).replace("SCENE", repr(scene)) \
            .replace("SPP", spp)
        c = json.loads(subprocess.run([sys.executable, "-c", code], check=True, capture_output=True,
                                      text=True).stdout.strip().splitlines()[-1])
        rc, rs = c[0] + c[1], c[2]
        print(os.path.basename(lib), f"closest rays {rc:.0f} shadow {rs:.0f} | per closest ray: nodes "
              f"{c[4] / max(rc, 1):.2f} leaves {c[5] / max(rc, 1):.2f} prims {c[6] / max(rc, 1):.2f} | per shadow "
              f"ray: nodes {c[7] / max(rs, 1):.2f} leaves {c[8] / max(rs, 1):.2f} prims {c[9] / max(rs, 1):.2f}",
              flush=True)
        if c[10] > 0:  # MFX_DIAG_OCCLUSION builds: occluded shadow rays
            print(f"  occluded shadow rays {c[10] / max(rs, 1):.3f}: nodes {c[11] / c[10]:.2f} leaves "
                  f"{c[12] / c[10]:.2f} per occluded ray; unoccluded: nodes {(c[7] - c[11]) / max(rs - c[10], 1):.2f} "
                  f"leaves {(c[8] - c[12]) / max(rs - c[10], 1):.2f}; closest rays after their first hit: "
                  f"nodes {c[13] / max(rc, 1):.2f} leaves {c[14] / max(rc, 1):.2f} per ray", flush=True)
