#!/usr/bin/env python3
"""Per-iteration traversal work of one traced sample set (MFX_DIAG_ITER=1 with MFX_F_COUNT_STATS):
node / leaf / primitive visits per closest and per shadow ray of each bounce, from the cumulative
counters the library prints after every iteration. Usage: iter_stats.py [SCENE] [SPP]"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys
sys.path.insert(0, ROOT)
from mafrixraytracing_amd.abi import MFX_F_COUNT_STATS
from mafrixraytracing_amd.native import NativeContext, DEFAULT_SEED
from mafrixraytracing_amd.scene_io import load_scene_file
ctx = NativeContext(load_scene_file(SCENE), seed=DEFAULT_SEED, flags=MFX_F_COUNT_STATS)
ctx.trace_accumulate(SPP, 0); ctx.sync(); ctx.ray_counts()
'''


def main():
    scene = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "scenes", "spot.xml")
    spp = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    env = dict(os.environ, MFX_DIAG_ITER="1", MFX_CAMERA_PACKETS="0")
    code = CHILD.replace("ROOT", repr(ROOT)).replace("SCENE", repr(scene)).replace("SPP", str(spp))
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=300)
    prev = [0.0] * 9
    N = r"([\d.]+)"
    pat = re.compile(rf"iter (\d+): cumulative primary {N} ext {N} shadow {N}; extend {N} ms shadow {N} ms;.*"
                     rf"cumulative traversal closest {N} {N} {N} shadow {N} {N} {N}")
    for line in p.stderr.splitlines():
        m = pat.search(line)
        if not m:
            continue
        it = int(m.group(1))
        v = [float(m.group(k)) for k in (2, 3, 4, 7, 8, 9, 10, 11, 12)]
        d = [a - b for a, b in zip(v, prev)]
        prev = v
        closest = d[0] + d[1]
        print(f"iter {it}: closest rays {closest:.0f}  nodes/leaves/prims per ray "
              f"{d[3] / max(closest, 1):.2f} {d[4] / max(closest, 1):.2f} {d[5] / max(closest, 1):.2f} | shadow rays {d[2]:.0f}  "
              f"{d[6] / max(d[2], 1):.2f} {d[7] / max(d[2], 1):.2f} {d[8] / max(d[2], 1):.2f} | extend {m.group(5)} ms shadow {m.group(6)} ms")
    if p.returncode:
        print(p.stderr[-2000:])


if __name__ == "__main__":
    main()
