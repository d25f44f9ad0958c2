#!/usr/bin/env python3
"""Per-bounce ray counts, node/leaf/primitive visits per ray and kernel times of the wavefront
(MFX_DIAG_ITER with MFX_F_COUNT_STATS; stderr lines from mfx_api.cpp). Usage: diag_iter_stats.py [SCENE] [SPP]"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
scene = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "scenes", "spot.xml")
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 16
code = f"""
import sys; sys.path.insert(0, {ROOT!r})
from mafrixraytracing_amd.abi import MFX_F_COUNT_STATS, MFX_F_WAVEFRONT
from mafrixraytracing_amd.native import NativeContext, DEFAULT_SEED
from mafrixraytracing_amd.scene_io import load_scene_file
for flags in (MFX_F_WAVEFRONT, MFX_F_COUNT_STATS | MFX_F_WAVEFRONT):
    with NativeContext(load_scene_file({scene!r}), seed=DEFAULT_SEED, flags=flags) as c:
        c.accum_clear(); c.trace_accumulate({spp}, 0); c.sync()
        print("RUN", flags, file=sys.stderr, flush=True)
"""
env = dict(os.environ, MFX_DIAG_ITER="1")
p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=600)
runs, cur = [], []
for line in p.stderr.splitlines():
    if line.startswith("RUN"):
        runs.append(cur)
        cur = []
    elif line.startswith("gen"):
        cur.append([float(x) for x in re.findall(r"[-+]?\d*\.?\d+(?:e[-+]?\d+)?", line.split(":", 1)[1])])
timed, stats = runs[0], runs[1]
prev_t = [0.0] * 20
prev_s = [0.0] * 20
print(f"{os.path.basename(scene)} {spp} spp: per bounce (timing run without counters; visits from the counting run)")
for t, s in zip(timed, stats):
    # fields: primary ext shadow extend_ms shadow_ms stamps(4) outer node  cn cl cp sn sl sp
    ext_rays = (t[0] + t[1]) - (prev_t[0] + prev_t[1])
    shd_rays = t[2] - prev_t[2]
    dcn, dcl, dcp = (s[11] - prev_s[11], s[12] - prev_s[12], s[13] - prev_s[13])
    dsn, dsl, dsp = (s[14] - prev_s[14], s[15] - prev_s[15], s[16] - prev_s[16])
    print(f"  closest {ext_rays / 1e6:8.2f} M in {t[3]:6.3f} ms ({ext_rays / t[3] / 1e6:6.2f} G/s), "
          f"nodes {dcn / max(ext_rays, 1):5.2f} leaves {dcl / max(ext_rays, 1):5.2f} prims {dcp / max(ext_rays, 1):5.2f} | "
          f"shade+shadow {shd_rays / 1e6:8.2f} M in {t[4]:6.3f} ms ({shd_rays / t[4] / 1e6:6.2f} G/s), "
          f"nodes {dsn / max(shd_rays, 1):5.2f} leaves {dsl / max(shd_rays, 1):5.2f} prims {dsp / max(shd_rays, 1):5.2f}")
    prev_t, prev_s = t, s
