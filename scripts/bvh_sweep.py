#!/usr/bin/env python3
"""Sweep the traversal-BVH build parameters (MFX_LEAF_MAX, MFX_SAH_CI) on a scene: Mrays/s,
stage times and traversal counters per setting. Usage: bvh_sweep.py SCENE SPP LEAF:CI,..."""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mafrixraytracing_amd.abi import MFX_F_COUNT_STATS
from mafrixraytracing_amd.native import NativeContext, DEFAULT_SEED
from mafrixraytracing_amd.scene_io import load_scene_file

scene, spp = sys.argv[1], int(sys.argv[2])
a = load_scene_file(scene)
for cfg in sys.argv[3].split(","):
    lm, ci = cfg.split(":")
    os.environ["MFX_LEAF_MAX"], os.environ["MFX_SAH_CI"] = lm, ci
    with NativeContext(a, seed=DEFAULT_SEED) as ctx:
        best = None
        for k in range(3):
            ctx.accum_clear(); t = time.perf_counter(); ctx.trace_accumulate(spp, k * spp); ctx.sync()
            dt = time.perf_counter() - t
            best = dt if best is None else min(best, dt)
        c = ctx.ray_counts(); tm = ctx.trace_timing()
    with NativeContext(a, seed=DEFAULT_SEED, flags=MFX_F_COUNT_STATS) as sc:
        sc.trace_accumulate(1, 10 ** 6)
        s = sc.ray_counts()
    rc, rs = s[0] + s[1], s[2]
    print(cfg, "Mrays/s %.1f" % ((c[0] + c[1] + c[2]) / best / 1e6), "ext %.2f shd %.2f" % (tm["extend_ms"], tm["shadow_ms"]),
          "closest n/l/p %.2f %.2f %.2f" % (s[4] / rc, s[5] / rc, s[6] / rc),
          "shadow n/l/p %.2f %.2f %.2f" % (s[7] / rs, s[8] / rs, s[9] / rs), flush=True)
