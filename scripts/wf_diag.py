#!/usr/bin/env python3
"""Stage timing of the wavefront pipeline (pool size x sub-pools) vs the megakernel on the bench
workload. Usage: wf_diag.py SCENE SPP MODES, MODES = comma list of "mega" or "POOL:NSUB"."""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mafrixraytracing_amd.abi import MFX_F_MEGAKERNEL, MFX_F_NONE
from mafrixraytracing_amd.native import NativeContext, DEFAULT_SEED
from mafrixraytracing_amd.scene_io import load_scene_file

scene = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "scenes", "spot.xml")
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 64
modes = (sys.argv[3] if len(sys.argv) > 3 else "mega,16777216:1,16777216:2").split(",")
a = load_scene_file(scene)
for mode in modes:
    if mode != "mega":
        pool, nsub = mode.split(":")
        os.environ["MFX_POOL"] = pool
        os.environ["MFX_SUBPOOLS"] = nsub
    ctx = NativeContext(a, seed=DEFAULT_SEED, flags=MFX_F_MEGAKERNEL if mode == "mega" else MFX_F_NONE)
    best = None
    for k in range(3):
        ctx.accum_clear(); t = time.perf_counter(); ctx.trace_accumulate(spp, k * spp); ctx.sync(); dt = time.perf_counter() - t
        best = dt if best is None else min(best, dt)
    c = ctx.ray_counts(); tm = ctx.trace_timing()
    rays = c[0] + c[1] + c[2]
    print(mode, "wall %.1f ms" % (best * 1e3), "Mrays/s %.1f" % (rays / best / 1e6),
          json.dumps({k: round(v, 2) for k, v in tm.items()}), flush=True)
    ctx.close()
