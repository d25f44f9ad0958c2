#!/usr/bin/env python3
"""Stage timing of the wavefront pipeline vs the megakernel on the bench workload."""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mafrixraytracing_amd.abi import MFX_F_MEGAKERNEL, MFX_F_NONE
from mafrixraytracing_amd.native import NativeContext, DEFAULT_SEED
from mafrixraytracing_amd.scene_io import load_scene_file

scene = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "scenes", "spot.xml")
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 64
pools = [int(x) for x in (sys.argv[3].split(",") if len(sys.argv) > 3 else ["2097152"])]
a = load_scene_file(scene)
for mode in ["mega"] + [f"wf{p}" for p in pools]:
    if mode.startswith("wf"):
        os.environ["MFX_POOL"] = mode[2:]
    ctx = NativeContext(a, seed=DEFAULT_SEED, flags=MFX_F_MEGAKERNEL if mode == "mega" else MFX_F_NONE)
    for k in range(3):
        ctx.accum_clear(); t = time.perf_counter(); ctx.trace_accumulate(spp, k * spp); ctx.sync(); dt = time.perf_counter() - t
    c = ctx.ray_counts(); tm = ctx.trace_timing()
    rays = c[0] + c[1] + c[2]
    print(mode, "wall %.1f ms" % (dt * 1e3), "Mrays/s %.1f" % (rays / dt / 1e6), json.dumps({k: round(v, 2) for k, v in tm.items()}), flush=True)
    ctx.close()
