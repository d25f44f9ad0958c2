#!/usr/bin/env python3
"""Diagnostic: device time of mfx_trace_accumulate at small spp (the Scene.Render regime, 1 spp per
call) vs spp, for the wavefront at several chunk sizes and for the megakernel. Device time only
(HIP events around the call's kernels), no readback. Run on the GPU box:
    python3 scripts/diag_small_frames.py [scene.xml]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mafrixraytracing_amd.abi import MFX_F_MEGAKERNEL, MFX_F_NONE  # noqa: E402
from mafrixraytracing_amd.native import DEFAULT_SEED, NativeContext  # noqa: E402
from mafrixraytracing_amd.scene_io import load_scene_file  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "scenes", "spot.xml")
a = load_scene_file(scene)
variants = [("wavefront chunk=default", MFX_F_NONE, None)] + \
           [(f"wavefront chunk={c}", MFX_F_NONE, str(c)) for c in (256, 512, 4096)] + \
           [("megakernel", MFX_F_MEGAKERNEL, None)]
for name, flags, chunk in variants:
    if chunk:
        os.environ["MFX_CHUNK"] = chunk
    else:
        os.environ.pop("MFX_CHUNK", None)
    with NativeContext(a, seed=DEFAULT_SEED, flags=flags) as ctx:
        base = 0
        for spp in (1, 1, 2, 4, 8, 16, 64):
            reps = 5 if spp < 16 else 2
            ms = []
            t0 = time.perf_counter()
            for _ in range(reps):
                ctx.accum_clear()
                ctx.trace_accumulate(spp, base)
                base += spp
                ms.append(ctx.last_trace_ms())
            wall = (time.perf_counter() - t0) / reps * 1e3
            c = ctx.ray_counts()
            rays = c[0] + c[1] + c[2]
            tm = ctx.trace_timing()
            dev = min(ms)
            print(f"{name:26s} spp {spp:3d}: device {dev:8.3f} ms (min of {reps}), wall {wall:8.3f} ms, "
                  f"{rays / dev / 1e3:8.1f} Mrays/s, extend {tm['extend_ms']:.3f} shadow {tm['shadow_ms']:.3f}",
                  flush=True)
