#!/usr/bin/env python3
"""Per-iteration stage times (MFX_DIAG_ITER=1) of one libmafrix_rt variant on a scene:
diag_variant.py LIB.so [SCENE] [SPP]. Runs one warm-up and one timed trace."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["MFX_DIAG_ITER"] = "1"
import mafrixraytracing_amd.abi as abi  # noqa: E402

abi._lib = abi.load_library(sys.argv[1])
from mafrixraytracing_amd.native import DEFAULT_SEED, NativeContext  # noqa: E402
from mafrixraytracing_amd.scene_io import load_scene_file  # noqa: E402

scene = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "scenes", "spot.xml")
spp = int(sys.argv[3]) if len(sys.argv) > 3 else 64
ctx = NativeContext(load_scene_file(scene), seed=DEFAULT_SEED)
for k in range(2):
    print(f"--- {os.path.basename(sys.argv[1])} trace {k}", file=sys.stderr, flush=True)
    ctx.accum_clear()
    ctx.trace_accumulate(spp, k * spp)
    ctx.sync()
print(os.path.basename(sys.argv[1]), ctx.trace_timing(), file=sys.stderr, flush=True)
