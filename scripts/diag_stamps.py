#!/usr/bin/env python3
"""Phase shares of the wavefront kernels from a stamp build (-DMFX_DIAG_STAMPS=1 k_extend, =2
k_shadow): wave-cycles spent in fetch/scan, node steps, leaf tests and result writes.
Usage: diag_stamps.py LIB.so [SCENE] [SPP]"""
import os, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import mafrixraytracing_amd.abi as abi
lib = sys.argv[1]
abi._lib = abi.load_library(lib)
from mafrixraytracing_amd.native import NativeContext, DEFAULT_SEED
from mafrixraytracing_amd.abi import MFX_F_COUNT_STATS
from mafrixraytracing_amd.scene_io import load_scene_file
scene = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "scenes", "spot.xml")
spp = int(sys.argv[3]) if len(sys.argv) > 3 else 64
ctx = NativeContext(load_scene_file(scene), seed=DEFAULT_SEED, flags=MFX_F_COUNT_STATS)
ctx.accum_clear(); ctx.trace_accumulate(spp, 0); ctx.sync()
c = ctx.ray_counts()
ph = dict(zip(["fetch", "node", "leaf", "fin"], c[10:14]))
tot = sum(ph.values())
nw = ctx.trace_timing()["launches"]
ext = "extend" in open(lib, "rb").read().decode("latin1") and os.path.basename(lib) == "st1.so"
ln, ll, lp = (c[4], c[5], c[6]) if os.path.basename(lib).startswith("st1") else (c[7], c[8], c[9])
print("per launch: outer %.4g, wave node iters %.4g (%.1f lanes each), lane leaf visits %.4g, lane prim tests %.4g; rays %s"
      % (c[14] / nw, c[15] / nw, ln / max(c[15], 1), ll / nw, lp / nw, c[:3] / nw))
print(os.path.basename(lib), json.dumps({k: round(v / tot, 4) for k, v in ph.items()}), "total wave-cycles %.4g" % tot,
      json.dumps(ctx.trace_timing()))
