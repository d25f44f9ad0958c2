#!/usr/bin/env python3
"""Traversal counters (node visits, leaf visits, primitive tests per ray) of a library build on a
scene, from one counted pass (MFX_F_COUNT_STATS). Usage: stats_counts.py LIB.so [SCENE] [SPP]"""
import os, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import mafrixraytracing_amd.abi as abi
abi._lib = abi.load_library(sys.argv[1])
from mafrixraytracing_amd.abi import MFX_F_COUNT_STATS
from mafrixraytracing_amd.native import NativeContext, DEFAULT_SEED
from mafrixraytracing_amd.scene_io import load_scene_file
scene = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "scenes", "spot.xml")
spp = int(sys.argv[3]) if len(sys.argv) > 3 else 2
with NativeContext(load_scene_file(scene), seed=DEFAULT_SEED, flags=MFX_F_COUNT_STATS) as ctx:
    ctx.trace_accumulate(spp, 0)
    s = ctx.ray_counts()
rc, rs = s[0] + s[1], s[2]
print(os.path.basename(sys.argv[1]), json.dumps({
    "closest": [round(s[4] / rc, 3), round(s[5] / rc, 3), round(s[6] / rc, 3)],
    "shadow": [round(s[7] / rs, 3), round(s[8] / rs, 3), round(s[9] / rs, 3)],
    # camera packets (k_camera): wave node steps and leaf slots per camera ray
    "camera_packets": [round(s[10] / s[3], 3), round(s[11] / s[3], 3)]}))
