#!/usr/bin/env python3
"""Scene-preparation timings (mfx_build_info) of the C2/C4/C5 scenes: GPU images vs the host build,
and the instanced C5. Second context of each kind timed (the first warms the device)."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mafrixraytracing_amd.abi import MFX_F_HOST_BVH, MFX_F_FLATTEN
from mafrixraytracing_amd.native import NativeContext
from mafrixraytracing_amd.scene_io import load_scene_file
out = {}
for name in ("spot", "renault", "spot16", "spot16_instanced"):
    a = load_scene_file(os.path.join(ROOT, "scenes", name + ".xml"))
    for label, flags in (("gpu", 0), ("host", MFX_F_HOST_BVH)):
        for _ in range(2):
            with NativeContext(a, flags=flags) as c:
                b = c.build_info()
        out[f"{name}/{label}"] = {k: (round(v, 2) if isinstance(v, float) else v) for k, v in b.items() if k != "digest"}
        out[f"{name}/{label}"]["digest"] = hex(b["digest"])
print(json.dumps(out, indent=1))
