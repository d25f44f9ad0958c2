#!/usr/bin/env python3
"""Freeze the per-config algorithmic bytes per ray before kernel tuning.

B_ray = N_node x 32 B + N_tri x 36 B + 64 B, with N_node = BVH2 node visits (internal-node visits +
leaf visits of the cluster BVH2) and N_tri = primitive tests, per traced ray of the kind the
kernel handles, counted by the kernels' own traversal counters (MFX_F_COUNT_STATS) at 1 spp of
each config scene. Committed as profiles/bray_fixture.json; bench.py prices the roofline with
these fixed values, so later traversal improvements show up as speed, not as changed bytes.
Run on the GPU box: python scripts/make_bray_fixture.py [LIB.so] (the library to count with; the
committed fixture was made with the round-1 kernels before the leaf-test shortcuts)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import mafrixraytracing_amd.abi as abi  # noqa: E402
from mafrixraytracing_amd.abi import MFX_F_COUNT_STATS  # noqa: E402
from mafrixraytracing_amd.native import DEFAULT_SEED, NativeContext  # noqa: E402
from mafrixraytracing_amd.scene_io import load_scene_file  # noqa: E402

SCENES = ["spot", "cube_cornell", "renault", "spot16", "cornell", "two_spheres_plane"]


def bray(nodes, prims):
    return 32.0 * nodes + 36.0 * prims + 64.0


def main():
    if len(sys.argv) > 1:
        abi._lib = abi.load_library(sys.argv[1])
    out = {"formula": "B_ray = 32*N_node + 36*N_tri + 64 (SURVEY.md 8d); N_node = internal + leaf visits",
           "seed": DEFAULT_SEED, "spp": 1, "scenes": {}}
    for name in SCENES:
        a = load_scene_file(os.path.join(ROOT, "scenes", name + ".xml"))
        with NativeContext(a, seed=DEFAULT_SEED, flags=MFX_F_COUNT_STATS) as c:
            c.trace_accumulate(1, 10 ** 6)
            s = c.ray_counts()
        rc, rs = s[0] + s[1], s[2]
        e = {"closest_rays": rc, "shadow_rays": rs,
             "closest": {"N_node": (s[4] + s[5]) / rc, "N_tri": s[6] / rc},
             "shadow": {"N_node": (s[7] + s[8]) / rs, "N_tri": s[9] / rs}}
        for k in ("closest", "shadow"):
            e[k]["B_ray"] = bray(e[k]["N_node"], e[k]["N_tri"])
        out["scenes"][name] = e
        print(name, json.dumps(e), flush=True)
    with open(os.path.join(ROOT, "gpurun_out", "bray_fixture.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    main()
