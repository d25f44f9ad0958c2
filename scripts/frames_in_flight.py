#!/usr/bin/env python3
"""Two frames in flight: consecutive frames on two contexts (two path pools, two HIP streams on
one GPU) against one context, for the C2 frame and for one rank's share of it at N GPUs (tile
rows 0 mod N, MFX_F_ROW_PARTITION). Every persistent launch fills the GPU, so a second stream's
launches only get CUs as the first stream's blocks retire: the next frame's dense first launches
run in the previous frame's tails. Frames are independent (each its own accumulator; a renderer's
next frame does not read the previous one's), the rays are the same. Prints one JSON line."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(ctxs, spp, steps):
    for c in ctxs:  # warm (pool allocation)
        c.trace_accumulate(spp, 0)
    for c in ctxs:
        c.sync()
        c.ray_counts_total(reset=True)
    t0 = time.perf_counter()
    for k in range(steps):
        c = ctxs[k % len(ctxs)]
        c.accum_clear()
        c.trace_accumulate(spp, (k + 1) * spp)
    for c in ctxs:
        c.sync()
    ms = (time.perf_counter() - t0) / steps * 1e3
    rays = sum(float(sum(c.ray_counts_total(reset=True)[:3])) for c in ctxs)
    return ms, rays / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default=os.path.join(ROOT, "scenes", "spot.xml"))
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--parts", default="1,2,4,8")
    ap.add_argument("--modes", default="1,2", help="contexts in flight per run, comma-separated")
    ap.add_argument("--torch", default="", help="'import' or 'cuda': import torch (and initialize its HIP context) first")
    a = ap.parse_args()
    if a.torch:
        import torch
        if a.torch == "cuda":
            torch.zeros(1, device="cuda")
    from mafrixraytracing_amd.abi import MFX_F_IN_FLIGHT, MFX_F_ROW_PARTITION
    from mafrixraytracing_amd.native import DEFAULT_SEED, NativeContext
    from mafrixraytracing_amd.scene_io import load_scene_file
    arr = load_scene_file(a.scene)
    out = {"scene": os.path.basename(a.scene), "spp": a.spp, "steps": a.steps}
    modes = [int(m) for m in a.modes.split(",")]
    for parts in (int(p) for p in a.parts.split(",")):
        kw = dict(flags=MFX_F_ROW_PARTITION, part_index=0, part_count=parts) if parts > 1 else {}
        row = {}
        for inflight in modes + modes:  # interleaved
            k2 = dict(kw)
            if inflight > 1:  # what bench.py's ranks create (MFX_F_IN_FLIGHT)
                k2["flags"] = k2.get("flags", 0) | MFX_F_IN_FLIGHT
            ctxs = [NativeContext(arr, seed=DEFAULT_SEED, **k2) for _ in range(inflight)]
            ms, rays = run(ctxs, a.spp, a.steps * max(1, parts // 2))
            for c in ctxs:
                c.close()
            r = row.setdefault(str(inflight), {"ms_per_frame": [], "rays_per_frame": rays})
            r["ms_per_frame"].append(round(ms, 3))
        for r in row.values():
            r["best_ms"] = min(r["ms_per_frame"])
            r["mrays_per_s"] = round(r["rays_per_frame"] / (r["best_ms"] / 1e3) / 1e6, 1)
        out["whole_film" if parts == 1 else f"share_1_of_{parts}"] = row
    print(json.dumps(out))


if __name__ == "__main__":
    main()
