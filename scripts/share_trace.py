#!/usr/bin/env python3
"""One rank's share of the strong-scaled C2 job, for a rocprofv3 kernel trace (scripts/share_timeline.py
reads it): rank R of N traces all spp samples of its tile rows (MFX_F_ROW_PARTITION) over NIF contexts,
frames alternating as bench.py's ranks run them (distributed.frames_in_flight). Warmup frames, a
100 ms idle gap (the timeline splits the warmup off at it), then the timed frames back to back.
Prints one JSON line per (nif) setting with the host-clock ms per frame.
Usage: share_trace.py [--parts 8] [--rank 0] [--nif 1,3] [--steps 20] [--spp 64] [--scene FILE]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--parts", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--nif", default="1,3")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--scene", default=os.path.join(ROOT, "scenes", "spot.xml"))
    a = ap.parse_args()
    from mafrixraytracing_amd.abi import MFX_F_IN_FLIGHT, MFX_F_ROW_PARTITION
    from mafrixraytracing_amd.native import DEFAULT_SEED, NativeContext
    from mafrixraytracing_amd.scene_io import load_scene_file
    arrays = load_scene_file(a.scene)
    for nif in [int(x) for x in a.nif.split(",")]:
        fl = MFX_F_ROW_PARTITION | (MFX_F_IN_FLIGHT if nif > 1 else 0)
        cs = [NativeContext(arrays, seed=DEFAULT_SEED, flags=fl, part_index=a.rank, part_count=a.parts)
              for _ in range(nif)]
        for k, c in enumerate(cs):  # pools allocated, warm
            c.accum_clear()
            c.trace_accumulate(a.spp, k * a.spp)
        for c in cs:
            c.sync()
        time.sleep(0.1)  # the timeline's split
        t0 = time.perf_counter()
        for k in range(a.steps):
            c = cs[k % nif]
            c.accum_clear()
            c.trace_accumulate(a.spp, (k + 10) * a.spp)
        for c in cs:
            c.sync()
        ms = (time.perf_counter() - t0) / a.steps * 1e3
        print(json.dumps({"parts": a.parts, "rank": a.rank, "nif": nif, "steps": a.steps, "ms_per_frame": round(ms, 4)}),
              flush=True)
        for c in cs:
            c.close()
        time.sleep(0.1)


if __name__ == "__main__":
    main()
