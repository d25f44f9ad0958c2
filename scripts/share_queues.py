#!/usr/bin/env python3
"""Which hardware queues a strong-share child's contexts land on (rocprofv3 kernel trace Queue_Id)
and how fast its shares ran: `share_queues.py DIR` reads DIR/p*/trace/**/*kernel_trace.csv and
DIR/p*/run.json (bench.py --strong-share-child 0 0 under rocprofv3, gpu_run step `sharequeues`).
For every run of back-to-back frames of the wavefront kernels (a rank's timed frames: split at idle
gaps > 20 ms), it prints the distinct Queue_Ids its kernels used and the frames' span."""
import csv
import glob
import json
import os
import sys
from collections import Counter


def main(d):
    for p in sorted(glob.glob(os.path.join(d, "p*"))):
        rj = os.path.join(p, "run.json")
        share = json.load(open(rj)) if os.path.exists(rj) and os.path.getsize(rj) else None
        sl = {n: v["slowest_rank_ms"] for n, v in share["shares"].items()} if share else None
        f = sorted(glob.glob(os.path.join(p, "trace", "**", "*kernel_trace.csv"), recursive=True))
        if not f:
            continue
        rows = [r for r in csv.DictReader(open(f[0])) if r["Kernel_Name"].lstrip("void ").startswith("k_")]
        rows.sort(key=lambda r: int(r["Start_Timestamp"]))
        segs, cur, end = [], [], None
        for r in rows:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if end is not None and s - end > 20e6:
                segs.append(cur)
                cur = []
            cur.append(r)
            end = e if end is None else max(end, e)
        segs.append(cur)
        print(os.path.basename(p), "slowest per N:", sl)
        for sg in segs:
            if len(sg) < 60:
                continue
            q = Counter(r["Queue_Id"] for r in sg)
            span = (max(int(r["End_Timestamp"]) for r in sg) - int(sg[0]["Start_Timestamp"])) / 1e6
            cams = sum(1 for r in sg if "k_camera" in r["Kernel_Name"])
            print(f"   {len(sg):4d} launches, {cams:3d} frames, {span / max(cams, 1):7.3f} ms per frame, queues {dict(q)}")


if __name__ == "__main__":
    main(sys.argv[1])
