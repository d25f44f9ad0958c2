#!/usr/bin/env python3
"""Timeline of a rocprofv3 kernel trace of scripts/share_trace.py: the dispatches are split into
segments at idle gaps of more than 50 ms (share_trace.py leaves 100 ms before each timed run); for
each segment with at least `min` dispatches: frames (k_camera launches), span per frame, the union of
busy time per frame, the time two or more launches ran at once, and per launch position of a frame
(camera, shadow 0, extend 1, ..., resolve, memsets) the mean duration.
Usage: share_timeline.py DIR_OR_CSV [min_dispatches]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def short(name):
    n = name.replace("void ", "").split("(")[0].split("<")[0]
    return "memset" if "fillBuffer" in n else n


def load(path):
    if os.path.isdir(path):
        path = sorted(glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True))[0]
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                     int(r.get("Queue_Id", 0) or 0), int(r.get("Stream_Id", 0) or 0)))
    rows.sort()
    return rows


def segments(rows, gap_ns=50e6):
    seg, out, end = [], [], None
    for r in rows:
        if end is not None and r[0] - end > gap_ns:
            out.append(seg)
            seg = []
        seg.append(r)
        end = r[1] if end is None else max(end, r[1])
    if seg:
        out.append(seg)
    return out


def union_and_overlap(seg):
    ev = []
    for s, e, *_ in seg:
        ev.append((s, 1))
        ev.append((e, -1))
    ev.sort()
    busy = over = 0
    depth, last = 0, ev[0][0]
    for t, d in ev:
        if depth >= 1:
            busy += t - last
        if depth >= 2:
            over += t - last
        depth += d
        last = t
    return busy, over


def main(path, min_n=40):
    rows = load(path)
    for i, seg in enumerate(segments(rows)):
        if len(seg) < min_n:
            continue
        frames = sum(1 for r in seg if r[2] == "k_camera") or 1
        span = (max(r[1] for r in seg) - seg[0][0]) / 1e6
        busy, over = union_and_overlap(seg)
        streams = sorted(set(r[4] for r in seg))
        tot = defaultdict(float)
        for s, e, k, q, st in seg:
            tot[k] += (e - s) / 1e6
        print(f"segment {i}: {len(seg)} dispatches, {frames} frames, {len(streams)} streams; per frame: span "
              f"{span / frames:.4f} ms, busy {busy / 1e6 / frames:.4f} ms, 2+ launches at once {over / 1e6 / frames:.4f} ms, "
              f"sum of launch durations {sum(tot.values()) / frames:.4f} ms")
        print("   per frame by kernel: " + ", ".join(f"{k} {v / frames:.4f}" for k, v in sorted(tot.items())))
        # per launch position within a stream's frames (a frame starts at its k_camera)
        pos = defaultdict(list)
        for st in streams:
            n = -1
            for s, e, k, q, sid in seg:
                if sid != st:
                    continue
                if k == "k_camera":
                    n = 0
                elif n < 0:
                    continue
                pos[n].append((k, (e - s) / 1e6))
                n += 1
        line = []
        for n in sorted(pos):
            ks = defaultdict(list)
            for k, d in pos[n]:
                ks[k].append(d)
            line.append(" / ".join(f"{n}:{k} {sum(v) / len(v):.4f}" for k, v in ks.items()))
        print("   by position: " + "; ".join(line))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 40)
