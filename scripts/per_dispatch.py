#!/usr/bin/env python3
"""Per-dispatch view of a scripts/profile_traffic.sh directory (or any rocprofv3 output with a
kernel-trace pass under trace/ and FETCH_SIZE / WRITE_SIZE passes under fetch/ and write/): for
each trace kernel launch of the last frame, in order, its duration, HBM bytes, start offset and the idle gap
before it (FETCH_SIZE x2 by
the gfx950 correction, WRITE_SIZE as reported). The wavefront's launches of one frame run
k_camera, then (k_shadow, k_extend) per bounce, so the order names the bounce.
Usage: per_dispatch.py DIR"""
import csv
import glob
import os
import sys

KERNELS = ("k_camera", "k_extend", "k_shadow", "k_resolve")


def one(pattern):
    f = sorted(glob.glob(pattern, recursive=True))
    return f[0] if f else None


def short(name):
    return name.replace("void ", "").split("(")[0].split("<")[0]


def pmc(path, counter):
    rows = []
    if path:
        for r in csv.DictReader(open(path)):
            if r["Counter_Name"] == counter and short(r["Kernel_Name"]) in KERNELS:
                rows.append((int(r["Dispatch_Id"]), short(r["Kernel_Name"]), float(r["Counter_Value"])))
    rows.sort()
    return rows


def main(d):
    tr = one(os.path.join(d, "trace", "**", "*kernel_trace.csv"))
    durs = []
    if tr:
        for r in csv.DictReader(open(tr)):
            k = short(r["Kernel_Name"])
            if k in KERNELS:
                durs.append((int(r["Dispatch_Id"]), k, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6,
                             int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
        durs.sort()
    fetch = pmc(one(os.path.join(d, "fetch", "**", "*counter_collection.csv")), "FETCH_SIZE")
    write = pmc(one(os.path.join(d, "write", "**", "*counter_collection.csv")), "WRITE_SIZE")

    def last_frame(rows):  # from the last k_camera launch on
        idx = [i for i, r in enumerate(rows) if r[1] == "k_camera"]
        return rows[idx[-1]:] if idx else rows

    durs, fetch, write = last_frame(durs), last_frame(fetch), last_frame(write)
    n = max(len(durs), len(fetch), len(write))
    print(f"{'#':>3} {'kernel':10} {'ms':>8} {'fetch GB':>9} {'write GB':>9} {'start ms':>9} {'gap ms':>7}")
    t0 = durs[0][3] if durs else 0
    for i in range(n):
        k = (durs[i][1] if i < len(durs) else fetch[i][1] if i < len(fetch) else write[i][1])
        ms = f"{durs[i][2]:8.3f}" if i < len(durs) else " " * 8
        fb = f"{2.0 * fetch[i][2] * 1024 / 1e9:9.3f}" if i < len(fetch) else " " * 9
        wb = f"{write[i][2] * 1024 / 1e9:9.3f}" if i < len(write) else " " * 9
        st = f"{(durs[i][3] - t0) / 1e6:9.3f}" if i < len(durs) else " " * 9
        gp = f"{(durs[i][3] - durs[i - 1][4]) / 1e6:7.3f}" if 0 < i < len(durs) else " " * 7
        print(f"{i:3d} {k:10} {ms} {fb} {wb} {st} {gp}")
    if durs:
        busy = sum(d[2] for d in durs)
        span = (durs[-1][4] - durs[0][3]) / 1e6
        print(f"frame span {span:.3f} ms, kernels busy {busy:.3f} ms, gaps {span - busy:.3f} ms")


if __name__ == "__main__":
    main(sys.argv[1])
