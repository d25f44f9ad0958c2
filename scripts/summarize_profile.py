#!/usr/bin/env python3
"""Summarise a scripts/profile_traffic.sh output directory: per-kernel launch count and average
duration (kernel trace) and HBM bytes per launch from the separate FETCH_SIZE / WRITE_SIZE
passes. FETCH_SIZE is doubled (MI355X_MICROARCH.md: gfx950 tallies 128-B requests at 64 B);
WRITE_SIZE is taken as reported (calibrated for 16-B stores and dword atomics; the FP64 pixel
atomics of k_logic are uncalibrated). Writes <dir>/traffic.json."""
import collections
import csv
import glob
import json
import os
import sys


def one(pattern):
    f = glob.glob(pattern, recursive=True)
    return f[0] if f else None


def pmc(path, counter):
    acc = collections.defaultdict(lambda: [0.0, 0])
    if path:
        for r in csv.DictReader(open(path)):
            if r["Counter_Name"] == counter:
                a = acc[r["Kernel_Name"]]
                a[0] += float(r["Counter_Value"])
                a[1] += 1
    return acc


def main(d, bench_args=()):
    stats = one(os.path.join(d, "trace", "**", "*kernel_stats.csv"))
    kern = {}
    if stats:
        for r in csv.DictReader(open(stats)):
            kern[r["Name"]] = {"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6,
                               "total_ms": float(r["TotalDurationNs"]) / 1e6, "pct": float(r["Percentage"])}
    fetch = pmc(one(os.path.join(d, "fetch", "**", "*counter_collection.csv")), "FETCH_SIZE")
    write = pmc(one(os.path.join(d, "write", "**", "*counter_collection.csv")), "WRITE_SIZE")
    out = {}
    for name in set(fetch) | set(write):
        short = name.replace("void ", "").split("(")[0]
        fs, fn = fetch.get(name, [0.0, 0])
        ws, wn = write.get(name, [0.0, 0])
        fb = 2.0 * fs * 1024 / fn if fn else 0.0
        wb = ws * 1024 / wn if wn else 0.0
        out[short] = {"launches_profiled": max(fn, wn), "fetch_bytes_per_launch": fb, "write_bytes_per_launch": wb,
                      "hbm_bytes_per_launch": fb + wb}
    # the bench workload the passes ran (bench.py --config / --spp), so bench.py only pairs this
    # traffic with the same workload
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import CONFIGS
    a = list(bench_args)
    cfg = a[a.index("--config") + 1] if "--config" in a else "C2"
    spp = int(a[a.index("--spp") + 1]) if "--spp" in a else CONFIGS[cfg][1]
    res = {"config": cfg, "scene": CONFIGS[cfg][0], "spp": spp, "kernels": out, "trace": kern,
           "note": "FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE, per launch, from separate --pmc passes"}
    with open(os.path.join(d, "traffic.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
