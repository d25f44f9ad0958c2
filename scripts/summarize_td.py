"""Summarise scripts/pmc_td_roof.sh's passes into profiles/td_<scene>.json (bench.py roofline.td).

Per trace kernel, per launch: TCP_TOTAL_ACCESSES (line lookups), TD / TA busy cycles (summed over
the 256 TDs / TAs) and GRBM_GUI_ACTIVE (GPU clocks of the dispatch); the dispatch's duration gives
the clock the pass ran at. The roof is the same counters over the td_gather peak case: line
lookups per GPU clock when every lane of every wave loads a distinct L1-resident line. The
fraction a kernel reaches of it is (its lookups per clock) / (the peak's), clock-independent.
Usage: python3 scripts/summarize_td.py OUTDIR [bench args...]"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N_TD = 256  # one TD and one TA per CU


def per_dispatch(path):
    d = collections.defaultdict(dict)
    for f in glob.glob(os.path.join(path, "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = (r["Dispatch_Id"], r["Kernel_Name"].split("(")[0].strip())
            d[k][r["Counter_Name"]] = float(r["Counter_Value"])
            d[k]["ns"] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    return d


def main():
    out = sys.argv[1]
    args = sys.argv[2:]
    scene = "spot"
    cfg = "C2"
    if "--config" in args:
        cfg = args[args.index("--config") + 1]
    sys.path.insert(0, ROOT)
    import bench
    scene = os.path.splitext(bench.CONFIGS[cfg][0])[0]
    if "--scene" in args:
        scene = os.path.splitext(os.path.basename(args[args.index("--scene") + 1]))[0]
    ub = [v for (i, k), v in per_dispatch(os.path.join(out, "ubench")).items() if k.startswith("void gather") or "gather" in k]
    ub = [v for v in ub if v.get("GRBM_GUI_ACTIVE", 0) > 0]
    peak_lpc = max(v["TCP_TOTAL_ACCESSES_sum"] / v["GRBM_GUI_ACTIVE"] for v in ub)
    peak_v = max(ub, key=lambda v: v["TCP_TOTAL_ACCESSES_sum"] / v["GRBM_GUI_ACTIVE"])
    kern = collections.defaultdict(lambda: collections.defaultdict(float))
    for (i, k), v in per_dispatch(os.path.join(out, "bench")).items():
        name = k.replace("void ", "")
        if not (name.startswith("k_extend") or name.startswith("k_shadow") or name.startswith("k_resolve")
                or name.startswith("trace_kernel")):
            continue
        for c, x in v.items():
            kern[name][c] += x
        kern[name]["launches"] += 1
    res = {"scene": scene, "config": cfg, "counters": "TCP_TOTAL_ACCESSES_sum TD_TD_BUSY_sum TA_TA_BUSY_sum GRBM_GUI_ACTIVE",
           "peak": {"case": "scripts/ubench/td_gather peak: 64 active lanes, each a distinct 64-B line of a 16 KB "
                            "(L1-resident) table, 16-B loads, 4 independent per round",
                    "lines_per_clock": peak_lpc,
                    "td_busy_frac": peak_v["TD_TD_BUSY_sum"] / (peak_v["GRBM_GUI_ACTIVE"] * N_TD),
                    "clock_mhz": peak_v["GRBM_GUI_ACTIVE"] / peak_v["ns"] * 1e3},
           "kernels": {}}
    for name, v in kern.items():
        n = v["launches"]
        cyc = v["GRBM_GUI_ACTIVE"]
        res["kernels"][name] = {
            "launches": n,
            "tcp_accesses_per_launch": v["TCP_TOTAL_ACCESSES_sum"] / n,
            "td_busy_per_launch": v["TD_TD_BUSY_sum"] / n,
            "ta_busy_per_launch": v["TA_TA_BUSY_sum"] / n,
            "gpu_clocks_per_launch": cyc / n,
            "ms_per_launch": v["ns"] / n / 1e6,
            "clock_mhz": cyc / v["ns"] * 1e3,
            "lines_per_clock": v["TCP_TOTAL_ACCESSES_sum"] / cyc,
            "frac_of_peak": v["TCP_TOTAL_ACCESSES_sum"] / cyc / peak_lpc,
            "td_busy_frac": v["TD_TD_BUSY_sum"] / (cyc * N_TD),
            "ta_busy_frac": v["TA_TA_BUSY_sum"] / (cyc * N_TD),
        }
    dst = os.path.join(ROOT, "profiles", f"td_{scene}.json")
    with open(os.path.join(out, "td.json"), "w") as f:
        json.dump(res, f, indent=1)
    with open(dst, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
