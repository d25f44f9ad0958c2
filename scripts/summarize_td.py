"""Summarise scripts/pmc_td_roof.sh's passes into profiles/td_<scene>.json (bench.py roofline.td).

Per trace kernel, per launch: TCP_TOTAL_CACHE_ACCESSES (L1 tag lookups: cache lines touched per
wave memory instruction), TCP_TCC_READ_REQ (L1 misses read from L2), TD busy cycles (summed over
the 256 TDs) and GRBM_GUI_ACTIVE (GPU clocks of the dispatch, summed over the 8 XCDs); the
dispatch's duration gives the clock the pass ran at. (TCP_TOTAL_ACCESSES counts lanes, 64 per wave
instruction whatever the lines: round 2's per-instruction figure.) The roof is the same counters
over the td_gather peak case, every lane of every wave a distinct L1-resident line: its lookups per
GPU clock and its TD busy fraction. A kernel's fraction is (its lookups per clock) / (the peak's),
clock-independent; td_busy_frac is the share of TD cycles the kernel keeps busy.
Usage: python3 scripts/summarize_td.py OUTDIR [bench args...]"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N_TD = 256  # one TD per CU
N_XCD = 8  # GRBM_GUI_ACTIVE is summed over the XCDs


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
    for v in ub:
        v["cyc"] = v["GRBM_GUI_ACTIVE"] / N_XCD
    peak_v = max(ub, key=lambda v: v["TCP_TOTAL_CACHE_ACCESSES_sum"] / v["cyc"])
    peak_lpc = peak_v["TCP_TOTAL_CACHE_ACCESSES_sum"] / peak_v["cyc"]
    kern = collections.defaultdict(lambda: collections.defaultdict(float))
    for (i, k), v in per_dispatch(os.path.join(out, "bench")).items():
        name = k.replace("void ", "")
        if not (name.startswith("k_extend") or name.startswith("k_shadow") or name.startswith("k_resolve")
                or name.startswith("k_camera") or name.startswith("trace_kernel")):
            continue
        for c, x in v.items():
            kern[name][c] += x
        kern[name]["launches"] += 1
    res = {"scene": scene, "config": cfg,
           "counters": "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE",
           "peak": {"case": "scripts/ubench/td_gather peak: 64 active lanes, each a distinct 64-B line of a 16 KB "
                            "(L1-resident) table, 16-B loads, 4 independent per round",
                    "lines_per_clock": peak_lpc,
                    "td_busy_frac": peak_v["TD_TD_BUSY_sum"] / (peak_v["cyc"] * N_TD),
                    "clock_mhz": peak_v["cyc"] / peak_v["ns"] * 1e3},
           "kernels": {}}
    for name, v in kern.items():
        n = v["launches"]
        cyc = v["GRBM_GUI_ACTIVE"] / N_XCD
        res["kernels"][name] = {
            "launches": n,
            "line_lookups_per_launch": v["TCP_TOTAL_CACHE_ACCESSES_sum"] / n,
            "l2_reads_per_launch": v["TCP_TCC_READ_REQ_sum"] / n,
            "td_busy_per_launch": v["TD_TD_BUSY_sum"] / n,
            "gpu_clocks_per_launch": cyc / n,
            "ms_per_launch": v["ns"] / n / 1e6,
            "clock_mhz": cyc / v["ns"] * 1e3,
            "lines_per_clock": v["TCP_TOTAL_CACHE_ACCESSES_sum"] / cyc,
            "frac_of_peak": v["TCP_TOTAL_CACHE_ACCESSES_sum"] / cyc / peak_lpc,
            "td_busy_frac": v["TD_TD_BUSY_sum"] / (cyc * N_TD),
        }
    # the scalar-memory pass (k_camera's roof): SQ_INSTS_SMEM per GPU clock against scripts/ubench/sload's
    # peak case (wave-uniform 128-B nodes from a 256 KB table, two 64-B loads each, 4 waves per SIMD)
    sub = per_dispatch(os.path.join(out, "ubench_smem"))
    sp = [v for (i, k), v in sub.items() if "sgather" in k and v.get("GRBM_GUI_ACTIVE", 0) > 0]
    if sp:
        for v in sp:
            v["cyc"] = v["GRBM_GUI_ACTIVE"] / N_XCD
        pv = max(sp, key=lambda v: v["SQ_INSTS_SMEM"] / v["cyc"])
        speak = pv["SQ_INSTS_SMEM"] / pv["cyc"]
        res["smem_peak"] = {"case": "scripts/ubench/sload peak: wave-uniform 128-B nodes (two s_load_dwordx16) at "
                                    "hashed indices of a 256 KB table, 4 independent per round, 16 waves per CU",
                            "smem_per_clock": speak, "clock_mhz": pv["cyc"] / pv["ns"] * 1e3}
        sk = collections.defaultdict(lambda: collections.defaultdict(float))
        for (i, k), v in per_dispatch(os.path.join(out, "bench_smem")).items():
            name = k.replace("void ", "")
            if name in res["kernels"]:
                for c, x in v.items():
                    sk[name][c] += x
                sk[name]["launches"] += 1
        for name, v in sk.items():
            cyc = v["GRBM_GUI_ACTIVE"] / N_XCD
            res["kernels"][name].update({"smem_per_launch": v["SQ_INSTS_SMEM"] / v["launches"],
                                         "smem_per_clock": v["SQ_INSTS_SMEM"] / cyc,
                                         "smem_frac_of_peak": v["SQ_INSTS_SMEM"] / cyc / speak,
                                         "smem_gpu_clocks_per_launch": cyc / v["launches"],
                                         "smem_ms_per_launch": v["ns"] / v["launches"] / 1e6})
    dst = os.path.join(ROOT, "profiles", f"td_{scene}.json")
    with open(os.path.join(out, "td.json"), "w") as f:
        json.dump(res, f, indent=1)
    with open(dst, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
