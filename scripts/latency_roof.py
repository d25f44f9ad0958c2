#!/usr/bin/env python3
"""Latency roof of the per-lane traversal kernels (VERDICT r05 Next #3): how much of k_extend's and
k_shadow's time their dependent node-step chain (load the node -> slab tests -> next node) explains.

Three child runs of scripts/diag_variant.py (MFX_DIAG_ITER=1, one warm-up trace and one measured
trace of SCENE at SPP): the shipped library (per-iteration HIP-event times of every launch, and the
launch shapes), and the stamp builds st1 (-DMFX_DIAG -DMFX_DIAG_STAMPS=1, k_extend) and st2 (=2,
k_shadow) from build_variants/ (scripts/build_variant.sh). A stamp build counts per launch the
wave-level node steps (node_iters: one per wave iteration of the node loop), every wave's cycles in
each phase, and `lat`: the cycles from each node step's loads issuing to their first use (s_memtime
around the loads in node_step), i.e. the step's loaded round trip.

Per kernel (its launches pooled):
  L_step   = lat / node_iters                    the loaded round trip of one node step (cycles)
  lat_share = lat / wave-cycles                  share of every wave's life spent waiting on one
  f        = wave-cycles / (waves resident x stamp-build time)    the clock s_memtime counts
  peak     = f / L_step                          node steps per second per wave if each waits one
                                                 round trip (the latency roof)
  achieved = node_iters / waves resident / T     with T the shipped kernel's HIP-event time
  frac     = achieved / peak                     = node_iters x L_step / (waves x f x T)
A frac near 1 says the kernel's time is its node chain's round trips, with every resident wave
waiting; the rest of the time is leaf tests, scans and shading. The loaded round trip against the
idle one (profiles/ubench_chase_r01.txt: 573-602 cycles for an L2-resident table, one load per step)
says how much of it is queueing behind other waves' requests.
Writes JSON (profiles/latency_<scene>.json, which bench.py reads for roofline.latency).
Usage: latency_roof.py [--scene FILE] [--spp 64] [--out FILE]"""
import argparse
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
LINE = re.compile(r"gen (\d+) iter (\d+): .*?extend ([\d.]+) ms shadow ([\d.]+) ms; stamps (\S+) (\S+) (\S+) (\S+) "
                  r"outer (\S+) node (\S+);.*scan (\S+) shade (\S+) lat (\S+)")
SHAPE = re.compile(r"blocks/CU extend (\d+) shadow (\d+) \((\d)-wave build\)")
L_IDLE = {"cycles": 573.0, "source": "profiles/ubench_chase_r01.txt (256 KB table, 1 load per step, 4 waves/CU)"}


def run(lib, scene, spp, timeout=300):
    cmd = [sys.executable, os.path.join(ROOT, "scripts", "diag_variant.py"), lib, scene, str(spp)]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=dict(os.environ, MFX_DIAG_ITER="1"))
    if p.returncode != 0:
        raise RuntimeError(f"{lib}: {p.stderr[-2000:]}")
    return p.stderr


def parse(err):
    """Per-iteration deltas of the last trace (the cumulative counters restart at each trace)."""
    trace = err.split("--- ")[-1]
    rows = []
    for m in LINE.finditer(trace):
        v = [float(x) for x in m.groups()]
        rows.append({"iter": int(v[1]), "extend_ms": v[2], "shadow_ms": v[3], "fetch": v[4], "node": v[5],
                     "leaf": v[6], "fin": v[7], "outer": v[8], "node_iters": v[9], "scan": v[10], "shade": v[11],
                     "lat": v[12]})
    out, prev = [], None
    for r in rows:
        d = dict(r)
        if prev is not None:
            for k in ("fetch", "node", "leaf", "fin", "outer", "node_iters", "scan", "shade", "lat"):
                d[k] = r[k] - prev[k]
        out.append(d)
        prev = r
    shape = SHAPE.search(err)
    return out, (tuple(int(x) for x in shape.groups()) if shape else None)


def kernel(name, stamp, prod, waves, simds, iters):
    s = [r for r in stamp if r["iter"] in iters]
    p = [r for r in prod if r["iter"] in iters]
    key = "extend_ms" if name == "k_extend" else "shadow_ms"
    wc = sum(r["fetch"] + r["node"] + r["leaf"] + r["fin"] + r["scan"] + r["shade"] for r in s)
    lat = sum(r["lat"] for r in s)
    ni = sum(r["node_iters"] for r in s)
    t_stamp = sum(r[key] for r in s) / 1e3
    t_prod = sum(r[key] for r in p) / 1e3
    nw = waves * simds
    f = wc / (nw * t_stamp)
    l_step = lat / ni
    peak = f / l_step
    ach = ni / nw / t_prod
    per = []
    for rs, rp in zip(s, p):
        wci = rs["fetch"] + rs["node"] + rs["leaf"] + rs["fin"] + rs["scan"] + rs["shade"]
        if rs["node_iters"] <= 0 or wci <= 0:
            continue
        li = rs["lat"] / rs["node_iters"]
        fi = wci / (nw * rs[key] / 1e3)
        per.append({"iteration": rs["iter"] - 1, "node_steps_per_wave": round(rs["node_iters"] / nw, 1),
                    "L_step_cycles": round(li, 1), "lat_share_stamp_build": round(rs["lat"] / wci, 4),
                    "node_phase_share": round(rs["node"] / wci, 4),
                    "phase_shares": {k: round(rs[k] / wci, 4) for k in ("fetch", "scan", "shade", "node", "leaf", "fin")},
                    "ms_shipped": rp[key], "ms_stamp_build": rs[key],
                    "frac": round(rs["node_iters"] / nw / (rp[key] / 1e3) / (fi / li), 4)})
    return {"bound": "latency", "achieved": round(ach / 1e6, 4), "peak": round(peak / 1e6, 4),
            "unit": "M node steps/s per resident wave", "frac": round(ach / peak, 4),
            "L_step_cycles": round(l_step, 1), "L_idle_cycles": L_IDLE["cycles"],
            "loaded_over_idle": round(l_step / L_IDLE["cycles"], 3), "clock_mhz": round(f / 1e6, 1),
            "waves_per_simd": waves, "node_steps_per_launch": ni / len(s), "launches": len(s),
            "node_steps_per_wave": round(ni / nw, 1), "lat_share_stamp_build": round(lat / wc, 4),
            "ms_shipped": round(t_prod * 1e3, 4), "ms_stamp_build": round(t_stamp * 1e3, 4),
            "per_launch": per}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default=os.path.join(ROOT, "scenes", "spot.xml"))
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--out", default=None)
    ap.add_argument("--simds", type=int, default=1024, help="256 CUs x 4 SIMDs (MI355X)")
    # a variant's roof (VERDICT r05 Next #4): its library and its own stamp builds
    ap.add_argument("--lib", default=os.path.join(ROOT, "mafrixraytracing_amd", "libmafrix_rt.so"))
    ap.add_argument("--st1", default=os.path.join(ROOT, "build_variants", "st1.so"))
    ap.add_argument("--st2", default=os.path.join(ROOT, "build_variants", "st2.so"))
    ap.add_argument("--st3", default=os.path.join(ROOT, "build_variants", "st3.so"))
    a = ap.parse_args()
    prod, shape = parse(run(a.lib, a.scene, a.spp))
    st1, _ = parse(run(a.st1, a.scene, a.spp))
    st2, _ = parse(run(a.st2, a.scene, a.spp))
    ebpc, sbpc, _ = shape  # 256-lane blocks per CU = waves per SIMD
    nit = max(r["iter"] for r in prod)
    cam = None
    st3p = a.st3
    if os.path.exists(st3p):  # k_camera's phases (-DMFX_DIAG_STAMPS=3), VERDICT r05 Next #5
        st3, _ = parse(run(st3p, a.scene, a.spp))
        r = [x for x in st3 if x["iter"] == 1][0]
        p = [x for x in prod if x["iter"] == 1][0]
        ph = {"window_scan": r["fetch"], "camera_ray": r["node"], "node_steps": r["leaf"], "leaf_tests": r["fin"],
              "result_writes": r["outer"]}
        tot = sum(ph.values())
        from mafrixraytracing_amd.scene_io import load_scene_file
        arr = load_scene_file(a.scene)
        tiles = (arr.width + 7) // 8 * ((arr.height + 7) // 8) * a.spp
        cam = {"share": {k: round(v / tot, 4) for k, v in ph.items()},
               "wave_cycles_per_tile": {k: round(v / tiles, 1) for k, v in ph.items()},
               "node_steps_per_tile": round(r["node_iters"] / tiles, 3), "leaf_visits_per_tile": round(r["scan"] / tiles, 3),
               "cycles_per_node_step": round(ph["node_steps"] / max(r["node_iters"], 1), 1),
               "cycles_per_leaf_visit": round(ph["leaf_tests"] / max(r["scan"], 1), 1),
               "ms_shipped": p["extend_ms"], "ms_stamp_build": r["extend_ms"], "tiles": tiles}
    res = {"scene": os.path.relpath(a.scene, ROOT), "spp": a.spp, "L_idle": L_IDLE, "k_camera_phases": cam,
           "kernels": {"k_extend": kernel("k_extend", st1, prod, ebpc, a.simds, range(2, nit + 1)),
                       "k_shadow": kernel("k_shadow", st2, prod, sbpc, a.simds, range(1, nit + 1))},
           "note": "frac = node steps x loaded round trip / (resident waves x clock x shipped HIP-event time): the "
                   "share of the kernel's time its node chain's round trips explain with every resident wave "
                   "waiting (scripts/latency_roof.py)"}
    txt = json.dumps(res, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
