#!/usr/bin/env python3
"""A/B of one GPU's strong-scaling shares between library builds (build_ab_share/*.so by default): for
each build, in its own process, every rank r of PARTS traces its 1/PARTS share (MFX_F_ROW_PARTITION,
all spp samples of its tile rows) over NIF contexts for STEPS frames, as bench.py's strong_share does;
builds interleaved over ROUNDS. Prints per build and round the ranks' ms per frame and ray shares.
Usage: share_ab.py [--dir build_ab_share] [--parts 8] [--nif 3] [--steps 20] [--rounds 2] [--spp 64]"""
import argparse
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys, json, time, os
sys.path.insert(0, ROOT)
import mafrixraytracing_amd.abi as abi
abi._lib = abi.load_library(LIB, strict=False)
from mafrixraytracing_amd.native import NativeContext, DEFAULT_SEED
from mafrixraytracing_amd.scene_io import load_scene_file
a = load_scene_file(os.path.join(ROOT, "scenes", "spot.xml"))
ms, rays = [], []
for r in range(PARTS):
    cs = [NativeContext(a, seed=DEFAULT_SEED, flags=64 | (128 if NIF > 1 else 0), part_index=r, part_count=PARTS)
          for _ in range(NIF)]
    for c in cs:
        c.trace_accumulate(SPP, 0)
    for c in cs:
        c.sync(); c.ray_counts_total(reset=True)
    t0 = time.perf_counter()
    for k in range(STEPS):
        c = cs[k % NIF]
        c.accum_clear(); c.trace_accumulate(SPP, (k + 1) * SPP)
    for c in cs:
        c.sync()
    ms.append((time.perf_counter() - t0) / STEPS * 1e3)
    rays.append(sum(float(sum(c.ray_counts_total(reset=True)[:3])) for c in cs))
    for c in cs:
        c.close()
print(json.dumps({"ms": ms, "rays": rays}))
'''


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", default="build_ab_share")
    ap.add_argument("--parts", type=int, default=8)
    ap.add_argument("--nif", type=int, default=3)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--spp", type=int, default=64)
    a = ap.parse_args()
    libs = sorted(glob.glob(os.path.join(ROOT, a.dir, "*.so")))
    res = {os.path.basename(l): [] for l in libs}
    for rd in range(a.rounds):
        for l in libs:
            code = CHILD.replace("ROOT", repr(ROOT)).replace("LIB", repr(l)).replace("PARTS", str(a.parts)) \
                .replace("NIF", str(a.nif)).replace("STEPS", str(a.steps)).replace("SPP", str(a.spp))
            p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
            if p.returncode != 0:
                print(os.path.basename(l), "FAILED", p.stderr[-1500:], flush=True)
                continue
            d = json.loads(p.stdout.strip().splitlines()[-1])
            tot = sum(d["rays"])
            res[os.path.basename(l)].append(max(d["ms"]))
            print(os.path.basename(l), "round", rd, "rank ms", [round(x, 3) for x in d["ms"]], "slowest", round(max(d["ms"]), 3),
                  "mean", round(sum(d["ms"]) / len(d["ms"]), 3),
                  "ray shares", [round(r / tot * a.parts, 4) for r in d["rays"]], flush=True)
    print("SUMMARY slowest-rank ms", json.dumps({k: [round(x, 3) for x in v] for k, v in res.items()}))


if __name__ == "__main__":
    main()
