#!/usr/bin/env python3
"""A/B timing of libmafrix_rt variants (build_variants/*.so) on the bench workload, each in its own
process, interleaved over rounds (cdna_hip_programming.md §5.4 rule 24). MFX_AB_STATS=1 adds each
variant's per-ray node / leaf / primitive visits (one MFX_F_COUNT_STATS sample)."""
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
abi.load_library(LIB); abi._lib = abi.load_library(LIB)
from mafrixraytracing_amd.native import NativeContext, DEFAULT_SEED
from mafrixraytracing_amd.scene_io import load_scene_file
a = load_scene_file(SCENE)
ctx = NativeContext(a, seed=DEFAULT_SEED)
res = []
for k in range(STEPS + 1):
    ctx.accum_clear(); t = time.perf_counter(); ctx.trace_accumulate(SPP, k * SPP); ctx.sync(); dt = time.perf_counter() - t
    c = ctx.ray_counts(); ms = ctx.last_trace_ms(); tt = ctx.trace_timing()
    if k: res.append(((c[0] + c[1] + c[2]) / dt / 1e6, ms, tt["total_ms"] - tt["extend_ms"] - tt["shadow_ms"],
                      tt["camera_ms"], tt["extend_ms"] - tt["camera_ms"], tt["shadow_ms"]))
st = {}
if os.environ.get("MFX_AB_STATS") == "1":  # per-ray traversal work of one sample (per-lane camera rays)
    os.environ["MFX_CAMERA_PACKETS"] = "0"
    cs = NativeContext(a, seed=DEFAULT_SEED, flags=1)
    cs.trace_accumulate(1, 0); cs.sync(); c = cs.ray_counts()
    st = {"nodes/closest": c[4] / (c[0] + c[1]), "leaves/closest": c[5] / (c[0] + c[1]), "prims/closest": c[6] / (c[0] + c[1]),
          "nodes/shadow": c[7] / max(c[2], 1), "leaves/shadow": c[8] / max(c[2], 1), "prims/shadow": c[9] / max(c[2], 1)}
print(json.dumps({"mrays": [r[0] for r in res], "ms": [r[1] for r in res], "rest": [r[2] for r in res],
                  "stage": [[r[3], r[4], r[5]] for r in res], "stats": st}))
'''


def main():
    # MFX_AB_DIR: the directory of candidates (default build_variants/; build_ab/ keeps A/B builds apart
    # from the diagnostic and experiment builds)
    libs = sorted(glob.glob(os.path.join(ROOT, os.environ.get("MFX_AB_DIR", "build_variants"), "*.so")))
    scene = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "scenes", "spot.xml")
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    spp = int(sys.argv[3]) if len(sys.argv) > 3 else 64
    out = {os.path.basename(l): [] for l in libs}
    for r in range(rounds):
        for l in libs:
            code = CHILD.replace("ROOT", repr(ROOT)).replace("LIB", repr(l)).replace("SCENE", repr(scene)) \
                .replace("STEPS", str(min(20, max(2, 64 // spp)))).replace("SPP", str(spp))
            env = dict(os.environ)
            ef = l[:-3] + ".env"  # optional KEY=VALUE lines for this variant (e.g. MFX_CHUNK=1024)
            if os.path.exists(ef):
                for line in open(ef):
                    if "=" in line:
                        k, v = line.strip().split("=", 1)
                        env[k] = v
            p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, env=env)
            if p.returncode != 0:
                print(os.path.basename(l), "FAILED", p.stderr[-2000:], flush=True)
                continue
            d = json.loads(p.stdout.strip().splitlines()[-1])
            out[os.path.basename(l)] += d["mrays"]
            print(os.path.basename(l), "round", r, ["%.1f" % x for x in d["mrays"]], "ms", ["%.2f" % x for x in d["ms"]],
                  "rest ms (resolve + memsets)", ["%.3f" % x for x in d.get("rest", [])],
                  "camera/extend/shadow ms", ["/".join("%.2f" % y for y in x) for x in d.get("stage", [])], flush=True)
            if d.get("stats"):
                print(os.path.basename(l), "stats", {k: round(v, 3) for k, v in d["stats"].items()}, flush=True)
    print("SUMMARY", json.dumps({k: (max(v) if v else None) for k, v in out.items()}))


if __name__ == "__main__":
    main()
