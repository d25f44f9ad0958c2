#!/usr/bin/env python3
"""mfx_sample under a rocprofv3 kernel + memory-copy trace (gpu_run step `sampletrace`): C2 at 64 spp,
two warm calls then three traced ones, banded (default) and unbanded (MFX_SAMPLE_BANDS=0) in one
process, with a 100 ms idle gap before each traced set; prints the host-clock ms per call. The
timeline of the last call of each set (k_resolve bands, mean kernels, D2H copies, the host's end) is
read from the trace by `--timeline DIR`."""
import csv
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run():
    import numpy as np
    from mafrixraytracing_amd.native import DEFAULT_SEED, NativeContext
    from mafrixraytracing_amd.scene_io import load_scene_file
    a = load_scene_file(os.path.join(ROOT, "scenes", "spot.xml"))
    frame = np.empty((a.width * a.height, 4))
    out = {}
    with NativeContext(a, seed=DEFAULT_SEED) as ctx:
        modes = {"banded": {}, "unbanded": {"MFX_SAMPLE_BANDS": "0"}}
        for b in (4, 8):
            for cs in (1, 2):
                modes[f"bands{b}_streams{cs}"] = {"MFX_SAMPLE_BANDS": str(b), "MFX_SAMPLE_COPY_STREAMS": str(cs)}
                modes[f"bands{b}_streams{cs}_zerocopy"] = {"MFX_SAMPLE_BANDS": str(b), "MFX_SAMPLE_COPY_STREAMS": str(cs),
                                                           "MFX_SAMPLE_ZEROCOPY": "1"}
        if os.environ.get("SAMPLE_TRACE_SWEEP") != "1":
            modes = {k: modes[k] for k in ("banded", "unbanded")}
        for mode, env in modes.items():
            for k in ("MFX_SAMPLE_BANDS", "MFX_SAMPLE_COPY_STREAMS", "MFX_SAMPLE_ZEROCOPY"):
                os.environ.pop(k, None)
            os.environ.update(env)
            for _ in range(2):
                ctx.sample(64, out=frame)
            time.sleep(0.1)
            t = []
            for _ in range(3):
                t0 = time.perf_counter()
                ctx.sample(64, out=frame)
                t.append(round((time.perf_counter() - t0) * 1e3, 3))
            out[mode] = t
            time.sleep(0.1)
    print(json.dumps(out), flush=True)


def timeline(d):
    def rows(pat):
        f = sorted(glob.glob(os.path.join(d, "**", pat), recursive=True))
        return list(csv.DictReader(open(f[0]))) if f else []
    ev = []
    for r in rows("*kernel_trace.csv"):
        n = r["Kernel_Name"].replace("void ", "").split("(")[0].split("<")[0]
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n))
    for r in rows("*memory_copy_trace.csv"):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy:" + r.get("Direction", "?") + ":" +
                   str(round(int(r.get("Bytes", 0) or 0) / 1e6, 1)) + "MB"))
    ev.sort()
    # the last k_resolve launches of each traced set: print from 0.3 ms before the first resolve band
    res = [i for i, e in enumerate(ev) if e[2] == "k_resolve"]
    if not res:
        return
    sets, cur = [], [res[0]]
    for i in res[1:]:
        if ev[i][0] - ev[cur[-1]][1] > 5e6:
            sets.append(cur)
            cur = []
        cur.append(i)
    sets.append(cur)
    for s in sets[-8:]:
        t0 = ev[s[0]][0]
        end = max(e[1] for e in ev[s[0]:s[-1] + 40])
        print(f"--- resolve set of {len(s)} launches; from its start to the last event: {(end - t0) / 1e6:.3f} ms")
        for e in ev[s[0]:s[-1] + 40]:
            if e[0] - t0 > 5e6:
                break
            print(f"  {(e[0] - t0) / 1e6:8.3f} {(e[1] - t0) / 1e6:8.3f}  {e[2]}")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--timeline":
        timeline(sys.argv[2])
    else:
        run()
