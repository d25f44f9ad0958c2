#!/usr/bin/env python3
"""A context's trace time after other contexts came and went in the process (round 6: mfx_sample's
context traced C2 in 32.8-33.5 ms in two contexts of six, 30.5 ms in the others). With a long-lived
context beside them, as bench.py's line context: twelve contexts one after another, each 2 warm + 3
timed 64-spp traces (HIP-event device time). (Round 6 ran it with a finished context's pool kept for
the next one and freed, interleaved: all twelve 30.0-30.2 ms, r06final2.) One JSON line per context."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from mafrixraytracing_amd.native import DEFAULT_SEED, NativeContext
    from mafrixraytracing_amd.scene_io import load_scene_file
    a = load_scene_file(os.path.join(ROOT, "scenes", "spot.xml"))
    line = NativeContext(a, seed=DEFAULT_SEED)
    line.trace_accumulate(64, 0)
    line.sync()
    for i in range(12):
        with NativeContext(a, seed=DEFAULT_SEED) as c:
            ms = []
            for k in range(5):
                c.accum_clear()
                c.trace_accumulate(64, k * 64)
                c.sync()
                if k >= 2:
                    ms.append(round(c.last_trace_ms(), 3))
        print(json.dumps({"context": i, "trace_ms": ms}), flush=True)
    line.close()


if __name__ == "__main__":
    main()
