#!/usr/bin/env python3
"""bench.py's strong_share in a fresh process (no other contexts, streams or torch allocations
before it) against the same call after a whole-film context has traced: per-rank share times.
Prints one JSON line per setting; run it with and without GPU_MAX_HW_QUEUES=8 in the environment."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
# (GPU_MAX_HW_QUEUES counts only from the environment the process starts with: set it outside)


def main():
    import bench
    from mafrixraytracing_amd.native import DEFAULT_SEED, NativeContext
    from mafrixraytracing_amd.scene_io import load_scene_file
    a = load_scene_file(bench.SPOT_SCENE)
    for mode in ("fresh", "after_whole_film"):
        ctx = None
        if mode == "after_whole_film":
            ctx = NativeContext(a, seed=DEFAULT_SEED)
            for k in range(3):
                ctx.trace_accumulate(64, k * 64)
            ctx.sync()
        sh = bench.strong_share(a, DEFAULT_SEED, 64, 11000.0, 31.0, steps=10)
        print(json.dumps({"mode": mode, "rank_ms": {n: v["rank_ms_per_step"] for n, v in sh["shares"].items()}}),
              flush=True)
        if ctx is not None:
            ctx.close()


if __name__ == "__main__":
    main()
