#!/usr/bin/env python3
"""mfx_sample's rate in bench.py's process state (VERDICT r05 Next #6): the line's context traces its
timed steps, render_api runs, then bench.sample_api, per readback setting (MFX_SAMPLE_BANDS,
MFX_SAMPLE_COPY_STREAMS read per call), interleaved over two rounds. Prints one JSON line per run.
SAMPLE_PROBE_SETTINGS=name,...: only those settings; --lone: no bench state first (a process that
only samples); MFX_SAMPLE_TIMING=1 prints the host's per-piece arrival and copy times on stderr."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    from mafrixraytracing_amd.native import DEFAULT_RENDER_AHEAD, DEFAULT_SEED, NativeContext
    from mafrixraytracing_amd.scene_io import load_scene_file
    a = load_scene_file(bench.SPOT_SCENE)
    lone = "--lone" in sys.argv
    ctx = None
    if not lone:
        ctx = NativeContext(a, seed=DEFAULT_SEED)
        for k in range(25):
            ctx.accum_clear()
            ctx.trace_accumulate(64, k * 64)
        ctx.sync()
        bench.render_api(a, DEFAULT_SEED, 2 * DEFAULT_RENDER_AHEAD, render_ahead=DEFAULT_RENDER_AHEAD)
    settings = [("bands8_streams1", {"MFX_SAMPLE_BANDS": "8", "MFX_SAMPLE_COPY_STREAMS": "1"}),
                ("bands8_streams2", {"MFX_SAMPLE_BANDS": "8", "MFX_SAMPLE_COPY_STREAMS": "2"}),
                ("bands4_streams1", {"MFX_SAMPLE_BANDS": "4", "MFX_SAMPLE_COPY_STREAMS": "1"}),
                ("unbanded", {"MFX_SAMPLE_BANDS": "0"}),
                ("bands4_noprobe", {"MFX_SAMPLE_BANDS": "4", "MFX_COPY_PROBE": "1"}),
                ("bands4_fp32nodes", {"MFX_SAMPLE_BANDS": "4", "MFX_NODE_F32": "1"})]
    if os.environ.get("SAMPLE_PROBE_SETTINGS"):
        keep = os.environ["SAMPLE_PROBE_SETTINGS"].split(",")
        settings = [x for x in settings if x[0] in keep]
    for rd in range(2):
        for name, env in settings:
            for k in ("MFX_SAMPLE_BANDS", "MFX_SAMPLE_COPY_STREAMS", "MFX_COPY_PROBE", "MFX_NODE_F32"):
                os.environ.pop(k, None)
            os.environ.update(env)
            r = bench.sample_api(a, DEFAULT_SEED, 64)
            print(json.dumps({"round": rd, "setting": name, "lone": lone, "ms_per_call": r["ms_per_call"],
                              "trace_device_ms": r["trace_device_ms_per_call"],
                              "min": r["ms_per_call_min"], "median": r["ms_per_call_median"]}), flush=True)
    if ctx is not None:
        ctx.close()


if __name__ == "__main__":
    main()
