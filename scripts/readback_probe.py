#!/usr/bin/env python3
"""Where mfx_sample's time beyond the trace goes (VERDICT r05 Next #6): on C2 (1080p, 64 spp) the
trace alone (mfx_trace_accumulate + sync), mfx_accum_read_mean (the mean kernel + the 66 MB x-major
FP64 frame's readback through the library's page-locked staging), the whole mfx_sample, and for
scale the raw rates: a device-to-host DMA of 66 MB into page-locked memory (torch) and a host copy of
66 MB from page-locked to pageable memory. Prints one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def best(fn, reps=5):
    fn()
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        t.append((time.perf_counter() - t0) * 1e3)
    return round(min(t), 3), round(sorted(t)[len(t) // 2], 3)


def main():
    import numpy as np
    from mafrixraytracing_amd.native import DEFAULT_SEED, NativeContext
    from mafrixraytracing_amd.scene_io import load_scene_file
    a = load_scene_file(os.path.join(ROOT, "scenes", "spot.xml"))
    spp = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    frame = np.empty((a.width * a.height, 4))
    out = {}
    with NativeContext(a, seed=DEFAULT_SEED) as ctx:
        def trace():
            ctx.accum_clear()
            ctx.trace_accumulate(spp, 0)
            ctx.sync()
        out["trace_ms"] = best(trace, 3)
        import ctypes as C
        fp = frame.ctypes.data_as(C.POINTER(C.c_double))
        out["accum_read_mean_ms"] = best(lambda: ctx.lib.mfx_accum_read_mean(ctx._h, float(spp), fp))
        out["sample_ms"] = best(lambda: ctx.sample(spp, out=frame), 3)
        os.environ["MFX_SAMPLE_BANDS"] = "0"  # the unbanded path: trace, then mean + staged readback
        out["sample_ms_unbanded"] = best(lambda: ctx.sample(spp, out=frame), 3)
        os.environ.pop("MFX_SAMPLE_BANDS")
        # host_readback's pieces x copy threads (read per call from the environment)
        sweep = {}
        for pieces, threads in ((4, 4), (8, 4), (8, 8), (8, 12), (4, 8), (8, 16)):
            os.environ["MFX_READBACK_PIECES"], os.environ["MFX_READBACK_THREADS"] = str(pieces), str(threads)
            sweep[f"{pieces}x{threads}"] = best(lambda: ctx.lib.mfx_accum_read_mean(ctx._h, float(spp), fp))[0]
        os.environ.pop("MFX_READBACK_PIECES")
        os.environ.pop("MFX_READBACK_THREADS")
        out["accum_read_mean_ms_pieces_x_threads"] = sweep
    import torch
    dev = torch.empty(a.width * a.height * 4, dtype=torch.float64, device="cuda")
    pin = torch.empty(dev.shape, dtype=torch.float64, pin_memory=True)
    page = np.empty(dev.shape[0])

    def dma():
        pin.copy_(dev, non_blocking=True)
        torch.cuda.synchronize()
    out["dma_66MB_to_pinned_ms"] = best(dma)
    pn = pin.numpy()
    out["host_copy_66MB_pinned_to_pageable_1thread_ms"] = best(lambda: np.copyto(page, pn))
    out["bytes"] = dev.numel() * 8
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
