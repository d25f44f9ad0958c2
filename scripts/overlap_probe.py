#!/usr/bin/env python3
"""Does an exchange kernel or copy overlap the persistent trace kernels? (VERDICT r04 Next #3)

The bench pipelines frame k's exchange under frame k+1's trace. `k_extend` / `k_shadow` are
persistent grids sized to fill every CU, so an exchange that needs CUs (RCCL's reduce or gather
kernels, RowGather's pack/unpack) may wait for them. Measured on one GPU with the C2 workload's
strong share (the same trace a rank of an 8-GPU job runs): the trace alone; each side operation
alone (an FP64 add kernel over `--mb` MB, a device-to-device copy of that size, and RowGather's
pack + unpack of an 8-rank 1080p frame); and each side operation enqueued on a second stream 1 ms
after the trace started, with its completion time measured from its own start event, plus the
trace's time beside it. Prints one JSON object."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default=os.path.join(ROOT, "scenes", "spot.xml"))
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--parts", type=int, default=8, help="the trace is tile rows 0 mod parts (a rank's share)")
    ap.add_argument("--mb", type=float, default=49.8, help="side operation size (C2's FP64 accumulator: 49.8 MB)")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()

    import torch
    from mafrixraytracing_amd.abi import MFX_F_ROW_PARTITION
    from mafrixraytracing_amd.distributed import RowGather
    from mafrixraytracing_amd.native import DEFAULT_SEED, NativeContext
    from mafrixraytracing_amd.scene_io import load_scene_file

    arr = load_scene_file(a.scene)
    W, H = arr.width, arr.height
    dev = torch.device("cuda:0")
    n = int(a.mb * 1e6 / 8)
    x = torch.zeros(n, dtype=torch.float64, device=dev)
    y = torch.ones(n, dtype=torch.float64, device=dev)
    z = torch.empty_like(x)
    acc = torch.zeros(3 * W * H, dtype=torch.float64, device=dev)
    g = RowGather(acc, W, H, 0, a.parts)
    side = torch.cuda.Stream(device=dev)
    ops = {"add_kernel": lambda: x.add_(y), "d2d_copy": lambda: z.copy_(x),
           "rowgather_pack_unpack": lambda: (g.pack(acc), g.unpack(acc))}

    def alone(fn):
        ts = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(side):
                e0.record()
                fn()
                e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        return min(ts)

    out = {"scene": os.path.basename(a.scene), "spp": a.spp, "share": f"tile rows 0 mod {a.parts}",
           "side_mb": a.mb, "alone_ms": {}, "during_trace": {}}
    with NativeContext(arr, seed=DEFAULT_SEED, flags=MFX_F_ROW_PARTITION, part_index=0, part_count=a.parts) as ctx:
        ctx.trace_accumulate(a.spp, 0)
        ctx.sync()
        tt = []
        for k in range(a.reps):
            ctx.trace_accumulate(a.spp, (k + 1) * a.spp)
            tt.append(ctx.last_trace_ms())
        out["trace_alone_ms"] = min(tt)
        for name, fn in ops.items():
            out["alone_ms"][name] = alone(fn)
            lat, tr = [], []
            for k in range(a.reps):
                ctx.trace_accumulate(a.spp, (k + 10) * a.spp)  # enqueued, not waited for
                time.sleep(1e-3)  # the persistent grid is resident by now
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                with torch.cuda.stream(side):
                    e0.record()
                    fn()
                    e1.record()
                e1.synchronize()
                lat.append(e0.elapsed_time(e1))
                tr.append(ctx.last_trace_ms())
            out["during_trace"][name] = {"completion_ms": min(lat), "completion_ms_median": sorted(lat)[len(lat) // 2],
                                         "trace_ms": min(tr)}
    out["note"] = ("completion_ms: the side operation's own start-to-end time when enqueued 1 ms into the trace; "
                   "near alone_ms: it ran beside the persistent grid; near the rest of the trace: it waited for CUs")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
