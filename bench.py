#!/usr/bin/env python3
"""Benchmark: Mrays/s (primary + secondary) of the path-tracing hot path on MI355X.

Workload (BASELINE.json configs[1]; --config C3/C4/C5 for the others):
scenes/spot.xml — spot (5,856 triangles)
on a floor quad under a quad light, 1920x1080, 64 samples per pixel, maxDepth 3.
A step = one frame: every GPU traces every sample of its disjoint set of the film's 8-pixel tile
rows (image partition: one of each N consecutive tile rows, serpentine, MFX_F_ROW_PARTITION) into an FP64 accumulator, then
(N > 1) the ranks' rows are gathered to GPU 0 (RowGather over RCCL: 1/N of the [3][w*h] buffer per
rank; the merged frame is the 1-GPU frame bit for bit).
  --scaling strong (default): the job renders the metric's 1080p x 64 spp, each GPU 1/N of the film;
  --scaling weak: 64 spp of a whole film per GPU (the N-GPU job renders 64*N spp); each N > 1 line
  carries the other scaling of the same job, measured in the same run, as a sub-object.
N > 1 runs one process per GPU under torch.distributed.run (the driver's launch;
mafrixraytracing_amd/distributed.py, RCCL through torch.distributed), or with --single-process
one process whose library context drives all N devices (mfx_options.devices: the same tile-row
partition, merged with the library's own RCCL communicator; the path the F# host binds).
--api render times the reference's real call pattern instead: Scene.Render = 1 spp per call,
mfx_render_rgba8(ctx, 1, buf) with the 8 MB RGBA8 readback, the config's spp calls per step.

Rays counted = primary + extension (closest-hit queries actually traced) + shadow rays, read
from the kernel's own counters. Inputs (scene, BVH) are resident in HBM before timing starts.

Extra objects on the JSON line:
  roofline      the dominant kernel of the wavefront pipeline (k_extend<false>: path start +
                closest-hit traversal; k_shadow<false>: shading + shadow-ray traversal; whichever
                takes the larger share of the step, the other in `other_kernel`) — algorithmic
                bytes per launch / its HIP-event duration vs HBM 8 TB/s; bytes per ray frozen in
                profiles/bray_fixture.json; traffic = PMC HBM bytes per launch
                (profiles/traffic_<scene>.json, scripts/profile_traffic.sh)
  render_api    (N = 1) the same workload through Scene.Render's call pattern: the config's spp
                calls of mfx_render_rgba8(ctx, 1, buf), each with film, post and readback
  cpu_baseline  the CPU oracle timed on this host on a bounded random sample of the same
                workload's paths (rank 0, N = 1 only): "strict" (the FP64 restatement of the
                reference algorithm; `value`) and "fast" (SAH BVH2, tMax culling, any-hit
                shadows), with the thread count, nproc and CPU model
  sample_api    (N = 1) mfx_sample: the trace, the mean kernel and the FP64 frame's readback
  strong_share  (N = 1) every rank's share of the strong job at N = 2, 4, 8 timed on this GPU in a
                fresh process (--strong-share-child), frames in flight as the N-GPU ranks keep
                them, the exchange's pack/unpack measured and its transfer modeled, and the
                predicted efficiency with and without the measured overlap

A rank whose frame is small rotates frames over three contexts (distributed.frames_in_flight,
MFX_F_IN_FLIGHT); their streams need hardware queues of their own, so bench.py runs with
GPU_MAX_HW_QUEUES=8 (relaunching itself as a child when the environment lacks it; under a profiler,
which has initialised the GPU before bench.py starts, it refuses instead: set it in the environment).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# Hardware queues per process. A rank keeps up to three contexts' streams in flight
# (distributed.frames_in_flight) beside torch's and RCCL's; with HIP's default of 4 queues two of
# them share one and serialize: C2's 1/8 share 4.59 instead of 4.26 ms per step in bench.py's
# strong_share (profiles/r05/r05zm_*, r05zo_*). The HIP runtime takes GPU_MAX_HW_QUEUES from the
# environment the process starts with (setting os.environ here is too late), so without it bench.py
# runs itself as a child process with GPU_MAX_HW_QUEUES=8 and exits with the child's code, before
# anything here touches the GPU (signals are forwarded). An explicit setting wins.
HW_QUEUES = "8"


def _relaunch_with_hw_queues():
    import signal
    env = dict(os.environ, GPU_MAX_HW_QUEUES=HW_QUEUES)
    child = subprocess.Popen([sys.executable] + sys.argv, env=env)
    for sig in (signal.SIGTERM, signal.SIGINT):
        signal.signal(sig, lambda s, f: child.send_signal(s))
    sys.exit(child.wait())

METRIC = "Mrays/s (primary+secondary) at 1080p/64spp; 1/2/4/8-GPU scaling"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
XGMI_LINK_GBS = 153.0  # one xGMI link of MI355X (7 per GPU): the exchange models move each rank's bytes over one link
SPOT_SCENE = os.path.join(ROOT, "scenes", "spot.xml")
# BASELINE.json configs: scene, spp per GPU per step at N = 1, label. C4 and C5 are
# 8-GPU configs; at N = 1 a step is one GPU's share of them (256/8 and 512/8 spp).
CONFIGS = {
    "C2": ("spot.xml", 64, "C2 spot (5856 tris) + floor/light stage"),
    "C3": ("cube_cornell.xml", 1024, "C3 Cube (12 tris) in the synthetic Cornell box"),
    "C4": ("renault.xml", 32, "C4 Renault12TL (36996 tris) + stage, per-GPU share of 256 spp over 8 GPUs"),
    "C5": ("spot16_instanced.xml", 64,
           "C5 spot x16 instanced (16 x 5856 tris; the library flattens it: its flat image fits the budget) + stage, "
           "per-GPU share of 512 spp over 8 GPUs"),
    "C5T": ("spot16_instanced.xml", 64,
            "C5 spot x16 instanced, two-level BVH forced (MFX_F_TWO_LEVEL) + stage, per-GPU share of 512 spp over 8 GPUs"),
    "C5F": ("spot16.xml", 64, "C5 scene flattened (93696 tris, one BVH) + stage, per-GPU share of 512 spp over 8 GPUs"),
}
CONFIG_FLAGS = {"C5T": 32}  # mafrixraytracing_amd.abi.MFX_F_TWO_LEVEL


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="C2", choices=sorted(CONFIGS),
                    help="BASELINE.json workload (C2 default: the metric's configuration)")
    ap.add_argument("--spp", type=int, default=None, help="samples per pixel per GPU per step (default: the config's)")
    ap.add_argument("--scene", default=None, help="scene file (default: the config's)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU-baseline time budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-stats", action="store_true", help="skip the traversal-counter pass")
    ap.add_argument("--megakernel", action="store_true", help="persistent megakernel instead of the wavefront")
    ap.add_argument("--scaling", default="strong", choices=["weak", "strong"],
                    help="strong: the config's spp per job, each GPU 1/N of the film; weak: config spp of a whole film per GPU")
    ap.add_argument("--partition", default="rows", choices=["rows", "samples"],
                    help="N > 1 ranks: rows = image partition + RowGather (default); samples = sample partition + sum-reduce")
    ap.add_argument("--single-process", action="store_true",
                    help="N > 1 from one process: one library context over N devices (its own RCCL reduce)")
    ap.add_argument("--render-ahead", type=int, default=0,
                    help="--api render: mfx_options.render_ahead (one-sample calls served from batches of K samples)")
    ap.add_argument("--api", default="batch", choices=["batch", "render"],
                    help="batch: mfx_trace_accumulate of the frame's spp; render: spp x mfx_render_rgba8(1)")
    ap.add_argument("--no-render-api", action="store_true", help="skip the render_api sub-measurement")
    ap.add_argument("--sample-base", type=int, default=0,
                    help="global sample index of the first warmup step's first sample (steps follow on)")
    ap.add_argument("--no-verify", action="store_true",
                    help="N > 1: skip the merged-frame check against one GPU (merged_equals_1gpu)")
    # internal: measure strong_share in this (fresh) process for the parent run's VALUE_1GPU, MS_1GPU
    ap.add_argument("--strong-share-child", nargs=2, type=float, default=None, help=argparse.SUPPRESS)
    return ap.parse_args()


def relaunch_distributed(args):
    """`python bench.py --gpus N` without torchrun: start torchrun as a child (before any GPU
    use in this process) and exit with its status."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def host_cpu():
    """(nproc, CPUs this process may run on, CPU model name)."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        allowed = len(os.sched_getaffinity(0))
    except AttributeError:
        allowed = os.cpu_count() or 1
    return os.cpu_count() or 1, allowed, model


def cpu_baseline(arrays, spp, seed, budget_s):
    """Oracle (port) on random (pixel, sample) paths of the same workload, time-boxed: "strict"
    (the reference algorithm) for `value`, then "fast" for half the budget.

    Threads: the job's CPU share. On the GPU box OMP_NUM_THREADS (16, the share of one GPU's
    job) is set and honoured — the box's rules forbid sizing a pool to the whole machine, whose
    nproc it reports. Without it, every CPU this process may run on. The per-thread rate and
    its linear extrapolation to nproc are reported beside it as an estimate."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    pyoracle.build()
    nproc, allowed, model = host_cpu()
    nthreads = int(os.environ.get("OMP_NUM_THREADS") or allowed)
    o = pyoracle.OracleScene(arrays)
    res = {}
    for mode, budget in (("strict", budget_s), ("fast", budget_s / 2)):
        rng = np.random.default_rng(7)
        rays = paths = 0.0
        t_total = 0.0
        batch = 20000
        while t_total < budget:
            px = rng.integers(0, arrays.width, batch)
            py = rng.integers(0, arrays.height, batch)
            sm = rng.integers(0, spp, batch)
            _, st = o.paths(px, py, sm, seed, nthreads=nthreads, mode=mode)
            rays += st[0] + st[1] + st[2]
            paths += st[3]
            t_total += st[7]
        res[mode] = (rays / t_total / 1e6, paths, rays, t_total)
    o.close()
    v, paths, rays, t = res["strict"]
    return {"value": round(v, 4), "unit": "Mrays/s", "cores": nthreads, "kind": "port",
            "strict": round(v, 4), "fast": round(res["fast"][0], 4),
            "nproc": nproc, "cpus_allowed": allowed, "model": model,
            "per_thread_strict": round(v / nthreads, 4),
            "nproc_estimate_strict": round(v / nthreads * nproc, 2),
            "sample": f"{int(paths)} random (pixel, sample) paths of the same {arrays.width}x{arrays.height}x{spp} workload "
                      f"({int(rays)} rays, {t:.1f} s), oracle/mfx_oracle.c strict FP64 restatement of the reference "
                      f"algorithm, OpenMP {nthreads} threads; fast = the same paths' integrator over a SAH BVH2 "
                      f"with tMax culling and any-hit shadows ({res['fast'][3]:.1f} s); nproc_estimate = "
                      f"per-thread rate x nproc (linear, not measured)"}


def render_api(arrays, seed, calls, devices=None, render_ahead=0, flags=0):
    """Scene.Render's call pattern (Scene.fs:331-333): `calls` x mfx_render_rgba8(ctx, 1, buf), each
    one 1-spp frame into the film, ACES/sqrt/RGBA8 post and the RGBA8 readback to host memory.
    Rays from the kernels' counters of every call; wall time per call by the host clock.
    render_ahead = K > 1: the context serves one-sample calls from batches of K samples
    (mfx_options.render_ahead); the warmup is one whole batch and `calls` a multiple of K, so the
    timed calls trace exactly the samples they consume."""
    import numpy as np
    from mafrixraytracing_amd.native import NativeContext
    ctx = NativeContext(arrays, seed=seed, devices=devices, render_ahead=render_ahead, flags=flags)
    if render_ahead > 1:  # whole batches; at least two, so the background batch is in steady state
        calls = max(2, calls // render_ahead) * render_ahead
    buf = np.empty(arrays.width * arrays.height * 4, dtype=np.uint8)
    import ctypes as C
    bp = buf.ctypes.data_as(C.POINTER(C.c_uint8))
    from mafrixraytracing_amd.abi import check
    for _ in range(render_ahead if render_ahead > 1 else 3):
        check(ctx.lib.mfx_render_rgba8(ctx._h, 1, bp), "mfx_render_rgba8")
    wall, dev, rays = [], [], 0.0
    for _ in range(calls):
        t0 = time.perf_counter()
        check(ctx.lib.mfx_render_rgba8(ctx._h, 1, bp), "mfx_render_rgba8")
        wall.append(time.perf_counter() - t0)
        r, sec = ctx.stats()
        rays += r
        dev.append(sec)
    ctx.close()
    total = sum(wall)
    return {"value": round(rays / total / 1e6, 2), "unit": "Mrays/s", "calls": calls,
            "ms_per_call": round(total / calls * 1e3, 4), "ms_per_call_min": round(min(wall) * 1e3, 4),
            "trace_device_ms_per_call": round(sum(dev) / calls * 1e3, 4),
            "rays_per_call": round(rays / calls, 1), "render_ahead": render_ahead,
            "ms_per_call_max": round(max(wall) * 1e3, 4),
            "includes": "per call: mfx_render_rgba8(ctx, 1, buf) = trace of 1 spp (all bounces), film add, "
                        "ACES/sqrt/RGBA8 post, 8 MB RGBA8 copy to pageable host memory, synchronize" +
                        (f"; render-ahead K = {render_ahead}: the calls take their frames from batches of "
                         f"{render_ahead} samples traced in one wavefront pass, their film add + post run ahead on "
                         "the GPU, and the next batch is traced in the background while one is served "
                         "(the call reporting a batch reports its rays and device time)" if render_ahead > 1 else "")}


def sample_api(arrays, seed, spp, calls=5, flags=0):
    """SURVEY §8(d)'s metric to the letter: Mrays/s over the wall time of mfx_sample(spp) — the trace,
    the mean and the FP64 x-major RGBA readback (66 MB at 1080p; on one device the last resolve runs in
    column bands, each band's mean and DMA overlapping the next band) — per call; `value` over all
    timed calls, the per-call min and median beside it."""
    from mafrixraytracing_amd.native import NativeContext
    import numpy as np
    frame = np.empty((arrays.width * arrays.height, 4))  # the Color[w,h] the integrator owns
    with NativeContext(arrays, seed=seed, flags=flags) as ctx:
        for _ in range(2):  # warmup (pool, staging and copy streams, first touch of the frame)
            ctx.sample(spp, out=frame)
        wall, rays, dev = [], 0.0, []
        for _ in range(calls):
            t0 = time.perf_counter()
            ctx.sample(spp, out=frame)
            wall.append(time.perf_counter() - t0)
            c = ctx.ray_counts()
            rays += c[0] + c[1] + c[2]
            dev.append(ctx.last_trace_ms())  # the call's kernels (HIP events), readback excluded
    tot = sum(wall)
    return {"value": round(rays / tot / 1e6, 2), "unit": "Mrays/s", "calls": calls, "spp": spp,
            "ms_per_call": round(tot / calls * 1e3, 3), "ms_per_call_min": round(min(wall) * 1e3, 3),
            "ms_per_call_median": round(sorted(wall)[calls // 2] * 1e3, 3),
            "trace_device_ms_per_call": round(sum(dev) / calls, 3),
            "includes": "per call: mfx_sample(ctx, spp, frame) = trace, mean, FP64 RGBA x-major readback "
                        "to pageable host memory (banded: overlapped with the last resolve), synchronize"}


SHARE_PROCESSES = 3  # fresh processes strong_share runs in (bench.py --strong-share-child)


def progress(what):
    """A line on stderr per phase (the JSON line alone goes to stdout): a long run shows it is alive."""
    print(f"bench.py: {what} ({time.strftime('%H:%M:%S')})", file=sys.stderr, flush=True)


def _hip_stream():
    """A non-blocking HIP stream on the current device, created through the HIP runtime directly."""
    import ctypes as C
    hip = C.CDLL("libamdhip64.so")
    s = C.c_void_p()
    if hip.hipStreamCreateWithFlags(C.byref(s), 1) != 0:  # hipStreamNonBlocking
        raise RuntimeError("hipStreamCreateWithFlags failed")
    return s.value


def combine_shares(runs, value_1gpu, ms_1gpu):
    """strong_share from several fresh processes (raw: no predictions yet): per N the process with the
    median slowest rank (its whole entry), plus every process's slowest rank and predictions and their
    spread, all against the N = 1 line's rate and step time."""
    for r in runs:
        for n, e in r["shares"].items():
            share_efficiency(e, int(n), value_1gpu, ms_1gpu)
    out = {"shares": {}, "processes": len(runs), "partition": runs[0]["partition"],
           "note": runs[0]["note"] + f"; measured in {len(runs)} fresh processes: per N the median process's entry, "
                                     "`processes_slowest_rank_ms` / `processes_predicted_efficiency` from each and "
                                     "`spread_over_processes` = (max - min) / median of their slowest ranks"}
    for n in runs[0]["shares"]:
        ent = sorted((r["shares"][n] for r in runs), key=lambda e: e["slowest_rank_ms"])
        med = dict(ent[len(ent) // 2])
        sl = [e["slowest_rank_ms"] for e in ent]
        med["processes_slowest_rank_ms"] = [r["shares"][n]["slowest_rank_ms"] for r in runs]
        med["processes_predicted_efficiency"] = [r["shares"][n]["predicted_efficiency"] for r in runs]
        med["processes_predicted_efficiency_pipelined"] = [r["shares"][n]["predicted_efficiency_pipelined"] for r in runs]
        med["spread_over_processes"] = round((max(sl) - min(sl)) / med["slowest_rank_ms"], 4)
        out["shares"][n] = med
    return out


def share_efficiency(e, n, value_1gpu, ms_1gpu):
    """The predictions of one N's share entry against the full frame's rate and time (the N = 1 line):
    predicted_efficiency = (t_1GPU / N) / (t_slowest_rank + the exchange), the exchange not overlapped;
    _pipelined: the exchange runs beside the next frame's trace (measured: it completes within that
    trace and the trace keeps its time), so a step is the slowest rank's trace slowed by the measured
    factor."""
    t_rank, t_ex, ov = e["slowest_rank_ms"], e["exchange_ms"], e["overlap_measured"]
    e["vs_full_step_rate"] = round(e["job_rays_per_step"] / n / (t_rank / 1e3) / 1e6 / value_1gpu, 4)
    e["predicted_efficiency"] = round((ms_1gpu / n) / (t_rank + t_ex), 4)
    e["predicted_efficiency_per_repeat"] = [round((ms_1gpu / n) / (t + t_ex), 4) for t in e["per_repeat_slowest_ms"]]
    e["predicted_efficiency_pipelined"] = round(
        (ms_1gpu / n) / (t_rank * max(1.0, ov["trace_ms_beside_it"] / ov["trace_ms_alone"]) +
                         (0.0 if ov["exchange_completion_ms"] < t_rank else t_ex)), 4)
    return e


def strong_share(arrays, seed, spp, value_1gpu=None, ms_1gpu=None, steps=8, flags=0, repeats=2):
    """Every rank's share of the strong-scaled job at N = 2, 4, 8 GPUs (the line's image partition),
    measured on this GPU: rank r traces all `spp` samples of the film's tile rows of band r of N
    (MFX_F_ROW_PARTITION). Each share is timed as a rank runs it (clear + trace + sync, the frame's
    fixed per-generation costs included); the slowest rank is the step's trace. The exchange is
    RowGather: its pack (the largest rank's rows) and rank 0's unpack of the others' are timed here
    (torch index kernels on this accumulator); the transfer is modeled as the largest sending rank's
    bytes over one xGMI link (every rank sends to rank 0 over its own link, in parallel).
    predicted_efficiency = (t_1GPU / N) / (t_slowest_rank + t_pack + t_transfer + t_unpack): the
    exchange not overlapped (the bench overlaps it with the next frame's trace; not counted here).
    Each rank's share is timed `repeats` times (its contexts kept, the steps run again) and its median
    taken (one run's 1/8 share varied by 7 % between runs); `spread` = (max - min) / median
    of the slowest rank's repeats, and the predictions from each repeat's slowest rank beside them."""
    import torch
    from mafrixraytracing_amd.abi import MFX_F_IN_FLIGHT, MFX_F_ROW_PARTITION
    from mafrixraytracing_amd.distributed import RowGather, frames_in_flight
    from mafrixraytracing_amd.native import NativeContext
    W, H = arrays.width, arrays.height
    acc = torch.zeros(3 * W * H, dtype=torch.float64, device="cuda")
    if os.environ.get("MFX_SHARE_TORCH_FIRST") == "1":  # (scripts/share_modes.py) torch's stream pools first
        torch.cuda.Stream()

    def timed(fn, reps=20):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps * 1e3

    def overlap(ctx, g, reps=3):
        """The exchange's pack + unpack enqueued on a second stream 1 ms into this rank's trace (the
        bench's pipelined frames): its completion time from its own start, and the trace's time
        beside it against alone (scripts/overlap_probe.py measures the same for other operations)."""
        # a HIP stream of its own, not torch's: torch.cuda.Stream() creates torch's stream pools (dozens of
        # streams), after which the HIP runtime maps the next contexts' streams onto shared hardware
        # queues and a rank's frames in flight serialize (r06k, scripts/share_queues.py: two queues for
        # three contexts, the 1/8 share 8 % slower)
        side = torch.cuda.ExternalStream(_hip_stream())
        lat, tr, al = [], [], []
        for k in range(reps):
            ctx.trace_accumulate(spp, (k + 20) * spp)
            al.append(ctx.last_trace_ms())
            ctx.trace_accumulate(spp, (k + 40) * spp)
            time.sleep(1e-3)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(side):
                e0.record()
                g.pack(acc)
                g.unpack(acc)
                e1.record()
            e1.synchronize()
            lat.append(e0.elapsed_time(e1))
            tr.append(ctx.last_trace_ms())
        return {"exchange_completion_ms": round(min(lat), 4), "trace_ms_beside_it": round(min(tr), 3),
                "trace_ms_alone": round(min(al), 3)}

    out = {}
    for n in (2, 4, 8):
        rank_ms, rank_rays, rank_reps = [], [], []
        ov = None
        nif = frames_in_flight(W, H, spp, n)  # the bench's rank alternates its frames over nif contexts
        for r in range(n):
            fl = flags | MFX_F_ROW_PARTITION | (MFX_F_IN_FLIGHT if nif > 1 else 0)
            cs = [NativeContext(arrays, seed=seed, flags=fl, part_index=r, part_count=n) for _ in range(nif)]
            for c in cs:
                c.trace_accumulate(spp, 0)  # the pool's first allocation, untimed
            for c in cs:
                c.sync()
                c.ray_counts_total(reset=True)
            reps, rays = [], 0.0
            for rp in range(repeats):
                t0 = time.perf_counter()
                for k in range(steps):  # back to back, as the bench's steps run
                    c = cs[k % nif]
                    c.accum_clear()
                    c.trace_accumulate(spp, (rp * steps + k + 1) * spp)
                for c in cs:
                    c.sync()
                reps.append((time.perf_counter() - t0) / steps * 1e3)
                for c in cs:
                    t = c.ray_counts_total(reset=True)
                    rays += t[0] + t[1] + t[2]
            rank_reps.append(reps)
            rank_ms.append(sorted(reps)[len(reps) // 2])
            rank_rays.append(rays / steps / repeats)
            if r == 0:
                ov = overlap(cs[0], RowGather(acc, W, H, 0, n))
            for c in cs:
                c.close()
        g0 = RowGather(acc, W, H, 0, n)
        t_pack = timed(lambda: g0.pack(acc))  # rank 0 holds the most rows: the largest pack
        t_unpack = timed(lambda: g0.unpack(acc))
        t_xfer = max(g0.bytes_per_rank[1:]) / (XGMI_LINK_GBS * 1e9) * 1e3
        t_rank = max(rank_ms)
        t_ex = t_pack + t_xfer + t_unpack
        job_rays = sum(rank_rays)
        slow = rank_reps[rank_ms.index(t_rank)]
        per_rep_slowest = [max(r[i] for r in rank_reps) for i in range(repeats)]
        out[str(n)] = {"film_share_per_gpu": round(1.0 / n, 6), "spp_per_gpu": spp, "frames_in_flight": nif,
                       "rank_ms_per_step": [round(t, 3) for t in rank_ms],
                       "rank_rays_rel": [round(r / (job_rays / n), 4) for r in rank_rays],
                       "slowest_rank_ms": round(t_rank, 3), "repeats": repeats,
                       "slowest_rank_repeats_ms": [round(t, 3) for t in slow],
                       "per_repeat_slowest_ms": [round(t, 4) for t in per_rep_slowest],
                       "spread": round((max(slow) - min(slow)) / t_rank, 4),
                       "imbalance": round(t_rank / (sum(rank_ms) / n), 4),
                       "mrays_per_s_per_gpu": round(job_rays / n / (t_rank / 1e3) / 1e6, 2),
                       "job_rays_per_step": job_rays,
                       "gather_ms": {"pack": round(t_pack, 4), "transfer_modeled": round(t_xfer, 4),
                                     "unpack": round(t_unpack, 4)},
                       "exchange_ms": t_ex,
                       "overlap_measured": ov}
        if value_1gpu:
            share_efficiency(out[str(n)], n, value_1gpu, ms_1gpu)
    return {"shares": out, "partition": "image: serpentine tile-row band r of N per rank (MFX_F_ROW_PARTITION), "
                                        "RowGather to rank 0",
            "note": "every rank's share of --scaling strong at N GPUs, measured on one GPU one after another, in a fresh "
                    "process (bench.py --strong-share-child); "
                    "the exchange's pack/unpack measured here, its transfer modeled at one xGMI link "
                    f"({XGMI_LINK_GBS:.0f} GB/s) per sending rank; predicted_efficiency counts the exchange in full "
                    "(not overlapped); predicted_efficiency_pipelined uses overlap_measured (rank 0's pack + unpack "
                    "on a second stream 1 ms into its trace: its completion time and the trace's time beside it)"}


def topology(ctx, use_dist, dist, backend, local, world, single_process):
    """Where the job ran: the process group (world, backend) and every rank's device (ordinal, and
    the device's UUID where torch reports one), or for one process the library context's device list
    and the RCCL communicators it created (mfx_device_info). One process per GPU must use distinct
    devices unless the one-GPU rehearsal (MFX_BENCH_DEVICE) pins them all to one: anything else fails."""
    out = {}
    if use_dist:
        import torch
        uid = None
        try:
            uid = str(torch.cuda.get_device_properties(local).uuid)
        except Exception:
            pass
        mine = {"device": local, "uuid": uid}
        allv = [None] * world
        dist.all_gather_object(allv, mine)
        devs = [(v["device"], v["uuid"]) for v in allv]
        distinct = len(set(devs)) == len(devs)
        pinned = os.environ.get("MFX_BENCH_DEVICE") is not None
        if not distinct and not pinned:
            raise RuntimeError(f"ranks share a device: {devs}")
        out.update({"rccl_world": dist.get_world_size(), "backend": dist.get_backend(), "requested_backend": backend,
                    "rank_devices": [d for d, _ in devs], "rank_device_uuids": [u for _, u in devs],
                    "distinct_devices": distinct, "pinned_one_device": pinned})
    info = ctx.device_info()
    out["library_context"] = info
    if single_process:
        out["single_process_devices"] = info["devices"]
        out["communicators"] = info["communicators"]
    return out


def verify_merge(arrays, ctx, ctxs, pr, accs, gathers, rank, world, local, backend, spp, mode, rows, single_process,
                 devices, npix):
    """One more frame of the line's job, untimed: traced as the timed steps trace it (every rank its
    partition, merged to rank 0 by the line's exchange; or the one-process context over its device
    list and the library's merge), then the same samples traced whole on one GPU by a fresh context.
    merged_equals_1gpu: the two FP64 accumulators are equal bit for bit (the image partition's claim).
    A sample partition merges sums in another order: exact equality is not expected there, and its
    max_abs_diff is reported. Every rank joins (collectives); rank 0 returns the result."""
    import hashlib
    import time as _t
    import torch
    from mafrixraytracing_amd.distributed import PipelinedNativeRender
    from mafrixraytracing_amd.native import DEFAULT_SEED, NativeContext
    vbase = 1 << 30  # a sample range no timed step used
    dev = devices[0] if single_process else local
    nbytes = 3 * npix * 8
    if pr is not None:
        pr.drain()
        pv = PipelinedNativeRender(ctxs[:1], accs[:2], rank, world, gathers=gathers[:2] if gathers else None)
        pv.frame(spp, vbase, all_ranks=backend == "gloo")
        pv.drain()
        merged = pv.buffer(0)
        import torch.distributed as dist
        dist.barrier()
    else:
        merged = torch.zeros(3 * npix, dtype=torch.float64, device=f"cuda:{dev}")
        ctx.accum_attach(merged.data_ptr(), nbytes)
        ctx.accum_clear()
        ctx.trace_accumulate(spp, vbase)
        ctx.accum_reduce()
        ctx.sync()
        ctx.accum_attach(None)
    if rank != 0:
        return None
    ref = torch.zeros(3 * npix, dtype=torch.float64, device=f"cuda:{dev}")
    t0 = _t.perf_counter()
    with NativeContext(arrays, seed=DEFAULT_SEED, device=dev, flags=mode) as rc:  # whole film, every sample
        rc.accum_attach(ref.data_ptr(), nbytes)
        rc.accum_clear()
        rc.trace_accumulate(spp, vbase)
        rc.sync()
        rc.accum_attach(None)
    ms = (_t.perf_counter() - t0) * 1e3
    torch.cuda.synchronize(dev)
    exact = bool(torch.equal(merged, ref))
    diff = float((merged - ref).abs().max().item())
    dig = lambda t: hashlib.blake2b(t.cpu().numpy().tobytes(), digest_size=8).hexdigest()
    image_part = rows or single_process
    return {"merged_equals_1gpu": exact, "exact_expected": bool(image_part), "max_abs_diff": diff,
            "digest_merged": dig(merged), "digest_1gpu": dig(ref), "spp": spp, "sample_base": vbase,
            "nonzero_pixels_1gpu": int((ref[:npix] != 0).sum().item()), "ms_1gpu_check": round(ms, 2),
            "note": "one more frame of the line's job after the timed steps (untimed), merged as the steps merge it, "
                    "against a fresh one-GPU context tracing the same samples of the whole film; FP64 accumulators "
                    "compared bit for bit (digest: blake2b-64 of their bytes)"}


def main():
    args = parse()
    # the JSON line is the only thing on stdout: libraries that print banners there (RCCL prints
    # its version at communicator creation) are sent to stderr instead
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    cfg_scene, cfg_spp, cfg_label = CONFIGS[args.config]
    if args.scene is None:
        args.scene = os.path.join(ROOT, "scenes", cfg_scene)
    if args.spp is None:
        args.spp = cfg_spp
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.strong_share_child is not None:  # a fresh process, as a rank's own process runs its share
        from mafrixraytracing_amd.native import DEFAULT_SEED
        from mafrixraytracing_amd.scene_io import load_scene_file
        share = strong_share(load_scene_file(args.scene), DEFAULT_SEED, args.spp, args.strong_share_child[0] or None,
                             args.strong_share_child[1] or None, steps=args.steps, flags=CONFIG_FLAGS.get(args.config, 0))
        print(json.dumps(share), file=json_out, flush=True)
        return
    if args.gpus > 1 and not args.single_process and "RANK" not in os.environ:
        sys.exit(relaunch_distributed(args))
    # strong_share: every rank's share of the N-GPU job timed on this GPU, each rank over the line's own
    # step count (its frames-in-flight pipeline fills and drains between the barriers, as an N-GPU
    # run's steps do), in SHARE_PROCESSES fresh processes started before this one touches the GPU, as a
    # rank's own process runs it alone on its GPU: started later, beside this process's contexts, a
    # third of the children ran every share 8 % slower (r06f: 4.82 / 4.46 / 4.82 ms at N = 8), started
    # from a process with no GPU context all nine agreed within 0.4 % (r06g, scripts/share_modes.py).
    # Never from a profiled process (the profiler initialised the GPU before this one started).
    share_runs = []
    # (the metric's configuration only: C3's 1024 spp in three fresh processes would take minutes)
    if (int(os.environ.get("WORLD_SIZE", "1")) == 1 and args.gpus == 1 and args.api == "batch" and not args.no_render_api
            and not args.megakernel and not _under_profiler() and args.config == "C2"):
        cmd = [sys.executable, os.path.abspath(__file__), "--config", args.config, "--scene", args.scene,
               "--steps", str(args.steps), "--strong-share-child", "0", "0"] + \
              (["--spp", str(args.spp)] if args.spp is not None else [])
        for _ in range(SHARE_PROCESSES):
            pc = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
            if pc.returncode != 0:
                raise RuntimeError("strong_share child failed: " + pc.stderr[-2000:])
            share_runs.append(json.loads(pc.stdout.strip().splitlines()[-1]))
            progress(f"strong_share process {len(share_runs)} of {SHARE_PROCESSES} done")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # Rehearsal of the N-rank job on a one-GPU box (tests/test_gpu_distributed.py): every rank on
    # device MFX_BENCH_DEVICE, the process group over MFX_BENCH_BACKEND (gloo: RCCL refuses two ranks
    # on one device). The driver's run sets neither: one GPU per rank, nccl (= RCCL).
    if os.environ.get("MFX_BENCH_DEVICE") is not None:
        local = int(os.environ["MFX_BENCH_DEVICE"])
    backend = os.environ.get("MFX_BENCH_BACKEND", "nccl")
    ngpu = args.gpus if args.single_process else world  # GPUs of the job
    if args.api == "render" and world > 1:
        sys.exit("--api render is one process (use --single-process for N > 1)")
    if args.single_process and world > 1:
        sys.exit("--single-process drives every GPU from one process: do not launch it under torchrun")
    # MFX_BENCH_FORCE_DIST=1: run the multi-process path (process group, attached torch accumulator,
    # RCCL reduce) even at world 1 — how tests/test_gpu_distributed.py runs the driver's N-GPU
    # sequence on a one-GPU box
    use_dist = world > 1 or os.environ.get("MFX_BENCH_FORCE_DIST") == "1"

    import numpy as np
    from mafrixraytracing_amd.abi import (MFX_F_COUNT_STATS, MFX_F_IN_FLIGHT, MFX_F_MEGAKERNEL, MFX_F_NONE,
                                          MFX_F_ROW_PARTITION, MFX_F_WAVEFRONT)
    from mafrixraytracing_amd.distributed import PipelinedNativeRender, RowGather, frames_in_flight, step_spp
    from mafrixraytracing_amd.native import DEFAULT_RENDER_AHEAD, DEFAULT_SEED, NativeContext
    from mafrixraytracing_amd.scene_io import load_scene_file

    dist = torch = None
    if use_dist:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group(backend=backend)  # nccl = RCCL over xGMI

    arrays = load_scene_file(args.scene)
    W, H = arrays.width, arrays.height
    npix = W * H
    # the whole job's spp per step (strong: the config's spp over the job; weak: per GPU)
    spp_step = step_spp(args.spp, ngpu, args.scaling)
    rows = args.partition == "rows"
    mode = (MFX_F_MEGAKERNEL if args.megakernel else MFX_F_NONE) | CONFIG_FLAGS.get(args.config, 0)
    # one process per GPU: rank r traces tile-row band r of N (image partition) or samples r mod N
    rank_mode = mode | (MFX_F_ROW_PARTITION if rows else 0)
    devices = None
    if args.single_process:  # one context over the device list (the library's own tile-row partition)
        devices = list(range(args.gpus))
        if os.environ.get("MFX_BENCH_DEVICE") is not None:  # the one-GPU rehearsal: every device is that one
            devices = [int(os.environ["MFX_BENCH_DEVICE"])] * args.gpus
    # one process per GPU: a rank whose frame is small (its share at 4+ GPUs) alternates its frames
    # over several contexts, frames in flight (distributed.frames_in_flight; MFX_F_IN_FLIGHT), for the
    # line's job and for the other scaling's job measured after it
    nif = frames_in_flight(W, H, spp_step, world, rows) if use_dist and args.api == "batch" else 1
    o_nif = (frames_in_flight(W, H, step_spp(args.spp, ngpu, "weak" if args.scaling == "strong" else "strong"),
                              world, rows) if use_dist and args.api == "batch" and ngpu > 1 else 1)
    nctx = max(nif, o_nif)
    if nctx > 1:
        rank_mode |= MFX_F_IN_FLIGHT
    # MFX_BENCH_FAULT=partition (tests only): rank r > 0 traces rank r - 1's partition, so one partition
    # is traced twice and one not at all: the merged-frame check must catch it
    part = max(0, rank - 1) if os.environ.get("MFX_BENCH_FAULT") == "partition" else rank
    ctx = NativeContext(arrays, seed=DEFAULT_SEED, device=local, flags=rank_mode, part_index=part, part_count=world,
                        devices=devices, render_ahead=args.render_ahead if args.api == "render" else 0)
    ctxs = [ctx] + [NativeContext(arrays, seed=DEFAULT_SEED, device=local, flags=rank_mode, part_index=part,
                                  part_count=world) for _ in range(nctx - 1)]

    def totals():  # the timed steps' rays, summed on the device over this rank's contexts
        t = np.zeros(16)
        for c in ctxs:
            t += c.ray_counts_total(reset=True)
        return t
    pr = None
    if use_dist:
        # attached accumulators (two, or one per context in flight): frame k's exchange runs while
        # the next frames trace. The image partition gathers each rank's rows to rank 0 (RCCL); gloo
        # (the one-GPU rehearsal, CUDA tensors) has no CUDA gather, so there the rows merge by
        # all_reduce (an exact sum too)
        accs = [torch.zeros(3 * npix, dtype=torch.float64, device=f"cuda:{local}") for _ in range(max(2, nctx))]
        gathers = [RowGather(a, W, H, rank, world) for a in accs] if rows and backend != "gloo" else None
        pr = PipelinedNativeRender(ctxs[:nif], accs, rank, world, gathers=gathers)
    # a context allocates its path pool in its first trace: the line's extra contexts trace one
    # untimed frame of its size now, so no allocation falls into a timed step
    for c in ctxs[1:nif]:
        c.trace_accumulate(spp_step, 0)
    rbuf = np.empty(npix * 4, dtype=np.uint8)  # Scene.Render's byte[w*h*4]

    def barrier():
        if pr is not None:
            pr.drain()  # every frame's exchange has finished
        if use_dist:
            dist.barrier()
            torch.cuda.synchronize()
        for c in ctxs:
            c.sync()

    def step(k):
        base = args.sample_base + k * spp_step
        if args.api == "render":  # Scene.Render x spp: 1 spp per call, film + post + readback
            for _ in range(spp_step):
                ctx.render_rgba8(1, out=rbuf)
        elif pr is not None:  # one process per GPU: trace own partition, gather (or reduce) via torch
            pr.frame(spp_step, base, all_ranks=backend == "gloo")  # (gloo reduces CUDA tensors with all_reduce)
        else:  # one GPU, or one context over the device list (the library's RCCL merge); no host wait:
            # steps run back to back on the context's stream(s), as a render loop enqueues them
            ctx.accum_clear()
            ctx.trace_accumulate(spp_step, base)
            if devices:
                ctx.accum_reduce()

    progress(f"{args.warmup} warmup + {args.steps} timed steps")
    for k in range(args.warmup):
        step(k)
    barrier()
    totals()  # the timed steps' rays: device-side totals, read after the final barrier
    t0 = time.perf_counter()
    rays = 0.0
    closest_rays = 0.0
    primary_rays = 0.0
    timings = []
    call_s = 0.0  # --api render: host time inside the render calls (counters are read between calls)
    for k in range(args.steps):
        if args.api == "render":
            for _ in range(spp_step):
                tc = time.perf_counter()
                ctx.render_rgba8(1, out=rbuf)
                call_s += time.perf_counter() - tc
                c = ctx.ray_counts()
                rays += c[0] + c[1] + c[2]
                closest_rays += c[0] + c[1]
                primary_rays += c[0]
                timings.append(ctx.trace_timing())
            continue
        step(args.warmup + k)  # enqueued; the steps run back to back (no per-step host read)
    barrier()
    elapsed = time.perf_counter() - t0
    if args.api == "render":
        elapsed = call_s
    else:
        c = totals()  # every timed step's counters, summed on the device
        rays, closest_rays, primary_rays = c[0] + c[1] + c[2], c[0] + c[1], c[0]
        # per-stage device times (HIP events around each launch) from two more steps of the same
        # workload, each read after it (the timed steps above carry no per-step host read)
        for k in range(2):
            step(args.warmup + args.steps + k)
            timings.append(ctx.trace_timing())
        barrier()

    def job_max_sum(el, ry):  # the slowest rank's time, the job's rays
        if not use_dist:
            return el, ry
        t = torch.tensor([el], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        r = torch.tensor([ry], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(r, op=dist.ReduceOp.SUM)
        return float(t.item()), float(r.item())

    elapsed, rays_all = job_max_sum(elapsed, rays)

    other = None
    if ngpu > 1 and args.api == "batch":
        # the same job under the other scaling, in the same run (barriers, max over ranks): strong
        # lines carry the weak job (the config's spp of a whole film per GPU), weak lines the strong
        # one (the config's spp split over the GPUs)
        o_scaling = "weak" if args.scaling == "strong" else "strong"
        o_spp = step_spp(args.spp, ngpu, o_scaling)
        po = pr
        if pr is not None:  # the other job's frames in flight, by its own frame size
            pr.drain()
            po = PipelinedNativeRender(ctxs[:o_nif], accs, rank, world, gathers=gathers)

        def other_step(k):
            base = args.sample_base + (args.warmup + args.steps) * spp_step + k * o_spp
            if po is not None:
                po.frame(o_spp, base, all_ranks=backend == "gloo")
            else:
                ctx.accum_clear()
                ctx.trace_accumulate(o_spp, base)
                ctx.accum_reduce()
        other_step(0)
        for c in ctxs[1:o_nif]:  # (the other job's extra contexts: their pools, untimed)
            c.trace_accumulate(o_spp, 0)
        if po is not None:
            po.drain()
        barrier()
        totals()
        ts = time.perf_counter()
        for k in range(args.steps):
            other_step(1 + k)
        if po is not None:
            po.drain()
        barrier()
        c = totals()
        o_el, o_rays = job_max_sum(time.perf_counter() - ts, c[0] + c[1] + c[2])
        other = {"scaling": o_scaling, "global_spp_per_step": o_spp,
                 "first_timed_sample": args.sample_base + (args.warmup + args.steps) * spp_step + o_spp,
                 "frames_in_flight": frames_in_flight(W, H, o_spp, world, rows) if use_dist else 1,
                 "spp_per_gpu": o_spp if rows else o_spp / ngpu,
                 "film_share_per_gpu": round(1.0 / ngpu, 6) if rows else 1.0,
                 "value": round(o_rays / o_el / 1e6, 2), "unit": "Mrays/s", "steps": args.steps,
                 "ms_per_step": round(o_el / args.steps * 1e3, 3), "rays_per_step": o_rays / args.steps,
                 "note": f"the same job {o_scaling}-scaled (whole-job Mrays/s), measured after the line's steps"}
    # N > 1 (and the forced multi-process path): the job's merged frame against the same samples traced
    # whole on one GPU, after every timed measurement (VERDICT r05 Next #2), and the topology it ran on
    verify = topo = None
    if ngpu > 1 or use_dist:
        topo = topology(ctx, use_dist, dist, backend, local, world, args.single_process)
        if args.api == "batch" and not args.no_verify:
            verify = verify_merge(arrays, ctx, ctxs, pr, accs if use_dist else None, gathers if use_dist else None,
                                  rank, world, local, backend, spp_step, mode, rows, args.single_process, devices, npix)
    stage_ms = {k: float(np.mean([t[k] for t in timings]))
                for k in ("total_ms", "camera_ms", "extend_ms", "camera_launches", "shadow_ms", "iterations", "launches",
                          "generations")}

    result = None
    # launches per timed unit: a step, or (--api render) one 1-spp call
    nt = args.steps * (spp_step if args.api == "render" else 1)
    if rank == 0:
        # traversal counters (separate, untimed pass at 1 spp of the same frame)
        stats = None
        if not args.no_stats:
            # per-ray counters: the camera rays' packet walk (k_camera) would count its union of
            # visits for every lane, so this pass traces them one ray per lane
            old = os.environ.get("MFX_CAMERA_PACKETS")
            os.environ["MFX_CAMERA_PACKETS"] = "0"
            with NativeContext(arrays, seed=DEFAULT_SEED, device=local, flags=MFX_F_COUNT_STATS | mode) as sc:
                sc.trace_accumulate(1, 10 ** 6)
                s = sc.ray_counts()
            if old is None:
                del os.environ["MFX_CAMERA_PACKETS"]
            else:
                os.environ["MFX_CAMERA_PACKETS"] = old
            # the camera-ray packets' own fetches (k_camera's bytes: each node and slot once per wave)
            pk = None
            if not args.megakernel and stage_ms["camera_launches"] > 0:
                # (a 1-spp call runs the megakernel unless the wavefront is pinned: k_camera must run)
                with NativeContext(arrays, seed=DEFAULT_SEED, device=local,
                                   flags=MFX_F_COUNT_STATS | MFX_F_WAVEFRONT | mode) as sc:
                    sc.trace_accumulate(1, 10 ** 6)
                    sp = sc.ray_counts()
                if sp[10] > 0:
                    pk = {"node_fetches_per_ray": sp[10] / sp[0], "slot_fetches_per_ray": sp[11] / sp[0]}
            rc, rs = s[0] + s[1], s[2]
            # closest-hit traversal counters in s[4..6], shadow in s[7..9]
            stats = {"closest": {"node_visits_per_ray": s[4] / rc, "cluster_visits_per_ray": s[5] / rc,
                                 "prim_tests_per_ray": s[6] / rc},
                     "shadow": {"node_visits_per_ray": s[7] / rs, "cluster_visits_per_ray": s[8] / rs,
                                "prim_tests_per_ray": s[9] / rs},
                     "all": {"node_visits_per_ray": (s[4] + s[7]) / (rc + rs),
                             "cluster_visits_per_ray": (s[5] + s[8]) / (rc + rs),
                             "prim_tests_per_ray": (s[6] + s[9]) / (rc + rs)},
                     "rays_per_path": (rc + rs) / s[0]}
            if pk:
                stats["camera_packets"] = pk

        def bytes_per_ray(c):
            # SURVEY.md §8d / DESIGN.md §7: 32 B per BVH2 node visit (internal or leaf), 36 B per
            # primitive test, 64 B ray record; priced from the frozen fixture when it has the scene
            return 32.0 * (c["node_visits_per_ray"] + c["cluster_visits_per_ray"]) + \
                36.0 * c["prim_tests_per_ray"] + 64.0

        fixture = None
        fx = os.path.join(ROOT, "profiles", "bray_fixture.json")
        sname = os.path.splitext(os.path.basename(args.scene))[0]
        if os.path.exists(fx):
            with open(fx) as f:  # an instanced scene is priced as its flat expansion (the same workload)
                fixture = json.load(f)["scenes"].get(sname.replace("_instanced", ""))

        roofline = None
        if stats is not None:
            tfile = os.path.join(ROOT, "profiles", f"traffic_{sname}.json")
            if sname == "spot":
                tfile = os.path.join(ROOT, "profiles", "traffic_spot_1080p.json")
            tdata = None
            if os.path.exists(tfile) and ngpu == 1 and args.api == "batch":
                with open(tfile) as f:
                    tdata = json.load(f)
                if tdata.get("spp", args.spp) != args.spp:
                    tdata = None  # profiled on another workload

            tdroof = None  # profiles/td_<scene>.json (scripts/pmc_td_roof.sh): the TD / L1 line-request roof
            tdfile = os.path.join(ROOT, "profiles", f"td_{sname}.json")
            if os.path.exists(tdfile) and ngpu == 1 and args.api == "batch" and not CONFIG_FLAGS.get(args.config):
                with open(tdfile) as f:
                    tdroof = json.load(f)

            def td_roofline(kname, kms, launches):
                """The bound these kernels sit under: vector-memory line requests. achieved = the PMC
                pass's TCP line lookups per launch over this run's HIP-event launch time; peak = the
                td_gather peak case's lookups per GPU clock x the clock the PMC pass ran at. A kernel's
                instances (in place / ray queues, MFX_RAY_QUEUE) are pooled: per launch = their sums over
                their launches, as the HIP-event average pools them."""
                if not tdroof:
                    return None
                base = kname.split("<")[0]
                ks = [kv for kk, kv in tdroof["kernels"].items() if kk.split("<")[0] == base]
                if not ks:
                    return None
                n = sum(kv.get("launches", 1.0) for kv in ks)
                tot = lambda f: sum(kv[f] * kv.get("launches", 1.0) for kv in ks)
                lines = tot("line_lookups_per_launch") / n
                clocks = tot("gpu_clocks_per_launch") if all("gpu_clocks_per_launch" in kv for kv in ks) else None
                ms = tot("ms_per_launch") if all("ms_per_launch" in kv for kv in ks) else None
                mhz = clocks / ms / 1e3 if clocks and ms else ks[0]["clock_mhz"]
                # busy share of the TDs, weighted by each instance's clocks
                busy = sum(kv["td_busy_frac"] * kv["gpu_clocks_per_launch"] * kv.get("launches", 1.0) for kv in ks) / clocks \
                    if clocks else ks[0]["td_busy_frac"]
                ach = lines / (kms / launches / 1e3) / 1e9
                peak = tdroof["peak"]["lines_per_clock"] * mhz * 1e6 / 1e9
                pass_frac = (lines * n / clocks) / tdroof["peak"]["lines_per_clock"] if clocks else ks[0]["frac_of_peak"]
                return {"bound": "td", "achieved": round(ach, 2), "peak": round(peak, 2),
                        "unit": "G line-lookups/s", "frac": round(ach / peak, 4),
                        "frac_pmc_pass": round(pass_frac, 4),
                        "td_busy_frac": round(busy, 4),
                        "td_busy_frac_peak_case": round(tdroof["peak"]["td_busy_frac"], 4),
                        "lines_per_launch": lines, "l2_reads_per_launch": tot("l2_reads_per_launch") / n,
                        "clock_mhz_pmc_pass": round(mhz, 1), "instances": len(ks),
                        "peak_case": tdroof["peak"]["case"],
                        "source": os.path.relpath(tdfile, ROOT) + " (scripts/pmc_td_roof.sh)"}

            latf = os.path.join(ROOT, "profiles", f"latency_{sname}.json")  # scripts/latency_roof.py
            lat = None
            if os.path.exists(latf) and ngpu == 1 and args.api == "batch" and not CONFIG_FLAGS.get(args.config):
                with open(latf) as f:
                    lat = json.load(f)
                if lat.get("spp", args.spp) != args.spp:
                    lat = None

            def latency_roofline(kname, kms, launches):
                """The per-lane kernels' latency roof (VERDICT r05 Next #3): the node steps per launch and
                the loaded round trip of a node step (L_step, s_memtime around the node loads) from the
                stamp builds' pass; achieved = node steps per resident wave per second over this run's
                HIP-event launch time, peak = clock / L_step (every wave waiting one round trip per
                step): frac = the share of the launch its node chain's round trips explain."""
                if not lat or kname.split("<")[0] not in lat["kernels"]:
                    return None
                kv = lat["kernels"][kname.split("<")[0]]
                waves = kv["waves_per_simd"] * 1024  # 256 CUs x 4 SIMDs
                ach = kv["node_steps_per_launch"] / waves / (kms / launches / 1e3) / 1e6
                return {"bound": "latency", "achieved": round(ach, 4), "peak": kv["peak"], "unit": kv["unit"],
                        "frac": round(ach / kv["peak"], 4), "frac_profile_run": kv["frac"],
                        "L_step_cycles": kv["L_step_cycles"], "L_idle_cycles": kv["L_idle_cycles"],
                        "loaded_over_idle": kv["loaded_over_idle"], "clock_mhz": kv["clock_mhz"],
                        "waves_per_simd": kv["waves_per_simd"], "node_steps_per_wave_launch":
                            round(kv["node_steps_per_launch"] / waves, 1),
                        "lat_share_stamp_build": kv["lat_share_stamp_build"],
                        "source": os.path.relpath(latf, ROOT) + " (scripts/latency_roof.py)"}

            def smem_roofline(kname, kms, launches):
                """k_camera's roof: scalar-memory instructions (SQ_INSTS_SMEM, the PMC pass of
                scripts/pmc_td_roof.sh) per launch over this run's HIP-event launch time, against
                scripts/ubench/sload's peak rate at the clock the pass ran at."""
                if not tdroof or "smem_peak" not in tdroof:
                    return None
                ks = [kv for kk, kv in tdroof["kernels"].items() if kk.split("<")[0] == kname and "smem_per_launch" in kv]
                if not ks:
                    return None
                kv = ks[0]
                mhz = kv["smem_gpu_clocks_per_launch"] / kv["smem_ms_per_launch"] / 1e3
                ach = kv["smem_per_launch"] / (kms / launches / 1e3) / 1e9
                peak = tdroof["smem_peak"]["smem_per_clock"] * mhz * 1e6 / 1e9
                return {"bound": "smem", "achieved": round(ach, 3), "peak": round(peak, 3),
                        "unit": "G scalar-load instructions/s", "frac": round(ach / peak, 4),
                        "frac_pmc_pass": round(kv["smem_frac_of_peak"], 4),
                        "smem_per_launch": kv["smem_per_launch"], "peak_case": tdroof["smem_peak"]["case"],
                        "source": os.path.relpath(tdfile, ROOT) + " (scripts/pmc_td_roof.sh)"}

            def kernel_roofline(kname, kms, krays, launches, bray):
                # per launch: (rays/launch * B/ray) / (ms/launch) == per-step totals
                achieved = krays * bray / (kms / 1e3) / 1e9
                traffic = None
                if tdata:  # rocprof names the instance: k_shadow<false> or k_shadow<false, SPILL, ...>;
                    # the instances' bytes pooled over their launches (in place / ray queues)
                    base = kname.split(">")[0]
                    ks = [kv for kk, kv in tdata.get("kernels", {}).items() if kk == kname or kk.startswith(base + ",")]
                    nl = sum(kv.get("launches_profiled", 1) for kv in ks)
                    if ks and nl:
                        traffic = sum(kv.get("hbm_bytes_per_launch", 0.0) * kv.get("launches_profiled", 1) for kv in ks) / nl
                return {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                        "traffic_note": "PMC HBM bytes per launch, an upper bound: FETCH_SIZE x2 (the gfx950 "
                                        "correction measured for wide streaming reads) is applied to these gathers "
                                        "too, and MALL hits count as fabric traffic" if traffic else None,
                        "td": td_roofline(kname, kms, launches),
                        "latency": latency_roofline(kname, kms, launches),
                        "kernel": kname, "launches_per_step": launches,
                        "avg_launch_ms": round(kms / launches, 4),
                        "bytes_per_ray": round(bray, 1), "bytes_per_ray_source":
                            "profiles/bray_fixture.json (frozen)" if fixture else "live counters",
                        "rays_per_launch": round(krays / launches, 1)}

            if args.megakernel or stage_ms["shadow_ms"] == 0:  # the megakernel ran (also: 1-spp calls)
                bray = bytes_per_ray(stats["all"])
                if fixture:
                    fc, fs = fixture["closest"], fixture["shadow"]
                    n_c, n_s = fixture["closest_rays"], fixture["shadow_rays"]
                    bray = (fc["B_ray"] * n_c + fs["B_ray"] * n_s) / (n_c + n_s)
                roofline = kernel_roofline("trace_kernel<false>", stage_ms["total_ms"], rays / nt, 1, bray)
            else:
                # the two wavefront kernels; the roofline object is the one with the larger share of
                # the step (the dominant kernel), the other is reported beside it
                # the wavefront's kernels: k_camera (each generation's camera rays as packets, flat
                # scenes), k_extend (the other closest-hit launches), k_shadow; each priced with its
                # own rays, launches and HIP-event time
                launches = stage_ms["launches"]
                cl = stage_ms["camera_launches"]
                bc = fixture["closest"]["B_ray"] if fixture else bytes_per_ray(stats["closest"])
                bs = fixture["shadow"]["B_ray"] if fixture else bytes_per_ray(stats["shadow"])
                ks = []
                b_cam = bc
                if cl > 0:
                    # k_camera's bytes are its packets' own fetches: per camera ray its
                    # share of the wave-uniform 128-B node steps and 80-B slot prefixes (scalar loads,
                    # once per wave), plus its state word read and hit point + state word written (32 B)
                    pkc = stats.get("camera_packets")
                    b_cam = (128.0 * pkc["node_fetches_per_ray"] + 80.0 * pkc["slot_fetches_per_ray"] + 32.0) if pkc else bc
                    kc = kernel_roofline("k_camera<false>", stage_ms["camera_ms"], primary_rays / nt, cl, b_cam)
                    kc["bytes_per_ray_source"] = ("packet fetch counters (mfx_ray_counts out[10], out[11], "
                                                  "MFX_F_COUNT_STATS pass)" if pkc else kc["bytes_per_ray_source"])
                    kc["td"] = None  # its nodes and slots do not pass the TD: the scalar-load roof is kc["smem"]
                    kc["latency"] = None  # (a packet walk: one wave-uniform chain, VALU-bound; the smem roof)
                    kc["smem"] = smem_roofline("k_camera", stage_ms["camera_ms"], cl)
                    kc["note"] = ("HBM index priced at the bytes the packets fetch (each node and slot once per wave, "
                                  "through the scalar cache); its binding roof is the scalar-load rate (smem)")
                    ks.append((stage_ms["camera_ms"], kc))
                ext_rays = (closest_rays - (primary_rays if cl > 0 else 0.0)) / nt
                ext_ms = stage_ms["extend_ms"] - stage_ms["camera_ms"]
                ks.append((ext_ms, kernel_roofline("k_extend<false>", ext_ms, ext_rays, launches - cl, bc)))
                ks.append((stage_ms["shadow_ms"], kernel_roofline("k_shadow<false>", stage_ms["shadow_ms"],
                                                                  (rays - closest_rays) / nt, launches, bs)))
                ks.sort(key=lambda x: -x[0])
                roofline = dict(ks[0][1])
                roofline["other_kernels"] = [k for _, k in ks[1:]]
                # the whole step priced with each kernel's own bytes per ray: camera rays at k_camera's
                # packet bytes when they ran as packets (pricing them at k_extend's 628 B
                # put this entry above 1), extension rays at the closest-hit figure, shadow rays at theirs
                cam_rays = primary_rays if cl > 0 else 0.0
                step_bytes = (cam_rays * b_cam + (closest_rays - cam_rays) * bc + (rays - closest_rays) * bs) / nt
                roofline["step"] = {"achieved": round(step_bytes / (stage_ms["total_ms"] / 1e3) / 1e9, 2),
                                    "frac": round(step_bytes / (stage_ms["total_ms"] / 1e3) / 1e9 / HBM_PEAK_GBS, 5),
                                    "note": "every kernel's algorithmic bytes (camera rays at k_camera's packet bytes, "
                                            "extension and shadow rays at the frozen fixture's) over the whole traced step"}
                # the same SURVEY §8(d) formula on this run's own traversal counters (BVH4 visits as
                # the kernels count them) instead of the frozen BVH2 fixture: what the bytes are now
                lc, ls = bytes_per_ray(stats["closest"]), bytes_per_ray(stats["shadow"])
                live_step = (cam_rays * b_cam + (closest_rays - cam_rays) * lc + (rays - closest_rays) * ls) / nt
                roofline["live_bytes_per_ray"] = {
                    "closest": round(lc, 1), "shadow": round(ls, 1), "camera_packets": round(b_cam, 1),
                    "step_achieved": round(live_step / (stage_ms["total_ms"] / 1e3) / 1e9, 2),
                    "step_frac": round(live_step / (stage_ms["total_ms"] / 1e3) / 1e9 / HBM_PEAK_GBS, 5),
                    "note": "32 B per node or leaf-cluster visit + 36 B per primitive test + 64 B per ray (SURVEY.md "
                            "§8d) on this run's MFX_F_COUNT_STATS counters (the kernels' BVH4 visits), not the "
                            "frozen BVH2 fixture"}
            roofline["note"] = ("the hbm entry is a speed index: SURVEY §8(d)'s algorithmic bytes of a frozen BVH2 walk "
                                "(profiles/bray_fixture.json) over the HIP-event launch time, kept comparable across rounds; "
                                "the bytes the kernels move are `traffic` (PMC) and live_bytes_per_ray; the roof that binds "
                                "the per-lane kernels is `latency` (their node chain's round trips; DESIGN.md §7)")
            roofline["stage_ms"] = {k: round(v, 3) for k, v in stage_ms.items()}
            roofline["counters"] = {g: ({k: round(v, 3) for k, v in d.items()} if isinstance(d, dict)
                                        else round(d, 4)) for g, d in stats.items()}
        value = rays_all / elapsed / 1e6
        rapi = sapi = share = None
        if ngpu == 1 and args.api == "batch" and not args.no_render_api and not args.megakernel:
            # the shipped binding's default (fsharp/Native.fs DefaultRenderAhead, native.Scene): Scene.Render
            # served from batches of DEFAULT_RENDER_AHEAD samples
            cf = CONFIG_FLAGS.get(args.config, 0)
            progress("render_api")
            rapi = render_api(arrays, DEFAULT_SEED, 2 * DEFAULT_RENDER_AHEAD, render_ahead=DEFAULT_RENDER_AHEAD, flags=cf)
            rapi["vs_batch"] = round(rapi["value"] / value, 4)
            rapi["binding_default"] = True
            # the same calls one sample at a time (render_ahead = 0)
            plain = render_api(arrays, DEFAULT_SEED, args.spp, flags=cf)
            plain["vs_batch"] = round(plain["value"] / value, 4)
            rapi["without_render_ahead"] = plain
            progress("sample_api")
            sapi = sample_api(arrays, DEFAULT_SEED, args.spp, flags=cf)
            sapi["vs_batch"] = round(sapi["value"] / value, 4)
            # the shares were measured before this process touched the GPU (share_runs, main's start)
            share = combine_shares(share_runs, value, elapsed / args.steps * 1e3) if share_runs else \
                {"skipped": "under a profiler" if _under_profiler() else "measured on the metric's configuration (C2)"}
        cpu = None
        if ngpu == 1 and not args.no_cpu_baseline:
            progress("cpu_baseline")
            cpu = cpu_baseline(arrays, args.spp, DEFAULT_SEED, args.cpu_seconds)
        if ngpu == 1 and use_dist:
            par = ("one GPU through the one-process-per-GPU path (process group, attached accumulators, reduce "
                   "overlapped with the next frame's trace)")
        elif ngpu == 1:
            par = "one GPU"
        elif args.single_process:
            par = (f"image partition x{ngpu} (serpentine tile-row bands), one process, the library's RCCL merge "
                   "(mfx_options.devices)")
        elif rows:
            par = (f"image partition x{ngpu} (a serpentine tile-row band per rank, MFX_F_ROW_PARTITION), one process per GPU, "
                   + ("rows gathered to rank 0 over RCCL (RowGather)" if backend != "gloo" else
                      "rows merged by gloo all_reduce (the one-GPU rehearsal)")
                   + "; frame k's exchange overlapped with frame k+1's trace")
        else:
            par = (f"sample-partition x{ngpu}, one process per GPU, RCCL reduce via torch.distributed "
                   "(frame k's reduce overlapped with frame k+1's trace)")
        image_part = ngpu > 1 and (rows or args.single_process)
        per_gpu = spp_step if image_part else spp_step / ngpu
        api = ("Scene.Render pattern: mfx_render_rgba8(ctx, 1, buf) x spp, readback included"
               if args.api == "render" else "mfx_trace_accumulate of the step's spp (inputs resident in HBM)")
        result = {
            "metric": METRIC, "value": round(value, 2), "unit": "Mrays/s", "n_gpus": ngpu,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "rays_per_step": rays_all / args.steps,
            "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None, "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": f"{cfg_label}, {W}x{H}, {spp_step} spp per step over {ngpu} GPU(s)",
                       "baseline_config": args.config,
                       "scene": os.path.relpath(args.scene, ROOT), "width": W, "height": H,
                       "spp_per_gpu": per_gpu, "global_spp_per_step": spp_step, "max_depth": 3,
                       "film_share_per_gpu": round(1.0 / ngpu, 6) if image_part else 1.0,
                       "frames_in_flight": nif,
                       "pipeline": "megakernel" if args.megakernel else "wavefront", "api": api,
                       "parallelism": par},
            "roofline": roofline, "render_api": rapi, "sample_api": sapi, "strong_share": share, "cpu_baseline": cpu,
        }
        if topo is not None:
            result["topology"] = topo
        if verify is not None:
            result["verify"] = verify
            result["merged_equals_1gpu"] = verify["merged_equals_1gpu"]
        if other is not None:
            result[other["scaling"]] = other
        print(json.dumps(result), file=json_out, flush=True)
    for c in ctxs:
        c.close()
    if use_dist:
        dist.barrier()
        dist.destroy_process_group()
    return result


def _under_profiler():
    """rocprofv3 (or another ROCm profiler) preloads a library that initialises the GPU before this
    script starts: a process it started must not start bench.py again."""
    if any(k.startswith(("ROCPROF", "ROCP_")) for k in os.environ):
        return True
    return "rocprof" in os.environ.get("LD_PRELOAD", "")


if __name__ == "__main__":
    if os.environ.get("GPU_MAX_HW_QUEUES") is None:
        if _under_profiler():
            sys.exit("bench.py: under a profiler GPU_MAX_HW_QUEUES must be set in the environment "
                     "(e.g. GPU_MAX_HW_QUEUES=8 rocprofv3 ... -- python3 bench.py); bench.py does not start "
                     "a copy of itself from a profiled process")
        _relaunch_with_hw_queues()
    main()
