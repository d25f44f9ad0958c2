"""The driver's multi-process composition on a real GPU (VERDICT r02 Next #1).

bench.py --gpus N runs one process per GPU under torch.distributed.run: each rank attaches a torch
device tensor as its context's accumulator (mfx_accum_attach), clears it, traces its sample
partition, waits for the context's stream and reduces over the process group
(distributed.native_partitioned_render). That replaces the reference's in-process fan-out
(Integrators.fs:164). A one-GPU box cannot run N > 1 ranks on N GPUs, so the sequence is pinned
here in the shapes it can take:
- a world-1 nccl (= RCCL) group: the whole attach / clear / trace / sync / reduce sequence with a
  real collective, bit-identical to a plain context's accumulator, for several frames;
- two ranks sharing device 0 over gloo with CUDA tensors (all_reduce): the reduced accumulator is
  bit for bit the two partitioned contexts' sum and matches the oracle;
- bench.py itself under torch.distributed.run with the multi-process path forced at world 1.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT, SEED

pytestmark = pytest.mark.gpu

W, H = 64, 36


def _free_port():
    """A port free now, outside the kernel's ephemeral range (32768-60999 by default): an ephemeral
    port released by this probe can be taken by any outgoing connection (RCCL / gloo bootstrap
    sockets) before the rendezvous binds it (r06h: EADDRINUSE)."""
    import random
    rng = random.Random()
    for _ in range(200):
        p = rng.randrange(20000, 30000)
        s = socket.socket()
        try:
            s.bind(("127.0.0.1", p))
            return p
        except OSError:
            continue
        finally:
            s.close()
    raise RuntimeError("no free port in 20000-30000")


def _plain_accumulators(name, frames, part_index=0, part_count=1):
    """Per frame (spp, base): a plain context's accumulator after clear + trace, as 3 x npix."""
    from conftest import scene
    from mafrixraytracing_amd.native import NativeContext
    a = scene(name, W, H)
    out = []
    with NativeContext(a, seed=SEED, part_index=part_index, part_count=part_count) as ctx:
        for spp, base in frames:
            ctx.accum_clear()
            ctx.trace_accumulate(spp, base)
            m = ctx.accum_read_mean(1.0)
            out.append(np.concatenate([m[:, c] for c in range(3)]))
    return out


def _rank_worker(rank, world, init, backend, name, frames, outdir, all_ranks, pipelined=False, rows=False,
                 nctx=1):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch
    import torch.distributed as dist

    from conftest import scene
    from mafrixraytracing_amd.abi import MFX_F_IN_FLIGHT, MFX_F_ROW_PARTITION
    from mafrixraytracing_amd.distributed import PipelinedNativeRender, RowGather, native_partitioned_render
    from mafrixraytracing_amd.native import NativeContext

    torch.cuda.set_device(0)
    dist.init_process_group(backend, init_method=init, rank=rank, world_size=world)
    a = scene(name, W, H)
    acc = torch.zeros(3 * W * H, dtype=torch.float64, device="cuda:0")
    gather = rows and backend == "nccl"  # (gloo has no CUDA gather: rows merge by all_reduce there)
    flags = (MFX_F_ROW_PARTITION if rows else 0) | (MFX_F_IN_FLIGHT if nctx > 1 else 0)
    ctxs = [NativeContext(a, seed=SEED, device=0, part_index=rank, part_count=world, flags=flags)
            for _ in range(nctx)]
    ctx = ctxs[0]
    try:
        got = []
        if pipelined:  # back to back, no waits between frames; the last B buffers checked after drain
            accs = [acc] + [torch.zeros_like(acc) for _ in range(max(2, nctx) - 1)]
            gs = [RowGather(b, W, H, rank, world) for b in accs] if gather else None
            pr = PipelinedNativeRender(ctxs if nctx > 1 else ctx, accs, rank, world, gathers=gs)
            for spp, base in frames:
                pr.frame(spp, base, all_ranks=all_ranks)
            pr.drain()
            got = [pr.buffer(k).cpu().numpy().copy() for k in range(len(frames) - len(accs), len(frames))]
            pr.close()
        else:
            pr = native_partitioned_render(ctx, acc, rank, world,
                                           exchange=RowGather(acc, W, H, rank, world) if gather else None)
            for spp, base in frames:
                pr.frame(spp, base, all_ranks=all_ranks)
                got.append(acc.cpu().numpy().copy())
            ctx.accum_attach(None)
    finally:
        for c in ctxs:
            c.close()
    if rank == 0:
        np.save(os.path.join(outdir, "frames.npy"), np.stack(got))
    dist.barrier()
    dist.destroy_process_group()


def _spawn(world, backend, name, frames, outdir, all_ranks, pipelined=False, rows=False, nctx=1):
    import torch.multiprocessing as mp
    # file rendezvous (no port to race for)
    init = "file://" + os.path.join(str(outdir), "pg_init")
    mp.start_processes(_rank_worker, args=(world, init, backend, name, frames, str(outdir), all_ranks,
                                           pipelined, rows, nctx),
                       nprocs=world, join=True, start_method="spawn")
    return np.load(os.path.join(outdir, "frames.npy"))


FRAMES = [(3, 0), (5, 3), (1, 8), (4, 9)]  # (spp, sample base) per frame: one-sample frames included


def test_world1_nccl_sequence_bit_identical(gpu, tmp_path):
    """World-1 RCCL group through native_partitioned_render: attach, clear, trace, sync, a real
    reduce, torch sync — the accumulator of every frame equals a plain context's bit for bit."""
    got = _spawn(1, "nccl", "spot", FRAMES, tmp_path, False)
    want = _plain_accumulators("spot", FRAMES)
    for k in range(len(FRAMES)):
        assert np.array_equal(got[k], want[k]), k


def test_world1_nccl_pipelined_frames_bit_identical(gpu, tmp_path):
    """The bench's pipelined form (PipelinedNativeRender: two attached accumulators, frame k's
    reduce on torch's stream overlapping frame k + 1's trace): frames run back to back with no host
    wait between them, and the last two buffers — each reused once — hold exactly the plain
    context's accumulators of their frames."""
    got = _spawn(1, "nccl", "spot", FRAMES, tmp_path, False, pipelined=True)
    want = _plain_accumulators("spot", FRAMES)
    for k in range(2):
        assert np.array_equal(got[k], want[len(FRAMES) - 2 + k]), k


@pytest.mark.parametrize("pipelined", [False, True])
def test_world1_nccl_row_gather_bit_identical(gpu, tmp_path, pipelined):
    """The bench's default exchange at world 1: MFX_F_ROW_PARTITION context, RowGather (pack, RCCL
    gather, unpack) per frame, plain and pipelined — every checked frame equals the plain context's."""
    got = _spawn(1, "nccl", "spot", FRAMES, tmp_path, False, pipelined=pipelined, rows=True)
    want = _plain_accumulators("spot", FRAMES)
    ks = range(len(FRAMES) - 2, len(FRAMES)) if pipelined else range(len(FRAMES))
    for i, k in enumerate(ks):
        assert np.array_equal(got[i], want[k]), k


@pytest.mark.parametrize("nctx", [2, 3])
def test_world1_nccl_frames_in_flight(gpu, tmp_path, nctx):
    """Frames alternating over two or three contexts (their own pools and streams, MFX_F_IN_FLIGHT's
    larger chunks: frames_in_flight), one buffer per context, row gather, pipelined: the last
    buffers equal the plain context's accumulators bit for bit."""
    got = _spawn(1, "nccl", "spot", FRAMES, tmp_path, False, pipelined=True, rows=True, nctx=nctx)
    want = _plain_accumulators("spot", FRAMES)
    nb = max(2, nctx)
    for i, k in enumerate(range(len(FRAMES) - nb, len(FRAMES))):
        assert np.array_equal(got[i], want[k]), k


def test_two_ranks_row_partition_gloo_merge_exact(gpu, tmp_path):
    """Two ranks sharing device 0, each tracing its tile rows (MFX_F_ROW_PARTITION, 36 rows = 5 tile
    rows, the last partial), pipelined, merged by gloo all_reduce: every merged accumulator is the
    whole-film context's bit for bit (a pixel is non-zero on one rank only)."""
    frames = [(2, 0), (3, 2), (1, 5), (2, 6)]
    got = _spawn(2, "gloo", "cube_cornell", frames, tmp_path, True, pipelined=True, rows=True)
    want = _plain_accumulators("cube_cornell", frames)
    for k in range(2):
        assert np.array_equal(got[k], want[len(frames) - 2 + k]), k


def test_two_ranks_pipelined_gloo_allreduce(gpu, tmp_path):
    """Two ranks sharing device 0, pipelined frames, gloo all_reduce: the last two frames' buffers are
    the sums of the two partitioned contexts' accumulators."""
    frames = [(2, 0), (3, 2), (1, 5), (2, 6)]
    got = _spawn(2, "gloo", "cube_cornell", frames, tmp_path, True, pipelined=True)
    p0 = _plain_accumulators("cube_cornell", frames, 0, 2)
    p1 = _plain_accumulators("cube_cornell", frames, 1, 2)
    for k in range(2):
        j = len(frames) - 2 + k
        assert np.array_equal(got[k], p0[j] + p1[j]), k


def test_two_ranks_on_one_device_gloo_allreduce(gpu, oracle, tmp_path):
    """Two ranks sharing device 0, gloo all_reduce on CUDA tensors: the reduced accumulator is the
    sum of the two partitioned contexts' (a0 + a1, exact for two terms in either order), and the
    image is within 1e-12 of the oracle's whole sample set."""
    frames = [(4, 0), (3, 4)]
    got = _spawn(2, "gloo", "cube_cornell", frames, tmp_path, True)
    p0 = _plain_accumulators("cube_cornell", frames, 0, 2)
    p1 = _plain_accumulators("cube_cornell", frames, 1, 2)
    from conftest import scene
    o = oracle.OracleScene(scene("cube_cornell", W, H))
    npix = W * H
    for k, (spp, base) in enumerate(frames):
        assert np.array_equal(got[k], p0[k] + p1[k]), k
        ref = o.sample(spp, SEED, sample_base=base)
        img = np.stack([got[k][c * npix:(c + 1) * npix] for c in range(3)], 1) / spp
        assert np.abs(img - ref[:, :3]).max() <= 1e-12, k


def test_bench_multiprocess_path_under_torchrun(gpu, tmp_path):
    """bench.py under torch.distributed.run (the driver's launch) with the multi-process path
    forced at world 1: process group, attached accumulator and RCCL reduce in the timed step; one
    JSON line with the metric, and the same ray count as the plain single-process run."""
    env = dict(os.environ, MFX_BENCH_FORCE_DIST="1")
    common = ["--steps", "2", "--warmup", "1", "--spp", "2", "--no-cpu-baseline", "--no-stats", "--no-render-api"]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py")] + common
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    r1 = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + common, capture_output=True, text=True,
                        timeout=300, cwd=ROOT)
    assert r1.returncode == 0, r1.stderr[-3000:]
    plain = json.loads(r1.stdout.strip().splitlines()[-1])
    assert line["metric"] == plain["metric"] and line["n_gpus"] == 1
    assert "process group" in line["config"]["parallelism"]
    # the forced multi-process path checks its merged frame too (world 1 over RCCL)
    assert line["merged_equals_1gpu"] is True and line["verify"]["exact_expected"] is True
    assert line["topology"]["rccl_world"] == 1 and line["topology"]["backend"] == "nccl"
    # rays per step are a property of the sample set: equal whichever path traced it
    assert line["rays_per_step"] == plain["rays_per_step"] > 0


def _bench(args, env=None, torchrun=0):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py")] + args
    if torchrun:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={torchrun}",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port())] + cmd[1:]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_bench_two_ranks_rehearsal_under_torchrun(gpu):
    """The driver's N-GPU launch rehearsed on one GPU: bench.py under torch.distributed.run with 2
    ranks, both on device 0 over gloo (MFX_BENCH_DEVICE / MFX_BENCH_BACKEND; RCCL refuses two ranks
    on one device). The whole world > 1 path runs — the image partition, pipelined frames and row
    merges, the barrier, max-over-ranks timing, the rays summed over ranks — and the line reports 2
    GPUs, strong scaling of the metric's job (the config's spp over the whole film, each rank half of
    the rows) with the rays of a 1-rank run of that job; the weak sub-object has the rays of the 2x
    larger sample set."""
    common = ["--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--no-stats", "--no-render-api"]
    env = dict(os.environ, MFX_BENCH_DEVICE="0", MFX_BENCH_BACKEND="gloo")
    line = _bench(["--spp", "2"] + common, env=env, torchrun=2)
    assert line["n_gpus"] == 2 and line["scaling"] == "strong"
    assert line["config"]["global_spp_per_step"] == 2 and line["config"]["film_share_per_gpu"] == 0.5
    assert "image partition" in line["config"]["parallelism"]
    one = _bench(["--spp", "2"] + common)
    assert line["rays_per_step"] == one["rays_per_step"] > 0
    # the line proves its own merge: the 2-rank frame is the 1-GPU frame bit for bit
    assert line["merged_equals_1gpu"] is True and line["verify"]["max_abs_diff"] == 0.0
    assert line["verify"]["digest_merged"] == line["verify"]["digest_1gpu"]
    topo = line["topology"]
    assert topo["rccl_world"] == 2 and topo["backend"] == "gloo" and topo["rank_devices"] == [0, 0]
    assert topo["pinned_one_device"] is True
    wk = line["weak"]
    assert wk["scaling"] == "weak" and wk["global_spp_per_step"] == 4
    # the sub-object continues the sample sequence after the line's steps: a 1-rank run of the same
    # 4-spp-per-step job over the same samples (its first timed step at the same global sample) has
    # exactly its rays
    first = wk["first_timed_sample"]
    four = _bench(["--spp", "4", "--sample-base", str(first - 4 * 1)] + common)  # warmup 1 step of 4 spp
    assert wk["rays_per_step"] == four["rays_per_step"] > 0 and wk["value"] > 0


def test_bench_merge_check_catches_a_wrong_partition(gpu):
    """The merged-frame check is not vacuous: with rank 1 tracing rank 0's rows instead of its own
    (MFX_BENCH_FAULT=partition), the 2-rank line reports merged_equals_1gpu false."""
    common = ["--steps", "1", "--warmup", "1", "--spp", "2", "--no-cpu-baseline", "--no-stats", "--no-render-api"]
    env = dict(os.environ, MFX_BENCH_DEVICE="0", MFX_BENCH_BACKEND="gloo", MFX_BENCH_FAULT="partition")
    line = _bench(common, env=env, torchrun=2)
    assert line["merged_equals_1gpu"] is False and line["verify"]["max_abs_diff"] > 0
    assert line["verify"]["digest_merged"] != line["verify"]["digest_1gpu"]


def test_bench_single_process_device_list_rehearsal(gpu):
    """bench.py --single-process --gpus 2 on the one-GPU box (MFX_BENCH_DEVICE=0: the device list
    [0, 0]): the library's own image partition and merge in the timed step, the batch line and the
    Scene.Render line (--api render, render-ahead on the device list), each with the rays of the
    one-GPU run of the same job."""
    common = ["--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--no-stats", "--no-render-api"]
    env = dict(os.environ, MFX_BENCH_DEVICE="0")
    line = _bench(["--spp", "4", "--single-process", "--gpus", "2"] + common, env=env)
    one = _bench(["--spp", "4"] + common)
    assert line["n_gpus"] == 2 and line["scaling"] == "strong" and line["rays_per_step"] == one["rays_per_step"]
    assert line["merged_equals_1gpu"] is True
    topo = line["topology"]
    # a repeated device cannot form a communicator: the library merges by device-ordered adds
    assert topo["single_process_devices"] == [0, 0] and topo["communicators"] == 0
    assert topo["library_context"]["merge"] == "ordered_adds"
    ra = ["--spp", "8", "--api", "render", "--render-ahead", "4"]
    rl = _bench(ra + ["--single-process", "--gpus", "2"] + common, env=env)
    r1 = _bench(ra + common)
    assert rl["n_gpus"] == 2 and rl["rays_per_step"] == r1["rays_per_step"] > 0


def test_bench_two_ranks_on_two_devices_over_rccl(gpu):
    """the default multi-GPU exchange for real — bench.py under torch.distributed.run with
    2 ranks on 2 distinct devices, RowGather over RCCL (nccl) — merges to the 1-GPU frame bit for bit
    (the line's own merged_equals_1gpu check) on distinct devices. Needs 2 GPUs: skipped on the
    one-GPU box (the 2-rank gloo rehearsal above runs the same code path there)."""
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("needs 2 GPUs")
    common = ["--steps", "2", "--warmup", "1", "--spp", "2", "--no-cpu-baseline", "--no-stats", "--no-render-api"]
    env = {k: v for k, v in os.environ.items() if k not in ("MFX_BENCH_DEVICE", "MFX_BENCH_BACKEND")}
    line = _bench(common, env=env, torchrun=2)
    topo = line["topology"]
    assert topo["backend"] == "nccl" and topo["rccl_world"] == 2 and topo["distinct_devices"] is True
    assert line["merged_equals_1gpu"] is True and line["verify"]["exact_expected"] is True
    one = _bench(common)
    assert line["rays_per_step"] == one["rays_per_step"] > 0


def test_bench_single_process_two_devices(gpu):
    """The library's own multi-device path on 2 distinct GPUs (ncclCommInitAll: 2 communicators, RCCL
    reduce) merges to the 1-GPU frame bit for bit. Needs 2 GPUs (the [0, 0] rehearsal runs on one)."""
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("needs 2 GPUs")
    common = ["--steps", "2", "--warmup", "1", "--spp", "4", "--no-cpu-baseline", "--no-stats", "--no-render-api"]
    env = {k: v for k, v in os.environ.items() if k != "MFX_BENCH_DEVICE"}
    line = _bench(common + ["--single-process", "--gpus", "2"], env=env)
    topo = line["topology"]
    assert topo["single_process_devices"] == [0, 1] and topo["communicators"] == 2
    assert topo["library_context"]["merge"] == "rccl_reduce"
    assert line["merged_equals_1gpu"] is True
