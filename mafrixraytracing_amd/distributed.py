"""Multi-GPU composition across processes: one process per GPU, an image partition, one exchange.
This is the path `bench.py --gpus N` runs under torch.distributed.run.

Every (pixel, sample) path is independent (Integrators.fs:164-171), so rank r of W traces every
sample of the film's 8-pixel tile rows it owns — one of each W consecutive ones, serpentine
(tile_row_owner) — (mfx_options.flags MFX_F_ROW_PARTITION,
part_index / part_count) into an FP64 accumulator it owns, which stays +0.0 outside its rows. Every
pixel's sample-order sum runs on one rank, so the merged frame is the 1-rank frame bit for bit, and
the only exchange is moving each rank's rows to rank 0:
- `RowGather` (default over RCCL): each rank packs its rows (3 x w x its rows, 1/W of the buffer) and
  rank 0 gathers and unpacks them — 1/W of the accumulator per rank over its own xGMI link;
- `reduce_accumulator`: a sum-reduce of the whole [3][w*h] buffer, an exact merge too (a pixel is
  non-zero on one rank only); the form gloo's CUDA-tensor all_reduce can run (the one-GPU rehearsal).
(torch.distributed backend "nccl" == RCCL on ROCm.) The sample partition (part_index / part_count
without the flag: rank r traces samples s % W == r of the whole film) composes the same way with a
sum-reduce, which is exact only up to FP64 summation order.

(A single process can drive the same partition itself: a context over a device list,
mfx_options.devices, partitions tile rows over its devices and merges with the library's own RCCL
communicator — `bench.py --single-process`.)

`PartitionedRender` is the per-rank frame: clear, trace this rank's partition, wait for the
trace, exchange. `native_partitioned_render` wires it to a HIP context (`NativeContext`) whose
accumulator is the exchange buffer; the gloo tests drive the same classes with a CPU tracer.
"""
from __future__ import annotations

from typing import Callable

import numpy as np


def partition_samples(spp: int, rank: int, world: int) -> np.ndarray:
    """Sample indices (within one call of spp samples) that `rank` renders (sample partition)."""
    return np.arange(rank, spp, world, dtype=np.int64)


def tile_row_owner(t, world: int):
    """The rank that owns 8-pixel tile row t under the image partition (csrc/mfx_device.h
    band_tile_row): each group of `world` consecutive tile rows gives one row to every rank, in rank
    order in even groups and in reverse order in odd ones (serpentine, so a gradient of work down a
    group does not load one rank more than another)."""
    g, o = np.divmod(np.asarray(t, dtype=np.int64), world)
    return np.where(g % 2 == 0, o, world - 1 - o)


def partition_rows(height: int, rank: int, world: int) -> np.ndarray:
    """Film rows y that `rank` renders under the image partition: the rows of the 8-pixel tile rows
    it owns (tile_row_owner; MFX_F_ROW_PARTITION, and a device list's device g of G likewise)."""
    y = np.arange(height, dtype=np.int64)
    return y[tile_row_owner(y // 8, world) == rank]


def step_spp(config_spp: int, world: int, scaling: str) -> int:
    """Samples per pixel of one whole-job step: strong scaling keeps the job at config_spp (each
    GPU traces config_spp over its 1/world of the film), weak scaling keeps config_spp of a whole
    film per GPU (the job renders config_spp * world)."""
    if scaling == "weak":
        return config_spp * world
    if scaling == "strong":
        return config_spp
    raise ValueError(f"scaling must be 'weak' or 'strong', not {scaling!r}")


def reduce_accumulator(acc, dst: int = 0, all_ranks: bool = False):
    """Sum-reduce a rank's accumulator tensor (torch) across the process group, in place. A group of
    one rank still runs the collective (so a 1-GPU job exercises the N-GPU sequence); without a
    process group there is nothing to reduce."""
    import torch.distributed as dist
    if not dist.is_available() or not dist.is_initialized():
        return acc
    if all_ranks:
        dist.all_reduce(acc, op=dist.ReduceOp.SUM)
    else:
        dist.reduce(acc, dst=dst, op=dist.ReduceOp.SUM)
    return acc


class RowGather:
    """The image partition's exchange: rank r's rows of the [3][w*h] x-major accumulator (pixel =
    x * h + y) packed into a 3 x w x n buffer (n = the most rows any rank has, so every rank sends
    the same shape), gathered to rank 0 and unpacked there into its accumulator; rank 0's own rows
    stay in place. Rank 0's accumulator is then the whole frame; the other ranks' are unchanged.
    Packing and unpacking run on torch's current stream (after the trace, before the next clear)."""

    def __init__(self, acc, width: int, height: int, rank: int, world: int):
        import torch
        self.w, self.h, self.rank, self.world = width, height, rank, world
        rows = [partition_rows(height, r, world) for r in range(world)]
        self.n = [len(r) for r in rows]
        self.nmax = max(self.n)
        self.idx = [torch.as_tensor(r, device=acc.device) for r in rows]
        self.send = torch.zeros((3, width, self.nmax), dtype=acc.dtype, device=acc.device)
        self.recv = [torch.zeros_like(self.send) for _ in range(world)] if rank == 0 else None
        self.bytes_per_rank = [3 * width * n * acc.element_size() for n in self.n]

    def _view(self, acc):
        return acc[:3 * self.w * self.h].view(3, self.w, self.h)

    def pack(self, acc):
        n = self.n[self.rank]
        if n:
            self.send[:, :, :n].copy_(self._view(acc).index_select(2, self.idx[self.rank]))

    def unpack(self, acc):
        if self.rank != 0:
            return
        v = self._view(acc)
        for r in range(1, self.world):
            if self.n[r]:
                v.index_copy_(2, self.idx[r], self.recv[r][:, :, :self.n[r]])

    def __call__(self, acc, async_op: bool = False):
        """Pack, gather to rank 0 (async_op: return the work handle; unpack after it), unpack."""
        import torch.distributed as dist
        self.pack(acc)
        if not dist.is_available() or not dist.is_initialized():
            return None
        work = dist.gather(self.send, self.recv if self.rank == 0 else None, dst=0, async_op=async_op)
        if not async_op:
            self.unpack(acc)
        return work


class PartitionedRender:
    """One rank's share of a frame: clear, trace own partition into `acc`, wait, exchange.

    render_fn(acc, spp, sample_base, rank, world) traces; clear_fn() zeroes the accumulator
    (default acc.zero_()); sync_fn() waits for the trace before the exchange reads the buffer (a
    HIP context traces on its own stream, the exchange runs on torch's); exchange(acc) moves the
    partitions to rank 0 (default: the sum-reduce, `reduce_accumulator`; a `RowGather` for the
    image partition)."""

    def __init__(self, render_fn: Callable, acc, rank: int, world: int,
                 clear_fn: Callable | None = None, sync_fn: Callable | None = None, after_reduce: Callable | None = None,
                 exchange: Callable | None = None):
        self.render_fn = render_fn
        self.acc = acc
        self.rank = rank
        self.world = world
        self.clear_fn = clear_fn or acc.zero_
        self.sync_fn = sync_fn
        self.after_reduce = after_reduce
        self.exchange = exchange

    def frame(self, spp: int, sample_base: int, all_ranks: bool = False):
        self.clear_fn()
        self.render_fn(self.acc, spp, sample_base, self.rank, self.world)
        if self.sync_fn is not None:
            self.sync_fn()
        if self.exchange is not None:
            self.exchange(self.acc)
            out = self.acc
        else:
            out = reduce_accumulator(self.acc, 0, all_ranks)
        if self.after_reduce is not None:
            self.after_reduce()
        return out


def native_partitioned_render(ctx, acc, rank: int, world: int, exchange: Callable | None = None) -> PartitionedRender:
    """PartitionedRender over a HIP context: `acc` (a device tensor on the context's GPU, at least
    3*w*h doubles) becomes the context's accumulator (mfx_accum_attach), so the trace writes
    straight into the buffer the exchange reads. The context must render partition `rank` of
    `world` (rows with MFX_F_ROW_PARTITION and a RowGather exchange, or samples with the default
    sum-reduce). A context over a device list (mfx_options.devices) first merges its devices into the
    primary's accumulator with its own reduce (mfx_accum_reduce), so no device's rows are dropped.

    Stream order: clear and trace run on the context's HIP stream; sync_fn (mfx_sync) waits for
    them before the collective, which torch enqueues on its own stream; after_reduce waits for
    that stream, so the next frame's clear cannot overwrite the buffer while RCCL still reads it."""
    ctx.accum_attach(acc.data_ptr(), acc.numel() * acc.element_size())
    multi = len(getattr(ctx, "devices", [0])) > 1

    def render(a, spp, base, r, w):
        ctx.trace_accumulate(spp, base)
        if multi:
            ctx.accum_reduce()

    def sync_torch():  # the exchange ran on torch's stream
        import torch
        if acc.is_cuda:
            torch.cuda.synchronize(acc.device)

    return PartitionedRender(render_fn=render, acc=acc, rank=rank, world=world,
                             clear_fn=ctx.accum_clear, sync_fn=ctx.sync, after_reduce=sync_torch, exchange=exchange)


def frames_in_flight(width: int, height: int, spp: int, world: int, rows: bool = True) -> int:
    """Contexts a rank alternates frames over: 3 when its frame is at most 2^25 paths (one rank's
    image-partition share at 4 or more GPUs), else 1. Every persistent launch fills the GPU, so
    another context's launches (its own pool and stream) take CUs as the first one's blocks retire:
    the next frames' dense launches fill the previous frame's tails. The contexts are created with
    MFX_F_IN_FLIGHT (larger chunk fetches: the tails are covered). Measured on C2: two contexts, a 1/8
    share +8.5 %, 1/4 +2.3 %, 1/2 -2 %, the whole film -4 % (profiles/r05/r05i_frames_in_flight.json:
    two frames' working sets in one L2); three with MFX_F_IN_FLIGHT, the 1/8 share 4.55 -> 4.37 ms and
    the 1/4 share 8.82 -> 8.63 ms against two (profiles/r05/r05s_sweep_small_frames.txt)."""
    tr = (height + 7) // 8
    rows_per_rank = -(-tr // world) if rows else tr
    paths = ((width + 7) // 8) * rows_per_rank * 64 * spp
    import os
    small = int(os.environ.get("MFX_FRAMES_IN_FLIGHT", "3"))  # (an A/B knob: scripts/share_modes.py)
    return small if paths <= (1 << 25) else 1


class PipelinedNativeRender:
    """Frames over B >= 2 attached accumulators, so a frame's exchange overlaps the next frames'
    traces: frame k traces into accs[k % B] on the HIP stream of context ctxs[k % len(ctxs)]
    (len(ctxs) <= B); torch's stream waits for that trace (an event on the context stream, no host
    sync) and runs the exchange — a RowGather per buffer (image partition) or the sum-reduce; frame
    k + B reuses the buffer only after that exchange has finished (an event on torch's stream, waited
    on the host just before the buffer is cleared, while the GPU is still tracing the frames between).
    With several contexts (their own pools and streams: frames_in_flight) the next frames' traces run
    beside frame k's. Each frame is the same clear / trace / exchange as PartitionedRender.frame;
    only the waits move. drain() waits for every outstanding exchange; `buffer(k)` is where frame k's
    merged accumulator lands (on rank 0)."""

    def __init__(self, ctx, accs, rank: int, world: int, gathers: list | None = None):
        import torch
        self.ctxs = list(ctx) if isinstance(ctx, (list, tuple)) else [ctx]
        self.ctx = self.ctxs[0]
        self.accs = list(accs)
        self.nbuf = len(self.accs)
        assert self.nbuf >= max(2, len(self.ctxs)) and all(a.is_cuda for a in self.accs)
        self.gathers = gathers
        assert gathers is None or len(gathers) == self.nbuf
        self.rank, self.world = rank, world
        self.multi = len(getattr(self.ctx, "devices", [0])) > 1
        self.device = self.accs[0].device
        self.ctx_streams = [torch.cuda.ExternalStream(c.stream(), device=self.device) for c in self.ctxs]
        self.pending = [None] * self.nbuf
        self.k = 0

    def buffer(self, k: int):
        return self.accs[k % self.nbuf]

    def _wait(self, i: int):
        if self.pending[i] is not None:
            self.pending[i].synchronize()
            self.pending[i] = None

    def frame(self, spp: int, sample_base: int, all_ranks: bool = False):
        import torch
        import torch.distributed as dist
        i = self.k % self.nbuf
        ci = self.k % len(self.ctxs)
        self.k += 1
        acc = self.accs[i]
        ctx = self.ctxs[ci]
        self._wait(i)  # frame k - B's exchange has read this buffer
        ctx.accum_attach(acc.data_ptr(), acc.numel() * acc.element_size())
        ctx.accum_clear()
        ctx.trace_accumulate(spp, sample_base)
        if self.multi:
            ctx.accum_reduce()
        traced = torch.cuda.Event()
        traced.record(self.ctx_streams[ci])
        cur = torch.cuda.current_stream(self.device)
        cur.wait_event(traced)
        if self.gathers is not None:
            g = self.gathers[i]
            work = g(acc, async_op=True)
            if work is not None:
                work.wait()  # the current stream waits for the collective's stream (no host wait)
            g.unpack(acc)
        elif dist.is_available() and dist.is_initialized():
            work = (dist.all_reduce(acc, op=dist.ReduceOp.SUM, async_op=True) if all_ranks
                    else dist.reduce(acc, dst=0, op=dist.ReduceOp.SUM, async_op=True))
            work.wait()  # the current stream waits for the collective's stream (no host wait)
        done = torch.cuda.Event()
        done.record(cur)
        self.pending[i] = done
        return acc

    def drain(self):
        for i in range(self.nbuf):
            self._wait(i)
        for c in self.ctxs:
            c.sync()

    def close(self):
        self.drain()
        for c in self.ctxs:
            c.accum_attach(None)
