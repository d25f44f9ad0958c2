"""Multi-GPU composition across processes: one process per GPU, disjoint sample partitions, one
RCCL reduce. This is the path `bench.py --gpus N` runs under torch.distributed.run.

Every (pixel, sample) path is independent (Integrators.fs:164-171), so rank r of W renders the
global samples s with s % W == r (mfx_options.part_index/part_count) into an FP64 accumulator it
owns; the only exchange is one sum-reduce of the [3][w*h] accumulator to rank 0 over RCCL
(torch.distributed backend "nccl" == RCCL on ROCm). The counter RNG is keyed on the global
sample index, so the W-rank image equals the 1-rank image up to FP64 summation order.

(A single process can drive the same partitions itself: a context over a device list,
mfx_options.devices, reduces with the library's own RCCL communicator — `bench.py
--single-process`.)

`PartitionedRender` is the per-rank frame: clear, trace this rank's partition, wait for the
trace, reduce. `native_partitioned_render` wires it to a HIP context (`NativeContext`) whose
accumulator is the reduce buffer; the gloo tests drive the same class with a CPU tracer.
"""
from __future__ import annotations

from typing import Callable

import numpy as np


def partition_samples(spp: int, rank: int, world: int) -> np.ndarray:
    """Sample indices (within one call of spp samples) that `rank` renders."""
    return np.arange(rank, spp, world, dtype=np.int64)


def step_spp(config_spp: int, world: int, scaling: str) -> int:
    """Samples per pixel of one whole-job step: weak scaling keeps config_spp per GPU (the job
    renders config_spp * world), strong scaling keeps the job at config_spp (each GPU renders
    about config_spp / world)."""
    if scaling == "weak":
        return config_spp * world
    if scaling == "strong":
        if config_spp < world:
            raise ValueError(f"strong scaling needs spp >= GPUs ({config_spp} < {world})")
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


class PartitionedRender:
    """One rank's share of a frame: clear, trace own partition into `acc`, wait, reduce to rank 0.

    render_fn(acc, spp, sample_base, rank, world) traces; clear_fn() zeroes the accumulator
    (default acc.zero_()); sync_fn() waits for the trace before the reduce reads the buffer (a
    HIP context traces on its own stream, the reduce runs on torch's)."""

    def __init__(self, render_fn: Callable, acc, rank: int, world: int,
                 clear_fn: Callable | None = None, sync_fn: Callable | None = None, after_reduce: Callable | None = None):
        self.render_fn = render_fn
        self.acc = acc
        self.rank = rank
        self.world = world
        self.clear_fn = clear_fn or acc.zero_
        self.sync_fn = sync_fn
        self.after_reduce = after_reduce

    def frame(self, spp: int, sample_base: int, all_ranks: bool = False):
        self.clear_fn()
        self.render_fn(self.acc, spp, sample_base, self.rank, self.world)
        if self.sync_fn is not None:
            self.sync_fn()
        out = reduce_accumulator(self.acc, 0, all_ranks)
        if self.after_reduce is not None:
            self.after_reduce()
        return out


def native_partitioned_render(ctx, acc, rank: int, world: int) -> PartitionedRender:
    """PartitionedRender over a HIP context: `acc` (a device tensor on the context's GPU, at least
    3*w*h doubles) becomes the context's accumulator (mfx_accum_attach), so the trace writes
    straight into the buffer RCCL reduces. The context must render partition `rank` of `world`.
    A context over a device list (mfx_options.devices) first sums its devices into the primary's
    accumulator with its own reduce (mfx_accum_reduce), so no device's samples are dropped.

    Stream order: clear and trace run on the context's HIP stream; sync_fn (mfx_sync) waits for
    them before the collective, which torch enqueues on its own stream; after_reduce waits for
    that stream, so the next frame's clear cannot overwrite the buffer while RCCL still reads it."""
    ctx.accum_attach(acc.data_ptr(), acc.numel() * acc.element_size())
    multi = len(getattr(ctx, "devices", [0])) > 1

    def render(a, spp, base, r, w):
        ctx.trace_accumulate(spp, base)
        if multi:
            ctx.accum_reduce()

    def sync_torch():  # the reduce ran on torch's stream
        import torch
        if acc.is_cuda:
            torch.cuda.synchronize(acc.device)

    return PartitionedRender(render_fn=render, acc=acc, rank=rank, world=world,
                             clear_fn=ctx.accum_clear, sync_fn=ctx.sync, after_reduce=sync_torch)


class PipelinedNativeRender:
    """Frames over two attached accumulators, so a frame's reduce overlaps the next frame's trace:
    frame k traces into accs[k % 2] on the context's HIP stream; torch's stream waits for that trace
    (an event on the context stream, no host sync) and runs the reduce; frame k + 2 reuses the
    buffer only after that reduce has finished (an event on torch's stream, waited on the host just
    before the buffer is cleared, while the GPU is still tracing frame k + 1). Each frame is the
    same clear / trace / reduce as PartitionedRender.frame; only the waits move. drain() waits for
    every outstanding reduce; `buffer(k)` is where frame k's reduced accumulator lands."""

    def __init__(self, ctx, accs, rank: int, world: int):
        import torch
        self.ctx = ctx
        self.accs = list(accs)
        assert len(self.accs) == 2 and all(a.is_cuda for a in self.accs)
        self.rank, self.world = rank, world
        self.multi = len(getattr(ctx, "devices", [0])) > 1
        self.device = self.accs[0].device
        self.ctx_stream = torch.cuda.ExternalStream(ctx.stream(), device=self.device)
        self.pending = [None, None]
        self.k = 0

    def buffer(self, k: int):
        return self.accs[k % 2]

    def _wait(self, i: int):
        if self.pending[i] is not None:
            self.pending[i].synchronize()
            self.pending[i] = None

    def frame(self, spp: int, sample_base: int, all_ranks: bool = False):
        import torch
        import torch.distributed as dist
        i = self.k % 2
        self.k += 1
        acc = self.accs[i]
        self._wait(i)  # frame k - 2's reduce has read this buffer
        self.ctx.accum_attach(acc.data_ptr(), acc.numel() * acc.element_size())
        self.ctx.accum_clear()
        self.ctx.trace_accumulate(spp, sample_base)
        if self.multi:
            self.ctx.accum_reduce()
        traced = torch.cuda.Event()
        traced.record(self.ctx_stream)
        cur = torch.cuda.current_stream(self.device)
        cur.wait_event(traced)
        if dist.is_available() and dist.is_initialized():
            work = (dist.all_reduce(acc, op=dist.ReduceOp.SUM, async_op=True) if all_ranks
                    else dist.reduce(acc, dst=0, op=dist.ReduceOp.SUM, async_op=True))
            work.wait()  # the current stream waits for the collective's stream (no host wait)
        done = torch.cuda.Event()
        done.record(cur)
        self.pending[i] = done
        return acc

    def drain(self):
        for i in (0, 1):
            self._wait(i)
        self.ctx.sync()

    def close(self):
        self.drain()
        self.ctx.accum_attach(None)
