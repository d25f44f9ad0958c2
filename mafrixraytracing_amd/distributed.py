"""Multi-GPU composition: one process per GPU, disjoint sample partitions, one RCCL reduce.

Every (pixel, sample) path is independent (Integrators.fs:164-171), so rank r of W renders the
global samples s with s % W == r (mfx_options.part_index/part_count) into an FP64 accumulator it
owns; the only exchange is one sum-reduce of the [3][w*h] accumulator to rank 0 over RCCL
(torch.distributed backend "nccl" == RCCL on ROCm). The counter RNG is keyed on the global
sample index, so the W-rank image equals the 1-rank image up to FP64 summation order.

`render_fn` is the per-rank tracer; in production it drives the HIP context
(`native.NativeContext.trace_accumulate` writing straight into the reduce buffer), and the
gloo tests substitute a CPU function of the same signature to check the composition.
"""
from __future__ import annotations

from typing import Callable

import numpy as np


def partition_samples(spp: int, rank: int, world: int) -> np.ndarray:
    """Sample indices (within one call of spp samples) that `rank` renders."""
    return np.arange(rank, spp, world, dtype=np.int64)


def reduce_accumulator(acc, dst: int = 0, all_ranks: bool = False):
    """Sum-reduce a rank's accumulator tensor (torch) across the process group, in place."""
    import torch.distributed as dist
    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size() == 1:
        return acc
    if all_ranks:
        dist.all_reduce(acc, op=dist.ReduceOp.SUM)
    else:
        dist.reduce(acc, dst=dst, op=dist.ReduceOp.SUM)
    return acc


class PartitionedRender:
    """One rank's share of a frame: trace own partition into `acc`, then reduce to rank 0."""

    def __init__(self, render_fn: Callable, acc, rank: int, world: int):
        self.render_fn = render_fn
        self.acc = acc
        self.rank = rank
        self.world = world

    def frame(self, spp: int, sample_base: int, all_ranks: bool = False):
        self.acc.zero_()
        self.render_fn(self.acc, spp, sample_base, self.rank, self.world)
        return reduce_accumulator(self.acc, 0, all_ranks)
