"""Multi-rank composition on CPU: world_size 2 and 3 over gloo. Each rank renders its
partition into an FP64 accumulator — its tile rows (the image partition bench.py runs: RowGather to
rank 0) or its samples (a sum-reduce) — and rank 0's merged accumulator must equal the single-rank
image (the rows: bit for bit). The ranks run `native_partitioned_render` — the function bench.py's
multi-process path runs — over a stand-in context whose trace is the CPU oracle (the container has
no GPU), so the clear / trace / sync / exchange sequence tested is the bench's."""
import os
import sys

import numpy as np
import pytest

from conftest import ROOT, SEED

W, H, SPP = 20, 12, 5


class OracleContext:
    """Stand-in for NativeContext with the methods native_partitioned_render calls; its trace adds
    this rank's partition of the frame (global samples s = base + part_index mod part_count,
    mfx_trace_accumulate's contract) to the attached accumulator, with the CPU oracle."""

    def __init__(self, oscene, acc, part_index, part_count, rows=False):
        self.o, self.acc, self.pi, self.pc, self.rows = oscene, acc, part_index, part_count, rows
        self.calls = []

    def accum_attach(self, ptr, nbytes):
        assert ptr == self.acc.data_ptr() and nbytes == self.acc.numel() * 8
        self.calls.append("attach")

    def accum_clear(self):
        self.acc.zero_()
        self.calls.append("clear")

    def sync(self):
        self.calls.append("sync")

    def trace_accumulate(self, spp, base):
        import torch
        from mafrixraytracing_amd.distributed import partition_rows, partition_samples
        if self.rows:  # MFX_F_ROW_PARTITION: every sample of this rank's tile rows
            s = np.arange(spp, dtype=np.int64) + base
            ys = partition_rows(H, self.pi, self.pc)
        else:
            s = partition_samples(spp, self.pi, self.pc) + base
            ys = np.arange(H)
        px, py, ss = np.meshgrid(np.arange(W), ys, s, indexing="ij")
        out, _ = self.o.paths(px.ravel(), py.ravel(), ss.ravel(), SEED, nthreads=2)
        pix = (px.ravel() * H + py.ravel())
        npix = W * H
        acc_np = np.zeros(3 * npix)
        # per pixel in sample order (the kernels' k_resolve order): meshgrid's last axis is the sample
        for c in range(3):
            np.add.at(acc_np, c * npix + pix, out[:, c])
        self.acc += torch.from_numpy(acc_np)
        self.calls.append("trace")


def _worker(rank, world, init, outdir, rows):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch
    import torch.distributed as dist

    import pyoracle
    from conftest import scene
    from mafrixraytracing_amd.distributed import RowGather, native_partitioned_render

    dist.init_process_group("gloo", init_method=init, rank=rank, world_size=world)
    a = scene("spot", W, H)
    acc = torch.zeros(3 * W * H, dtype=torch.float64)
    ctx = OracleContext(pyoracle.OracleScene(a), acc, rank, world, rows=rows)
    ex = RowGather(acc, W, H, rank, world) if rows else None
    pr = native_partitioned_render(ctx, acc, rank, world, exchange=ex)
    for k, base in enumerate((7, 12)):  # two frames: the gather buffers are reused
        pr.frame(SPP, sample_base=base)
        if rank == 0:
            np.save(os.path.join(outdir, f"merged{k}.npy"), acc.numpy())
    assert ctx.calls == ["attach"] + ["clear", "trace", "sync"] * 2, ctx.calls
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,rows", [(2, False), (2, True), (3, True)])
def test_ranks_merge_to_the_single_rank_image(oracle, tmp_path, world, rows):
    """rows: the image partition with RowGather (12 rows = 2 tile rows, the second partial: with 3
    ranks one rank owns none) — rank 0's accumulator is the single-rank image bit for bit. Else the
    sample partition with a sum-reduce, within FP64 summation order."""
    import torch.multiprocessing as mp
    init = "file://" + str(tmp_path / "pg_init")  # file rendezvous: no port to race for
    mp.start_processes(_worker, args=(world, init, str(tmp_path), rows), nprocs=world, join=True, start_method="spawn")
    from conftest import scene
    o = oracle.OracleScene(scene("spot", W, H))
    npix = W * H
    for k, base in enumerate((7, 12)):
        acc = np.load(tmp_path / f"merged{k}.npy")
        ref = o.sample(SPP, SEED, sample_base=base)
        got = np.stack([acc[c * npix:(c + 1) * npix] for c in range(3)], 1) / SPP
        if rows:
            assert np.array_equal(got, ref[:, :3]), k
        assert np.abs(got - ref[:, :3]).max() < 1e-12, k


def test_partition_rows_cover_every_row_once():
    from mafrixraytracing_amd.distributed import partition_rows, tile_row_owner
    for h in (1, 8, 12, 37, 1080):
        for world in (1, 2, 3, 8):
            allr = np.concatenate([partition_rows(h, r, world) for r in range(world)])
            assert sorted(allr.tolist()) == list(range(h))
            for r in range(world):
                assert all(tile_row_owner(y // 8, world) == r for y in partition_rows(h, r, world))


def test_partition_covers_every_sample_once():
    from mafrixraytracing_amd.distributed import partition_samples
    for spp in (1, 7, 64):
        for world in (1, 2, 3, 8):
            allp = np.concatenate([partition_samples(spp, r, world) for r in range(world)])
            assert sorted(allp.tolist()) == list(range(spp))


def test_step_spp_weak_and_strong():
    from mafrixraytracing_amd.distributed import step_spp
    assert step_spp(64, 8, "weak") == 512 and step_spp(64, 1, "weak") == 64
    assert step_spp(64, 8, "strong") == 64
    assert step_spp(4, 8, "strong") == 4  # the image partition splits rows, not samples
    with pytest.raises(ValueError):
        step_spp(64, 2, "linear")


def test_frames_in_flight_policy():
    """Two contexts per rank exactly when a rank's frame is at most 2^25 paths: C2's 1080p x 64 spp
    share at 4 and 8 GPUs (profiles/r05/r05i_frames_in_flight.json: +2.3 %, +8.5 %), one context for
    the whole film and the half share (-4 %, -2 %)."""
    from mafrixraytracing_amd.distributed import frames_in_flight
    assert [frames_in_flight(1920, 1080, 64, n) for n in (1, 2, 4, 8)] == [1, 1, 3, 3]
    assert frames_in_flight(1920, 1080, 512, 8) == 1  # the weak job's share: 8x the paths
    assert frames_in_flight(1920, 1080, 64, 8, rows=False) == 1  # a sample partition keeps the whole film


def test_band_rows_match_the_library(tmp_path):
    """The kernels' band mapping (csrc/mfx_device.h band_tile_row / band_row_count, compiled here for
    the host) is the partition distributed.py gathers by: for every band count and film height each
    band's tile rows are exactly the rows tile_row_owner gives it, in increasing order, and the bands
    cover every tile row once."""
    import subprocess
    from mafrixraytracing_amd.distributed import tile_row_owner
    src = tmp_path / "bt.cpp"
    src.write_text('#include "mfx_device.h"\n#include <cstdio>\nint main() {\n'
                   '  for (int bc = 1; bc <= 9; ++bc) for (int tr = 0; tr <= 40; ++tr) for (int bi = 0; bi < bc; ++bi) {\n'
                   '    int n = band_row_count(bi, bc, tr); printf("%d %d %d", bc, tr, bi);\n'
                   '    for (int k = 0; k < n; ++k) printf(" %d", band_tile_row(bi, bc, k)); printf("\\n"); } }\n')
    exe = tmp_path / "bt"
    subprocess.run(["g++", "-std=c++17", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
                    "-I" + os.path.join(ROOT, "mafrixraytracing_amd", "csrc"), "-o", str(exe), str(src)], check=True)
    seen = {}
    for line in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.splitlines():
        v = [int(x) for x in line.split()]
        bc, tr, bi, rows = v[0], v[1], v[2], v[3:]
        want = [t for t in range(tr) if int(tile_row_owner(t, bc)) == bi]
        assert rows == want, (bc, tr, bi, rows, want)
        seen.setdefault((bc, tr), []).extend(rows)
    for (bc, tr), rows in seen.items():
        assert sorted(rows) == list(range(tr)), (bc, tr)
