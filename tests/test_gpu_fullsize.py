"""GPU parity at BASELINE.json's full film sizes (C2-C5: 1920x1080, spot16 at 3840x2160).

The oracle renders one sample per pixel of the full frame (all 2.07 M / 8.29 M paths) in a few
seconds on the host cores, so the comparison is per pixel against the CPU restatement, at a
non-zero global sample index: bit for bit. At the configs' full sample counts the size-independent
properties are checked instead: the wavefront and megakernel pipelines (independent traversal
and integrator schedules) produce identical ray counts and images equal up to FP64 summation
order, and sample partitions (the multi-GPU decomposition) sum to the whole.
"""
import numpy as np
import pytest

from conftest import SEED, scene

pytestmark = pytest.mark.gpu

FULL = ["spot", "cube_cornell", "renault", "spot16", "spot16_instanced@2l"]  # C2-C5 at their film sizes (C5 flat and two-level)


@pytest.mark.parametrize("name", FULL)
def test_full_frame_one_spp_matches_oracle(gpu, oracle, name):
    from mafrixraytracing_amd.native import NativeContext
    a = scene(name)
    base = 5  # global sample index 5: a mid-stream sample, not the first
    ref, st = oracle.OracleScene(a).sample(1, SEED, sample_base=base, with_stats=True)
    with NativeContext(a, seed=SEED) as ctx:
        ctx.accum_clear()
        ctx.trace_accumulate(1, base)
        img = ctx.accum_read_mean(1.0)
        counts = ctx.ray_counts()
    assert tuple(counts[:3]) == tuple(st[:3]), (counts[:3], st[:3])
    # every path's radiance is folded in the reference's recursion order: the frame is the oracle's bit for bit
    assert np.array_equal(img[:, :3], ref[:, :3]), np.abs(img[:, :3] - ref[:, :3]).max()


@pytest.mark.parametrize("name,spp", [("spot", 64), ("cube_cornell", 32), ("renault", 16), ("spot16", 4)])
def test_full_size_pipelines_agree(gpu, name, spp):
    from mafrixraytracing_amd.abi import MFX_F_MEGAKERNEL, MFX_F_NONE
    from mafrixraytracing_amd.native import NativeContext
    a = scene(name)
    out = {}
    for mode in (MFX_F_NONE, MFX_F_MEGAKERNEL):
        with NativeContext(a, seed=SEED, flags=mode) as ctx:
            ctx.accum_clear()
            ctx.trace_accumulate(spp, 0)
            out[mode] = (ctx.accum_read_mean(float(spp)), ctx.ray_counts()[:3].copy())
    (iw, cw), (im, cm) = out[MFX_F_NONE], out[MFX_F_MEGAKERNEL]
    assert np.array_equal(cw, cm), (cw, cm)
    assert np.abs(iw[:, :3] - im[:, :3]).max() <= 1e-12 * max(1.0, np.abs(im).max())


def test_full_size_partitions_sum_to_whole(gpu):
    from mafrixraytracing_amd.native import NativeContext
    a = scene("spot")
    spp, G = 8, 2
    with NativeContext(a, seed=SEED) as ctx:
        ctx.accum_clear()
        ctx.trace_accumulate(spp, 0)
        whole = ctx.accum_read_mean(1.0)
        cw = ctx.ray_counts()[:3].copy()
    total = np.zeros_like(whole)
    ct = np.zeros(3)
    for g in range(G):
        with NativeContext(a, seed=SEED, part_index=g, part_count=G) as ctx:
            ctx.accum_clear()
            ctx.trace_accumulate(spp, 0)  # spp is the global count; this partition renders spp / G of it
            total += ctx.accum_read_mean(1.0)
            ct += ctx.ray_counts()[:3]
    assert np.array_equal(ct, cw)
    assert np.abs(total[:, :3] - whole[:, :3]).max() <= 1e-12 * max(1.0, np.abs(whole).max())


@pytest.mark.parametrize("name", ["two_spheres_plane", "cornell"])
def test_c1_config_matches_oracle(gpu, oracle, name):
    """BASELINE.json configs[0] at its own size: Scene.xml's two spheres + plane (and the Cornell
    fallback scene), 256x256, 4 spp, through mfx_sample — the Color[w,h] image, the ray counters and
    the first Scene.Render frames against the oracle, bit for bit."""
    from mafrixraytracing_amd.native import NativeContext
    a = scene(name, 256, 256)
    o = oracle.OracleScene(a)
    ref, st = o.sample(4, SEED, sample_base=0, with_stats=True)
    with NativeContext(a, seed=SEED) as ctx:
        img = ctx.sample(4)
        counts = ctx.ray_counts()
    assert tuple(counts[:3]) == tuple(st[:3]), (counts[:3], st[:3])
    assert np.array_equal(img, ref), np.abs(img[:, :3] - ref[:, :3]).max()


def test_full_size_row_partition_merges_exactly(gpu):
    """C2 at 1920x1080, 8 spp, split over 8 MFX_F_ROW_PARTITION ranks (the multi-GPU image
    partition, one rank per GPU): the ranks' accumulators sum to the whole-film context's bit for
    bit, and their ray counts to its counts (135 tile rows: 17 or 16 per rank)."""
    from mafrixraytracing_amd.abi import MFX_F_ROW_PARTITION
    from mafrixraytracing_amd.native import NativeContext
    a = scene("spot")
    spp, P = 8, 8
    with NativeContext(a, seed=SEED) as ctx:
        ctx.trace_accumulate(spp, 3)
        whole = ctx.accum_read_mean(1.0)
        cw = ctx.ray_counts()[:3].copy()
    total = np.zeros_like(whole)
    ct = np.zeros(3)
    for p in range(P):
        with NativeContext(a, seed=SEED, flags=MFX_F_ROW_PARTITION, part_index=p, part_count=P) as ctx:
            ctx.trace_accumulate(spp, 3)
            total[:, :3] += ctx.accum_read_mean(1.0)[:, :3]
            ct += ctx.ray_counts()[:3]
    assert np.array_equal(ct, cw)
    assert np.array_equal(total[:, :3], whole[:, :3])


def test_full_size_render_ahead_device_list(gpu):
    """Scene.Render at C2's film size on a two-device list with render-ahead (K = 4): 10 frames
    byte-identical to the one-device context's, then the film."""
    from mafrixraytracing_amd.native import NativeContext
    a = scene("spot")
    with NativeContext(a, seed=SEED) as c1, NativeContext(a, seed=SEED, devices=[0, 0], render_ahead=4) as c2:
        for k in range(10):
            assert np.array_equal(c1.render_rgba8(1), c2.render_rgba8(1)), k
        assert np.array_equal(c1.film_mean(), c2.film_mean())


def test_pool_shrinks_when_the_device_is_short_of_memory(gpu):
    """A context created while the device had room, traced after other allocations left it short:
    the wavefront pool's allocation fails, the trace retries with half-size generations until it
    fits (wf_trace), and the accumulator and ray counts equal an unconstrained context's bit for bit.
    C2 at 64 spp: 132.7 M paths, a ~23 GB pool in one generation; 8 GB are left free (the pool fits
    at a quarter of the generation, with room for the runtime's own allocations)."""
    import torch
    from mafrixraytracing_amd.native import NativeContext
    a = scene("spot")  # 1920 x 1080
    with NativeContext(a, seed=SEED) as ref_ctx:
        ref_ctx.trace_accumulate(64, 0)
        want = ref_ctx.accum_read_mean(1.0)
        want_counts = ref_ctx.ray_counts()[:3]
    ctx = NativeContext(a, seed=SEED)
    try:
        free, _ = torch.cuda.mem_get_info()
        hog = torch.empty(max(0, free - (8 << 30)), dtype=torch.uint8, device="cuda")
        try:
            ctx.trace_accumulate(64, 0)
            got = ctx.accum_read_mean(1.0)
            counts = ctx.ray_counts()[:3]
            gens_short = ctx.trace_timing()["generations"]
        finally:
            del hog
            torch.cuda.empty_cache()
        # the shrink holds for that call only: with the memory back, the next trace of the same context
        # runs the frame as one generation again
        ctx.accum_clear()
        ctx.trace_accumulate(64, 0)
        again = ctx.accum_read_mean(1.0)
        gens_after = ctx.trace_timing()["generations"]
    finally:
        ctx.close()
    assert np.array_equal(got, want)
    assert np.array_equal(counts, want_counts)
    assert gens_short > 1 and gens_after == 1
    assert np.array_equal(again, want)


def test_trace_after_a_refused_pool_allocation(gpu, monkeypatch):
    """The pool's hipMalloc itself refused (another process took the memory between the headroom check
    and the allocation; MFX_POOL_FAIL_ONCE=1 asks for a size no device holds): wf_trace retries, and the
    refusal must not surface as the next launch's error (HIP's last error, which the launches return:
    r06p, eight ranks on one GPU failed "mfx_wf_iteration: out of memory"). The frame equals a plain
    context's bit for bit."""
    from mafrixraytracing_amd.native import NativeContext
    a = scene("cube_cornell", 64, 36)
    with NativeContext(a, seed=SEED) as c:
        c.trace_accumulate(4, 0)
        want = c.accum_read_mean(4.0)
    monkeypatch.setenv("MFX_POOL_FAIL_ONCE", "1")
    with NativeContext(a, seed=SEED) as c:
        c.trace_accumulate(4, 0)
        got = c.accum_read_mean(4.0)
    assert np.array_equal(got, want)

