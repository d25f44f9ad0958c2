"""Multi-device contexts through the C ABI (mfx_options.devices).

One context drives a device list from one process by an image partition: device g of G traces the
film's 8-pixel tile rows of band g of G (serpentine: one of each G consecutive tile rows; every
sample) on its own stream, so every per-pixel operation
runs on one device in the one-device order and every output is the one-device context's, bit for
bit. FP64 buffers (mfx_sample's accumulator, mfx_film_mean's film) merge on devices[0]:
- a list of distinct devices with RCCL (a communicator the library creates with ncclCommInitAll);
  devices=[0] runs that code path on the 1-GPU box (a 1-rank reduce);
- a list that repeats a device (devices=[0,0]) by device-ordered adds.
A pixel is +0.0 on every device but its own, so either sum is an exact merge. The 8-GPU case is the
driver's; every bit of bookkeeping it uses is exercised here with G = 1-3.
"""
import ctypes as C

import numpy as np
import pytest

from conftest import SEED, scene

pytestmark = pytest.mark.gpu


def test_single_device_list_is_bit_identical(gpu):
    """devices=[0] (RCCL communicator of one rank + its reduce) == the plain single-device context."""
    from mafrixraytracing_amd.native import NativeContext
    a = scene("spot", 64, 36)
    with NativeContext(a, seed=SEED) as c1, NativeContext(a, seed=SEED, devices=[0]) as c2:
        for _ in range(2):
            assert np.array_equal(c1.sample(3), c2.sample(3))
            assert np.array_equal(c1.render_rgba8(2), c2.render_rgba8(2))
        assert np.array_equal(c1.film_mean(), c2.film_mean())
        assert np.array_equal(c1.ray_counts(), c2.ray_counts())


@pytest.mark.parametrize("G", [2, 3])
def test_repeated_device_list_partitions_rows_exactly(gpu, oracle, G):
    """devices=[0]*G: device g traces the tile rows of band g; after the merge the primary's accumulator is
    the one-device context's bit for bit, and so are the Sample image and the ray counters; the
    image matches the oracle. cube_cornell at 48x27: 4 tile rows, the last one partial."""
    from mafrixraytracing_amd.native import NativeContext
    a = scene("cube_cornell", 48, 27)
    spp = 7
    with NativeContext(a, seed=SEED) as s:
        s.accum_clear()
        s.trace_accumulate(spp, 0)
        want = s.accum_read_mean(1.0)
        want_counts = s.ray_counts()
    with NativeContext(a, seed=SEED, devices=[0] * G) as m:
        m.accum_clear()
        m.trace_accumulate(spp, 0)
        counts = m.ray_counts()
        m.accum_reduce()
        got = m.accum_read_mean(1.0)
        img = m.sample(spp)  # the same frame through mfx_sample (trace_accumulate does not advance it)
    assert np.array_equal(got, want)
    assert np.array_equal(counts[:4], want_counts[:4])
    ref = oracle.OracleScene(a).sample(spp, SEED, sample_base=0)
    assert np.array_equal(img, ref)


@pytest.mark.parametrize("P", [2, 3])
def test_row_partition_ranks_merge_exactly(gpu, P):
    """MFX_F_ROW_PARTITION (the multi-process image partition): P one-device contexts, rank p traces
    every sample of the tile rows of band p (distributed.tile_row_owner); each rank's accumulator is +0.0 outside its rows, and the sum
    over the ranks is the whole-film context's accumulator bit for bit (so is the ray total)."""
    from mafrixraytracing_amd.abi import MFX_F_ROW_PARTITION
    from mafrixraytracing_amd.distributed import tile_row_owner
    from mafrixraytracing_amd.native import NativeContext
    w, h = 50, 29  # 4 tile rows, the last one partial; 7 tile columns, the last one partial
    a = scene("spot", w, h)
    spp = 5
    with NativeContext(a, seed=SEED) as s:
        s.trace_accumulate(spp, 11)
        want = s.accum_read_mean(1.0)
        want_rays = s.ray_counts()[:4]
    total = np.zeros_like(want)
    rays = np.zeros(4)
    rows = np.arange(h) // 8
    for p in range(P):
        with NativeContext(a, seed=SEED, flags=MFX_F_ROW_PARTITION, part_index=p, part_count=P) as c:
            c.trace_accumulate(spp, 11)
            part = c.accum_read_mean(1.0)
            rays += c.ray_counts()[:4]
        own = np.tile(tile_row_owner(rows, P) == p, w)  # x-major pixels: pixel = x * h + y
        assert not np.any(part[~own, :3]), p
        assert np.array_equal(part[own], want[own]), p
        total[:, :3] += part[:, :3]
    total[:, 3] = want[:, 3]
    assert np.array_equal(total, want)
    assert np.array_equal(rays, want_rays)


def test_repeated_device_reduce_orders_later_work(gpu):
    """mfx_accum_reduce then, with no mfx_sync, another trace onto the same accumulators: the peers'
    streams wait for the primary's copies of their buffers, so the reduced frame holds
    only the first trace's samples — equal to the same calls with a sync after the reduce."""
    from mafrixraytracing_amd.native import NativeContext
    a = scene("cube_cornell", 48, 27)
    out = []
    for synced in (False, True):
        with NativeContext(a, seed=SEED, devices=[0, 0, 0]) as m:
            m.accum_clear()
            m.trace_accumulate(6, 0)
            m.accum_reduce()
            if synced:
                m.sync()
            m.trace_accumulate(5, 6)  # no clear: every device adds onto its buffer
            m.accum_reduce()
            out.append(m.accum_read_mean(1.0))
    assert np.array_equal(out[0], out[1])


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0]])
def test_repeated_device_render_and_stats(gpu, devices):
    """Scene.Render (no render-ahead) on a device list: each device adds its rows to its band of the
    film and copies its rows of the RGBA8 frame; frames, the merged film and the ray counts equal the
    one-device context's, bit for bit, across spp != 1 calls and a reset."""
    from mafrixraytracing_amd.native import NativeContext
    a = scene("two_spheres_plane", 40, 30)
    with NativeContext(a, seed=SEED, devices=devices) as m, NativeContext(a, seed=SEED) as s:
        for k in range(5):
            spp = 1 + (k % 3)
            assert np.array_equal(m.render_rgba8(spp), s.render_rgba8(spp)), k
            if k == 2:
                m.reset()
                s.reset()
        assert np.array_equal(m.film_mean(), s.film_mean())
        rays, sec = m.stats()
        n = s.ray_counts()
        assert rays == n[0] + n[1] + n[2] and sec > 0


def test_sample_mean_divides_by_the_count(gpu):
    """mfx_sample(49) divides by 49 itself (Integrators.fs:171): 1/(1/49) != 49 in FP64, so a
    reciprocal round trip would be 1 ulp off here."""
    from mafrixraytracing_amd.native import NativeContext
    assert 1.0 / (1.0 / 49.0) != 49.0
    a = scene("cornell", 16, 16)
    with NativeContext(a, seed=SEED) as c1, NativeContext(a, seed=SEED) as c2:
        img = c1.sample(49)
        c2.accum_clear()
        c2.trace_accumulate(49, 0)
        acc = c2.accum_read_mean(1.0)
        assert np.array_equal(c2.accum_read_mean(49.0), img)
    assert np.array_equal(img[:, :3], acc[:, :3] / 49.0)


def test_bad_device_lists_fail_loudly(gpu):
    from mafrixraytracing_amd.abi import MfxError
    from mafrixraytracing_amd.native import NativeContext
    a = scene("cornell", 8, 8)
    n = gpu.mfx_device_count()
    with pytest.raises(MfxError):
        NativeContext(a, seed=SEED, devices=[0, n])  # no such device
    with pytest.raises(MfxError):  # partitioned contexts compose through trace_accumulate, not Sample
        with NativeContext(a, seed=SEED, devices=[0, 0], part_index=0, part_count=2) as m:
            m.sample(1)
    _ = C


def test_one_sample_calls_megakernel_equals_wavefront(gpu):
    """A call in which the device renders one sample per pixel (Scene.Render) runs the megakernel
    by default; MFX_F_WAVEFRONT pins the wavefront. Same paths, same per-path arithmetic, one path
    per pixel (exact accumulation): identical bits, counters and bytes."""
    from mafrixraytracing_amd.abi import MFX_F_WAVEFRONT
    from mafrixraytracing_amd.native import NativeContext
    a = scene("spot", 96, 54)
    with NativeContext(a, seed=SEED) as auto, NativeContext(a, seed=SEED, flags=MFX_F_WAVEFRONT) as wf:
        for _ in range(3):
            assert np.array_equal(auto.render_rgba8(1), wf.render_rgba8(1))
            assert np.array_equal(auto.ray_counts()[:4], wf.ray_counts()[:4])
            tw = wf.trace_timing()  # 4 bounce-synchronous iterations
            assert auto.trace_timing()["launches"] == 1
            assert tw["launches"] == 4, tw
        assert np.array_equal(auto.film_mean(), wf.film_mean())
        assert np.array_equal(auto.sample(1), wf.sample(1))
    # two devices of one sample each: every device takes the megakernel
    with NativeContext(a, seed=SEED, devices=[0, 0]) as m2, NativeContext(a, seed=SEED, devices=[0, 0],
                                                                         flags=MFX_F_WAVEFRONT) as w2:
        assert np.array_equal(m2.sample(2), w2.sample(2))


@pytest.mark.parametrize("devices", [None, [0, 0]])
def test_ray_counts_total_sums_back_to_back_traces(gpu, devices):
    """mfx_ray_counts_total: the counters of traces enqueued back to back (no host read between
    them, as the bench's timed steps run) summed on the device, over every device of a list; equal
    to the per-trace counters read one by one; reset zeroes them."""
    from mafrixraytracing_amd.native import NativeContext
    a = scene("spot", 48, 27)
    frames = [(3, 0), (1, 3), (5, 4)]  # a one-sample frame runs the megakernel: counted too
    with NativeContext(a, seed=SEED, devices=devices) as one:
        want = np.zeros(16)
        for spp, base in frames:
            one.trace_accumulate(spp, base)
            want += one.ray_counts()
    with NativeContext(a, seed=SEED, devices=devices) as c:
        c.trace_accumulate(2, 100)
        c.ray_counts_total(reset=True)
        for spp, base in frames:
            c.accum_clear()
            c.trace_accumulate(spp, base)
        got = c.ray_counts_total(reset=True)
        assert np.array_equal(got[:3], want[:3]) and got[3] == got[0]
        assert not np.any(c.ray_counts_total(reset=False)[:3])


@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0]])
def test_accum_read_mean_after_render_merges_the_device_list(gpu, devices):
    """a render call on a device list leaves each device's rows in its own accumulator;
    mfx_accum_read_mean merges them before reading (and only once: a second read, or a read after an
    explicit mfx_accum_reduce, is the same), so it equals the one-device context's accumulator."""
    from mafrixraytracing_amd.native import NativeContext
    a = scene("cube_cornell", 48, 27)
    with NativeContext(a, seed=SEED) as s:
        s.render_rgba8(3)
        want = s.accum_read_mean(3.0)
    with NativeContext(a, seed=SEED, devices=devices) as m:
        m.render_rgba8(3)
        got = m.accum_read_mean(3.0)
        again = m.accum_read_mean(3.0)
        m.accum_reduce()
        third = m.accum_read_mean(3.0)
    assert np.array_equal(got, want) and np.array_equal(again, want) and np.array_equal(third, want)
