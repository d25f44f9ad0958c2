"""Render-ahead (mfx_options.render_ahead; DESIGN.md §7 "Scene.Render"): one-sample render calls
served from a batch of the next K samples traced at once by the wavefront, whose k_resolve adds
them to the film in call order and writes each call's frame. Every frame must be the bytes of the
one-sample-per-call path, which the
oracle pins (test_gpu_parity.test_film_render_rgba8_matches_oracle_post); here both contexts run
side by side, and the first frames are also checked against the oracle's film directly."""
import numpy as np
import pytest

from conftest import SEED, scene

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,w,h,K", [("spot", 67, 37, 4), ("cube_cornell", 48, 27, 5),
                                         ("spot16_instanced@2l", 40, 24, 3), ("two_spheres_plane", 32, 32, 2)])
def test_render_ahead_frames_are_the_one_sample_frames(gpu, name, w, h, K):
    """12 Scene.Render calls with a reset after the 7th and an spp = 2 call in between (traced by
    the plain path; the next one-sample call needs a batch traced again from the film as it is then): identical
    RGBA8 bytes every call and an identical film."""
    from mafrixraytracing_amd.native import NativeContext
    a = scene(name, w, h)
    rays_plain = rays_ahead = 0.0
    with NativeContext(a, seed=SEED) as c1, NativeContext(a, seed=SEED, render_ahead=K) as c2:
        for k in range(12):
            spp = 2 if k == 4 else 1
            assert np.array_equal(c1.render_rgba8(spp), c2.render_rgba8(spp)), (name, k)
            rays_plain += c1.stats()[0]
            rays_ahead += c2.stats()[0]
            if k == 6:
                c1.reset()
                c2.reset()
        assert np.array_equal(c1.film_mean(), c2.film_mean())
    assert rays_plain > 0 and rays_ahead > 0


def test_render_ahead_pipeline_survives_interleaved_calls(gpu):
    """30 calls over ~8 batches (the next batch traced and post-processed in the background while
    one is served): frames without pixels (rgba = NULL), an mfx_sample call that moves the sample
    sequence mid-batch, a film read mid-batch and a reset; every frame, the Sample image and the
    film equal the one-sample-per-call context's."""
    from mafrixraytracing_amd.native import NativeContext
    a = scene("spot", 51, 29)
    with NativeContext(a, seed=SEED) as c1, NativeContext(a, seed=SEED, render_ahead=4) as c2:
        for k in range(30):
            if k == 6:
                assert np.array_equal(c1.sample(3), c2.sample(3))
            if k == 11:
                assert np.array_equal(c1.film_mean(), c2.film_mean())
            if k == 17:
                c1.reset()
                c2.reset()
            want = k % 3 != 1
            r1 = c1.render_rgba8(1, want_pixels=want)
            r2 = c2.render_rgba8(1, want_pixels=want)
            if want:
                assert np.array_equal(r1, r2), k
        assert np.array_equal(c1.film_mean(), c2.film_mean())


@pytest.mark.parametrize("budget,label", [(1024, "none fits: one sample per call"),
                                          (300_000, "one buffer, no background batch")])
def test_render_ahead_memory_fallbacks(gpu, monkeypatch, budget, label):
    """Render-ahead under a memory budget (MFX_RENDER_AHEAD_MAX_BYTES caps the quarter of free HBM
    the buffers may take): with no room for two samples the context falls back to one sample per
    call (the buffers freed, the film kept); with room for one buffer only it serves batches with
    no background trace. Either way every frame and the film are the one-sample path's."""
    from mafrixraytracing_amd.native import NativeContext
    monkeypatch.setenv("MFX_RENDER_AHEAD_MAX_BYTES", str(budget))
    a = scene("spot", 67, 37)
    with NativeContext(a, seed=SEED) as c1, NativeContext(a, seed=SEED, render_ahead=16) as c2:
        for k in range(40):
            if k == 23:
                c1.reset()
                c2.reset()
            assert np.array_equal(c1.render_rgba8(1), c2.render_rgba8(1)), (label, k)
        assert np.array_equal(c1.film_mean(), c2.film_mean()), label


def test_render_ahead_stats_account_for_whole_batches(gpu):
    """The batch call reports K samples' rays and device time; held calls report 0 rays in 0 s;
    over K calls the rays equal K one-sample calls'."""
    from mafrixraytracing_amd.native import NativeContext
    a = scene("spot", 64, 36)
    K = 4
    with NativeContext(a, seed=SEED) as c1, NativeContext(a, seed=SEED, render_ahead=K) as c2:
        plain = []
        for _ in range(2 * K):
            c1.render_rgba8(1, want_pixels=False)
            plain.append(c1.stats()[0])
        ahead = []
        for k in range(2 * K):
            c2.render_rgba8(1, want_pixels=False)
            r, sec = c2.stats()
            ahead.append(r)
            if k % K:
                assert r == 0 and sec < 1e-4  # events recorded back to back
            else:
                assert r > 0 and sec > 0.0
        assert ahead[0] == sum(plain[:K]) and ahead[K] == sum(plain[K:])


def test_render_ahead_matches_oracle_film(gpu, oracle):
    """Frames 1..5 of a render-ahead context (K = 3: a batch boundary inside) against the oracle's
    Film.AddSample + PostProcessAndToScreenBuffer, bit for bit."""
    from mafrixraytracing_amd.abi import dptr
    from mafrixraytracing_amd.native import NativeContext
    w, h = 40, 30
    a = scene("two_spheres_plane", w, h)
    o = oracle.OracleScene(a)
    npix = w * h
    accum, target, fc = np.zeros((npix, 4)), np.zeros((npix, 4)), np.zeros(1)
    with NativeContext(a, seed=SEED, render_ahead=3) as ctx:
        for k in range(5):
            rgba = ctx.render_rgba8(1)
            fr = o.sample(1, SEED, sample_base=k)
            oracle.lib().oracle_film_add(dptr(accum), dptr(target), dptr(fc), dptr(fr), npix)
            assert np.array_equal(rgba, oracle.post_rgba8(target, w, h)), k
        assert np.array_equal(ctx.film_mean()[:, :3], target[:, :3])


def test_render_ahead_option_validated(gpu):
    from mafrixraytracing_amd.abi import MfxError
    from mafrixraytracing_amd.native import NativeContext
    a = scene("spot", 16, 16)
    with pytest.raises(MfxError):
        NativeContext(a, seed=SEED, render_ahead=-1)
    with pytest.raises(MfxError):
        NativeContext(a, seed=SEED, render_ahead=1 << 20)


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0]])
@pytest.mark.parametrize("name,w,h,K", [("spot", 67, 37, 4), ("cube_cornell", 48, 27, 5)])
def test_render_ahead_on_a_device_list(gpu, devices, name, w, h, K):
    """Scene(state, devices) — the F# binding's device-list context — serving Scene.Render from
    batches on every device (image partition: device g traces the tile rows of band g of G of each batch and
    copies its rows of each frame). 14 calls with an spp = 2 call, a film read mid-batch, a reset and
    an mfx_sample call in between: every RGBA8 frame, the Sample image, the film and the rays equal
    the one-device context without render-ahead, bit for bit. (37 rows: 5 tile rows, the last one
    partial, so with 3 devices one device's band ends in the partial row.)"""
    from mafrixraytracing_amd.native import NativeContext
    a = scene(name, w, h)
    rays_plain = rays_multi = 0.0
    with NativeContext(a, seed=SEED) as c1, NativeContext(a, seed=SEED, devices=devices, render_ahead=K) as c2:
        for k in range(14):
            spp = 2 if k == 4 else 1
            if k == 6:
                assert np.array_equal(c1.film_mean(), c2.film_mean()), k
            if k == 9:
                c1.reset()
                c2.reset()
            if k == 11:
                assert np.array_equal(c1.sample(3), c2.sample(3))
            assert np.array_equal(c1.render_rgba8(spp), c2.render_rgba8(spp)), (name, devices, k)
            rays_plain += c1.stats()[0]
            rays_multi += c2.stats()[0]
        assert np.array_equal(c1.film_mean(), c2.film_mean())
    # the last batch may hold samples no call has taken yet: only whole served batches compare
    assert rays_multi > 0 and rays_plain > 0


def test_render_ahead_device_list_with_an_empty_band(gpu):
    """A film of one tile row on three devices: devices 1 and 2 own no row (no trace, no copy) and
    the frames are still the one-device frames."""
    from mafrixraytracing_amd.native import NativeContext
    a = scene("spot", 24, 8)
    with NativeContext(a, seed=SEED) as c1, NativeContext(a, seed=SEED, devices=[0, 0, 0], render_ahead=3) as c2, \
            NativeContext(a, seed=SEED, devices=[0, 0, 0]) as c3:
        for k in range(7):
            r1 = c1.render_rgba8(1)
            assert np.array_equal(r1, c2.render_rgba8(1)), k
            assert np.array_equal(r1, c3.render_rgba8(1)), k
        assert np.array_equal(c1.film_mean(), c2.film_mean())
        assert np.array_equal(c1.sample(2), c3.sample(2))


def test_film_mean_mid_batch_traces_each_sample_once(gpu):
    """Render and mfx_film_mean alternating inside one batch: each film read traces only
    the samples served since the last one (film only), not the batch prefix again; the films are the
    one-sample path's."""
    from mafrixraytracing_amd.native import NativeContext
    a = scene("spot", 40, 24)
    K = 8
    with NativeContext(a, seed=SEED) as c1, NativeContext(a, seed=SEED, render_ahead=K) as c2:
        for k in range(2 * K):
            assert np.array_equal(c1.render_rgba8(1), c2.render_rgba8(1)), k
            assert np.array_equal(c1.film_mean(), c2.film_mean()), k


def test_trace_timing_keeps_to_eight_doubles(gpu):
    """mfx_trace_timing writes exactly out[8], also for a call served from held frames (ADVICE r04:
    the render-ahead branch cleared 12 doubles): a guard after the buffer stays untouched."""
    import ctypes as C
    from mafrixraytracing_amd.abi import check, dptr
    from mafrixraytracing_amd.native import NativeContext
    a = scene("spot", 32, 16)
    with NativeContext(a, seed=SEED, render_ahead=4) as c:
        for k in range(6):
            c.render_rgba8(1, want_pixels=False)
            buf = np.full(16, 12345.0)
            check(c.lib.mfx_trace_timing(c._h, dptr(buf)), "mfx_trace_timing")
            assert np.all(buf[8:] == 12345.0), k
    _ = C
