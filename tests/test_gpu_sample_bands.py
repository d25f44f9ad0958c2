"""mfx_sample's banded readback (VERDICT r05 Next #6): on one device the last generation's k_resolve
runs in column bands of tiles, each band's mean and readback enqueued behind it on the copy stream.
Every Sample frame must be the unbanded path's (MFX_SAMPLE_BANDS=0) and the oracle's bit for bit:
films whose width is not a multiple of 8 (a partial last tile column), fewer tile columns than bands,
several generations (MFX_POOL: only the last one is banded), one sample per pixel (the megakernel,
no bands) and back-to-back calls that reuse the staging buffer. The bands' means are staged as RGB and
widened to RGBA by the host (alpha 1.0); MFX_SAMPLE_RGBA=1 stages the RGBA frame itself."""
import numpy as np
import pytest

from conftest import SEED, scene

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,w,h,spp", [("spot", 61, 37, 3), ("cube_cornell", 20, 13, 4), ("renault", 96, 54, 2),
                                          ("spot", 64, 36, 1)])
def test_banded_sample_equals_unbanded_and_oracle(gpu, oracle, monkeypatch, name, w, h, spp):
    from mafrixraytracing_amd.native import NativeContext
    a = scene(name, w, h)
    with NativeContext(a, seed=SEED) as c:
        banded = [c.sample(spp) for _ in range(2)]
    monkeypatch.setenv("MFX_SAMPLE_ZEROCOPY", "1")  # the means written straight into page-locked memory
    with NativeContext(a, seed=SEED) as c:
        zero = [c.sample(spp) for _ in range(2)]
    monkeypatch.delenv("MFX_SAMPLE_ZEROCOPY")
    monkeypatch.setenv("MFX_SAMPLE_RGBA", "1")  # the whole RGBA frame staged (no host-written alpha)
    with NativeContext(a, seed=SEED) as c:
        rgba = [c.sample(spp) for _ in range(2)]
    monkeypatch.delenv("MFX_SAMPLE_RGBA")
    monkeypatch.setenv("MFX_SAMPLE_BANDS", "0")
    with NativeContext(a, seed=SEED) as c:
        plain = [c.sample(spp) for _ in range(2)]
    for b, z, r, p in zip(banded, zero, rgba, plain):
        assert np.array_equal(b, p) and np.array_equal(z, p) and np.array_equal(r, p)
    o = oracle.OracleScene(a)
    assert np.array_equal(banded[1], o.sample(spp, SEED, sample_base=spp))


def test_banded_sample_several_generations_and_full_film(gpu, monkeypatch):
    """C2's film (1080p, 240 tile columns in 8 bands of 30; the staged 66 MB readback) at 2 spp, and
    the same frame traced in generations of 2^20 paths (MFX_POOL): only the last generation's resolve
    is banded; both equal the unbanded frame."""
    from mafrixraytracing_amd.native import NativeContext
    a = scene("spot")
    with NativeContext(a, seed=SEED) as c:
        banded = c.sample(2)
        counts = c.ray_counts()
    monkeypatch.setenv("MFX_POOL", str(1 << 20))
    with NativeContext(a, seed=SEED) as c:
        gens = c.sample(2)
        assert c.trace_timing()["generations"] > 1
    monkeypatch.delenv("MFX_POOL")
    monkeypatch.setenv("MFX_SAMPLE_BANDS", "0")
    with NativeContext(a, seed=SEED) as c:
        plain = c.sample(2)
        assert np.array_equal(c.ray_counts()[:4], counts[:4])
    assert np.array_equal(banded, plain) and np.array_equal(gens, plain)
