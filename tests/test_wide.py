"""The per-lane traversal's BVH8 (mfx_wide.cpp), host-only: built from each scene's BVH4 and checked
by the library itself (mfx_wide_info: every BVH4 leaf reached exactly once, every FP16 box, back in
the world frame, containing the FP32 boxes of its subtree — the conservative-search property the
exact leaf semantics rest on). The GPU tests then hold the images bit-exact against
the oracle with this image in the loop (test_gpu_parity.py, test_gpu_edge_parity.py)."""
import numpy as np
import pytest

from conftest import scene
from test_gpu_build import soup


def check(a):
    from mafrixraytracing_amd.abi import wide_info
    r = wide_info(a)
    assert r["nodes"] >= 1 and r["leaves"] >= 1
    assert 1 <= r["stack"] <= 96
    assert r["depth"] <= max(r["depth4"], 1)  # (depth4 counts a lone root as 0)
    assert 1.0 <= r["mean_entries"] <= 8.0
    s = r["scale"]
    assert s > 0 and np.log2(s) == round(np.log2(s))  # a power of 2: the ray transform is exact
    return r


@pytest.mark.parametrize("name", ["spot", "cube_cornell", "cornell", "two_spheres_plane", "spot16"])
def test_wide_image_of_scene(name):
    r = check(scene(name, 64, 36))
    if name in ("spot", "spot16"):
        assert r["mean_entries"] > 4.5  # the collapse fills the nodes


@pytest.mark.parametrize("n,grid,zoom", [(1, False, 1.0), (5, True, 1.0), (777, True, 1.0), (5000, False, 1.0),
                                         (3000, False, 1e5), (3000, True, 1e-4)])
def test_wide_image_of_soup(n, grid, zoom):
    """Duplicates, flat boxes, and coordinates far outside FP16's range (x 1e5) or deep in its
    subnormals (x 1e-4): the frame's power-of-2 scale keeps every plane finite and outward."""
    a = soup(n, np.random.default_rng(300 + n), grid=grid)
    a.prims["p"] *= zoom
    check(a)


def test_half_rounding_is_directed():
    """mfx_half_round through the image: a single primitive's box, its planes at awkward values."""
    from mafrixraytracing_amd.abi import PRIM_DTYPE, SceneArrays
    base = scene("spot", 32, 18)
    for v in (1.0 / 3.0, 65504.0 * 0.9, 1e-7, 12345.678, -2.0 ** -14):
        p = np.zeros(1, dtype=PRIM_DTYPE)
        p["p"][0, :3] = [[v, v, v], [v * 1.5 + 1e-3, v, v], [v, v * 1.25 + 1e-3, v]]
        check(SceneArrays(p, base.albedo[:1], base.light, base.camera, 32, 18))
