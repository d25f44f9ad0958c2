"""On-GPU traversal-BVH build (the reference builds on the host, Bvh.Build,
BvhNode.fs:24-61) against the host build: mfx_build.hip builds the same binned-SAH tree as
mfx_scene.cpp's SahBuilder, so the device images are byte-identical (equal FNV digests) and every
traversal, counter and image is identical too. The default context builds on the GPU, so every
other GPU parity test also runs on the GPU-built tree."""
import numpy as np
import pytest

from conftest import SEED, scene

pytestmark = pytest.mark.gpu

SCENES = ["two_spheres_plane", "cornell", "spot", "cube_cornell", "renault", "spot16", "spot16_instanced", "spot16_instanced@2l"]


def both(a):
    from mafrixraytracing_amd.abi import MFX_F_HOST_BVH
    from mafrixraytracing_amd.native import NativeContext
    with NativeContext(a, seed=SEED) as g:
        bg = g.build_info()
    with NativeContext(a, seed=SEED, flags=MFX_F_HOST_BVH) as h:
        bh = h.build_info()
    return bg, bh


@pytest.mark.parametrize("name", SCENES)
def test_gpu_bvh_equals_host_bvh(gpu, name):
    a = scene(name, 16, 16)
    bg, bh = both(a)
    assert bg["gpu_bvh"] and not bh["gpu_bvh"]
    # flat (and auto-flattened) scenes: collapse and layout on the GPU too
    assert bg["gpu_images"] == (a.instancing is None or not a.two_level)
    for k in ("nodes2", "nodes4", "slots"):
        assert bg[k] == bh[k], (k, bg[k], bh[k])
    assert bg["digest"] == bh["digest"]


def soup(n, rng, dup_frac=0.2, grid=False):
    """Random triangles with duplicated and axis-aligned ones: coincident centroids, flat boxes and
    equal SAH costs exercise the tie rules and the all-centroids-equal split."""
    from mafrixraytracing_amd.abi import PRIM_DTYPE, SceneArrays
    base = scene("spot", 32, 18)
    p = np.zeros(n, dtype=PRIM_DTYPE)
    v0 = rng.uniform(-1, 1, size=(n, 3))
    if grid:
        v0 = np.round(v0 * 4) / 4
    p["p"][:, 0] = v0
    p["p"][:, 1] = v0 + rng.uniform(-0.05, 0.05, size=(n, 3))
    p["p"][:, 2] = v0 + rng.uniform(-0.05, 0.05, size=(n, 3))
    nd = int(n * dup_frac)
    p[n - nd:] = p[:nd]  # exact duplicates
    flat = rng.random(n) < 0.1
    p["p"][flat, :, 1] = p["p"][flat, 0:1, 1]  # flat in y (zero box extent)
    p["kind"] = 0
    return SceneArrays(p, base.albedo[:1], base.light, base.camera, 32, 18)


@pytest.mark.parametrize("n,grid", [(1, False), (2, False), (5, True), (777, True), (20000, False), (60000, True)])
def test_gpu_bvh_equals_host_bvh_on_triangle_soup(gpu, n, grid):
    bg, bh = both(soup(n, np.random.default_rng(n), grid=grid))
    assert bg["digest"] == bh["digest"], (bg, bh)


def test_gpu_bvh_build_time_reported(gpu):
    bg, bh = both(scene("spot16", 16, 16))
    assert bg["bvh_ms"] > 0 and bh["bvh_ms"] > 0 and bg["levels"] > 1
    print(f"spot16 BVH2: GPU {bg['bvh_ms']:.1f} ms ({bg['levels']} levels), host {bh['bvh_ms']:.1f} ms; "
          f"reference grouping {bh['ref_bvh_ms']:.1f} ms; scene {bg['scene_ms']:.1f} / {bh['scene_ms']:.1f} ms")
