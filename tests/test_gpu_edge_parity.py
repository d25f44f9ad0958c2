"""GPU parity on edge-case geometry and rays (SURVEY.md §8(a) A9/A10 semantics): random triangle
soups with exact duplicates (equal-t ties: the first minimum wins, BvhNode.fs:70,80), flat and
grid-aligned triangles (zero-extent boxes), near-degenerate slivers (|div| < 1e-6 cull,
Trangle.fs:130), and axis-aligned rays whose zero direction components (+0.0 and -0.0) make the
slab test divide by zero (±inf / NaN, IHitable.fs:18-54). Closest hits and occlusion must be
identical to the oracle, images within the parity bar of test_gpu_parity.py."""
import numpy as np
import pytest

from conftest import SEED
from test_gpu_build import soup

pytestmark = pytest.mark.gpu


def edge_rays(n, rng, grid):
    o = rng.uniform(-1.2, 1.2, size=(n, 3))
    if grid:  # origins on the soup's grid planes: rays run inside zero-extent boxes
        o[: n // 2] = np.round(o[: n // 2] * 4) / 4
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    q = n // 4
    axes = np.eye(3)[rng.integers(0, 3, size=q)] * rng.choice([-1.0, 1.0], size=(q, 1))
    d[:q] = axes
    d[:q][d[:q] == 0] = 0.0
    neg = rng.random(q) < 0.5  # -0.0 components (count as >= 0 in the slab test's branch)
    d[:q][neg] = np.where(d[:q][neg] == 0, -0.0, d[:q][neg])
    # one zero component, the other two normalised
    d2 = rng.normal(size=(q, 3))
    d2[np.arange(q), rng.integers(0, 3, size=q)] = 0.0
    d2 /= np.linalg.norm(d2, axis=1, keepdims=True)
    d[q:2 * q] = d2
    return np.concatenate([o, d], axis=1)


def slivers(a, rng, k):
    """Replace k triangles with slivers whose Möller–Trumbore determinant straddles 1e-6."""
    p = a.prims["p"]
    idx = rng.choice(len(p), size=k, replace=False)
    e = rng.uniform(1e-7, 1e-5, size=k)
    p[idx, 2] = p[idx, 0] + (p[idx, 1] - p[idx, 0]) * 0.5 + e[:, None] * np.array([0.0, 1.0, 0.0])
    return a


@pytest.mark.parametrize("n,grid", [(5, True), (777, True), (5000, False)])
def test_soup_closest_and_shadow_exact(gpu, oracle, n, grid):
    from mafrixraytracing_amd.native import NativeContext
    rng = np.random.default_rng(100 + n)
    a = slivers(soup(n, rng, grid=grid), rng, max(1, n // 20))
    rays = edge_rays(8000, rng, grid)
    o = oracle.OracleScene(a)
    ot, op, on = o.closest_hit(rays)
    tmax = rng.uniform(0.05, 3.0, size=len(rays))
    occ_o = o.any_hit(rays, tmax)
    with NativeContext(a) as ctx:
        gt, gp, gn = ctx.closest_hit(rays)
        occ_g = ctx.any_hit(rays, tmax)
    assert np.array_equal(gp, op), f"prim mismatch on {(gp != op).sum()} rays"
    assert np.array_equal(gt, ot)
    assert np.array_equal(gn, on)
    assert np.array_equal(occ_g, occ_o), f"occlusion mismatch on {(occ_g != occ_o).sum()} rays"
    if n > 5:
        assert (op >= 0).mean() > 0.01


@pytest.mark.parametrize("scale,offset", [(1e3, 5e3), (0.05, 0.0), (1.0, 3e4)])
def test_soup_far_from_unit_scale_exact(gpu, oracle, scale, offset):
    """The FP32 search stays conservative away from unit scale: the soup and its rays scaled by
    1e3 and moved 5e3 off the origin, shrunk to 0.05 (smaller, and the reference's absolute
    |div| < 1e-6 cull, Trangle.fs:130, leaves nothing to hit), and moved 3e4 away (FP32 spacing
    2^-9 there against triangles 0.05 across). Closest hits, normals and occlusion equal the
    oracle's."""
    from mafrixraytracing_amd.native import NativeContext
    rng = np.random.default_rng(400)
    a = soup(3000, rng, grid=True)
    a.prims["p"] = a.prims["p"] * scale + offset
    rays = edge_rays(6000, rng, True)
    rays[:, :3] = rays[:, :3] * scale + offset
    o = oracle.OracleScene(a)
    ot, op, on = o.closest_hit(rays)
    tmax = rng.uniform(0.05, 3.0, size=len(rays)) * scale
    occ_o = o.any_hit(rays, tmax)
    with NativeContext(a) as ctx:
        gt, gp, gn = ctx.closest_hit(rays)
        occ_g = ctx.any_hit(rays, tmax)
    assert np.array_equal(gp, op), f"prim mismatch on {(gp != op).sum()} rays"
    assert np.array_equal(gt, ot)
    assert np.array_equal(gn, on)
    assert np.array_equal(occ_g, occ_o), f"occlusion mismatch on {(occ_g != occ_o).sum()} rays"
    assert (op >= 0).mean() > 0.01


@pytest.mark.parametrize("name", ["cube_cornell", "spot"])
def test_scene_moved_far_from_origin_image_exact(gpu, oracle, name):
    """A whole scene (geometry, light and camera) moved (1e4, -3e3, 2e4) away: the FP32 search's
    widening grows with the coordinates and the FP64 paths see larger rounding
    (self-hits near tMin = 1e-6 among them); the 4-spp image is still the oracle's bit for bit."""
    from conftest import scene
    from mafrixraytracing_amd.abi import SceneArrays
    from mafrixraytracing_amd.native import NativeContext
    a = scene(name, 48, 27)
    off = np.array([1e4, -3e3, 2e4])
    assert np.all(a.prims["kind"] != 2)  # (a sphere's p[1] is its radius, not a point)
    prims = a.prims.copy()
    prims["p"] = prims["p"] + off
    light = dict(a.light, p=[list(np.asarray(q) + off) for q in a.light["p"]])
    cam = dict(a.camera, position=list(np.asarray(a.camera["position"]) + off))
    b = SceneArrays(prims, a.albedo, light, cam, a.width, a.height, a.max_depth)
    ref, st = oracle.OracleScene(b).sample(4, SEED, with_stats=True)
    with NativeContext(b, seed=SEED) as ctx:
        img = ctx.sample(4)
        counts = ctx.ray_counts()
    assert tuple(counts[:3]) == tuple(st[:3])
    assert np.array_equal(img, ref), np.abs(img - ref).max()
    assert img[:, :3].max() > 0


@pytest.mark.parametrize("n", [777, 5000])
def test_soup_image_parity(gpu, oracle, n):
    from mafrixraytracing_amd.native import NativeContext
    rng = np.random.default_rng(200 + n)
    a = slivers(soup(n, rng, grid=True), rng, n // 20)
    ref, st = oracle.OracleScene(a).sample(4, SEED, with_stats=True)
    with NativeContext(a, seed=SEED) as ctx:
        img = ctx.sample(4)
        counts = ctx.ray_counts()
    assert tuple(counts[:3]) == tuple(st[:3]), (counts[:3], st[:3])
    assert np.array_equal(img, ref), np.abs(img - ref).max()  # bit for bit
