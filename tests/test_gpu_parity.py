"""GPU parity: the HIP path (through the C ABI) against the CPU oracle on identical inputs.

Bar: discrete results (hit/miss, primitive, occlusion, ray counts, reference-leaf
grouping, RGBA8 bytes) identical; FP64 hit distances and normals bit-identical; images bit-identical
too: both pipelines fold a path's vertices in the reference's recursion order, and the wavefront
adds a pixel's samples in sample order like the oracle. The one exception is the megakernel at
more than one sample per pixel, which adds a pixel's paths with FP64 atomics in arrival order:
within 1e-12 there (and inside north_star's 1e-4 per-channel RMSE gate, asserted too).
"""
import os

import numpy as np
import pytest

from conftest import SEED, scene

pytestmark = pytest.mark.gpu

# spot16_instanced: the library's default flags (flattened, it fits the budget); @2l: two-level forced
SCENES = ["two_spheres_plane", "cornell", "spot", "cube_cornell", "renault", "spot16", "spot16_instanced",
          "spot16_instanced@2l"]


def random_rays(arrays, n, rng, camera_frac=0.5):
    p = arrays.prims["p"]
    k = arrays.prims["kind"]
    pts = p[k != 2][:, :3, :].reshape(-1, 3)
    sph = p[k == 2]
    if len(sph):
        pts = np.concatenate([pts, sph[:, 0, :]])
    lo, hi = pts.min(0), pts.max(0)
    pad = 0.1 * (hi - lo) + 1e-3
    lo, hi = lo - pad, hi + pad
    nc = int(n * camera_frac)
    o = rng.uniform(lo, hi, size=(n, 3))
    o[:nc] = np.asarray(arrays.camera["position"], dtype=np.float64)
    tgt = rng.uniform(lo, hi, size=(n, 3))
    d = tgt - o
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return np.concatenate([o, d], axis=1)


@pytest.mark.parametrize("name", SCENES)
def test_ref_leaf_grouping_identical(gpu, oracle, name):
    from mafrixraytracing_amd.native import NativeContext
    a = scene(name, 16, 16)
    with NativeContext(a) as ctx:
        gi, gf, gc = ctx.ref_leaves()
    oi, of, oc = oracle.OracleScene(a).bvh_leaves()
    assert np.array_equal(gi, oi)
    assert np.array_equal(gf, of) and np.array_equal(gc, oc)


@pytest.mark.parametrize("name", SCENES)
def test_closest_hit_bit_exact(gpu, oracle, name):
    from mafrixraytracing_amd.native import NativeContext
    a = scene(name, 16, 16)
    rays = random_rays(a, 20000, np.random.default_rng(1))
    o = oracle.OracleScene(a)
    ot, op, on = o.closest_hit(rays)
    with NativeContext(a) as ctx:
        gt, gp, gn = ctx.closest_hit(rays)
    assert np.array_equal(gp, op), f"prim mismatch on {(gp != op).sum()} rays"
    assert np.array_equal(gt, ot)
    assert np.array_equal(gn, on)
    assert (op >= 0).mean() > 0.05  # the ray set actually hits things


@pytest.mark.parametrize("name", SCENES)
def test_shadow_query_exact(gpu, oracle, name):
    """Shadow rays from hit points toward the light, tmax = dist - 1e-6 (Integrators.fs:44),
    including the reference's leaf quirk (Triangle.Hit ignores tMax)."""
    from mafrixraytracing_amd.native import NativeContext
    a = scene(name, 16, 16)
    rng = np.random.default_rng(2)
    rays = random_rays(a, 20000, rng)
    o = oracle.OracleScene(a)
    t, prim, _ = o.closest_hit(rays)
    hit = prim >= 0
    hp = rays[hit, :3] + rays[hit, 3:] * t[hit, None]
    L = np.asarray(a.light["p"], dtype=np.float64)
    uv = rng.uniform(0, 1, size=(hit.sum(), 2))
    lp = L[0] + uv[:, :1] * (L[1] - L[0]) + uv[:, 1:] * (L[3] - L[0])
    to = lp - hp
    dist = np.linalg.norm(to, axis=1)
    srays = np.concatenate([hp, to / dist[:, None]], axis=1)
    tmax = dist - 1e-6
    occ_o = o.any_hit(srays, tmax)
    with NativeContext(a) as ctx:
        occ_g = ctx.any_hit(srays, tmax)
    assert np.array_equal(occ_g, occ_o), f"occlusion mismatch on {(occ_g != occ_o).sum()} rays"


def test_fp64_device_math_bit_exact(gpu):
    from mafrixraytracing_amd.native import fp64_selftest
    rng = np.random.default_rng(3)
    a = np.concatenate([rng.uniform(0, 4, 100000), 10.0 ** rng.uniform(-300, 300, 100000)])
    b = np.concatenate([rng.uniform(-3, 3, 100000), 10.0 ** rng.uniform(-300, 300, 100000)])
    dv, sq = fp64_selftest(a, b)
    assert np.array_equal(dv, a / b)
    assert np.array_equal(sq, np.sqrt(a))


@pytest.mark.parametrize("name,w,h,spp", [
    ("two_spheres_plane", 64, 64, 8),
    ("cornell", 48, 48, 8),
    ("spot", 64, 36, 8),
    ("cube_cornell", 64, 36, 8),
    ("renault", 64, 36, 4),
    ("spot16", 64, 36, 4),
    ("spot16_instanced", 64, 36, 4),
    ("spot16_instanced@2l", 64, 36, 4),
])
@pytest.mark.parametrize("mode", ["wavefront", "megakernel"])
def test_image_parity(gpu, oracle, name, w, h, spp, mode):
    from mafrixraytracing_amd.abi import MFX_F_MEGAKERNEL, MFX_F_NONE
    from mafrixraytracing_amd.native import NativeContext
    a = scene(name, w, h)
    o = oracle.OracleScene(a)
    ref, st = o.sample(spp, SEED, with_stats=True)
    flags = MFX_F_MEGAKERNEL if mode == "megakernel" else MFX_F_NONE
    with NativeContext(a, seed=SEED, flags=flags) as ctx:
        img = ctx.sample(spp)
        counts = ctx.ray_counts()
    assert counts[0] == st[0] and counts[1] == st[1] and counts[2] == st[2], (counts[:3], st[:3])
    diff = np.abs(img[:, :3] - ref[:, :3])
    rmse = np.sqrt((diff ** 2).mean(axis=0))
    assert np.all(rmse <= 1e-4), rmse  # north_star gate
    if mode == "wavefront":
        assert np.array_equal(img, ref), diff.max()  # bit for bit
    else:  # FP64 atomics add a pixel's paths in arrival order
        assert diff.max() <= 1e-12 * max(1.0, np.abs(ref).max()), diff.max()
    assert np.all(img[:, 3] == 1.0)


def test_default_flags_two_level_when_over_budget(gpu, oracle, monkeypatch):
    """An instanced scene over the flatten budget takes the two-level traversal with the default
    flags (no MFX_F_TWO_LEVEL): images and ray counts still equal the oracle's on the expansion."""
    from mafrixraytracing_amd.native import NativeContext
    monkeypatch.setenv("MFX_FLATTEN_MAX_BYTES", "1024")
    a = scene("spot16_instanced", 48, 27)
    ref, st = oracle.OracleScene(a).sample(2, SEED, with_stats=True)
    with NativeContext(a, seed=SEED) as ctx:
        assert ctx.instancing_info()["instances"] == 16  # two-level
        img = ctx.sample(2)
        counts = ctx.ray_counts()
    assert counts[0] == st[0] and counts[1] == st[1] and counts[2] == st[2], (counts[:3], st[:3])
    assert np.array_equal(img, ref)


def test_successive_sample_calls_continue_the_stream(gpu, oracle):
    """Sample(n) twice == oracle with sample_base 0 then n (the reference's RNG keeps running)."""
    from mafrixraytracing_amd.native import NativeContext
    a = scene("cornell", 24, 24)
    o = oracle.OracleScene(a)
    with NativeContext(a, seed=SEED) as ctx:
        f1 = ctx.sample(3)
        f2 = ctx.sample(3)
    r1 = o.sample(3, SEED, sample_base=0)
    r2 = o.sample(3, SEED, sample_base=3)
    assert np.array_equal(f1, r1) and np.array_equal(f2, r2)


def test_film_render_rgba8_matches_oracle_post(gpu, oracle):
    """Scene.Render x3 (1 spp each) == Film.AddSample x3 + PostProcessAndToScreenBuffer."""
    from mafrixraytracing_amd.native import NativeContext
    a = scene("two_spheres_plane", 40, 30)
    o = oracle.OracleScene(a)
    npix = 40 * 30
    accum = np.zeros((npix, 4))
    target = np.zeros((npix, 4))
    fc = np.zeros(1)
    import ctypes as C
    from mafrixraytracing_amd.abi import dptr
    with NativeContext(a, seed=SEED) as ctx:
        for k in range(3):
            rgba = ctx.render_rgba8(1)
            fr = o.sample(1, SEED, sample_base=k)
            oracle.lib().oracle_film_add(dptr(accum), dptr(target), dptr(fc), dptr(fr), npix)
        mean = ctx.film_mean()
    assert np.array_equal(mean[:, :3], target[:, :3])
    ref = oracle.post_rgba8(target, 40, 30)
    assert np.array_equal(rgba, ref), (rgba != ref).sum()  # the same bytes
    _ = C


def test_partitioned_contexts_sum_to_whole(gpu, oracle):
    """Sample partitions (the multi-GPU decomposition) sum to the single image."""
    from mafrixraytracing_amd.native import NativeContext
    a = scene("spot", 48, 27)
    spp, G = 8, 3
    total = np.zeros((48 * 27, 4))
    for g in range(G):
        with NativeContext(a, seed=SEED, part_index=g, part_count=G) as ctx:
            ctx.accum_clear()
            ctx.trace_accumulate(spp, 0)
            total += ctx.accum_read_mean(1.0)
    ref = oracle.OracleScene(a).sample(spp, SEED)
    assert np.abs(total[:, :3] / spp - ref[:, :3]).max() < 1e-12


@pytest.mark.parametrize("pool", [256, 4096])
def test_wavefront_small_pool_many_iterations(gpu, oracle, pool, monkeypatch):
    """A pool far smaller than the path count forces many logic/extend/shade/shadow iterations
    with slot reuse; the image must not change."""
    monkeypatch.setenv("MFX_POOL", str(pool))
    from mafrixraytracing_amd.native import NativeContext
    a = scene("cube_cornell", 40, 24)
    ref = oracle.OracleScene(a).sample(6, SEED)
    with NativeContext(a, seed=SEED) as ctx:
        img = ctx.sample(6)
        tm = ctx.trace_timing()
    assert tm["generations"] > 1
    assert np.array_equal(img, ref)


def test_wavefront_image_is_deterministic(gpu):
    """k_resolve adds each pixel's paths in sample order (no atomics): two runs are bit-identical,
    also across generations (a small pool forces several)."""
    from mafrixraytracing_amd.native import NativeContext
    a = scene("spot", 64, 36)
    with NativeContext(a, seed=SEED) as ctx:
        f1 = ctx.sample(8)
    with NativeContext(a, seed=SEED) as ctx:
        f2 = ctx.sample(8)
    assert np.array_equal(f1, f2)


def test_megakernel_and_wavefront_counters_agree(gpu, monkeypatch):
    """The same per-ray traversal in both pipelines: identical ray counts and visit counters. (The
    wavefront's camera rays run as packets by default, k_camera, whose counters add the packet's
    union of visits; MFX_CAMERA_PACKETS=0 gives them the per-ray traversal compared here.)"""
    from mafrixraytracing_amd.abi import MFX_F_COUNT_STATS, MFX_F_MEGAKERNEL
    from mafrixraytracing_amd.native import NativeContext
    monkeypatch.setenv("MFX_CAMERA_PACKETS", "0")
    a = scene("spot", 96, 54)
    with NativeContext(a, seed=SEED, flags=MFX_F_COUNT_STATS) as w:  # the per-lane kernels on FP16 nodes
        w.sample(2)
        c16 = w.ray_counts()
    monkeypatch.setenv("MFX_NODE_F32", "1")  # the per-lane kernels on the FP32 nodes the megakernel walks
    with NativeContext(a, seed=SEED, flags=MFX_F_COUNT_STATS) as w:
        w.sample(2)
        cw = w.ray_counts()
    with NativeContext(a, seed=SEED, flags=MFX_F_COUNT_STATS | MFX_F_MEGAKERNEL) as m:
        m.sample(2)
        cm = m.ray_counts()
    assert np.array_equal(cw[:4], cm[:4]) and np.array_equal(c16[:4], cm[:4])
    # identical traversal algorithm per ray -> identical visit counts
    assert np.array_equal(cw[4:10], cm[4:10])
    # FP16 boxes contain the FP32 ones: a superset of the visits, the same rays
    assert np.all(c16[4:10] >= cw[4:10])


@pytest.mark.gpu
def test_survey_named_entry_points(gpu):
    """mfx_accumulate_render_rgba8 (SURVEY §8(b)'s name) == mfx_render_rgba8 on a twin context, and
    mfx_stats reports the last call's rays (primary + extension + shadow) and device time."""
    import ctypes as C
    from mafrixraytracing_amd.native import NativeContext
    a = scene("two_spheres_plane", 40, 30)
    with NativeContext(a, seed=SEED) as c1, NativeContext(a, seed=SEED) as c2:
        for _ in range(2):
            r1 = c1.render_rgba8(2)
            r2 = np.empty(40 * 30 * 4, dtype=np.uint8)
            rc = c2.lib.mfx_accumulate_render_rgba8(c2._h, 2, r2.ctypes.data_as(C.POINTER(C.c_uint8)))
            assert rc == 0
            assert np.array_equal(r1, r2)
        rays, sec = c2.stats()
        n = c2.ray_counts()
        assert rays == n[0] + n[1] + n[2] and rays > 0
        assert 0 < sec < 10 and abs(sec * 1e3 - c2.last_trace_ms()) < 1e-9


@pytest.mark.parametrize("name", ["spot", "cube_cornell"])
def test_colored_and_gray_light_records(gpu, oracle, monkeypatch, name):
    """A lit vertex's direct term is recorded as a_v itself for a gray light (one double) and as its
    operands cs and solid otherwise (k_resolve evaluates a_v per channel): a colored light through the
    second form equals the oracle bit for bit, and the scene's own gray light gives the same image and
    frames through either form (MFX_NO_GRAY_LIGHT pins the general one)."""
    from mafrixraytracing_amd.native import NativeContext
    a = scene(name, 40, 24)
    a.light = dict(a.light, intensity=(3.0, 2.5, 1.0))
    ref = oracle.OracleScene(a).sample(6, SEED, sample_base=0)
    with NativeContext(a, seed=SEED) as ctx:
        assert np.array_equal(ctx.sample(6), ref)
    g = scene(name, 40, 24)
    out = []
    for general in (False, True):
        if general:
            monkeypatch.setenv("MFX_NO_GRAY_LIGHT", "1")
        with NativeContext(g, seed=SEED) as ctx, NativeContext(g, seed=SEED, render_ahead=3) as ra:
            out.append((ctx.sample(5), [ra.render_rgba8(1) for _ in range(4)]))
    assert np.array_equal(out[0][0], out[1][0])
    assert all(np.array_equal(x, y) for x, y in zip(out[0][1], out[1][1]))
    assert np.array_equal(out[0][0], oracle.OracleScene(g).sample(5, SEED, sample_base=0))


_SUBPACKET_CHILD = r"""
import os, sys
import numpy as np
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "oracle")); sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import mafrixraytracing_amd.abi as abi
abi._lib = abi.load_library(LIB)
import pyoracle
pyoracle.build()
from conftest import scene
from test_gpu_parity import random_rays
from shadow_packets import tile_shadow_rays
from mafrixraytracing_amd.native import NativeContext
for name in ("spot", "renault", "cube_cornell", "two_spheres_plane"):
    a = scene(name, 96, 54)
    rng = np.random.default_rng(5)
    with NativeContext(a) as ctx:
        srays, tmax = tile_shadow_rays(ctx, a, 2)
        rr = random_rays(a, 4000, rng)
        srays = np.concatenate([srays, rr])
        tmax = np.concatenate([tmax, rng.uniform(0.1, 5.0, len(rr))])
        os.environ.pop("MFX_ANYHIT_PACKET", None)
        single = ctx.any_hit(srays, tmax)
        os.environ["MFX_ANYHIT_PACKET"] = "16"
        packet = ctx.any_hit(srays, tmax)
        os.environ.pop("MFX_ANYHIT_PACKET")
    assert np.array_equal(single, packet), (name, int((single != packet).sum()))
    assert np.array_equal(single, pyoracle.OracleScene(a).any_hit(srays, tmax)), name
    print(name, "ok", len(srays))
"""


def test_shadow_subpackets_answer_like_single_rays(gpu):
    """The 16-lane sub-packet any-hit experiment (anyhit_packet16_kernel, MFX_ANYHIT_PACKET=16; measured
    and lost, so built only into build_variants/pk16.so by the Makefile's `experiments` target, which
    __graft_entry__.build() runs): first-vertex shadow rays in k_shadow's tile order and random rays,
    every answer the per-lane kernel's and the oracle's. The variant runs in a child process (two
    copies of the library in one process would interpose each other's symbols)."""
    import subprocess
    import sys as _sys
    from conftest import ROOT
    lib = os.path.join(ROOT, "build_variants", "pk16.so")
    if not os.path.exists(lib):
        pytest.skip("build_variants/pk16.so not built (make -C mafrixraytracing_amd/csrc experiments)")
    code = f"ROOT = {ROOT!r}; LIB = {lib!r}\n" + _SUBPACKET_CHILD
    r = subprocess.run([_sys.executable, "-c", code], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    assert r.stdout.count(" ok ") == 4, r.stdout


_CONE_CAMERAS = [
    # (scene, camera): the camera on a wall's plane, at a vertex, grazing the floor, inside the
    # mesh, close to it, far and narrow
    ("cube_cornell", {"position": (0.0, 0.0, 0.5), "direction": (0.0, 0.2, -1.0), "fov": 100.0}),
    ("cube_cornell", {"position": (-1.0, 0.0, 0.99), "direction": (1.0, 0.8, -1.0), "fov": 90.0}),
    ("cube_cornell", {"position": (0.0, 1e-7, 0.9), "direction": (0.0, 0.0, -1.0), "fov": 120.0}),
    ("spot", {"position": (0.0, 0.0, 0.0), "direction": (0.3, -0.2, 1.0), "fov": 110.0}),
    ("spot", {"position": (0.33, -0.39, 0.45), "direction": (-0.1, -0.05, -1.0), "fov": 60.0}),
    ("spot", {"position": (240.0, 120.0, -340.0), "direction": (-2.4, -1.2, 3.4), "fov": 0.6}),
    ("renault", None),
]


@pytest.mark.parametrize("name,cam", _CONE_CAMERAS)
def test_camera_packets_at_edge_case_cameras(gpu, oracle, name, cam):
    """Camera-ray packets (k_camera) at cameras on a triangle's plane, at a vertex, grazing a wall,
    inside the mesh, far and narrow: images equal the oracle's bit for bit."""
    from mafrixraytracing_amd.abi import SceneArrays
    from mafrixraytracing_amd.native import NativeContext
    a = scene(name, 40, 24)
    if cam is not None:
        c = dict(a.camera)
        c.update(cam)
        a = SceneArrays(a.prims, a.albedo, a.light, c, a.width, a.height, a.max_depth)
    ref = oracle.OracleScene(a).sample(2, SEED)
    with NativeContext(a, seed=SEED) as ctx:
        img = ctx.sample(2)
    assert np.array_equal(img, ref), np.abs(img - ref).max()
