"""Known-answer tests pinning the CPU oracle, one reference function at a time.

The reference ships no tests, golden images or fixtures and cannot run here (no .NET), so each
expected value below is derived by hand from the F# source (file:line in each test) — an
independent restatement of the arithmetic, not oracle output.
"""
import math

import numpy as np
import pytest

from conftest import SEED


# ---- AABB.hit — IHitable.fs:18-54 ---------------------------------------------------------
def test_aabb_basic_hit_and_tmax(oracle):
    box = ([0, 0, 0], [1, 1, 1])
    assert oracle.kat_aabb(*box, [-1, 0.5, 0.5], [1, 0, 0], 1e-6, 10.0)
    # entry at t = 1: `tmin < tMax` fails for tMax = 0.5
    assert not oracle.kat_aabb(*box, [-1, 0.5, 0.5], [1, 0, 0], 1e-6, 0.5)
    # box behind the origin: `tmax > tMin` fails
    assert not oracle.kat_aabb(*box, [2, 0.5, 0.5], [1, 0, 0], 1e-6, 10.0)


def test_aabb_flat_box_is_hit(oracle):
    """Flat boxes (walls, floor) are common: pmin.y == pmax.y gives tymin == tymax."""
    assert oracle.kat_aabb([0, 0, 0], [1, 0, 1], [0.5, 1, 0.5], [0, -1, 0], 1e-6, 10.0)


def test_aabb_negative_zero_direction_misses(oracle):
    """`dir.x >= 0.` is true for -0.0, so (pmin-o)/-0.0 = +inf becomes tmin: such a ray misses."""
    assert oracle.kat_aabb([0, 0, 0], [1, 0, 1], [0.5, 1, 0.5], [0.0, -1, 0], 1e-6, 10.0)
    assert not oracle.kat_aabb([0, 0, 0], [1, 0, 1], [0.5, 1, 0.5], [-0.0, -1, 0], 1e-6, 10.0)


# ---- Triangle.Hit — Trangle.fs:120-155 ------------------------------------------------------
TRI = [[0, 0, 0], [1, 0, 0], [0, 1, 0]]


def test_triangle_hit_values(oracle):
    hit, t, p, n = oracle.kat_prim_hit(0, TRI, [0.25, 0.25, 1], [0, 0, -1], 1e-6, 1e8)
    assert hit and t == 1.0
    assert list(p) == [0.25, 0.25, 0.0] and list(n) == [0.0, 0.0, 1.0]


def test_triangle_ignores_tmax(oracle):
    hit, t, _, _ = oracle.kat_prim_hit(0, TRI, [0.25, 0.25, 1], [0, 0, -1], 1e-6, 0.5)
    assert hit and t == 1.0  # tMax is never checked (Trangle.fs:148)


def test_triangle_edge_and_backface_rules(oracle):
    # b1 + b2 >= 1 is rejected (the hypotenuse is excluded)
    assert not oracle.kat_prim_hit(0, TRI, [0.5, 0.5, 1], [0, 0, -1], 1e-6, 1e8)[0]
    # two-sided: hit from below
    hit, t, _, n = oracle.kat_prim_hit(0, TRI, [0.25, 0.25, -1], [0, 0, 1], 1e-6, 1e8)
    assert hit and t == 1.0 and list(n) == [0.0, 0.0, 1.0]
    # parallel ray: divisor 0
    assert not oracle.kat_prim_hit(0, TRI, [-1, 0.25, 0], [1, 0, 0], 1e-6, 1e8)[0]
    # origin on the plane: t = 0 is not > tMin
    assert not oracle.kat_prim_hit(0, TRI, [0.25, 0.25, 0], [0, 0, -1], 1e-6, 1e8)[0]


def test_triangle_absolute_divisor_cull(oracle):
    """|s1.e1| < 1e-6 is culled absolutely: a 0.9e-3-sided triangle hit head-on has divisor
    8.1e-7 and is missed; 1e-3-sided has exactly 1e-6 and is hit."""
    big = [[0, 0, 0], [1e-3, 0, 0], [0, 1e-3, 0]]
    small = [[0, 0, 0], [0.9e-3, 0, 0], [0, 0.9e-3, 0]]
    assert oracle.kat_prim_hit(0, big, [2e-4, 2e-4, 1], [0, 0, -1], 1e-6, 1e8)[0]
    assert not oracle.kat_prim_hit(0, small, [2e-4, 2e-4, 1], [0, 0, -1], 1e-6, 1e8)[0]


# ---- Rect.Hit — Rect.fs:11-31 -----------------------------------------------------------------
def test_rect_two_triangles(oracle):
    quad = [[0, 0, 0], [1, 0, 0], [1, 1, 0], [0, 1, 0]]
    for x, y in [(0.75, 0.25), (0.25, 0.75), (0.5, 0.1)]:
        hit, t, p, n = oracle.kat_prim_hit(1, quad, [x, y, 2], [0, 0, -1], 1e-6, 1e8)
        assert hit and t == 2.0 and list(n) == [0.0, 0.0, 1.0]
    assert not oracle.kat_prim_hit(1, quad, [1.5, 0.5, 2], [0, 0, -1], 1e-6, 1e8)[0]


# ---- Sphere.Hit — Sphere.fs:21-43 -------------------------------------------------------------
def test_sphere_roots(oracle):
    sph = [[0, 0, 0], [1, 0, 0]]  # center, radius in p[1][0]
    hit, t, p, n = oracle.kat_prim_hit(2, sph, [0, 0, 5], [0, 0, -1], 1e-6, 1e8)
    # b = -10, c = 24, disc = 4, q = 6, t0 = 6, t1 = 24/6 = 4 -> tmin = 4
    assert hit and t == 4.0 and list(p) == [0, 0, 1.0] and list(n) == [0, 0, 1.0]
    # from inside: t0 = -1 < tMin, so the far root t = 1
    hit, t, _, n = oracle.kat_prim_hit(2, sph, [0, 0, 0], [1, 0, 0], 1e-6, 1e8)
    assert hit and t == 1.0 and list(n) == [1.0, 0, 0]
    # Sphere.Hit does check tMax: both roots beyond tMax = 3
    assert not oracle.kat_prim_hit(2, sph, [0, 0, 5], [0, 0, -1], 1e-6, 3.0)[0]


# ---- PinholeCamera — Camera.fs:96-139 -----------------------------------------------------
def test_camera_scene_xml(oracle):
    """Scene.xml camera: pos (0,1,3), dir (0,0,-1), fov 120, aspect 1 -> half-angle fov/4."""
    h = math.tan(0.5 * 120 * math.pi / 360.0)
    o, d = oracle.kat_camera_ray([0, 1, 3], [0, 0, -1], 120, 1.0, 0.5, 0.5)
    assert list(o) == [0, 1, 3] and np.allclose(d, [0, 0, -1], atol=1e-15)
    o, d = oracle.kat_camera_ray([0, 1, 3], [0, 0, -1], 120, 1.0, 0.0, 0.0)
    ref = np.array([-0.5 * h, 0.5 * h, -0.5])
    assert np.allclose(d, ref / np.linalg.norm(ref), atol=1e-15)
    # effective full horizontal FOV = fov / 2 = 60 degrees
    _, dl = oracle.kat_camera_ray([0, 1, 3], [0, 0, -1], 120, 1.0, 0.0, 0.5)
    assert math.isclose(2 * math.degrees(math.atan2(-dl[0], -dl[2])), 60.0, rel_tol=1e-12)


def test_camera_right_not_normalised(oracle):
    """right = fwd x (0,1,0) is not normalised (Camera.fs:99): looking 45 degrees down, |right|
    = sin(135 deg) = 1/sqrt(2), which narrows the horizontal field of view."""
    _, dc = oracle.kat_camera_ray([0, 0, 0], [0, -1, -1], 90, 1.0, 0.5, 0.5)
    _, dr = oracle.kat_camera_ray([0, 0, 0], [0, -1, -1], 90, 1.0, 1.0, 0.5)
    h = math.tan(0.5 * 90 * math.pi / 360.0)
    fwd = np.array([0, -1, -1]) / math.sqrt(2)
    assert np.allclose(dc, fwd, atol=1e-15)
    # target = pos + 0.5 fwd + 0.5 right, so x / (d . fwd) = |right| = h / sqrt(2)
    assert math.isclose(dr[0] / np.dot(dr, fwd), h / math.sqrt(2), rel_tol=1e-12)


# ---- Triangle.SamplePoint — Trangle.fs:157-169 ---------------------------------------------
def test_tri_sample_point_mapping(oracle):
    v0, v1, v2 = [0, 0, 0], [1, 0, 0], [0, 1, 0]
    p = oracle.kat_tri_sample(v0, v1, v2, 0.3, 0.4)
    sq = math.sqrt(1 - 0.3)
    assert list(p) == [1 - sq, 0.4 * sq, 0.0]
    p = oracle.kat_tri_sample(v0, v1, v2, 0.8, 0.6)  # fold to (0.2, 0.4)
    sq = math.sqrt(1 - (1 - 0.8))
    assert list(p) == [1 - sq, (1 - 0.6) * sq, 0.0]


def test_tri_sample_covers_half_the_triangle(oracle):
    """s2 = v*sqrt(1-u) <= (1-s1)^3 for every sample: only half of each light triangle is
    reachable (area 1/4 of the unit square vs 1/2)."""
    rng = np.random.default_rng(0)
    for tu, tv in rng.uniform(0, 1, (2000, 2)):
        s1, s2, _ = oracle.kat_tri_sample([0, 0, 0], [1, 0, 0], [0, 1, 0], tu, tv)
        assert s2 <= (1 - s1) ** 3 + 1e-12


# ---- NewAreaLight.L — Light.fs:48-56 -------------------------------------------------------
def test_light_L(oracle):
    quad = [[-0.5, 1, 0.5], [-0.5, 1, -0.5], [0.5, 1, -0.5], [0.5, 1, 0.5]]  # area 1, facing -y
    L = oracle.kat_light_L(quad, [0, -1, 0], [10, 10, 10], [0, 2, 0])
    assert list(L) == [5.0, 5.0, 5.0]  # |cos_o| * A / |toLight|^2 = 2 * 1 / 4, times I
    assert list(oracle.kat_light_L(quad, [0, -1, 0], [10, 10, 10], [0, -2, 0])) == [0, 0, 0]


# ---- ACES + post — Scene.fs:273-330 ---------------------------------------------------------
def test_aces_values(oracle):
    assert list(oracle.kat_aces([0, 0, 0])) == [0, 0, 0]
    one = (1 * (2.51 * 1 + 0.03)) / (1 * (2.43 * 1 + 0.59) + 0.14)
    assert list(oracle.kat_aces([1, 1, 1])) == [one] * 3
    # negative radiance (the unclamped cosine, Integrators.fs:52) maps to 2.48 / 1.98 > 1 -> 1
    assert list(oracle.kat_aces([1e6, -1, 0.5])) == [1.0, 1.0, (0.5 * (2.51 * 0.5 + 0.03)) / (0.5 * (2.43 * 0.5 + 0.59) + 0.14)]


def test_post_rgba8_bytes(oracle):
    w, h = 2, 1
    frame = np.array([[0, 0, 0, 1], [1, 1, 1, 1]], dtype=np.float64)  # x-major: pixel (0,0), (1,0)
    rgba = oracle.post_rgba8(frame, w, h)
    v = int(255.99 * math.sqrt((2.51 + 0.03) / (2.43 + 0.59 + 0.14)))
    assert list(rgba) == [0, 0, 0, 255, v, v, v, 255]


# ---- counter RNG -------------------------------------------------------------
def _mix64(z):
    M = (1 << 64) - 1
    z ^= z >> 30
    z = (z * 0xBF58476D1CE4E5B9) & M
    z ^= z >> 27
    z = (z * 0x94D049BB133111EB) & M
    return z ^ (z >> 31)


def test_rng_stream_matches_spec(oracle):
    M = (1 << 64) - 1
    for pixel, sample in [(0, 0), (12345, 7), (2073599, 63)]:
        key = _mix64(SEED ^ _mix64(((pixel << 32) | sample) & M))
        ref = [(_mix64((key + n * 0x9E3779B97F4A7C15) & M) >> 11) * 2.0 ** -53 for n in range(1, 9)]
        assert list(oracle.rng_draws(SEED, pixel, sample, 8)) == ref


def test_hemisphere_rejection_sampler(oracle):
    """GetRandomInUnitSphere (Material.fs:9-14): n.p > 0, |p| < 1, 3 draws per trial; the
    normalised result is uniform on the hemisphere (E[cos] = 1/2)."""
    n = np.array([0.0, 0.6, 0.8])
    cos, draws = [], []
    for s in range(4000):
        wi, k = oracle.kat_hemisphere(n, SEED, 5, s)
        assert abs(np.linalg.norm(wi) - 1) < 1e-15 and np.dot(wi, n) > 0 and k % 3 == 0
        cos.append(np.dot(wi, n))
        draws.append(k)
    assert abs(np.mean(cos) - 0.5) < 0.02
    assert abs(np.mean(draws) / 3 - 1 / ((2 * math.pi / 3) / 8)) < 0.25  # acceptance (2pi/3)/8


def test_oracle_image_determinism(oracle):
    from conftest import scene
    a = scene("two_spheres_plane", 16, 16)
    o = oracle.OracleScene(a)
    f1 = o.sample(2, SEED, nthreads=1)
    f2 = o.sample(2, SEED, nthreads=4)
    assert np.array_equal(f1, f2)
