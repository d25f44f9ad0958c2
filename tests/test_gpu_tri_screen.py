"""The FP32 triangle screen (mfx_trace_common.h: tri_skip32) against the exact FP64 Triangle.Hit
(Trangle.fs:120-155) on the device (mfx_tri_screen_selftest). The screen may only skip a slot whose
FP64 test misses, or hits at beyond < t < tMax (a closest query's candidate that cannot win); the
cases aim at every decision boundary of the FP64 test: the |div| < 1e-6 cull, b1 = 0 / 1, b2 = 0,
b1 + b2 = 1 (edges and vertices), t = tMin, t = beyond, grazing rays and mixed scales."""
import numpy as np
import pytest

from conftest import scene

pytestmark = pytest.mark.gpu

TMIN, TMAX = 1e-6, 99999999.0


def _unit(v):
    return v / np.linalg.norm(v, axis=-1, keepdims=True)


def _cases(rng, n):
    scale = 10.0 ** rng.uniform(-3, 2.5, size=(n, 1))
    v0 = rng.uniform(-1, 1, size=(n, 3)) * scale * rng.choice([1.0, 30.0], size=(n, 1))
    e1 = rng.normal(size=(n, 3)) * scale
    e2 = rng.normal(size=(n, 3)) * scale
    d = _unit(rng.normal(size=(n, 3)))
    kind = rng.integers(0, 8, size=n)
    b1 = rng.uniform(-0.2, 1.2, size=n)
    b2 = rng.uniform(-0.2, 1.2, size=n)
    b1 = np.where(kind == 1, 0.0, b1)                       # on edge v0-v2
    b2 = np.where(kind == 2, 0.0, b2)                       # on edge v0-v1
    b2 = np.where(kind == 3, 1.0 - b1, b2)                  # on edge v1-v2
    b1 = np.where(kind == 4, rng.choice([0.0, 1.0], size=n), b1)  # vertices
    b2 = np.where(kind == 4, 0.0, b2)
    t = np.where(rng.random(n) < 0.3, rng.uniform(-1, 1, size=n) * 1e-6 + TMIN, rng.uniform(-2, 5, size=n) * scale[:, 0])
    p = v0 + b1[:, None] * e1 + b2[:, None] * e2
    o = p - t[:, None] * d
    # grazing / near-cull: the direction (almost) in the triangle's plane
    nrm = _unit(np.cross(e1, e2))
    graze = kind == 5
    d_g = _unit(_unit(e1) + nrm * rng.normal(size=(n, 1)) * 10.0 ** rng.uniform(-12, -3, size=(n, 1)))
    d = np.where(graze[:, None], d_g, d)
    o = np.where(graze[:, None], p - t[:, None] * d, o)
    # tiny triangles around the 1e-6 cull (|div| = 2 area |cos|)
    tiny = kind == 6
    s = 10.0 ** rng.uniform(-3.6, -2.6, size=(n, 1))
    e1 = np.where(tiny[:, None], e1 / scale * s, e1)
    e2 = np.where(tiny[:, None], e2 / scale * s, e2)
    beyond = np.where(rng.random(n) < 0.5, np.inf, np.abs(t) * (1 + rng.uniform(-1e-6, 1e-6, size=n)))
    beyond = np.where(rng.random(n) < 0.2, rng.uniform(0, 10, size=n) * scale[:, 0], beyond)
    rec = np.concatenate([o, d, v0, e1, e2, np.full((n, 1), TMIN), beyond[:, None], np.full((n, 1), TMAX)], 1)
    return rec


def _check(rec):
    from mafrixraytracing_amd.native import tri_screen_selftest
    hit, t, skip = tri_screen_selftest(rec)
    beyond, tmax = rec[:, 16], rec[:, 17]
    bad = skip & hit & ~((t > beyond) & (t < tmax))
    assert not bad.any(), f"{bad.sum()} wrong skips, e.g. {rec[np.argmax(bad)].tolist()} t={t[np.argmax(bad)]}"
    return hit, skip


def test_screen_never_skips_a_live_candidate(gpu):
    rng = np.random.default_rng(1234)
    hits = skips = misses = 0
    for _ in range(8):
        rec = _cases(rng, 250_000)
        hit, skip = _check(rec)
        hits += hit.sum()
        misses += (~hit).sum()
        skips += (skip & ~hit).sum()
    assert hits > 100_000 and misses > 100_000
    # it decides most misses (the point of the screen)
    assert skips > 0.6 * misses, (skips, misses)


def test_screen_on_scene_triangles(gpu):
    """Spot's triangles (as the leaf test sees them) with rays from the camera and from surface points."""
    from mafrixraytracing_amd.native import NativeContext
    a = scene("spot", 32, 18)
    rng = np.random.default_rng(7)
    tri = a.prims[a.prims["kind"] == 0]
    k = rng.integers(0, len(tri), size=400_000)
    v = tri["p"][k]
    v0, e1, e2 = v[:, 0], v[:, 1] - v[:, 0], v[:, 2] - v[:, 0]
    o = np.where(rng.random((len(k), 1)) < 0.5, np.array(a.camera["position"])[None, :],
                 v[rng.integers(0, len(k), size=len(k)), 0] + rng.normal(size=(len(k), 3)) * 1e-3)
    target = v0 + rng.uniform(-0.1, 0.7, size=(len(k), 1)) * e1 + rng.uniform(-0.1, 0.7, size=(len(k), 1)) * e2
    d = _unit(target - o)
    beyond = np.where(rng.random(len(k)) < 0.5, np.inf, rng.uniform(0, 3, size=len(k)))
    rec = np.concatenate([o, d, v0, e1, e2, np.full((len(k), 1), TMIN), beyond[:, None], np.full((len(k), 1), TMAX)], 1)
    hit, skip = _check(rec)
    assert hit.any() and (skip & ~hit).any()
    _ = NativeContext
