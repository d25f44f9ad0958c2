"""The exact FP32 screen in front of the reference-leaf box test (mfx_trace_common.h:
aabb_screen32) never contradicts the FP64 AABB.hit (IHitable.fs:18-54) it stands in for.

Every case the screen decides must match the FP64 answer bit for bit; the cases built to sit on
the decision boundaries (rays through box edges, corners and faces, flat boxes, tMin/tMax at the
entry and exit values, zero, tiny and negative-zero direction components, huge coordinates) must
either match or be left to the FP64 test. The FP64 answers are also checked against a numpy
restatement of AABB.hit, so the device division is the reference's."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def aabb_hit_np(r):
    """AABB.hit (IHitable.fs:18-54), vectorised: entry/exit per axis by the sign of d, the two
    early-outs, then tmin < tMax && tmax > tMin."""
    lo, hi, o, d, tmin_q, tmax_q = r[:, 0:3], r[:, 3:6], r[:, 6:9], r[:, 9:12], r[:, 12], r[:, 13]
    with np.errstate(all="ignore"):
        a = (lo - o) / d
        b = (hi - o) / d
    pos = d >= 0.0
    mn = np.where(pos, a, b)
    mx = np.where(pos, b, a)
    tmin, tmax = mn[:, 0].copy(), mx[:, 0].copy()
    ok = ~((tmin > mx[:, 1]) | (mn[:, 1] > tmax))
    tmin = np.where(mn[:, 1] > tmin, mn[:, 1], tmin)
    tmax = np.where(mx[:, 1] < tmax, mx[:, 1], tmax)
    ok &= ~((tmin > mx[:, 2]) | (mn[:, 2] > tmax))
    tmin = np.where(mn[:, 2] > tmin, mn[:, 2], tmin)
    tmax = np.where(mx[:, 2] < tmax, mx[:, 2], tmax)
    return (ok & (tmin < tmax_q) & (tmax > tmin_q)).astype(np.int32)


def cases(rng, n):
    out = []
    # 1. general: random boxes, origins and unit directions, the query interval of closest hits
    lo = rng.uniform(-10, 10, (n, 3))
    hi = lo + rng.exponential(1.0, (n, 3))
    o = rng.uniform(-20, 20, (n, 3))
    d = rng.normal(size=(n, 3))
    aim = rng.random(n) < 0.5  # half of them aimed into the box
    d[aim] = rng.uniform(lo[aim], hi[aim]) - o[aim]
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    out.append(np.c_[lo, hi, o, d, np.full(n, 1e-6), np.full(n, 99999999.0)])
    # 2. rays aimed at a box corner, an edge point or a face point, nudged by a few ulps
    lo = rng.uniform(-5, 5, (n, 3))
    hi = lo + rng.uniform(0, 2, (n, 3))
    tgt = np.where(rng.random((n, 3)) < 0.5, lo, hi)
    free = rng.integers(0, 4, n)  # 0: corner; 1..3: that axis slides inside the box
    for ax in range(3):
        m = free == ax + 1
        tgt[m, ax] = rng.uniform(lo[m, ax], hi[m, ax])
    o = rng.uniform(-20, 20, (n, 3))
    d = tgt - o
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    d = d + d * rng.integers(-4, 5, (n, 3)) * 2.0 ** -52
    out.append(np.c_[lo, hi, o, d, np.full(n, 1e-6), np.full(n, 99999999.0)])
    # 3. flat boxes (a quad's leaf: zero extent on one axis), rays through their plane
    lo = rng.uniform(-5, 5, (n, 3))
    hi = lo + rng.uniform(0, 2, (n, 3))
    ax = rng.integers(0, 3, n)
    hi[np.arange(n), ax] = lo[np.arange(n), ax]
    o = rng.uniform(-20, 20, (n, 3))
    d = rng.uniform(lo, hi) - o
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    out.append(np.c_[lo, hi, o, d, np.full(n, 1e-6), np.full(n, 99999999.0)])
    # 4. tMax / tMin at the FP64 entry and exit values themselves, and a few ulps either side
    base = out[0][: n].copy()
    with np.errstate(all="ignore"):
        a = (base[:, 0:3] - base[:, 6:9]) / base[:, 9:12]
        b = (base[:, 3:6] - base[:, 6:9]) / base[:, 9:12]
    entry = np.minimum(a, b).max(axis=1)
    exit_ = np.maximum(a, b).min(axis=1)
    k = rng.integers(-3, 4, n)
    t1 = base.copy()
    t1[:, 13] = entry + np.abs(entry) * k * 2.0 ** -52   # shadow-ray style tMax at the box entry
    t1[:, 12] = -1.0
    t2 = base.copy()
    t2[:, 12] = exit_ + np.abs(exit_) * k * 2.0 ** -52   # tMin at the box exit
    out += [t1, t2]
    # 5. axis-aligned and near-axis directions: 0, -0.0, subnormal and tiny components
    t3 = out[0][: n].copy()
    comp = rng.integers(0, 3, n)
    vals = np.array([0.0, -0.0, 5e-324, -1e-310, 1e-30, -1e-19, 2.0 ** -60, 3e-18])
    t3[np.arange(n), 9 + comp] = vals[rng.integers(0, len(vals), n)]
    out.append(t3)
    # 6. huge and tiny coordinates, and a huge query interval
    t4 = out[0][: n].copy()
    t4[:, 0:9] *= rng.choice([1e-25, 1e-12, 1e12, 1e19, 1e25], (n, 1))
    t4[:, 13] = rng.choice([99999999.0, 1e30, np.inf], n)
    out.append(t4)
    rec = np.concatenate(out)
    # no triangle of their own: a degenerate one at the box's lo corner (its vertex box lies inside)
    return np.c_[rec, rec[:, 0:3], np.zeros((len(rec), 7))]


def triangle_cases(rng, n, flat=False):
    """Triangles as the traversal slots hold them (v0, e1 = v1 - v0, e2 = v2 - v0 in FP64) inside
    reference-leaf boxes that are their own vertex box or its union with up to two neighbours,
    and rays aimed at points of the triangle: interior, within 1e-7 of an edge, or a vertex."""
    scale = rng.choice([1e-3, 1e-2, 1.0, 10.0], (n, 1))
    c = rng.uniform(-10, 10, (n, 3))
    v = c[:, None, :] + rng.normal(size=(n, 3, 3)) * scale[:, :, None]
    if flat:  # axis-aligned triangles (a quad's halves): one coordinate shared by all vertices
        ax = rng.integers(0, 3, n)
        v[np.arange(n), :, ax] = v[np.arange(n), 0, ax][:, None]
    lo, hi = v.min(axis=1), v.max(axis=1)
    for _ in range(2):
        m = rng.random(n) < 0.3
        w = c[:, None, :] + rng.normal(size=(n, 3, 3)) * scale[:, :, None]
        lo[m] = np.minimum(lo[m], w[m].min(axis=1))
        hi[m] = np.maximum(hi[m], w[m].max(axis=1))
    bc = rng.dirichlet([1, 1, 1], n)
    near = rng.random(n)
    e = rng.integers(0, 3, n)
    bc[near < 0.2, e[near < 0.2]] = 1e-7
    bc[(near >= 0.2) & (near < 0.3)] = np.eye(3)[e[(near >= 0.2) & (near < 0.3)]]
    bc /= bc.sum(axis=1, keepdims=True)
    tgt = np.einsum("nk,nkj->nj", bc, v)
    o = tgt + rng.normal(size=(n, 3)) * rng.choice([0.01, 1.0, 20.0], (n, 1))
    d = tgt - o
    dist = np.linalg.norm(d, axis=1)
    d /= dist[:, None]
    tmax = np.where(rng.random(n) < 0.5, 99999999.0, dist * rng.choice([0.5, 1 - 1e-9, 1.0, 1 + 1e-9, 2.0], n))
    return np.c_[lo, hi, o, d, np.full(n, 1e-6), tmax, v[:, 0], v[:, 1] - v[:, 0], v[:, 2] - v[:, 0], np.zeros(n)]


def test_screen_agrees_with_fp64_aabb():
    from mafrixraytracing_amd.native import aabb_selftest
    rng = np.random.default_rng(20261016)
    rec = cases(rng, 200_000)
    exact, screen, _ = aabb_selftest(rec)
    assert np.array_equal(exact, aabb_hit_np(rec))     # the device test is the reference's
    assert set(np.unique(screen)) <= {-1, 0, 1}
    decided = screen >= 0
    bad = np.flatnonzero(decided & (screen != exact))
    assert bad.size == 0, rec[bad[:5]]
    # general cases are nearly all decided in FP32; the boundary families mostly fall back
    n = 200_000
    for f in range(len(rec) // n):
        print(f"family {f + 1}: decided {decided[f * n:(f + 1) * n].mean():.4f} hits {exact[f * n:(f + 1) * n].mean():.3f}")
    assert decided[:n].mean() > 0.995
    assert (exact[:n] == 1).sum() > 1000 and (exact[:n] == 0).sum() > 1000
    # zero and subnormal direction components always go to the FP64 test
    t3 = rec[5 * n: 6 * n]
    small = (np.abs(t3[:, 9:12]) < 2.0 ** -60).any(axis=1)
    assert (screen[5 * n: 6 * n][small] == -1).all()


def test_vertex_box_proof_never_contradicts_fp64_aabb():
    """tri_box_pass (mfx_trace_common.h), which lets a triangle winner skip reading its reference
    leaf's box: whenever it claims the box test passes, the FP64 test on the real box passes."""
    from mafrixraytracing_amd.native import aabb_selftest
    rng = np.random.default_rng(7)
    n = 200_000
    fams = [triangle_cases(rng, n), triangle_cases(rng, n, flat=True), cases(rng, n // 4)]
    rec = np.concatenate(fams)
    exact, _, proof = aabb_selftest(rec)
    assert np.array_equal(exact, aabb_hit_np(rec))
    bad = np.flatnonzero((proof == 1) & (exact != 1))
    assert bad.size == 0, rec[bad[:5]]
    for f, name in enumerate(["triangles", "flat triangles"]):
        e, p = exact[f * n:(f + 1) * n], proof[f * n:(f + 1) * n]
        closest = rec[f * n:(f + 1) * n, 13] == 99999999.0  # the closest-hit query interval
        print(f"{name}: box test passes {e.mean():.4f}, proved {p.mean():.4f} ({p[e == 1].mean():.4f} of passes; "
              f"{p[closest & (e == 1)].mean():.4f} of closest-hit passes)")
        # most closest-hit winners never read their box (a third of these rays hit within 1e-7 of
        # an edge or at a vertex); tMax within 1e-9 of t is left to the FP64 test by design
        assert p[closest & (e == 1)].mean() > 0.8
