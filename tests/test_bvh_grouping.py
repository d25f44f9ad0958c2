"""Reference heap-BVH leaf grouping (BvhNode.fs:24-61) — three implementations must agree:
the oracle (C), the product's host builder (C++, via the host-only mfx_build_leaves), and the
pure-Python restatement below (including .NET 6's introsort tie order, which F#'s
Array.sortInPlaceBy reaches with a null comparer). Runs on CPU."""
import numpy as np
import pytest

from conftest import scene


# ---- pure-Python restatement ----------------------------------------------------------------
def _net_sort(keys, vals):
    k, v = keys, vals

    def swap(i, j):
        k[i], k[j] = k[j], k[i]
        v[i], v[j] = v[j], v[i]

    def sig(i, j):
        if k[i] > k[j]:
            swap(i, j)

    def insertion(lo, n):
        for i in range(n - 1):
            t, tv = k[lo + i + 1], v[lo + i + 1]
            j = i
            while j >= 0 and t < k[lo + j]:
                k[lo + j + 1], v[lo + j + 1] = k[lo + j], v[lo + j]
                j -= 1
            k[lo + j + 1], v[lo + j + 1] = t, tv

    def down(lo, i, n):
        d, dv = k[lo + i - 1], v[lo + i - 1]
        while i <= n >> 1:
            c = 2 * i
            if c < n and k[lo + c - 1] < k[lo + c]:
                c += 1
            if not (d < k[lo + c - 1]):
                break
            k[lo + i - 1], v[lo + i - 1] = k[lo + c - 1], v[lo + c - 1]
            i = c
        k[lo + i - 1], v[lo + i - 1] = d, dv

    def heap(lo, n):
        for i in range(n >> 1, 0, -1):
            down(lo, i, n)
        for i in range(n, 1, -1):
            swap(lo, lo + i - 1)
            down(lo, 1, i - 1)

    def part(lo, n):
        hi, mid = lo + n - 1, lo + ((n - 1) >> 1)
        sig(lo, mid); sig(lo, hi); sig(mid, hi)
        piv = k[mid]
        swap(mid, hi - 1)
        l, r = lo, hi - 1
        while l < r:
            l += 1
            while piv > k[l]:
                l += 1
            r -= 1
            while piv < k[r]:
                r -= 1
            if l >= r:
                break
            swap(l, r)
        if l != hi - 1:
            swap(l, hi - 1)
        return l - lo

    def intro(lo, n, depth):
        while n > 1:
            if n <= 16:
                if n == 2:
                    sig(lo, lo + 1)
                elif n == 3:
                    sig(lo, lo + 1); sig(lo, lo + 2); sig(lo + 1, lo + 2)
                else:
                    insertion(lo, n)
                return
            if depth == 0:
                heap(lo, n)
                return
            depth -= 1
            p = part(lo, n)
            intro(lo + p + 1, n - p - 1, depth)
            n = p

    n = len(k)
    if n >= 2:
        intro(0, n, 2 * (n.bit_length() - 1 + 1))


def py_leaves(lo, hi):
    """Bvh.Build over prim boxes (lo[i], hi[i]) -> (indices, leaf_first, leaf_count)."""
    n = len(lo)
    idx = list(range(n))
    lf, lc = [], []

    def bound(f, c):
        ids = idx[f:f + c]
        return lo[ids].min(0), hi[ids].max(0)

    def sub(f, c, b):
        if c <= 3:
            lf.append(f)
            lc.append(c)
            return
        d = b[1] - b[0]
        axis = 0 if (d[0] > d[1] and d[0] > d[2]) else (1 if d[1] > d[2] else 2)
        ids = idx[f:f + c]
        keys = [lo[i][axis] + (hi[i][axis] - lo[i][axis]) * 0.5 for i in ids]
        vals = list(ids)
        _net_sort(keys, vals)
        idx[f:f + c] = vals
        left = c // 2
        sub(f, left, bound(f, left))
        sub(f + left, c - left, bound(f + left, c - left))

    sub(0, n, bound(0, n))
    return np.array(idx), np.array(lf), np.array(lc)


def tri_scene(verts):
    """SceneArrays of triangles from an (n,3,3) array (film/camera irrelevant here)."""
    from mafrixraytracing_amd.abi import PRIM_DTYPE, SceneArrays
    prims = np.zeros(len(verts), dtype=PRIM_DTYPE)
    prims["kind"] = 0
    prims["p"][:, :3, :] = verts
    light = {"p": [[-1, 5, 1], [-1, 5, -1], [1, 5, -1], [1, 5, 1]], "normal": [0, -1, 0], "intensity": [1, 1, 1]}
    cam = {"position": [0, 0, 10], "direction": [0, 0, -1], "fov": 90, "aspect": 1.0}
    return SceneArrays(prims, np.array([[0.5, 0.5, 0.5]]), light, cam, 8, 8)


def boxes(verts):
    return verts.min(1), verts.max(1)


@pytest.mark.parametrize("n,quant", [(1, 0), (2, 0), (3, 0), (4, 0), (5, 0), (17, 0), (40, 3), (200, 2),
                                     (257, 0), (1000, 4), (3000, 0)])
def test_three_implementations_agree(oracle, n, quant):
    from mafrixraytracing_amd.abi import build_leaves
    rng = np.random.default_rng(n * 31 + quant)
    c = rng.uniform(-1, 1, (n, 1, 3))
    if quant:  # quantised centres -> many exact ties in the sort keys
        c = np.round(c * quant) / quant
    verts = c + rng.uniform(-0.05, 0.05, (n, 3, 3))
    if quant:
        verts = c + np.array([[0.02, 0, 0], [-0.01, 0.02, 0], [-0.01, -0.02, 0.01]])[None]
    a = tri_scene(verts)
    pi, pf, pc = py_leaves(*boxes(a.prims["p"][:, :3, :]))
    oi, of, oc = oracle.OracleScene(a).bvh_leaves()
    gi, gf, gc, info = build_leaves(a)
    assert np.array_equal(oi, pi) and np.array_equal(of, pf) and np.array_equal(oc, pc)
    assert np.array_equal(gi, pi) and np.array_equal(gf, pf) and np.array_equal(gc, pc)
    assert info["clusters"] == len(pf)
    assert set(pc.tolist()) <= {1, 2, 3}


def test_all_equal_keys_follow_dotnet_order(oracle):
    """Every key equal: the order .NET's introsort leaves them in (not a stable sort)."""
    from mafrixraytracing_amd.abi import build_leaves
    verts = np.tile(np.array([[[0, 0, 0], [1, 0, 0], [0, 1, 0]]], dtype=np.float64), (64, 1, 1))
    verts[:, :, 2] += np.arange(64)[:, None] * 1e-9  # distinct z, equal x/y keys on the split axis
    a = tri_scene(verts)
    pi, pf, pc = py_leaves(*boxes(a.prims["p"][:, :3, :]))
    gi, gf, gc, _ = build_leaves(a)
    assert np.array_equal(gi, pi)


@pytest.mark.parametrize("n,quant", [(20000, 0), (40000, 6)])
def test_threaded_grouping_matches_oracle(oracle, n, quant):
    """Ranges of >= 8,192 primitives split onto host threads (mfx_scene.cpp RefBvh): the leaves and
    their order equal the oracle's sequential recursion, with and without tied keys."""
    from mafrixraytracing_amd.abi import build_leaves
    rng = np.random.default_rng(n + quant)
    c = rng.uniform(-1, 1, (n, 1, 3))
    if quant:
        c = np.round(c * quant) / quant
    verts = c + rng.uniform(-0.05, 0.05, (n, 3, 3))
    a = tri_scene(verts)
    oi, of, oc = oracle.OracleScene(a).bvh_leaves()
    gi, gf, gc, _ = build_leaves(a)
    assert np.array_equal(gi, oi) and np.array_equal(gf, of) and np.array_equal(gc, oc)


@pytest.mark.parametrize("name", ["cornell", "cube_cornell", "spot", "two_spheres_plane", "renault", "spot16"])
def test_scene_grouping_matches_oracle(oracle, name):
    from mafrixraytracing_amd.abi import build_leaves
    a = scene(name, 8, 8)
    oi, of, oc = oracle.OracleScene(a).bvh_leaves()
    gi, gf, gc, info = build_leaves(a)
    assert np.array_equal(gi, oi) and np.array_equal(gf, of) and np.array_equal(gc, oc)
    assert 1 <= info["stack"] <= 96  # LDS traversal stack entries per lane
