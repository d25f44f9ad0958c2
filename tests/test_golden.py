"""Committed fixtures (tests/golden/oracle_golden.npz, made by scripts/make_golden.py): the
oracle must reproduce them bit for bit (CPU), and the GPU must match them (gpu)."""
import os

import numpy as np
import pytest

from conftest import ROOT, SEED, scene

G = np.load(os.path.join(ROOT, "tests", "golden", "oracle_golden.npz"))
NAMES = sorted({k.split("/")[0] for k in G.files})


@pytest.mark.parametrize("name", NAMES)
def test_oracle_reproduces_golden(oracle, name):
    w, h, spp = G[f"{name}/spec"].tolist()
    o = oracle.OracleScene(scene(name, w, h))
    img, st = o.sample(spp, SEED, with_stats=True)
    assert np.array_equal(img, G[f"{name}/image"])
    assert np.array_equal(st[:4], G[f"{name}/counts"])
    t, prim, _ = o.closest_hit(G[f"{name}/rays"])
    assert np.array_equal(t, G[f"{name}/t"]) and np.array_equal(prim, G[f"{name}/prim"])


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_gpu_matches_golden(gpu, name):
    from mafrixraytracing_amd.native import NativeContext
    w, h, spp = G[f"{name}/spec"].tolist()
    with NativeContext(scene(name, w, h), seed=SEED) as ctx:
        img = ctx.sample(spp)
        counts = ctx.ray_counts()
        t, prim, _ = ctx.closest_hit(G[f"{name}/rays"])
    ref = G[f"{name}/image"]
    assert np.array_equal(img, ref), np.abs(img - ref).max()  # bit for bit
    assert np.array_equal(counts[:3], G[f"{name}/counts"][:3])
    assert np.array_equal(t, G[f"{name}/t"]) and np.array_equal(prim, G[f"{name}/prim"])
