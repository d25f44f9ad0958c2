"""The oracle's "fast" mode (the CPU baseline's second figure): a SAH BVH2 with
tMax culling and any-hit shadows. It is not the reference algorithm, so it is checked for what it
is: the same integrator and RNG stream, the same path set and ray counts, and radiance equal to
strict's on (almost) every path — it can differ only where the reference's missing tMax check in
Triangle.Hit (the leaf quirk) decides an occlusion. CPU only."""
import numpy as np
import pytest

from conftest import SEED, scene


@pytest.mark.parametrize("name", ["cornell", "spot", "two_spheres_plane"])
def test_fast_mode_matches_strict_on_nearly_every_path(oracle, name):
    a = scene(name, 96, 54)
    o = oracle.OracleScene(a)
    rng = np.random.default_rng(3)
    n = 20000
    px, py, sm = rng.integers(0, 96, n), rng.integers(0, 54, n), rng.integers(0, 16, n)
    s_out, s_st = o.paths(px, py, sm, SEED, mode="strict")
    f_out, f_st = o.paths(px, py, sm, SEED, mode="fast")
    assert np.array_equal(s_st[:4], f_st[:4])  # same paths, same rays traced
    same = np.all(np.abs(s_out - f_out) <= 1e-12 * np.maximum(1.0, np.abs(s_out)), axis=1)
    assert same.mean() >= 0.995, same.mean()
    with pytest.raises(KeyError):
        o.paths(px[:4], py[:4], sm[:4], SEED, mode="quick")
