"""SURVEY.md §8(c)'s statistical check of the oracle's semantics: the reference draws the
Lambertian bounce by rejection from the unit ball (GetRandomInUnitSphere, Material.fs:9-14), whose
direction is uniform on the hemisphere around the geometric normal. The oracle's "direct" mode
draws that distribution by inversion instead (a different sample sequence). Both estimate the same
image, so their difference is pure noise: its RMSE over pixels falls as 1/sqrt(spp), and its mean
stays within the noise (no bias). A sampler that drifted from the reference's distribution (a
cosine-weighted or normal-flipped hemisphere, say) would leave a floor the RMSE stops at."""
import numpy as np
import pytest

from conftest import SEED, scene

W, H = 24, 14
SPPS = (16, 64, 256, 1024)


def images(o, spp, mode, seed):
    px, py, smp = np.meshgrid(np.arange(W), np.arange(H), np.arange(spp), indexing="ij")
    out, _ = o.paths(px.ravel(), py.ravel(), smp.ravel(), seed, mode=mode)
    return out.reshape(W * H, spp, 3).mean(axis=1)


@pytest.mark.parametrize("name", ["cube_cornell", "two_spheres_plane"])
def test_rejection_and_direct_hemisphere_agree_in_distribution(oracle, name):
    o = oracle.OracleScene(scene(name, W, H))
    rmse, bias = [], []

    def z(d):  # mean difference against its own standard error (pixels x channels independent)
        return abs(d.mean()) / (d.std(ddof=1) / np.sqrt(d.size))

    for spp in SPPS:
        a = images(o, spp, "strict", SEED)
        b = images(o, spp, "direct", SEED ^ 0x5A5A)
        d = a - b
        rmse.append(np.sqrt((d ** 2).mean()))
        bias.append(z(d))
    # negative control: the same statistic sees a 2 % gain error at the largest spp (z ~ 11)
    assert z(a * 1.02 - b) > 6.0
    rmse = np.array(rmse)
    ratios = rmse[1:] / rmse[:-1]  # expect 1/2 per 4x spp
    assert np.all((ratios > 0.35) & (ratios < 0.7)), (rmse, ratios)
    assert rmse[-1] / rmse[0] < 0.2, rmse  # 1/8 expected over 64x spp: no floor
    assert max(bias) < 4.5, bias
