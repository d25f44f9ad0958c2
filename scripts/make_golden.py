#!/usr/bin/env python3
"""Regenerate tests/golden/oracle_golden.npz: small images, ray counts and hit lists produced by
the CPU oracle (oracle/mfx_oracle.c) for the committed scenes. These pin the oracle (and through
it the GPU) against regressions; they are oracle outputs, not reference (F#) outputs — the
reference cannot run here."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pyoracle  # noqa: E402
from mafrixraytracing_amd.scene_io import load_scene_file  # noqa: E402

SEED = 0x4D414652
CASES = [("two_spheres_plane", 32, 32, 4), ("cornell", 32, 32, 4), ("spot", 48, 27, 2),
         ("cube_cornell", 48, 27, 4), ("renault", 48, 27, 2), ("spot16", 48, 27, 2)]


def rays_for(a, n, seed):
    rng = np.random.default_rng(seed)
    p = a.prims["p"]
    pts = p[a.prims["kind"] != 2][:, :3, :].reshape(-1, 3)
    lo, hi = pts.min(0) - 0.2, pts.max(0) + 0.2
    o = rng.uniform(lo, hi, (n, 3))
    o[: n // 2] = a.camera["position"]
    d = rng.uniform(lo, hi, (n, 3)) - o
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return np.concatenate([o, d], 1)


def main():
    pyoracle.build()
    out = {}
    for name, w, h, spp in CASES:
        a = load_scene_file(os.path.join(ROOT, "scenes", name + ".xml")).with_film(w, h)
        o = pyoracle.OracleScene(a)
        img, st = o.sample(spp, SEED, with_stats=True)
        out[f"{name}/image"] = img
        out[f"{name}/counts"] = st[:4]
        out[f"{name}/spec"] = np.array([w, h, spp])
        rays = rays_for(a, 2000, 11)
        t, prim, _ = o.closest_hit(rays)
        out[f"{name}/rays"] = rays
        out[f"{name}/t"] = t
        out[f"{name}/prim"] = prim
        print(name, img[:, :3].mean(0), st[:4])
    np.savez_compressed(os.path.join(ROOT, "tests", "golden", "oracle_golden.npz"), **out)


if __name__ == "__main__":
    main()
