#!/usr/bin/env python3
"""16-lane sub-packets for first-vertex shadow rays (VERDICT r04 Next #4a): an isolated A/B of the
traversal itself. First-vertex shadow rays are made the way k_shadow lists them — camera rays of
8x8 tiles (tile-major, one jittered sample per pixel, PinholeCamera as mfx_scene.cpp builds it),
their closest hits through the library, a light point sampled per hit, the hits compacted in tile
order (a shading batch is 64 consecutive hits of a scan window) — and traced twice through
mfx_any_hit: one ray per lane (anyhit_kernel, the per-lane walk) and four 16-lane sub-packets
per wave (anyhit_packet16_kernel, MFX_ANYHIT_PACKET=16). Answers must agree bit for bit; the
kernels' device times come from the rocprofv3 kernel trace of this script (gpu_run.sh step
`subpk`). Prints one JSON line with the ray count and the occluded fraction."""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def pinhole(cam):
    """(position, topleft, right, down) of PinholeCamera (Camera.fs:96-133, mfx_scene.cpp)."""
    def nz(v):
        v = np.asarray(v, dtype=np.float64)
        return v / np.linalg.norm(v)
    fwd = nz(cam["direction"])
    hori0 = np.cross(fwd, np.array([0.0, 1.0, 0.0]))
    vert0 = np.cross(hori0, fwd)
    hori = np.tan(0.5 * cam["fov"] * np.pi / 360.0)
    up, right = vert0 * (hori / cam["aspect"]), hori0 * hori
    pos = np.asarray(cam["position"], dtype=np.float64)
    tl = pos + fwd * 0.5 - right * 0.5 + up * 0.5
    return pos, tl, right, -up


def tile_shadow_rays(ctx, arrays, spp=1, seed=7):
    """First-vertex shadow rays in k_shadow's listing order: (rays n x 6, tmax n)."""
    W, H = arrays.width, arrays.height
    rng = np.random.default_rng(seed)
    tx, ty = (W + 7) // 8, (H + 7) // 8
    t = np.arange(tx * ty * 64)
    tile, within = t // 64, t % 64
    x = (tile % tx) * 8 + within % 8
    y = (tile // tx) * 8 + within // 8
    keep = (x < W) & (y < H)
    x, y = x[keep], y[keep]
    pos, tl, right, down = pinhole(arrays.camera)
    L = np.asarray(arrays.light["p"], dtype=np.float64)
    out_r, out_t = [], []
    for _ in range(spp):
        u = (x + rng.uniform(0, 1, x.size)) / W
        v = (y + rng.uniform(0, 1, y.size)) / H
        tgt = tl + right * u[:, None] + down * v[:, None]
        d = tgt - pos
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        rays = np.concatenate([np.broadcast_to(pos, d.shape), d], axis=1)
        th, prim, _ = ctx.closest_hit(rays)
        hit = prim >= 0
        hp = rays[hit, :3] + rays[hit, 3:] * th[hit, None]
        uv = rng.uniform(0, 1, size=(hit.sum(), 2))
        lp = L[0] + uv[:, :1] * (L[1] - L[0]) + uv[:, 1:] * (L[3] - L[0])
        to = lp - hp
        dist = np.linalg.norm(to, axis=1)
        out_r.append(np.concatenate([hp, to / dist[:, None]], axis=1))
        out_t.append(dist - 1e-6)
    return np.concatenate(out_r), np.concatenate(out_t)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default=os.path.join(ROOT, "scenes", "spot.xml"))
    ap.add_argument("--spp", type=int, default=4)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--lib", default=os.path.join(ROOT, "build_variants", "pk16.so"),
                    help="the experiment build that carries anyhit_packet16_kernel (Makefile `experiments`)")
    a = ap.parse_args()
    import mafrixraytracing_amd.abi as abi
    abi._lib = abi.load_library(a.lib)
    from mafrixraytracing_amd.native import DEFAULT_SEED, NativeContext
    from mafrixraytracing_amd.scene_io import load_scene_file
    arr = load_scene_file(a.scene)
    with NativeContext(arr, seed=DEFAULT_SEED) as ctx:
        rays, tmax = tile_shadow_rays(ctx, arr, a.spp)
        res = {}
        for mode in ("per_lane", "packet16"):
            if mode == "packet16":
                os.environ["MFX_ANYHIT_PACKET"] = "16"
            else:
                os.environ.pop("MFX_ANYHIT_PACKET", None)
            for _ in range(a.reps):
                res[mode] = ctx.any_hit(rays, tmax)
        os.environ.pop("MFX_ANYHIT_PACKET", None)
    same = bool(np.array_equal(res["per_lane"], res["packet16"]))
    print(json.dumps({"scene": os.path.basename(a.scene), "rays": int(len(rays)), "spp": a.spp,
                      "occluded_frac": round(float(res["per_lane"].mean()), 4), "answers_equal": same,
                      "note": "device times: rocprofv3 kernel stats of anyhit_kernel<false> vs anyhit_packet16_kernel<false>"}))
    return 0 if same else 1


if __name__ == "__main__":
    sys.exit(main())
