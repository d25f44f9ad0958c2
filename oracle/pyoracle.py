"""ctypes wrapper of the CPU oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg — never by the product package. See mfx_oracle.c for what it restates and
its parity status.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from mafrixraytracing_amd.abi import (MfxPinhole, MfxPrim, MfxQuadLight, MfxSceneDesc, SceneArrays,
                                      dptr, iptr)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, "liboracle.so")
_lib = None

_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int32)


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        L.oracle_create.restype = C.c_void_p
        L.oracle_create.argtypes = [C.POINTER(MfxSceneDesc)]
        L.oracle_destroy.argtypes = [C.c_void_p]
        L.oracle_sample.argtypes = [C.c_void_p, C.c_uint64, C.c_int32, C.c_int64, C.c_int32, _dp, _dp]
        L.oracle_paths.argtypes = [C.c_void_p, C.c_uint64, C.c_int64, _ip, _ip, C.POINTER(C.c_int64),
                                   C.c_int32, _dp, _dp]
        L.oracle_paths_mode.argtypes = [C.c_void_p, C.c_uint64, C.c_int64, _ip, _ip, C.POINTER(C.c_int64),
                                        C.c_int32, C.c_int32, _dp, _dp]
        L.oracle_closest_hit.argtypes = [C.c_void_p, C.c_int64, _dp, C.c_double, C.c_double, _dp, _ip, _dp]
        L.oracle_any_hit.argtypes = [C.c_void_p, C.c_int64, _dp, C.c_double, _dp, _ip]
        L.oracle_bvh_leaves.argtypes = [C.c_void_p, _ip, _ip, _ip, _ip]
        L.oracle_kat_aabb.argtypes = [_dp, _dp, _dp, _dp, C.c_double, C.c_double]
        L.oracle_kat_prim_hit.argtypes = [C.POINTER(MfxPrim), _dp, _dp, C.c_double, C.c_double, _dp]
        L.oracle_kat_camera_ray.argtypes = [C.POINTER(MfxPinhole), C.c_double, C.c_double, _dp]
        L.oracle_kat_tri_sample.argtypes = [_dp, _dp, _dp, C.c_double, C.c_double, _dp]
        L.oracle_kat_light_L.argtypes = [C.POINTER(MfxQuadLight), _dp, _dp]
        L.oracle_kat_hemisphere.argtypes = [_dp, C.c_uint64, C.c_uint64, C.c_uint64, C.c_int32, _dp]
        L.oracle_rng_draws.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, C.c_int32, _dp]
        L.oracle_kat_aces.argtypes = [_dp, _dp]
        L.oracle_post_rgba8.argtypes = [_dp, C.c_int32, C.c_int32, C.POINTER(C.c_uint8)]
        L.oracle_film_add.argtypes = [_dp, _dp, _dp, _dp, C.c_int64]
        L.oracle_num_threads.restype = C.c_int
        _lib = L
    return _lib


def _a3(x):
    return np.ascontiguousarray(x, dtype=np.float64).reshape(3)


class OracleScene:
    """The oracle's Scene (heap BVH + integrator state) for one SceneArrays."""

    def __init__(self, arrays: SceneArrays):
        self.arrays = arrays
        self._desc = arrays.desc()
        self.h = lib().oracle_create(C.byref(self._desc))
        if not self.h:
            raise ValueError("oracle_create rejected the scene")
        self.w, self.hgt = arrays.width, arrays.height

    def close(self):
        if self.h:
            lib().oracle_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def sample(self, spp: int, seed: int, sample_base: int = 0, nthreads: int = 0, with_stats: bool = False):
        """PixelIntegrator.Sample(spp): x-major (w*h, 4) mean frame."""
        frame = np.zeros((self.w * self.hgt, 4), dtype=np.float64)
        stats = np.zeros(8, dtype=np.float64)
        rc = lib().oracle_sample(self.h, seed, spp, sample_base, nthreads, dptr(frame), dptr(stats))
        assert rc == 0
        return (frame, stats) if with_stats else frame

    def paths(self, px, py, samples, seed: int, nthreads: int = 0, mode: str = "strict"):
        """Radiance of explicit (pixel, sample) paths. mode "strict" = the reference algorithm;
        "fast" = SAH BVH2 with tMax culling and any-hit shadows (a CPU-baseline figure only);
        "direct" = strict with the hemisphere drawn directly instead of by rejection (the same
        distribution, a different sample sequence: the statistical check of SURVEY.md §8(c))."""
        px = np.ascontiguousarray(px, dtype=np.int32)
        py = np.ascontiguousarray(py, dtype=np.int32)
        samples = np.ascontiguousarray(samples, dtype=np.int64)
        out = np.zeros((len(px), 3), dtype=np.float64)
        stats = np.zeros(8, dtype=np.float64)
        lib().oracle_paths_mode(self.h, seed, len(px), iptr(px), iptr(py),
                                samples.ctypes.data_as(C.POINTER(C.c_int64)), nthreads,
                                {"strict": 0, "fast": 1, "direct": 2}[mode], dptr(out), dptr(stats))
        return out, stats

    def closest_hit(self, rays: np.ndarray, tmin=1e-6, tmax=99999999.0):
        rays = np.ascontiguousarray(rays, dtype=np.float64).reshape(-1, 6)
        n = len(rays)
        t = np.zeros(n)
        prim = np.zeros(n, dtype=np.int32)
        nrm = np.zeros((n, 3))
        lib().oracle_closest_hit(self.h, n, dptr(rays), tmin, tmax, dptr(t), iptr(prim), dptr(nrm))
        return t, prim, nrm

    def any_hit(self, rays: np.ndarray, tmax: np.ndarray, tmin=1e-6):
        rays = np.ascontiguousarray(rays, dtype=np.float64).reshape(-1, 6)
        tmax = np.ascontiguousarray(tmax, dtype=np.float64)
        occ = np.zeros(len(rays), dtype=np.int32)
        lib().oracle_any_hit(self.h, len(rays), dptr(rays), tmin, dptr(tmax), iptr(occ))
        return occ

    def bvh_leaves(self):
        n = len(self.arrays.prims)
        idx = np.zeros(n, dtype=np.int32)
        lf = np.zeros(n, dtype=np.int32)
        lc = np.zeros(n, dtype=np.int32)
        nl = np.zeros(1, dtype=np.int32)
        lib().oracle_bvh_leaves(self.h, iptr(idx), iptr(lf), iptr(lc), iptr(nl))
        k = int(nl[0])
        return idx, lf[:k], lc[:k]


def post_rgba8(frame_xmajor: np.ndarray, w: int, h: int) -> np.ndarray:
    frame = np.ascontiguousarray(frame_xmajor, dtype=np.float64)
    out = np.zeros(w * h * 4, dtype=np.uint8)
    lib().oracle_post_rgba8(dptr(frame), w, h, out.ctypes.data_as(C.POINTER(C.c_uint8)))
    return out


def rng_draws(seed: int, pixel: int, sample: int, n: int) -> np.ndarray:
    out = np.zeros(n)
    lib().oracle_rng_draws(seed, pixel, sample, n, dptr(out))
    return out


def kat_aabb(pmin, pmax, o, d, tmin, tmax) -> bool:
    return bool(lib().oracle_kat_aabb(dptr(_a3(pmin)), dptr(_a3(pmax)), dptr(_a3(o)), dptr(_a3(d)), tmin, tmax))


def kat_prim_hit(kind: int, pts, o, d, tmin, tmax, material: int = 0):
    p = MfxPrim()
    p.kind = kind
    p.material = material
    pts = np.asarray(pts, dtype=np.float64)
    for k in range(min(4, len(pts))):
        for c in range(3):
            p.p[k][c] = float(pts[k][c]) if np.ndim(pts[k]) else (float(pts[k]) if c == 0 else 0.0)
    out = np.zeros(7)
    hit = lib().oracle_kat_prim_hit(C.byref(p), dptr(_a3(o)), dptr(_a3(d)), tmin, tmax, dptr(out))
    return bool(hit), out[0], out[1:4], out[4:7]


def kat_camera_ray(position, direction, fov, aspect, u, v):
    cam = MfxPinhole()
    for c in range(3):
        cam.position[c] = position[c]
        cam.direction[c] = direction[c]
    cam.fov, cam.aspect = fov, aspect
    out = np.zeros(6)
    lib().oracle_kat_camera_ray(C.byref(cam), u, v, dptr(out))
    return out[:3], out[3:]


def kat_tri_sample(v0, v1, v2, tu, tv):
    out = np.zeros(3)
    lib().oracle_kat_tri_sample(dptr(_a3(v0)), dptr(_a3(v1)), dptr(_a3(v2)), tu, tv, dptr(out))
    return out


def kat_light_L(p4, normal, intensity, to_light):
    L = MfxQuadLight()
    for k in range(4):
        for c in range(3):
            L.p[k][c] = p4[k][c]
    for c in range(3):
        L.normal[c] = normal[c]
        L.intensity[c] = intensity[c]
    out = np.zeros(3)
    lib().oracle_kat_light_L(C.byref(L), dptr(_a3(to_light)), dptr(out))
    return out


def kat_aces(rgb):
    out = np.zeros(3)
    lib().oracle_kat_aces(dptr(_a3(rgb)), dptr(out))
    return out


def kat_hemisphere(nm, seed, pixel, sample, skip=0):
    out = np.zeros(3)
    n = lib().oracle_kat_hemisphere(dptr(_a3(nm)), seed, pixel, sample, skip, dptr(out))
    return out, n
