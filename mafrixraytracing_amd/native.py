"""Host-side mirror of the reference's render API over the C ABI.

`Scene`, `NativePixelIntegrator` and `Film` keep the names and argument meaning of
EngineCore/Scene/Scene.fs:291-333, Core/Integrator/Integrators.fs:143-172 and
Core/Film.fs:13-34; all work happens in libmafrix_rt.so on the GPU.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from .abi import (INSTANCING_KEYS, MFX_F_NONE, MFX_F_TWO_LEVEL, MfxInstance, MfxOptions, SceneArrays, check, dptr, iptr, load_library)

DEFAULT_SEED = 0x4D414652
DEFAULT_RENDER_AHEAD = 64  # fsharp/Native.fs DefaultRenderAhead: Scene.Render served from batches of 64 samples


class NativeContext:
    """One mfx_ctx: a scene resident in HBM on one GPU."""

    def __init__(self, arrays: SceneArrays, seed: int = DEFAULT_SEED, device: int = 0, flags: int = MFX_F_NONE,
                 part_index: int = 0, part_count: int = 1, devices: list[int] | None = None,
                 instancing: bool = True, render_ahead: int = 0):
        """devices: drive this list of HIP devices from one context (mfx_options.devices; the
        library's own RCCL reduce sums them into devices[0]); None: the single `device`.
        instancing: a scene with instancing data is created through mfx_create_instanced (two-level
        traversal; MFX_F_FLATTEN flattens it in the library); False: mfx_create on the world list.
        render_ahead: mfx_options.render_ahead (one-sample render calls served from batches of K
        samples; 0 = off)."""
        self.lib = load_library()
        self.arrays = arrays
        self.w, self.h = arrays.width, arrays.height
        inst = instancing and arrays.instancing is not None
        if inst and getattr(arrays, "two_level", False):
            flags |= MFX_F_TWO_LEVEL
        self._desc = arrays.desc(templates=inst)
        self.devices = list(devices) if devices else [device]
        self._devs = (C.c_int32 * len(self.devices))(*self.devices)
        opt = MfxOptions(seed=seed, device=device, flags=flags, part_index=part_index, part_count=part_count,
                         ndevices=len(devices) if devices else 0, render_ahead=render_ahead,
                         devices=C.cast(self._devs, C.POINTER(C.c_int32)) if devices else None)
        h = C.c_void_p()
        if inst:
            self._inst = arrays.instancing[1]
            ip = self._inst.ctypes.data_as(C.POINTER(MfxInstance))
            check(self.lib.mfx_create_instanced(C.byref(self._desc), ip, len(self._inst), C.byref(opt), C.byref(h)),
                  "mfx_create_instanced")
        else:
            check(self.lib.mfx_create(C.byref(self._desc), C.byref(opt), C.byref(h)), "mfx_create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            self.lib.mfx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # -- reference API -------------------------------------------------------------------
    def sample(self, spp: int, out: np.ndarray | None = None) -> np.ndarray:
        """IPixelIntegrator.Sample(spp) into `out` (w*h x 4 doubles, x-major; allocated if None), as
        the reference writes the Color[w,h] array it owns (Integrators.fs:160-172)."""
        frame = out if out is not None else np.empty((self.w * self.h, 4), dtype=np.float64)
        assert frame.dtype == np.float64 and frame.size == self.w * self.h * 4 and frame.flags.c_contiguous
        check(self.lib.mfx_sample(self._h, spp, dptr(frame)), "mfx_sample")
        return frame

    def render_rgba8(self, spp: int = 1, want_pixels: bool = True, out: np.ndarray | None = None) -> np.ndarray | None:
        """Film.GetFrame(spp) + post into `out` (a uint8 buffer of w*h*4, allocated if None), as
        Scene.Render writes its byte[] (mfx_render_rgba8)."""
        if not want_pixels:
            check(self.lib.mfx_render_rgba8(self._h, spp, None), "mfx_render_rgba8")
            return None
        if out is None:
            out = np.empty(self.w * self.h * 4, dtype=np.uint8)
        assert out.dtype == np.uint8 and out.size == self.w * self.h * 4 and out.flags.c_contiguous
        check(self.lib.mfx_render_rgba8(self._h, spp, out.ctypes.data_as(C.POINTER(C.c_uint8))), "mfx_render_rgba8")
        return out

    def reset(self):
        check(self.lib.mfx_reset(self._h), "mfx_reset")

    def film_mean(self) -> np.ndarray:
        frame = np.empty((self.w * self.h, 4), dtype=np.float64)
        check(self.lib.mfx_film_mean(self._h, dptr(frame)), "mfx_film_mean")
        return frame

    # -- lower level ---------------------------------------------------------------------
    def trace_accumulate(self, spp: int, sample_base: int):
        check(self.lib.mfx_trace_accumulate(self._h, spp, sample_base), "mfx_trace_accumulate")

    def accum_reduce(self):
        """Multi-device context: sum the devices' accumulators into devices[0] (mfx_accum_reduce)."""
        check(self.lib.mfx_accum_reduce(self._h), "mfx_accum_reduce")

    def accum_clear(self):
        check(self.lib.mfx_accum_clear(self._h), "mfx_accum_clear")

    def accum_device_ptr(self) -> tuple[int, int]:
        p = C.c_void_p()
        n = C.c_int64()
        check(self.lib.mfx_accum_device_ptr(self._h, C.byref(p), C.byref(n)), "mfx_accum_device_ptr")
        return p.value, n.value

    def accum_attach(self, dptr: int | None, nbytes: int = 0):
        check(self.lib.mfx_accum_attach(self._h, C.c_void_p(dptr) if dptr else None, nbytes), "mfx_accum_attach")

    def accum_read_mean(self, count: float) -> np.ndarray:
        frame = np.empty((self.w * self.h, 4), dtype=np.float64)
        check(self.lib.mfx_accum_read_mean(self._h, float(count), dptr(frame)), "mfx_accum_read_mean")
        return frame

    def sync(self):
        check(self.lib.mfx_sync(self._h), "mfx_sync")

    def stream(self) -> int:
        s = C.c_void_p()
        check(self.lib.mfx_stream(self._h, C.byref(s)), "mfx_stream")
        return s.value or 0

    def ray_counts(self) -> np.ndarray:
        out = np.zeros(16)
        check(self.lib.mfx_ray_counts(self._h, dptr(out)), "mfx_ray_counts")
        return out

    def ray_counts_total(self, reset: bool = True) -> np.ndarray:
        """The ray counters summed over every trace since creation or the last reset
        (mfx_ray_counts_total): no host read between back-to-back traces."""
        out = np.zeros(16)
        check(self.lib.mfx_ray_counts_total(self._h, dptr(out), 1 if reset else 0), "mfx_ray_counts_total")
        return out

    def stats(self) -> tuple[float, float]:
        """(rays traced, device seconds) of the last trace call (mfx_stats)."""
        rays, sec = C.c_double(), C.c_double()
        check(self.lib.mfx_stats(self._h, C.byref(rays), C.byref(sec)), "mfx_stats")
        return rays.value, sec.value

    def last_trace_ms(self) -> float:
        ms = C.c_double()
        check(self.lib.mfx_last_trace_ms(self._h, C.byref(ms)), "mfx_last_trace_ms")
        return ms.value

    def trace_timing(self) -> dict:
        out = np.zeros(8)
        check(self.lib.mfx_trace_timing(self._h, dptr(out)), "mfx_trace_timing")
        return {"total_ms": out[0], "camera_ms": out[1], "extend_ms": out[2], "camera_launches": int(out[3]),
                "shadow_ms": out[4], "iterations": int(out[5]), "launches": int(out[6]), "generations": int(out[7])}

    def closest_hit(self, rays: np.ndarray, tmin: float = 1e-6, tmax: float = 99999999.0):
        rays = np.ascontiguousarray(rays, dtype=np.float64).reshape(-1, 6)
        n = len(rays)
        t = np.zeros(n)
        prim = np.zeros(n, dtype=np.int32)
        nrm = np.zeros((n, 3))
        check(self.lib.mfx_closest_hit(self._h, n, dptr(rays), tmin, tmax, dptr(t), iptr(prim), dptr(nrm)),
              "mfx_closest_hit")
        return t, prim, nrm

    def any_hit(self, rays: np.ndarray, tmax: np.ndarray, tmin: float = 1e-6):
        rays = np.ascontiguousarray(rays, dtype=np.float64).reshape(-1, 6)
        tmax = np.ascontiguousarray(tmax, dtype=np.float64)
        occ = np.zeros(len(rays), dtype=np.int32)
        check(self.lib.mfx_any_hit(self._h, len(rays), dptr(rays), tmin, dptr(tmax), iptr(occ)), "mfx_any_hit")
        return occ

    def build_info(self) -> dict:
        """How the scene was prepared (mfx_build_info): timings, BVH sizes, image digest."""
        out = np.zeros(8)
        dig = C.c_uint64()
        check(self.lib.mfx_build_info(self._h, dptr(out), C.byref(dig)), "mfx_build_info")
        return {"ref_bvh_ms": out[0], "bvh_ms": out[1], "scene_ms": out[2], "gpu_bvh": bool(out[3]),
                "gpu_images": bool(out[3] == 2),
                "nodes4": int(out[4]), "slots": int(out[5]), "nodes2": int(out[6]), "levels": int(out[7]),
                "digest": dig.value}

    def device_info(self) -> dict:
        """How the context's work lies over devices (mfx_device_info): the HIP ordinals, the RCCL
        communicators it created, how mfx_accum_reduce merges, and the primary's tile-row band."""
        out = np.zeros(5 + len(self.devices), dtype=np.int32)
        check(self.lib.mfx_device_info(self._h, iptr(out), len(out)), "mfx_device_info")
        g = int(out[0])
        return {"devices": [int(d) for d in out[5:5 + g]], "communicators": int(out[1]),
                "merge": {0: "none", 1: "rccl_reduce", 2: "ordered_adds"}[int(out[2])],
                "band_index": int(out[3]), "band_count": int(out[4])}

    def instancing_info(self) -> dict:
        """How instances are traced (mfx_instancing_info): two-level shape and image bytes."""
        out = np.zeros(8)
        check(self.lib.mfx_instancing_info(self._h, dptr(out)), "mfx_instancing_info")
        return {k: int(v) for k, v in zip(INSTANCING_KEYS, out)}

    def ref_leaves(self):
        n = len(self.arrays.prims)
        idx = np.zeros(n, dtype=np.int32)
        lf = np.zeros(n, dtype=np.int32)
        lc = np.zeros(n, dtype=np.int32)
        nl = C.c_int32()
        check(self.lib.mfx_ref_leaves(self._h, iptr(idx), iptr(lf), iptr(lc), C.byref(nl)), "mfx_ref_leaves")
        return idx, lf[:nl.value], lc[:nl.value]


def fp64_selftest(a: np.ndarray, b: np.ndarray, device: int = 0):
    lib = load_library()
    a = np.ascontiguousarray(a, dtype=np.float64)
    b = np.ascontiguousarray(b, dtype=np.float64)
    dv = np.zeros_like(a)
    sq = np.zeros_like(a)
    check(lib.mfx_fp64_selftest(device, len(a), dptr(a), dptr(b), dptr(dv), dptr(sq)), "mfx_fp64_selftest")
    return dv, sq


def aabb_selftest(rec: np.ndarray, device: int = 0):
    """(FP64 AABB.hit answers, FP32-screen answers: 1, 0 or -1 = left to FP64, vertex-box proofs:
    1 or 0) for n x 24 records (mfx_aabb_selftest)."""
    lib = load_library()
    rec = np.ascontiguousarray(rec, dtype=np.float64).reshape(-1, 24)
    out = np.zeros((len(rec), 3), dtype=np.int32)
    check(lib.mfx_aabb_selftest(device, len(rec), dptr(rec), iptr(out)), "mfx_aabb_selftest")
    return out[:, 0], out[:, 1], out[:, 2]


# ---- the reference's object model -----------------------------------------------------------
class Film:
    """Film (Film.fs:13-34): progressive accumulation; here the accumulator lives on the GPU."""

    def __init__(self, ctx: NativeContext):
        self._ctx = ctx
        self.Size = (ctx.w, ctx.h)

    def Reset(self):
        self._ctx.reset()

    def GetFrame(self, integrator: "NativePixelIntegrator", samples: int) -> np.ndarray:
        self._ctx.render_rgba8(samples, want_pixels=False)
        return self._ctx.film_mean()


class NativePixelIntegrator:
    """IPixelIntegrator (IIntegrator.fs:35-40) backed by the GPU: Sample(n) -> Color[w,h] x-major."""

    def __init__(self, ctx: NativeContext):
        self._ctx = ctx

    def Sample(self, n: int) -> np.ndarray:
        return self._ctx.sample(n)


class Scene:
    """Scene (Scene.fs:291-333) with the path-tracing hot path on the GPU. Render's one-sample calls
    are served from batches of `render_ahead` samples (the F# binding's DefaultRenderAhead;
    mfx_options.render_ahead): the same bytes per frame as one sample per call."""

    def __init__(self, state, seed: int = DEFAULT_SEED, device: int = 0, max_depth: int = 3,
                 render_ahead: int = DEFAULT_RENDER_AHEAD):
        arrays = state.arrays(max_depth=max_depth) if hasattr(state, "arrays") else state
        self._ctx = NativeContext(arrays, seed=seed, device=device, render_ahead=render_ahead)
        self.width, self.height = arrays.width, arrays.height
        self.film = Film(self._ctx)
        self.pixelIntegrator = NativePixelIntegrator(self._ctx)

    @property
    def ScreenSize(self):
        return (self.width, self.height)

    def Render(self, delta: float, buffer) -> None:
        """Scene.Render(delta, buffer) (Scene.fs:331-333): one 1-spp frame into the film, then
        ACES -> sqrt -> RGBA8 into `buffer` (byte[w*h*4], y-major)."""
        out = self._ctx.render_rgba8(1)
        mv = memoryview(buffer).cast("B")
        mv[:] = out.tobytes()

    def close(self):
        self._ctx.close()
