"""ctypes mirror of include/mafrix_rt.h and the loader for libmafrix_rt.so.

This is the Python stand-in for the F# P/Invoke declarations a maintainer adds to
EngineCore/Library.fs: the same structs, the same entry points.
The library is the HIP build for gfx950; there is no CPU fallback — loading fails loudly
if the shared object is missing.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

MFX_PRIM_TRIANGLE = 0
MFX_PRIM_RECT = 1
MFX_PRIM_SPHERE = 2

MFX_F_NONE = 0
MFX_F_COUNT_STATS = 1
MFX_F_MEGAKERNEL = 2
MFX_F_HOST_BVH = 4
MFX_F_WAVEFRONT = 8
MFX_F_FLATTEN = 16
MFX_F_TWO_LEVEL = 32
MFX_F_ROW_PARTITION = 64
MFX_F_IN_FLIGHT = 128
MFX_INSTANCE_VERBATIM = 1
MFX_MAX_DEVICES = 64
MFX_ABI_VERSION = 6

_HERE = os.path.dirname(os.path.abspath(__file__))
# MFX_LIB_PATH: another build of the same library (scripts' A/B and roof passes on a variant)
LIB_PATH = os.environ.get("MFX_LIB_PATH") or os.path.join(_HERE, "libmafrix_rt.so")


class MfxPrim(C.Structure):
    _fields_ = [("kind", C.c_int32), ("material", C.c_int32), ("p", (C.c_double * 3) * 4)]


class MfxQuadLight(C.Structure):
    _fields_ = [("p", (C.c_double * 3) * 4), ("normal", C.c_double * 3), ("intensity", C.c_double * 3)]


class MfxPinhole(C.Structure):
    _fields_ = [("position", C.c_double * 3), ("direction", C.c_double * 3),
                ("fov", C.c_double), ("aspect", C.c_double),
                ("topleft", C.c_double * 3), ("right", C.c_double * 3), ("down", C.c_double * 3),
                ("derived", C.c_int32), ("reserved", C.c_int32)]


class MfxSceneDesc(C.Structure):
    _fields_ = [("prims", C.POINTER(MfxPrim)), ("nprims", C.c_int64),
                ("albedo", C.POINTER(C.c_double)), ("nmat", C.c_int32),
                ("width", C.c_int32), ("height", C.c_int32), ("max_depth", C.c_int32),
                ("light", MfxQuadLight), ("camera", MfxPinhole)]


class MfxOptions(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("device", C.c_int32), ("flags", C.c_int32),
                ("part_index", C.c_int32), ("part_count", C.c_int32),
                ("ndevices", C.c_int32), ("render_ahead", C.c_int32), ("devices", C.POINTER(C.c_int32))]


class MfxInstance(C.Structure):
    _fields_ = [("first", C.c_int64), ("count", C.c_int64), ("offset", C.c_double * 3),
                ("flags", C.c_int32), ("reserved", C.c_int32)]


assert C.sizeof(MfxPrim) == 104
assert C.sizeof(MfxInstance) == 48

# numpy structured dtype with the same layout as mfx_prim (for building big prim arrays fast)
PRIM_DTYPE = np.dtype([("kind", "<i4"), ("material", "<i4"), ("p", "<f8", (4, 3))], align=True)
assert PRIM_DTYPE.itemsize == 104
# mfx_instance: template range, translation, flags
INSTANCE_DTYPE = np.dtype([("first", "<i8"), ("count", "<i8"), ("offset", "<f8", (3,)), ("flags", "<i4"),
                           ("reserved", "<i4")], align=True)
assert INSTANCE_DTYPE.itemsize == 48


class SceneArrays:
    """Owns the numpy buffers an MfxSceneDesc points into (keeps them alive).

    prims is the world primitive list (the reference's flat scene). `instancing`, when given, is
    (templates, instances): the same world scene as template primitives and mfx_instance entries
    whose expansion is `prims` (mfx_create_instanced: flattened when the flat image fits the library's
    budget, two-level otherwise). two_level: ask for the two-level traversal regardless
    (MFX_F_TWO_LEVEL)."""

    def __init__(self, prims: np.ndarray, albedo: np.ndarray, light: dict, camera: dict,
                 width: int, height: int, max_depth: int = 3, instancing=None, two_level: bool = False):
        self.prims = np.ascontiguousarray(prims, dtype=PRIM_DTYPE)
        self.two_level = bool(two_level)
        self.instancing = None
        if instancing is not None:
            self.instancing = (np.ascontiguousarray(instancing[0], dtype=PRIM_DTYPE),
                               np.ascontiguousarray(instancing[1], dtype=INSTANCE_DTYPE))
        self.albedo = np.ascontiguousarray(albedo, dtype=np.float64).reshape(-1, 3)
        self.light = light
        self.camera = camera
        self.width = int(width)
        self.height = int(height)
        self.max_depth = int(max_depth)

    def desc(self, templates: bool = False) -> MfxSceneDesc:
        """templates: point at the instancing template primitives instead of the world list."""
        d = MfxSceneDesc()
        pr = self.instancing[0] if templates else self.prims
        d.prims = pr.ctypes.data_as(C.POINTER(MfxPrim))
        d.nprims = len(pr)
        d.albedo = self.albedo.ctypes.data_as(C.POINTER(C.c_double))
        d.nmat = len(self.albedo)
        d.width, d.height, d.max_depth = self.width, self.height, self.max_depth
        for k in range(4):
            for c in range(3):
                d.light.p[k][c] = float(self.light["p"][k][c])
        for c in range(3):
            d.light.normal[c] = float(self.light["normal"][c])
            d.light.intensity[c] = float(self.light["intensity"][c])
            d.camera.position[c] = float(self.camera["position"][c])
            d.camera.direction[c] = float(self.camera["direction"][c])
        d.camera.fov = float(self.camera["fov"])
        d.camera.aspect = float(self.camera["aspect"])
        return d

    def with_film(self, width: int, height: int) -> "SceneArrays":
        return SceneArrays(self.prims, self.albedo, self.light, self.camera, width, height, self.max_depth,
                           self.instancing, self.two_level)

    def flat(self) -> "SceneArrays":
        """The same scene without its instancing (the reference's flat primitive list)."""
        return SceneArrays(self.prims, self.albedo, self.light, self.camera, self.width, self.height,
                           self.max_depth)


_P = C.POINTER
_dp = _P(C.c_double)
_ip = _P(C.c_int32)


def _bind(lib, strict: bool = True):
    sig = {
        "mfx_create": (C.c_int, [_P(MfxSceneDesc), _P(MfxOptions), _P(C.c_void_p)]),
        "mfx_create_instanced": (C.c_int, [_P(MfxSceneDesc), _P(MfxInstance), C.c_int32, _P(MfxOptions),
                                           _P(C.c_void_p)]),
        "mfx_expand_instances": (C.c_int, [_P(MfxPrim), C.c_int64, _P(MfxInstance), C.c_int32, _P(MfxPrim),
                                           C.c_int64, _P(C.c_int64)]),
        "mfx_instancing_info": (C.c_int, [C.c_void_p, _dp]),
        "mfx_build_instanced_info": (C.c_int, [_P(MfxSceneDesc), _P(MfxInstance), C.c_int32, C.c_int32, _dp, _ip]),
        "mfx_destroy": (None, [C.c_void_p]),
        "mfx_sample": (C.c_int, [C.c_void_p, C.c_int32, _dp]),
        "mfx_render_rgba8": (C.c_int, [C.c_void_p, C.c_int32, _P(C.c_uint8)]),
        "mfx_accumulate_render_rgba8": (C.c_int, [C.c_void_p, C.c_int32, _P(C.c_uint8)]),
        "mfx_stats": (C.c_int, [C.c_void_p, _dp, _dp]),
        "mfx_reset": (C.c_int, [C.c_void_p]),
        "mfx_film_mean": (C.c_int, [C.c_void_p, _dp]),
        "mfx_trace_accumulate": (C.c_int, [C.c_void_p, C.c_int32, C.c_int64]),
        "mfx_accum_clear": (C.c_int, [C.c_void_p]),
        "mfx_accum_reduce": (C.c_int, [C.c_void_p]),
        "mfx_accum_device_ptr": (C.c_int, [C.c_void_p, _P(C.c_void_p), _P(C.c_int64)]),
        "mfx_accum_read_mean": (C.c_int, [C.c_void_p, C.c_double, _dp]),
        "mfx_accum_attach": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64]),
        "mfx_sync": (C.c_int, [C.c_void_p]),
        "mfx_stream": (C.c_int, [C.c_void_p, _P(C.c_void_p)]),
        "mfx_ray_counts": (C.c_int, [C.c_void_p, _dp]),
        "mfx_last_trace_ms": (C.c_int, [C.c_void_p, _dp]),
        "mfx_trace_timing": (C.c_int, [C.c_void_p, _dp]),
        "mfx_ray_counts_total": (C.c_int, [C.c_void_p, _dp, C.c_int32]),
        "mfx_closest_hit": (C.c_int, [C.c_void_p, C.c_int64, _dp, C.c_double, C.c_double, _dp, _ip, _dp]),
        "mfx_any_hit": (C.c_int, [C.c_void_p, C.c_int64, _dp, C.c_double, _dp, _ip]),
        "mfx_ref_leaves": (C.c_int, [C.c_void_p, _ip, _ip, _ip, _ip]),
        "mfx_fp64_selftest": (C.c_int, [C.c_int32, C.c_int64, _dp, _dp, _dp, _dp]),
        "mfx_aabb_selftest": (C.c_int, [C.c_int32, C.c_int64, _dp, _ip]),
        "mfx_build_leaves": (C.c_int, [_P(MfxSceneDesc), _ip, _ip, _ip, _ip, _ip]),
        "mfx_build_info": (C.c_int, [C.c_void_p, _dp, _P(C.c_uint64)]),
        "mfx_device_info": (C.c_int, [C.c_void_p, _ip, C.c_int32]),
        "mfx_last_error": (C.c_char_p, []),
        "mfx_abi_version": (C.c_int, []),
        "mfx_device_count": (C.c_int, []),
    }
    for name, (res, args) in sig.items():
        if not strict and not hasattr(lib, name):  # (an older build under A/B: scripts only)
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


EXPORTED_SYMBOLS = [
    "mfx_create", "mfx_create_instanced", "mfx_expand_instances", "mfx_instancing_info", "mfx_build_instanced_info", "mfx_destroy", "mfx_sample", "mfx_render_rgba8", "mfx_accumulate_render_rgba8", "mfx_reset",
    "mfx_film_mean", "mfx_stats",
    "mfx_trace_accumulate", "mfx_accum_clear", "mfx_accum_reduce", "mfx_accum_device_ptr", "mfx_accum_attach", "mfx_accum_read_mean",
    "mfx_sync", "mfx_stream", "mfx_ray_counts", "mfx_last_trace_ms", "mfx_trace_timing", "mfx_ray_counts_total", "mfx_closest_hit", "mfx_any_hit", "mfx_ref_leaves",
    "mfx_fp64_selftest", "mfx_aabb_selftest", "mfx_build_leaves", "mfx_build_info", "mfx_device_info", "mfx_last_error", "mfx_abi_version", "mfx_device_count",
]

_lib = None


def load_library(path: str | None = None, strict: bool = True):
    """Load libmafrix_rt.so (the HIP build). Raises if it is missing — no fallback exists.
    strict=False (A/B scripts timing an older build) binds only the entry points it exports."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise RuntimeError(f"mafrix_rt native library not built: {p} (run __graft_entry__.build())")
    lib = _bind(C.CDLL(p, mode=C.RTLD_GLOBAL), strict)
    if path is None:
        _lib = lib
    return lib


class MfxError(RuntimeError):
    pass


def check(rc: int, what: str):
    if rc != 0:
        msg = load_library().mfx_last_error()
        raise MfxError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")


def dptr(a: np.ndarray):
    return a.ctypes.data_as(_dp)


def iptr(a: np.ndarray):
    return a.ctypes.data_as(_ip)


def build_leaves(arrays: SceneArrays):
    """Host-only: reference leaf grouping + traversal-BVH shape of a scene (no GPU needed)."""
    lib = load_library()
    d = arrays.desc()
    n = len(arrays.prims)
    idx = np.zeros(n, dtype=np.int32)
    lf = np.zeros(n, dtype=np.int32)
    lc = np.zeros(n, dtype=np.int32)
    nl = np.zeros(1, dtype=np.int32)
    info = np.zeros(4, dtype=np.int32)
    check(lib.mfx_build_leaves(C.byref(d), iptr(idx), iptr(lf), iptr(lc), iptr(nl), iptr(info)), "mfx_build_leaves")
    k = int(nl[0])
    return idx, lf[:k], lc[:k], {"clusters": int(info[0]), "nodes": int(info[1]), "stack": int(info[2]),
                                 "slots": int(info[3])}


def expand_instances(templates: np.ndarray, instances: np.ndarray) -> np.ndarray:
    """Host-only: the world primitive list the library derives from an instanced scene."""
    lib = load_library()
    t = np.ascontiguousarray(templates, dtype=PRIM_DTYPE)
    ins = np.ascontiguousarray(instances, dtype=INSTANCE_DTYPE)
    n = C.c_int64()
    tp = t.ctypes.data_as(_P(MfxPrim))
    ip = ins.ctypes.data_as(_P(MfxInstance))
    check(lib.mfx_expand_instances(tp, len(t), ip, len(ins), None, 0, C.byref(n)), "mfx_expand_instances")
    out = np.zeros(n.value, dtype=PRIM_DTYPE)
    check(lib.mfx_expand_instances(tp, len(t), ip, len(ins), out.ctypes.data_as(_P(MfxPrim)), len(out), C.byref(n)),
          "mfx_expand_instances")
    return out


INSTANCING_KEYS = ("instances", "templates", "top_nodes", "template_nodes", "template_slots", "top_slots",
                   "world_slots", "image_bytes")


def build_instanced_info(arrays: SceneArrays, flags: int = 0) -> dict:
    """Host-only: how an instanced scene's traversal images come out (no GPU needed)."""
    lib = load_library()
    d = arrays.desc(templates=True)
    ins = arrays.instancing[1]
    out = np.zeros(8)
    st = np.zeros(1, dtype=np.int32)
    check(lib.mfx_build_instanced_info(C.byref(d), ins.ctypes.data_as(_P(MfxInstance)), len(ins), flags, dptr(out),
                                       iptr(st)), "mfx_build_instanced_info")
    r = {k: int(v) for k, v in zip(INSTANCING_KEYS, out)}
    r["stack"] = int(st[0])
    return r
