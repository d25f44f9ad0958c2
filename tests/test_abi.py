"""The C-ABI library loads and exports exactly what include/mafrix_rt.h declares (CPU only: no
compute calls)."""
import os
import re
import subprocess

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "mafrix_rt.h")
LIB = os.path.join(ROOT, "mafrixraytracing_amd", "libmafrix_rt.so")


def declared():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"\b(mfx_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    from mafrixraytracing_amd.abi import EXPORTED_SYMBOLS, load_library
    lib = load_library()
    names = declared()
    assert len(names) >= 20
    for n in names:
        assert hasattr(lib, n), n
    assert sorted(EXPORTED_SYMBOLS) == names  # the ctypes mirror binds all of them
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True).stdout
    exported = sorted(set(re.findall(r"\bT (mfx_[a-z0-9_]+)$", out, re.M)))
    assert exported == names  # nothing undeclared leaks out


def test_struct_layouts_match_header():
    import ctypes as C
    from mafrixraytracing_amd.abi import MfxOptions, MfxPinhole, MfxPrim, MfxQuadLight, MfxSceneDesc
    assert C.sizeof(MfxPrim) == 104
    assert C.sizeof(MfxQuadLight) == 18 * 8
    assert C.sizeof(MfxPinhole) == 17 * 8 + 8
    assert C.sizeof(MfxOptions) == 24
    assert C.sizeof(MfxSceneDesc) == 8 + 8 + 8 + 4 * 4 + C.sizeof(MfxQuadLight) + C.sizeof(MfxPinhole)


def test_version_errors_and_no_cpu_fallback():
    import ctypes as C
    from mafrixraytracing_amd.abi import MfxOptions, load_library
    lib = load_library()
    assert lib.mfx_abi_version() == 1
    assert lib.mfx_device_count() >= 0
    h = C.c_void_p()
    opt = MfxOptions(seed=1, device=0, flags=0, part_index=0, part_count=1)
    assert lib.mfx_create(None, C.byref(opt), C.byref(h)) == -1
    assert b"null" in lib.mfx_last_error()
    rays, sec = C.c_double(), C.c_double()
    assert lib.mfx_stats(None, C.byref(rays), C.byref(sec)) == -1
    assert lib.mfx_accumulate_render_rgba8(None, 1, None) == -1
    opt.part_count = 0
    from conftest import scene
    d = scene("cornell", 4, 4).desc()
    assert lib.mfx_create(C.byref(d), C.byref(opt), C.byref(h)) == -1
    if lib.mfx_device_count() == 0:
        # without a GPU, creating a context fails loudly (MFX_E_DEVICE) instead of falling back
        opt.part_count = 1
        assert lib.mfx_create(C.byref(d), C.byref(opt), C.byref(h)) == -2


def test_empty_scene_rejected():
    import ctypes as C
    from mafrixraytracing_amd.abi import load_library
    from conftest import scene
    lib = load_library()
    a = scene("cornell", 4, 4)
    d = a.desc()
    d.nprims = 0  # Bvh.Build on an empty array throws in the reference (BvhNode.fs:26)
    info = (C.c_int32 * 4)()
    assert lib.mfx_build_leaves(C.byref(d), None, None, None, None, info) == -1
