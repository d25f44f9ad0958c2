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


def header_layouts(tmp_path):
    """sizeof and every field offset of the header's structs, as gcc lays them out."""
    from mafrixraytracing_amd import abi
    structs = {"mfx_prim": abi.MfxPrim, "mfx_quad_light": abi.MfxQuadLight, "mfx_pinhole": abi.MfxPinhole,
               "mfx_scene_desc": abi.MfxSceneDesc, "mfx_options": abi.MfxOptions, "mfx_instance": abi.MfxInstance}
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(void) {"]
    for cname, py in structs.items():
        lines.append(f'printf("{cname} size %zu\\n", sizeof({cname}));')
        for f in py._fields_:
            lines.append(f'printf("{cname} {f[0]} %zu\\n", offsetof({cname}, {f[0]}));')
    lines.append("return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-o", str(exe), str(src)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout
    return structs, {tuple(l.split()[:2]): int(l.split()[2]) for l in out.splitlines()}


def test_struct_layouts_match_header(tmp_path):
    """The ctypes mirror (and so the F# shim, whose fields follow it) has the C header's layout."""
    import ctypes as C
    structs, lay = header_layouts(tmp_path)
    for cname, py in structs.items():
        assert lay[(cname, "size")] == C.sizeof(py), cname
        for f in py._fields_:
            assert lay[(cname, f[0])] == getattr(py, f[0]).offset, (cname, f[0])
    assert lay[("mfx_prim", "size")] == 104 and lay[("mfx_options", "size")] == 40
    assert lay[("mfx_instance", "size")] == 48


def test_version_errors_and_no_cpu_fallback():
    import ctypes as C
    from mafrixraytracing_amd.abi import MfxOptions, load_library
    lib = load_library()
    assert lib.mfx_abi_version() == 6
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
    # a device list needs its array, and at most MFX_MAX_DEVICES entries
    opt.part_count = 1
    opt.ndevices = 2
    opt.devices = None
    assert lib.mfx_create(C.byref(d), C.byref(opt), C.byref(h)) == -1
    opt.ndevices = 65
    assert lib.mfx_create(C.byref(d), C.byref(opt), C.byref(h)) == -1
    assert lib.mfx_accum_reduce(None) == -4


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
