"""The F# binding (fsharp/Native.fs + the EngineCore.fsproj / Scene.fs / Library.fs diffs) against
the reference's declarations (tests/golden/ref_fsharp_decls.json, made from the reference by
scripts/extract_ref_decls.py). No .NET toolchain exists here; scripts/check_fsharp_shim.py checks
what a wrong binding fails to compile on. CPU only."""
import os
import shutil
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "scripts"))
from check_fsharp_shim import Checker  # noqa: E402

FS = os.path.join(ROOT, "fsharp")


def test_shim_resolves_against_the_reference():
    assert Checker().run() == []


def _mutated(tmp_path, fname, old, new):
    d = tmp_path / "fsharp"
    shutil.copytree(FS, d)
    p = d / fname
    s = p.read_text(encoding="utf-8")
    assert old in s
    p.write_text(s.replace(old, new, 1), encoding="utf-8")
    return str(d / "Native.fs"), str(d)


@pytest.mark.parametrize("fname,old,new,expect", [
    # round 1's module names: the reference's modules are Shapes.Triangle, Light, Material
    ("Native.fs", "open Engine.Core.Shapes.Triangle", "open Engine.Core.Shapes.Trangle", "does not declare"),
    ("Native.fs", "open Engine.Core.Light\n", "open Engine.Core.Lights.Light\n", "does not declare"),
    # a field the reference does not have
    ("Native.fs", "c.coord.right.x", "c.coord.rigth.x", "no field or member"),
    ("Native.fs", "l.rect.trig1.v0", "l.rect.tri1.v0", "no field or member"),
    # a type no opened module declares
    ("Native.fs", ":? SpecularTransmission", ":? Transmission", "not declared"),
    # a wrong constructor arity for a reference type
    ("Native.fs", "Texture2D<Color>(data, width, height)", "Texture2D<Color>(data, width)", "arguments"),
    # Native.fs after Scene.fs: Scene's constructor could not see it (round 1's Library.fs placement)
    ("EngineCore.fsproj.diff", ' <Compile Include="Models\\ObjModelLoader.fs" />\n+    <Compile Include="Native\\Native.fs" />\n  <Compile Include="Scene\\Scene.fs" />',
     ' <Compile Include="Models\\ObjModelLoader.fs" />\n     <Compile Include="Scene\\Scene.fs" />\n+    <Compile Include="Native\\Native.fs" />', "before Scene"),
    # a context line that is not the reference's
    ("Scene.fs.diff", "         let cam = state.camera", "         let camera = state.camera", "differs"),
    # the shim's constructor called with the wrong arity
    ("Scene.fs.diff", "new NativePixelIntegrator(objs, AreaLight, cam, w, h, devices, DefaultSeed)",
     "new NativePixelIntegrator(objs, AreaLight, cam, w, h, devices)", "takes"),
    # an extern whose parameter count differs from the header
    ("Native.fs", "extern int mfx_reset(nativeint ctx)", "extern int mfx_reset(nativeint ctx, int spp)", "parameters"),
    # a struct whose fields do not follow the C layout
    ("Native.fs", "    val mutable ndevices : int32\n    val mutable renderAhead : int32\n",
     "    val mutable ndevices : int32\n", "C layout"),
    # a binding written for another ABI, or one that never checks the loaded library's
    ("Native.fs", "let MFX_ABI_VERSION = 6", "let MFX_ABI_VERSION = 5", "ABI version"),
    ("Native.fs", "        checkAbi ()\n", "\n", "version check"),
    ("Native.fs", "    if v <> MFX_ABI_VERSION then", "    if v < 0 then", "checkAbi must compare"),
])
def test_checker_catches_binding_errors(tmp_path, fname, old, new, expect):
    if fname.endswith(".diff") and "Compile" in old:
        old, new = old.replace("\n  <", "\n     <"), new
    native, ddir = _mutated(tmp_path, fname, old, new)
    errs = Checker(native, ddir).run()
    assert any(expect in e for e in errs), errs
