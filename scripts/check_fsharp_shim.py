#!/usr/bin/env python3
"""Check the F# shim (fsharp/Native.fs + fsharp/*.diff) against the reference's declarations.

There is no .NET toolchain in this image, so the shim cannot be compiled here. This checker
does the part of the compiler's job that a wrong binding fails on, from the committed fixture
tests/golden/ref_fsharp_decls.json (scripts/extract_ref_decls.py, generated from the reference):

1. every diff applies to the reference: its context and removed lines equal the reference's
   lines at those positions (per-line SHA-1s in the fixture);
2. compile order: Native.fs is inserted into EngineCore.fsproj after every module it opens and
   before Scene/Scene.fs, which opens it (F# has no forward references);
3. every module Native.fs opens exists; every type it names (type tests, annotations, generic
   arguments, constructor calls) is declared by an opened module, by the shim, or is a .NET type;
4. every member chain on a typed value (`c.coord.right.x`, `l.rect.trig1.v0`, `mgr.materials`)
   resolves field by field through the reference's declarations; static members exist;
   constructor calls have a declared arity;
5. the names the diffs' added lines use exist: the ctor locals in the verified context, the
   shim's constructor arity and members, Scene's new constructor used by Library.fs;
6. the blittable structs have the C header's field sequence (via the ctypes mirror abi.py,
   whose offsets tests/test_abi.py checks against the header), and every `extern` names a
   declared C entry point with its parameter count; the shim's MFX_ABI_VERSION is the header's and
   it is checked (mfx_abi_version) before the first mfx_create.

Exit status 0 and "OK" when everything resolves; otherwise one line per problem.
"""
from __future__ import annotations

import hashlib
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
from extract_ref_decls import parse_file  # noqa: E402

FIXTURE = os.path.join(ROOT, "tests", "golden", "ref_fsharp_decls.json")
NATIVE = os.path.join(ROOT, "fsharp", "Native.fs")
DIFFS = {"EngineCore/EngineCore.fsproj": "EngineCore.fsproj.diff", "EngineCore/Scene/Scene.fs": "Scene.fs.diff",
         "EngineCore/Library.fs": "Library.fs.diff"}
HEADER = os.path.join(ROOT, "include", "mafrix_rt.h")

# .NET / FSharp.Core names the shim uses (not the reference's)
DOTNET = {"int", "int32", "int64", "uint64", "float", "double", "byte", "nativeint", "string", "bool", "obj", "unit",
          "IDisposable", "GCHandle", "GCHandleType", "Marshal", "Array", "Array2D", "DllImport", "StructLayout",
          "LayoutKind", "CallingConvention", "Struct", "byref", "System", "InteropServices", "Runtime"}


def sha(line: str) -> str:
    return hashlib.sha1(line.encode("utf-8")).hexdigest()[:16]


def parse_diff(path):
    hunks, cur = [], None
    for raw in open(path, encoding="utf-8").read().split("\n"):
        line = raw.lstrip("﻿")
        m = re.match(r"^@@ -(\d+)(?:,(\d+))? \+(\d+)(?:,(\d+))? @@", line)
        if m:
            cur = {"old": int(m.group(1)), "lines": []}
            hunks.append(cur)
        elif cur is not None and line[:1] in (" ", "-", "+"):
            if not line.startswith(("---", "+++")) or cur["lines"]:
                cur["lines"].append((line[0], raw[1:].lstrip("﻿") if raw[:1] in " -+" else raw))
    return hunks


def ident_type(t: str) -> str:
    """Base type name of an annotation: 'IHitable[]' -> 'IHitable', 'byref<MfxPrim>' -> 'MfxPrim'."""
    t = t.strip()
    m = re.match(r"byref<(\w+)>", t)
    if m:
        return m.group(1)
    return re.match(r"[\w\.]*", t).group(0).split(".")[-1]


class Checker:
    def __init__(self, native_path: str = NATIVE, diff_dir: str = os.path.join(ROOT, "fsharp")):
        self.fx = json.load(open(FIXTURE))
        self.errors = []
        self.diff_dir = diff_dir
        raw = open(native_path, encoding="utf-8").read()
        # code only: comments and string literals out, multi-line parenthesised headers joined
        code = re.sub(r'"(?:[^"\\]|\\.)*"', '""', raw)
        code = "\n".join(l.split("//")[0].rstrip() for l in code.split("\n"))
        joined, depth = [], 0
        for l in code.split("\n"):
            if depth > 0:
                joined[-1] += " " + l.strip()
            else:
                joined.append(l)
            depth += l.count("(") - l.count(")")
        self.native_lines = joined
        self.native_text = "\n".join(joined)
        self.own = parse_file("fsharp/Native.fs", self.native_lines)
        self.mod_name = next(iter(self.own))
        self.opens = self.own[self.mod_name]["opens"]

    def err(self, msg):
        self.errors.append(msg)

    # ---- type lookup -------------------------------------------------------------------------
    def types_in(self, modules):
        out = {}
        for m in modules:
            md = self.fx["modules"].get(m) or self.own.get(m)
            if not md:
                continue
            for k, v in md["types"].items():
                out.setdefault(k, v)
            for k, v in md.get("aliases", {}).items():
                out.setdefault(k, {"alias": v})
        return out

    def visible_types(self):
        vis = self.types_in(self.opens)
        for m, md in self.own.items():
            vis.update(md["types"])
        return vis

    # ---- 1. diffs apply to the reference ------------------------------------------------------
    def check_diffs(self):
        self.diffs = {}
        for ref_file, name in DIFFS.items():
            path = os.path.join(self.diff_dir, name)
            hashes = self.fx["line_sha1_16"][ref_file]
            hunks = parse_diff(path)
            if not hunks:
                self.err(f"{name}: no hunks")
            for h in hunks:
                ln = h["old"]
                for tag, text in h["lines"]:
                    if tag in (" ", "-"):
                        if ln - 1 >= len(hashes) or hashes[ln - 1] != sha(text):
                            self.err(f"{name}: line {ln} of {ref_file} differs from the diff's {text!r}")
                        ln += 1
            self.diffs[ref_file] = hunks

    # ---- 2. compile order --------------------------------------------------------------------
    def check_order(self):
        order = list(self.fx["compile_order"])
        new = order[:]
        for h in self.diffs["EngineCore/EngineCore.fsproj"]:
            prev = None
            for tag, text in h["lines"]:
                m = re.search(r'<Compile Include="([^"]+)"', text)
                if not m:
                    continue
                f = "EngineCore/" + m.group(1).replace("\\", "/")
                if tag == "+":
                    new.insert(new.index(prev) + 1 if prev else 0, f)
                    prev = f
                elif tag == " ":
                    prev = f
                elif tag == "-":
                    new.remove(f)
        self.order = new
        mine = "EngineCore/Native/Native.fs"
        if mine not in new:
            self.err("EngineCore.fsproj.diff does not add Native\\Native.fs")
            return
        pos = new.index(mine)
        for m in self.opens:
            if m.startswith("System"):
                continue
            md = self.fx["modules"].get(m)
            if md is None:
                self.err(f"Native.fs opens {m}, which the reference does not declare")
            elif new.index(md["file"]) >= pos:
                self.err(f"Native.fs opens {m} ({md['file']}), compiled after it")
        if new.index("EngineCore/Scene/Scene.fs") <= pos:
            self.err("Native.fs must compile before Scene/Scene.fs")
        if self.mod_name in self.fx["modules"]:
            self.err(f"module {self.mod_name} already exists in the reference")

    # ---- 3/4. types and member chains in Native.fs --------------------------------------------
    def blocks(self):
        """Top-level definitions of Native.fs (scopes for local names)."""
        cur = []
        for l in self.native_lines:
            if l and not l[0].isspace() and not l.startswith(("//", "[<", "///")) and cur:
                yield cur
                cur = []
            cur.append(l)
        if cur:
            yield cur

    def resolve_chain(self, tname, steps, vis, where):
        t = vis.get(tname)
        while t is not None and "alias" in t:
            t = vis.get(t["alias"].split(".")[-1])
        for s in steps:
            if t is None:
                return
            if s in t["fields"]:
                ft = t["fields"][s]
                if re.search(r"\[|array", ft):
                    return
                t = vis.get(ident_type(ft))
                if t is None and ident_type(ft) not in DOTNET:
                    self.err(f"{where}: field type {ft} of .{s} is not visible")
                continue
            if s in t["members"] or s in t["static"] or s in t["abstract"]:
                return
            self.err(f"{where}: {tname} has no field or member {s!r} (chain .{'.'.join(steps)})")
            return

    def check_native(self):
        vis = self.visible_types()
        own_types = {k for md in self.own.values() for k in md["types"]}
        text = self.native_text
        # every type name used in a type position
        used = set(re.findall(r":\?\s*(\w+)", text))
        used |= {ident_type(t) for t in re.findall(r"\w\s*:\s*([A-Za-z][\w\.]*(?:<[^>]*>)?(?:\[,*\])?)", text)}
        used |= set(re.findall(r"<(\w+)>", text))
        used |= set(re.findall(r"\bnew\s+(\w+)\s*\(", text))
        for t in sorted(used):
            if t not in vis and t not in DOTNET and t not in own_types:
                self.err(f"Native.fs: type {t} is not declared by an opened module")
        # constructor arities of reference types
        for t, args in re.findall(r"\b([A-Z]\w*)(?:<\w+>)?\(([^()]*)\)", text):
            info = vis.get(t)
            if info and t not in own_types and "alias" not in info:
                n = len([a for a in args.split(",") if a.strip()])
                ok = n == 0 or n == len(info["ctor_params"]) or n in info["ctors"]
                if not ok:
                    self.err(f"Native.fs: {t}({args}) has {n} arguments; the reference declares "
                             f"{len(info['ctor_params'])} / {info['ctors']}")
        # member chains inside each top-level definition
        for blk in self.blocks():
            b = "\n".join(blk)
            head = blk[0].strip()[:60]
            env = {}
            for v, t in re.findall(r":\?\s*(\w+)\s+as\s+(\w+)", b):
                env[t] = v
            for v, t in re.findall(r"\b([a-z]\w*)\s*:\s*([A-Za-z][\w\.]*(?:<[^>]*>)?(?:\[,*\])?)", b):
                if "[" not in t:
                    env.setdefault(v, ident_type(t))
            for v, t in re.findall(r"let\s+(?:mutable\s+)?([a-z]\w*)\s*=\s*([A-Z]\w*)(?:<\w+>)?\(", b):
                env.setdefault(v, t)
            for v, chain in re.findall(r"\b([a-z]\w*)((?:\.[A-Za-z_]\w*)+)", b):
                if v in env and v not in ("this",):
                    self.resolve_chain(env[v], chain.strip(".").split("."), {**vis, **{k: self.own_type(k) for k in own_types}},
                                       f"Native.fs [{head}]")
            for t, s in re.findall(r"\b([A-Z]\w*)\.([A-Z]\w*)\(", b):
                info = vis.get(t)
                if info and "alias" not in info and s not in info["static"] and s not in info["members"]:
                    self.err(f"Native.fs: {t}.{s} is not declared")

    def own_type(self, name):
        for md in self.own.values():
            if name in md["types"]:
                return md["types"][name]

    # ---- 5. the diffs' added lines --------------------------------------------------------------
    def check_added(self):
        ni = self.own_type("NativePixelIntegrator")
        scene = self.diffs["EngineCore/Scene/Scene.fs"]
        plus = [t for h in scene for tag, t in h["lines"] if tag == "+"]
        ctx = [t for h in scene for tag, t in h["lines"] if tag == " "]
        added = "\n".join(plus)
        for mod in re.findall(r"^open\s+([\w\.]+)", added, re.M):
            if mod != self.mod_name and mod not in self.fx["modules"]:
                self.err(f"Scene.fs.diff opens unknown module {mod}")
        for m in re.finditer(r"new\s+NativePixelIntegrator\(([^)]*)\)", added):
            args = [a.strip() for a in m.group(1).split(",")]
            if len(args) not in (len(ni["ctor_params"]), *ni["ctors"]):
                self.err(f"Scene.fs.diff: NativePixelIntegrator takes {len(ni['ctor_params'])} or {ni['ctors']} arguments, "
                         f"not {len(args)}")
            defined = set(re.findall(r"let\s+(\w+)\s*=", "\n".join(ctx))) | {"w", "h"} & set(
                re.findall(r"let\s+(\w+)\s*,\s*(\w+)", "\n".join(ctx))[0] if re.findall(r"let\s+(\w+)\s*,\s*(\w+)", "\n".join(ctx)) else set())
            for sig in re.findall(r"new\s*\(([^)]*)\)", added):
                defined |= set(re.findall(r"(\w+)\s*:", sig))
            own_lets = set(self.own[self.mod_name]["lets"])
            for a in args:
                if a not in defined and a not in own_lets:
                    self.err(f"Scene.fs.diff: {a!r} is not bound in the constructor's (verified) context")
        for mem in re.findall(r"\bni\.(\w+)\(", added):
            if mem not in ni["members"]:
                self.err(f"Scene.fs.diff: NativePixelIntegrator has no member {mem}")
        iface = self.types_in(self.fx["modules"]["Engine.Core.Scene"]["opens"])
        for t in re.findall(r":\s*(I\w+)", added) + re.findall(r":>\s*(I\w+)", added):
            if t not in iface:
                self.err(f"Scene.fs.diff: {t} is not visible in Scene.fs")
        scene_ctor_arities = set(self.fx["modules"]["Engine.Core.Scene"]["types"]["Scene"]["ctors"])
        for m in re.finditer(r"^\s*new\s*\(([^)]*)\)\s*=", added, re.M):
            scene_ctor_arities.add(len([a for a in m.group(1).split(",") if a.strip()]))
        lib = [t for h in self.diffs["EngineCore/Library.fs"] for tag, t in h["lines"] if tag == "+"]
        lt = "\n".join(lib)
        for mod in re.findall(r"open\s+([\w\.]+)", lt):
            if mod not in self.fx["modules"]:
                self.err(f"Library.fs.diff opens unknown module {mod}")
        for args in re.findall(r"new\s+Scene\(([^)]*)\)", lt):
            n = len([a for a in args.split(",") if a.strip()])
            if n not in scene_ctor_arities:
                self.err(f"Library.fs.diff: Scene has no {n}-argument constructor")
        sc = self.fx["modules"]["Engine.Core.Scene"]
        for t in re.findall(r":\s*(Scene\w*)\)", lt):
            if t not in sc["types"] and t not in sc["aliases"]:
                self.err(f"Library.fs.diff: {t} is not declared by Engine.Core.Scene")
        for mem in re.findall(r"\bscene\.(\w+)\(", lt):
            if mem not in sc["types"]["Scene"]["members"]:
                self.err(f"Library.fs.diff: Scene has no member {mem}")

    # ---- 6. layouts and externs ----------------------------------------------------------------
    def check_abi(self):
        import ctypes as C
        from mafrixraytracing_amd import abi
        fsz = {"int32": "i4", "int": "i4", "int64": "i8", "uint64": "u8", "float": "f8", "nativeint": "p8"}

        def flat_fs(tname):
            out = []
            for f, ft in self.own_type(tname)["fields"].items():
                out += flat_fs(ft) if self.own_type(ft) else [fsz[ft]]
            return out

        def flat_ct(ct):
            out = []
            for f, ftp in ct._fields_:
                out += flat_ctype(ftp)
            return out

        def flat_ctype(ftp):
            if hasattr(ftp, "_fields_"):
                return flat_ct(ftp)
            if hasattr(ftp, "_length_"):
                return flat_ctype(ftp._type_) * ftp._length_
            if ftp in (C.c_int32,):
                return ["i4"]
            if ftp in (C.c_int64,):
                return ["i8"]
            if ftp in (C.c_uint64,):
                return ["u8"]
            if ftp in (C.c_double,):
                return ["f8"]
            return ["p8"]  # pointers

        for fs, ct in [("MfxPrim", abi.MfxPrim), ("MfxQuadLight", abi.MfxQuadLight), ("MfxPinhole", abi.MfxPinhole),
                       ("MfxSceneDesc", abi.MfxSceneDesc), ("MfxOptions", abi.MfxOptions)]:
            if self.own_type(fs) is None:
                self.err(f"Native.fs: struct {fs} missing")
            elif flat_fs(fs) != flat_ct(ct):
                self.err(f"Native.fs: {fs} fields {flat_fs(fs)} != C layout {flat_ct(ct)}")
        hdr = open(HEADER).read()
        protos = {m.group(1): m.group(2) for m in re.finditer(r"\b(mfx_\w+)\s*\(([^)]*)\)\s*;", hdr)}
        for ret, name, params in re.findall(r"extern\s+(\w+)\s+(\w+)\(([^)]*)\)", self.native_text):
            if name not in protos:
                self.err(f"Native.fs: extern {name} is not declared in include/mafrix_rt.h")
                continue
            nc = 0 if protos[name].strip() in ("", "void") else len(protos[name].split(","))
            nf = len([p for p in params.split(",") if p.strip()])
            if nc != nf:
                self.err(f"Native.fs: extern {name} has {nf} parameters, the header {nc}")
        # the ABI version: the shim's constant is the header's, and the constructor checks the loaded
        # library against it before it creates a context (a stale .so fails loudly, not on a layout)
        hv = re.search(r"#define\s+MFX_ABI_VERSION\s+(\d+)", hdr)
        fv = re.search(r"let\s+MFX_ABI_VERSION\s*=\s*(\d+)", self.native_text)
        if not fv:
            self.err("Native.fs: no MFX_ABI_VERSION constant")
        elif hv and fv.group(1) != hv.group(1):
            self.err(f"Native.fs: MFX_ABI_VERSION {fv.group(1)} != the header's ABI version {hv.group(1)}")
        chk = re.search(r"let\s+checkAbi\s*\(\)\s*=(.*?)(?=\n\S)", self.native_text, re.S)
        if not chk or "Api.mfx_abi_version()" not in chk.group(1) or \
                not re.search(r"\bv\s*<>\s*MFX_ABI_VERSION\b|\bMFX_ABI_VERSION\s*<>\s*v\b", chk.group(1)):
            self.err("Native.fs: checkAbi must compare Api.mfx_abi_version() with MFX_ABI_VERSION")
        call = re.search(r"^\s+checkAbi \(\)\s*$", self.native_text, re.M)
        cc = self.native_text.find("Api.mfx_create(")
        if not call or cc < 0 or call.start() > cc:
            self.err("Native.fs: the ABI version check must run before mfx_create")

    def run(self):
        self.check_diffs()
        self.check_order()
        self.check_native()
        self.check_added()
        self.check_abi()
        return self.errors


def main():
    errs = Checker().run()
    for e in errs:
        print(e)
    print("OK" if not errs else f"{len(errs)} problem(s)")
    return 1 if errs else 0


if __name__ == "__main__":
    sys.exit(main())
