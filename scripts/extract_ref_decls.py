#!/usr/bin/env python3
"""Extract the F# reference's declarations into a committed fixture (tests/golden/ref_fsharp_decls.json).

The fixture is data about the reference, not its text: per module its file, compile position,
`open`s, the types it declares (with their fields and field types, member names, primary-
constructor parameters and struct-ness) and its top-level `let`s; plus, for the three files the
F# shim diffs (EngineCore.fsproj, Scene/Scene.fs, Library.fs), one SHA-1 per line so the diffs'
context and removed lines can be checked without the reference present.

scripts/check_fsharp_shim.py checks fsharp/Native.fs and fsharp/*.diff against it
(tests/test_fsharp_shim.py). Run from the repo root where /root/reference exists:

    python scripts/extract_ref_decls.py [/root/reference] [out.json]
"""
from __future__ import annotations

import hashlib
import json
import os
import re
import sys

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
OUT = sys.argv[2] if len(sys.argv) > 2 else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                         "tests", "golden", "ref_fsharp_decls.json")
PROJ = "EngineCore/EngineCore.fsproj"
HASHED = ["EngineCore/EngineCore.fsproj", "EngineCore/Scene/Scene.fs", "EngineCore/Library.fs"]


def read_lines(path):
    with open(path, encoding="utf-8-sig") as f:
        return [l.rstrip("\r\n") for l in f.read().split("\n")]


def strip_comments(lines):
    """Drop (* ... *) blocks and // line comments (string literals in the reference hold no //)."""
    out, depth = [], 0
    for l in lines:
        s, i, buf = l, 0, ""
        while i < len(s):
            if depth == 0 and s.startswith("//", i):
                break
            if s.startswith("(*", i) and not s.startswith("(*)", i):
                depth += 1
                i += 2
                continue
            if depth and s.startswith("*)", i):
                depth -= 1
                i += 2
                continue
            if depth == 0:
                buf += s[i]
            i += 1
        out.append(buf.rstrip())
    return out


def indent(l):
    return len(l) - len(l.lstrip(" "))


TYPE_RE = re.compile(r"^(?:type|and)\s+(?:\[<([^>]*)>\]\s*)?(?:private\s+|internal\s+)?(\w+)(<[^>]*>)?\s*(\((.*?)\))?")
VAL_RE = re.compile(r"^val\s+(?:mutable\s+)?(?:private\s+)?(\w+)\s*:\s*(.+?)\s*$")
MEMBER_RE = re.compile(r"^(?:override|default|member)\s+(?:private\s+|inline\s+)*(\w+)\.(\w+)")
STATIC_RE = re.compile(r"^static\s+member\s+(?:private\s+|inline\s+)*(?:\(([^)]*)\)|(\w+))")
ABSTRACT_RE = re.compile(r"^abstract\s+(?:member\s+)?(\w+)")
LET_RE = re.compile(r"^let\s+(?:private\s+|inline\s+|mutable\s+|rec\s+)*(\w+)")


def parse_file(rel, text_lines):
    lines = strip_comments(text_lines)
    modules = {}
    file_mod = None
    stack = []  # (indent, qualified name) of nested modules

    def cur_module():
        return stack[-1][1] if stack else file_mod

    cur_type = None  # (indent, module, name)
    pending_attrs = ""  # an attribute line ([<Struct>]) applies to the type declared next
    for raw in lines:
        if not raw.strip():
            continue
        ind = indent(raw)
        l = raw.strip()
        if cur_type and ind <= cur_type[0]:
            cur_type = None
        while stack and ind <= stack[-1][0]:
            stack.pop()
        m = re.match(r"^module\s+(?:rec\s+)?([\w\.]+)\s*$", l)
        if m and ind == 0 and file_mod is None:
            file_mod = m.group(1)
            modules.setdefault(file_mod, {"file": rel, "opens": [], "types": {}, "lets": [], "aliases": {}})
            continue
        m = re.match(r"^namespace\s+([\w\.]+)", l)
        if m and ind == 0:
            file_mod = m.group(1)
            modules.setdefault(file_mod, {"file": rel, "opens": [], "types": {}, "lets": [], "aliases": {},
                                          "namespace": True})
            continue
        m = re.match(r"^module\s+(\w+)\s*=", l)
        if m:
            q = f"{cur_module()}.{m.group(1)}" if cur_module() else m.group(1)
            stack.append((ind, q))
            modules.setdefault(q, {"file": rel, "opens": [], "types": {}, "lets": [], "aliases": {}})
            continue
        mod = cur_module()
        if mod is None:
            continue
        md = modules[mod]
        m = re.match(r"^open\s+([\w\.]+)", l)
        if m:
            md["opens"].append(m.group(1))
            continue
        if re.match(r"^\[<[^>]*>\]$", l):
            pending_attrs += l
            continue
        m = TYPE_RE.match(l)
        if m and (cur_type is None or ind <= cur_type[0]):
            attrs, name, gen, _, params = m.groups()
            attrs = (attrs or "") + pending_attrs
            pending_attrs = ""
            am = re.match(r"^(?:type|and)\s+(?:\[<[^>]*>\]\s*)?(\w+)\s*=\s*([\w\.]+)\s*$", l)
            if am and not re.match(r"^(struct|class|interface|\{)$", am.group(2)):
                md["aliases"][am.group(1)] = am.group(2)
                continue
            t = md["types"].setdefault(name, {"fields": {}, "members": [], "static": [], "abstract": [],
                                              "ctor_params": [], "struct": False, "ctors": []})
            if attrs and "Struct" in attrs:
                t["struct"] = True
            if params is not None:
                t["ctor_params"] = [p.strip() for p in re.split(r",(?![^\[]*\])", params) if p.strip()]
            cur_type = (ind, mod, name)
            continue
        if cur_type:
            t = modules[cur_type[1]]["types"][cur_type[2]]
            if l == "struct":
                t["struct"] = True
            m = VAL_RE.match(l)
            if m:
                t["fields"][m.group(1)] = m.group(2)
                continue
            m = MEMBER_RE.match(l)
            if m:
                if m.group(2) not in t["members"]:
                    t["members"].append(m.group(2))
                continue
            m = STATIC_RE.match(l)
            if m:
                nm = m.group(1) or m.group(2)
                if nm and nm not in t["static"]:
                    t["static"].append(nm.strip())
                continue
            m = ABSTRACT_RE.match(l)
            if m:
                if m.group(1) not in t["abstract"]:
                    t["abstract"].append(m.group(1))
                continue
            m = re.match(r"^new\s*\((.*)\)\s*=", l)
            if m:
                t["ctors"].append(len([p for p in re.split(r",(?![^<]*>)", m.group(1)) if p.strip()]))
                continue
        else:
            m = LET_RE.match(l)
            if m and (not stack or ind > stack[-1][0]) and (stack or ind == 0):
                md["lets"].append(m.group(1))
    return modules


def main():
    proj_lines = read_lines(os.path.join(REF, PROJ))
    order = [m.group(1).replace("\\", "/") for m in
             (re.search(r'<Compile Include="([^"]+)"', l) for l in proj_lines) if m]
    modules = {}
    for pos, rel in enumerate(order):
        path = os.path.join(REF, "EngineCore", rel)
        for name, md in parse_file("EngineCore/" + rel, read_lines(path)).items():
            md["position"] = pos
            modules[name] = md
    hashes = {}
    for rel in HASHED:
        hashes[rel] = [hashlib.sha1(l.encode("utf-8")).hexdigest()[:16] for l in read_lines(os.path.join(REF, rel))]
    out = {"generator": "scripts/extract_ref_decls.py", "reference": "NAIVEddd/MafrixRaytracing EngineCore",
           "compile_order": ["EngineCore/" + r for r in order], "modules": modules, "line_sha1_16": hashes}
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(f"{OUT}: {len(modules)} modules, {sum(len(m['types']) for m in modules.values())} types")


if __name__ == "__main__":
    main()
