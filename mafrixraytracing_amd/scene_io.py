"""Scene XML v0.1 + OBJ/MTL loading with the reference's semantics (host side, FP64).

Mirrors EngineCore/Scene/Scene.fs:26-271 (`InitSceneState`), Models/ObjModelLoader.fs:18-340
(`LoadObjModel`) and Models/Obj_Mtl.fs:50-217 (`LoadObjMtl`) closely enough that the same XML +
OBJ inputs produce the same primitive list, in the same order, with the same material indices:

  * MTL materials are added to the global MaterialManager first (as `Lambertian(Ka)`,
    Obj_Mtl.fs:195-196), XML <Materials> are appended after all shapes are parsed
    (Scene.fs:258-259), so an XML `material="i"` addresses slot i of that combined list.
  * 3-vertex faces become Triangle, 4-vertex faces Rect (ObjModelLoader.fs:76-92); negative
    OBJ indices count from the end (:63-64); `usemtl` defaults to "white" and an unknown
    name maps to 0 (Obj_Mtl.fs:30-35).
  * <Shape type="shapelist"> rebuilds every primitive of `model.group` with the XML material
    (Scene.fs:143-161); the light is the first primitive of its group, which must be a Rect:
    NewAreaLight(trig1.v0, trig1.v1, trig1.v2, trig2.v2, trig1.normal, I) (Scene.fs:180-194).
  * Camera defaults fov 60 / aspect 1.333 (Scene.fs:61-62), film defaults 800x800 (:203-204).

Documented extensions: `vt`/`vn`/`o`/`s` lines are accepted and ignored
(an `o` name may contain dots, which FindModel's `model.group` split rejects), trailing whitespace/CR is trimmed from group names (the
FParsec grammar as shipped rejects the bundled meshes — SURVEY.md §0.4); a `.npz` mesh
(converted OBJ, scripts/make_scenes.py) may stand in for an `.obj`; and
<Shape type="sphere"> adds a Sphere (the reference's scene graph has spheres, Scene.fs:159,
but no loader produces one); and <Shape type="instances"> adds translated copies of a group
(`obj_ref`, `material`, `offsets` = "x,y,z;x,y,z;..."): each copy's vertices (a sphere's centre)
are the group's + offset in FP64, appended to the shape list like a shapelist per offset, and the
scene carries that structure as instancing data (mfx_create_instanced). The reference has no
instancing: its flat list is exactly the expansion, which is what every result refers to.
"""
from __future__ import annotations

import math
import os
import xml.etree.ElementTree as ET
from dataclasses import dataclass, field

import numpy as np

from .abi import (INSTANCE_DTYPE, MFX_INSTANCE_VERBATIM, MFX_PRIM_RECT, MFX_PRIM_SPHERE, MFX_PRIM_TRIANGLE,
                  PRIM_DTYPE, SceneArrays)


class SceneError(ValueError):
    """Raised where the reference asserts or throws (Map.find, assert false, ...)."""


# --------------------------------------------------------------------------------------------
# MaterialManager — Core/Interfaces/IMaterial.fs:20-35 (a process-global, append-only list)
# --------------------------------------------------------------------------------------------
class MaterialManager:
    _default: "MaterialManager | None" = None

    def __init__(self):
        self.materials: list[tuple[float, float, float]] = []

    @classmethod
    def GetManager(cls) -> "MaterialManager":
        if cls._default is None:
            cls._default = MaterialManager()
        return cls._default

    @classmethod
    def reset_default(cls):
        cls._default = MaterialManager()

    def Add(self, albedo) -> int:
        self.materials.append(tuple(float(x) for x in albedo))
        return len(self.materials) - 1

    def albedo_table(self) -> np.ndarray:
        return np.array(self.materials, dtype=np.float64).reshape(-1, 3)


# --------------------------------------------------------------------------------------------
# FP64 helpers in the reference's operation order (Point.fs:50-58)
# --------------------------------------------------------------------------------------------
def _sub(a, b):
    return (a[0] - b[0], a[1] - b[1], a[2] - b[2])


def _cross(a, v):
    return (a[1] * v[2] - a[2] * v[1], a[2] * v[0] - a[0] * v[2], a[0] * v[1] - a[1] * v[0])


def tri_normal(v0, v1, v2):
    """Triangle ctor normal: a = e1 x e2; a / |a|  (Trangle.fs:108-113)."""
    a = _cross(_sub(v1, v0), _sub(v2, v0))
    al = math.sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2])
    return (a[0] / al, a[1] / al, a[2] / al)


# --------------------------------------------------------------------------------------------
# OBJ / MTL
# --------------------------------------------------------------------------------------------
@dataclass
class Prim:
    kind: int
    pts: tuple
    material: int


@dataclass
class ObjState:
    """ObjModelLoader.fs:18-53 — vertices plus faces grouped by name (insertion-ordered)."""
    vertices: list = field(default_factory=list)
    groups: dict = field(default_factory=lambda: {"default": []})


def load_mtl(path: str, manager: MaterialManager) -> dict:
    """LoadObjMtl (Obj_Mtl.fs:199-217): each `newmtl` becomes Lambertian(Ka) in the manager."""
    refs: dict[str, int] = {}
    name = None
    ka = (0.0, 0.0, 0.0)
    started = False

    def flush():
        if started:
            refs[name] = manager.Add(ka)

    with open(path, "r", encoding="utf-8", errors="replace") as f:
        for raw in f:
            line = raw.strip()
            if not line or line.startswith("#"):
                continue
            tok = line.split()
            if tok[0] == "newmtl":
                flush()
                started, name, ka = True, line[len("newmtl"):].strip(), (0.0, 0.0, 0.0)
            elif tok[0] == "Ka" and len(tok) >= 4:
                ka = (float(tok[1]), float(tok[2]), float(tok[3]))
    flush()
    return refs


def _vi(i: int, n: int) -> int:
    return i - 1 if i > 0 else n + i  # VertexReferencing.VI, ObjModelLoader.fs:63-64


def load_obj(path: str, manager: MaterialManager) -> ObjState:
    """LoadObjModel (ObjModelLoader.fs:306-340) plus the documented grammar extensions."""
    if path.endswith(".npz"):
        return load_npz_mesh(path, manager)
    st = ObjState()
    with open(path, "r", encoding="utf-8", errors="replace") as f:
        lines = f.read().split("\n")
    # the reference loads the first mtllib before replaying statements (:317-330)
    mtl_refs: dict[str, int] = {}
    for raw in lines:
        tok = raw.split()
        if tok and tok[0] == "mtllib":
            mtl_path = os.path.join(os.path.dirname(path), tok[1])
            mtl_refs = load_mtl(mtl_path, manager)
            break
    usemtl = "white"
    cur = "default"
    for raw in lines:
        line = raw.strip()
        if not line or line.startswith("#"):
            continue
        tok = line.split()
        key = tok[0]
        if key == "v":
            if len(tok) < 4:
                raise SceneError(f"{path}: vertex needs 3 coordinates: {line!r}")
            st.vertices.append((float(tok[1]), float(tok[2]), float(tok[3])))
        elif key in ("vt", "vn", "s", "o", "mtllib", "maplib", "usemap"):
            continue
        elif key == "g":
            cur = line[len(key):].strip()
            st.groups.setdefault(cur, [])
        elif key == "usemtl":
            usemtl = line[len("usemtl"):].strip()
        elif key == "f":
            refs = [int(t.split("/")[0]) for t in tok[1:]]
            n = len(st.vertices)
            pts = tuple(st.vertices[_vi(i, n)] for i in refs)
            mat = mtl_refs.get(usemtl, 0)
            if len(pts) == 3:
                st.groups[cur].append(Prim(MFX_PRIM_TRIANGLE, pts, mat))
            elif len(pts) == 4:
                st.groups[cur].append(Prim(MFX_PRIM_RECT, pts, mat))
            else:
                raise SceneError(f"{path}: face with {len(pts)} vertices (only 3 or 4 supported)")
    return st


def save_npz_mesh(path: str, st: ObjState, mtl: list[tuple[str, tuple]]):
    """Binary form of an ObjState + its MTL (scripts/make_scenes.py)."""
    names = list(st.groups.keys())
    faces, fgroup, fmat = [], [], []
    verts, vidx = [], {}
    for gi, g in enumerate(names):
        for p in st.groups[g]:
            idx = []
            for q in p.pts:
                if q not in vidx:
                    vidx[q] = len(verts)
                    verts.append(q)
                idx.append(vidx[q])
            while len(idx) < 4:
                idx.append(-1)
            faces.append(idx)
            fgroup.append(gi)
            fmat.append(p.material)
    np.savez_compressed(
        path,
        vertices=np.array(verts, dtype=np.float64).reshape(-1, 3),
        faces=np.array(faces, dtype=np.int32).reshape(-1, 4),
        face_group=np.array(fgroup, dtype=np.int32),
        face_mtl=np.array(fmat, dtype=np.int32),
        group_names=np.array(names),
        mtl_names=np.array([m[0] for m in mtl] if mtl else [], dtype=str),
        mtl_ka=np.array([m[1] for m in mtl], dtype=np.float64).reshape(-1, 3),
    )


def load_npz_mesh(path: str, manager: MaterialManager) -> ObjState:
    z = dict(np.load(path, allow_pickle=False))  # read every member once (NpzFile re-reads per access)
    base = len(manager.materials)
    for ka in z["mtl_ka"]:
        manager.Add(ka)
    st = ObjState(vertices=[], groups={})
    st.groups["default"] = []
    names = [str(s) for s in z["group_names"]]
    for g in names:
        st.groups.setdefault(g, [])
    V = z["vertices"].tolist()
    has_mtl = len(z["mtl_ka"]) > 0
    for f, gi, m in zip(z["faces"].tolist(), z["face_group"].tolist(), z["face_mtl"].tolist()):
        k = 3 if f[3] < 0 else 4
        pts = tuple(tuple(V[i]) for i in f[:k])
        mat = base + int(m) if has_mtl else 0
        st.groups[names[gi]].append(Prim(MFX_PRIM_TRIANGLE if k == 3 else MFX_PRIM_RECT, pts, mat))
    return st


# --------------------------------------------------------------------------------------------
# Scene XML v0.1 — Scene.fs:26-271
# --------------------------------------------------------------------------------------------
def _f3(node) -> tuple:
    v = node.get("value")
    parts = v.split(",")
    if len(parts) != 3:
        raise SceneError(f"expected 3 comma-separated floats, got {v!r}")
    return tuple(float(p.strip()) for p in parts)


@dataclass
class SceneState:
    """Parse.SceneState.State (Scene.fs:213-229), flattened."""
    camera: dict
    light: dict
    width: int
    height: int
    prims: list
    manager: MaterialManager
    # <Shape type="instances"> extension: ("verbatim", start, count) / ("instance", key, offset,
    # start, count) runs of `prims`, and the template primitives per key
    segments: list = field(default_factory=list)
    templates: dict = field(default_factory=dict)

    def arrays(self, max_depth: int = 3, width: int | None = None, height: int | None = None) -> SceneArrays:
        inst = None
        if any(sg[0] == "instance" for sg in self.segments):
            tmpl, rows, first_of = [], [], {}
            for sg in self.segments:
                if sg[0] == "instance":
                    _, key, off, _start, count = sg
                    if key not in first_of:
                        first_of[key] = len(tmpl)
                        tmpl.extend(self.templates[key])
                    rows.append((first_of[key], count, off, 0, 0))
                else:
                    _, start, count = sg
                    rows.append((len(tmpl), count, (0.0, 0.0, 0.0), MFX_INSTANCE_VERBATIM, 0))
                    tmpl.extend(self.prims[start:start + count])
            inst = (_prim_array(tmpl), np.array(rows, dtype=INSTANCE_DTYPE))
        return SceneArrays(_prim_array(self.prims), self.manager.albedo_table(), self.light, self.camera,
                           width or self.width, height or self.height, max_depth, instancing=inst)


def _prim_array(plist) -> np.ndarray:
    prims = np.zeros(len(plist), dtype=PRIM_DTYPE)
    for k, p in enumerate(plist):
        prims[k]["kind"] = p.kind
        prims[k]["material"] = p.material
        if p.kind == MFX_PRIM_SPHERE:
            prims[k]["p"][0] = p.pts[0]
            prims[k]["p"][1][0] = p.pts[1]
        else:
            for i, q in enumerate(p.pts):
                prims[k]["p"][i] = q
    return prims


def translate(p: Prim, off) -> Prim:
    """A translated copy (the instances extension): every vertex / a sphere's centre + off, FP64."""
    if p.kind == MFX_PRIM_SPHERE:
        c = p.pts[0]
        return Prim(p.kind, ((c[0] + off[0], c[1] + off[1], c[2] + off[2]), p.pts[1]), p.material)
    return Prim(p.kind, tuple((q[0] + off[0], q[1] + off[1], q[2] + off[2]) for q in p.pts), p.material)


def _find_model(ref: str, models: dict):
    nm = ref.split(".")
    if len(nm) != 2:
        raise SceneError(f"shape reference must be model.group: {ref!r}")
    if nm[0] not in models:
        raise SceneError(f"unknown model {nm[0]!r}")
    groups = models[nm[0]].groups
    if nm[1] not in groups:
        raise SceneError(f"model {nm[0]!r} has no group {nm[1]!r}")
    return groups[nm[1]]


# The light Scene.fs:194 builds when the light group's first primitive is not a Rect: there the
# reference asserts false, which a Release build compiles out, and returns this quad.
RELEASE_FALLBACK_LIGHT = {
    "p": ((-0.24, 1.98, 0.16), (-0.24, 1.98, -0.22), (0.23, 1.98, -0.22), (0.23, 1.98, 0.16)),
    "normal": (0.0, -1.0, 0.0),
    "intensity": (20.0, 20.0, 20.0),
}


def InitSceneState(xml_text: str, base_dir: str = ".", manager: MaterialManager | None = None,
                   light_fallback: str = "debug") -> SceneState:
    """InitSceneState (Scene.fs:265-271): parse XML *text*, version must be 0.1.

    light_fallback: what a light group whose first primitive is not a Rect does. "debug" (the
    default) raises SceneError, as the reference's Debug build does at `assert(false)`
    (Scene.fs:194); "release" returns the hard-coded NewAreaLight of the same line (I = 20,
    normal (0,-1,0)), as its Release build does, where the assert compiles out."""
    if light_fallback not in ("debug", "release"):
        raise ValueError("light_fallback must be 'debug' or 'release'")
    mgr = manager or MaterialManager.GetManager()
    root = ET.fromstring(xml_text)
    if root.get("version") != "0.1":
        raise SceneError("this scene loader only supports version 0.1")
    nodes = {}
    for n in root:
        if n.tag not in ("Camera", "Models", "Materials", "Shapes", "Light", "Film"):
            raise SceneError(f"unknown scene element {n.tag!r}")
        nodes[n.tag] = n
    # Camera (Scene.fs:57-76)
    cam = {"position": (0.0, 0.0, 0.0), "direction": (0.0, 0.0, 0.0), "fov": 60.0, "aspect": 1.333}
    cn = nodes.get("Camera")
    if cn is not None:
        if cn.get("type") != "pinhole":
            raise SceneError("camera type must be pinhole")
        for n in cn:
            a = n.get("name")
            if a == "position":
                cam["position"] = _f3(n)
            elif a == "direction":
                cam["direction"] = _f3(n)
            elif a == "fov":
                cam["fov"] = float(n.get("value"))
            elif a == "aspectratio":
                cam["aspect"] = float(n.get("value"))
            else:
                raise SceneError(f"unknown camera argument {a!r}")
    # Models (Scene.fs:103-135): loading adds MTL materials to the manager, in order
    models = {}
    mn = nodes.get("Models")
    for n in (mn if mn is not None else []):
        if n.get("type") != "obj":
            raise SceneError("model type must be obj")
        fname = ""
        for a in n:
            if a.get("name") == "filename":
                fname = a.get("value")
            else:
                raise SceneError(f"unknown model argument {a.get('name')!r}")
        models[n.get("name")] = load_obj(os.path.join(base_dir, fname), mgr)
    # Light (Scene.fs:179-199)
    ln = nodes.get("Light")
    if ln is None or ln.get("type") != "area":
        raise SceneError("an area light is required")
    ref, inten = "", (0.0, 0.0, 0.0)
    for a in ln:
        if a.get("name") == "shape_ref":
            ref = a.get("value")
        elif a.get("name") == "intensity":
            inten = _f3(a)
        else:
            raise SceneError(f"unknown light argument {a.get('name')!r}")
    grp = _find_model(ref, models)
    if not grp:  # FindModel(...).ToArray()[0] on an empty group throws in either build
        raise SceneError("the light's group has no primitive")
    if grp[0].kind != MFX_PRIM_RECT:
        if light_fallback == "debug":
            raise SceneError("the light's first primitive must be a quad (Rect)")
        light = dict(RELEASE_FALLBACK_LIGHT)
    else:
        q = grp[0].pts
        light = {"p": (q[0], q[1], q[2], q[3]), "normal": tri_normal(q[0], q[1], q[2]), "intensity": inten}
    # Film (Scene.fs:201-211)
    w, h = 800, 800
    fn = nodes.get("Film")
    for a in (fn if fn is not None else []):
        if a.get("name") == "width":
            w = int(a.get("value"))
        elif a.get("name") == "height":
            h = int(a.get("value"))
        else:
            raise SceneError(f"unknown film argument {a.get('name')!r}")
    # Materials (Scene.fs:78-101) — parsed now, added to the manager after the shapes
    xml_mats = []
    matn = nodes.get("Materials")
    for m in (matn if matn is not None else []):
        if m.get("type") != "lambert":
            raise SceneError("material type must be lambert")
        alb = (0.0, 0.0, 0.0)
        for a in m:
            if a.get("name") == "albedo":
                alb = _f3(a)
            else:
                raise SceneError(f"unknown material argument {a.get('name')!r}")
        xml_mats.append(alb)
    # Shapes (Scene.fs:137-177)
    prims = []
    segments, templates = [], {}
    sn = nodes.get("Shapes")
    for s in (sn if sn is not None else []):
        t = s.get("type")
        start = len(prims)
        if t == "instances":  # extension: translated copies of a group
            ref, mat, offs = "", 0, []
            for a in s:
                nm = a.get("name")
                if nm == "obj_ref":
                    ref = a.get("value")
                elif nm == "material":
                    mat = int(a.get("value"))
                elif nm == "offsets":
                    for o in a.get("value").split(";"):
                        if o.strip():
                            parts = o.split(",")
                            if len(parts) != 3:
                                raise SceneError(f"instance offset needs 3 floats: {o!r}")
                            offs.append(tuple(float(x.strip()) for x in parts))
                else:
                    raise SceneError(f"unknown instances argument {nm!r}")
            key = (ref, mat)
            if key not in templates:
                templates[key] = [Prim(p.kind, p.pts, mat) for p in _find_model(ref, models)]
            for off in offs:
                segments.append(("instance", key, off, len(prims), len(templates[key])))
                prims.extend(translate(p, off) for p in templates[key])
            continue
        if t == "shapelist":
            ref, mat = "", 0
            for a in s:
                if a.get("name") == "obj_ref":
                    ref = a.get("value")
                elif a.get("name") == "material":
                    mat = int(a.get("value"))
                else:
                    raise SceneError(f"unknown shape argument {a.get('name')!r}")
            for p in _find_model(ref, models):
                prims.append(Prim(p.kind, p.pts, mat))
        elif t == "sphere":  # extension
            c, r, mat = (0.0, 0.0, 0.0), 1.0, 0
            for a in s:
                nm = a.get("name")
                if nm == "center":
                    c = _f3(a)
                elif nm == "radius":
                    r = float(a.get("value"))
                elif nm == "material":
                    mat = int(a.get("value"))
                else:
                    raise SceneError(f"unknown sphere argument {nm!r}")
            prims.append(Prim(MFX_PRIM_SPHERE, (c, r), mat))
        else:
            raise SceneError(f"unknown shape type {t!r}")
        if len(prims) > start:
            segments.append(("verbatim", start, len(prims) - start))
    for alb in xml_mats:
        mgr.Add(alb)
    for p in prims:
        if not (0 <= p.material < len(mgr.materials)):
            raise SceneError(f"material index {p.material} out of range (manager has {len(mgr.materials)})")
    return SceneState(cam, light, w, h, prims, mgr, segments, templates)


def load_scene_file(path: str, fresh_manager: bool = True, light_fallback: str = "debug", **kw) -> SceneArrays:
    """Convenience: XML file -> SceneArrays, with a fresh MaterialManager (the reference's
    manager is process-global; a fresh one gives the index space of a first load)."""
    with open(path, "r", encoding="utf-8") as f:
        text = f.read()
    mgr = MaterialManager() if fresh_manager else None
    st = InitSceneState(text, base_dir=os.path.dirname(os.path.abspath(path)), manager=mgr,
                        light_fallback=light_fallback)
    return st.arrays(**kw)
