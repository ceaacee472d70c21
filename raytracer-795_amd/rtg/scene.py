"""Host-side scene model: the state the reference's Parser leaves in `Scene`.

Mirrors src/Parser.h (ParseSceneAttributes/Cameras/BRDF/Materials/Textures/
Transformations/Vertices/TextureCoordinates/Objects/Lights) and src/Scene.cpp:455-504,
including its quirks (texture-map state carried from one TextureMap to the next,
`ParseObjectTransformations` only recognising a composite as the first token,
quad faces of PLY meshes split into (0,1,2),(2,3,0)).  `Scene.to_desc()` flattens the
model into the C ABI descriptor of include/rtg.h; `write_xml()` serialises it back to
the reference's XML format (floats printed so they parse back bit-exactly).
"""
from __future__ import annotations

import ctypes as C
import math
import os
import re
import struct
import xml.etree.ElementTree as ET
from dataclasses import dataclass, field

import numpy as np

from . import _abi as A

f32 = np.float32


def _fmt(x) -> str:
    return np.format_float_positional(f32(x), unique=True, trim="-")


def _fmts(v) -> str:
    return " ".join(_fmt(x) for x in v)


def _f3(text: str | None, default=(0.0, 0.0, 0.0)):
    if text is None:
        return np.array(default, dtype=f32)
    vals = [float(t) for t in text.split()[:3]]
    while len(vals) < 3:
        vals.append(0.0)
    return np.array(vals, dtype=f32)


@dataclass
class Camera:                       # src/Camera.h, src/Parser.h:52-164
    id: int = 1
    position: np.ndarray = field(default_factory=lambda: np.zeros(3, f32))
    gaze: np.ndarray = field(default_factory=lambda: np.array([0, 0, -1], f32))
    up: np.ndarray = field(default_factory=lambda: np.array([0, 1, 0], f32))
    near_plane: tuple = (-1.0, 1.0, -1.0, 1.0)       # left right bottom top
    near_distance: float = 1.0
    nx: int = 64
    ny: int = 64
    image_name: str = "out.png"
    num_samples: int = 1
    focus_distance: float = 0.0
    aperture_size: float = 0.0
    is_dof: bool = False
    left_handed: bool = False
    integrator: int = A.INTEGRATOR_REFERENCE     # hw7 <Renderer>PathTracing</Renderer>
    pt_flags: int = 0                            # hw7 <RendererParams> (A.PT_*)
    tonemap: tuple | None = None                 # hw5 <Tonemap>: (key, burn %, saturation, gamma)
    # XML-only conveniences kept for write_xml round trips
    gaze_point: np.ndarray | None = None
    fov_y: float | None = None

    def desc(self) -> A.CameraDesc:
        d = A.CameraDesc()
        d.position = A.F3(*map(float, self.position))
        d.gaze = A.F3(*map(float, self.gaze))
        d.up = A.F3(*map(float, self.up))
        d.left, d.right, d.bottom, d.top = (float(f32(v)) for v in self.near_plane)
        d.near_distance = float(f32(self.near_distance))
        d.nx, d.ny = int(self.nx), int(self.ny)
        d.num_samples = int(self.num_samples)
        d.is_dof = int(bool(self.is_dof))
        d.focus_distance = float(f32(self.focus_distance))
        d.aperture_size = float(f32(self.aperture_size))
        d.left_handed = int(bool(self.left_handed))
        d.integrator = int(self.integrator)
        d.pt_flags = int(self.pt_flags)
        return d


@dataclass
class Material:                     # src/Material.h, src/Parser.h:304-474
    id: int = 1
    type: int = A.MAT_NORMAL
    brdf: int = A.BRDF_NONE
    phong_exp: int = 0
    is_rough: bool = False
    roughness: float = 0.0
    ambient: tuple = (0.1, 0.1, 0.1)
    diffuse: tuple = (0.5, 0.5, 0.5)
    specular: tuple = (0.0, 0.0, 0.0)
    mirror: tuple = (0.0, 0.0, 0.0)
    refraction_index: float = 0.0
    absorption_index: float = 0.0
    absorption_coeff: tuple = (0.0, 0.0, 0.0)
    brdf_id: int = -1               # XML BRDF attribute (write_xml)


@dataclass
class Texture:                      # src/Texture.h
    kind: int = A.TEX_IMAGE
    decal: int = A.DECAL_NONE
    interp: int = A.INTERP_NN
    noise_conv: int = A.NC_LINEAR
    normalizer: int = 255
    noise_scale: float = 1.0
    bump_factor: float = 1.0
    texels: np.ndarray | None = None   # (h, w, 3) float32, row 0 = first image row
    image_id: int = 0                   # XML ImageId (write_xml)


@dataclass
class Light:                        # src/Light.h
    type: int = A.LIGHT_POINT
    position: tuple = (0.0, 0.0, 0.0)
    direction: tuple = (0.0, -1.0, 0.0)
    intensity: tuple = (0.0, 0.0, 0.0)
    coverage_deg: float = 0.0
    falloff_deg: float = 0.0
    size: float = 0.0
    texture: int = -1                   # environment: 0-based texture index
    image_id: int = 0


@dataclass
class Object:                       # src/Shape.h (Sphere / Triangle / Mesh)
    type: int = A.OBJ_SPHERE
    id: int = 1
    material: int = 1
    textures: list = field(default_factory=list)
    texture_offset: int = 0
    smooth: bool = False
    xforms: list = field(default_factory=list)      # [(type, index)]
    blur: tuple = (0.0, 0.0, 0.0)
    center: int = 1
    radius: float = 1.0
    v: tuple = (1, 2, 3)
    faces: np.ndarray | None = None                 # (F,3) int32, 1-based, offsets applied
    ply_file: str | None = None                     # write_xml: emit faces as a PLY
    xml_vertex_offset: int = 0
    is_light: bool = False                          # hw7 <LightSphere> / <LightMesh>
    radiance: tuple = (0.0, 0.0, 0.0)


@dataclass
class Instance:                     # src/Instance.h
    base_object: int = 0
    id: int = 1
    material: int = 1
    reset_transform: bool = False
    xforms: list = field(default_factory=list)
    blur: tuple = (0.0, 0.0, 0.0)


@dataclass
class Scene:
    max_depth: int = 1
    shadow_eps: float = 0.002
    int_eps: float = 0.001
    background: tuple = (0.0, 0.0, 0.0)
    ambient: tuple = (0.0, 0.0, 0.0)
    cameras: list = field(default_factory=list)
    materials: list = field(default_factory=list)
    textures: list = field(default_factory=list)
    images: list = field(default_factory=list)          # image file paths (1-based ImageId)
    translations: list = field(default_factory=list)
    scalings: list = field(default_factory=list)
    rotations: list = field(default_factory=list)       # (angle_deg, x, y, z)
    composites: list = field(default_factory=list)      # 16 floats, glm column-major
    vertices: np.ndarray = field(default_factory=lambda: np.zeros((0, 3), f32))
    texcoords: np.ndarray = field(default_factory=lambda: np.zeros((0, 2), f32))
    objects: list = field(default_factory=list)
    instances: list = field(default_factory=list)
    lights: list = field(default_factory=list)
    background_texture: int = -1
    environment_light: int = -1

    # ------------------------------------------------------------------ C ABI
    def to_desc(self):
        """Return (SceneDesc, keepalive) — the descriptor of include/rtg.h."""
        keep = []

        def arr(a, dtype, ctype):
            a = np.ascontiguousarray(a, dtype=dtype)
            keep.append(a)
            if a.size == 0:
                return C.cast(None, C.POINTER(ctype)), a
            return a.ctypes.data_as(C.POINTER(ctype)), a

        d = A.SceneDesc()
        d.abi_version = A.loaded_abi()
        d.max_recursion_depth = int(self.max_depth)
        d.shadow_ray_eps = float(f32(self.shadow_eps))
        d.intersection_test_eps = float(f32(self.int_eps))
        d.background = A.F3(*map(float, np.asarray(self.background, f32)))
        d.ambient_light = A.F3(*map(float, np.asarray(self.ambient, f32)))
        d.background_texture = int(self.background_texture)
        d.environment_light = int(self.environment_light)
        d.vertices, v = arr(np.asarray(self.vertices, f32).reshape(-1, 3), f32, C.c_float)
        d.num_vertices = v.shape[0]
        d.texcoords, t = arr(np.asarray(self.texcoords, f32).reshape(-1, 2), f32, C.c_float)
        d.num_texcoords = t.shape[0]
        faces, face_first = [], []
        n = 0
        for o in self.objects:
            if o.type == A.OBJ_MESH:
                fa = np.asarray(o.faces, np.int32).reshape(-1, 3)
                face_first.append(n)
                faces.append(fa)
                n += fa.shape[0]
            else:
                face_first.append(0)
        allf = np.concatenate(faces) if faces else np.zeros((0, 3), np.int32)
        d.faces, fa = arr(allf, np.int32, C.c_int32)
        d.num_faces = fa.shape[0]
        d.translations, a = arr(np.asarray(self.translations, f32).reshape(-1, 3), f32, C.c_float)
        d.num_translations = a.shape[0]
        d.scalings, a = arr(np.asarray(self.scalings, f32).reshape(-1, 3), f32, C.c_float)
        d.num_scalings = a.shape[0]
        d.rotations, a = arr(np.asarray(self.rotations, f32).reshape(-1, 4), f32, C.c_float)
        d.num_rotations = a.shape[0]
        d.composites, a = arr(np.asarray(self.composites, f32).reshape(-1, 16), f32, C.c_float)
        d.num_composites = a.shape[0]
        refs = []
        objs = (A.ObjectDesc * max(1, len(self.objects)))()
        for i, o in enumerate(self.objects):
            od = objs[i]
            od.type = o.type
            od.id = o.id
            od.material = o.material
            od.num_textures = len(o.textures)
            for k, tx in enumerate(o.textures[:2]):
                od.textures[k] = tx
            od.texture_offset = o.texture_offset
            od.smooth = int(bool(o.smooth))
            od.xform_first = len(refs)
            od.xform_count = len(o.xforms)
            refs.extend(o.xforms)
            od.blur = A.F3(*map(float, np.asarray(o.blur, f32)))
            od.center = o.center
            od.radius = float(f32(o.radius))
            od.v = A.I3(*o.v)
            od.face_first = face_first[i]
            od.face_count = 0 if o.faces is None else int(np.asarray(o.faces).reshape(-1, 3).shape[0])
            od.is_light = int(bool(o.is_light))
            od.radiance = A.F3(*map(float, np.asarray(o.radiance, f32)))
        keep.append(objs)
        insts = (A.InstanceDesc * max(1, len(self.instances)))()
        for i, it in enumerate(self.instances):
            idd = insts[i]
            idd.base_object = it.base_object
            idd.id = it.id
            idd.material = it.material
            idd.reset_transform = int(bool(it.reset_transform))
            idd.xform_first = len(refs)
            idd.xform_count = len(it.xforms)
            refs.extend(it.xforms)
            idd.blur = A.F3(*map(float, np.asarray(it.blur, f32)))
        keep.append(insts)
        xr = (A.XformRef * max(1, len(refs)))()
        for i, (ty, ix) in enumerate(refs):
            xr[i].type, xr[i].index = ty, ix
        keep.append(xr)
        mats = (A.MaterialDesc * max(1, len(self.materials)))()
        for i, m in enumerate(self.materials):
            md = mats[i]
            md.type, md.brdf, md.phong_exp = m.type, m.brdf, m.phong_exp
            md.is_rough, md.roughness = int(bool(m.is_rough)), float(f32(m.roughness))
            md.ambient = A.F3(*map(float, np.asarray(m.ambient, f32)))
            md.diffuse = A.F3(*map(float, np.asarray(m.diffuse, f32)))
            md.specular = A.F3(*map(float, np.asarray(m.specular, f32)))
            md.mirror = A.F3(*map(float, np.asarray(m.mirror, f32)))
            md.refraction_index = float(f32(m.refraction_index))
            md.absorption_index = float(f32(m.absorption_index))
            md.absorption_coeff = A.F3(*map(float, np.asarray(m.absorption_coeff, f32)))
        keep.append(mats)
        texs = (A.TextureDesc * max(1, len(self.textures)))()
        for i, tx in enumerate(self.textures):
            td = texs[i]
            td.kind, td.decal, td.interp, td.noise_conv = tx.kind, tx.decal, tx.interp, tx.noise_conv
            td.normalizer = tx.normalizer
            td.noise_scale, td.bump_factor = float(f32(tx.noise_scale)), float(f32(tx.bump_factor))
            if tx.texels is not None:
                tex = np.ascontiguousarray(tx.texels, f32)
                keep.append(tex)
                td.height, td.width = tex.shape[0], tex.shape[1]
                td.texels = tex.ctypes.data_as(A.PF)
        keep.append(texs)
        lts = (A.LightDesc * max(1, len(self.lights)))()
        for i, l in enumerate(self.lights):
            ld = lts[i]
            ld.type = l.type
            ld.position = A.F3(*map(float, np.asarray(l.position, f32)))
            ld.direction = A.F3(*map(float, np.asarray(l.direction, f32)))
            ld.intensity = A.F3(*map(float, np.asarray(l.intensity, f32)))
            ld.coverage_deg, ld.falloff_deg = float(f32(l.coverage_deg)), float(f32(l.falloff_deg))
            ld.size = float(f32(l.size))
            ld.texture = l.texture
        keep.append(lts)
        d.xform_refs, d.num_xform_refs = xr, len(refs)
        d.objects, d.num_objects = objs, len(self.objects)
        d.instances, d.num_instances = insts, len(self.instances)
        d.materials, d.num_materials = mats, len(self.materials)
        d.textures, d.num_textures = texs, len(self.textures)
        d.lights, d.num_lights = lts, len(self.lights)
        return d, keep

    # ------------------------------------------------------------------ counts
    def num_triangles(self) -> int:
        n = 0
        for o in self.objects:
            if o.type == A.OBJ_MESH:
                n += int(np.asarray(o.faces).reshape(-1, 3).shape[0])
            elif o.type == A.OBJ_TRIANGLE:
                n += 1
        return n


# ============================================================================ XML parser
def _text(el, tag):
    c = el.find(tag)
    return None if c is None else (c.text or "")


def _attr_prefix(el, name_prefix: str, value_prefix: str) -> bool:
    """tinyxml2 attribute scan with strncmp semantics used by Parser.h."""
    for k, v in el.attrib.items():
        if k[:len(name_prefix)] == name_prefix:
            return v[:len(value_prefix)] == value_prefix
    return False


def _query_int(text: str | None, default: int) -> int:
    if text is None:
        return default
    m = re.match(r"\s*([-+]?\d+)", text)
    return int(m.group(1)) if m else default


def _query_float(text: str | None, default: float) -> float:
    if text is None:
        return default
    m = re.match(r"\s*([-+]?(?:\d+\.?\d*|\.\d+)(?:[eE][-+]?\d+)?)", text)
    return float(f32(float(m.group(1)))) if m else default


def parse_object_transformations(s: str) -> list:
    """Parser::ParseObjectTransformations (src/Parser.h:769-796), quirks included."""
    out = []
    kinds = {"t": A.XF_TRANSLATION, "s": A.XF_SCALING, "r": A.XF_ROTATION, "c": A.XF_COMPOSITE}
    cur, n = 0, len(s)
    while cur < n:
        ch = s[cur]
        if ch in kinds:
            m = re.match(r"\s*([-+]?\d+)", s[cur + 1:])
            out.append((kinds[ch], int(m.group(1)) if m else 0))
        cur += 1
        while cur < n and s[cur] not in "str":
            cur += 1
    return out


def _parse_textures_list(text: str) -> list:
    vals = [int(v) for v in re.findall(r"[-+]?\d+", text)]
    if " " in text:
        return vals[:2]
    return vals[:1]


def load_image(path: str) -> np.ndarray:
    """Decode an image texture the way src/Texture.cpp:133-300 exposes it: 8-bit RGB(A) raw
    values 0..255 as floats, row 0 first.  OpenEXR goes through the native decoder
    (librtghost rtgh_read_image, host/exr_read.cpp): LoadEXR's linear R, G, B floats."""
    low = path.lower()
    if low.endswith(".exr"):
        from . import native
        return native.read_image(path)
    if low.endswith(".ppm") or low.endswith(".pnm"):
        return read_ppm(path)
    from PIL import Image  # decode is host I/O, out of the hot path
    im = Image.open(path)
    if im.mode == "I;16" or im.mode == "I":
        im = im.point(lambda v: v / 256).convert("L")
    im = im.convert("RGB")
    return np.asarray(im, dtype=np.uint8).astype(f32)


def read_ppm(path: str) -> np.ndarray:
    with open(path, "rb") as fh:
        data = fh.read()
    toks = re.findall(rb"\S+", data[:64])
    magic = toks[0]
    w, h, mx = int(toks[1]), int(toks[2]), int(toks[3])
    if magic == b"P6":
        hdr = re.match(rb"P6\s+\d+\s+\d+\s+\d+\s", data)
        px = np.frombuffer(data[hdr.end():hdr.end() + w * h * 3], np.uint8)
        return px.reshape(h, w, 3).astype(f32) * f32(255.0 / mx) if mx != 255 else px.reshape(h, w, 3).astype(f32)
    vals = np.array([int(v) for v in re.findall(rb"\d+", data)[4:4 + w * h * 3]], dtype=f32)
    return vals.reshape(h, w, 3)


def read_ply(path: str):
    """Minimal PLY reader for what happly gives Parser.h (src/Parser.h:1020-1106):
    vertex x,y,z (+u,v) and face index lists.  ascii and binary_little_endian."""
    with open(path, "rb") as fh:
        data = fh.read()
    end = data.index(b"end_header")
    end = data.index(b"\n", end) + 1
    header = data[:end].decode("ascii").splitlines()
    fmt = None
    elements = []
    for line in header:
        p = line.split()
        if not p:
            continue
        if p[0] == "format":
            fmt = p[1]
        elif p[0] == "element":
            elements.append([p[1], int(p[2]), []])
        elif p[0] == "property":
            if p[1] == "list":
                elements[-1][2].append(("list", p[4], p[2], p[3]))
            else:
                elements[-1][2].append(("scalar", p[2], p[1]))
    tmap = {"char": "i1", "int8": "i1", "uchar": "u1", "uint8": "u1", "short": "i2", "int16": "i2",
            "ushort": "u2", "uint16": "u2", "int": "i4", "int32": "i4", "uint": "u4", "uint32": "u4",
            "float": "f4", "float32": "f4", "double": "f8", "float64": "f8"}
    verts, uvs, faces = None, None, []
    body = data[end:]
    if fmt == "ascii":
        toks = body.split()
        pos = 0
        for name, count, props in elements:
            if name == "vertex":
                names = [pp[1] for pp in props]
                vals = np.array(toks[pos:pos + count * len(props)], dtype=np.float64).reshape(count, len(props))
                pos += count * len(props)
                verts = vals[:, [names.index("x"), names.index("y"), names.index("z")]]
                if "u" in names:
                    uvs = vals[:, [names.index("u"), names.index("v")]]
            else:
                for _ in range(count):
                    for pp in props:
                        if pp[0] == "list":
                            k = int(toks[pos]); pos += 1
                            if name == "face":
                                faces.append([int(t) for t in toks[pos:pos + k]])
                            pos += k
                        else:
                            pos += 1
    elif fmt == "binary_little_endian":
        off = 0
        for name, count, props in elements:
            if all(pp[0] == "scalar" for pp in props):
                dt = np.dtype([(pp[1], "<" + tmap[pp[2]]) for pp in props])
                arr = np.frombuffer(body, dt, count, off)
                off += dt.itemsize * count
                if name == "vertex":
                    verts = np.stack([arr["x"], arr["y"], arr["z"]], 1).astype(np.float64)
                    if "u" in dt.names:
                        uvs = np.stack([arr["u"], arr["v"]], 1).astype(np.float64)
            else:
                cdt = None
                for _ in range(count):
                    for pp in props:
                        if pp[0] == "list":
                            ct = np.dtype("<" + tmap[pp[2]])
                            it = np.dtype("<" + tmap[pp[3]])
                            k = int(np.frombuffer(body, ct, 1, off)[0]); off += ct.itemsize
                            idx = np.frombuffer(body, it, k, off); off += it.itemsize * k
                            if name == "face":
                                faces.append(idx.tolist())
                        else:
                            off += np.dtype(tmap[pp[2]]).itemsize
                del cdt
    else:
        raise ValueError(f"unsupported PLY format {fmt}")
    return verts, uvs, faces


def write_ply_binary(path: str, verts: np.ndarray, quads_or_tris: np.ndarray, uvs: np.ndarray | None = None):
    """Little-endian binary PLY (float32 xyz[uv], uchar/int index lists)."""
    verts = np.asarray(verts, f32)
    f = np.asarray(quads_or_tris, np.int32)
    k = f.shape[1]
    with open(path, "wb") as fh:
        hdr = ["ply", "format binary_little_endian 1.0", f"element vertex {verts.shape[0]}",
               "property float x", "property float y", "property float z"]
        if uvs is not None:
            hdr += ["property float u", "property float v"]
        hdr += [f"element face {f.shape[0]}", "property list uchar int vertex_indices", "end_header"]
        fh.write(("\n".join(hdr) + "\n").encode())
        if uvs is not None:
            vv = np.concatenate([verts, np.asarray(uvs, f32)], 1)
        else:
            vv = verts
        fh.write(np.ascontiguousarray(vv, "<f4").tobytes())
        rec = np.zeros(f.shape[0], dtype=[("n", "u1"), ("i", "<i4", (k,))])
        rec["n"] = k
        rec["i"] = f
        fh.write(rec.tobytes())


def _dir_of(xml_path: str) -> str:
    # Parser.h keeps everything up to and including the last '/'
    i = xml_path.rfind("/")
    return xml_path[:i + 1] if i >= 0 else ""


def parse_xml(xml_path: str) -> Scene:
    """Parse a CENG795 scene file like `new Scene(xml)` (src/Scene.cpp:455-504)."""
    root = ET.parse(xml_path).getroot()
    sc = Scene()
    base = _dir_of(xml_path)
    # ParseSceneAttributes (src/Parser.h:17-50)
    sc.max_depth = _query_int(_text(root, "MaxRecursionDepth"), 1)
    sc.background = tuple(_f3(_text(root, "BackgroundColor")))
    sc.shadow_eps = _query_float(_text(root, "ShadowRayEpsilon"), float(f32(0.002)))
    sc.int_eps = _query_float(_text(root, "IntersectionTestEpsilon"), float(f32(0.001)))
    # ParseCameras (Parser.h:52-164)
    for ce in root.find("Cameras").findall("Camera"):
        cam = Camera()
        cam.id = int(ce.get("id", "0"))
        cam.left_handed = _attr_prefix(ce, "handedness", "left")
        if ce.find("FocusDistance") is not None:
            cam.focus_distance = _query_float(_text(ce, "FocusDistance"), 0.0)
            cam.is_dof = True
        if ce.find("ApertureSize") is not None:
            cam.aperture_size = _query_float(_text(ce, "ApertureSize"), 0.0)
        cam.num_samples = _query_int(_text(ce, "NumSamples"), 1)
        cam.position = _f3(_text(ce, "Position"))
        if ce.find("Gaze") is not None:
            cam.gaze = _f3(_text(ce, "Gaze"))
        if ce.find("GazePoint") is not None:
            gp = _f3(_text(ce, "GazePoint"))
            cam.gaze_point = gp
            cam.gaze = (gp - cam.position).astype(f32)
        cam.up = _f3(_text(ce, "Up"))
        cam.near_distance = _query_float(_text(ce, "NearDistance"), 1.0)
        res = [int(v) for v in _text(ce, "ImageResolution").split()[:2]]
        cam.nx, cam.ny = res
        cam.image_name = (_text(ce, "ImageName") or "").strip()
        if ce.find("NearPlane") is not None:
            cam.near_plane = tuple(float(f32(float(v))) for v in _text(ce, "NearPlane").split()[:4])
        if ce.find("FovY") is not None:
            fov = f32(_query_float(_text(ce, "FovY"), 0.0))
            cam.fov_y = float(fov)
            fovr = f32(float(f32(fov * f32(0.5))) * (math.pi / float(f32(180.0))))
            aspect = f32(cam.nx) / f32(cam.ny)
            y = f32(f32(math.tan(float(fovr))) * f32(cam.near_distance))
            x = f32(aspect * y)
            cam.near_plane = (float(-x), float(x), float(-y), float(y))
        # hw5 <Tonemap> (pages/Page5.md:47-53; no parser code in src/): Photographic TMO only
        tm = ce.find("Tonemap")
        if tm is not None and (_text(tm, "TMO") or "Photographic").strip().lower().startswith("photographic"):
            opts = [float(f32(float(v))) for v in (_text(tm, "TMOOptions") or "0.18 1").split()[:2]]
            while len(opts) < 2:
                opts.append(0.0)
            cam.tonemap = (opts[0], opts[1], _query_float(_text(tm, "Saturation"), 1.0),
                           _query_float(_text(tm, "Gamma"), float(f32(2.2))))
        # hw7 (pages/Page7.md; the reference parser has no such tags): <Renderer>PathTracing</Renderer>
        # and <RendererParams>ImportanceSampling NextEventEstimation RussianRoulette</RendererParams>
        ren = _text(ce, "Renderer")
        if ren is not None and ren.strip().lower().startswith("pathtracing"):
            cam.integrator = A.INTEGRATOR_PATH
        rp = _text(ce, "RendererParams")
        if rp is not None:
            for tok in rp.split():
                cam.pt_flags |= {"importancesampling": A.PT_IMPORTANCE, "nexteventestimation": A.PT_NEE,
                                 "russianroulette": A.PT_RUSSIAN_ROULETTE}.get(tok.strip().lower(), 0)
        sc.cameras.append(cam)
    # ParseBRDF (Parser.h:166-302)
    brdfs = []   # (type, id, exponent)
    be = root.find("BRDFs")
    if be is not None:
        for tag in ("ModifiedBlinnPhong", "OriginalBlinnPhong", "ModifiedPhong", "OriginalPhong", "TorranceSparrow"):
            for b in be.findall(tag):
                bid = int(b.get("id", "0"))
                ex = _query_int(_text(b, "Exponent"), 0)
                if tag == "ModifiedBlinnPhong":
                    ty = A.BRDF_MBPN if _attr_prefix(b, "normalized", "true") else A.BRDF_MBP
                elif tag == "OriginalBlinnPhong":
                    ty = A.BRDF_OBP
                elif tag == "ModifiedPhong":
                    ty = A.BRDF_MPN if _attr_prefix(b, "normalized", "true") else A.BRDF_MP
                elif tag == "OriginalPhong":
                    ty = A.BRDF_OP
                else:
                    ty = A.BRDF_TSF if _attr_prefix(b, "kdfresnel", "true") else A.BRDF_TS
                brdfs.append((ty, bid, ex))
    # ParseMaterials (Parser.h:304-474)
    for me in root.find("Materials").findall("Material"):
        m = Material()
        m.id = int(me.get("id", "0"))
        degamma = _attr_prefix(me, "degamma", "true")
        bidx = int(me.get("BRDF")) if me.get("BRDF") is not None else -1
        m.brdf_id = bidx
        if bidx != -1:
            for ty, bid, ex in brdfs:
                if bid == bidx:
                    m.phong_exp, m.brdf = ex, ty
        m.ambient = tuple(_f3(_text(me, "AmbientReflectance")))
        m.diffuse = tuple(_f3(_text(me, "DiffuseReflectance")))
        m.specular = tuple(_f3(_text(me, "SpecularReflectance")))
        if degamma:
            g = float(f32(2.2))
            m.ambient = tuple(f32(math.pow(float(v), g)) for v in m.ambient)
            m.diffuse = tuple(f32(math.pow(float(v), g)) for v in m.diffuse)
            m.specular = tuple(f32(math.pow(float(v), g)) for v in m.specular)
        if me.find("Roughness") is not None:
            m.roughness = _query_float(_text(me, "Roughness"), 0.0)
            m.is_rough = True
        m.mirror = tuple(_f3(_text(me, "MirrorReflectance")))
        if me.find("PhongExponent") is not None:
            m.phong_exp = _query_int(_text(me, "PhongExponent"), m.phong_exp)
        m.type = A.MAT_NORMAL
        for k, v in me.attrib.items():
            if k[:4] == "type":
                if v[:10] == "dielectric":
                    m.type = A.MAT_DIELECTRIC
                elif v[:9] == "conductor":
                    m.type = A.MAT_CONDUCTOR
                elif v[:6] == "mirror":
                    m.type = A.MAT_MIRROR
                break
        m.refraction_index = _query_float(_text(me, "RefractionIndex"), 0.0)
        m.absorption_index = _query_float(_text(me, "AbsorptionIndex"), 0.0)
        m.absorption_coeff = tuple(_f3(_text(me, "AbsorptionCoefficient")))
        sc.materials.append(m)
    # ParseTextures (Parser.h:476-605): state carries over between TextureMaps
    te = root.find("Textures")
    if te is not None:
        ie = te.find("Images")
        if ie is not None:
            for im in ie.findall("Image"):
                sc.images.append(base + (im.text or "").strip())
        state = dict(is_image=False, image_id=0, normalizer=255, noise_scale=1.0, bump=1.0,
                     dm=A.DECAL_NONE, nc=A.NC_LINEAR, interp=A.INTERP_NN)
        cache = {}
        for tm in te.findall("TextureMap"):
            for k, v in tm.attrib.items():
                if k[:4] == "type":
                    state["is_image"] = v[:5] == "image"
                    break
            if tm.find("ImageId") is not None:
                state["image_id"] = _query_int(_text(tm, "ImageId"), state["image_id"])
            dmt = _text(tm, "DecalMode")
            if dmt is not None:
                for pre, val in (("blend_kd", A.DECAL_BLEND_KD), ("replace_kd", A.DECAL_REPLACE_KD),
                                 ("replace_all", A.DECAL_REPLACE_ALL), ("bump_normal", A.DECAL_BUMP_NORMAL),
                                 ("replace_normal", A.DECAL_REPLACE_NORMAL),
                                 ("replace_background", A.DECAL_REPLACE_BACKGROUND)):
                    if dmt[:len(pre)] == pre:
                        state["dm"] = val
                        break
            nct = _text(tm, "NoiseConversion")
            if nct is not None:
                state["nc"] = A.NC_ABSVAL if nct[:6] == "absval" else A.NC_LINEAR
            it = _text(tm, "Interpolation")
            if it is not None:
                if it[:7] == "nearest":
                    state["interp"] = A.INTERP_NN
                elif it[:8] == "bilinear":
                    state["interp"] = A.INTERP_BILINEAR
            if tm.find("Normalizer") is not None:
                state["normalizer"] = _query_int(_text(tm, "Normalizer"), state["normalizer"])
            if tm.find("NoiseScale") is not None:
                state["noise_scale"] = _query_float(_text(tm, "NoiseScale"), state["noise_scale"])
            if tm.find("BumpFactor") is not None:
                state["bump"] = _query_float(_text(tm, "BumpFactor"), state["bump"])
            tx = Texture(decal=state["dm"], interp=state["interp"], normalizer=state["normalizer"],
                         bump_factor=state["bump"], noise_conv=state["nc"], noise_scale=state["noise_scale"])
            if state["is_image"]:
                tx.kind = A.TEX_IMAGE
                tx.image_id = state["image_id"]
                path = sc.images[state["image_id"] - 1]
                if path not in cache:
                    cache[path] = load_image(path)
                tx.texels = cache[path]
            else:
                tx.kind = A.TEX_PERLIN
            sc.textures.append(tx)
    # ParseTransformations (Parser.h:607-682)
    tr = root.find("Transformations")
    if tr is not None:
        for t in tr.findall("Translation"):
            sc.translations.append(tuple(_f3(t.text)))
        for t in tr.findall("Scaling"):
            sc.scalings.append(tuple(_f3(t.text)))
        for t in tr.findall("Rotation"):
            v = [float(f32(float(x))) for x in t.text.split()[:4]]
            sc.rotations.append(tuple(v))
        for t in tr.findall("Composite"):
            v = [float(f32(float(x))) for x in t.text.split()[:16]]
            col_major = [0.0] * 16
            for k, val in enumerate(v):      # XML row-major -> composite[col][row]
                row, col = divmod(k, 4)
                col_major[col * 4 + row] = val
            sc.composites.append(tuple(col_major))
    # ParseVertices / ParseTextureCoordinates (Parser.h:684-767): atof -> double -> float
    vd = root.find("VertexData")
    verts = []
    if vd is not None and vd.text:
        vals = np.array([float(x) for x in vd.text.split()], dtype=np.float64)
        verts = list(vals[: len(vals) // 3 * 3].reshape(-1, 3).astype(f32))
    tcd = root.find("TexCoordData")
    tcs = []
    if tcd is not None and tcd.text:
        vals = np.array([float(x) for x in tcd.text.split()], dtype=np.float64)
        tcs = list(vals[: len(vals) // 2 * 2].reshape(-1, 2).astype(f32))
    extra_v, extra_t = [], []

    def nverts():
        return len(verts) + sum(a.shape[0] for a in extra_v)

    def ntcs():
        return len(tcs) + sum(a.shape[0] for a in extra_t)

    # ParseObjects (Parser.h:798-1195)
    oe = root.find("Objects")

    def common(el, o):
        o.id = int(el.get("id", "0"))
        o.material = _query_int(_text(el, "Material"), 1)
        x = _text(el, "Transformations")
        if x is not None:
            o.xforms = parse_object_transformations(x)
        tx = _text(el, "Textures")
        if tx is not None:
            o.textures = _parse_textures_list(tx)
        mb = _text(el, "MotionBlur")
        if mb is not None:
            o.blur = tuple(_f3(mb))

    # object lights (hw7): <LightSphere> after the spheres, <LightMesh> after the meshes
    def light(el, o):
        o.is_light = True
        o.radiance = tuple(_f3(_text(el, "Radiance")))

    for tag in ("Sphere", "LightSphere"):
        for el in oe.findall(tag):
            o = Object(type=A.OBJ_SPHERE)
            common(el, o)
            o.center = _query_int(_text(el, "Center"), 1)
            o.radius = _query_float(_text(el, "Radius"), 1.0)
            if tag == "LightSphere":
                light(el, o)
            sc.objects.append(o)
    for el in oe.findall("Triangle"):
        o = Object(type=A.OBJ_TRIANGLE)
        common(el, o)
        o.v = tuple(int(v) for v in _text(el, "Indices").split()[:3])
        sc.objects.append(o)
    mesh_start = len(sc.objects)
    for el in oe.findall("Mesh") + oe.findall("LightMesh"):
        o = Object(type=A.OBJ_MESH)
        common(el, o)
        if el.tag == "LightMesh":
            light(el, o)
        o.smooth = _attr_prefix(el, "shadingMode", "smooth")
        fe = el.find("Faces")
        ply = None
        for k, v in fe.attrib.items():
            if k[:7] == "plyFile":
                ply = v
                break
        if ply is not None:
            o.ply_file = ply
            pv, puv, pf = read_ply(base + ply)
            texture_offset = ntcs() + 1
            if puv is not None:
                extra_t.append(puv.astype(f32))
            vertex_count = nverts() + 1
            tri = []
            for f in pf:
                if len(f) == 4:
                    tri.append((f[0] + vertex_count, f[1] + vertex_count, f[2] + vertex_count))
                    tri.append((f[2] + vertex_count, f[3] + vertex_count, f[0] + vertex_count))
                else:
                    tri.append((f[0] + vertex_count, f[1] + vertex_count, f[2] + vertex_count))
            o.faces = np.array(tri, np.int32).reshape(-1, 3)
            extra_v.append(np.asarray(pv, np.float64).astype(f32))
            o.texture_offset = texture_offset - vertex_count
        else:
            vo = int(fe.get("vertexOffset", "0"))
            to = int(fe.get("textureOffset", "0"))
            o.xml_vertex_offset = vo
            idx = np.array([int(v) for v in (fe.text or "").split()], np.int64)
            idx = idx[: len(idx) // 3 * 3].reshape(-1, 3) + vo
            o.faces = idx.astype(np.int32)
            o.texture_offset = to - vo
        sc.objects.append(o)
    for el in oe.findall("MeshInstance"):
        it = Instance()
        it.id = int(el.get("id", "0"))
        base_id = int(el.get("baseMeshId", "0"))
        rt = el.get("resetTransform", "false").strip().lower()
        it.reset_transform = rt in ("true", "1")
        it.material = _query_int(_text(el, "Material"), 1)
        x = _text(el, "Transformations")
        if x is not None:
            it.xforms = parse_object_transformations(x)
        mb = _text(el, "MotionBlur")
        if mb is not None:
            it.blur = tuple(_f3(mb))
        found = -1
        for i in range(mesh_start, len(sc.objects)):
            if sc.objects[i].id == base_id:
                found = i
        if found < 0:
            raise ValueError(f"MeshInstance {it.id}: base mesh {base_id} not found")
        it.base_object = found
        sc.instances.append(it)
    parts_v = [np.asarray(verts, f32).reshape(-1, 3)] + extra_v
    sc.vertices = np.concatenate(parts_v).astype(f32) if parts_v else np.zeros((0, 3), f32)
    parts_t = [np.asarray(tcs, f32).reshape(-1, 2)] + extra_t
    sc.texcoords = np.concatenate(parts_t).astype(f32)
    # ParseLights (Parser.h:1197-1315): Point, Directional, Spot, Area, SphericalDirectional
    le = root.find("Lights")
    amb = _text(le, "AmbientLight")
    sc.ambient = tuple(_f3(amb)) if amb is not None else (0.0, 0.0, 0.0)
    for l in le.findall("PointLight"):
        sc.lights.append(Light(type=A.LIGHT_POINT, position=tuple(_f3(_text(l, "Position"))),
                               intensity=tuple(_f3(_text(l, "Intensity")))))
    for l in le.findall("DirectionalLight"):
        sc.lights.append(Light(type=A.LIGHT_DIRECTIONAL, direction=tuple(_f3(_text(l, "Direction"))),
                               intensity=tuple(_f3(_text(l, "Radiance")))))
    for l in le.findall("SpotLight"):
        sc.lights.append(Light(type=A.LIGHT_SPOT, position=tuple(_f3(_text(l, "Position"))),
                               direction=tuple(_f3(_text(l, "Direction"))),
                               intensity=tuple(_f3(_text(l, "Intensity"))),
                               coverage_deg=_query_float(_text(l, "CoverageAngle"), 0.0),
                               falloff_deg=_query_float(_text(l, "FalloffAngle"), 0.0)))
    for l in le.findall("AreaLight"):
        rad = _text(l, "Radiance")
        if rad is None:
            rad = _text(l, "Intensity")
        sc.lights.append(Light(type=A.LIGHT_AREA, position=tuple(_f3(_text(l, "Position"))),
                               direction=tuple(_f3(_text(l, "Normal"))), intensity=tuple(_f3(rad)),
                               size=_query_float(_text(l, "Size"), 0.0)))
    sc.environment_light = -1
    for l in le.findall("SphericalDirectionalLight"):
        sc.environment_light = len(sc.lights)
        iid = _query_int(_text(l, "ImageId"), 1)
        tex = Texture(kind=A.TEX_IMAGE, decal=A.DECAL_NONE, interp=A.INTERP_BILINEAR, normalizer=1,
                      bump_factor=1.0, texels=load_image(sc.images[iid - 1]), image_id=iid)
        sc.textures.append(tex)
        sc.lights.append(Light(type=A.LIGHT_ENVIRONMENT, texture=len(sc.textures) - 1, image_id=iid))
    # Scene ctor: last replace_background texture (src/Scene.cpp:494-500)
    sc.background_texture = -1
    for i, tx in enumerate(sc.textures):
        if tx.decal == A.DECAL_REPLACE_BACKGROUND:
            sc.background_texture = i
    return sc


# ============================================================================ XML writer
_XF_CH = {A.XF_TRANSLATION: "t", A.XF_SCALING: "s", A.XF_ROTATION: "r", A.XF_COMPOSITE: "c"}


def write_xml(sc: Scene, xml_path: str, images: dict | None = None) -> str:
    """Serialise `sc` in the reference's scene format.  Meshes with `ply_file` set are
    written as binary PLY next to the XML (vertices referenced by a mesh's faces must then
    be exclusive to it and contiguous).  Image textures must have `image_id` pointing into
    `sc.images` (paths relative to the XML directory)."""
    d = os.path.dirname(os.path.abspath(xml_path))
    out = ["<Scene>"]
    out.append(f"<MaxRecursionDepth>{sc.max_depth}</MaxRecursionDepth>")
    out.append(f"<BackgroundColor>{_fmts(sc.background)}</BackgroundColor>")
    out.append(f"<ShadowRayEpsilon>{_fmt(sc.shadow_eps)}</ShadowRayEpsilon>")
    out.append(f"<IntersectionTestEpsilon>{_fmt(sc.int_eps)}</IntersectionTestEpsilon>")
    out.append("<Cameras>")
    for c in sc.cameras:
        hand = ' handedness="left"' if c.left_handed else ""
        out.append(f'<Camera id="{c.id}"{hand}>')
        out.append(f"<Position>{_fmts(c.position)}</Position>")
        out.append(f"<Gaze>{_fmts(c.gaze)}</Gaze>")
        out.append(f"<Up>{_fmts(c.up)}</Up>")
        out.append(f"<NearPlane>{_fmts(c.near_plane)}</NearPlane>")
        out.append(f"<NearDistance>{_fmt(c.near_distance)}</NearDistance>")
        out.append(f"<ImageResolution>{c.nx} {c.ny}</ImageResolution>")
        out.append(f"<NumSamples>{c.num_samples}</NumSamples>")
        if c.is_dof:
            out.append(f"<FocusDistance>{_fmt(c.focus_distance)}</FocusDistance>")
            out.append(f"<ApertureSize>{_fmt(c.aperture_size)}</ApertureSize>")
        out.append(f"<ImageName>{c.image_name}</ImageName>")
        if c.tonemap is not None:
            k, b, sat, g = c.tonemap
            out.append(f"<Tonemap><TMO>Photographic</TMO><TMOOptions>{_fmt(k)} {_fmt(b)}</TMOOptions>"
                       f"<Saturation>{_fmt(sat)}</Saturation><Gamma>{_fmt(g)}</Gamma></Tonemap>")
        if c.integrator == A.INTEGRATOR_PATH:
            out.append("<Renderer>PathTracing</Renderer>")
            toks = [n for f, n in ((A.PT_IMPORTANCE, "ImportanceSampling"), (A.PT_NEE, "NextEventEstimation"),
                                   (A.PT_RUSSIAN_ROULETTE, "RussianRoulette")) if c.pt_flags & f]
            if toks:
                out.append(f"<RendererParams>{' '.join(toks)}</RendererParams>")
        out.append("</Camera>")
    out.append("</Cameras>")
    # BRDFs referenced by materials
    brdf_tags = {A.BRDF_MBP: ("ModifiedBlinnPhong", ""), A.BRDF_MBPN: ("ModifiedBlinnPhong", ' normalized="true"'),
                 A.BRDF_OBP: ("OriginalBlinnPhong", ""), A.BRDF_MP: ("ModifiedPhong", ""),
                 A.BRDF_MPN: ("ModifiedPhong", ' normalized="true"'), A.BRDF_OP: ("OriginalPhong", ""),
                 A.BRDF_TS: ("TorranceSparrow", ""), A.BRDF_TSF: ("TorranceSparrow", ' kdfresnel="true"')}
    brdf_ids = []
    for i, m in enumerate(sc.materials):
        if m.brdf != A.BRDF_NONE:
            brdf_ids.append((i + 1, m))
    if brdf_ids:
        out.append("<BRDFs>")
        for bid, m in brdf_ids:
            tag, attr = brdf_tags[m.brdf]
            out.append(f'<{tag} id="{bid}"{attr}><Exponent>{m.phong_exp}</Exponent></{tag}>')
        out.append("</BRDFs>")
    out.append("<Materials>")
    tnames = {A.MAT_MIRROR: "mirror", A.MAT_CONDUCTOR: "conductor", A.MAT_DIELECTRIC: "dielectric"}
    for i, m in enumerate(sc.materials):
        attrs = f' id="{i + 1}"'
        if m.type in tnames:
            attrs += f' type="{tnames[m.type]}"'
        if m.brdf != A.BRDF_NONE:
            attrs += f' BRDF="{i + 1}"'
        out.append(f"<Material{attrs}>")
        out.append(f"<AmbientReflectance>{_fmts(m.ambient)}</AmbientReflectance>")
        out.append(f"<DiffuseReflectance>{_fmts(m.diffuse)}</DiffuseReflectance>")
        out.append(f"<SpecularReflectance>{_fmts(m.specular)}</SpecularReflectance>")
        out.append(f"<MirrorReflectance>{_fmts(m.mirror)}</MirrorReflectance>")
        if m.brdf == A.BRDF_NONE:
            out.append(f"<PhongExponent>{m.phong_exp}</PhongExponent>")
        if m.is_rough:
            out.append(f"<Roughness>{_fmt(m.roughness)}</Roughness>")
        out.append(f"<RefractionIndex>{_fmt(m.refraction_index)}</RefractionIndex>")
        out.append(f"<AbsorptionIndex>{_fmt(m.absorption_index)}</AbsorptionIndex>")
        out.append(f"<AbsorptionCoefficient>{_fmts(m.absorption_coeff)}</AbsorptionCoefficient>")
        out.append("</Material>")
    out.append("</Materials>")
    maps = [t for t in sc.textures if not (t.decal == A.DECAL_NONE and t.kind == A.TEX_IMAGE and t.normalizer == 1)]
    if sc.images or maps:
        out.append("<Textures>")
        if sc.images:
            out.append("<Images>")
            for i, p in enumerate(sc.images):
                rel = os.path.relpath(p, d) if os.path.isabs(p) else p
                out.append(f'<Image id="{i + 1}">{rel}</Image>')
            out.append("</Images>")
        dnames = {A.DECAL_REPLACE_KD: "replace_kd", A.DECAL_BLEND_KD: "blend_kd", A.DECAL_BUMP_NORMAL: "bump_normal",
                  A.DECAL_REPLACE_NORMAL: "replace_normal", A.DECAL_REPLACE_ALL: "replace_all",
                  A.DECAL_REPLACE_BACKGROUND: "replace_background"}
        for t in maps:
            ty = "image" if t.kind == A.TEX_IMAGE else "perlin"
            out.append(f'<TextureMap type="{ty}">')
            # every field is written: Parser.h carries unset fields over from the previous map
            if t.kind == A.TEX_IMAGE:
                out.append(f"<ImageId>{t.image_id}</ImageId>")
            out.append(f"<Interpolation>{'bilinear' if t.interp == A.INTERP_BILINEAR else 'nearest'}</Interpolation>")
            out.append(f"<NoiseConversion>{'absval' if t.noise_conv == A.NC_ABSVAL else 'linear'}</NoiseConversion>")
            out.append(f"<NoiseScale>{_fmt(t.noise_scale)}</NoiseScale>")
            if t.decal in dnames:
                out.append(f"<DecalMode>{dnames[t.decal]}</DecalMode>")
            out.append(f"<Normalizer>{t.normalizer}</Normalizer>")
            out.append(f"<BumpFactor>{_fmt(t.bump_factor)}</BumpFactor>")
            out.append("</TextureMap>")
        out.append("</Textures>")
    if sc.translations or sc.scalings or sc.rotations or sc.composites:
        out.append("<Transformations>")
        for i, t in enumerate(sc.translations):
            out.append(f'<Translation id="{i + 1}">{_fmts(t)}</Translation>')
        for i, t in enumerate(sc.scalings):
            out.append(f'<Scaling id="{i + 1}">{_fmts(t)}</Scaling>')
        for i, t in enumerate(sc.rotations):
            out.append(f'<Rotation id="{i + 1}">{_fmts(t)}</Rotation>')
        for i, t in enumerate(sc.composites):
            rowmajor = [t[(k % 4) * 4 + k // 4] for k in range(16)]
            out.append(f'<Composite id="{i + 1}">{_fmts(rowmajor)}</Composite>')
        out.append("</Transformations>")
    # vertices referenced by PLY meshes are written into the PLY files instead
    verts = np.asarray(sc.vertices, f32).reshape(-1, 3)
    ply_ranges = []
    for o in sc.objects:
        if o.type == A.OBJ_MESH and o.ply_file:
            f = np.asarray(o.faces)
            ply_ranges.append((int(f.min()), int(f.max())))
    n_xml = len(verts)
    if ply_ranges:
        n_xml = ply_ranges[0][0] - 1
        nxt = ply_ranges[0][0]
        for lo, hi in ply_ranges:
            if lo != nxt:
                raise ValueError("PLY-backed vertices must be the trailing vertices, in mesh order")
            nxt = hi + 1
        if nxt != len(verts) + 1:
            raise ValueError("PLY-backed vertices must be the trailing vertices, in mesh order")
    xml_verts = verts[:n_xml]
    out.append("<VertexData>")
    out.extend(_fmts(v) for v in xml_verts)
    out.append("</VertexData>")
    if len(sc.texcoords):
        out.append("<TexCoordData>")
        out.extend(_fmts(v) for v in np.asarray(sc.texcoords, f32).reshape(-1, 2))
        out.append("</TexCoordData>")
    out.append("<Objects>")

    def common(o, tag):
        lines = [f"<Material>{o.material}</Material>"]
        if o.xforms:
            lines.append("<Transformations>" + " ".join(f"{_XF_CH[t]}{i}" for t, i in o.xforms) + "</Transformations>")
        if o.textures:
            lines.append("<Textures>" + " ".join(str(t) for t in o.textures) + "</Textures>")
        if any(float(b) != 0.0 for b in o.blur):
            lines.append(f"<MotionBlur>{_fmts(o.blur)}</MotionBlur>")
        return lines

    def radiance(o):
        return [f"<Radiance>{_fmts(o.radiance)}</Radiance>"] if o.is_light else []

    for lt in (False, True):
        for o in sc.objects:
            if o.type == A.OBJ_SPHERE and bool(o.is_light) == lt:
                tag = "LightSphere" if lt else "Sphere"
                out.append(f'<{tag} id="{o.id}">')
                out.extend(common(o, tag))
                out.append(f"<Center>{o.center}</Center><Radius>{_fmt(o.radius)}</Radius>")
                out.extend(radiance(o))
                out.append(f"</{tag}>")
    for o in sc.objects:
        if o.type == A.OBJ_TRIANGLE:
            out.append(f'<Triangle id="{o.id}">')
            out.extend(common(o, "Triangle"))
            out.append(f"<Indices>{o.v[0]} {o.v[1]} {o.v[2]}</Indices>")
            out.append("</Triangle>")
    meshes = [o for o in sc.objects if o.type == A.OBJ_MESH]
    for o in [o for o in meshes if not o.is_light] + [o for o in meshes if o.is_light]:
        sm = ' shadingMode="smooth"' if o.smooth else ""
        tag = "LightMesh" if o.is_light else "Mesh"
        out.append(f'<{tag} id="{o.id}"{sm}>')
        out.extend(common(o, tag))
        out.extend(radiance(o))
        f = np.asarray(o.faces, np.int64).reshape(-1, 3)
        if o.ply_file:
            lo, hi = int(f.min()), int(f.max())
            write_ply_binary(os.path.join(d, o.ply_file), verts[lo - 1:hi], f - lo)
            out.append(f'<Faces plyFile="{o.ply_file}"/>')
        else:
            to = o.texture_offset
            out.append(f'<Faces textureOffset="{to}">')
            out.extend(f"{a} {b} {c}" for a, b, c in f)
            out.append("</Faces>")
        out.append(f"</{tag}>")
    for it in sc.instances:
        base = sc.objects[it.base_object]
        rt = ' resetTransform="true"' if it.reset_transform else ""
        out.append(f'<MeshInstance id="{it.id}" baseMeshId="{base.id}"{rt}>')
        out.append(f"<Material>{it.material}</Material>")
        if it.xforms:
            out.append("<Transformations>" + " ".join(f"{_XF_CH[t]}{i}" for t, i in it.xforms) + "</Transformations>")
        if any(float(b) != 0.0 for b in it.blur):
            out.append(f"<MotionBlur>{_fmts(it.blur)}</MotionBlur>")
        out.append("</MeshInstance>")
    out.append("</Objects>")
    out.append("<Lights>")
    out.append(f"<AmbientLight>{_fmts(sc.ambient)}</AmbientLight>")
    order = [A.LIGHT_POINT, A.LIGHT_DIRECTIONAL, A.LIGHT_SPOT, A.LIGHT_AREA, A.LIGHT_ENVIRONMENT]
    if [l.type for l in sc.lights] != sorted((l.type for l in sc.lights), key=order.index):
        raise ValueError("lights must be in the reference's parse order (point, directional, spot, area, env)")
    for i, l in enumerate(sc.lights):
        if l.type == A.LIGHT_POINT:
            out.append(f'<PointLight id="{i + 1}"><Position>{_fmts(l.position)}</Position>'
                       f"<Intensity>{_fmts(l.intensity)}</Intensity></PointLight>")
        elif l.type == A.LIGHT_DIRECTIONAL:
            out.append(f'<DirectionalLight id="{i + 1}"><Direction>{_fmts(l.direction)}</Direction>'
                       f"<Radiance>{_fmts(l.intensity)}</Radiance></DirectionalLight>")
        elif l.type == A.LIGHT_SPOT:
            out.append(f'<SpotLight id="{i + 1}"><Position>{_fmts(l.position)}</Position>'
                       f"<Direction>{_fmts(l.direction)}</Direction><Intensity>{_fmts(l.intensity)}</Intensity>"
                       f"<CoverageAngle>{_fmt(l.coverage_deg)}</CoverageAngle>"
                       f"<FalloffAngle>{_fmt(l.falloff_deg)}</FalloffAngle></SpotLight>")
        elif l.type == A.LIGHT_AREA:
            out.append(f'<AreaLight id="{i + 1}"><Position>{_fmts(l.position)}</Position>'
                       f"<Normal>{_fmts(l.direction)}</Normal><Radiance>{_fmts(l.intensity)}</Radiance>"
                       f"<Size>{_fmt(l.size)}</Size></AreaLight>")
        else:
            out.append(f'<SphericalDirectionalLight id="{i + 1}"><ImageId>{l.image_id}</ImageId>'
                       "</SphericalDirectionalLight>")
    out.append("</Lights>")
    out.append("</Scene>")
    with open(xml_path, "w") as fh:
        fh.write("\n".join(out) + "\n")
    return xml_path
