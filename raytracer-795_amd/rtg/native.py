"""ctypes binding of the native host library (librtghost.so, include/rtg_host.h): the C++
Parser / Image / renderScene loop, and a reader that turns any rtg_scene_desc into plain
Python data (used to check the native parser against rtg/scene.py field by field)."""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import _abi as A

LIB_PATH = os.path.join(A.PKG_DIR, "librtghost.so")
CLI_PATH = os.path.join(A.PKG_DIR, "rtg_cli")
_lib = None


def load():
    global _lib
    if _lib is None:
        A.load_library()                      # librtg first (one HIP runtime, see _abi)
        if not os.path.exists(LIB_PATH):
            raise A.RtgError(f"{LIB_PATH} missing: run __graft_entry__.build()")
        lib = C.CDLL(LIB_PATH)
        lib.rtgh_last_error.restype = C.c_char_p
        lib.rtgh_parse_xml.argtypes = [C.c_char_p, C.POINTER(C.c_void_p)]
        lib.rtgh_parse_xml.restype = C.c_int32
        lib.rtgh_scene_desc.argtypes = [C.c_void_p]
        lib.rtgh_scene_desc.restype = C.POINTER(A.SceneDesc)
        lib.rtgh_num_cameras.argtypes = [C.c_void_p]
        lib.rtgh_num_cameras.restype = C.c_int32
        lib.rtgh_camera.argtypes = [C.c_void_p, C.c_int32, C.POINTER(A.CameraDesc), C.c_char_p, C.c_int32]
        lib.rtgh_camera.restype = C.c_int32
        lib.rtgh_camera_tonemap.argtypes = [C.c_void_p, C.c_int32, C.POINTER(A.TonemapDesc)]
        lib.rtgh_camera_tonemap.restype = C.c_int32
        lib.rtgh_free.argtypes = [C.c_void_p]
        lib.rtgh_free.restype = None
        lib.rtgh_save_image.argtypes = [C.c_char_p, A.PF, C.c_int32, C.c_int32]
        lib.rtgh_save_image.restype = C.c_int32
        lib.rtgh_render_scene.argtypes = [C.c_char_p, C.c_int32, C.c_uint64, C.c_char_p]
        lib.rtgh_render_scene.restype = C.c_int32
        lib.rtgh_render_scene_multi.argtypes = [C.c_char_p, C.c_int32, C.c_int32, C.c_uint64, C.c_char_p]
        lib.rtgh_render_scene_multi.restype = C.c_int32
        lib.rtgh_read_image.argtypes = [C.c_char_p, C.POINTER(A.PF), C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
        lib.rtgh_read_image.restype = C.c_int32
        lib.rtgh_free_image.argtypes = [A.PF]
        lib.rtgh_free_image.restype = None
        _lib = lib
    return _lib


def _check(rc):
    if rc != 0:
        raise A.RtgError(f"{A.STATUS.get(rc, rc)}: {_lib.rtgh_last_error().decode()}")


def read_image(path: str) -> np.ndarray:
    """rtgh_read_image: the texels a texture sees, (h, w, 3) float32 (raw 0..255 for
    PNG/JPEG/PPM, linear floats for OpenEXR)."""
    lib = load()
    p = A.PF()
    w, h = C.c_int32(), C.c_int32()
    _check(lib.rtgh_read_image(path.encode(), C.byref(p), C.byref(w), C.byref(h)))
    try:
        return np.ctypeslib.as_array(p, shape=(h.value, w.value, 3)).copy()
    finally:
        lib.rtgh_free_image(p)


class NativeScene:
    """rtgh_parse_xml result: .desc (rtg_scene_desc) and .cameras [(CameraDesc, image_name)]."""

    def __init__(self, xml_path: str):
        self.lib = load()
        h = C.c_void_p()
        _check(self.lib.rtgh_parse_xml(xml_path.encode(), C.byref(h)))
        self.handle = h
        self.desc = self.lib.rtgh_scene_desc(h).contents
        self.cameras = []
        for i in range(self.lib.rtgh_num_cameras(h)):
            cd = A.CameraDesc()
            name = C.create_string_buffer(4096)
            _check(self.lib.rtgh_camera(h, i, C.byref(cd), name, 4096))
            self.cameras.append((cd, name.value.decode()))
        self.tonemaps = []
        for i in range(len(self.cameras)):
            tm = A.TonemapDesc()
            has = self.lib.rtgh_camera_tonemap(h, i, C.byref(tm))
            self.tonemaps.append((tm.key, tm.burn_percent, tm.saturation, tm.gamma) if has == 1 else None)

    def close(self):
        if getattr(self, "handle", None):
            self.lib.rtgh_free(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def save_image(name: str, rgb: np.ndarray):
    lib = load()
    a = np.ascontiguousarray(rgb, np.float32)
    _check(lib.rtgh_save_image(name.encode(), a.ctypes.data_as(A.PF), a.shape[1], a.shape[0]))


def render_scene(xml_path: str, device: int = 0, seed: int = 0x5EED2026, out_dir: str | None = None,
                 num_devices: int = 1):
    lib = load()
    _check(lib.rtgh_render_scene_multi(xml_path.encode(), device, num_devices, seed,
                                       out_dir.encode() if out_dir else None))


def _struct(s) -> dict:
    out = {}
    for name, typ in s._fields_:
        v = getattr(s, name)
        if isinstance(v, C.Array):
            v = list(v)
        elif isinstance(v, (C._Pointer, bytes, str)):
            continue
        out[name] = v
    return out


def desc_to_dict(d: A.SceneDesc) -> dict:
    """Every value an rtg_scene_desc carries, pointers dereferenced (for equality checks)."""
    def arr(ptr, n, width, dtype=np.float32):
        if n == 0:
            return np.zeros((0, width), dtype)
        return np.ctypeslib.as_array(ptr, shape=(n * width,)).reshape(n, width).astype(dtype).copy()

    out = {k: getattr(d, k) for k in ("abi_version", "max_recursion_depth", "shadow_ray_eps", "intersection_test_eps",
                                      "background_texture", "environment_light")}
    out["background"] = list(d.background)
    out["ambient_light"] = list(d.ambient_light)
    out["vertices"] = arr(d.vertices, d.num_vertices, 3)
    out["texcoords"] = arr(d.texcoords, d.num_texcoords, 2)
    out["faces"] = arr(d.faces, d.num_faces, 3, np.int32)
    out["translations"] = arr(d.translations, d.num_translations, 3)
    out["scalings"] = arr(d.scalings, d.num_scalings, 3)
    out["rotations"] = arr(d.rotations, d.num_rotations, 4)
    out["composites"] = arr(d.composites, d.num_composites, 16)
    out["xform_refs"] = [(d.xform_refs[i].type, d.xform_refs[i].index) for i in range(d.num_xform_refs)]
    out["objects"] = [_struct(d.objects[i]) for i in range(d.num_objects)]
    out["instances"] = [_struct(d.instances[i]) for i in range(d.num_instances)]
    out["materials"] = [_struct(d.materials[i]) for i in range(d.num_materials)]
    texs = []
    for i in range(d.num_textures):
        t = d.textures[i]
        e = _struct(t)
        e["texels"] = (np.ctypeslib.as_array(t.texels, shape=(t.width * t.height * 3,)).copy()
                       if bool(t.texels) and t.width * t.height > 0 else None)
        texs.append(e)
    out["textures"] = texs
    out["lights"] = [_struct(d.lights[i]) for i in range(d.num_lights)]
    return out
