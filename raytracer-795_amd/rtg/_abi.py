"""ctypes mirror of include/rtg.h and the loader for the in-tree librtg.so.

The product path is the HIP library; there is no CPU fallback.  `load_library()`
raises if librtg.so is missing or was built for a different ABI version.
"""
from __future__ import annotations

import ctypes as C
import os

RTG_ABI_VERSION = 9

RTG_OK = 0
RTG_DEVICE_HOST_ONLY = -1
STATUS = {0: "RTG_OK", -1: "RTG_ERR_INVALID", -2: "RTG_ERR_NO_DEVICE", -3: "RTG_ERR_OOM",
          -4: "RTG_ERR_HIP", -5: "RTG_ERR_UNSUPPORTED"}

# enums (src/defs.h:8-11, src/Material.h:7-8, src/Light.h:12)
OBJ_SPHERE, OBJ_TRIANGLE, OBJ_MESH = 0, 1, 2
XF_TRANSLATION, XF_SCALING, XF_ROTATION, XF_COMPOSITE = 1, 2, 3, 4
MAT_NORMAL, MAT_MIRROR, MAT_CONDUCTOR, MAT_DIELECTRIC = 0, 1, 2, 3
(BRDF_NONE, BRDF_OBP, BRDF_MBP, BRDF_MBPN, BRDF_OP, BRDF_MP, BRDF_MPN, BRDF_TS, BRDF_TSF) = range(9)
(DECAL_REPLACE_KD, DECAL_BLEND_KD, DECAL_BUMP_NORMAL, DECAL_REPLACE_NORMAL, DECAL_REPLACE_ALL,
 DECAL_REPLACE_BACKGROUND, DECAL_NONE) = range(7)
INTERP_NN, INTERP_BILINEAR = 0, 1
TEX_IMAGE, TEX_PERLIN = 0, 1
NC_ABSVAL, NC_LINEAR, NC_NONE = 0, 1, 2
LIGHT_POINT, LIGHT_AREA, LIGHT_DIRECTIONAL, LIGHT_SPOT, LIGHT_ENVIRONMENT = 0, 1, 2, 3, 4
INTEGRATOR_REFERENCE, INTEGRATOR_PATH = 0, 1
PT_IMPORTANCE, PT_NEE, PT_RUSSIAN_ROULETTE = 1, 2, 4
PT_MAX_BOUNCES = 32

F3 = C.c_float * 3
I2 = C.c_int32 * 2
I3 = C.c_int32 * 3
PF = C.POINTER(C.c_float)
PI = C.POINTER(C.c_int32)


class XformRef(C.Structure):
    _fields_ = [("type", C.c_int32), ("index", C.c_int32)]


class ObjectDesc(C.Structure):
    _fields_ = [("type", C.c_int32), ("id", C.c_int32), ("material", C.c_int32), ("num_textures", C.c_int32),
                ("textures", I2), ("texture_offset", C.c_int32), ("smooth", C.c_int32),
                ("xform_first", C.c_int32), ("xform_count", C.c_int32), ("blur", F3),
                ("center", C.c_int32), ("radius", C.c_float), ("v", I3),
                ("face_first", C.c_int32), ("face_count", C.c_int32),
                ("is_light", C.c_int32), ("radiance", F3)]


class InstanceDesc(C.Structure):
    _fields_ = [("base_object", C.c_int32), ("id", C.c_int32), ("material", C.c_int32),
                ("reset_transform", C.c_int32), ("xform_first", C.c_int32), ("xform_count", C.c_int32),
                ("blur", F3)]


class MaterialDesc(C.Structure):
    _fields_ = [("type", C.c_int32), ("brdf", C.c_int32), ("phong_exp", C.c_int32), ("is_rough", C.c_int32),
                ("roughness", C.c_float), ("ambient", F3), ("diffuse", F3), ("specular", F3), ("mirror", F3),
                ("refraction_index", C.c_float), ("absorption_index", C.c_float), ("absorption_coeff", F3)]


class TextureDesc(C.Structure):
    _fields_ = [("kind", C.c_int32), ("decal", C.c_int32), ("interp", C.c_int32), ("noise_conv", C.c_int32),
                ("normalizer", C.c_int32), ("noise_scale", C.c_float), ("bump_factor", C.c_float),
                ("width", C.c_int32), ("height", C.c_int32), ("texels", PF)]


class LightDesc(C.Structure):
    _fields_ = [("type", C.c_int32), ("position", F3), ("direction", F3), ("intensity", F3),
                ("coverage_deg", C.c_float), ("falloff_deg", C.c_float), ("size", C.c_float),
                ("texture", C.c_int32)]


class SceneDesc(C.Structure):
    _fields_ = [("abi_version", C.c_int32), ("max_recursion_depth", C.c_int32),
                ("shadow_ray_eps", C.c_float), ("intersection_test_eps", C.c_float),
                ("background", F3), ("ambient_light", F3),
                ("background_texture", C.c_int32), ("environment_light", C.c_int32),
                ("vertices", PF), ("num_vertices", C.c_int32),
                ("texcoords", PF), ("num_texcoords", C.c_int32),
                ("faces", PI), ("num_faces", C.c_int32),
                ("translations", PF), ("num_translations", C.c_int32),
                ("scalings", PF), ("num_scalings", C.c_int32),
                ("rotations", PF), ("num_rotations", C.c_int32),
                ("composites", PF), ("num_composites", C.c_int32),
                ("xform_refs", C.POINTER(XformRef)), ("num_xform_refs", C.c_int32),
                ("objects", C.POINTER(ObjectDesc)), ("num_objects", C.c_int32),
                ("instances", C.POINTER(InstanceDesc)), ("num_instances", C.c_int32),
                ("materials", C.POINTER(MaterialDesc)), ("num_materials", C.c_int32),
                ("textures", C.POINTER(TextureDesc)), ("num_textures", C.c_int32),
                ("lights", C.POINTER(LightDesc)), ("num_lights", C.c_int32)]


class CameraDesc(C.Structure):
    _fields_ = [("position", F3), ("gaze", F3), ("up", F3),
                ("left", C.c_float), ("right", C.c_float), ("bottom", C.c_float), ("top", C.c_float),
                ("near_distance", C.c_float), ("nx", C.c_int32), ("ny", C.c_int32),
                ("num_samples", C.c_int32), ("is_dof", C.c_int32), ("focus_distance", C.c_float),
                ("aperture_size", C.c_float), ("left_handed", C.c_int32),
                ("integrator", C.c_int32), ("pt_flags", C.c_int32)]


class RenderOpts(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("row_offset", C.c_int32), ("row_stride", C.c_int32),
                ("traversal", C.c_int32), ("max_batch_rays", C.c_int32), ("collect_stats", C.c_int32),
                ("collect_timing", C.c_int32), ("streams", C.c_int32), ("row_block", C.c_int32),
                ("compact_rows", C.c_int32), ("num_devices", C.c_int32), ("devices", C.POINTER(C.c_int32)),
                ("schedule", C.c_int32), ("tile_band", C.c_int32), ("segment_pixels", C.c_int32),
                ("segment_nodes", C.c_int32), ("pad_abi8", C.c_int32)]


SCHEDULE_AUTO, SCHEDULE_PASSES, SCHEDULE_STREAM = 0, 1, 2


class RenderStats(C.Structure):
    _fields_ = [("primary_rays", C.c_uint64), ("secondary_rays", C.c_uint64), ("shadow_rays", C.c_uint64),
                ("total_rays", C.c_uint64), ("render_ms", C.c_double), ("passes", C.c_int32),
                ("max_level", C.c_int32), ("node_visits", C.c_uint64), ("tri_tests", C.c_uint64),
                ("shadow_node_visits", C.c_uint64), ("shadow_tri_tests", C.c_uint64), ("trace_ms", C.c_double),
                ("shadow_ms", C.c_double), ("trace_launches", C.c_int32), ("shadow_launches", C.c_int32),
                ("trace_steps", C.c_uint64), ("shadow_steps", C.c_uint64),
                ("trace_lane_slots", C.c_uint64), ("shadow_lane_slots", C.c_uint64),
                ("shade_ms", C.c_double), ("shade_launches", C.c_int32), ("devices", C.c_int32),
                ("gather_ms", C.c_double), ("shadow_blocked", C.c_uint64), ("shadow_blocked_steps", C.c_uint64),
                ("shadow_blocked_tris", C.c_uint64), ("resolve_ms", C.c_double), ("accumulate_ms", C.c_double),
                ("resolve_launches", C.c_int32), ("accumulate_launches", C.c_int32),
                ("trace_entry_visits", C.c_uint64), ("trace_entry_slots", C.c_uint64),
                ("shadow_entry_visits", C.c_uint64), ("shadow_entry_slots", C.c_uint64),
                ("shadow_hist_before", C.c_uint64 * 8), ("shadow_hist_after", C.c_uint64 * 8),
                ("shadow_blocked_steps_before", C.c_uint64),
                ("shadow_blocked_steps_before_wavemin", C.c_uint64),
                ("trace_entry_cycles", C.c_uint64 * 16), ("shadow_entry_cycles", C.c_uint64 * 16),
                ("pt_shade_cycles", C.c_uint64 * 4),
                # ABI 9: the flat group's lane work / slots and set-up / test cycles
                ("trace_group_work", C.c_uint64), ("trace_group_slots", C.c_uint64),
                ("shadow_group_work", C.c_uint64), ("shadow_group_slots", C.c_uint64),
                ("trace_group_cycles", C.c_uint64 * 2), ("shadow_group_cycles", C.c_uint64 * 2)]

RTG_COMM_ID_BYTES = 128


class Ray(C.Structure):
    _fields_ = [("origin", F3), ("direction", F3), ("time", C.c_float)]


class BuildOpts(C.Structure):
    _fields_ = [("bvh_builder", C.c_int32), ("tlas", C.c_int32), ("traversal_tree", C.c_int32),
                ("uniform_walk", C.c_int32)]


class BuildStats(C.Structure):
    _fields_ = [("bvh_build_ms", C.c_double), ("bvh_gpu_objects", C.c_int32), ("num_objects", C.c_int32),
                ("tlas_nodes", C.c_int32), ("flat_group_entries", C.c_int32),
                ("validate_ms", C.c_double), ("prep_ms", C.c_double), ("median_tree_ms", C.c_double),
                ("records_ms", C.c_double), ("traversal_tree_ms", C.c_double), ("top_level_ms", C.c_double),
                ("upload_ms", C.c_double), ("total_ms", C.c_double), ("upload_bytes", C.c_uint64),
                ("sah_gpu_objects", C.c_int32), ("pad_abi8", C.c_int32), ("traversal_nodes", C.c_uint64),
                ("traversal_hash", C.c_uint64)]


RTG_BVH_AUTO, RTG_BVH_HOST, RTG_BVH_GPU = 0, 1, 2


class TonemapDesc(C.Structure):
    _fields_ = [("tmo", C.c_int32), ("key", C.c_float), ("burn_percent", C.c_float), ("saturation", C.c_float),
                ("gamma", C.c_float)]


TMO_PHOTOGRAPHIC = 0


class Hit(C.Structure):
    _fields_ = [("full", C.c_int32), ("object", C.c_int32), ("prim", C.c_int32), ("material", C.c_int32),
                ("t", C.c_float), ("point", F3), ("normal", F3)]


# Every entry point declared in include/rtg.h (checked by tests/test_abi.py).
EXPORTS = {
    "rtg_abi_version": (C.c_int32, []),
    "rtg_last_error": (C.c_char_p, []),
    "rtg_device_count": (C.c_int32, []),
    "rtg_scene_create": (C.c_int32, [C.POINTER(SceneDesc), C.c_int32, C.POINTER(C.c_void_p)]),
    "rtg_scene_create_ex": (C.c_int32, [C.POINTER(SceneDesc), C.c_int32, C.POINTER(BuildOpts),
                                         C.POINTER(C.c_void_p)]),
    "rtg_scene_build_stats": (C.c_int32, [C.c_void_p, C.POINTER(BuildStats)]),
    "rtg_scene_destroy": (C.c_int32, [C.c_void_p]),
    "rtg_render": (C.c_int32, [C.c_void_p, C.POINTER(CameraDesc), C.POINTER(RenderOpts), PF]),
    "rtg_render_device": (C.c_int32, [C.c_void_p, C.POINTER(CameraDesc), C.POINTER(RenderOpts), C.c_void_p,
                                      C.c_void_p]),
    "rtg_last_render_stats": (C.c_int32, [C.c_void_p, C.POINTER(RenderStats)]),
    "rtg_shard_rows": (C.c_int32, [C.c_int32, C.c_int32, C.c_int32, C.c_int32]),
    "rtg_pass_rays": (C.c_int64, [C.c_int32, C.c_int32, C.c_int32, C.c_uint64]),
    "rtg_tonemap": (C.c_int32, [C.c_int32, PF, C.c_int32, C.c_int32, C.POINTER(TonemapDesc), PF]),
    "rtg_tonemap_device": (C.c_int32, [C.c_int32, C.c_void_p, C.c_int32, C.c_int32, C.POINTER(TonemapDesc), C.c_void_p,
                                       C.c_void_p]),
    "rtg_trace_closest": (C.c_int32, [C.c_void_p, C.POINTER(Ray), C.c_int32, C.POINTER(Hit), C.c_int32]),
    "rtg_scene_object_bvh": (C.c_int32, [C.c_void_p, C.c_int32, PI, PI, PI, PI, PF]),
    "rtg_scene_object_matrices": (C.c_int32, [C.c_void_p, C.c_int32, PF, PF]),
    "rtg_scene_vertex_normals": (C.c_int32, [C.c_void_p, PF]),
    "rtg_comm_unique_id": (C.c_int32, [C.c_void_p]),
    "rtg_comm_init_rank": (C.c_int32, [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.POINTER(C.c_void_p)]),
    "rtg_comm_init_rank_timeout": (C.c_int32, [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                               C.POINTER(C.c_void_p)]),
    "rtg_comm_destroy": (C.c_int32, [C.c_void_p]),
    "rtg_render_ranked": (C.c_int32, [C.c_void_p, C.POINTER(CameraDesc), C.POINTER(RenderOpts), C.c_void_p,
                                      C.c_void_p, C.c_void_p]),
}

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "librtg.so")

_lib = None


class RtgError(RuntimeError):
    pass


def load_library(path: str | None = None):
    """Load librtg.so (in-tree).  Raises RtgError if it is missing or mismatched."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or os.environ.get("RTG_LIBRARY") or LIB_PATH   # RTG_LIBRARY: dev builds of variants
    if not os.path.exists(p):
        raise RtgError(f"librtg.so not found at {p}: run `python -c 'import __graft_entry__ as g; g.build()'`")
    # PyTorch-ROCm ships its own libamdhip64.so.7.  Loading torch first makes librtg bind to
    # that same HIP runtime (one runtime per process), so torch streams / allocations can be
    # handed to rtg_render_device.  Loading librtg first would pull /opt/rocm's runtime in as
    # a second instance and torch would then see no GPU.
    try:
        import torch  # noqa: F401
    except Exception:
        pass
    lib = C.CDLL(p)
    for name, (res, args) in EXPORTS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    v = lib.rtg_abi_version()
    # dev A/B variants (RTG_LIBRARY) may be one ABI older: ABI 9 only appended rtg_render_stats fields,
    # which then read 0 (the structure is zero-initialised and the older library writes its own prefix)
    if v != RTG_ABI_VERSION and not (os.environ.get("RTG_LIBRARY") and v == RTG_ABI_VERSION - 1 == 8):
        raise RtgError("librtg.so ABI version mismatch")
    if path is None:
        _lib = lib
    return lib


def loaded_abi() -> int:
    """The ABI version of the library in use (RTG_ABI_VERSION, or a dev variant's one older: the scene
    descriptor's layout is the same in ABI 8 and 9)."""
    try:
        return int(load_library().rtg_abi_version())
    except (RtgError, OSError):
        return RTG_ABI_VERSION


def check(rc: int, lib=None):
    if rc != RTG_OK:
        lib = lib or _lib
        msg = lib.rtg_last_error().decode() if lib is not None else ""
        raise RtgError(f"{STATUS.get(rc, rc)}: {msg}")
