"""C ABI checks that need no GPU: the library loads, exports exactly what include/rtg.h
declares, the ctypes mirror has the C struct layouts, and descriptor validation rejects
malformed scenes before any device call."""
import ctypes as C
import os
import re
import subprocess
import tempfile

import numpy as np
import pytest

import rtg
from rtg import _abi as A
from rtg import scenegen

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "rtg.h")


def declared_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int32_t|int64_t|const char\*)\s+(rtg_\w+)\s*\(", src, re.M)))


def test_header_matches_ctypes_exports():
    assert declared_functions() == sorted(A.EXPORTS)


def test_library_exports_every_declared_symbol(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", A.LIB_PATH], capture_output=True, text=True, check=True)
    syms = set(re.findall(r"\sT\s(rtg_\w+)", out.stdout))
    missing = [f for f in declared_functions() if f not in syms]
    assert not missing, missing
    assert lib.rtg_abi_version() == A.RTG_ABI_VERSION


def test_struct_layouts_match_c():
    structs = ["rtg_xform_ref", "rtg_object_desc", "rtg_instance_desc", "rtg_material_desc", "rtg_texture_desc",
               "rtg_light_desc", "rtg_scene_desc", "rtg_camera_desc", "rtg_render_opts", "rtg_render_stats",
               "rtg_ray", "rtg_hit", "rtg_build_opts", "rtg_build_stats", "rtg_tonemap_desc"]
    py = [A.XformRef, A.ObjectDesc, A.InstanceDesc, A.MaterialDesc, A.TextureDesc, A.LightDesc, A.SceneDesc,
          A.CameraDesc, A.RenderOpts, A.RenderStats, A.Ray, A.Hit, A.BuildOpts, A.BuildStats, A.TonemapDesc]
    body = "\n".join(f'printf("%zu\\n", sizeof({s}));' for s in structs)
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "s.c")
        with open(c, "w") as fh:
            fh.write(f'#include <stdio.h>\n#include "{HEADER}"\nint main(void){{{body} return 0;}}\n')
        subprocess.run(["gcc", "-o", os.path.join(d, "s"), c], check=True)
        sizes = [int(x) for x in subprocess.run([os.path.join(d, "s")], capture_output=True, text=True).stdout.split()]
    assert sizes == [C.sizeof(p) for p in py]


def _create(lib, sc, device=A.RTG_DEVICE_HOST_ONLY if hasattr(A, "RTG_DEVICE_HOST_ONLY") else -1):
    desc, keep = sc.to_desc()
    h = C.c_void_p()
    rc = lib.rtg_scene_create(C.byref(desc), device, C.byref(h))
    return rc, h, keep


def test_host_only_scene_cannot_render(lib):
    sc = scenegen.simple(8, 8)
    rc, h, _ = _create(lib, sc)
    assert rc == A.RTG_OK
    cam = sc.cameras[0].desc()
    out = np.zeros((8, 8, 3), np.float32)
    rc = lib.rtg_render(h, C.byref(cam), None, out.ctypes.data_as(A.PF))
    assert rc == -2 and b"host-only" in lib.rtg_last_error()
    rays = (A.Ray * 1)()
    hits = (A.Hit * 1)()
    assert lib.rtg_trace_closest(h, rays, 1, hits, 0) == -2
    assert lib.rtg_scene_destroy(h) == 0


@pytest.mark.parametrize("mutate,msg", [
    (lambda sc: setattr(sc.objects[0], "material", 99), b"material"),
    (lambda sc: setattr(sc.objects[0], "center", 0), b"sphere center"),
    (lambda sc: setattr(sc.objects[3], "v", (1, 2, 999)), b"triangle index"),
    (lambda sc: setattr(sc.objects[0], "xforms", [(A.XF_TRANSLATION, 5)]), b"transformation"),
    (lambda sc: setattr(sc.objects[0], "textures", [3]), b"texture"),
])
def test_validation_rejects_malformed_descriptors(lib, mutate, msg):
    sc = scenegen.simple(8, 8)
    mutate(sc)
    rc, h, _ = _create(lib, sc)
    assert rc == -1
    assert msg in lib.rtg_last_error()


def test_abi_version_mismatch_rejected(lib):
    desc, keep = scenegen.simple(8, 8).to_desc()
    desc.abi_version = 999
    h = C.c_void_p()
    assert lib.rtg_scene_create(C.byref(desc), -1, C.byref(h)) == -1


def test_device_count_without_gpu_is_safe(lib):
    assert lib.rtg_device_count() >= 0


def test_missing_library_fails_loudly(tmp_path):
    with pytest.raises(rtg.RtgError):
        A.load_library(str(tmp_path / "nope.so"))


def test_pass_size_shrinks_with_the_lights(lib):
    """rtg_pass_rays: the per-pass ray count is capped at 24M and shrinks so that the level
    buffers of the passes in flight (68 B per ray and light) fit half the device memory."""
    gb = 288 << 30                                       # one MI355X
    one = lib.rtg_pass_rays(1, 0, 8, gb)
    assert one == 24 << 20
    sizes = [lib.rtg_pass_rays(n, 0, 8, gb) for n in (1, 8, 24, 64)]
    assert sizes == sorted(sizes, reverse=True) and sizes[-1] < sizes[0]
    for n, k in zip((1, 8, 24, 64), sizes):
        per_ray = 2 * (16 + 48 + 68 * n + 96)
        assert k * per_ray * 8 <= gb // 2 or k == 1 << 16
    assert lib.rtg_pass_rays(64, 1, 8, gb) < lib.rtg_pass_rays(64, 0, 8, gb)   # path records
    assert lib.rtg_pass_rays(64, 0, 1, gb) > lib.rtg_pass_rays(64, 0, 8, gb)   # fewer lanes
    assert lib.rtg_pass_rays(64, 0, 8, 0) == 24 << 20                          # no limit known
    assert lib.rtg_pass_rays(64, 0, 8, 1 << 20) == 1 << 16                     # floor
