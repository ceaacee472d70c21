"""Edge cases of the render path on the GPU, each against the oracle bit for bit: empty and
light-less scenes, degenerate image sizes, MaxRecursionDepth 0, many lights (the in-order
light sum of Scene::RecursiveShading, src/Scene.cpp:148-219), every primary ray missing,
glass far from the origin (Beer's law on overflowing distances), and empty / NaN ray batches
for rtg_trace_closest (src/Helper.cpp:28-30 returns {} on NaN)."""
import numpy as np
import pytest

import pyoracle
import rtg
from rtg import _abi as A
from rtg import scenegen
from rtg.scene import Light, Material, Object, Scene

pytestmark = pytest.mark.gpu


def _same(sc, **kw):
    with rtg.Renderer(sc, device=0) as r:
        img = r.render(0, **kw)
    ref = pyoracle.Oracle(sc).render(0, **kw)[0]      # same row shard (others stay 0)
    assert img.shape == ref.shape
    assert np.array_equal(np.isnan(img), np.isnan(ref))
    assert np.array_equal(np.nan_to_num(img).view(np.int32), np.nan_to_num(ref).view(np.int32))
    return img


def test_empty_scene_is_background(gpu):
    sc = Scene(background=(12, 34, 56), ambient=(1, 1, 1))
    sc.cameras.append(scenegen._cam((0, 0, 0), (0, 0, -1), (0, 1, 0), 7, 5, spp=3))
    img = _same(sc)
    assert np.all(img == np.float32([12, 34, 56]))


def test_scene_without_lights_is_ambient_only(gpu):
    sc = scenegen.simple(20, 14)
    sc.lights = []
    _same(sc)


@pytest.mark.parametrize("nx,ny,spp", [(1, 1, 1), (1, 1, 5), (1, 9, 2), (13, 1, 1), (37, 13, 3)])
def test_degenerate_image_sizes(gpu, nx, ny, spp):
    sc = scenegen.multilight(nx, ny, spp=spp)
    _same(sc)
    if ny > 1:
        _same(sc, row_offset=1, row_stride=2, row_block=4)


def test_max_recursion_depth_zero(gpu):
    sc = scenegen.multilight(32, 24)
    sc.max_depth = 0
    _same(sc)


def test_many_lights_in_order(gpu):
    sc = scenegen.simple(24, 18)
    rng = np.random.default_rng(3)
    for k in range(24):
        kind = (A.LIGHT_POINT, A.LIGHT_DIRECTIONAL, A.LIGHT_SPOT)[k % 3]
        sc.lights.append(Light(type=kind, position=tuple(rng.uniform(-3, 3, 3) + (0, 4, 0)),
                               direction=tuple(rng.uniform(-1, 1, 3) - (0, 1, 0)),
                               intensity=tuple(rng.uniform(10, 400, 3)), coverage_deg=40, falloff_deg=20))
    _same(sc)


def test_all_primary_rays_miss(gpu):
    sc = scenegen.simple(16, 12)
    sc.cameras[0].gaze = np.float32([0, 1, 0])        # looking up, away from every object
    sc.cameras[0].up = np.float32([0, 0, 1])
    img = _same(sc)
    assert np.all(img == 0)


@pytest.mark.parametrize("scale", [1.0, 3e17, 1e18, 1e19])
@pytest.mark.parametrize("intensity", [0.0, 500.0])
def test_far_glass_beer_distance(gpu, scale, intensity):
    """A non-absorbing glass sphere in front of a diffuse one, the scene scaled so hit points reach
    1e18-1e19: Beer's law (src/Scene.cpp:110) then sees |q0 - p| overflow (exp(-0 * inf) = NaN) or
    not, so the refracted child's hit point must reach the bottom-up pass even where the child is
    a final diffuse node without a shadow query (light intensity 0: no queries at all)."""
    S = scale
    sc = Scene(max_depth=3, background=(10, 20, 30), ambient=(20, 20, 20))
    sc.cameras.append(scenegen._cam((0, 0, 0), (0, 0, -1), (0, 1, 0), 24, 16, fov_deg=50, spp=2))
    sc.materials += [
        Material(type=A.MAT_DIELECTRIC, ambient=(0, 0, 0), diffuse=(0, 0, 0), specular=(0, 0, 0),
                 refraction_index=1.5, absorption_coeff=(0, 0, 0)),
        Material(ambient=(1, 1, 1), diffuse=(0.6, 0.4, 0.3), specular=(0.2, 0.2, 0.2), phong_exp=8),
    ]
    v = scenegen._add_vertices(sc, [(0.2 * S, 0.0, -3.0 * S), (-0.3 * S, 0.1 * S, -6.0 * S)])
    sc.objects.append(Object(type=A.OBJ_SPHERE, id=1, material=1, center=v, radius=1.0 * S))
    sc.objects.append(Object(type=A.OBJ_SPHERE, id=2, material=2, center=v + 1, radius=1.5 * S))
    sc.lights.append(Light(type=A.LIGHT_POINT, position=(0, 4 * S, -1 * S), intensity=(intensity,) * 3))
    _same(sc)


@pytest.mark.parametrize("kind", ["point", "directional", "spot", "area"])
@pytest.mark.parametrize("blur", [False, True])
def test_single_light_shadow_records(gpu, kind, blur):
    """One light of each kind, with and without motion blur: the lit-node shadow records (k_shade
    stores the lit colour, k_shadow restores the ambient term of a blocked query; the lean origin-only
    records, and the blurred lean records whose mode travels in L.w) against the oracle, with a mirror
    (a second level) and shadows cast on the floor by the spheres."""
    sc = scenegen.simple(40, 30)
    sc.cameras[0].num_samples = 4
    sc.max_depth = 2
    sc.materials[1].type = A.MAT_MIRROR
    sc.materials[1].mirror = (0.6, 0.6, 0.6)
    if blur:
        sc.objects[0].blur = (0.0, 0.25, 0.0)
    L = {"point": Light(type=A.LIGHT_POINT, position=(0.3, 3.0, -1.0), intensity=(900, 800, 700)),
         "directional": Light(type=A.LIGHT_DIRECTIONAL, direction=(0.2, -1.0, -0.3), intensity=(0.9, 0.8, 0.7)),
         "spot": Light(type=A.LIGHT_SPOT, position=(0.0, 3.0, -1.5), direction=(0.0, -1.0, -0.1),
                       intensity=(900, 800, 700), coverage_deg=35, falloff_deg=20),
         "area": Light(type=A.LIGHT_AREA, position=(0.0, 3.0, -1.5), direction=(0.0, -1.0, 0.0),
                       intensity=(900, 800, 700), size=1.5)}[kind]
    sc.lights = [L]
    _same(sc)


def test_trace_empty_and_nan_batches(gpu):
    sc = scenegen.simple(8, 8)
    with rtg.Renderer(sc, device=0) as r:
        h = r.trace(np.zeros((0, 3), np.float32), np.zeros((0, 3), np.float32))
        assert len(h["full"]) == 0
        nan = np.float32(np.nan)
        h = r.trace([(0, 0, 0), (nan, 0, 0), (0, 0, 0)], [(0, 0, -1), (0, 0, -1), (nan, 0, -1)])
        assert list(h["full"]) == [1, 0, 0]


def test_too_wide_image_is_rejected(gpu):
    """A band of tile_pixel's widest tiles must stay below 2^31 pixels (32-bit band arithmetic):
    an image wider than 2^28 pixels is refused before any work, not mis-tiled."""
    import torch
    sc = scenegen.simple(8, 1)
    cam = sc.cameras[0]
    cam.nx = (1 << 28) + 1
    out = torch.zeros(3, device="cuda:0")
    with rtg.Renderer(sc, device=0) as r:
        with pytest.raises(A.RtgError, match="wider than"):
            r.render_device(cam, out.data_ptr())
