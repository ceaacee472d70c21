"""GPU parity of the hw7 path tracer (pages/Page7.md; no reference code exists, so the CPU
restatement in oracle/rtg_oracle.c pt_sample() is the specification).

The GPU wavefront (k_pt_shade / k_shadow, radiance carried with each path) must reproduce the oracle's paths on
the same Philox stream: same image within the north_star bar (L-inf < 1e-3 on the float
framebuffer) and the same number of traced rays, for every combination of the hw7 renderer
parameters (uniform / importance sampling, next event estimation, Russian roulette).
"""
import numpy as np
import pytest

import pyoracle
import rtg
from rtg import _abi as A
from rtg import scenegen

pytestmark = pytest.mark.gpu

TOL = 1e-3
I, N, R = A.PT_IMPORTANCE, A.PT_NEE, A.PT_RUSSIAN_ROULETTE
FLAGS = [0, I, N, I | N, R, I | R, N | R, I | N | R]


def _cmp(img, ref):
    d = np.abs(img.astype(np.float64) - ref.astype(np.float64))
    nan_mismatch = int(np.sum(np.isnan(img) != np.isnan(ref)))
    d = np.where(np.isnan(d), 0.0, d)
    return float(d.max()), float((d > 0).mean()), nan_mismatch


def _phong(sc):
    """Same scene through the non-BRDF (reference Blinn-Phong) response: the simple shading variant."""
    for m in sc.materials:
        if m.brdf != A.BRDF_NONE:
            m.brdf = A.BRDF_NONE
            m.diffuse = tuple(float(v) / np.pi for v in m.diffuse)
            m.phong_exp = max(m.phong_exp, 1)
    return sc


@pytest.mark.parametrize("flags", [I | N | R, N])
def test_path_trace_torrance_sparrow_variant_matches_oracle(gpu, flags):
    """BRDF-only scene with Torrance-Sparrow materials: the k_pt_shade<false, false, 2> variant (the
    cornell_pt default, without them, runs k_pt_shade<false, false, 1>; round 4)."""
    sc = scenegen.cornell_pt(32, 24, spp=4, flags=flags)
    sc.materials[0].brdf = A.BRDF_TS
    sc.materials[3].brdf = A.BRDF_TSF
    sc.materials[3].refraction_index, sc.materials[3].absorption_index = 1.3, 2.0
    with rtg.Renderer(sc, device=gpu) as r:
        img = r.render(0)
    ref, _, _, _ = pyoracle.Oracle(sc).render(0)
    linf, frac, nanm = _cmp(img, ref)
    assert nanm == 0
    assert linf < TOL


@pytest.mark.parametrize("flags", FLAGS)
def test_path_trace_matches_oracle(gpu, flags):
    sc = scenegen.cornell_pt(40, 30, spp=6, flags=flags)
    with rtg.Renderer(sc, device=gpu) as r:
        img = r.render(0)
        st = r.stats()
    o = pyoracle.Oracle(sc)
    ref, _, _, _ = o.render(0)
    linf, frac, nanm = _cmp(img, ref)
    print(f"flags={flags}: Linf={linf:.3g} differing={frac:.2e} rays={st['total_rays']}")
    assert nanm == 0
    assert linf < TOL
    c = o.ray_counts()
    assert (st["primary_rays"], st["secondary_rays"]) == (c["primary"], c["secondary"])
    # zero-contribution queries of the scene's reference lights are not traced (see light_sample)
    assert st["shadow_rays"] <= c["shadow"]


@pytest.mark.parametrize("flags", [I | N | R, N])
def test_path_trace_simple_variant_matches_oracle(gpu, flags):
    """Scene without BRDFs / textures: the k_pt_shade<false, ...> specialisation."""
    sc = _phong(scenegen.cornell_pt(32, 24, spp=4, flags=flags))
    with rtg.Renderer(sc, device=gpu) as r:
        img = r.render(0)
    ref, _, _, _ = pyoracle.Oracle(sc).render(0)
    linf, frac, nanm = _cmp(img, ref)
    assert nanm == 0
    assert linf < TOL


def test_path_trace_single_sample_and_single_light(gpu):
    """spp = 1 (SingleSample camera path) and exactly one object light (k_shadow's direct add)."""
    sc = scenegen.cornell_pt(48, 36, spp=1, flags=I | N, light_sphere=False)
    with rtg.Renderer(sc, device=gpu) as r:
        img = r.render(0)
    ref, _, _, _ = pyoracle.Oracle(sc).render(0)
    linf, _, nanm = _cmp(img, ref)
    assert nanm == 0
    assert linf < TOL


@pytest.mark.parametrize("flags", [I, 0, N, I | R])
def test_furnace_on_gpu(gpu, flags):
    """Analytic: a convex kd/pi-Lambertian sphere inside a LightSphere of radiance Le has
    radiance kd * Le (exact per sample with importance sampling, unbiased otherwise)."""
    sc = scenegen.furnace(16, 12, spp=256, flags=flags)
    with rtg.Renderer(sc, device=gpu) as r:
        img = r.render(0)
    want = 0.6 * np.array([10.0, 20.0, 40.0])
    centre = img[4:8, 6:10].reshape(-1, 3).mean(0)
    tol = 1e-5 if flags == I else 0.03
    assert np.allclose(centre, want, rtol=tol), (centre, want)


def test_path_trace_row_shards_and_batching(gpu):
    """Row shards of the multi-GPU partition sum to the single-device frame bit for bit, and
    the frame does not depend on pass batching or streams in flight."""
    sc = scenegen.cornell_pt(36, 27, spp=5)
    with rtg.Renderer(sc, device=gpu) as r:
        full = r.render(0)
        acc = np.zeros_like(full)
        for rank in range(2):
            acc += r.render(0, row_offset=rank, row_stride=2, row_block=8)
        b = r.render(0, max_batch_rays=777, streams=2)
        c = r.render(0, max_batch_rays=3, streams=1)       # sample chunks accumulate in order
    assert np.array_equal(acc.view(np.int32), full.view(np.int32))
    assert np.array_equal(b.view(np.int32), full.view(np.int32))
    assert np.array_equal(c.view(np.int32), full.view(np.int32))


def test_reference_integrator_ignores_object_lights(gpu):
    """With the reference integrator an object light is an ordinary object (the reference
    parser has no light objects); the Whitted path still matches the oracle."""
    sc = scenegen.cornell_pt(32, 24, spp=2)
    sc.cameras[0].integrator = A.INTEGRATOR_REFERENCE
    with rtg.Renderer(sc, device=gpu) as r:
        img = r.render(0)
    ref, _, _, _ = pyoracle.Oracle(sc).render(0)
    linf, _, nanm = _cmp(img, ref)
    assert nanm == 0
    assert linf < TOL


@pytest.mark.parametrize("name,make", [
    ("textured", lambda: scenegen.textured(32, 24, spp=2)),          # textures, BRDFs, spot + directional
    ("cornell_area_dof", lambda: scenegen.cornell(32, 24, spp=4)),   # area light, instances, blur, DoF
    ("multilight", lambda: scenegen.multilight(32, 24, spp=2)),      # spots, rough mirror, conductor, glass
])
@pytest.mark.parametrize("flags", [I | N | R, 0])
def test_path_trace_full_variant_matches_oracle(gpu, name, make, flags):
    """The reference scenes path traced (classical lights as BasicShading at every vertex):
    the full k_pt_shade specialisation (textures / area light / every material type)."""
    sc = make()
    sc.cameras[0].integrator = A.INTEGRATOR_PATH
    sc.cameras[0].pt_flags = flags
    with rtg.Renderer(sc, device=gpu) as r:
        img = r.render(0)
    ref, _, _, _ = pyoracle.Oracle(sc).render(0)
    linf, frac, nanm = _cmp(img, ref)
    print(f"{name} flags={flags}: Linf={linf:.3g} differing={frac:.2e}")
    assert nanm == 0
    assert linf < TOL


@pytest.mark.parametrize("flags", [I | N | R, N | R, I])
def test_stream_schedule_equals_pass_schedule(gpu, flags, monkeypatch):
    """The stream schedule (steps mixing the survivors of every level with new camera samples,
    DESIGN.md §4 "Schedules") renders the pass schedule's frame bit for bit and traces the same
    rays: small steps (many regenerating steps per lane, levels mixed in every launch), one or
    three lanes, and segments of a few pixels (the radiance buffer reused)."""
    sc = scenegen.cornell_pt(37, 23, spp=7, flags=flags)
    with rtg.Renderer(sc, device=gpu) as r:
        ref = r.render(0, schedule=A.SCHEDULE_PASSES)
        st0 = r.stats()
        for batch, streams in ((0, 0), (500, 1), (1300, 3), (64, 2)):
            img = r.render(0, schedule=A.SCHEDULE_STREAM, max_batch_rays=batch, streams=streams, segment_pixels=97)
            st = r.stats()
            assert np.array_equal(img.view(np.int32), ref.view(np.int32)), (batch, streams)
            assert (st["primary_rays"], st["secondary_rays"], st["shadow_rays"]) == \
                   (st0["primary_rays"], st0["secondary_rays"], st0["shadow_rays"]), (batch, streams)
    o = pyoracle.Oracle(sc)
    want, _, _, _ = o.render(0)
    linf, _, nanm = _cmp(img, want)
    assert nanm == 0 and linf < TOL
