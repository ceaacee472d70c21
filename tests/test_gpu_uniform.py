"""The wave-uniform traversal walk (`visit_object<..., UNI>`): waves of camera samples and
the shadow queries of camera-sample nodes walk the SAH traversal tree together (node / triangle indices
uniform, scalar-cache loads, slots visited when any lane needs them), every lane pruning and accepting by
its own window, test and reachability gate.  A lane then sees a superset of its own walk's candidates,
each valid, so the winner -- the minimum of the total order (dist, -leaf_start, prim) that the
reference's recursive walk returns (src/BVH.cpp:137-210) -- and every frame are unchanged.  Checked
here bitwise against the per-lane walk (rtg_build_opts.uniform_walk = 1) on both schedules and both
integrators, and against the oracle."""
import numpy as np
import pytest

import pyoracle
import rtg
from rtg import _abi as A
from rtg import scenegen

pytestmark = pytest.mark.gpu

SCENES = {
    # 64 spp: a wave is one pixel's samples (the coherent case the walk is for)
    "dragon": lambda: scenegen.dragon1m(48, 32, spp=64, nu=200, nv=100),
    # 1 spp: a wave spans 64 neighbouring pixels
    "bunny": lambda: scenegen.bunny5k(64, 48, level=3),
    "cornell": lambda: scenegen.cornell(40, 30, spp=16),
    "glass_nest": lambda: scenegen.glass_nest(32, 24, spp=8, max_depth=6),
}


def _same(a, b):
    return np.array_equal(np.ascontiguousarray(a).view(np.int32), np.ascontiguousarray(b).view(np.int32))


def _render_pair(sc, gpu, monkeypatch, **kw):
    with rtg.Renderer(sc, device=gpu) as r:
        uni = r.render(0, **kw)
        st_uni = r.stats()
    with rtg.Renderer(sc, device=gpu, uniform_walk=1) as r:
        lane = r.render(0, **kw)
        st_lane = r.stats()
    return uni, lane, st_uni, st_lane


@pytest.mark.parametrize("name", sorted(SCENES))
@pytest.mark.parametrize("schedule", [A.SCHEDULE_PASSES, A.SCHEDULE_STREAM])
def test_uniform_walk_equals_per_lane_walk(gpu, name, schedule, monkeypatch):
    uni, lane, su, sl = _render_pair(SCENES[name](), gpu, monkeypatch, schedule=schedule)
    assert _same(uni, lane), (name, schedule)
    assert (su["primary_rays"], su["secondary_rays"], su["shadow_rays"]) == \
           (sl["primary_rays"], sl["secondary_rays"], sl["shadow_rays"])


def test_uniform_walk_path_tracer(gpu, monkeypatch):
    """hw7 path tracer (stream schedule: camera waves of each step's new samples, and the NEE queries
    of those nodes) against the per-lane walk and the oracle."""
    sc = scenegen.cornell_pt(24, 18, spp=16)
    uni, lane, _, _ = _render_pair(sc, gpu, monkeypatch)
    assert _same(uni, lane)
    ref = pyoracle.Oracle(sc).render(0)[0]
    assert _same(np.nan_to_num(uni), np.nan_to_num(ref))


def test_uniform_walk_dragon_matches_oracle(gpu):
    sc = SCENES["dragon"]()
    with rtg.Renderer(sc, device=gpu) as r:
        img = r.render(0)
    ref = pyoracle.Oracle(sc).render(0)[0]
    assert _same(np.nan_to_num(img), np.nan_to_num(ref))
