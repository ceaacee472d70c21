"""The persistent lane-refill closest-hit kernel (k_trace_refill, env RTG_REFILL=1; an experiment,
DESIGN.md §4) returns the same frames as k_trace bit for bit: the entry order, candidate keys and
acceptance (src/Helper.cpp:32-73, src/BVH.cpp:137-210) do not depend on which rays share a wave."""
import os

import numpy as np
import pytest

import rtg
from rtg import scenegen

pytestmark = pytest.mark.gpu


def _bits(a):
    return np.nan_to_num(np.ascontiguousarray(a, np.float32)).view(np.int32)


SCENES = {
    "dragon": lambda: scenegen.dragon1m(96, 54, spp=4, nu=200, nv=100),
    "bunny": lambda: scenegen.bunny5k(80, 60, level=3),
    "cornell": lambda: scenegen.cornell(48, 36, spp=4),
    "cornell_pt": lambda: scenegen.cornell_pt(32, 24, spp=8),
    "glass_nest": lambda: scenegen.glass_nest(32, 24, spp=2, max_depth=6),
}


@pytest.fixture
def refill_env():
    keep = {k: os.environ.get(k) for k in ("RTG_REFILL", "RTG_REFILL_MIN", "RTG_REFILL_WAVES")}
    yield os.environ
    for k, v in keep.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v


@pytest.mark.parametrize("name", list(SCENES))
def test_refill_frames_equal_k_trace(gpu, refill_env, name):
    sc = SCENES[name]()
    with rtg.Renderer(sc, device=gpu) as r:
        refill_env.pop("RTG_REFILL", None)
        ref = r.render(0)
        st = r.stats()
        refill_env["RTG_REFILL"] = "1"
        for mn, waves in ((16, 4096), (1, 7), (64, 3)):
            refill_env["RTG_REFILL_MIN"], refill_env["RTG_REFILL_WAVES"] = str(mn), str(waves)
            img = r.render(0)
            assert np.array_equal(_bits(img), _bits(ref)), (name, mn, waves)
            assert r.stats()["total_rays"] == st["total_rays"]
