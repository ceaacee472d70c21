"""The stream schedule (DESIGN.md §4 "Schedules", rtg_render_opts.schedule): steps that carry the
survivors of every ray-tree level together with new camera samples, instead of one launch per
level of each pass.  Both schedules compute every sample from the same rays in the same order
(src/Scene.cpp:148-219 bottom-up per sample, 386-411 per pixel in sample order), so frames and
ray counts must be bit-identical -- under small steps (levels mixed in every launch), one or
several lanes, and segments closed early by a small node-record budget (the reference integrator
resolves and sums a segment before it takes new samples again)."""
import numpy as np
import pytest

import pyoracle
import rtg
from rtg import _abi as A
from rtg import scenegen

pytestmark = pytest.mark.gpu

SCENES = {
    "dragon_ms": lambda: scenegen.dragon1m(40, 24, spp=4, nu=60, nv=30),     # meta-free Whitted, mirror + glass
    "glass_nest": lambda: scenegen.glass_nest(32, 24, spp=2, max_depth=6),   # rays double per level
    "cornell": lambda: scenegen.cornell(36, 27, spp=3),                      # area light, blur, DoF, rough mirror
    "textured_ms": lambda: scenegen.textured(32, 24, spp=2),                 # full variant, BRDFs, textures
    "multilight": lambda: scenegen.multilight(40, 30),                       # several lights, spp 1 (SingleSample)
    "bgtex": lambda: scenegen.bgtex(48, 32, spp=1),                          # transposed background at 1 spp
}


def _same(a, b):
    return np.array_equal(np.ascontiguousarray(a).view(np.int32), np.ascontiguousarray(b).view(np.int32))


@pytest.mark.parametrize("name", sorted(SCENES))
def test_stream_equals_passes_reference_integrator(gpu, name, monkeypatch):
    sc = SCENES[name]()
    with rtg.Renderer(sc, device=gpu) as r:
        ref = r.render(0, schedule=A.SCHEDULE_PASSES)
        st0 = r.stats()
        for batch, streams in ((0, 0), (300, 1), (1000, 3), (64, 2)):
            img = r.render(0, schedule=A.SCHEDULE_STREAM, max_batch_rays=batch, streams=streams,
                           segment_nodes=4200)       # ~4 K nodes: several segments
            st = r.stats()
            assert _same(img, ref), (name, batch, streams)
            assert (st["primary_rays"], st["secondary_rays"], st["shadow_rays"]) == \
                   (st0["primary_rays"], st0["secondary_rays"], st0["shadow_rays"]), (name, batch, streams)
        assert st["passes"] >= 1


def test_stream_matches_oracle_and_shards(gpu):
    """The reference integrator on the stream schedule (the pass schedule is its default since
    round 4: DESIGN.md §4 "Schedules"): against the oracle, and row shards gathered bit-exactly."""
    sc = scenegen.glass_nest(30, 20, spp=3, max_depth=6)
    with rtg.Renderer(sc, device=gpu) as r:
        img = r.render(0, schedule=A.SCHEDULE_STREAM)
        acc = np.zeros_like(img)
        for rank in range(3):
            acc += r.render(0, row_offset=rank, row_stride=3, row_block=4, schedule=A.SCHEDULE_STREAM)
    ref, _, _, _ = pyoracle.Oracle(sc).render(0)
    assert _same(np.nan_to_num(img), np.nan_to_num(ref))
    assert _same(acc, img)
