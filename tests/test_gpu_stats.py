"""collect_stats counters of the traversal kernels (rtg_render_stats, ABI 9): the flat group's lane
work and slots and its set-up / test cycle split, which bench.py's SIMD efficiency and
roofline.kernels.*.flat_group are computed from."""
import pytest

import rtg
from rtg import scenegen

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("make", [lambda: scenegen.cornell(48, 32, spp=4),
                                  lambda: scenegen.cornell_pt(40, 24, spp=4)])
def test_flat_group_counters(gpu, make):
    sc = make()
    with rtg.Renderer(sc, device=gpu) as r:
        r.render(0, collect_stats=1)
        st = r.stats()
        assert r.build_stats()["flat_group_entries"] >= 2
    for p in ("trace", "shadow"):
        work, slots = st[f"{p}_group_work"], st[f"{p}_group_slots"]
        assert 0 < work <= slots, (p, work, slots)
        assert slots % 64 == 0
        setup, tests = st[f"{p}_group_cycles"]
        assert setup > 0 and tests > 0
        # the group's slot of the per-entry cycles holds its whole time, the split holds its parts
        assert st[f"{p}_entry_cycles"][15] > 0
    # the all-work SIMD efficiency bench.py reports is a fraction
    eff = (st["trace_steps"] + st["trace_entry_visits"] + st["trace_group_work"]) / \
          (st["trace_lane_slots"] + st["trace_entry_slots"] + st["trace_group_slots"])
    assert 0.0 < eff <= 1.0


def test_frames_do_not_depend_on_collect_stats(gpu):
    """The counting instantiations run the same traversal: frames bit-identical with and without."""
    import numpy as np
    sc = scenegen.cornell_pt(32, 20, spp=3)
    with rtg.Renderer(sc, device=gpu) as r:
        a = r.render(0)
        b = r.render(0, collect_stats=1)
    assert np.array_equal(a.view(np.int32), b.view(np.int32))
