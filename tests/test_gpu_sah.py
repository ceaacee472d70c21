"""The SAH traversal tree for meshes (rtg_build_opts.traversal_tree = 0) against the reference's
own tree walk (src/BVH.cpp:167-195 via Triangle::bvhIntersect, src/Shape.cpp:297-345): a
candidate only wins when the reference walk could reach it (its leaf's parent box passes the
exact slab test), so images and hit records must equal the oracle's bit for bit with either
tree."""
import numpy as np
import pytest

import pyoracle
import rtg
from rtg import scenegen

pytestmark = pytest.mark.gpu

SAH, REF_TREE = 0, 1


def _bits(a):
    return np.nan_to_num(np.ascontiguousarray(a, np.float32)).view(np.int32)


SCENES = {
    "bunny": lambda: scenegen.bunny5k(48, 36, level=2),
    "dragon": lambda: scenegen.dragon1m(48, 27, spp=2, nu=60, nv=30),
    "cornell": lambda: scenegen.cornell(40, 30, spp=3),
    "textured": lambda: scenegen.textured(40, 30),
    "cornell_pt": lambda: scenegen.cornell_pt(24, 18, spp=4),
}


@pytest.mark.parametrize("name", list(SCENES))
def test_sah_render_matches_oracle(gpu, name):
    sc = SCENES[name]()
    ref = pyoracle.Oracle(sc).render(0)[0]
    for tree in (SAH, REF_TREE):
        with rtg.Renderer(sc, device=0, traversal_tree=tree) as r:
            img = r.render(0)
        assert np.array_equal(np.isnan(img), np.isnan(ref))
        assert np.array_equal(_bits(img), _bits(ref)), f"{name} tree={tree}"


@pytest.mark.parametrize("name", ["bunny", "dragon"])
def test_sah_random_rays_match_oracle(gpu, name):
    """Origins inside and around the mesh, directions random, a slice with one tiny component
    (the reference tree's exact walk) and a slice grazing along box faces."""
    sc = SCENES[name]()
    v = np.asarray(sc.vertices, np.float32)
    lo, hi = v.min(0), v.max(0)
    ext = hi - lo
    rng = np.random.default_rng(31)
    n = 30000
    o = rng.uniform(lo - 0.3 * ext, hi + 0.3 * ext, (n, 3)).astype(np.float32)
    tgt = rng.uniform(lo, hi, (n, 3)).astype(np.float32)
    d = tgt - o
    d[: n // 10] = rng.standard_normal((n // 10, 3))
    d[n // 10: n // 5, 0] *= 1e-9                                  # gett() on a tiny component
    k = slice(n // 5, n // 4)
    o[k, 1] = rng.choice(v[:, 1], n // 4 - n // 5)               # in the plane of a vertex
    d[k, 1] = 0.0
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    ref = pyoracle.Oracle(sc).trace(o, d)
    for tree in (SAH, REF_TREE):
        with rtg.Renderer(sc, device=0, traversal_tree=tree) as r:
            h = r.trace(o, d)
        for key in ("full", "object", "prim", "material"):
            assert np.array_equal(h[key], ref[key]), (tree, key)
        m = ref["full"] == 1
        for key in ("t", "point", "normal"):
            assert np.array_equal(h[key][m].view(np.int32), ref[key][m].view(np.int32)), (tree, key)
