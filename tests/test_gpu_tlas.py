"""Top-level BVH over objects and instances (rtg_build_opts.tlas) against the reference's linear
object loop (src/Helper.cpp:32-73): the same winner, including the first-object-wins rule for
equal distances (`distance < nearestDistance`, objects before instances, src/Helper.cpp:43, 64).
Every image and hit record must equal the oracle's bit for bit, with the TLAS forced on scenes
that would not use it by default and off on the many-sphere scene that would."""
import numpy as np
import pytest

import pyoracle
import rtg
from rtg import scenegen
from rtg.scene import Instance, Object

pytestmark = pytest.mark.gpu

TLAS_AUTO, TLAS_OFF, TLAS_ON = 0, 1, 2


def _bits(a):
    return np.nan_to_num(np.ascontiguousarray(a, np.float32)).view(np.int32)


def _render(sc, tlas, **kw):
    with rtg.Renderer(sc, device=0, tlas=tlas) as r:
        img = r.render(0, **kw)
        return img, r.stats(), r.build_stats()


SCENES = {
    "spheres": lambda: scenegen.spheres(64, 40, spp=2),
    "spheres_1spp": lambda: scenegen.spheres(56, 40, spp=1),
    "cornell": lambda: scenegen.cornell(40, 30, spp=3),
    "bunny": lambda: scenegen.bunny5k(48, 36, level=2),
    "multilight": lambda: scenegen.multilight(40, 30),
    "textured": lambda: scenegen.textured(40, 30),
    "envmap": lambda: scenegen.envmap(32, 24, spp=2),
    "dragon": lambda: scenegen.dragon1m(48, 27, spp=2, nu=60, nv=30),
    "cornell_pt": lambda: scenegen.cornell_pt(24, 18, spp=4),
}


@pytest.mark.parametrize("name", list(SCENES))
def test_tlas_render_matches_oracle(gpu, name):
    sc = SCENES[name]()
    ref = pyoracle.Oracle(sc).render(0)[0]
    for tlas in (TLAS_ON, TLAS_OFF):
        img, st, bs = _render(sc, tlas)
        assert (bs["tlas_nodes"] > 0) == (tlas == TLAS_ON)
        assert np.array_equal(np.isnan(img), np.isnan(ref))
        assert np.array_equal(_bits(img), _bits(ref)), f"{name} tlas={tlas}"


def test_many_spheres_use_the_tlas_by_default(gpu):
    sc = SCENES["spheres"]()
    img, st, bs = _render(sc, TLAS_AUTO)
    assert bs["tlas_nodes"] >= len(sc.objects) + len(sc.instances) - 1


def _tie_scene():
    """Coincident entries: the same sphere three times (materials 1, 2, 3) and the same mesh as an
    object and as two instances with identity transforms (materials 4, 5, 6) -- every hit is a tie
    broken by the loop order."""
    sc = scenegen.simple(40, 30)
    sc.objects = []
    c = len(sc.vertices) + 1
    sc.vertices = np.concatenate([np.asarray(sc.vertices, np.float32),
                                  np.float32([[0.0, 0.0, -2.0], [-1, -0.5, -1.5], [1, -0.5, -1.5], [0, 0.7, -3.0]])])
    while len(sc.materials) < 6:
        sc.materials.append(sc.materials[len(sc.materials) % 3])
    for m in (2, 1, 3):
        sc.objects.append(Object(type=0, id=len(sc.objects) + 1, material=m, center=c, radius=0.5))
    sc.objects.append(Object(type=2, id=10, material=4, faces=np.array([[c + 1, c + 2, c + 3]], np.int32)))
    base = len(sc.objects) - 1
    sc.instances.append(Instance(base_object=base, id=11, material=5, reset_transform=False))
    sc.instances.append(Instance(base_object=base, id=12, material=6, reset_transform=True))
    return sc


def test_ties_go_to_the_first_entry(gpu):
    sc = _tie_scene()
    rng = np.random.default_rng(5)
    n = 6000
    o = np.tile(np.float32([0, 0, 1.5]), (n, 1)) + rng.normal(0, 0.05, (n, 3)).astype(np.float32)
    tgt = rng.uniform([-1.1, -0.7, -3.1], [1.1, 0.8, -1.4], (n, 3)).astype(np.float32)
    d = tgt - o
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    ref = pyoracle.Oracle(sc).trace(o, d)
    for tlas in (TLAS_ON, TLAS_OFF):
        with rtg.Renderer(sc, device=0, tlas=tlas) as r:
            h = r.trace(o, d)
        for k in ("full", "object", "prim", "material"):
            assert np.array_equal(h[k], ref[k]), (tlas, k)
        m = ref["full"] == 1
        assert np.array_equal(h["t"][m].view(np.int32), ref["t"][m].view(np.int32))
    assert set(np.unique(ref["object"][ref["full"] == 1])) <= {0, 3}       # always the first copy


def test_tlas_trace_random_rays_match_oracle(gpu):
    """Random rays through the sphere field (origins inside it too): hit records bit-exact."""
    sc = scenegen.spheres(8, 6, spp=1, n=300)
    rng = np.random.default_rng(17)
    n = 20000
    lo = np.float32([-17, -1.2, -23])
    hi = np.float32([17, 3, 11])
    o = rng.uniform(lo, hi, (n, 3)).astype(np.float32)
    d = rng.standard_normal((n, 3)).astype(np.float32)
    d[: n // 4, 1] = -np.abs(d[: n // 4, 1])                 # a quarter aimed downwards
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    t = rng.random(n).astype(np.float32)
    ref = pyoracle.Oracle(sc).trace(o, d, t)
    with rtg.Renderer(sc, device=0, tlas=TLAS_ON) as r:
        h = r.trace(o, d, t)
    for k in ("full", "object", "prim", "material"):
        assert np.array_equal(h[k], ref[k]), k
    m = ref["full"] == 1
    for k in ("t", "point", "normal"):
        assert np.array_equal(h[k][m].view(np.int32), ref[k][m].view(np.int32)), k


def test_tlas_gett_ties_from_a_tiny_direction_component(gpu):
    """gett() divides by the first nonzero direction component (src/Ray.cpp:21-36): with a tiny x
    component it quantises t so coarsely that spheres at different depths tie, and the first in
    the loop must win.  The ray below is one such case from the 1080p64 spheres frame (level-1
    reflection, row 519); the batch around it varies the tiny component and the origin."""
    sc = scenegen.spheres(8, 6, spp=1)
    rng = np.random.default_rng(23)
    n = 20000
    o = np.float32([-1.411496639251709, -0.4932418763637543, -4.315512657165527]) + \
        rng.uniform(-3, 3, (n, 3)).astype(np.float32) * np.float32([1, 0.1, 1])
    d = np.empty((n, 3), np.float32)
    d[:, 0] = rng.choice([-1, 1], n) * 10.0 ** rng.uniform(-8, -5, n)
    ang = rng.uniform(-0.6, 0.3, n)
    d[:, 1] = np.sin(ang)
    d[:, 2] = -np.cos(ang)
    d[0] = [6.705522537231445e-07, -0.2306806743144989, -0.9730295538902283]
    o[0] = [-1.411496639251709, -0.4932418763637543, -4.315512657165527]
    ref = pyoracle.Oracle(sc).trace(o, d)
    with rtg.Renderer(sc, device=0, tlas=TLAS_ON) as r:
        h = r.trace(o, d)
    for k in ("full", "object", "prim", "material"):
        assert np.array_equal(h[k], ref[k]), k
    m = ref["full"] == 1
    assert np.array_equal(h["t"][m].view(np.int32), ref["t"][m].view(np.int32))


def test_full_frame_tlas_equals_linear_loop(gpu):
    """The 1080p spheres frame (8 spp): the TLAS and the linear object loop give the same image
    bit for bit and the same ray counts (the size at which the gett() tie above was found)."""
    sc = scenegen.spheres(1920, 1080, spp=8)
    a, sa, _ = _render(sc, TLAS_OFF)
    b, sb, bs = _render(sc, TLAS_ON)
    assert bs["tlas_nodes"] > 0
    assert np.array_equal(_bits(a), _bits(b))
    for k in ("primary_rays", "secondary_rays", "shadow_rays"):
        assert sa[k] == sb[k], k
