"""GPU parity: librtg (HIP, gfx950) against the CPU restatement (oracle).

Bars (north_star): hit object / primitive indices bit-exact; image L-inf error < 1e-3 on
the reference's 0..255 float framebuffer.  The oracle is parity-unpinned (see
oracle/rtg_oracle.h); the GPU must match it on the same seeded inputs.
"""
import numpy as np
import pytest

import pyoracle
import rtg
from rtg import scenegen
from rtg import _abi as A

pytestmark = pytest.mark.gpu

TOL = 1e-3

SCENES = {
    "simple": lambda: scenegen.simple(96, 96),
    "bunny": lambda: scenegen.bunny5k(80, 60, level=3),
    "dragon": lambda: scenegen.dragon1m(80, 45, spp=1, nu=120, nv=60),
    "dragon_ms": lambda: scenegen.dragon1m(40, 24, spp=4, nu=60, nv=30),
    "cornell": lambda: scenegen.cornell(48, 36, spp=4),
    "cornell_nodof": lambda: scenegen.cornell(48, 36, spp=3, dof=False),
    "textured": lambda: scenegen.textured(64, 48),
    "textured_ms": lambda: scenegen.textured(32, 24, spp=2),
    "multilight": lambda: scenegen.multilight(64, 48),
    "multilight_ms": lambda: scenegen.multilight(32, 24, spp=3),
    "envmap": lambda: scenegen.envmap(48, 36, spp=2),
    "bgtex": lambda: scenegen.bgtex(48, 32, spp=1),
    "bgtex_ms": lambda: scenegen.bgtex(48, 32, spp=3, interp=1),
    "glass_nest": lambda: scenegen.glass_nest(32, 24, spp=2, max_depth=6),   # rays double per level
    # the full shading variants by light set (round 4, SceneView::heavy): textures / BRDFs without a
    # spot or environment light, and an area light together with a spot light
    "textured_point": lambda: _spot_to_point(scenegen.textured(48, 36)),
    "cornell_spot": lambda: _with_spot(scenegen.cornell(40, 30, spp=2)),
}


def _spot_to_point(sc):
    for L in sc.lights:
        if L.type == rtg._abi.LIGHT_SPOT:
            L.type = rtg._abi.LIGHT_POINT
    assert all(L.type not in (rtg._abi.LIGHT_SPOT, rtg._abi.LIGHT_ENVIRONMENT) for L in sc.lights)
    return sc


def _with_spot(sc):
    sc.lights.append(rtg.Light(type=rtg._abi.LIGHT_SPOT, position=(2.0, 8.0, 2.0), direction=(-0.3, -1.0, -0.4),
                               intensity=(600.0, 500.0, 400.0), coverage_deg=50.0, falloff_deg=30.0))
    return sc


def _cmp(img, ref):
    d = np.abs(img.astype(np.float64) - ref.astype(np.float64))
    nan_mismatch = int(np.sum(np.isnan(img) != np.isnan(ref)))
    d = np.where(np.isnan(d), 0.0, d)
    return float(d.max()), float((d > 0).mean()), nan_mismatch


@pytest.mark.parametrize("name", list(SCENES))
@pytest.mark.parametrize("traversal", [0, 1])
def test_render_matches_oracle(gpu, name, traversal):
    sc = SCENES[name]()
    with rtg.Renderer(sc, device=gpu) as r:
        img = r.render(0, traversal=traversal)
    ref, _, _, _ = pyoracle.Oracle(sc).render(0)
    linf, frac, nanm = _cmp(img, ref)
    print(f"{name} traversal={traversal}: Linf={linf:.3g} differing={frac:.2e}")
    assert nanm == 0
    assert linf < TOL


@pytest.mark.parametrize("name", ["simple", "bunny", "dragon", "cornell", "textured", "multilight"])
def test_trace_matches_oracle(gpu, name):
    sc = SCENES[name]()
    rng = np.random.default_rng(11)
    n = 4000
    lo = np.asarray(sc.vertices).min(0) - 1
    hi = np.asarray(sc.vertices).max(0) + 1
    o = rng.uniform(lo, hi, (n, 3)).astype(np.float32)
    d = rng.standard_normal((n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    t = rng.random(n).astype(np.float32)
    ref = pyoracle.Oracle(sc).trace(o, d, t)
    with rtg.Renderer(sc, device=gpu) as r:
        for trav in (0, 1):
            h = r.trace(o, d, t, traversal=trav)
            assert np.array_equal(h["full"], ref["full"])
            assert np.array_equal(h["object"], ref["object"])
            assert np.array_equal(h["prim"], ref["prim"])
            assert np.array_equal(h["material"], ref["material"])
            m = ref["full"] == 1
            assert np.array_equal(h["t"][m].view(np.int32), ref["t"][m].view(np.int32))
            assert np.array_equal(h["point"][m].view(np.int32), ref["point"][m].view(np.int32))
            assert np.array_equal(h["normal"][m].view(np.int32), ref["normal"][m].view(np.int32))


@pytest.mark.parametrize("name", ["cornell", "dragon"])
def test_trace_from_surface_points_matches_oracle(gpu, name):
    """Rays starting on (or within +-2 eps of) the scenes' triangles, as shadow and secondary rays
    do: the t >= -eps acceptance (src/Shape.cpp:330) with the top-level t > 0 rule
    (src/Helper.cpp:39-49) lets a candidate just behind the origin hide the rest of its object.
    Covers the flat meshes (cornell's walls, the 2-triangle quads: triangles tested without a
    node) and the root-box window (entries wholly behind the origin skipped) against the literal
    oracle, pruned and exhaustive."""
    sc = SCENES[name]()
    rng = np.random.default_rng(23)
    V = np.asarray(sc.vertices, np.float64)
    faces = np.concatenate([np.asarray(ob.faces) - 1 for ob in sc.objects if ob.faces is not None])
    # degenerate faces (the dragon's pole triangles have a zero cross product) have no normal to
    # offset along; drop them so every origin is a finite surface point
    cr = np.cross(V[faces[:, 1]] - V[faces[:, 0]], V[faces[:, 2]] - V[faces[:, 0]])
    faces = faces[np.linalg.norm(cr, axis=1) > 0]
    n = 6000
    f = faces[rng.integers(0, len(faces), n)]
    a, b, c = V[f[:, 0]], V[f[:, 1]], V[f[:, 2]]
    u, v = rng.random(n), rng.random(n)
    flip = u + v > 1
    u[flip], v[flip] = 1 - u[flip], 1 - v[flip]
    nrm = np.cross(b - a, c - a)
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    off = rng.uniform(-2, 2, n) * float(sc.int_eps)
    o = (a + (b - a) * u[:, None] + (c - a) * v[:, None] + nrm * off[:, None]).astype(np.float32)
    d = rng.standard_normal((n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    d = d.astype(np.float32)
    t = rng.random(n).astype(np.float32)
    assert np.isfinite(o).all(1).sum() >= 5000
    ref = pyoracle.Oracle(sc).trace(o, d, t)
    with rtg.Renderer(sc, device=gpu) as r:
        for trav in (0, 1):
            h = r.trace(o, d, t, traversal=trav)
            assert np.array_equal(h["full"], ref["full"])
            assert np.array_equal(h["object"], ref["object"])
            assert np.array_equal(h["prim"], ref["prim"])
            m = ref["full"] == 1
            assert np.array_equal(h["t"][m].view(np.int32), ref["t"][m].view(np.int32))
            assert np.array_equal(h["point"][m].view(np.int32), ref["point"][m].view(np.int32))


@pytest.mark.parametrize("name", ["cornell", "dragon"])
def test_trace_at_flat_box_edges_matches_oracle(gpu, name):
    """Round 5's pairwise slab decision (box_pairs): a line crossing a zero-thickness box -- the root
    and gate boxes of axis-aligned walls and floors -- meets it at one parameter, so the whole-box
    band test is always undecided; the six cross-axis exit/entry pairs decide it instead.  Rays aimed
    at the boxes' edges and corners (exactly, and a few ulp inside / outside), from inside and
    outside the scene, where a pair falls inside the band and the exact divisions must decide:
    every field bitwise against the literal oracle, pruned and exhaustive."""
    sc = SCENES[name]()
    rng = np.random.default_rng(41)
    V = np.asarray(sc.vertices, np.float32)
    pts = []
    for ob in sc.objects:
        if ob.faces is None or len(ob.faces) > 8:
            continue
        P = V[np.asarray(ob.faces).reshape(-1) - 1]
        lo, hi = P.min(0), P.max(0)
        for _ in range(400):
            q = rng.uniform(lo, hi).astype(np.float32)
            k = rng.integers(0, 3)
            q[k] = (lo if rng.random() < 0.5 else hi)[k]              # an edge / corner plane
            q = np.nextafter(q, rng.choice([-np.inf, np.inf], 3).astype(np.float32)) if rng.random() < 0.5 else q
            pts.append(q)
    pts = np.asarray(pts, np.float32)
    n = len(pts)
    c = V.mean(0)
    o = (c + rng.normal(0, 1, (n, 3)) * (V.max(0) - V.min(0)) * 0.4).astype(np.float32)
    d = (pts - o).astype(np.float64)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    d = d.astype(np.float32)
    t = rng.random(n).astype(np.float32)
    ref = pyoracle.Oracle(sc).trace(o, d, t)
    with rtg.Renderer(sc, device=gpu) as r:
        for trav in (0, 1):
            h = r.trace(o, d, t, traversal=trav)
            assert np.array_equal(h["full"], ref["full"])
            assert np.array_equal(h["object"], ref["object"])
            assert np.array_equal(h["prim"], ref["prim"])
            m = ref["full"] == 1
            assert np.array_equal(h["t"][m].view(np.int32), ref["t"][m].view(np.int32))
            assert np.array_equal(h["point"][m].view(np.int32), ref["point"][m].view(np.int32))


def test_trace_transformed_entries_any_time_matches_oracle(gpu):
    """cornell_dynamic's transformed entries (scaled / rotated instances, the motion-blurred sphere
    and instance) are skipped before their ray transform when the ray line misses their world box
    (TopObject::wbox, blur swept over times in [0, 1]).  Times outside [0, 1], direction components
    of exactly zero and rays from outside the room take the paths where that skip must not fire
    (or the exact division tests), against the literal oracle, pruned and exhaustive."""
    sc = scenegen.cornell(48, 36, spp=4)
    rng = np.random.default_rng(31)
    n = 6000
    lo = np.asarray(sc.vertices).min(0) - 3
    hi = np.asarray(sc.vertices).max(0) + 3
    o = rng.uniform(lo, hi, (n, 3)).astype(np.float32)
    d = rng.standard_normal((n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    zero = rng.random((n, 3)) < 0.08                  # some components exactly +-0
    d[zero] = 0.0
    d[np.all(d == 0, axis=1), 1] = -1.0
    d = d.astype(np.float32)
    t = rng.uniform(-0.5, 1.5, n).astype(np.float32)
    ref = pyoracle.Oracle(sc).trace(o, d, t)
    with rtg.Renderer(sc, device=gpu) as r:
        for trav in (0, 1):
            h = r.trace(o, d, t, traversal=trav)
            assert np.array_equal(h["full"], ref["full"])
            assert np.array_equal(h["object"], ref["object"])
            assert np.array_equal(h["prim"], ref["prim"])
            m = ref["full"] == 1
            assert np.array_equal(h["t"][m].view(np.int32), ref["t"][m].view(np.int32))
            assert np.array_equal(h["point"][m].view(np.int32), ref["point"][m].view(np.int32))
            assert np.array_equal(h["normal"][m].view(np.int32), ref["normal"][m].view(np.int32))


@pytest.mark.parametrize("name", ["cornell_pt", "spheres_small"])
def test_trace_untransformed_spheres_signed_zeros_matches_oracle(gpu, name):
    """Untransformed spheres (inverse = identity up to the signs of its zeros, zero blur) skip the
    ray transform (TopObject::ident, rtg_host.cpp): the world ray equals the object-space ray in value,
    not always in the signs of its zeros.  Origins and directions with components of exactly +0 and
    -0, aimed at the sphere centres or at random, against the literal oracle (hit records and the
    shading point / normal bitwise), pruned and exhaustive."""
    sc = scenegen.cornell_pt(32, 24, spp=1) if name == "cornell_pt" else scenegen.spheres(32, 24, spp=1, n=64)
    rng = np.random.default_rng(47)
    n = 8000
    cen = np.asarray([np.asarray(sc.vertices)[ob.center - 1] for ob in sc.objects
                      if ob.type == A.OBJ_SPHERE], np.float64)
    lo = np.asarray(sc.vertices).min(0) - 2
    hi = np.asarray(sc.vertices).max(0) + 2
    o = rng.uniform(lo, hi, (n, 3))
    tgt = cen[rng.integers(0, len(cen), n)]
    d = np.where(rng.random((n, 1)) < 0.7, tgt - o, rng.standard_normal((n, 3)))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    sgn = np.where(rng.random((n, 3)) < 0.5, -0.0, 0.0)
    zd = rng.random((n, 3)) < 0.15
    d[zd] = sgn[zd]
    d[np.all(d == 0, axis=1), 1] = -1.0
    zo = rng.random((n, 3)) < 0.15
    o[zo] = np.where(rng.random((n, 3)) < 0.5, -0.0, 0.0)[zo]
    o, d = o.astype(np.float32), d.astype(np.float32)
    t = np.zeros(n, np.float32)
    ref = pyoracle.Oracle(sc).trace(o, d, t)
    assert (ref["object"] >= 0).mean() > 0.3
    with rtg.Renderer(sc, device=gpu) as r:
        for trav in (0, 1):
            h = r.trace(o, d, t, traversal=trav)
            assert np.array_equal(h["full"], ref["full"])
            assert np.array_equal(h["object"], ref["object"])
            assert np.array_equal(h["prim"], ref["prim"])
            m = ref["full"] == 1
            for k in ("t", "point", "normal"):
                assert np.array_equal(h[k][m].view(np.int32), ref[k][m].view(np.int32)), k


@pytest.mark.parametrize("name", ["cornell_pt", "dragon_small"])
def test_trace_bounding_sphere_silhouette_matches_oracle(gpu, name):
    """Mesh entries with a world box whose world bounding sphere is tight (TopObject::bsph: cornell_pt's
    scaled, translated icosphere; the dragon's displaced sphere, untransformed but with glm's signed-zero
    inverse) are skipped by lanes whose ray line misses the sphere.  Rays grazing the sphere's
    silhouette (0.97-1.03 of its radius) from near and far origins (up to 400 units), a quarter of them
    turned away (the sphere behind the origin: its parameter test), against the literal oracle, pruned
    and exhaustive."""
    rng = np.random.default_rng(59)
    n = 8000
    if name == "cornell_pt":
        sc = scenegen.cornell_pt(32, 24, spp=1)
        c, rad = np.array([-1.2, 1.4, -2.0]), 1.4
        ico = next(k for k, ob in enumerate(sc.objects) if ob.type == A.OBJ_MESH and ob.xforms)
    else:
        sc = scenegen.dragon1m(32, 24, spp=1, nu=80, nv=40)
        ico = next(k for k, ob in enumerate(sc.objects) if ob.type == A.OBJ_MESH and len(ob.faces) > 100)
        v = np.asarray(sc.vertices, np.float64)[np.unique(np.asarray(sc.objects[ico].faces)) - 1]
        c = 0.5 * (v.min(0) + v.max(0))
        rad = np.sqrt(((v - c) ** 2).sum(1)).max()
    u = rng.standard_normal((n, 3))
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    dist = np.where(rng.random(n) < 0.5, rng.uniform(1.5, 12.0, n), rng.uniform(12.0, 400.0, n))
    o = c + u * dist[:, None]
    # a target on a random tangent offset: the line passes at 0.97-1.03 x the radius from the centre
    w = rng.standard_normal((n, 3))
    w -= (w * u).sum(1, keepdims=True) * u
    w /= np.linalg.norm(w, axis=1, keepdims=True)
    tgt = c + w * (rad * rng.uniform(0.97, 1.03, n))[:, None]
    d = tgt - o
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    d[rng.random(n) < 0.25] *= -1.0       # the sphere behind the origin (the parameter test)
    o, d = o.astype(np.float32), d.astype(np.float32)
    t = np.zeros(n, np.float32)
    ref = pyoracle.Oracle(sc).trace(o, d, t)
    assert (ref["object"] == ico).mean() > 0.05
    with rtg.Renderer(sc, device=gpu) as r:
        for trav in (0, 1):
            h = r.trace(o, d, t, traversal=trav)
            assert np.array_equal(h["object"], ref["object"])
            assert np.array_equal(h["prim"], ref["prim"])
            m = ref["full"] == 1
            assert np.array_equal(h["t"][m].view(np.int32), ref["t"][m].view(np.int32))


@pytest.mark.parametrize("block", [1, 2, 4, 5, 8])
def test_row_shards_sum_to_full_frame(gpu, block):
    """Multi-GPU partition (rows (y // block) % G == rank, incl. a partial last block) +
    exact sum == the single-device frame; each shard writes exactly its own rows."""
    from rtg.shard import owned_rows
    sc = scenegen.cornell(40, 30, spp=2)
    with rtg.Renderer(sc, device=gpu) as r:
        full = r.render(0)
        acc = np.zeros_like(full)
        for rank in range(3):
            part = r.render(0, row_offset=rank, row_stride=3, row_block=block)
            mask = np.zeros(30, bool)
            mask[owned_rows(30, rank, 3, block)] = True
            assert not part[~mask].any()
            compact = r.render(0, row_offset=rank, row_stride=3, row_block=block, compact_rows=1)
            assert np.array_equal(compact.view(np.int32), part[mask].view(np.int32))
            acc += part
    assert np.array_equal(acc.view(np.int32), full.view(np.int32))


def test_pruned_equals_exhaustive_dragon(gpu):
    """Full-resolution property: the ordered/pruned traversal returns the literal line-test
    result (1M-triangle BVH, 1 spp, 1920x1080 primary + secondary + shadow rays)."""
    sc = scenegen.dragon1m(1920, 1080, spp=1)
    with rtg.Renderer(sc, device=gpu) as r:
        a = r.render(0, traversal=0)
        b = r.render(0, traversal=1)
    linf, frac, nanm = _cmp(a, b)
    print(f"dragon1m 1080p pruned vs exhaustive: Linf={linf:.3g} differing={frac:.2e}")
    assert nanm == 0
    assert np.array_equal(np.nan_to_num(a).view(np.int32), np.nan_to_num(b).view(np.int32))


def test_reference_quirks_on_gpu(gpu):
    """The quirk cases pinned in test_oracle_kat.py give the same answers on the GPU:
    axis-parallel / tiny-component rays and a mesh hidden by a candidate behind the origin."""
    from test_oracle_kat import QUIRK_DIRS, _scene_with, quirk_mesh_scene
    from rtg import _abi as A
    from rtg.scene import Object
    sc = quirk_mesh_scene()
    with rtg.Renderer(sc, device=gpu) as r:
        for trav in (0, 1):
            h = r.trace([(0.01, 0.02, 0)] * 4, QUIRK_DIRS, traversal=trav)
            assert list(h["full"]) == [0, 0, 0, 1]
    verts = [(-1, -1, 0.0005), (1, -1, 0.0005), (0, 1, 0.0005), (-1, -1, -2), (1, -1, -2), (0, 1, -2)]
    sc2 = _scene_with([Object(type=A.OBJ_MESH, faces=np.array([[1, 2, 3], [4, 5, 6]], np.int32))], verts)
    with rtg.Renderer(sc2, device=gpu) as r:
        for trav in (0, 1):
            assert r.trace([(0, 0, 0)], [(0, 0, -1)], traversal=trav)["full"][0] == 0


def test_render_is_deterministic(gpu):
    sc = scenegen.cornell(64, 48, spp=8)
    with rtg.Renderer(sc, device=gpu) as r:
        a = r.render(0)
        b = r.render(0)
        c = r.render(0, max_batch_rays=1000)          # different pass batching, same sample order
        others = [r.render(0, max_batch_rays=1000, streams=k) for k in (1, 2, 8)]   # passes in flight
    assert np.array_equal(a.view(np.int32), b.view(np.int32))
    assert np.array_equal(a.view(np.int32), c.view(np.int32))
    for x in others:
        assert np.array_equal(a.view(np.int32), x.view(np.int32))


def test_sample_chunks_accumulate_in_order(gpu):
    """spp above the ray batch: sample chunks of one pixel range run as successive passes on
    one stream, so the in-order sum of MultiSample (src/Scene.cpp:386-409) is kept bit for bit."""
    sc = scenegen.cornell(24, 18, spp=8)
    with rtg.Renderer(sc, device=gpu) as r:
        a = r.render(0)
        for k in (1, 3):
            b = r.render(0, max_batch_rays=3, streams=k)   # ns_chunk = 3: chunks 0-2, 3-5, 6-7
            assert np.array_equal(a.view(np.int32), b.view(np.int32))


def test_ray_counts_match_oracle(gpu):
    """Point-light scenes: the GPU traces exactly the primary / secondary rays of the reference
    loop, and its shadow queries minus those whose light contributes exactly +0 (skipped: blocked
    or not, they add the same +0, rtg_device.hip light_sample)."""
    sc = scenegen.bunny5k(48, 36, level=3)
    with rtg.Renderer(sc, device=gpu) as r:
        r.render(0)
        st = r.stats()
    o = pyoracle.Oracle(sc)
    o.render(0)
    c = o.ray_counts()
    assert (st["primary_rays"], st["secondary_rays"]) == (c["primary"], c["secondary"])
    assert 0 < st["shadow_rays"] <= c["shadow"]


def test_render_device_into_torch_tensor(gpu):
    import torch
    sc = scenegen.simple(40, 30)
    with rtg.Renderer(sc, device=gpu) as r:
        host = r.render(0)
        t = torch.full((30, 40, 3), -1.0, device=f"cuda:{gpu}")
        r.render_device(0, t.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
    assert np.array_equal(t.cpu().numpy().view(np.int32), host.view(np.int32))


def test_xml_scene_renders_like_generated(gpu, tmp_path):
    from rtg.scene import parse_xml, write_xml
    sc = scenegen.dragon1m(48, 27, spp=2, nu=80, nv=40)
    back = parse_xml(write_xml(sc, str(tmp_path / "d.xml")))
    with rtg.Renderer(sc, device=gpu) as r:
        a = r.render(0)
    with rtg.Renderer(back, device=gpu) as r:
        b = r.render(0)
    assert np.array_equal(a.view(np.int32), b.view(np.int32))


@pytest.mark.parametrize("name", ["bunny5k", "cornell"])
def test_pruned_equals_exhaustive_full_res(gpu, name):
    sc = scenegen.bunny5k(1920, 1080) if name == "bunny5k" else scenegen.cornell(960, 540, spp=4)
    with rtg.Renderer(sc, device=gpu) as r:
        a = r.render(0, traversal=0)
        b = r.render(0, traversal=1)
    linf, frac, nanm = _cmp(a, b)
    print(f"{name} pruned vs exhaustive: Linf={linf:.3g} differing={frac:.2e}")
    assert nanm == 0
    assert np.array_equal(np.nan_to_num(a).view(np.int32), np.nan_to_num(b).view(np.int32))


def test_full_frame_shards_sum_exactly(gpu):
    """1080p dragon1m at 2 spp split over 4 row shards (bench's 8-row blocks) sums to the
    single-device frame."""
    from rtg.shard import shard_opts
    sc = scenegen.dragon1m(1920, 1080, spp=2)
    with rtg.Renderer(sc, device=gpu) as r:
        full = r.render(0)
        acc = np.zeros_like(full)
        for rank in range(4):
            acc += r.render(0, **shard_opts(rank, 4))
    assert np.array_equal(acc.view(np.int32), full.view(np.int32))


# One point / spot / directional light takes the lean shadow-record path (k_shadow rebuilds the
# direction and t bound, SceneView::lean_shadow); a rough mirror keeps the child RayMeta
# records (SceneView::meta_free off); two lights take the full four-plane records.
# "point_blur": one point light with a motion-blurred sphere -- the lean records keep their
# time lanes (SceneView::has_blur), as do the queued rays (RayQ time plane).
@pytest.mark.parametrize("kind", ["point", "spot", "directional", "two_lights", "rough_mirror", "point_blur"])
def test_shadow_record_paths_match_oracle(gpu, kind):
    from rtg import _abi as A
    from rtg.scene import Light
    sc = scenegen.bunny5k(64, 48, level=3, spp=2)
    L = sc.lights[0]
    if kind == "spot":
        sc.lights[0] = Light(type=A.LIGHT_SPOT, position=L.position, direction=(-0.4, -1.0, -0.6),
                             intensity=L.intensity, coverage_deg=50, falloff_deg=25)
    elif kind == "directional":
        sc.lights[0] = Light(type=A.LIGHT_DIRECTIONAL, direction=(-0.3, -1.0, -0.5), intensity=(3, 3, 3))
    elif kind == "two_lights":
        sc.lights.append(Light(type=A.LIGHT_DIRECTIONAL, direction=(0.5, -1.0, 0.2), intensity=(2, 2, 2)))
    elif kind == "rough_mirror":
        sc.materials[1].is_rough, sc.materials[1].roughness = True, 0.15
    elif kind == "point_blur":
        sph = next(ob for ob in sc.objects if ob.type == A.OBJ_SPHERE)
        sph.blur = (0.0, 0.3, 0.2)
    with rtg.Renderer(sc, device=gpu) as r:
        img = r.render(0)
        st = r.stats()
    o = pyoracle.Oracle(sc)
    ref, _, _, _ = o.render(0)
    linf, frac, nanm = _cmp(img, ref)
    print(f"{kind}: Linf={linf:.3g} differing={frac:.2e} shadow={st['shadow_rays']}/{o.ray_counts()['shadow']}")
    assert nanm == 0
    assert linf < TOL
    assert np.array_equal(np.nan_to_num(img).view(np.int32), np.nan_to_num(ref).view(np.int32)), kind
    assert 0 < st["shadow_rays"] <= o.ray_counts()["shadow"]
