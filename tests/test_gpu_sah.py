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


# ---------------------------------------------------------------- GPU-built traversal tree (round 5)
HOST_B, GPU_B = 1, 2   # rtg_bvh_builder: RTG_BVH_HOST, RTG_BVH_GPU


def _soup(n, seed, nx=40, ny=30):
    """n random triangles (no two with the same centroid) in the unit cube, camera and a point light."""
    from rtg import _abi as A
    from rtg.scene import Light, Material, Object, Scene
    rng = np.random.default_rng(seed)
    sc = Scene(max_depth=2, background=(10, 10, 20), ambient=(20, 20, 20))
    sc.cameras.append(scenegen._cam((0.5, 0.5, 3.0), (0, 0, -1), (0, 1, 0), nx, ny, fov_deg=40))
    sc.materials.append(Material(ambient=(1, 1, 1), diffuse=(0.7, 0.6, 0.5), specular=(0.3, 0.3, 0.3), phong_exp=20))
    c = rng.uniform(0, 1, (n, 1, 3))
    v = (c + rng.normal(0, 0.02, (n, 3, 3))).astype(np.float32).reshape(-1, 3)
    b = scenegen._add_vertices(sc, v)
    faces = (np.arange(3 * n, dtype=np.int32).reshape(n, 3) + b).astype(np.int32)
    sc.objects.append(Object(type=A.OBJ_MESH, id=1, material=1, faces=faces))
    sc.lights.append(Light(type=A.LIGHT_POINT, position=(0.5, 3, 3), intensity=(800, 800, 800)))
    return sc


def _tree(sc, builder):
    with rtg.Renderer(sc, device=0, bvh_builder=builder) as r:
        bs = r.build_stats()
        img = r.render(0)
    return bs, img


@pytest.mark.parametrize("n", [2, 5, 300, 512, 513, 1025, 2048, 2049, 5000, 70000])
def test_gpu_sah_tree_equals_host_tree(gpu, n):
    """The GPU binned-SAH build applies the host's split rule to the same record sets, so both trees
    have the same nodes (box + triangle count; order-independent hash) and every frame is identical.
    Sizes at the one-wave subtree limit (kSmall = 512 records in rtg_sah_gpu.hip: 512 is built by one
    wave, 513 takes one level step first, ~1025 splits into halves at about the limit) and in the level
    phase (70000)."""
    sc = _soup(n, seed=n)
    bh, ih = _tree(sc, HOST_B)
    bg, ig = _tree(sc, GPU_B)
    assert bh["sah_gpu_objects"] == 0 and bg["sah_gpu_objects"] == 1
    assert bg["traversal_nodes"] == bh["traversal_nodes"] > 0
    assert bg["traversal_hash"] == bh["traversal_hash"]
    assert np.array_equal(_bits(ig), _bits(ih))


def test_gpu_sah_dragon_tree_and_frames(gpu):
    """The C3 mesh at 160 K triangles: the level phase, then subtrees; same tree as the host's, frames
    and random hit records bit-identical to the oracle."""
    sc = scenegen.dragon1m(48, 27, spp=2, nu=400, nv=200)
    bh, ih = _tree(sc, HOST_B)
    bg, ig = _tree(sc, GPU_B)
    assert bg["sah_gpu_objects"] >= 1
    assert bg["traversal_hash"] == bh["traversal_hash"] and bg["traversal_nodes"] == bh["traversal_nodes"]
    ref = pyoracle.Oracle(sc).render(0)[0]
    assert np.array_equal(_bits(ig), _bits(ref))


def test_gpu_sah_duplicate_centroids_match_oracle(gpu):
    """Ranges whose centroids are all equal are halved by count; the two builders may then put
    different members in each half (trees may differ), but every result stays the oracle's."""
    sc = _soup(3000, seed=7)
    v = np.asarray(sc.vertices, np.float32).copy()
    v[-3 * 600:] = np.tile(v[-3:], (600, 1))                   # 600 copies of one triangle
    sc.vertices = v
    _, ig = _tree(sc, GPU_B)
    ref = pyoracle.Oracle(sc).render(0)[0]
    assert np.array_equal(_bits(ig), _bits(ref))
    rng = np.random.default_rng(3)
    o = rng.uniform(-0.5, 1.5, (20000, 3)).astype(np.float32)
    d = rng.standard_normal((20000, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    with rtg.Renderer(sc, device=0, bvh_builder=GPU_B) as r:
        h = r.trace(o, d)
    hr = pyoracle.Oracle(sc).trace(o, d)
    for key in ("full", "object", "prim"):
        assert np.array_equal(h[key], hr[key]), key
