"""Known-answer tests that pin the CPU restatement (oracle/) where something outside it can:
Random123's published Philox4x32-10 vectors, analytic ray/primitive geometry, BVH
construction invariants of src/BVH.cpp:64-135, and the reference quirks the restatement
must keep (SURVEY.md §7 hard parts).  The reference ships no fixtures of its own, so the
oracle's render output itself stays parity-unpinned."""
import math

import numpy as np
import pytest

import pyoracle
from rtg import _abi as A
from rtg import scenegen
from rtg.scene import Camera, Light, Material, Object, Scene

f32 = np.float32


# Random123 kat_vectors, philox4x32 10 rounds: (ctr, key) -> out
PHILOX_KAT = [
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


@pytest.mark.parametrize("ctr,key,out", PHILOX_KAT)
def test_philox_known_answers(ctr, key, out):
    assert tuple(pyoracle.philox4x32_10(ctr, key)) == out


def test_uniform_mapping_is_generate_canonical():
    # (float)u / 2^32 clamped below 1 (libstdc++ generate_canonical<float,24>)
    vals = [pyoracle.rng_uniform(s, 3, 4, 5, 1, 0, 0, lane) for s in range(50) for lane in range(4)]
    assert all(0.0 <= v < 1.0 for v in vals)
    assert abs(np.mean(vals) - 0.5) < 0.08


def _scene_with(objects, vertices, materials=None, lights=None, eps=0.001):
    sc = Scene(int_eps=eps, shadow_eps=0.002, max_depth=1)
    sc.vertices = np.asarray(vertices, f32).reshape(-1, 3)
    sc.materials = materials or [Material()]
    sc.objects = objects
    sc.lights = lights or []
    sc.cameras = [Camera(nx=4, ny=4)]
    return sc


def test_sphere_analytic_hit():
    sc = _scene_with([Object(type=A.OBJ_SPHERE, center=1, radius=1.0)], [(0, 0, -5)])
    h = pyoracle.Oracle(sc).trace([(0, 0, 0)], [(0, 0, -1)])
    assert h["full"][0] == 1 and h["object"][0] == 0
    assert h["t"][0] == pytest.approx(4.0, abs=1e-6)
    np.testing.assert_allclose(h["point"][0], (0, 0, -4), atol=1e-6)
    np.testing.assert_allclose(h["normal"][0], (0, 0, 1), atol=1e-6)


def test_sphere_origin_inside_picks_positive_root():
    sc = _scene_with([Object(type=A.OBJ_SPHERE, center=1, radius=2.0)], [(0, 0, 0)])
    h = pyoracle.Oracle(sc).trace([(0, 0, 0)], [(1, 0, 0)])
    assert h["full"][0] == 1 and h["t"][0] == pytest.approx(2.0, abs=1e-6)


def test_triangle_barycentric_epsilon_band():
    # Triangle a=(0,0,-1) b=(1,0,-1) c=(0,1,-1); accept iff beta,gamma >= -eps, beta+gamma <= 1
    verts = [(0, 0, -1), (1, 0, -1), (0, 1, -1)]
    sc = _scene_with([Object(type=A.OBJ_TRIANGLE, v=(1, 2, 3))], verts, eps=0.01)
    o = pyoracle.Oracle(sc)
    h = o.trace([(-0.005, 0.5, 0), (-0.02, 0.5, 0), (0.6, 0.39, 0), (0.6, 0.41, 0)], [(0, 0, -1)] * 4)
    assert list(h["full"]) == [1, 0, 1, 0]
    assert h["t"][0] == pytest.approx(1.0, abs=1e-6)


def test_object_rejected_when_nearest_candidate_is_behind_origin():
    """src/BVH.cpp:159-173 + src/Helper.cpp:39-49: a mesh whose nearest candidate has
    t in [-eps, 0] contributes nothing, even if it has a valid hit further along."""
    verts = [(-1, -1, 0.0005), (1, -1, 0.0005), (0, 1, 0.0005),       # just behind the origin
             (-1, -1, -2), (1, -1, -2), (0, 1, -2)]                     # in front
    mesh = Object(type=A.OBJ_MESH, faces=np.array([[1, 2, 3], [4, 5, 6]], np.int32))
    sc = _scene_with([mesh], verts)
    h = pyoracle.Oracle(sc).trace([(0, 0, 0)], [(0, 0, -1)])
    assert h["full"][0] == 0
    # the same triangles as two separate objects: the front one is found
    sc2 = _scene_with([Object(type=A.OBJ_TRIANGLE, v=(1, 2, 3)), Object(type=A.OBJ_TRIANGLE, v=(4, 5, 6))], verts)
    h2 = pyoracle.Oracle(sc2).trace([(0, 0, 0)], [(0, 0, -1)])
    assert h2["full"][0] == 1 and h2["object"][0] == 1


def quirk_mesh_scene():
    v, f = scenegen.icosphere(1)
    mesh = Object(type=A.OBJ_MESH, faces=(f + 1).astype(np.int32))
    return _scene_with([mesh], v - np.array([0, 0, 3.0]))


QUIRK_DIRS = [(0.0, 0.0, -1.0), (-0.0, -0.0, -1.0), (1e-30, 1e-30, -1.0), (1e-7, 1e-7, -1.0)]


def test_axis_parallel_and_tiny_direction_quirks():
    """BVH::RayBBoxIntersection (src/BVH.cpp:212-233): a zero direction component takes the
    `else` branch, (max-o)/0 = +inf becomes the slab entry and the box is missed (glm's
    mat4*vec4 turns -0 into +0, so both signs miss).  Ray::gett (src/Ray.cpp:21-36) then
    rejects a tiny x component: p.x rounds back to o.x, t = 0, and `distance > 0` fails."""
    o = pyoracle.Oracle(quirk_mesh_scene())
    h = o.trace([(0.01, 0.02, 0)] * 4, QUIRK_DIRS)
    assert list(h["full"]) == [0, 0, 0, 1]


def test_bvh_invariants():
    sc = scenegen.bunny5k(8, 8, level=3)
    o = pyoracle.Oracle(sc)
    mesh_idx = [i for i, ob in enumerate(sc.objects) if ob.type == A.OBJ_MESH][0]
    perm, nodes, boxes = o.bvh(mesh_idx)
    n = len(sc.objects[mesh_idx].faces)
    assert sorted(perm.tolist()) == list(range(n))
    faces = np.asarray(sc.objects[mesh_idx].faces)[perm]
    verts = np.asarray(sc.vertices)
    centers = ((verts[faces[:, 0] - 1] + verts[faces[:, 1] - 1]) + verts[faces[:, 2] - 1]) / f32(3)

    def walk(k, depth):
        left, right, s, e = nodes[k]
        if left < 0 and right < 0:
            assert e - s == 1 or depth >= 30
            return depth
        axis = depth % 3
        ls = nodes[left] if left >= 0 else None
        rs = nodes[right] if right >= 0 else None
        split = ls[3] if ls is not None else s
        assert (ls is None or (ls[2] == s)) and (rs is None or rs[3] == e)
        if ls is not None and rs is not None:
            assert ls[3] == rs[2]
            # in-place partition around the median: left centres < split <= right centres
            assert centers[s:split, axis].max() < centers[split:e, axis].min()
        # box contains children's boxes
        for c in (left, right):
            if c >= 0:
                assert np.all(boxes[c][:3] >= boxes[k][:3]) and np.all(boxes[c][3:] <= boxes[k][3:])
        return max(walk(c, depth + 1) for c in (left, right) if c >= 0)

    assert walk(0, 0) <= 30


def test_rotation_matrix_against_float64():
    sc = _scene_with([Object(type=A.OBJ_SPHERE, center=1, radius=1.0,
                             xforms=[(A.XF_TRANSLATION, 1), (A.XF_ROTATION, 1), (A.XF_SCALING, 1)])], [(0, 0, 0)])
    sc.translations = [(1.0, 2.0, 3.0)]
    sc.rotations = [(30.0, 0.0, 1.0, 0.0)]
    sc.scalings = [(2.0, 2.0, 2.0)]
    inv, _ = pyoracle.Oracle(sc).matrices(0)
    M = np.linalg.inv(np.asarray(inv, np.float64).reshape(4, 4).T)
    c, s = math.cos(math.radians(30)), math.sin(math.radians(30))
    T = np.eye(4); T[:3, 3] = (1, 2, 3)
    Rm = np.eye(4); Rm[0, 0], Rm[0, 2], Rm[2, 0], Rm[2, 2] = c, s, -s, c
    S = np.diag([2.0, 2.0, 2.0, 1.0])
    np.testing.assert_allclose(M, S @ Rm @ T, atol=1e-5)   # "t1 r1 s1": translate first


def test_oracle_render_is_deterministic_and_finite():
    sc = scenegen.cornell(24, 18, spp=4)
    o = pyoracle.Oracle(sc)
    a = o.render(0)[0]
    b = o.render(0, nthreads=1)[0]
    assert np.array_equal(a.view(np.int32), b.view(np.int32))
    assert np.isfinite(a).all()


def test_background_texture_transposed_at_1spp():
    """Scene::SingleSample passes (row = x, col = y) to GetBackgroundColor (src/Scene.cpp:365-380,
    544-566), so at 1 spp a replace_background texture is looked up at (u, v) = (y/nx, x/ny);
    MultiSample (> 1 spp) uses (x/nx, y/ny); coordinates wrap (GetColorAtCoordinates, src/Texture.cpp:111-119)."""
    nx, ny = 48, 32
    for spp in (1, 4):
        sc = scenegen.bgtex(nx, ny, spp=spp)
        img, obj, _, _ = pyoracle.Oracle(sc).render(0)
        tex = sc.textures[0].texels
        h, w, _ = tex.shape
        ys, xs = np.nonzero(obj == -1)
        assert len(ys) > 100
        for y, x in zip(ys[::37], xs[::37]):
            if spp == 1:
                u, v = np.float32(y) / np.float32(nx), np.float32(x) / np.float32(ny)
            else:
                u, v = np.float32(x) / np.float32(nx), np.float32(y) / np.float32(ny)
            u, v = u - np.floor(u), v - np.floor(v)          # Texture::GetColorAtCoordinates wrap
            i, j = min(int(u * np.float32(w)), w - 1), min(int(v * np.float32(h)), h - 1)
            if spp == 1:
                assert np.array_equal(img[y, x], tex[j, i]), (y, x)
            else:   # every sample of a background pixel sees the same texel at NN
                assert np.allclose(img[y, x], tex[j, i], rtol=1e-6), (y, x)
