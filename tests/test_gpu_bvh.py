"""GPU BVH construction (rtg_bvh_gpu.hip) against the recursive builder.

Both must give the reference's tree (src/BVH.cpp:64-135, 268-303) bit for bit: the same
primitive permutation, the same pre-order topology and the same node boxes.  The host builder
is itself pinned to the oracle (tests/test_host_structures.py), so equality here pins the GPU
build transitively; the small cases are also checked against the oracle directly."""
import numpy as np
import pytest

import pyoracle
import rtg
from rtg import _abi as A
from rtg import scenegen
from rtg.scene import Object

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a).view(np.int32)


def _mesh_scene(verts, faces):
    sc = scenegen.simple(8, 8)
    base = len(sc.vertices) + 1
    sc.vertices = np.concatenate([sc.vertices, np.asarray(verts, np.float32)])
    sc.objects.append(Object(type=A.OBJ_MESH, id=9, material=1, faces=(np.asarray(faces, np.int32) + base)))
    return sc


def _random_mesh(n, seed, quant=None, dup=0.0):
    rng = np.random.default_rng(seed)
    v = rng.uniform(-2, 2, (3 * n, 3)).astype(np.float32)
    if quant:                                   # many equal centre coordinates (ties at the median)
        v = (np.round(v * quant) / quant).astype(np.float32)
    f = np.arange(3 * n).reshape(n, 3)
    if dup:                                     # repeated triangles: identical centres
        k = int(n * dup)
        f[:k] = f[0]
    return v, f


def _signed_zero_mesh(n, seed):
    """Coordinates that are exactly +0 or -0: box folds must keep the first of equal zeros."""
    rng = np.random.default_rng(seed)
    v = rng.uniform(-1, 1, (3 * n, 3)).astype(np.float32)
    m = rng.random(v.shape) < 0.3
    v[m] = np.where(rng.random(m.sum()) < 0.5, np.float32(0.0), np.float32(-0.0))
    return v, np.arange(3 * n).reshape(n, 3)


CASES = {
    "bunny": lambda: scenegen.bunny5k(8, 8, level=4),
    "dragon_200k": lambda: scenegen.dragon1m(8, 8, spp=1, nu=316, nv=316),
    "dragon1m_full": lambda: scenegen.dragon1m(8, 8, spp=1),
    "random_5k": lambda: _mesh_scene(*_random_mesh(5000, 1)),
    "quantised_20k": lambda: _mesh_scene(*_random_mesh(20000, 2, quant=4)),
    "duplicates_3k": lambda: _mesh_scene(*_random_mesh(3000, 3, dup=0.5)),
    "all_equal_600": lambda: _mesh_scene([(0, 0, -3), (1, 0, -3), (0, 1, -3)], [[0, 1, 2]] * 600),
    "signed_zero_4k": lambda: _mesh_scene(*_signed_zero_mesh(4000, 4)),
    "tiny_2": lambda: _mesh_scene(*_random_mesh(2, 5)),
    "tiny_3": lambda: _mesh_scene(*_random_mesh(3, 6)),
}


@pytest.mark.parametrize("name", list(CASES))
def test_gpu_bvh_equals_host_bvh(gpu, name):
    sc = CASES[name]()
    with rtg.Renderer(sc, device=gpu, bvh_builder=A.RTG_BVH_HOST) as a, \
            rtg.Renderer(sc, device=gpu, bvh_builder=A.RTG_BVH_GPU) as b:
        sa, sb = a.build_stats(), b.build_stats()
        meshes = [i for i, o in enumerate(sc.objects) if o.type != A.OBJ_SPHERE]
        assert sa["bvh_gpu_objects"] == 0 and sb["bvh_gpu_objects"] == len(meshes)
        print(f"{name}: host {sa['bvh_build_ms']:.1f} ms, gpu {sb['bvh_build_ms']:.1f} ms")
        for i in range(len(sc.objects)):
            p1, n1, b1 = a.bvh(i)
            p2, n2, b2 = b.bvh(i)
            assert np.array_equal(p1, p2), f"object {i} permutation"
            assert np.array_equal(n1, n2), f"object {i} topology"
            assert np.array_equal(bits(b1), bits(b2)), f"object {i} boxes"
    if name.startswith(("tiny", "random", "all_equal", "signed_zero", "duplicates")):
        o = pyoracle.Oracle(sc)
        p3, n3, b3 = o.bvh(len(sc.objects) - 1)
        o.close()
        assert np.array_equal(p2, p3) and np.array_equal(n2, n3) and np.array_equal(bits(b2), bits(b3))


def test_gpu_bvh_renders_identically(gpu):
    sc = scenegen.dragon1m(64, 36, spp=2, nu=200, nv=100)
    with rtg.Renderer(sc, device=gpu, bvh_builder=A.RTG_BVH_HOST) as a:
        x = a.render(0)
    with rtg.Renderer(sc, device=gpu, bvh_builder=A.RTG_BVH_GPU) as b:
        y = b.render(0)
    assert np.array_equal(bits(x), bits(y))
