"""Product host-side flattening (librtg, RTG_DEVICE_HOST_ONLY) against the oracle,
bit for bit: per-object BVH permutation / topology / boxes (src/BVH.cpp:64-135),
inverse and inverse-transpose matrices (src/Helper.cpp:135-226) and smooth vertex normals
(src/Scene.cpp:302-318).  The product builds its BVH with nth_element selection and the
oracle with a full sort per node (as the reference does); both must agree exactly."""
import ctypes as C

import numpy as np
import pytest

import pyoracle
from rtg import _abi as A
from rtg import scenegen
from rtg.render import _bvh

SCENES = {
    "simple": lambda: scenegen.simple(8, 8),
    "bunny": lambda: scenegen.bunny5k(8, 8, level=4),
    "dragon_200k": lambda: scenegen.dragon1m(8, 8, spp=1, nu=316, nv=316),
    "dragon1m_full": lambda: scenegen.dragon1m(8, 8, spp=1),          # the bench BVH (1,000,000 tris)
    "cornell": lambda: scenegen.cornell(8, 8, spp=1),
    "textured": lambda: scenegen.textured(8, 8),
}


def bits(a):
    return np.ascontiguousarray(a).view(np.int32)


@pytest.mark.parametrize("name", list(SCENES))
def test_host_structures_bit_identical(lib, name):
    sc = SCENES[name]()
    desc, keep = sc.to_desc()
    h = C.c_void_p()
    assert lib.rtg_scene_create(C.byref(desc), A.RTG_DEVICE_HOST_ONLY, C.byref(h)) == 0, lib.rtg_last_error()
    o = pyoracle.Oracle(sc)
    try:
        for i in range(len(sc.objects)):
            p1, n1, b1 = _bvh(lib.rtg_scene_object_bvh, h, i)
            p2, n2, b2 = o.bvh(i)
            assert np.array_equal(p1, p2), f"object {i} permutation"
            assert np.array_equal(n1, n2), f"object {i} topology"
            assert np.array_equal(bits(b1), bits(b2)), f"object {i} boxes"
        for t in range(len(sc.objects) + len(sc.instances)):
            inv = np.zeros(16, np.float32)
            it = np.zeros(16, np.float32)
            assert lib.rtg_scene_object_matrices(h, t, inv.ctypes.data_as(A.PF), it.ctypes.data_as(A.PF)) == 0
            a, b = o.matrices(t)
            assert np.array_equal(bits(inv), bits(a)) and np.array_equal(bits(it), bits(b))
        vn = np.zeros((len(sc.vertices), 3), np.float32)
        assert lib.rtg_scene_vertex_normals(h, vn.ctypes.data_as(A.PF)) == 0
        assert np.array_equal(bits(vn), bits(o.vertex_normals()))
    finally:
        lib.rtg_scene_destroy(h)
        o.close()


def test_degenerate_centres_hit_depth_cap(lib):
    """Identical centroids never split (src/BVH.cpp:95-106): the builder must stop at depth 30
    with a multi-primitive leaf, exactly like the reference."""
    sc = scenegen.simple(8, 8)
    base = len(sc.vertices) + 1
    sc.vertices = np.concatenate([sc.vertices, np.array([(0, 0, -3), (1, 0, -3), (0, 1, -3)], np.float32)])
    faces = np.array([[base, base + 1, base + 2]] * 40, np.int32)
    from rtg.scene import Object
    sc.objects.append(Object(type=A.OBJ_MESH, id=9, material=1, faces=faces))
    desc, keep = sc.to_desc()
    h = C.c_void_p()
    assert lib.rtg_scene_create(C.byref(desc), A.RTG_DEVICE_HOST_ONLY, C.byref(h)) == 0
    p1, n1, _ = _bvh(lib.rtg_scene_object_bvh, h, len(sc.objects) - 1)
    p2, n2, _ = pyoracle.Oracle(sc).bvh(len(sc.objects) - 1)
    lib.rtg_scene_destroy(h)
    assert np.array_equal(p1, p2) and np.array_equal(n1, n2)
    leaves = n1[(n1[:, 0] < 0) & (n1[:, 1] < 0)]
    assert (leaves[:, 3] - leaves[:, 2]).max() == 40


def test_parallel_root_box_keeps_the_reference_fold_with_nan(lib):
    """the top levels of a >= 64K-triangle host build (construct_par) reduce their node
    boxes in chunks.  The reference's fold (ComputeBoundingBox, src/BVH.cpp:268-283, min/maxOfTwo
    as `a <= b ? a : b`) drops everything before the last NaN, which a merge of chunk results does
    not; a mesh with a NaN vertex coordinate must get the sequential fold (the oracle's).  The NaN
    sits in the third vertex's z of one triangle three quarters into the face list, so the
    triangle's box z is NaN (minOfThree(a, b, NaN) = NaN): the reference's root box z then comes from
    the triangles after it only, while a chunked merge would also take the earlier chunks'."""
    sc = scenegen.dragon1m(8, 8, spp=1, nu=300, nv=150)     # 90,000 triangles in the mesh
    mesh = len(sc.objects) - 1
    faces = sc.objects[mesh].faces
    f = faces[(3 * len(faces)) // 4]
    sc.vertices = np.array(sc.vertices, np.float32, copy=True)
    sc.vertices[f[2] - 1, 2] = np.nan
    desc, keep = sc.to_desc()
    h = C.c_void_p()
    assert lib.rtg_scene_create(C.byref(desc), A.RTG_DEVICE_HOST_ONLY, C.byref(h)) == 0, lib.rtg_last_error()
    o = pyoracle.Oracle(sc)
    try:
        p1, n1, b1 = _bvh(lib.rtg_scene_object_bvh, h, mesh)
        p2, n2, b2 = o.bvh(mesh)
        assert np.isnan(b2).any(), "the fixture must put a NaN into a node box"
        # Nodes down to depth 2 (x, y splits: the NaN is only in a z coordinate, so these medians
        # are well defined): same ranges and bit-identical boxes, found by their path from the root.
        # Below, a z split over a NaN centroid depends on the sort algorithm (the reference's
        # std::sort with NaN is unspecified), so the permutation is not compared there.
        def walk(n, b, node, depth, path, out):
            out[path] = (tuple(n[node][2:4]), bits(b[node]).tobytes())
            if depth < 2:
                for k, child in ((0, n[node][0]), (1, n[node][1])):
                    if child >= 0:
                        walk(n, b, child, depth + 1, path + "LR"[k], out)
        a, r = {}, {}
        walk(n1, b1, 0, 0, "", a)
        walk(n2, b2, 0, 0, "", r)
        assert a == r
    finally:
        lib.rtg_scene_destroy(h)
        o.close()
