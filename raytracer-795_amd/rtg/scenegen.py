"""Synthetic scenes for the BASELINE.json configs.

The reference ships no scene files, so every benchmark / parity scene is generated here
with fixed seeds:
  C1 simple          3 spheres + 1 triangle, point light, 800x800, 1 spp, depth 1
  C2 bunny5k         displaced icosphere (5,120 tris, flat), mirror floor, glass sphere, depth 6
  C3 dragon1m        1000x500-quad displaced UV sphere (1,000,000 tris) + mirror & glass spheres
  C4 cornell_dynamic cornell walls mesh, 2 mesh instances (resetTransform on/off), motion-blurred
                     sphere, area light, DoF camera, 64 spp
  C5 cornell_pt      C4 geometry at 256 spp, 1920x1080 (distribution ray tracing: the reference
                     has no path tracer in src/)
`size` arguments shrink resolution / tessellation for parity tests.
"""
from __future__ import annotations

import math

import numpy as np

from . import _abi as A
from .scene import Camera, Instance, Light, Material, Object, Scene, Texture

f32 = np.float32


def _perlin3(p: np.ndarray, seed: int) -> np.ndarray:
    """Small value-noise used only to jitter generated geometry (not the renderer's Perlin)."""
    rng = np.random.default_rng(seed)
    lat = rng.random((16, 16, 16))
    q = p * 4.0
    i = np.floor(q).astype(np.int64)
    f = q - i
    w = f * f * (3 - 2 * f)
    out = np.zeros(len(p))
    for dx in (0, 1):
        for dy in (0, 1):
            for dz in (0, 1):
                v = lat[(i[:, 0] + dx) % 16, (i[:, 1] + dy) % 16, (i[:, 2] + dz) % 16]
                wt = (w[:, 0] if dx else 1 - w[:, 0]) * (w[:, 1] if dy else 1 - w[:, 1]) * (w[:, 2] if dz else 1 - w[:, 2])
                out += v * wt
    return out - 0.5


def icosphere(level: int):
    t = (1.0 + math.sqrt(5.0)) / 2.0
    v = [(-1, t, 0), (1, t, 0), (-1, -t, 0), (1, -t, 0), (0, -1, t), (0, 1, t), (0, -1, -t), (0, 1, -t),
         (t, 0, -1), (t, 0, 1), (-t, 0, -1), (-t, 0, 1)]
    v = [np.array(x, float) / np.linalg.norm(x) for x in v]
    f = [(0, 11, 5), (0, 5, 1), (0, 1, 7), (0, 7, 10), (0, 10, 11), (1, 5, 9), (5, 11, 4), (11, 10, 2), (10, 7, 6),
         (7, 1, 8), (3, 9, 4), (3, 4, 2), (3, 2, 6), (3, 6, 8), (3, 8, 9), (4, 9, 5), (2, 4, 11), (6, 2, 10),
         (8, 6, 7), (9, 8, 1)]
    for _ in range(level):
        cache = {}
        nf = []

        def mid(a, b):
            key = (min(a, b), max(a, b))
            if key not in cache:
                m = (v[a] + v[b]) / 2
                v.append(m / np.linalg.norm(m))
                cache[key] = len(v) - 1
            return cache[key]

        for a, b, c in f:
            ab, bc, ca = mid(a, b), mid(b, c), mid(c, a)
            nf += [(a, ab, ca), (b, bc, ab), (c, ca, bc), (ab, bc, ca)]
        f = nf
    return np.array(v), np.array(f, np.int64)


def uv_sphere(nu: int, nv: int, seed: int = 20261015):
    """(nu x nv) quads -> 2*nu*nv triangles (quad split (0,1,2),(2,3,0) as Parser.h:1069-1079),
    radius 1 + 0.05 sin(13 theta) sin(17 phi) + jitter."""
    th = np.linspace(0.0, math.pi, nv + 1)
    ph = np.linspace(0.0, 2 * math.pi, nu + 1)
    T, P = np.meshgrid(th, ph, indexing="ij")            # (nv+1, nu+1)
    dirs = np.stack([np.sin(T) * np.cos(P), np.cos(T), np.sin(T) * np.sin(P)], -1).reshape(-1, 3)
    r = 1.0 + 0.05 * np.sin(13 * T) * np.sin(17 * P)
    r = r.reshape(-1) + 0.02 * _perlin3(dirs + 1.5, seed)
    verts = dirs * r[:, None]
    idx = np.arange((nv + 1) * (nu + 1)).reshape(nv + 1, nu + 1)
    a = idx[:-1, :-1].reshape(-1)
    b = idx[1:, :-1].reshape(-1)
    c = idx[1:, 1:].reshape(-1)
    d = idx[:-1, 1:].reshape(-1)
    quads = np.stack([a, d, c, b], 1)          # counter-clockwise seen from outside
    tris = np.empty((quads.shape[0] * 2, 3), np.int64)
    tris[0::2] = quads[:, [0, 1, 2]]
    tris[1::2] = quads[:, [2, 3, 0]]
    return verts, tris


def _cam(pos, gaze, up, nx, ny, fov_deg=45.0, dist=1.0, spp=1, name="out.png", **kw):
    half = math.tan(math.radians(fov_deg) / 2) * dist
    aspect = nx / ny
    c = Camera(position=np.array(pos, f32), gaze=np.array(gaze, f32), up=np.array(up, f32),
               near_plane=(float(f32(-half * aspect)), float(f32(half * aspect)), float(f32(-half)), float(f32(half))),
               near_distance=dist, nx=nx, ny=ny, num_samples=spp, image_name=name)
    for k, v in kw.items():
        setattr(c, k, v)
    return c


def _add_vertices(sc: Scene, v: np.ndarray) -> int:
    """Append vertices, return the 1-based index of the first one."""
    base = len(sc.vertices) + 1
    sc.vertices = np.concatenate([np.asarray(sc.vertices, f32).reshape(-1, 3), np.asarray(v, f32)])
    return base


def simple(nx=800, ny=800) -> Scene:
    """C1: hw1 simple.xml analogue."""
    sc = Scene(max_depth=1, background=(0, 0, 0), ambient=(25, 25, 25))
    sc.cameras.append(_cam((0, 0, 0), (0, 0, -1), (0, 1, 0), nx, ny, fov_deg=60, name="simple.png"))
    sc.materials += [
        Material(ambient=(1, 1, 1), diffuse=(1, 0.2, 0.2), specular=(1, 1, 1), phong_exp=1),
        Material(ambient=(1, 1, 1), diffuse=(0.2, 1, 0.2), specular=(1, 1, 1), phong_exp=10),
        Material(ambient=(1, 1, 1), diffuse=(0.2, 0.2, 1), specular=(1, 1, 1), phong_exp=100),
        Material(ambient=(1, 1, 1), diffuse=(0.8, 0.8, 0.8), specular=(0, 0, 0), phong_exp=1),
    ]
    b = _add_vertices(sc, [(-0.875, 0.0, -2.0), (0.0, 0.0, -2.0), (0.875, 0.0, -2.0),
                           (-10, -0.5, 10), (10, -0.5, 10), (0, -0.5, -100)])
    for k in range(3):
        sc.objects.append(Object(type=A.OBJ_SPHERE, id=k + 1, material=k + 1, center=b + k, radius=0.3))
    sc.objects.append(Object(type=A.OBJ_TRIANGLE, id=1, material=4, v=(b + 3, b + 4, b + 5)))
    sc.lights.append(Light(type=A.LIGHT_POINT, position=(0, 4, 0), intensity=(1000, 1000, 1000)))
    return sc


def bgtex(nx=48, ny=32, spp=1, interp=A.INTERP_NN) -> Scene:
    """`simple` in front of a replace_background image texture (src/Scene.cpp:413-435): at 1 spp
    SingleSample passes (row = x, col = y), so the background is looked up transposed; at > 1
    spp it is not (src/Scene.cpp:365-411)."""
    sc = simple(nx, ny)
    sc.cameras[0].num_samples = spp
    sc.cameras[0].image_name = "bgtex.png"
    v, u = np.mgrid[0:12, 0:20].astype(f32)
    img = np.stack([u * 12.0, v * 20.0, ((u + v) % 3) * 100.0], -1).astype(f32)
    sc.textures.append(Texture(kind=A.TEX_IMAGE, decal=A.DECAL_REPLACE_BACKGROUND, interp=interp, normalizer=255,
                               bump_factor=1.0, texels=img, image_id=1))
    sc.images = ["bg.ppm"]
    sc.background_texture = len(sc.textures) - 1
    return sc


def bunny5k(nx=1920, ny=1080, level=4, spp=1) -> Scene:
    """C2: ~5K-tri displaced icosphere (flat), mirror floor, glass sphere, Whitted depth 6."""
    sc = Scene(max_depth=6, background=(10, 10, 20), ambient=(20, 20, 20))
    sc.cameras.append(_cam((0, 0.6, 3.2), (0, -0.15, -1), (0, 1, 0), nx, ny, fov_deg=50, spp=spp, name="bunny.png"))
    sc.materials += [
        Material(ambient=(1, 1, 1), diffuse=(0.8, 0.6, 0.4), specular=(0.5, 0.5, 0.5), phong_exp=20),
        Material(type=A.MAT_MIRROR, ambient=(0.1, 0.1, 0.1), diffuse=(0.2, 0.2, 0.2), specular=(0.2, 0.2, 0.2),
                 mirror=(0.6, 0.6, 0.6), phong_exp=10),
        Material(type=A.MAT_DIELECTRIC, ambient=(0, 0, 0), diffuse=(0, 0, 0), specular=(0, 0, 0),
                 refraction_index=1.5, absorption_coeff=(0.05, 0.1, 0.2)),
    ]
    v, f = icosphere(level)
    rng = np.random.default_rng(795)
    disp = 1.0 + 0.08 * _perlin3(v + 2.0, 7) + 0.01 * rng.standard_normal(len(v))
    v = v * disp[:, None] * 0.7
    b = _add_vertices(sc, v)
    b2 = _add_vertices(sc, [(-0.9, -0.2, 0.9), (0, 0, 0)])
    fl = _add_vertices(sc, [(-6, -0.75, 6), (6, -0.75, 6), (6, -0.75, -6), (-6, -0.75, -6)])
    sc.objects.append(Object(type=A.OBJ_SPHERE, id=1, material=3, center=b2, radius=0.35))
    sc.objects.append(Object(type=A.OBJ_MESH, id=1, material=1, faces=(f + b).astype(np.int32)))
    sc.objects.append(Object(type=A.OBJ_MESH, id=2, material=2,
                             faces=np.array([[fl, fl + 1, fl + 2], [fl, fl + 2, fl + 3]], np.int32)))
    sc.lights.append(Light(type=A.LIGHT_POINT, position=(2, 4, 3), intensity=(40000, 40000, 40000)))
    return sc


def dragon1m(nx=1920, ny=1080, spp=64, nu=1000, nv=500) -> Scene:
    """C3: 1,000,000-triangle BVH scene, mirror + dielectric spheres, recursive shading."""
    sc = Scene(max_depth=6, background=(15, 15, 30), ambient=(15, 15, 15))
    sc.cameras.append(_cam((0, 0.35, 3.6), (0, -0.08, -1), (0, 1, 0), nx, ny, fov_deg=45, spp=spp,
                           name="dragon.png"))
    sc.materials += [
        Material(ambient=(1, 1, 1), diffuse=(0.7, 0.55, 0.3), specular=(0.6, 0.6, 0.6), phong_exp=30),
        Material(type=A.MAT_MIRROR, ambient=(0.05, 0.05, 0.05), diffuse=(0.1, 0.1, 0.1),
                 specular=(0.3, 0.3, 0.3), mirror=(0.8, 0.8, 0.8), phong_exp=50),
        Material(type=A.MAT_DIELECTRIC, ambient=(0, 0, 0), diffuse=(0, 0, 0), specular=(0, 0, 0),
                 refraction_index=1.5, absorption_coeff=(0, 0, 0)),
        Material(ambient=(1, 1, 1), diffuse=(0.5, 0.5, 0.55), specular=(0, 0, 0), phong_exp=1),
    ]
    s = _add_vertices(sc, [(-1.7, -0.3, -0.3), (1.2, -0.55, 1.2)])
    fl = _add_vertices(sc, [(-20, -1.05, 20), (20, -1.05, 20), (20, -1.05, -20), (-20, -1.05, -20)])
    sc.objects.append(Object(type=A.OBJ_SPHERE, id=1, material=2, center=s, radius=0.7))
    sc.objects.append(Object(type=A.OBJ_SPHERE, id=2, material=3, center=s + 1, radius=0.45))
    sc.objects.append(Object(type=A.OBJ_MESH, id=2, material=4,
                             faces=np.array([[fl, fl + 1, fl + 2], [fl, fl + 2, fl + 3]], np.int32)))
    v, f = uv_sphere(nu, nv)
    b = _add_vertices(sc, v)
    sc.objects.append(Object(type=A.OBJ_MESH, id=1, material=1, faces=(f + b).astype(np.int32),
                             ply_file="dragon1m.ply",
                             texture_offset=len(sc.texcoords) + 1 - b))   # what Parser.h:1051, 1099-1102 derives
    sc.lights.append(Light(type=A.LIGHT_POINT, position=(3, 5, 4), intensity=(22000, 22000, 22000)))
    return sc


def cornell(nx=1920, ny=1080, spp=64, dof=True, level=2) -> Scene:
    """C4: cornell box walls mesh, two instances (resetTransform on/off), motion-blurred sphere,
    area light, depth-of-field camera."""
    sc = Scene(max_depth=4, background=(0, 0, 0), ambient=(10, 10, 10))
    cam = _cam((0, 5, 13.5), (0, 0, -1), (0, 1, 0), nx, ny, fov_deg=45, spp=spp, name="cornell.png")
    if dof:
        cam.is_dof, cam.focus_distance, cam.aperture_size = True, 13.0, 0.25
    sc.cameras.append(cam)
    sc.materials += [
        Material(ambient=(1, 1, 1), diffuse=(0.8, 0.8, 0.8), specular=(0, 0, 0), phong_exp=1),
        Material(ambient=(1, 1, 1), diffuse=(0.8, 0.1, 0.1), specular=(0, 0, 0), phong_exp=1),
        Material(ambient=(1, 1, 1), diffuse=(0.1, 0.8, 0.1), specular=(0, 0, 0), phong_exp=1),
        Material(type=A.MAT_MIRROR, ambient=(0.1, 0.1, 0.1), diffuse=(0.1, 0.1, 0.1), specular=(0.4, 0.4, 0.4),
                 mirror=(0.7, 0.7, 0.7), phong_exp=40, is_rough=True, roughness=0.08),
        Material(ambient=(1, 1, 1), diffuse=(0.3, 0.4, 0.9), specular=(0.6, 0.6, 0.6), phong_exp=60),
        Material(type=A.MAT_CONDUCTOR, ambient=(0.1, 0.1, 0.1), diffuse=(0.1, 0.1, 0.1),
                 specular=(0.5, 0.5, 0.5), mirror=(0.9, 0.7, 0.4), phong_exp=80, refraction_index=0.37,
                 absorption_index=2.82),
    ]
    w = _add_vertices(sc, [(-5, 0, 5), (5, 0, 5), (5, 0, -5), (-5, 0, -5),
                           (-5, 10, 5), (5, 10, 5), (5, 10, -5), (-5, 10, -5)])
    q = lambda a, b, c, d: [[a, b, c], [a, c, d]]
    walls_white = np.array(q(w, w + 1, w + 2, w + 3) + q(w + 4, w + 7, w + 6, w + 5) + q(w + 3, w + 2, w + 6, w + 7),
                           np.int32)
    red = np.array(q(w, w + 3, w + 7, w + 4), np.int32)
    green = np.array(q(w + 1, w + 5, w + 6, w + 2), np.int32)
    iv, ifc = icosphere(level)
    ib = _add_vertices(sc, iv)
    sph = _add_vertices(sc, [(2.2, 1.6, 1.5)])
    sc.translations += [(-2.2, 1.4, -1.5), (0.0, 1.0, 0.0), (1.5, 0.0, 2.0)]
    sc.scalings += [(1.4, 1.4, 1.4), (1.0, 1.6, 1.0)]
    sc.rotations += [(30.0, 0.0, 1.0, 0.0)]
    sc.objects.append(Object(type=A.OBJ_SPHERE, id=1, material=6, center=sph, radius=1.2, blur=(0.0, 0.8, 0.0)))
    sc.objects.append(Object(type=A.OBJ_MESH, id=1, material=1, faces=walls_white))
    sc.objects.append(Object(type=A.OBJ_MESH, id=2, material=2, faces=red))
    sc.objects.append(Object(type=A.OBJ_MESH, id=3, material=3, faces=green))
    sc.objects.append(Object(type=A.OBJ_MESH, id=4, material=5, faces=(ifc + ib).astype(np.int32), smooth=True,
                             xforms=[(A.XF_TRANSLATION, 1), (A.XF_SCALING, 1)]))
    sc.instances.append(Instance(base_object=4, id=5, material=4, reset_transform=False,
                                 xforms=[(A.XF_TRANSLATION, 3), (A.XF_ROTATION, 1)]))
    sc.instances.append(Instance(base_object=4, id=6, material=5, reset_transform=True,
                                 xforms=[(A.XF_TRANSLATION, 2), (A.XF_SCALING, 2)], blur=(0.3, 0.0, 0.0)))
    sc.lights.append(Light(type=A.LIGHT_AREA, position=(0, 9.9, 0), direction=(0, -1, 0),
                           intensity=(3000, 3000, 3000), size=2.5))
    return sc


def spheres(nx=1920, ny=1080, spp=64, n=1024, seed=3) -> Scene:
    """hw3 "Spheres DOF" analogue (pages/Page3.md:61) for the top-level BVH: `n` spheres, each its
    own object (the reference tests every object per ray, src/Helper.cpp:32-51), jittered on a
    ground quad; some transformed (scaling / translation / rotation), a few motion-blurred, two
    instances of a small mesh; diffuse, mirror, glass and conductor materials; DoF camera, point
    light, Whitted depth 3."""
    rng = np.random.default_rng(seed)
    sc = Scene(max_depth=3, background=(20, 30, 50), ambient=(12, 12, 12))
    cam = _cam((0, 3.0, 15.0), (0, -0.2, -1), (0, 1, 0), nx, ny, fov_deg=50, spp=spp, name="spheres.png")
    if spp > 1:
        cam.is_dof, cam.focus_distance, cam.aperture_size = True, 14.0, 0.3
    sc.cameras.append(cam)
    cols = [(0.8, 0.2, 0.2), (0.2, 0.7, 0.2), (0.2, 0.3, 0.85), (0.8, 0.7, 0.2), (0.7, 0.3, 0.7), (0.9, 0.9, 0.9)]
    for c in cols:
        sc.materials.append(Material(ambient=(1, 1, 1), diffuse=c, specular=(0.5, 0.5, 0.5), phong_exp=30))
    sc.materials.append(Material(type=A.MAT_MIRROR, ambient=(0.1, 0.1, 0.1), diffuse=(0.1, 0.1, 0.1),
                                 specular=(0.4, 0.4, 0.4), mirror=(0.8, 0.8, 0.8), phong_exp=60))
    sc.materials.append(Material(type=A.MAT_DIELECTRIC, ambient=(0, 0, 0), diffuse=(0, 0, 0), specular=(0, 0, 0),
                                 refraction_index=1.5, absorption_coeff=(0.05, 0.02, 0.01)))
    sc.materials.append(Material(type=A.MAT_CONDUCTOR, ambient=(0.1, 0.1, 0.1), diffuse=(0.1, 0.1, 0.1),
                                 specular=(0.5, 0.5, 0.5), mirror=(0.9, 0.7, 0.4), phong_exp=80,
                                 refraction_index=0.37, absorption_index=2.82))
    sc.materials.append(Material(ambient=(1, 1, 1), diffuse=(0.5, 0.5, 0.5), specular=(0, 0, 0), phong_exp=1))
    side = int(math.ceil(math.sqrt(n)))
    r = rng.uniform(0.2, 0.42, n).astype(f32)
    gx = (np.arange(n) % side).astype(f32)
    gz = (np.arange(n) // side).astype(f32)
    x = (gx - side / 2 + 0.5) * (32.0 / side) + rng.uniform(-0.2, 0.2, n)
    z = (gz - side / 2 + 0.5) * (32.0 / side) + rng.uniform(-0.2, 0.2, n) - 6.0
    y = -1.0 + r
    c = _add_vertices(sc, np.stack([x, y, z], -1))
    sc.translations += [(0.0, 0.3, 0.0), (0.4, 0.0, -0.3)]
    sc.scalings += [(1.0, 1.6, 1.0), (0.7, 0.7, 0.7)]
    sc.rotations += [(25.0, 0.0, 0.0, 1.0)]
    mats = rng.choice(len(sc.materials) - 1, n, p=[0.13] * 6 + [0.08, 0.08, 0.06]) + 1
    for k in range(n):
        xf = []
        if k % 11 == 3:
            xf = [(A.XF_TRANSLATION, 1), (A.XF_SCALING, 1)]
        elif k % 13 == 5:
            xf = [(A.XF_ROTATION, 1), (A.XF_SCALING, 2), (A.XF_TRANSLATION, 2)]
        blur = (0.0, 0.25, 0.0) if k % 37 == 7 else (0.0, 0.0, 0.0)
        sc.objects.append(Object(type=A.OBJ_SPHERE, id=k + 1, material=int(mats[k]), center=c + k, radius=float(r[k]),
                                 xforms=xf, blur=blur))
    fl = _add_vertices(sc, [(-40, -1.0, 40), (40, -1.0, 40), (40, -1.0, -40), (-40, -1.0, -40)])
    sc.objects.append(Object(type=A.OBJ_MESH, id=n + 1, material=len(sc.materials),
                             faces=np.array([[fl, fl + 1, fl + 2], [fl, fl + 2, fl + 3]], np.int32)))
    iv, ifc = icosphere(1)
    ib = _add_vertices(sc, iv * 0.6)
    sc.objects.append(Object(type=A.OBJ_MESH, id=n + 2, material=5, faces=(ifc + ib).astype(np.int32),
                             xforms=[(A.XF_TRANSLATION, 1)]))
    sc.translations += [(-3.0, 0.0, 2.0), (3.0, 0.2, 1.0)]
    base = len(sc.objects) - 1
    sc.instances.append(Instance(base_object=base, id=n + 3, material=7, reset_transform=False,
                                 xforms=[(A.XF_TRANSLATION, 3)]))
    sc.instances.append(Instance(base_object=base, id=n + 4, material=8, reset_transform=True,
                                 xforms=[(A.XF_TRANSLATION, 4), (A.XF_SCALING, 1)], blur=(0.2, 0.0, 0.0)))
    sc.lights.append(Light(type=A.LIGHT_POINT, position=(2, 12, 8), intensity=(60000, 60000, 60000)))
    return sc


PT_ALL = A.PT_IMPORTANCE | A.PT_NEE | A.PT_RUSSIAN_ROULETTE


def cornell_pt(nx=1920, ny=1080, spp=256, flags=PT_ALL, max_depth=6, light_sphere=True, level=2) -> Scene:
    """C5 (hw7 cornellbox path tracing, pages/Page7.md): cornell box with a ceiling LightMesh and a
    LightSphere, normalised-BRDF walls, a glossy instanced icosphere, glass and mirror spheres,
    path traced with `flags` (A.PT_*)."""
    sc = Scene(max_depth=max_depth, background=(0, 0, 0), ambient=(0, 0, 0))
    sc.cameras.append(_cam((0, 5, 13.5), (0, 0, -1), (0, 1, 0), nx, ny, fov_deg=45, spp=spp, name="cornell_pt.exr",
                           integrator=A.INTEGRATOR_PATH, pt_flags=flags))
    z3 = (0.0, 0.0, 0.0)
    sc.materials += [
        Material(brdf=A.BRDF_MBPN, phong_exp=1, ambient=z3, diffuse=(0.75, 0.75, 0.75), specular=z3),
        Material(brdf=A.BRDF_MBPN, phong_exp=1, ambient=z3, diffuse=(0.75, 0.1, 0.1), specular=z3),
        Material(brdf=A.BRDF_MBPN, phong_exp=1, ambient=z3, diffuse=(0.1, 0.75, 0.1), specular=z3),
        Material(brdf=A.BRDF_MBPN, phong_exp=40, ambient=z3, diffuse=(0.2, 0.3, 0.7), specular=(0.4, 0.4, 0.4)),
        Material(type=A.MAT_MIRROR, ambient=z3, diffuse=z3, specular=z3, mirror=(0.9, 0.9, 0.9)),
        Material(type=A.MAT_DIELECTRIC, ambient=z3, diffuse=z3, specular=z3, refraction_index=1.5,
                 absorption_coeff=(0.02, 0.05, 0.1)),
    ]
    w = _add_vertices(sc, [(-5, 0, 5), (5, 0, 5), (5, 0, -5), (-5, 0, -5),
                           (-5, 10, 5), (5, 10, 5), (5, 10, -5), (-5, 10, -5)])
    q = lambda a, b, c, d: [[a, b, c], [a, c, d]]
    walls_white = np.array(q(w, w + 1, w + 2, w + 3) + q(w + 4, w + 7, w + 6, w + 5) + q(w + 3, w + 2, w + 6, w + 7),
                           np.int32)
    red = np.array(q(w, w + 3, w + 7, w + 4), np.int32)
    green = np.array(q(w + 1, w + 5, w + 6, w + 2), np.int32)
    lq = _add_vertices(sc, [(-1.25, 9.98, 1.25), (1.25, 9.98, 1.25), (1.25, 9.98, -1.25), (-1.25, 9.98, -1.25)])
    iv, ifc = icosphere(level)
    ib = _add_vertices(sc, iv)
    sph = _add_vertices(sc, [(2.2, 1.3, 1.2), (-2.4, 1.5, 2.0), (-3.2, 8.2, -2.5)])
    sc.translations += [(-1.2, 1.4, -2.0)]
    sc.scalings += [(1.4, 1.4, 1.4)]
    sc.objects.append(Object(type=A.OBJ_SPHERE, id=1, material=6, center=sph, radius=1.3))
    sc.objects.append(Object(type=A.OBJ_SPHERE, id=2, material=5, center=sph + 1, radius=1.0))
    if light_sphere:
        sc.objects.append(Object(type=A.OBJ_SPHERE, id=3, material=1, center=sph + 2, radius=0.4, is_light=True,
                                 radiance=(160.0, 120.0, 80.0)))
    sc.objects.append(Object(type=A.OBJ_MESH, id=1, material=1, faces=walls_white))
    sc.objects.append(Object(type=A.OBJ_MESH, id=2, material=2, faces=red))
    sc.objects.append(Object(type=A.OBJ_MESH, id=3, material=3, faces=green))
    sc.objects.append(Object(type=A.OBJ_MESH, id=4, material=4, faces=(ifc + ib).astype(np.int32), smooth=True,
                             xforms=[(A.XF_TRANSLATION, 1), (A.XF_SCALING, 1)]))
    sc.objects.append(Object(type=A.OBJ_MESH, id=5, material=1, faces=np.array(q(lq + 3, lq + 2, lq + 1, lq), np.int32),
                             is_light=True, radiance=(600.0, 560.0, 500.0)))
    return sc


def furnace(nx=8, ny=6, spp=64, flags=A.PT_IMPORTANCE, kd=0.6, Le=(10.0, 20.0, 40.0), radius=50.0) -> Scene:
    """Analytic case: a convex diffuse sphere (normalised Lambertian kd/pi) inside a LightSphere of
    radiance Le.  Every visible point sees only the light, so its radiance is exactly kd * Le."""
    sc = Scene(max_depth=1, background=(0, 0, 0), ambient=(0, 0, 0))
    sc.cameras.append(_cam((0, 0, 4), (0, 0, -1), (0, 1, 0), nx, ny, fov_deg=20, spp=spp, name="furnace.exr",
                           integrator=A.INTEGRATOR_PATH, pt_flags=flags))
    sc.materials.append(Material(brdf=A.BRDF_MBPN, phong_exp=1, ambient=(0, 0, 0), diffuse=(kd, kd, kd),
                                 specular=(0, 0, 0)))
    c = _add_vertices(sc, [(0, 0, 0)])
    sc.objects.append(Object(type=A.OBJ_SPHERE, id=1, material=1, center=c, radius=1.0))
    sc.objects.append(Object(type=A.OBJ_SPHERE, id=2, material=1, center=c, radius=radius, is_light=True,
                             radiance=Le))
    return sc


def checker_texture(n=64, c0=(230, 230, 230), c1=(40, 60, 160)) -> np.ndarray:
    i = np.arange(n)
    m = ((i[:, None] // 8) + (i[None, :] // 8)) % 2
    img = np.where(m[..., None] == 0, np.array(c0, f32), np.array(c1, f32)).astype(f32)
    grad = (np.linspace(0, 60, n)[None, :, None]).astype(f32)
    return np.clip(img + grad, 0, 255).astype(np.uint8).astype(f32)


def textured(nx=96, ny=72, spp=1) -> Scene:
    """Feature scene: image/Perlin textures (replace_kd, blend_kd, bump, replace_normal,
    replace_all), spot + directional lights and the BRDF models."""
    sc = Scene(max_depth=2, background=(5, 5, 5), ambient=(20, 20, 20))
    sc.cameras.append(_cam((0, 1.2, 5), (0, -0.2, -1), (0, 1, 0), nx, ny, fov_deg=55, spp=spp, name="tex.png"))
    tex = checker_texture()
    for decal, interp in ((A.DECAL_REPLACE_KD, A.INTERP_NN), (A.DECAL_BLEND_KD, A.INTERP_BILINEAR),
                          (A.DECAL_BUMP_NORMAL, A.INTERP_BILINEAR), (A.DECAL_REPLACE_NORMAL, A.INTERP_NN),
                          (A.DECAL_REPLACE_ALL, A.INTERP_BILINEAR)):
        sc.textures.append(Texture(kind=A.TEX_IMAGE, decal=decal, interp=interp, normalizer=255,
                                   bump_factor=2.0, texels=tex, image_id=1))
    sc.textures.append(Texture(kind=A.TEX_PERLIN, decal=A.DECAL_REPLACE_KD, noise_conv=A.NC_ABSVAL, noise_scale=3.0))
    sc.textures.append(Texture(kind=A.TEX_PERLIN, decal=A.DECAL_BUMP_NORMAL, noise_conv=A.NC_LINEAR,
                               noise_scale=5.0, bump_factor=0.5))
    brdfs = [A.BRDF_NONE, A.BRDF_MBP, A.BRDF_MBPN, A.BRDF_OBP, A.BRDF_MP, A.BRDF_MPN, A.BRDF_OP, A.BRDF_TS,
             A.BRDF_TSF]
    for k, br in enumerate(brdfs):
        sc.materials.append(Material(ambient=(0.5, 0.5, 0.5), diffuse=(0.6, 0.5 + 0.05 * k, 0.4),
                                     specular=(0.7, 0.7, 0.7), phong_exp=20 + 5 * k, brdf=br,
                                     refraction_index=1.8, absorption_index=0.5))
    centers = [(-2.4, 0.5, -1), (-1.2, 0.5, -1), (0, 0.5, -1), (1.2, 0.5, -1), (2.4, 0.5, -1),
               (-1.8, 0.5, 0.4), (-0.6, 0.5, 0.4), (0.6, 0.5, 0.4), (1.8, 0.5, 0.4)]
    c0 = _add_vertices(sc, centers)
    texsets = [[1], [2], [3], [4], [5], [6], [7], [1, 7], []]
    for k in range(9):
        sc.objects.append(Object(type=A.OBJ_SPHERE, id=k + 1, material=k + 1, center=c0 + k, radius=0.5,
                                 textures=texsets[k]))
    fl = _add_vertices(sc, [(-4, 0, 3), (4, 0, 3), (4, 0, -4), (-4, 0, -4)])
    sc.texcoords = np.array([(0, 0), (3, 0), (3, 3), (0, 3)], f32)
    sc.objects.append(Object(type=A.OBJ_MESH, id=1, material=1, textures=[2, 3],
                             faces=np.array([[fl, fl + 1, fl + 2], [fl, fl + 2, fl + 3]], np.int32),
                             texture_offset=-(fl - 1)))
    sc.images = ["checker.ppm"]
    sc.lights.append(Light(type=A.LIGHT_POINT, position=(0, 5, 3), intensity=(20000, 20000, 20000)))
    sc.lights.append(Light(type=A.LIGHT_DIRECTIONAL, direction=(-0.3, -1, -0.4), intensity=(1.5, 1.5, 1.5)))
    sc.lights.append(Light(type=A.LIGHT_SPOT, position=(-3, 4, 2), direction=(0.6, -1, -0.6),
                           intensity=(30000, 20000, 20000), coverage_deg=50, falloff_deg=25))
    return sc


def multilight(nx=320, ny=240, spp=1) -> Scene:
    """Untextured scene with several light kinds (point, directional, two spots) and every
    material type (rough mirror, conductor, dielectric): exercises the untextured shading
    variant with spot lights and the in-order multi-light sum."""
    sc = Scene(max_depth=4, background=(5, 5, 12), ambient=(12, 12, 12))
    sc.cameras.append(_cam((0, 1.6, 6.0), (0, -0.2, -1), (0, 1, 0), nx, ny, fov_deg=50, spp=spp,
                           name="multilight.png"))
    sc.materials += [
        Material(ambient=(1, 1, 1), diffuse=(0.7, 0.7, 0.7), specular=(0.2, 0.2, 0.2), phong_exp=8),
        Material(type=A.MAT_MIRROR, ambient=(0.05, 0.05, 0.05), diffuse=(0.1, 0.1, 0.1),
                 specular=(0.4, 0.4, 0.4), mirror=(0.7, 0.7, 0.7), phong_exp=40, is_rough=True, roughness=0.1),
        Material(type=A.MAT_CONDUCTOR, ambient=(0.1, 0.1, 0.1), diffuse=(0.1, 0.1, 0.1),
                 specular=(0.5, 0.5, 0.5), mirror=(0.9, 0.6, 0.3), phong_exp=70, refraction_index=0.27,
                 absorption_index=2.77),
        Material(type=A.MAT_DIELECTRIC, ambient=(0, 0, 0), diffuse=(0, 0, 0), specular=(0, 0, 0),
                 refraction_index=1.45, absorption_coeff=(0.1, 0.05, 0.02)),
        Material(ambient=(1, 1, 1), diffuse=(0.3, 0.5, 0.8), specular=(0.8, 0.8, 0.8), phong_exp=120),
    ]
    c = _add_vertices(sc, [(-1.6, 0.6, -0.5), (0.0, 0.6, -1.2), (1.6, 0.6, -0.5), (0.6, 0.35, 1.0)])
    for k, mat in enumerate([2, 3, 4, 5]):
        sc.objects.append(Object(type=A.OBJ_SPHERE, id=k + 1, material=mat, center=c + k,
                                 radius=0.6 if k < 3 else 0.35))
    fl = _add_vertices(sc, [(-6, 0, 6), (6, 0, 6), (6, 0, -6), (-6, 0, -6)])
    sc.objects.append(Object(type=A.OBJ_MESH, id=1, material=1,
                             faces=np.array([[fl, fl + 1, fl + 2], [fl, fl + 2, fl + 3]], np.int32)))
    v, f = icosphere(2)
    b = _add_vertices(sc, v * 0.45 + np.array([-0.7, 0.45, 1.3], f32))
    sc.objects.append(Object(type=A.OBJ_MESH, id=2, material=5, faces=(f + b).astype(np.int32), smooth=True))
    sc.lights.append(Light(type=A.LIGHT_POINT, position=(2, 5, 4), intensity=(9000, 9000, 9000)))
    sc.lights.append(Light(type=A.LIGHT_DIRECTIONAL, direction=(0.4, -1, -0.3), intensity=(0.8, 0.8, 0.9)))
    sc.lights.append(Light(type=A.LIGHT_SPOT, position=(-3, 4, 2), direction=(0.6, -1, -0.5),
                           intensity=(20000, 15000, 12000), coverage_deg=40, falloff_deg=20))
    sc.lights.append(Light(type=A.LIGHT_SPOT, position=(3, 3, -2), direction=(-0.7, -1, 0.4),
                           intensity=(8000, 12000, 16000), coverage_deg=60, falloff_deg=45))
    return sc


def glass_nest(nx=64, ny=48, spp=1, max_depth=6) -> Scene:
    """Camera inside two concentric dielectric spheres inside a mirror sphere, with a point light in
    the gap: every ray hits something and every dielectric hit spawns two children, so the ray
    count roughly doubles per level (the device-driven level loop's overflow case)."""
    sc = Scene(max_depth=max_depth, background=(20, 20, 30), ambient=(10, 10, 10))
    sc.cameras.append(_cam((0, 0, 0), (0, 0, -1), (0, 1, 0), nx, ny, fov_deg=60, spp=spp, name="glass_nest.png"))
    sc.materials += [
        Material(type=A.MAT_DIELECTRIC, ambient=(0, 0, 0), diffuse=(0, 0, 0), specular=(0, 0, 0),
                 refraction_index=1.5, absorption_coeff=(0.01, 0.02, 0.03)),
        Material(type=A.MAT_MIRROR, ambient=(0.2, 0.2, 0.2), diffuse=(0.3, 0.3, 0.3), specular=(0.2, 0.2, 0.2),
                 mirror=(0.6, 0.6, 0.6), phong_exp=20),
    ]
    c = _add_vertices(sc, [(0, 0, 0)])
    sc.objects.append(Object(type=A.OBJ_SPHERE, id=1, material=1, center=c, radius=2.0))
    sc.objects.append(Object(type=A.OBJ_SPHERE, id=2, material=1, center=c, radius=4.0))
    sc.objects.append(Object(type=A.OBJ_SPHERE, id=3, material=2, center=c, radius=8.0))
    sc.lights.append(Light(type=A.LIGHT_POINT, position=(1.0, 5.5, 1.0), intensity=(400, 400, 400)))
    return sc


def sky_texture(w=64, h=32, sun=(0.3, 0.28), sun_radiance=40.0) -> np.ndarray:
    """Linear HDR latitude-longitude sky (what an .exr environment map decodes to): a
    horizon-to-zenith gradient, a dark ground half and a small bright sun disc.  Values are
    rounded through float16 so that an OpenEXR HALF file round-trips them exactly."""
    v, u = np.mgrid[0:h, 0:w].astype(f32)
    v = (v + 0.5) / h
    u = (u + 0.5) / w
    up = np.clip(1.0 - 2.0 * v, 0.0, 1.0)[..., None]
    sky = (np.array([0.9, 1.0, 1.1], f32) * (1 - up) + np.array([0.25, 0.45, 1.0], f32) * up) * 1.5
    ground = np.array([0.18, 0.15, 0.12], f32) * np.ones_like(sky)
    img = np.where((v < 0.5)[..., None], sky, ground)
    du = np.minimum(np.abs(u - sun[0]), 1 - np.abs(u - sun[0]))
    d2 = (du * 2) ** 2 + (v - sun[1]) ** 2
    img = img + (d2 < 0.004)[..., None] * np.array([1.0, 0.9, 0.7], f32) * sun_radiance
    return img.astype(np.float16).astype(f32)


def envmap(nx=96, ny=72, spp=4, max_depth=3) -> Scene:
    """hw6 image-based lighting: a SphericalDirectionalLight (src/Light.cpp:551-660) over an
    HDR sky (`sky_texture`, written as `sky.exr` by tests) lighting diffuse, Blinn-Phong,
    BRDF, mirror and dielectric objects; primary misses show the environment map
    (src/Scene.cpp:413-435)."""
    sc = Scene(max_depth=max_depth, background=(0, 0, 0), ambient=(0, 0, 0))
    sc.cameras.append(_cam((0, 1.3, 5.5), (0, -0.15, -1), (0, 1, 0), nx, ny, fov_deg=55, spp=spp,
                           name="env.exr"))
    sc.materials += [
        Material(ambient=(0, 0, 0), diffuse=(0.6, 0.6, 0.6), specular=(0, 0, 0), phong_exp=1),
        Material(ambient=(0, 0, 0), diffuse=(0.7, 0.3, 0.2), specular=(0.4, 0.4, 0.4), phong_exp=30),
        Material(type=A.MAT_MIRROR, ambient=(0, 0, 0), diffuse=(0.05, 0.05, 0.05), specular=(0, 0, 0),
                 mirror=(0.85, 0.85, 0.85), phong_exp=1),
        Material(type=A.MAT_DIELECTRIC, ambient=(0, 0, 0), diffuse=(0, 0, 0), specular=(0, 0, 0),
                 refraction_index=1.5, absorption_coeff=(0.05, 0.02, 0.01)),
        Material(ambient=(0, 0, 0), diffuse=(0.3, 0.5, 0.7), specular=(0.5, 0.5, 0.5), phong_exp=50,
                 brdf=A.BRDF_MBPN),
    ]
    c = _add_vertices(sc, [(-1.7, 0.6, -0.6), (0.0, 0.6, -1.2), (1.7, 0.6, -0.6), (0.8, 0.4, 0.9)])
    for k, mat in enumerate([2, 3, 4, 5]):
        sc.objects.append(Object(type=A.OBJ_SPHERE, id=k + 1, material=mat, center=c + k,
                                 radius=0.6 if k < 3 else 0.4))
    fl = _add_vertices(sc, [(-5, 0, 5), (5, 0, 5), (5, 0, -5), (-5, 0, -5)])
    sc.objects.append(Object(type=A.OBJ_MESH, id=1, material=1,
                             faces=np.array([[fl, fl + 1, fl + 2], [fl, fl + 2, fl + 3]], np.int32)))
    sc.images = ["sky.exr"]
    sc.textures.append(Texture(kind=A.TEX_IMAGE, decal=A.DECAL_NONE, interp=A.INTERP_BILINEAR, normalizer=1,
                               bump_factor=1.0, texels=sky_texture(), image_id=1))
    sc.environment_light = len(sc.lights)
    sc.lights.append(Light(type=A.LIGHT_ENVIRONMENT, texture=len(sc.textures) - 1, image_id=1))
    return sc


CONFIGS = {
    "simple": simple,
    "bunny5k": bunny5k,
    "dragon1m": dragon1m,
    "cornell_dynamic": cornell,
    "cornell_pt": cornell_pt,
    "textured": textured,
    "multilight": multilight,
    "envmap": envmap,
}
