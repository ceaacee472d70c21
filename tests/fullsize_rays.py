"""Ray sets for the full-size parity tests (tests/test_gpu_fullsize.py): rays of the kinds the
render loop traces on the BASELINE headline scene (C3 dragon1m, 1,000,002 triangles + 2 spheres), built from
the scene's own camera, light and the oracle's hit records:

  camera     pixel centres + jitter of the 1920x1080 camera (Camera::getPrimaryRay /
             getSampleRay, src/Camera.cpp:63-113: m = pos + gaze*dist + u*right + v*up)
  reflected  MirrorReflectance origins / directions from primary hits (src/Scene.cpp:32-55)
  refracted  DielectricRefraction (src/Scene.cpp:57-118) from primary hits: eta 1.5, origin p - n*eps
  shadow     toward the point light from p + n*eps (PointLight::IsShadow, src/Light.cpp:188-204)
  grazing    nearly tangent to the surface at a hit point
  tiny       camera rays with one direction component 0, denormal or tiny: the exact-division
             slab test (src/BVH.cpp:224-233) and Ray::gett's fall-through (src/Ray.cpp:21-36)

Hit records come from the oracle (test infrastructure), so these rays are inputs, not results.
"""
from __future__ import annotations

import numpy as np

f32 = np.float32


def _norm(v):
    return (v / np.linalg.norm(v, axis=-1, keepdims=True)).astype(f32)


def camera_rays(cam, n: int, rng) -> tuple[np.ndarray, np.ndarray]:
    pos = np.asarray(cam.position, np.float64)
    gaze = _norm(np.asarray(cam.gaze, np.float64)).astype(np.float64)
    up = np.asarray(cam.up, np.float64)
    w = -gaze
    right = np.cross(up, w)
    right /= np.linalg.norm(right)
    upv = np.cross(w, right)
    l, r, b, t = cam.near_plane
    col = rng.integers(0, cam.nx, n) + rng.random(n)
    row = rng.integers(0, cam.ny, n) + rng.random(n)
    u = l + (r - l) * col / cam.nx
    v = t - (t - b) * row / cam.ny
    m = pos + gaze * cam.near_distance + u[:, None] * right + v[:, None] * upv
    return np.repeat(pos[None].astype(f32), n, 0), _norm(m - pos)


def build(scene, oracle, n_camera: int = 40000, seed: int = 2026) -> dict[str, tuple[np.ndarray, np.ndarray]]:
    """Returns {kind: (origins, directions)}; about 2.6 rays per camera ray in total."""
    rng = np.random.default_rng(seed)
    cam = scene.cameras[0]
    eps = f32(scene.shadow_eps)
    o_cam, d_cam = camera_rays(cam, n_camera, rng)
    h = oracle.trace(o_cam, d_cam)
    hit = h["full"] == 1
    p = h["point"][hit].astype(f32)
    nrm = h["normal"][hit].astype(f32)
    d_in = d_cam[hit]
    out = {"camera": (o_cam, d_cam)}
    # MirrorReflectance: wr = -wo + n*2*(n.wo), origin p + n*eps
    wo = -d_in
    wr = _norm(-wo + nrm * 2 * np.sum(nrm * wo, 1, keepdims=True))
    out["reflected"] = ((p + nrm * eps).astype(f32), wr)
    # refraction into / out of an eta = 1.5 medium (the sign of d.n picks the side)
    dn = np.sum(d_in * nrm, 1, keepdims=True)
    nn = np.where(dn < 0, nrm, -nrm)
    eta = np.where(dn < 0, 1 / 1.5, 1.5)
    cos_t = -np.sum(d_in * nn, 1, keepdims=True)
    k = 1 - eta ** 2 * (1 - cos_t ** 2)
    ok = (k >= 0)[:, 0]
    td = _norm((d_in + nn * cos_t) * eta - nn * np.sqrt(np.maximum(k, 0)))
    out["refracted"] = ((p - nn * eps).astype(f32)[ok], td[ok])
    # shadow rays toward the first point light
    L = np.asarray(scene.lights[0].position, f32)
    out["shadow"] = ((p + nrm * eps).astype(f32), _norm(L[None] - p))
    # grazing: a tangent direction tilted 1e-3 off the surface, from just above it
    tang = _norm(np.cross(nrm, rng.standard_normal(nrm.shape)))
    gsel = rng.random(len(p)) < 0.5
    out["grazing"] = ((p + nrm * f32(1e-3)).astype(f32)[gsel], _norm(tang + nrm * f32(1e-3))[gsel])
    # tiny / zero / denormal direction components on camera rays
    m = n_camera // 4
    dt = d_cam[:m].copy()
    which = rng.integers(0, 3, m)
    vals = np.array([0.0, -0.0, 1e-38, -1e-40, 1e-31, 3e-30], f32)[rng.integers(0, 6, m)]
    dt[np.arange(m), which] = vals
    out["tiny"] = (o_cam[:m].copy(), dt.astype(f32))
    return out
