"""Rebuild the spheres frame's rays of one image row level by level (camera rays with DoF,
mirror / refraction children, shadow rays) in float32 numpy and trace them with the TLAS on and
off; print every ray whose hit record differs, and the oracle's answer for it."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "raytracer-795_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pyoracle  # noqa: E402
import rtg  # noqa: E402
from rtg import scenegen  # noqa: E402

f32 = np.float32
row = int(sys.argv[1]) if len(sys.argv) > 1 else 519
spp = 64
sc = scenegen.spheres(1920, 1080, spp=spp)
cam = sc.cameras[0]
nx, ny = cam.nx, cam.ny


def nrm(v):
    n = np.sqrt(v[:, 0] * v[:, 0] + (v[:, 1] * v[:, 1] + v[:, 2] * v[:, 2]))
    return v / n[:, None]


def cross(a, b):
    return np.stack([a[..., 1] * b[..., 2] - a[..., 2] * b[..., 1], a[..., 2] * b[..., 0] - a[..., 0] * b[..., 2],
                     a[..., 0] * b[..., 1] - a[..., 1] * b[..., 0]], -1).astype(f32)


def dot(a, b):
    return a[:, 0] * b[:, 0] + (a[:, 1] * b[:, 1] + a[:, 2] * b[:, 2])


pos = np.asarray(cam.position, f32)
gz = np.asarray(cam.gaze, f32)[None]
up = np.asarray(cam.up, f32)[None]
g = nrm(gz)[0]
w = nrm(-gz)[0]
right = nrm(cross(up[0], w)[None])[0]
up2 = cross(w, right)
l, r_, b_, t_ = (f32(v) for v in cam.near_plane)
dist = f32(cam.near_distance)
nxDA, nyDA = f32(1.0) / f32(nx), f32(1.0) / f32(ny)
pw, ph = (r_ - l) * nxDA, (t_ - b_) * nyDA
sc_n = 1
while sc_n * sc_n < spp:
    sc_n += 1
sw, sh = pw / f32(sc_n), ph / f32(sc_n)
xs = np.repeat(np.arange(nx), spp)
ss = np.tile(np.arange(spp), nx)
pix = (row * nx + xs).astype(np.uint32)
seed = 0x5EED2026
xi = np.zeros((len(xs), 4), f32)
for k in range(len(xs)):
    for lane in range(4):
        xi[k, lane] = pyoracle.rng_uniform(seed, int(pix[k]), int(ss[k]), 1, 1, 0, 0, lane)
u = l + xs.astype(f32) * pw
v = t_ - f32(row + 1) * ph
m = pos + g * dist
m = m + right[None] * u[:, None]
m = m + up2[None] * v
ii = (ss % sc_n).astype(f32)
jj = (ss // sc_n).astype(f32)
m = m + right[None] * ((ii + xi[:, 0]) * sw)[:, None]
m = m + up2[None] * ((jj + xi[:, 1]) * sh)[:, None]
d = nrm(m - pos)
xa, xb = xi[:, 2] - f32(0.5), xi[:, 3] - f32(0.5)
ap = f32(cam.aperture_size)
q = pos + right[None] * (ap * xa)[:, None]
q = q + up2[None] * (ap * xb)[:, None]
dr = nrm(m - pos)
tfd = f32(cam.focus_distance) / dot(dr, np.broadcast_to(g, dr.shape))
p = pos + d * tfd[:, None]
o = q.astype(f32)
d = nrm(p - q)
tm = np.zeros(len(o), f32)

ron = rtg.Renderer(sc, device=0, tlas=2)
roff = rtg.Renderer(sc, device=0, tlas=1)
orc = pyoracle.Oracle(sc)
eps = f32(sc.shadow_eps)
light = np.asarray(sc.lights[0].position, f32)
mats = sc.materials


def compare(tag, o, d, t):
    a = roff.trace(o, d, t)
    b = ron.trace(o, d, t)
    bad = np.nonzero((a["object"] != b["object"]) | (a["prim"] != b["prim"]) |
                     (a["t"].view(np.int32) != b["t"].view(np.int32)))[0]
    print(tag, len(o), "rays, differing:", len(bad), flush=True)
    if len(bad):
        ref = orc.trace(o[bad], d[bad], t[bad])
        for j, k in enumerate(bad[:10]):
            print("  ray", k, "o", o[k].tolist(), "d", d[k].tolist(), "linear", a["object"][k], a["t"][k],
                  "tlas", b["object"][k], b["t"][k], "oracle", ref["object"][j], ref["t"][j], flush=True)
    return a


level = 0
while len(o) and level < 4:
    h = compare(f"level {level}", o, d, tm)
    full = h["full"] == 1
    P = h["point"].astype(f32)
    N = h["normal"].astype(f32)
    sh_o = (P + N * eps)[full]
    Ld = light[None] - P[full]
    sh_d = nrm(Ld)
    compare(f"shadow {level}", sh_o, sh_d, tm[full])
    co, cd, ct = [], [], []
    for k in np.nonzero(full)[0]:
        mt = mats[h["material"][k] - 1]
        if mt.type == 0:
            continue
        n = N[k][None]
        dd = d[k][None]
        wo = -dd
        nwo = dot(n, wo)
        wr = nrm(-wo + (n * f32(2)) * nwo[:, None])
        co.append((P[k][None] + n * eps)[0]); cd.append(wr[0]); ct.append(tm[k])
        if mt.type == 3:
            dp = dot(dd, n)[0]
            nt = f32(mt.refraction_index)
            if dp < 0:
                snell, nn = f32(1.0) / nt, n
            else:
                snell, nn = nt, -n
            cos_t = -dot(dd, nn)
            left = (dd + nn * cos_t[:, None]) * snell
            srp = f32(1 - np.float64(snell) ** 2 * (1 - np.float64(cos_t[0]) ** 2))
            if srp >= 0:
                tdir = nrm(left - nn * np.sqrt(srp))
                co.append((P[k][None] - nn * eps)[0]); cd.append(tdir[0]); ct.append(tm[k])
    o = np.asarray(co, f32).reshape(-1, 3)
    d = np.asarray(cd, f32).reshape(-1, 3)
    tm = np.asarray(ct, f32)
    level += 1
