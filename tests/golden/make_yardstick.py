"""SURVEY §8(d) yardstick per bench workload -> tests/golden/yardstick.json.

The algorithmic bytes per ray that bench.py's `roofline.model` prices,
    B = 64 + 32 N_node + 36 N_tri + 16 N_sphere,
with N_node / N_tri / N_sphere the mean child records read and primitive tests of the
CANONICAL ordered early-exit traversal over the reference's own median-split trees
(oracle/rtg_oracle.c canon_count: closest hit for primary + secondary rays, first hit up to
the light for shadow rays), measured by the CPU restatement on a fixed row sample of the
bench frame.  Fixed per workload: it does not move when the GPU's traversal changes.

usage: python tests/golden/make_yardstick.py [workload ...]     (about a minute on 8 cores)
"""
from __future__ import annotations

import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "raytracer-795_amd"), os.path.join(ROOT, "oracle")]

import pyoracle  # noqa: E402
from rtg import scenegen  # noqa: E402

OUT = os.path.join(HERE, "yardstick.json")
# workload -> (scenegen factory, spp, row stride of the sample, row offset)
WORKLOADS = {
    "dragon1m": ("dragon1m", 64, 54, 27),
    "bunny": ("bunny5k", 1, 4, 2),
    "cornell": ("cornell", 64, 54, 27),
    "cornell_pt": ("cornell_pt", 256, 108, 54),
    "spheres": ("spheres", 64, 540, 270),
}
NODE_B, TRI_B, SPH_B, RAY_B = 32, 36, 16, 64


def bytes_per_ray(n_node, n_tri, n_sph):
    return RAY_B + NODE_B * n_node + TRI_B * n_tri + SPH_B * n_sph


def measure(name: str) -> dict:
    make, spp, stride, off = WORKLOADS[name]
    sc = getattr(scenegen, make)(1920, 1080, spp=spp)
    o = pyoracle.Oracle(sc)
    o.canonical_counts(True)
    t0 = time.time()
    o.render(0, row_stride=stride, row_offset=off)
    dt = time.time() - t0
    c = o.canonical_counts(False)
    o.close()
    out = {"sample": f"rows y % {stride} == {off} of the 1920x1080x{spp} frame", "seconds": round(dt, 1)}
    for pre, k in (("", "rays"), ("shadow_", "shadow_rays")):
        n = max(c[k], 1)
        nn, nt, ns = c[pre + "nodes"] / n, c[pre + "tris"] / n, c[pre + "spheres"] / n
        out.update({pre + "rays": c[k], pre + "n_node": round(nn, 4), pre + "n_tri": round(nt, 4),
                    pre + "n_sphere": round(ns, 4), pre + "bytes_per_ray": round(bytes_per_ray(nn, nt, ns), 2)})
    return out


def main():
    names = sys.argv[1:] or list(WORKLOADS)
    data = json.load(open(OUT)) if os.path.exists(OUT) else {}
    data["_model"] = ("B = 64 + 32 N_node + 36 N_tri + 16 N_sphere bytes per ray (SURVEY §8(d)); N_* = mean child "
                      "records / primitive tests of the canonical ordered early-exit traversal on the reference's "
                      "median-split trees (oracle canon_count), shadow rays: first hit up to the light")
    for n in names:
        data[n] = measure(n)
        print(n, data[n], flush=True)
    json.dump(data, open(OUT, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
