"""Regenerate tests/golden/ (run from the repo root: python tests/golden/make_golden.py).

The reference ships no fixtures and cannot be built here (Eigen / glm are
absent), so these files are of two kinds, kept apart:

* known_answers.json — answers that do not come from this repository: Random123's published
  Philox4x32-10 vectors, and analytic ray/primitive intersections evaluated in float64
  (checked against the oracle and the GPU with a stated tolerance);
* oracle_regression.npz — bit-exact outputs of the CPU restatement (oracle/) on small seeded
  scenes: a drift guard for the restatement (tests/test_golden.py) and a fixed target the GPU
  must hit (tests/test_golden.py::test_gpu_matches_golden), NOT reference outputs.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "raytracer-795_amd"), os.path.join(ROOT, "oracle")]

import pyoracle  # noqa: E402
from rtg import scenegen  # noqa: E402

# small, fast scenes covering every integrator feature; names are the fixture keys
SCENES = {
    "simple": lambda: scenegen.simple(24, 24),
    "bunny": lambda: scenegen.bunny5k(20, 15, level=2),
    "cornell_dof": lambda: scenegen.cornell(16, 12, spp=4),
    "textured": lambda: scenegen.textured(20, 15),
    "multilight": lambda: scenegen.multilight(20, 15, spp=2),
    "dragon_small": lambda: scenegen.dragon1m(16, 9, spp=2, nu=40, nv=20),
    "cornell_pt": lambda: scenegen.cornell_pt(12, 9, spp=3),
    "furnace_pt": lambda: scenegen.furnace(8, 6, spp=4),
    "envmap": lambda: scenegen.envmap(16, 12, spp=2),
    "bgtex_1spp": lambda: scenegen.bgtex(16, 12, spp=1),
    "bgtex_ms": lambda: scenegen.bgtex(16, 12, spp=2, interp=1),
}
SEED = 0x5EED2026
TRACE_SCENES = ["simple", "bunny", "cornell_dof", "dragon_small"]


def trace_rays(sc, n=256, seed=11):
    rng = np.random.default_rng(seed)
    lo = np.asarray(sc.vertices).min(0) - 1
    hi = np.asarray(sc.vertices).max(0) + 1
    o = rng.uniform(lo, hi, (n, 3)).astype(np.float32)
    d = rng.standard_normal((n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    t = rng.random(n).astype(np.float32)
    return o, d, t


def known_answers():
    philox = [  # Random123 kat_vectors, philox4x32 10 rounds
        {"ctr": [0, 0, 0, 0], "key": [0, 0], "out": [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]},
        {"ctr": [0xFFFFFFFF] * 4, "key": [0xFFFFFFFF] * 2, "out": [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]},
        {"ctr": [0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], "key": [0xA4093822, 0x299F31D0],
         "out": [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]},
    ]
    # unit sphere at the origin hit from (0,0,5) towards -z etc.: t = |o| - 1, n = hit point
    spheres = []
    for o, d in (((0, 0, 5), (0, 0, -1)), ((3, 4, 0), (-0.6, -0.8, 0)), ((0.3, -0.2, 4), (0, 0, -1))):
        o, d = np.array(o, float), np.array(d, float)
        b = d @ o
        t = -b - np.sqrt(b * b - (o @ o - 1.0))
        p = o + t * d
        spheres.append({"origin": o.tolist(), "direction": d.tolist(), "t": t, "point": p.tolist(), "normal": p.tolist()})
    return {"philox4x32_10": philox, "unit_sphere_hits": spheres}


def main():
    with open(os.path.join(HERE, "known_answers.json"), "w") as f:
        json.dump(known_answers(), f, indent=1)
    out = {}
    for name, make in SCENES.items():
        sc = make()
        orc = pyoracle.Oracle(sc)
        rgb, obj, prim, t = orc.render(0, seed=SEED)
        out[f"{name}/rgb"] = rgb
        out[f"{name}/prim_obj"] = obj
        c = orc.ray_counts()
        out[f"{name}/ray_counts"] = np.array([c["primary"], c["secondary"], c["shadow"]], np.int64)
        if name in TRACE_SCENES:
            o, d, tt = trace_rays(sc)
            h = orc.trace(o, d, tt)
            for k in ("full", "object", "prim", "material", "t", "point", "normal"):
                out[f"{name}/trace_{k}"] = h[k]
        orc.close()
    np.savez_compressed(os.path.join(HERE, "oracle_regression.npz"), **out)
    print("wrote", sorted({k.split("/")[0] for k in out}))


if __name__ == "__main__":
    main()
