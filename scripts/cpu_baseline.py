"""CPU restatement (oracle/rtg_oracle.c, literal visit-both-children BVH) timed on a centred row
sample of each bench workload's full frame -- BASELINE.md §3's CPU column.  Runs on any host (no
GPU): `python scripts/cpu_baseline.py [--threads N] [workload:rows ...]`, one JSON line each."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "raytracer-795_amd")]
import bench  # noqa: E402
from rtg import scenegen  # noqa: E402

DEFAULT = ["dragon1m:270", "bunny:1080", "cornell:60", "cornell_pt:8", "spheres:30"]

ap = argparse.ArgumentParser()
ap.add_argument("--threads", type=int, default=os.cpu_count())
ap.add_argument("jobs", nargs="*", default=DEFAULT)
args = ap.parse_args()
for job in args.jobs:
    wl, rows = job.split(":")
    make, spp, text, _ = bench.WORKLOADS[wl]
    scene = getattr(scenegen, make)(1920, 1080, spp=spp)
    r = bench.cpu_baseline(scene, int(rows), args.threads)
    print(json.dumps({"workload": wl, "spp": spp, "host_cpus": os.cpu_count(), **r}), flush=True)
