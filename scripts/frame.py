"""Render the bench frame N times (no stats, no timing) — the workload for PMC passes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracer-795_amd"))
import rtg  # noqa: E402
from rtg import scenegen  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1
w = os.environ.get("RTG_WORKLOAD", "dragon1m")      # any rtg.scenegen factory
sc = getattr(scenegen, w)(1920, 1080, spp=int(os.environ.get("RTG_SPP", "256" if w == "cornell_pt" else "64")))
r = rtg.Renderer(sc, 0)
stride = int(os.environ.get("RTG_ROW_STRIDE", "1"))     # one multi-GPU rank's row shard
for _ in range(n):
    r.render(0, row_offset=0, row_stride=stride, row_block=int(os.environ.get("RTG_ROW_BLOCK", "8")))
print("frame ms", round(r.stats()["render_ms"], 1))
