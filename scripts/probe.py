"""Dev probe: render the bench scene once with timing/stats and print a breakdown."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracer-795_amd"))
import rtg  # noqa: E402
from rtg import scenegen  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "dragon1m"
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 64
if name == "dragon1m":
    sc = scenegen.dragon1m(1920, 1080, spp=spp)
elif name == "bunny5k":
    sc = scenegen.bunny5k(1920, 1080, spp=spp)
else:
    sc = scenegen.cornell(1920, 1080, spp=spp)
if len(sys.argv) > 3:
    sc.max_depth = int(sys.argv[3])     # e.g. 0: primary rays only (fixed trace input across variants)
t0 = time.time()
r = rtg.Renderer(sc, 0)
print("create", round(time.time() - t0, 2), "s", flush=True)
r.render(0)
base = {"max_batch_rays": int(os.environ.get("RTG_BATCH", "0"))}
for kw in ({"collect_stats": 1}, {"collect_timing": 1}, {}):
    kw = {**base, **kw}
    t0 = time.time()
    r.render(0, **kw)
    st = r.stats()
    st["wall_ms"] = round((time.time() - t0) * 1e3, 1)
    st["Mray_s"] = round(st["total_rays"] / st["render_ms"] / 1e3, 1)
    if st["trace_lane_slots"]:
        st["simd_eff_trace"] = round(st["trace_steps"] / st["trace_lane_slots"], 3)
        st["simd_eff_shadow"] = round(st["shadow_steps"] / st["shadow_lane_slots"], 3)
        tr = st["primary_rays"] + st["secondary_rays"]
        st["steps_per_ray"] = round(st["trace_steps"] / tr, 2)
        st["steps_per_shadow"] = round(st["shadow_steps"] / max(st["shadow_rays"], 1), 2)
    print(json.dumps({"opts": kw, **st}), flush=True)
