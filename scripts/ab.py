"""A/B of librtg variants (RTG_LIBRARY): median frame time at the default streams and the
isolated trace / shadow kernel times (streams=1 timing frame).  usage: ab.py [workload]"""
import json, os, statistics, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracer-795_amd"))
import rtg
from rtg import scenegen
w = sys.argv[1] if len(sys.argv) > 1 else "dragon1m"
fn, spp = {"bunny": ("bunny5k", 1), "cornell_pt": ("cornell_pt", 256)}.get(w, (w, 64))   # bench.py's workloads
sc = getattr(scenegen, fn)(1920, 1080, spp=spp)
# AB_OPTS "key=int,key=int": render options of this variant (e.g. tile_band=8)
kw = {k: int(v) for k, v in (p.split("=") for p in os.environ.get("AB_OPTS", "").split(",") if p)}
# AB_BUILD "key=int,...": build options (e.g. bvh_builder=1)
bkw = {k: int(v) for k, v in (p.split("=") for p in os.environ.get("AB_BUILD", "").split(",") if p)}
r = rtg.Renderer(sc, 0, **bkw)
r.render(0, **kw)
ms = []
for _ in range(int(os.environ.get("AB_FRAMES", "5"))):
    r.render(0, **kw)
    ms.append(r.stats()["render_ms"])
r.render(0, collect_stats=1, **kw)
ss = r.stats()
kw1 = {k: v for k, v in kw.items() if k != "streams"}
r.render(0, collect_timing=1, streams=1, **kw1)
r.render(0, collect_timing=1, streams=1, **kw1)
st = r.stats()
def breakdown(ss, p):
    """Entry-cycle shares, the flat group's set-up share and the all-work SIMD efficiency (ABI 9)."""
    cyc = list(ss.get(f"{p}_entry_cycles", []))
    tot = max(sum(cyc), 1)
    gc = list(ss.get(f"{p}_group_cycles", [0, 0]))
    work = ss[f"{p}_steps"] + ss.get(f"{p}_entry_visits", 0) + ss.get(f"{p}_group_work", 0)
    slots = ss[f"{p}_lane_slots"] + ss.get(f"{p}_entry_slots", 0) + ss.get(f"{p}_group_slots", 0)
    return {"entry_frac": [round(c / tot, 3) for c in cyc if c], "group_setup_frac": round(gc[0] / max(sum(gc), 1), 3),
            "group_frac": round(sum(gc) / tot, 3), "simd_eff_all": round(work / max(slots, 1), 4)}


print(json.dumps({"lib": os.environ.get("AB_TAG", os.environ.get("RTG_LIBRARY", "librtg")), "workload": w, "frame_ms": round(statistics.median(ms), 2),
                  "frames": [round(x, 2) for x in ms], "trace_ms": round(st["trace_ms"], 2),
                  "shadow_ms": round(st["shadow_ms"], 2), "shade_ms": round(st["shade_ms"], 2),
                  "resolve_ms": round(st["resolve_ms"], 2), "accumulate_ms": round(st["accumulate_ms"], 2),
                  "streams1_ms": round(st["render_ms"], 2),
                  "trace_steps_per_ray": round(ss["trace_steps"] / max(ss["primary_rays"] + ss["secondary_rays"], 1), 3),
                  "shadow_steps_per_query": round(ss["shadow_steps"] / max(ss["shadow_rays"], 1), 3),
                  "shadow_blocked_steps": round(ss["shadow_blocked_steps"] / max(ss["shadow_blocked"], 1), 3),
                  "trace_simd_eff": round(ss["trace_steps"] / max(ss["trace_lane_slots"], 1), 4),
                  "shadow_simd_eff": round(ss["shadow_steps"] / max(ss["shadow_lane_slots"], 1), 4),
                  **{f"{p}_{k}": v for p in ("trace", "shadow") for k, v in breakdown(ss, p).items()}}), flush=True)
