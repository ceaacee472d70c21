"""Benchmark: Mray/s + ms/frame at 1920x1080, 64 spp (BASELINE.json metric) on the
C3 `dragon1m` scene (1,000,004-triangle BVH, mirror + dielectric spheres, Whitted depth 6).

One step = one full frame.  With N ranks (torch.distributed.run, one process per GPU) rank r
renders every sample of the rows with (y // 4) % N == r compactly, and librtg gathers the
shards' rows onto rank 0's frame with RCCL point-to-point transfers (rtg_comm_init_rank +
rtg_render_ranked: the same shard + gather code as rtg_render_opts.num_devices and
`rtg_cli --devices N`; the fan-out it replaces is src/Scene.cpp:340-356).  value = rays traced
by all ranks / max-over-ranks frame time.  --ranked takes that RCCL path even at N = 1 (a
1-rank communicator).  RTG_BENCH_REHEARSE=1 rehearses the N-rank path on one GPU (every rank
on cuda:0, gloo gather through host memory); its numbers are not a scaling measurement.

Prints ONE JSON line (rank 0).  Extra objects:
  roofline     the dominant kernel (k_trace, closest hit) against the ceiling that binds it, VALU
               issue (MI355X_MICROARCH.md: 256 CUs x 4 SIMD-32, one wave64 VALU instruction per 2
               cycles at 2.4 GHz = 1228.8 G wave-instructions/s), from the committed PMC counters
               (profiles/counters_<workload>.json: SQ_INSTS_VALU per launch) divided by the live
               HIP-event launch time; `kernels` holds the same for k_shadow, k_shade (k_pt_shade), k_resolve2 (Whitted) and
               k_accumulate plus each kernel's measured HBM bytes (FETCH_SIZE x 2 + WRITE_SIZE)
               against 8 TB/s, and the traversal kernels' SIMD lane efficiency (node steps / lane
               slots of a collect_stats frame) with the lane-adjusted VALU fraction; `model` holds
               SURVEY §8(d)'s fixed algorithmic byte model (B = 64 + 32 N_node + 36 N_tri +
               16 N_sphere per ray, N_* from tests/golden/yardstick.json); `frame_hbm` the whole
               frame's measured HBM bytes over ms_per_step.
  cpu_baseline the CPU restatement (oracle/) on a bounded row sample of the same frame (N = 1).
  parity       that row sample against the same rows of the GPU frame (bitwise).
  multi        N > 1 (or --ranked): rank 0 renders the full frame alone after the timed loop and
               compares it with the gathered frame (gathered_equals_single).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "raytracer-795_amd"))

METRIC = "Mray/s + ms/frame at 1920×1080, 64 spp; 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0                       # MI355X_MICROARCH.md chip table: HBM3E 8.0 TB/s (spec)
L2_PEAK_GBS = 34500.0                       # MI355X_MICROARCH.md §L2: ~34.5 TB/s aggregate
VALU_PEAK_GIPS = 256 * 4 * 2.4 / 2          # G wave64-VALU-instructions/s (see the docstring)
PROFILES = os.path.join(ROOT, "profiles")
YARDSTICK = os.path.join(ROOT, "tests", "golden", "yardstick.json")


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def load_counters(workload: str) -> dict:
    """Per-dispatch PMC counter means of the last committed profiling run of this workload
    (scripts/pmc_counters.py): profiles/counters_<workload>.json (or, first, $RTG_COUNTERS_DIR's), or
    counters_current.json when it was taken on this workload."""
    dirs = [os.environ["RTG_COUNTERS_DIR"]] if os.environ.get("RTG_COUNTERS_DIR") else []
    cands = [os.path.join(d, f"counters_{workload}.json") for d in dirs + [PROFILES]]
    for f in cands + [os.path.join(PROFILES, "counters_current.json")]:
        try:
            with open(f) as fh:
                c = json.load(fh)
        except (OSError, ValueError):
            continue
        if c.get("workload", "dragon1m") == workload:
            return c
    return {}


def kernel_roof(counters: dict, name: str, avg_ms: float, launches: int) -> dict | None:
    c = counters.get("kernels", {}).get(name)
    if c is None or avg_ms <= 0:
        return None
    s = avg_ms * 1e-3
    out = {"kernel": name, "avg_launch_ms": round(avg_ms, 4), "launches": launches}
    if "SQ_INSTS_VALU" in c:
        a = c["SQ_INSTS_VALU"] / s / 1e9
        out["valu"] = {"achieved": round(a, 1), "peak": VALU_PEAK_GIPS, "unit": "G wave-inst/s",
                       "frac": round(a / VALU_PEAK_GIPS, 4), "insts_per_launch": c["SQ_INSTS_VALU"]}
    if "hbm_bytes" in c:
        a = c["hbm_bytes"] / s / 1e9
        out["hbm"] = {"achieved": round(a, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(a / HBM_PEAK_GBS, 4),
                      "bytes_per_launch": round(c["hbm_bytes"])}
    if "SQ_WAVE_CYCLES" in c and c["SQ_WAVE_CYCLES"] > 0:
        w = c["SQ_WAVE_CYCLES"]
        out["wave_cycles"] = {"issuing": round(c.get("SQ_ACTIVE_INST_ANY", 0) / w, 3),
                              "waiting_on_memory": round(c.get("SQ_WAIT_ANY", 0) / w, 3),
                              "issue_stalled": round(c.get("SQ_WAIT_INST_ANY", 0) / w, 3)}
    if c.get("TCC_HIT_sum", 0) + c.get("TCC_MISS_sum", 0) > 0:
        out["l2_hit_rate"] = round(c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"]), 4)
    if c.get("TCP_TOTAL_CACHE_ACCESSES_sum", 0) > 0:
        out["l1_to_l2_read_reqs_per_access"] = round(c["TCP_TCC_READ_REQ_sum"] / c["TCP_TOTAL_CACHE_ACCESSES_sum"], 4)
    return out


def _targs(k: str) -> list:
    return [a.strip() for a in k[k.index("<") + 1:k.rindex(">")].split(",")] if "<" in k else []


def frame_hbm_bytes(counters: dict, shade_name: str, shade_per_frame: int) -> float | None:
    """Measured HBM bytes of one rendered frame: every kernel's per-dispatch bytes x its dispatches in
    the profiled run, over the frames of that run (k_shade dispatches / k_shade launches per frame).
    The profiled run also creates the scene (twice): its build kernels (rocprim sorts, rtg::anon::
    kernels of rtg_bvh_gpu / rtg_sah_gpu; "rtg::" in counter files written before the names kept
    the namespace) are not frame traffic.  One of its frames is the collect_stats frame (the lane
    efficiencies): its traversal kernels are the STATS instantiations (second template argument
    true), which also write counters; they are left out and the plain traversal kernels divided by
    the other frames (the stats frames counted from the camera-ray launches, GEN = true)."""
    ks = counters.get("kernels", {})
    sh = ks.get(shade_name)
    if not sh or "dispatches_WRITE_SIZE" not in sh or shade_per_frame <= 0:
        return None
    frames = sh["dispatches_WRITE_SIZE"] / shade_per_frame

    def n_of(c):
        return min(c["dispatches_FETCH_SIZE"], c["dispatches_WRITE_SIZE"])

    def walk(k):
        return k.startswith(("rtg::k_trace<", "rtg::k_shadow<"))
    gen = {False: 0.0, True: 0.0}
    for k, c in ks.items():
        a = _targs(k)
        if k.startswith("rtg::k_trace<") and len(a) >= 3 and a[2] == "true" and "dispatches_WRITE_SIZE" in c:
            gen[a[1] == "true"] += n_of(c)
    stats_frames = frames * gen[True] / (gen[True] + gen[False]) if gen[True] > 0 and gen[False] > 0 else 0.0
    tot = 0.0
    for k, c in ks.items():
        if k.endswith("*>") or "hbm_bytes" not in c:       # combined entries double-count
            continue
        if k == "rtg::" or k.startswith(("rocprim::", "rtg::anon::")):
            continue
        if walk(k):
            if _targs(k)[1:2] == ["true"]:
                continue
            tot += c["hbm_bytes"] * n_of(c) / (frames - stats_frames)
        else:
            tot += c["hbm_bytes"] * n_of(c) / frames
    return tot


def cpu_baseline(scene, rows: int, threads: int):
    """The oracle on rows [y0, y0+rows) of the same frame: (cpu_baseline object, rgb rows)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle

    cam = scene.cameras[0]
    o = pyoracle.Oracle(scene)
    y0 = cam.ny // 2 - rows // 2
    t0 = time.perf_counter()
    rgb, _, _, _ = o.render(0, nthreads=threads, row_begin=y0, row_end=y0 + rows)
    dt = time.perf_counter() - t0
    c = o.ray_counts()
    nrays = c["primary"] + c["secondary"] + c["shadow"]
    o.close()
    host = host_cpu_info()
    v = nrays / dt / 1e6
    cpu = {"value": v, "unit": "Mray/s", "threads": threads, "host_cpus": host["host_cpus"],
           "cpus_granted": host["cpus_granted"], "kind": "port",
           "sample": f"rows {y0}..{y0 + rows - 1} of the same 1920x1080x{cam.num_samples}spp frame "
                     f"({rows * cam.nx} px, {nrays} rays, {dt:.1f} s, literal visit-both-children BVH)",
           # SURVEY 8(d) asks for threads = cores.  The GPU box grants this job `cpus_granted` of the host's
           # `host_cpus` CPUs (its CPU share; pools are sized to it, per the pool's rules), so the measured
           # figure runs at that many threads; the all-host-cores figure is a linear extrapolation of it
           # (the oracle's rows are independent: it scales with cores), labelled as such, never measured.
           "all_host_cpus_extrapolated": {"value": v * host["host_cpus"] / max(threads, 1),
                                          "threads": host["host_cpus"], "measured": False},
           "granted_source": host["source"]}
    return cpu, (y0, y0 + rows), rgb[y0:y0 + rows]


def host_cpu_info() -> dict:
    """The host's CPU count and the CPUs this process may use (affinity, then the cgroup v2 quota)."""
    host = os.cpu_count() or 1
    granted, src = host, "os.cpu_count"
    try:
        granted, src = len(os.sched_getaffinity(0)), "sched_getaffinity"
    except (AttributeError, OSError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            granted, src = min(granted, max(1, int(int(q) // int(per)))), "cgroup cpu.max"
    except (OSError, ValueError):
        pass
    env = os.environ.get("OMP_NUM_THREADS", "")
    if env.isdigit() and 0 < int(env) < granted:
        granted, src = int(env), "OMP_NUM_THREADS (the box's CPU share)"
    return {"host_cpus": host, "cpus_granted": granted, "source": src}


def compare_rows(gpu_rows: np.ndarray, ref_rows: np.ndarray, rows) -> dict:
    g, r = np.ascontiguousarray(gpu_rows, np.float32), np.ascontiguousarray(ref_rows, np.float32)
    nanm = int(np.sum(np.isnan(g) != np.isnan(r)))
    d = np.abs(g.astype(np.float64) - r.astype(np.float64))
    d = np.where(np.isnan(d), 0.0, d)
    diff = int(np.sum(np.nan_to_num(g).view(np.int32) != np.nan_to_num(r).view(np.int32)))
    return {"rows": [int(rows[0]), int(rows[1]) - 1], "values": int(g.size), "linf": float(d.max()) if d.size else 0.0,
            "differing": diff, "differing_frac": diff / max(g.size, 1), "nan_mismatch": nanm,
            "against": "oracle/ CPU restatement (cpu_baseline's rows), bitwise on the 0..255 float framebuffer"}


def load_yardstick(workload: str) -> dict:
    try:
        with open(YARDSTICK) as f:
            return json.load(f).get(workload, {})
    except (OSError, ValueError):
        return {}


# BASELINE.json configs -> (rtg.scenegen factory, default spp, config.workload text, data text)
WORKLOADS = {
    "dragon1m": ("dragon1m", 64,
                 "C3 dragon1m: 1,000,004-triangle BVH + mirror & dielectric spheres, point light, Whitted depth 6",
                 "synthetic (scenegen.dragon1m, seed 20261015)"),
    "bunny": ("bunny5k", 1,
              "C2 bunny5k: 5,120-triangle displaced icosphere, mirror floor, glass sphere, Whitted depth 6",
              "synthetic (scenegen.bunny5k)"),
    "cornell": ("cornell", 64,
                "C4 cornell_dynamic: instancing (resetTransform on/off), motion blur, area light, DoF, "
                "rough mirror, conductor; distribution ray tracing depth 4",
                "synthetic (scenegen.cornell)"),
    "cornell_pt": ("cornell_pt", 256,
                   "C5 cornell_pt (hw7): path tracing with importance sampling + NEE + Russian roulette, "
                   "LightMesh + LightSphere, BRDF walls, glass / mirror spheres",
                   "synthetic (scenegen.cornell_pt)"),
    "spheres": ("spheres", 64,
                "hw3 Spheres-DOF analogue: 1,024 spheres (one object each) on a ground quad, DoF camera, "
                "point light, Whitted depth 3",
                "synthetic (scenegen.spheres)"),
}


def kernel_table(counters, st_roof, st_stats, pt: bool) -> dict:
    """roofline.kernels: every frame kernel with a live launch time and committed counters."""
    ks = counters.get("kernels", {})

    def first(prefix):
        names = sorted((k for k in ks if k.startswith(prefix)),
                       key=lambda k: (not k.endswith("*>"), -ks[k].get("dispatches_SQ_INSTS_VALU", 0)))
        return names[0] if names else ""

    shade = first("rtg::k_pt_shade<" if pt else "rtg::k_shade<")
    # the shadow kernel's TLAS instantiation (k_shadow<false, false, true>) runs on scenes with a
    # top-level BVH (spheres)
    rows = [("k_trace", "rtg::k_trace<false, false, *>", "trace"),
            ("k_shadow", first("rtg::k_shadow<false, false"), "shadow"),
            ("k_pt_shade" if pt else "k_shade", shade, "shade"),
            ("k_accumulate", first("rtg::k_accumulate<"), "accumulate")]
    # the bottom-up pass (Whitted only): k_resolve2 resolves two levels per launch (round 5); the path
    # tracer has no bottom-up pass since round 6 (radiance rides with the path, k_pt_gather is gone)
    if not pt:
        rows.append(("k_resolve2", first("rtg::k_resolve2"), "resolve"))
    out = {}
    for key, name, slot in rows:
        n = st_roof.get(f"{slot}_launches", 0)
        avg = st_roof.get(f"{slot}_ms", 0.0) / max(n, 1)
        kr = kernel_roof(counters, name, avg, n)
        if kr:
            out[key] = kr
    # SIMD lane efficiency of the traversal kernels (collect_stats frame): node steps / lane slots
    # of the BVH walks (simd_eff_walk) and, all work included, (node steps + top-level entries visited
    # + the flat group's triangle tests) / (walk lane slots + 64 x the entries each wave's object loop
    # went through + 64 x the group tests each wave ran): the reference's linear object loop
    # (src/Helper.cpp:33-73) costs every lane its entry-start work whether or not the lane walks that
    # entry, and the flat group (round 5) tests its triangles per lane without node steps -- round 6
    #  counts that work, which the walk-only figure missed.  The lane-adjusted VALU
    # fraction uses the all-work figure.
    for key, pre in (("k_trace", "trace"), ("k_shadow", "shadow")):
        slots = st_stats.get(f"{pre}_lane_slots", 0)
        if key in out and slots > 0:
            walk = st_stats[f"{pre}_steps"] / slots
            ev, es = st_stats.get(f"{pre}_entry_visits", 0), st_stats.get(f"{pre}_entry_slots", 0)
            gw, gs = st_stats.get(f"{pre}_group_work", 0), st_stats.get(f"{pre}_group_slots", 0)
            eff = (st_stats[f"{pre}_steps"] + ev + gw) / (slots + es + gs) if es + gs > 0 else walk
            out[key]["simd_eff_walk"] = round(walk, 4)
            out[key]["simd_eff"] = round(eff, 4)
            if es > 0:
                out[key]["entry_lane_activity"] = {
                    "entries_visited_per_lane_slot": round(ev / es, 4),
                    "entry_visits": ev, "entry_slots": es,
                    "node_steps": st_stats[f"{pre}_steps"], "walk_lane_slots": slots}
            if gs > 0:
                gc = list(st_stats.get(f"{pre}_group_cycles", [0, 0]))
                out[key]["flat_group"] = {
                    "lane_work": gw, "lane_slots": gs, "simd_eff": round(gw / gs, 4),
                    "cycles_setup_frac": round(gc[0] / max(sum(gc), 1), 4),
                    "note": "triangle tests the lanes ran (every member's fast rejection, then each lane's own "
                            "candidates' exact tests) over 64 x the tests their waves ran; cycles: set-up "
                            "(transform, reciprocals, window) vs tests, of the group's slot in entry_cycles_frac"}
            if "valu" in out[key]:
                out[key]["valu"]["lane_adjusted_frac"] = round(out[key]["valu"]["frac"] * eff, 4)
    # where the traversal's wave time goes: s_memtime cycles per top-level entry of the linear loop
    # (collect_stats frame; entries >= 15 pooled in the last slot)
    for key, pre in (("k_trace", "trace"), ("k_shadow", "shadow")):
        cyc = list(st_stats.get(f"{pre}_entry_cycles", []))
        while cyc and cyc[-1] == 0:
            cyc.pop()
        if key in out and cyc and sum(cyc) > 0:
            out[key]["entry_cycles_frac"] = [round(c / sum(cyc), 4) for c in cyc]
    pc = list(st_stats.get("pt_shade_cycles", []))
    if pt and "k_pt_shade" in out and sum(pc) > 0:
        out["k_pt_shade"]["phase_cycles_frac"] = dict(zip(("hit_setup", "nee", "continuation", "compaction_stores"),
                                                          [round(c / sum(pc), 4) for c in pc]))
    sq = st_stats.get("shadow_rays", 0)
    if "k_shadow" in out and sq > 0:
        b = st_stats["shadow_blocked"]
        ub = max(sq - b, 1)
        out["k_shadow"]["queries"] = {
            "blocked_frac": round(b / sq, 4),
            "steps_per_blocked": round(st_stats["shadow_blocked_steps"] / max(b, 1), 3),
            "steps_per_unblocked": round((st_stats["shadow_steps"] - st_stats["shadow_blocked_steps"]) / ub, 3),
            "tris_per_blocked": round(st_stats["shadow_blocked_tris"] / max(b, 1), 3),
            "tris_per_unblocked": round((st_stats["shadow_tri_tests"] - st_stats["shadow_blocked_tris"]) / ub, 3)}
        if "shadow_hist_before" in st_stats and b > 0:
            # finding the blocker vs proving it nearest (Light::IsShadow, src/Light.cpp:188-204)
            out["k_shadow"]["queries"]["blocked_steps_split"] = {
                "steps_before_blocker_per_blocked": round(st_stats["shadow_blocked_steps_before"] / b, 3),
                "wave_min_steps_before_blocker_per_blocked": round(
                    st_stats.get("shadow_blocked_steps_before_wavemin", 0) / b, 3),
                "steps_after_blocker_per_blocked": round(
                    (st_stats["shadow_blocked_steps"] - st_stats["shadow_blocked_steps_before"]) / b, 3),
                "bins": ["0", "1", "2", "3-4", "5-8", "9-16", "17-32", ">32"],
                "hist_before": st_stats["shadow_hist_before"], "hist_after": st_stats["shadow_hist_after"]}
    return out, shade


def roofline(counters, st_roof, st_stats, workload: str, ms_per_step: float, pt: bool) -> dict:
    kern, shade = kernel_table(counters, st_roof, st_stats, pt)
    # fixed algorithmic bytes per closest-hit ray (tests/golden/yardstick.json), priced
    # over the k_trace launches' rays and live launch time
    ys = load_yardstick(workload)
    trace_avg = st_roof["trace_ms"] / max(st_roof["trace_launches"], 1)
    traced = st_stats["primary_rays"] + st_stats["secondary_rays"]
    model = None
    if ys:
        bpr = ys["bytes_per_ray"]
        rays_per_launch = (st_roof["primary_rays"] + st_roof["secondary_rays"]) / max(st_roof["trace_launches"], 1)
        gbs = bpr * rays_per_launch / (trace_avg * 1e-3) / 1e9 if trace_avg > 0 else 0.0
        model = {"bytes_per_ray": bpr, "n_node": ys["n_node"], "n_tri": ys["n_tri"], "n_sphere": ys["n_sphere"],
                 "shadow_bytes_per_ray": ys["shadow_bytes_per_ray"], "source": "tests/golden/yardstick.json (" +
                 ys["sample"] + ", canonical ordered early-exit traversal of the reference trees)",
                 "requested": round(gbs, 1), "unit": "GB/s (requested, cache-served)",
                 "frac_of_l2_peak": round(gbs / L2_PEAK_GBS, 4),
                 "note": "bytes the canonical traversal requests per ray; the vL1D / L2 / MALL serve most of "
                         "them (measured HBM bytes: kernels.k_trace.hbm), so this rate is priced against the "
                         "aggregate L2 bandwidth only, never against HBM"}
    gpu_walk = {"node_records_per_ray": round(st_stats["node_visits"] / max(traced, 1), 3),
                "tri_tests_per_ray": round(st_stats["tri_tests"] / max(traced, 1), 3),
                "shadow_node_records_per_query": round(st_stats["shadow_node_visits"] / max(st_stats["shadow_rays"], 1), 3),
                "shadow_tri_tests_per_query": round(st_stats["shadow_tri_tests"] / max(st_stats["shadow_rays"], 1), 3)}
    tr = kern.get("k_trace", {})
    roof = {"bound": "valu", "kernel": "k_trace<false,false,*> (closest hit; GEN=true generates the primary "
                                       "rays at level 0, GEN=false traces secondary levels)",
            "achieved": tr.get("valu", {}).get("achieved"), "peak": VALU_PEAK_GIPS, "unit": "G wave-inst/s",
            "frac": tr.get("valu", {}).get("frac"),
            "traffic": tr.get("hbm", {}).get("bytes_per_launch"),
            "traffic_unit": "HBM bytes per launch (PMC FETCH_SIZE x 2 + WRITE_SIZE, profiles/counters_<workload>.json)",
            "peak_source": "MI355X_MICROARCH.md: 256 CUs x 4 SIMD-32, wave64 VALU instruction per 2 cycles, 2400 MHz",
            "avg_launch_ms": round(trace_avg, 4), "launches": st_roof["trace_launches"],
            "timing": "HIP events around each launch in a streams=1 frame outside the timed region",
            "counters": counters.get("source"), "roofline_frame_ms": round(st_roof["render_ms"], 2),
            "kernels": kern, "model": model, "gpu_walk": gpu_walk}
    fb = frame_hbm_bytes(counters, shade, st_roof["shade_launches"]) if shade else None
    if fb:
        roof["frame_hbm"] = {"bytes_per_frame": round(fb), "achieved": round(fb / (ms_per_step * 1e-3) / 1e9, 1),
                             "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": round(fb / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
    return roof


def create_phases(bs: dict, create_ms: float) -> dict:
    """rtg_build_stats' wall-time split of rtg_scene_create (ABI 7), plus the Python descriptor
    build around it (Renderer(scene) - the library call)."""
    keys = ("validate_ms", "prep_ms", "median_tree_ms", "records_ms", "traversal_tree_ms", "top_level_ms",
            "upload_ms", "total_ms")
    out = {k[:-3]: round(bs[k], 1) for k in keys if k in bs}
    if "total_ms" in bs:
        out["desc_python"] = round(create_ms - bs["total_ms"], 1)
        out["upload_MB"] = round(bs["upload_bytes"] / 1e6, 1)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=0, help="0 = the workload's spp (64; cornell_pt 256)")
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="dragon1m",
                    help="dragon1m = the BASELINE metric line (C3); the others are the configs' own scenes")
    ap.add_argument("--cpu-rows", type=int, default=0,
                    help="rows of the CPU baseline sample (0: about 10-30 s of CPU work for the workload)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="oracle threads for cpu_baseline; 0 = every CPU this job is granted (host_cpu_info)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--ranked", action="store_true",
                    help="render through rtg_render_ranked (RCCL shard + gather) even with one rank")
    ap.add_argument("--tlas", choices=["auto", "off", "on"], default="auto",
                    help="top-level BVH over objects / instances (rtg_build_opts.tlas; auto: from 16 entries)")
    ap.add_argument("--streams", type=int, default=0,
                    help="HIP streams (lanes) of every frame (rtg_render_opts.streams; 0 = library default). "
                         "PMC passes use 1 so each dispatch is one pass's launch (scripts/pmc_counters.py)")
    ap.add_argument("--timeout-s", type=int, default=300,
                    help="N > 1: bound on every wait for a peer rank (process group set-up, id exchange, "
                         "librtg's RCCL set-up / failure agreement / gather); a dead peer is an error, not a hang")
    args = ap.parse_args()
    # stdout carries exactly the one JSON line: libraries that print banners there (RCCL's
    # "RCCL version ..." at communicator init) are sent to stderr with everything else
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)

    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    rehearse = os.environ.get("RTG_BENCH_REHEARSE") == "1"
    if rehearse:
        local = 0
    torch.cuda.set_device(local)
    id_group = None
    if world > 1:
        from datetime import timedelta

        import torch.distributed as dist
        tmo = timedelta(seconds=args.timeout_s)
        if rehearse:
            dist.init_process_group("gloo", timeout=tmo)
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=tmo)
            id_group = dist.new_group(backend="gloo", timeout=tmo)     # host-side id exchange

    import rtg
    from rtg import _abi as rtg_abi
    from rtg import scenegen
    from rtg.shard import ROW_BLOCK, exchange_comm_id, gather_frame, max_shard_rows, shard_opts

    t0 = time.perf_counter()
    make, spp_default, wl_text, data_text = WORKLOADS[args.workload]
    if args.cpu_rows <= 0:
        args.cpu_rows = {"cornell_pt": 96, "spheres": 32}.get(args.workload, 540)
    scene = getattr(scenegen, make)(args.width, args.height, spp=args.spp or spp_default)
    log(f"[rank {rank}] scene: {scene.num_triangles()} triangles, gen {time.perf_counter() - t0:.1f}s")
    # The process's first kernel launch pays the HIP runtime's one-time set-up (100-170 ms on MI355X,
    # profiles/history/r4i_hip_init_probe_kernel_first.txt: torch's own first fill).  It is timed here on its
    # own (end_to_end_ms.runtime_init) so that scene_create is the library's cost in a process whose
    # device is in use, as in any PyTorch program; librtg's own code-object load stays in it.
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    torch.zeros(1, device=f"cuda:{local}")
    torch.cuda.synchronize()
    runtime_init_ms = (time.perf_counter() - t0) * 1e3
    t0 = time.perf_counter()
    r = rtg.Renderer(scene, device=local, tlas={"auto": 0, "off": 1, "on": 2}[args.tlas])
    create_ms = (time.perf_counter() - t0) * 1e3
    log(f"[rank {rank}] rtg_scene_create (BVH build + upload) {create_ms:.0f} ms")
    cam = scene.cameras[0]
    pt = cam.integrator == rtg_abi.INTEGRATOR_PATH
    frame = torch.zeros((cam.ny, cam.nx, 3), dtype=torch.float32, device=f"cuda:{local}")
    host = torch.empty((cam.ny, cam.nx, 3), dtype=torch.float32, pin_memory=True)
    stream = torch.cuda.current_stream().cuda_stream
    comm = None
    part = None
    if (world > 1 or args.ranked) and not rehearse:
        # librtg's own RCCL communicator (ncclCommInitRank, non-blocking with a deadline); its id
        # travels over a gloo group of torch.distributed, bounded by the same timeout
        uid = exchange_comm_id(dist, rank, rtg.Comm.unique_id, group=id_group) if dist is not None \
            else rtg.Comm.unique_id()
        comm = rtg.Comm(uid, world, rank, local, timeout_ms=args.timeout_s * 1000)
    elif world > 1:
        part = torch.zeros((max_shard_rows(cam.ny, world), cam.nx, 3), dtype=torch.float32, device=frame.device)
    sharded = comm is not None or part is not None

    def single(buf, **kw):
        kw.setdefault("streams", args.streams)
        r.render_device(0, buf.data_ptr(), stream, **kw)
        return r.stats()

    def step(**kw):
        kw.setdefault("streams", args.streams)
        if comm is not None:       # shard + RCCL gather inside librtg (rtg_render_ranked)
            r.render_ranked(0, comm, frame.data_ptr(), stream, row_block=ROW_BLOCK, **kw)
        elif part is not None:     # rehearsal: compact shard, gloo gather in Python
            r.render_device(0, part.data_ptr(), stream, **shard_opts(rank, world), compact_rows=1, **kw)
            st = r.stats()
            torch.cuda.synchronize()
            tg = time.perf_counter()
            gather_frame(part, frame, rank, world, dist)
            return dict(st, gather_ms=(time.perf_counter() - tg) * 1e3)
        else:
            r.render_device(0, frame.data_ptr(), stream, **kw)
        return r.stats()

    def roofline_frames(buf):
        """traversal statistics (collect_stats) and the per-launch timing frame: passes one at a
        time (streams=1) so every launch is timed alone by its HIP events (the timed frames overlap
        passes on several streams, where an event pair would also count other streams' work); the
        first streams=1 frame also grows that lane's level buffers, so it is run twice."""
        st_stats = single(buf, collect_stats=1)
        single(buf, collect_timing=1, streams=1)
        return st_stats, single(buf, collect_timing=1, streams=1)

    # one frame to the host right after the upload: the end-to-end time of a fresh scene
    t0 = time.perf_counter()
    step()
    if rank == 0:
        host.copy_(frame, non_blocking=True)
    torch.cuda.synchronize()
    first_frame_ms = (time.perf_counter() - t0) * 1e3
    st_stats = st_roof = None
    if not sharded:
        st_stats, st_roof = roofline_frames(frame)
    for _ in range(args.warmup):
        step()

    def timed(to_host: bool):
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        rays = 0
        st = None
        for i in range(args.steps):
            st = step()
            if to_host and rank == 0:
                host.copy_(frame, non_blocking=True)
            rays += st["total_rays"]
            log(f"[rank {rank}] step {i}{' (+D2H)' if to_host else ''}: {st['render_ms']:.1f} ms, rays {st['total_rays']}")
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        gather_max = st.get("gather_ms", 0.0) if st else 0.0
        if dist is not None:
            dev = frame.device if not rehearse else "cpu"
            t = torch.tensor([elapsed, gather_max], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed, gather_max = float(t[0].item()), float(t[1].item())
            if st is not None:
                st = dict(st, gather_ms_max_over_ranks=gather_max)
            rt = torch.tensor([rays], dtype=torch.float64, device=dev)
            dist.all_reduce(rt, op=dist.ReduceOp.SUM)
            rays = int(rt.item())
            # every rank's shard time (its render minus its agreement + gather) of the last step
            shard = float(st["render_ms"] - st.get("gather_ms", 0.0)) if st else 0.0
            if comm is None and st is not None:
                shard = float(st["render_ms"])          # rehearsal: render_ms is the shard alone
            parts = [torch.zeros(1, dtype=torch.float64, device=dev) for _ in range(world)]
            dist.all_gather(parts, torch.tensor([shard], dtype=torch.float64, device=dev))
            if st is not None:
                st = dict(st, shard_ms_per_rank=[round(float(x.item()), 3) for x in parts])
        return elapsed, rays, st

    elapsed, rays, st = timed(False)
    elapsed_h, _, _ = timed(True)
    ms_per_step = elapsed * 1e3 / args.steps
    value = rays / elapsed / 1e6
    rays_frame = rays // max(args.steps, 1)

    multi = None
    if sharded and rank == 0:
        # rank 0 alone: the full frame on its own device vs the gathered frame (bit for bit), then
        # its single-device roofline frames (same kernels and counters as the N = 1 line)
        full = torch.zeros_like(frame)
        t0 = time.perf_counter()
        single(full)
        torch.cuda.synchronize()
        single_ms = (time.perf_counter() - t0) * 1e3
        same = bool(torch.equal(full.view(torch.int32), frame.view(torch.int32)))
        log(f"[rank 0] gathered frame == single-device frame: {same}")
        multi = {"gathered_equals_single": same, "ranks": world,
                 "gather": "rehearsal: gloo gather through host memory (all ranks on one GPU)" if rehearse
                 else "RCCL point-to-point rows gather inside librtg (rtg_render_ranked)",
                 "single_device_frame_ms": round(single_ms, 2), "row_block": ROW_BLOCK,
                 "gather_ms_rank0": round(st.get("gather_ms", 0.0), 3),
                 "gather_ms_max_over_ranks": round(st.get("gather_ms_max_over_ranks", 0.0), 3),
                 "shard_ms_per_rank": st.get("shard_ms_per_rank"),
                 "gather_note": ("per rank: the Python gloo gather of the compact rows after the rank's shard "
                                 "(host memory), last timed step" if rehearse else
                                 "per rank: librtg's failure agreement + RCCL rows gather after the rank's shard "
                                 "finished (rtg_render_stats.gather_ms), last timed step"),
                 "shard_note": "shard_ms_per_rank: each rank's own shard render of the last timed step"
                               + (" -- all ranks share one GPU in a rehearsal, so each shard takes about the "
                                  "whole GPU's frame time" if rehearse else ""),
                 "timeout_s": args.timeout_s}
        if rehearse and not same:
            raise SystemExit("rehearsal: gathered frame differs from the single-device frame")
        st_stats, st_roof = roofline_frames(full)
        del full
    if dist is not None:
        dist.barrier()

    if rank == 0:
        # the same scene created again in this process (outside every timed region): the first
        # rtg_scene_create also pays the HIP runtime's one-time first-use set-up, ~100-150 ms for the
        # first launch / copy of a process (scripts/micro/init_probe.hip, profiles/history/r4m_init_probe.txt)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r2 = rtg.Renderer(scene, device=local, tlas={"auto": 0, "off": 1, "on": 2}[args.tlas])
        again_ms = (time.perf_counter() - t0) * 1e3
        again = {"ms": round(again_ms, 1), "phases": create_phases(r2.build_stats(), again_ms),
                 "note": "a second Renderer(scene) in the same process (librtg's code objects loaded, its "
                         "host threads and device allocator warm)"}
        r2.close()
        counters = load_counters(args.workload)
        roof = roofline(counters, st_roof, st_stats, args.workload, ms_per_step, pt)
        if sharded:
            roof["note"] = "rank 0's single-device roofline frames after the timed loop (the sharded frame's passes " \
                           "are smaller; the counters are per launch of the full frame)"
        cpu = parity = None
        cpu_note = None
        if args.no_cpu:
            cpu_note = "skipped (--no-cpu)"
        elif world > 1:
            cpu_note = "measured on the N = 1 line only (rank 0, N = 1 per the bench contract); see BENCH N=1"
        else:
            log("[rank 0] cpu baseline ...")
            cpu, rows, ref_rows = cpu_baseline(scene, args.cpu_rows,
                                               args.cpu_threads or host_cpu_info()["cpus_granted"])
            parity = compare_rows(host.numpy()[rows[0]:rows[1]], ref_rows, rows)
            log(f"[rank 0] parity rows {rows}: linf={parity['linf']} differing={parity['differing']}")
        if world == 1 and comm is None:
            par = "single GPU"
        elif rehearse:
            par = f"{ROW_BLOCK}-row-block pixel shards x{world} + gloo gather (rehearsal, all ranks on one GPU)"
        else:
            par = f"{ROW_BLOCK}-row-block pixel shards x{world}, one process per GPU + RCCL gather inside librtg"
        line = {"metric": METRIC, "value": round(value, 2), "unit": "Mray/s", "n_gpus": world,
                "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 2),
                "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
                "data": data_text,
                "config": {"workload": wl_text, "resolution": f"{cam.nx}x{cam.ny}", "spp": cam.num_samples,
                           "parallelism": par, "tlas": args.tlas, "tlas_nodes": r.build_stats()["tlas_nodes"]},
                "rays_per_frame": rays_frame,
                "primary_msamples_s": round(cam.nx * cam.ny * cam.num_samples / (ms_per_step * 1e-3) / 1e6, 1),
                "ms_per_frame_to_host": round(elapsed_h * 1e3 / args.steps, 2),
                "end_to_end_ms": {"runtime_init": round(runtime_init_ms, 1),
                                  "scene_create": round(create_ms, 1), "first_frame_to_host": round(first_frame_ms, 1),
                                  "total": round(runtime_init_ms + create_ms + first_frame_ms, 1),
                                  "scene_create_phases": create_phases(r.build_stats(), create_ms),
                                  "scene_create_again": again,
                                  "note": "runtime_init = the process's first kernel launch (torch.zeros, the HIP "
                                          "runtime's one-time set-up); Renderer(scene) = the Python host's descriptor "
                                          "(desc_python) + rtg_scene_create (library phases), then the first frame incl. "
                                          "its D2H copy"},
                "rays_rank0": {k: st[k] for k in ("primary_rays", "secondary_rays", "shadow_rays")},
                "kernel_ms_rank0_streams1": {k: round(st_roof[f"{k}_ms"], 2)
                                             for k in ("trace", "shade", "shadow", "resolve", "accumulate")},
                "roofline": roof, "cpu_baseline": cpu, "parity": parity, "multi": multi}
        if cpu_note:
            line["cpu_baseline_note"] = cpu_note
        print(json.dumps(line), file=json_out, flush=True)
    if comm is not None:
        comm.close()
    r.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
