"""Benchmark: Mray/s + ms/frame at 1920x1080, 64 spp (BASELINE.json metric) on the
C3 `dragon1m` scene (1,000,004-triangle BVH, mirror + dielectric spheres, Whitted depth 6).

One step = one full frame.  With N ranks (torch.distributed.run, one process per GPU) rank r
renders every sample of the rows with (y // 4) % N == r compactly, and librtg gathers the
shards' rows onto rank 0's frame with RCCL point-to-point transfers (rtg_comm_init_rank +
rtg_render_ranked: the same shard + gather code as rtg_render_opts.num_devices and
`rtg_cli --devices N`).  value = rays traced by all ranks / max-over-ranks frame time.
RTG_BENCH_REHEARSE=1 rehearses the N-rank path on one GPU (every rank on cuda:0, gloo gather
through host memory); its numbers are not a scaling measurement.

Prints ONE JSON line (rank 0).  Extra objects:
  roofline     the dominant kernel (k_trace, closest hit) against the ceiling that binds it, VALU
               issue (MI355X_MICROARCH.md: 256 CUs x 4 SIMD-32, one wave64 VALU instruction per 2
               cycles at 2.4 GHz = 1228.8 G wave-instructions/s), from the committed PMC counters
               (profiles/counters_current.json: SQ_INSTS_VALU per launch) divided by the live
               HIP-event launch time; `kernels` holds the same for k_shadow and k_shade plus each
               kernel's measured HBM bytes (FETCH_SIZE x 2 + WRITE_SIZE) against 8 TB/s; `model`
               holds SURVEY §8(d)'s algorithmic byte model (B = 64 + 32 N_node + 36 N_tri per ray);
               `frame_hbm` the whole frame's measured HBM bytes over ms_per_step.
  cpu_baseline the CPU restatement (oracle/) on a bounded row sample of the same frame.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "raytracer-795_amd"))

METRIC = "Mray/s + ms/frame at 1920×1080, 64 spp; 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0                       # MI355X_MICROARCH.md chip table: HBM3E 8.0 TB/s (spec)
L2_PEAK_GBS = 34500.0                       # MI355X_MICROARCH.md §L2: ~34.5 TB/s aggregate
VALU_PEAK_GIPS = 256 * 4 * 2.4 / 2          # G wave64-VALU-instructions/s (see the docstring)
COUNTERS = os.path.join(ROOT, "profiles", "counters_current.json")


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def load_counters() -> dict:
    """Per-dispatch PMC counter means of the last committed profiling run (scripts/pmc_counters.py)."""
    try:
        with open(COUNTERS) as f:
            return json.load(f)
    except (OSError, ValueError):
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


def frame_hbm_bytes(counters: dict, shade_name: str, shade_per_frame: int) -> float | None:
    """Measured HBM bytes of one whole frame: every kernel's per-dispatch bytes x its dispatches in
    the profiled run, over the frames of that run (k_shade dispatches / k_shade launches per frame)."""
    ks = counters.get("kernels", {})
    sh = ks.get(shade_name)
    if not sh or "dispatches_WRITE_SIZE" not in sh or shade_per_frame <= 0:
        return None
    frames = sh["dispatches_WRITE_SIZE"] / shade_per_frame
    tot = 0.0
    for k, c in ks.items():
        if k.endswith("*>") or "hbm_bytes" not in c:       # combined entries double-count
            continue
        tot += c["hbm_bytes"] * min(c["dispatches_FETCH_SIZE"], c["dispatches_WRITE_SIZE"])
    return tot / frames


def cpu_baseline(scene, rows: int, threads: int) -> dict:
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle

    cam = scene.cameras[0]
    o = pyoracle.Oracle(scene)
    y0 = cam.ny // 2 - rows // 2
    t0 = time.perf_counter()
    o.render(0, nthreads=threads, row_begin=y0, row_end=y0 + rows)
    dt = time.perf_counter() - t0
    c = o.ray_counts()
    nrays = c["primary"] + c["secondary"] + c["shadow"]
    o.close()
    return {"value": nrays / dt / 1e6, "unit": "Mray/s", "cores": threads, "kind": "port",
            "sample": f"rows {y0}..{y0 + rows - 1} of the same 1920x1080x{cam.num_samples}spp frame "
                      f"({rows * cam.nx} px, {nrays} rays, {dt:.1f} s, literal visit-both-children BVH)"}


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
    ap.add_argument("--cpu-rows", type=int, default=540)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--tlas", choices=["auto", "off", "on"], default="auto",
                    help="top-level BVH over objects / instances (rtg_build_opts.tlas; auto: from 16 entries)")
    args = ap.parse_args()

    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    rehearse = os.environ.get("RTG_BENCH_REHEARSE") == "1"
    if rehearse:
        local = 0
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    import rtg
    from rtg import scenegen
    from rtg.shard import ROW_BLOCK, gather_frame, max_shard_rows, shard_opts

    t0 = time.perf_counter()
    make, spp_default, wl_text, data_text = WORKLOADS[args.workload]
    scene = getattr(scenegen, make)(args.width, args.height, spp=args.spp or spp_default)
    log(f"[rank {rank}] scene: {scene.num_triangles()} triangles, gen {time.perf_counter() - t0:.1f}s")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = rtg.Renderer(scene, device=local, tlas={"auto": 0, "off": 1, "on": 2}[args.tlas])
    create_ms = (time.perf_counter() - t0) * 1e3
    log(f"[rank {rank}] rtg_scene_create (BVH build + upload) {create_ms:.0f} ms")
    cam = scene.cameras[0]
    frame = torch.zeros((cam.ny, cam.nx, 3), dtype=torch.float32, device=f"cuda:{local}")
    host = torch.empty((cam.ny, cam.nx, 3), dtype=torch.float32, pin_memory=True)
    stream = torch.cuda.current_stream().cuda_stream
    comm = None
    part = None
    if world > 1 and not rehearse:
        # librtg's own RCCL communicator (ncclCommInitRank); its id travels over torch.distributed
        uid = [rtg.Comm.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        comm = rtg.Comm(uid[0], world, rank, local)
    elif world > 1:
        part = torch.zeros((max_shard_rows(cam.ny, world), cam.nx, 3), dtype=torch.float32, device=frame.device)

    def step(**kw):
        if world == 1:
            r.render_device(0, frame.data_ptr(), stream, **kw)
        elif comm is not None:     # shard + RCCL gather inside librtg (rtg_render_ranked)
            r.render_ranked(0, comm, frame.data_ptr(), stream, row_block=ROW_BLOCK, **kw)
        else:                      # rehearsal: compact shard, gloo gather in Python
            r.render_device(0, part.data_ptr(), stream, **shard_opts(rank, world), compact_rows=1, **kw)
            st = r.stats()
            gather_frame(part, frame, rank, world, dist)
            return st
        return r.stats()

    # one frame to the host right after the upload: the end-to-end time of a fresh scene
    t0 = time.perf_counter()
    step()
    if rank == 0:
        host.copy_(frame, non_blocking=True)
    torch.cuda.synchronize()
    first_frame_ms = (time.perf_counter() - t0) * 1e3
    # traversal statistics for the byte model (outside the timed region)
    st_stats = step(collect_stats=1)
    # roofline frame (outside the timed region): passes one at a time (streams=1) so every
    # trace / shade / shadow launch is timed alone by its HIP events; the timed frames below
    # overlap passes on several streams, where an event pair would also count other streams'
    # work (twice: the first streams=1 frame also grows that lane's level buffers)
    step(collect_timing=1, streams=1)
    st_roof = step(collect_timing=1, streams=1)
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
        if dist is not None:
            dev = frame.device if not rehearse else "cpu"
            t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
            rt = torch.tensor([rays], dtype=torch.float64, device=dev)
            dist.all_reduce(rt, op=dist.ReduceOp.SUM)
            rays = int(rt.item())
        return elapsed, rays, st

    elapsed, rays, st = timed(False)
    elapsed_h, _, _ = timed(True)
    ms_per_step = elapsed * 1e3 / args.steps
    value = rays / elapsed / 1e6
    rays_frame = rays // max(args.steps, 1)

    if rehearse and rank == 0 and world > 1:
        # the gathered frame must equal this rank's own single-device frame bit for bit
        full = torch.zeros_like(frame)
        r.render_device(0, full.data_ptr(), stream)
        torch.cuda.synchronize()
        same = bool(torch.equal(full.view(torch.int32), frame.view(torch.int32)))
        log(f"[rank 0] rehearsal: gathered frame == single-device frame: {same}")
        if not same:
            raise SystemExit("rehearsal: gathered frame differs from the single-device frame")

    if rank == 0:
        counters = load_counters()
        trace_avg = st_roof["trace_ms"] / max(st_roof["trace_launches"], 1)
        shadow_avg = st_roof["shadow_ms"] / max(st_roof["shadow_launches"], 1)
        shade_avg = st_roof["shade_ms"] / max(st_roof["shade_launches"], 1)
        shade_names = sorted((k for k in counters.get("kernels", {}) if k.startswith("rtg::k_shade<")),
                             key=lambda k: -counters["kernels"][k].get("dispatches_SQ_INSTS_VALU", 0))
        same_wl = counters.get("workload", "dragon1m") == args.workload and world == 1
        kern = {}
        if same_wl:
            for key, name, avg, n in (("k_trace", "rtg::k_trace<false, false, *>", trace_avg, st_roof["trace_launches"]),
                                      ("k_shadow", "rtg::k_shadow<false, false, false>", shadow_avg, st_roof["shadow_launches"]),
                                      ("k_shade", shade_names[0] if shade_names else "", shade_avg, st_roof["shade_launches"])):
                kr = kernel_roof(counters, name, avg, n)
                if kr:
                    kern[key] = kr
        # SURVEY §8(d) algorithmic byte model of the closest-hit kernel
        traced = st_stats["primary_rays"] + st_stats["secondary_rays"]
        n_node = st_stats["node_visits"] / max(traced, 1)
        n_tri = st_stats["tri_tests"] / max(traced, 1)
        bytes_per_ray = 64 + 32 * n_node + 36 * n_tri
        trace_rays = st_roof["primary_rays"] + st_roof["secondary_rays"]
        model_gbs = (bytes_per_ray * trace_rays / max(st_roof["trace_launches"], 1)) / (trace_avg * 1e-3) / 1e9 \
            if trace_avg > 0 else 0.0
        model = {"bytes_per_ray": round(bytes_per_ray, 1), "n_node": round(n_node, 2), "n_tri": round(n_tri, 2),
                 "achieved": round(model_gbs, 1), "unit": "GB/s",
                 "frac_of_hbm_peak": round(model_gbs / HBM_PEAK_GBS, 4),
                 "frac_of_l2_peak": round(model_gbs / L2_PEAK_GBS, 4),
                 "note": "node / triangle bytes the traversal requests; most are served by the vL1D / L2 "
                         "(compare kernels.k_trace.hbm), so this is not an HBM roofline"}
        tr = kern.get("k_trace", {})
        roof = {"bound": "valu", "kernel": "k_trace<false,false,*> (closest hit; GEN=true generates the primary "
                                           "rays at level 0, GEN=false traces secondary levels)",
                "achieved": tr.get("valu", {}).get("achieved"), "peak": VALU_PEAK_GIPS, "unit": "G wave-inst/s",
                "frac": tr.get("valu", {}).get("frac"),
                "traffic": tr.get("hbm", {}).get("bytes_per_launch"),
                "traffic_unit": "HBM bytes per launch (PMC FETCH_SIZE x 2 + WRITE_SIZE, profiles/counters_current.json)",
                "peak_source": "MI355X_MICROARCH.md: 256 CUs x 4 SIMD-32, wave64 VALU instruction per 2 cycles, 2400 MHz",
                "avg_launch_ms": round(trace_avg, 4), "launches": st_roof["trace_launches"],
                "timing": "HIP events around each launch in a streams=1 frame outside the timed region",
                "counters": counters.get("source"), "roofline_frame_ms": round(st_roof["render_ms"], 2),
                "kernels": kern, "model": model}
        fb = frame_hbm_bytes(counters, shade_names[0], st_roof["shade_launches"]) if (same_wl and shade_names) else None
        if fb:
            roof["frame_hbm"] = {"bytes_per_frame": round(fb), "achieved": round(fb / (ms_per_step * 1e-3) / 1e9, 1),
                                 "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                 "frac": round(fb / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
        cpu = None
        if not args.no_cpu and world == 1:
            log("[rank 0] cpu baseline ...")
            cpu = cpu_baseline(scene, args.cpu_rows, args.cpu_threads)
        if world == 1:
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
                "end_to_end_ms": {"scene_create": round(create_ms, 1), "first_frame_to_host": round(first_frame_ms, 1),
                                  "total": round(create_ms + first_frame_ms, 1),
                                  "note": "rtg_scene_create (BVH build + upload) + the first frame incl. its D2H copy"},
                "rays_rank0": {k: st[k] for k in ("primary_rays", "secondary_rays", "shadow_rays")},
                "kernel_ms_rank0_streams1": {"trace": round(st_roof["trace_ms"], 2), "shade": round(st_roof["shade_ms"], 2),
                                             "shadow": round(st_roof["shadow_ms"], 2)},
                "roofline": roof, "cpu_baseline": cpu}
        print(json.dumps(line), flush=True)
    if comm is not None:
        comm.close()
    r.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
