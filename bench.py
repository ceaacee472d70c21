"""Benchmark: Mray/s + ms/frame at 1920x1080, 64 spp (BASELINE.json metric) on the
C3 `dragon1m` scene (1,000,000-triangle BVH, mirror + dielectric spheres, Whitted depth 6).

One step = one full frame.  With N ranks (torch.distributed.run, one GPU each) every rank
renders the rows y % N == rank into a zero-initialised full-frame accumulator and the
frames are summed onto rank 0 with one RCCL reduce (exact: disjoint pixel support).
value = rays traced by all ranks / max-over-ranks frame time.

Prints ONE JSON line (rank 0).  Extra objects:
  roofline     dominant kernel k_trace (closest hit), algorithmic bytes per launch from the
               SURVEY §8(d) model B = 64 + 32*N_node + 36*N_tri per ray (N_* measured by a
               stats frame outside the timed region), divided by its HIP-event launch time.
  cpu_baseline the CPU restatement (oracle/) on a bounded row sample of the same frame.
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
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def pmc_traffic(kernel: str):
    """HBM bytes per launch of `kernel` from the last committed PMC passes (separate
    `rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE` runs of this bench, gfx950-corrected by
    scripts/pmc_traffic.py); None when absent."""
    p = os.path.join(ROOT, "profiles", "traffic_current.json")
    try:
        with open(p) as f:
            k = json.load(f)["kernels"].get(kernel)
        return None if k is None else k["hbm_bytes_per_launch"]
    except (OSError, ValueError, KeyError):
        return None


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
    args = ap.parse_args()

    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # RTG_BENCH_REHEARSE=1: rehearse the N>1 path on a 1-GPU box (every rank on cuda:0, gloo
    # collectives through host memory); the numbers of such a run are not a scaling measurement
    rehearse = os.environ.get("RTG_BENCH_REHEARSE") == "1"
    if rehearse:
        local = 0
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(local)

    import rtg

    t0 = time.perf_counter()
    from rtg import scenegen
    from rtg.shard import ROW_BLOCK, gather_frame, max_shard_rows, shard_opts
    make, spp_default, wl_text, data_text = WORKLOADS[args.workload]
    scene = getattr(scenegen, make)(args.width, args.height, spp=args.spp or spp_default)
    log(f"[rank {rank}] scene: {scene.num_triangles()} triangles, gen {time.perf_counter() - t0:.1f}s")
    t0 = time.perf_counter()
    r = rtg.Renderer(scene, device=local)
    log(f"[rank {rank}] rtg_scene_create (BVH build + upload) {time.perf_counter() - t0:.1f}s")
    cam = scene.cameras[0]
    frame = torch.zeros((cam.ny, cam.nx, 3), dtype=torch.float32, device=f"cuda:{local}")
    stream = torch.cuda.current_stream().cuda_stream
    # N > 1: each rank renders its owned rows compactly (1/N of the frame) and rank 0 gathers
    # them over RCCL (point-to-point xGMI) into the frame — exact, and 1/N of a reduce's bytes
    part = (torch.zeros((max_shard_rows(cam.ny, world), cam.nx, 3), dtype=torch.float32, device=frame.device)
            if world > 1 else None)

    def step(**kw):
        if part is None:
            r.render_device(0, frame.data_ptr(), stream, **kw)
            return r.stats()
        r.render_device(0, part.data_ptr(), stream, **shard_opts(rank, world), compact_rows=1, **kw)
        st = r.stats()
        gather_frame(part, frame, rank, world, dist)
        return st

    # traversal statistics for the roofline model (outside the timed region)
    st_stats = step(collect_stats=1)
    # roofline frame (outside the timed region): passes one at a time (streams=1) so every
    # closest-hit launch is timed alone by its HIP events; the timed frames below overlap
    # passes on several streams, where an event pair would also count the other streams' work
    # (twice: the first streams=1 frame also grows that lane's level buffers — hipMalloc of
    # fresh memory — so only the second one's frame time is representative)
    step(collect_timing=1, streams=1)
    st_roof = step(collect_timing=1, streams=1)
    for _ in range(args.warmup):
        step()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rays = 0
    for i in range(args.steps):
        st = step()
        rays += st["total_rays"]
        log(f"[rank {rank}] step {i}: {st['render_ms']:.1f} ms device, rays {st['total_rays']}")
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=frame.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        rt = torch.tensor([rays], dtype=torch.float64, device=frame.device)
        dist.all_reduce(rt, op=dist.ReduceOp.SUM)
        rays = int(rt.item())
    trace_ms = st_roof["trace_ms"]
    trace_launches = st_roof["trace_launches"]
    trace_rays = st_roof["primary_rays"] + st_roof["secondary_rays"]

    ms_per_step = elapsed * 1e3 / args.steps
    value = rays / elapsed / 1e6
    # roofline of the dominant kernel (closest-hit trace)
    traced = st_stats["primary_rays"] + st_stats["secondary_rays"]
    n_node = st_stats["node_visits"] / max(traced, 1)
    n_tri = st_stats["tri_tests"] / max(traced, 1)
    bytes_per_ray = 64 + 32 * n_node + 36 * n_tri
    avg_launch_ms = trace_ms / max(trace_launches, 1)
    bytes_per_launch = bytes_per_ray * trace_rays / max(trace_launches, 1)
    achieved = bytes_per_launch / (avg_launch_ms * 1e-3) / 1e9 if avg_launch_ms > 0 else 0.0
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": pmc_traffic("rtg::k_trace<false, false, *>") if args.workload == "dragon1m" else None,
            "traffic_unit": "bytes/launch (PMC, profiles/traffic_current.json)",
            "kernel": "k_trace<false,false,*> (closest hit: GEN=true generates the primary rays at level 0, GEN=false traces secondary levels)",
            "avg_launch_ms": round(avg_launch_ms, 3), "launches": trace_launches,
            "bytes_per_ray": round(bytes_per_ray, 1), "n_node": round(n_node, 2), "n_tri": round(n_tri, 2),
            "timing": "HIP events around each launch in a streams=1 frame outside the timed region",
            "roofline_frame_ms": round(st_roof["render_ms"], 2)}

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
        cpu = None
        if not args.no_cpu and world == 1:
            log("[rank 0] cpu baseline ...")
            cpu = cpu_baseline(scene, args.cpu_rows, args.cpu_threads)
        line = {"metric": METRIC, "value": round(value, 2), "unit": "Mray/s", "n_gpus": world,
                "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 2),
                "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
                "data": data_text,
                "config": {"workload": wl_text,
                           "resolution": f"{cam.nx}x{cam.ny}", "spp": cam.num_samples,
                           "parallelism": (f"{ROW_BLOCK}-row-block interleaved pixel shards x{world} + "
                                           + ("gloo gather (rehearsal, all ranks on one GPU)" if rehearse
                                              else "RCCL gather") if world > 1 else "single GPU")},
                "rays_per_frame": rays // max(args.steps, 1),
                "rays_rank0": {k: st[k] for k in ("primary_rays", "secondary_rays", "shadow_rays")},
                "kernel_ms_rank0_streams1": {"trace": round(st_roof["trace_ms"], 2),
                                             "shadow": round(st_roof["shadow_ms"], 2)},
                "roofline": roof, "cpu_baseline": cpu}
        print(json.dumps(line), flush=True)
    r.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
