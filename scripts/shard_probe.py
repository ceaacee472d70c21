"""Per-rank frame time of the N-GPU row shards on one GPU (what each rank of bench.py --gpus N
renders): render_ms of every shard k of N (row_offset k, row_stride N, the bench's row block),
compact owned rows left in HBM.  usage: python scripts/shard_probe.py [N ...]
RTG_PROBE_OPTS="tile_band=16,streams=4" adds render options (integers)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracer-795_amd"))
import torch  # noqa: E402
import rtg  # noqa: E402
from rtg import scenegen  # noqa: E402
from rtg.shard import shard_opts  # noqa: E402

wl = os.environ.get("RTG_WORKLOAD", "dragon1m")      # dragon1m | cornell_pt | cornell | spheres
sc = getattr(scenegen, wl)(1920, 1080) if wl != "dragon1m" else scenegen.dragon1m(1920, 1080, spp=64)
r = rtg.Renderer(sc, 0)
out = torch.empty((1080, 1920, 3), dtype=torch.float32, device="cuda:0")
extra = {k: int(v) for k, v in (kv.split("=") for kv in os.environ.get("RTG_PROBE_OPTS", "").split(",") if kv)}
for n in [int(a) for a in sys.argv[1:]] or [1, 2, 4, 8]:
    ms = []
    for k in range(n):
        kw = dict(shard_opts(k, n), compact_rows=1 if n > 1 else 0,
                  max_batch_rays=int(os.environ.get("RTG_BATCH", "0")), **extra)
        r.render_device(0, out.data_ptr(), **kw)          # warm (buffers sized for this shard)
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(3):
            r.render_device(0, out.data_ptr(), **kw)
            torch.cuda.synchronize()
            best = min(best, r.stats()["render_ms"])
        ms.append(best)
    print(f"{wl} batch={os.environ.get('RTG_BATCH', '0')} opts={extra} N={n}: per-rank render_ms max {max(ms):.2f} min {min(ms):.2f}", flush=True)
if os.environ.get("RTG_KT"):
    # per-kernel device time of one frame with the passes serialised (streams=1, HIP events)
    r.render_device(0, out.data_ptr(), collect_timing=1, streams=1)
    torch.cuda.synchronize()
    st = r.stats()
    print(f"  kernels (streams=1): trace {st['trace_ms']:.2f} shade {st['shade_ms']:.2f} shadow {st['shadow_ms']:.2f} "
          f"render {st['render_ms']:.2f} ms", flush=True)
