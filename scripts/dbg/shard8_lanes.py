"""N=8 shard: pass size x lanes, repeated (median of 3 runs of 5 frames), max over 3 ranks."""
import statistics, sys, time
sys.path[:0] = ['raytracer-795_amd']
import torch
import rtg
from rtg import scenegen
from rtg.shard import shard_opts
sc = scenegen.dragon1m(1920, 1080, spp=64)
r = rtg.Renderer(sc, device=0)
frame = torch.zeros((1080, 1920, 3), device="cuda:0")
st = torch.cuda.current_stream().cuda_stream


def timed(**kw):
    r.render_device(0, frame.data_ptr(), st, **kw)
    torch.cuda.synchronize()
    runs = []
    for _ in range(3):
        t = time.perf_counter()
        for _ in range(5):
            r.render_device(0, frame.data_ptr(), st, **kw)
        torch.cuda.synchronize()
        runs.append((time.perf_counter() - t) / 5 * 1e3)
    return statistics.median(runs)


for mb, lanes in [tuple(float(x) for x in c.split(":")) for c in (sys.argv[1] if len(sys.argv) > 1 else "0:0,2:8,3:4,2:8,0:0,3:4,2.5:5,2.5:4").split(",")]:
    lanes = int(lanes)
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    ranks = (0, 1, 5) if N == 8 else tuple(range(N))[:3]
    ts = [timed(**shard_opts(rank, N), streams=lanes, max_batch_rays=int(mb * (1 << 20))) for rank in ranks]
    print(f"N={N} batch={mb}M lanes={lanes}: ranks{ranks} " + " ".join(f"{t:.2f}" for t in ts) +
          f"  max {max(ts):.2f} passes={r.stats()['passes']}", flush=True)
