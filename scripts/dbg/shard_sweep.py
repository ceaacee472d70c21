"""N=8 per-rank work on one GPU: batch size x streams sweep."""
import sys, time
sys.path[:0] = ['raytracer-795_amd']
import torch
import rtg
from rtg import scenegen
sc = scenegen.dragon1m(1920, 1080, spp=64)
r = rtg.Renderer(sc, device=0)
frame = torch.zeros((1080, 1920, 3), device="cuda:0")
st = torch.cuda.current_stream().cuda_stream
for N in (8, 4, 1):
    for mb in (8 << 20, 4 << 20, 3 << 20, 2 << 20, 1 << 20):
        for streams in (3, 4, 6):
            if N == 1 and mb < (4 << 20):
                continue
            kw = dict(row_offset=0, row_stride=N, streams=streams, max_batch_rays=mb)
            r.render_device(0, frame.data_ptr(), st, **kw)
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(4):
                r.render_device(0, frame.data_ptr(), st, **kw)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t) / 4 * 1e3
            print(f"N={N} batch={mb >> 20}M streams={streams}: {ms:.2f} ms passes={r.stats()['passes']}", flush=True)
