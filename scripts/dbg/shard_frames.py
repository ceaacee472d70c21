"""Render one multi-GPU rank's row shard K times into device memory (workload for rocprof)."""
import os, sys
sys.path[:0] = ['raytracer-795_amd']
import torch
import rtg
from rtg import scenegen
from rtg.shard import shard_opts
N, K = int(sys.argv[1]), int(sys.argv[2])
rank = int(sys.argv[3]) if len(sys.argv) > 3 else 0
sc = scenegen.dragon1m(1920, 1080, spp=64)
r = rtg.Renderer(sc, device=0)
frame = torch.zeros((1080, 1920, 3), device="cuda:0")
st = torch.cuda.current_stream().cuda_stream
for _ in range(K):
    r.render_device(0, frame.data_ptr(), st, **shard_opts(rank, N))
torch.cuda.synchronize()
print("ms", r.stats()["render_ms"])
