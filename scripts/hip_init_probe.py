"""One-time costs of the HIP runtime in a fresh process after torch's device init: a kernel first, then pinned, then
pageable host-to-device copies (12 MB), device-to-host copies, each twice.
usage: python scripts/hip_init_probe.py"""
import time

import torch

torch.cuda.set_device(0)
torch.cuda.synchronize()


def timed(what, f):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = f()
    torch.cuda.synchronize()
    print(f"{what:40s} {(time.perf_counter() - t0) * 1e3:8.2f} ms", flush=True)
    return r


n = 3 << 20
src = torch.arange(n, dtype=torch.float32)
for k in range(2):
    d = timed(f"[{k}] device alloc 12 MB", lambda: torch.empty(n, device="cuda"))
    timed(f"[{k}] first kernel (fill)", lambda: d.fill_(1.0))
    timed(f"[{k}] second kernel (fill)", lambda: d.fill_(2.0))
    pin = timed(f"[{k}] pinned host alloc 12 MB", lambda: torch.empty(n, pin_memory=True))
    pin.copy_(src)
    timed(f"[{k}] H2D pinned 12 MB", lambda: d.copy_(pin, non_blocking=True))
    timed(f"[{k}] D2H pinned 12 MB", lambda: pin.copy_(d, non_blocking=True))
    timed(f"[{k}] H2D pageable 12 MB", lambda: d.copy_(src))
    timed(f"[{k}] D2H pageable 12 MB", lambda: src.copy_(d))
    d2 = torch.empty(16 << 20, device="cuda")
    timed(f"[{k}] D2H pageable 64 MB", lambda: d2.cpu())
