"""Multi-GPU pixel sharding.

Rank r of G renders the rows y with (y // B) % G == r, B = ROW_BLOCK = 8 (the reference
interleaves pixel columns over its 8 threads, src/Scene.cpp:400-423; 8-row blocks keep
each GPU's 8x8 pixel tiles image-contiguous, so its rays stay as coherent as on one GPU,
while the fine interleave keeps the ranks' loads balanced) into a zero-initialised
full-frame accumulator.  Summing the G frames is exact because
their supports are disjoint (x + 0 == x), so one reduce (RCCL over xGMI on GPUs, gloo on
CPU) yields the single-device frame bit for bit.
"""
from __future__ import annotations

import numpy as np


ROW_BLOCK = 8


def owned_rows(ny: int, rank: int, world: int, block: int = ROW_BLOCK) -> np.ndarray:
    y = np.arange(ny)
    return y[(y // max(block, 1)) % world == rank]


def shard_opts(rank: int, world: int, block: int = ROW_BLOCK) -> dict:
    return {"row_offset": rank, "row_stride": world, "row_block": block}


def reduce_frame(frame, dist, dst: int = 0):
    """Sum the per-rank frames onto `dst` (torch tensor, any backend)."""
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        dist.reduce(frame, dst=dst, op=dist.ReduceOp.SUM)
    return frame


def render_sharded(render_rows, ny: int, nx: int, rank: int, world: int, dist=None):
    """render_rows(**shard_opts(rank, world)) -> (ny, nx, 3) float32 frame with only the owned
    rows written (others zero).  Returns the reduced frame on rank 0 (torch CPU tensor)."""
    import torch

    part = np.asarray(render_rows(**shard_opts(rank, world)), np.float32)
    mask = np.zeros(ny, bool)
    mask[owned_rows(ny, rank, world)] = True
    part = np.where(mask[:, None, None], part, np.float32(0.0)).astype(np.float32)
    t = torch.from_numpy(np.ascontiguousarray(part))
    reduce_frame(t, dist)
    return t
