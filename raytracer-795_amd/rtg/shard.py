"""Multi-GPU pixel sharding.

Rank r of G renders the rows y with (y // B) % G == r, B = ROW_BLOCK = 4 (the reference
interleaves pixel columns over its 8 threads, src/Scene.cpp:269-292; the library tiles a
shard's pixels 16x4 for B = 4, so each tile stays image-contiguous and its rays as coherent
as on one GPU, while 270 blocks over the ranks keep their loads balanced) into a
zero-initialised full-frame accumulator, or compactly (gather_frame).  Summing the G frames is exact because
their supports are disjoint (x + 0 == x), so one reduce (RCCL over xGMI on GPUs, gloo on
CPU) yields the single-device frame bit for bit.
"""
from __future__ import annotations

import numpy as np


ROW_BLOCK = 4


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


def gather_frame(part, frame, rank: int, world: int, dist, block: int = ROW_BLOCK, dst: int = 0):
    """Collect the ranks' compact owned-row buffers (`part`: (max_rows, nx, 3), rows beyond the
    rank's own count unused) onto `dst` and place them in `frame` ((ny, nx, 3), same device).
    One gather of 1/G of the frame per rank instead of a full-frame reduce: rank `dst` receives
    G-1 buffers over its point-to-point links; exact (a copy, not a sum)."""
    import torch

    ny = frame.shape[0]
    if dist is None or not dist.is_initialized() or world == 1:
        rows = _row_index(ny, rank, world, block, frame.device)
        frame.index_copy_(0, rows, part[:len(rows)])
        return frame
    staged = part.is_cuda and dist.get_backend() == "gloo"   # gloo gathers host tensors only
    src = part.cpu() if staged else part
    key = (id(part), world, staged)
    if rank == dst and _GATHER_BUFS.get("key") != key:
        _GATHER_BUFS.update(key=key, bufs=[torch.empty_like(src) for _ in range(world)])
    parts = _GATHER_BUFS["bufs"] if rank == dst else None
    dist.gather(src, parts, dst=dst)
    if staged and rank == dst:
        parts = [q.to(frame.device) for q in parts]
    if rank == dst:
        for r in range(world):
            rows = _row_index(ny, r, world, block, frame.device)
            frame.index_copy_(0, rows, parts[r][:len(rows)])
    return frame


_GATHER_BUFS: dict = {}
_ROW_INDEX: dict = {}


def _row_index(ny, rank, world, block, device):
    """Owned-row index tensor on `device`, built once (no host->device copy per frame)."""
    import torch

    k = (ny, rank, world, block, str(device))
    if k not in _ROW_INDEX:
        _ROW_INDEX[k] = torch.as_tensor(owned_rows(ny, rank, world, block), device=device)
    return _ROW_INDEX[k]


def exchange_comm_id(dist, rank: int, make_id, group=None) -> bytes:
    """Rank 0's communicator id (make_id(): rtg.Comm.unique_id) to every rank -- the set-up of the
    one-process-per-GPU path (bench.py N > 1).  Bounded: the broadcast runs on `group` (a gloo group;
    default: the default group), whose timeout the caller sets at init_process_group / new_group, so a
    peer that died or never joined makes every other rank raise RuntimeError instead of blocking.
    The librtg side bounds its own waits (rtg.Comm(timeout_ms=...), rtg_comm_init_rank_timeout)."""
    obj = [make_id() if rank == 0 else None]
    try:
        dist.broadcast_object_list(obj, src=0, group=group)
    except Exception as e:          # gloo: peer closed / timed out
        raise RuntimeError(f"rank {rank}: communicator id exchange failed (a peer did not join): {e}") from e
    if not isinstance(obj[0], (bytes, bytearray)) or len(obj[0]) != 128:
        raise RuntimeError(f"rank {rank}: bad communicator id from rank 0")
    return bytes(obj[0])


def max_shard_rows(ny: int, world: int, block: int = ROW_BLOCK) -> int:
    return max(len(owned_rows(ny, r, world, block)) for r in range(world))


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
