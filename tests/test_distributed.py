"""N>1 path on CPU: world_size-2 gloo.  Each rank renders its row shard ((y // 8) % 2 == rank)
and the frames are summed onto rank 0 with one reduce — the same partition + collective
bench.py uses over RCCL.  The oracle stands in for the GPU renderer here (test infra);
the reduced frame must equal the single-process frame bit for bit."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_path):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "raytracer-795_amd"))
    sys.path.insert(0, os.path.join(root, "oracle"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import pyoracle
    from rtg import scenegen
    from rtg.shard import render_sharded

    sc = scenegen.cornell(24, 17, spp=2)
    orc = pyoracle.Oracle(sc)

    def rows(row_offset, row_stride, row_block):
        return orc.render(0, nthreads=1, row_offset=row_offset, row_stride=row_stride, row_block=row_block)[0]

    frame = render_sharded(rows, 17, 24, rank, world, dist)
    if rank == 0:
        np.save(out_path, frame.numpy())
    dist.barrier()
    dist.destroy_process_group()


def _gather_worker(rank, world, port, out_path):
    """bench.py's N>1 exchange: compact owned rows per rank, one gather onto rank 0."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "raytracer-795_amd"))
    sys.path.insert(0, os.path.join(root, "oracle"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import pyoracle
    from rtg import scenegen
    from rtg.shard import gather_frame, max_shard_rows, owned_rows, shard_opts

    sc = scenegen.cornell(24, 19, spp=2)
    full = pyoracle.Oracle(sc).render(0, nthreads=1, **shard_opts(rank, world))[0]
    rows = owned_rows(19, rank, world)
    part = torch.zeros((max_shard_rows(19, world), 24, 3))
    part[:len(rows)] = torch.from_numpy(full[rows])
    frame = torch.full((19, 24, 3), float("nan"))
    gather_frame(part, frame, rank, world, dist)
    if rank == 0:
        np.save(out_path, frame.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_compact_shards_gather_to_single_frame(tmp_path, world):
    import pyoracle
    from rtg import scenegen

    out = str(tmp_path / "frame.npy")
    mp.spawn(_gather_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    got = np.load(out)
    ref = pyoracle.Oracle(scenegen.cornell(24, 19, spp=2)).render(0)[0]
    assert np.array_equal(got.view(np.int32), ref.view(np.int32))


@pytest.mark.parametrize("world", [2])
def test_row_shards_reduce_to_single_frame(tmp_path, world):
    import pyoracle
    from rtg import scenegen

    out = str(tmp_path / "frame.npy")
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    got = np.load(out)
    ref = pyoracle.Oracle(scenegen.cornell(24, 17, spp=2)).render(0)[0]
    assert np.array_equal(got.view(np.int32), ref.view(np.int32))


def test_owned_rows_partition():
    from rtg.shard import owned_rows
    for world in (1, 2, 3, 8):
        for ny, block in ((1080, 8), (1080, 1), (37, 8), (5, 8)):
            rows = np.concatenate([owned_rows(ny, r, world, block) for r in range(world)])
            assert sorted(rows.tolist()) == list(range(ny))
