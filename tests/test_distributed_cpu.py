"""Replica sharding + end-of-run gather, world size 2 over gloo on CPU."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from spgg_amd.distributed import gather_rows, shard, shard_range


@pytest.mark.parametrize("n,world", [(0, 2), (1, 2), (7, 2), (105, 8), (64, 8), (5, 3), (8, 1)])
def test_shard_range_partitions(n, world):
    seen = []
    sizes = []
    for r in range(world):
        a, b = shard_range(n, world, r)
        seen.extend(range(a, b))
        sizes.append(b - a)
    assert seen == list(range(n))
    assert max(sizes) - min(sizes) <= 1
    assert sum(len(shard(list(range(n)), world, r)) for r in range(world)) == n


def test_shard_range_rejects_bad_rank():
    with pytest.raises(ValueError):
        shard_range(10, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        a, b = shard_range(n, world, rank)
        local = np.array([[i, i * 0.5, -i] for i in range(a, b)], dtype=np.float64).reshape(-1, 3)
        out = gather_rows(local, n)
        root = gather_rows(local, n, dst=1)   # to rank 1 only
        q.put((rank, out, root))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n", [7, 2, 1])
def test_gather_rows_world2_gloo(n):
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = np.array([[i, i * 0.5, -i] for i in range(n)], dtype=np.float64)
    for rank, out, root in res:
        assert np.array_equal(out, want)
        if rank == 1:
            assert np.array_equal(root, want)
        else:
            assert root is None
