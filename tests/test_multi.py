"""N>1 path on CPU: world_size-2 gloo rehearsal of bench.py's sharding and timing reduction."""
import os
import socket

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


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    seeds = bench.shard_seeds(1000, rank, 5)
    out = [None] * world
    dist.all_gather_object(out, seeds)
    tmax = bench.reduce_max(float(rank + 1) * 0.5, dist, "cpu")
    if rank == 0:
        q.put((out, tmax))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharding_and_max_reduction(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    shards, tmax = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    flat = [s for sh in shards for s in sh]
    assert len(flat) == len(set(flat)) == 5 * world          # disjoint shards
    assert sorted(flat) == list(range(1000, 1000 + 5 * world))  # covering the job
    assert tmax == 0.5 * world                                  # slowest rank's time
