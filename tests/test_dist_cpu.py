"""bench.py's multi-rank logic on CPU with the gloo backend, world_size 2:
per-rank shards are independent tables (different seeds, identical shapes),
the timing barrier holds, MAX-over-ranks picks the slowest rank, and the
whole-job rate is the sum of every rank's bytes over that time."""
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import bench


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        r, w, local = bench.dist_env()
        plan = bench.shard_plan(r, w)
        bench.barrier(w)
        slowest = bench.max_over_ranks(0.010 * (r + 1), w)  # rank 1 is "slower"
        q.put((r, w, local, plan["seed"], plan["n"], slowest))
    finally:
        dist.destroy_process_group()


def test_two_rank_gloo():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    got = sorted(q.get(timeout=10) for _ in range(world))
    assert [g[0] for g in got] == [0, 1] and all(g[1] == 2 for g in got)
    seeds = [g[3] for g in got]
    assert len(set(seeds)) == 2                       # independent tables per rank
    assert len({g[4] for g in got}) == 1              # same shape: weak scaling
    assert all(g[5] == pytest.approx(0.020) for g in got)  # max over ranks everywhere


def test_aggregate_is_whole_job():
    # 2 ranks x 1 GiB each, 10 steps in 0.01 s of max-rank wall time -> 2000 GiB/s
    assert bench.aggregate(0.01, 10, 2, 1 << 30) == pytest.approx(2000.0)
    assert bench.shard_plan(3, 8)["seed"] == bench.CFG2["seed"] + 3000
