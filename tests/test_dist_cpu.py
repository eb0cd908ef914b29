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
        bench.init_side_group()  # the cross-GPU leg's CPU-side waits
        bench.side_barrier(w)
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


def _cfg5_worker(rank, world, port, q, per_table):
    """Rank `rank` builds its key range of the cfg 5 tables exactly as
    bench.compaction_leg does (on the CPU), compacts it with the oracle (the
    reference loop, src/sstable/manager.rs:199-234) and gathers every rank's
    slices and outputs over gloo."""
    import numpy as np
    from horreum_amd import synth
    from oracle import oracle
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        datas = []
        for t, keys in enumerate(bench.cfg5_rank_keys(rank, 3, per_table)):
            buf, _ = synth.keyed_table(keys, np.full(keys.size, 100),
                                       seed=bench.cfg5_value_seed(rank, t), device="cpu")
            datas.append(buf.numpy())
        out, _, n = oracle.compacted_table(datas)
        got = [None] * world
        dist.all_gather_object(got, (rank, [d.tobytes() for d in datas], out.tobytes(), n))
        q.put(got if rank == 0 else None)
    finally:
        dist.destroy_process_group()


def test_cfg5_key_range_split_gloo():
    """The N > 1 cfg 5 leg splits the compaction by key range with no data
    movement: rank r compacts range r of every table.  Over gloo, world size 2:
    the ranks' ranges are disjoint and ascending, and their compacted outputs
    concatenated in rank order equal the compaction of the whole tables (each
    table = its ranges concatenated in rank order), byte for byte."""
    import numpy as np
    from oracle import oracle
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_cfg5_worker, args=(r, world, port, q, 3000)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    got = sorted(next(r for r in res if r is not None))
    whole = [np.frombuffer(b"".join(g[1][t] for g in got), np.uint8) for t in range(3)]
    want, _, wn = oracle.compacted_table(whole)
    assert sum(g[3] for g in got) == wn
    assert b"".join(g[2] for g in got) == want.tobytes()
    # disjoint ascending ranges: rank 0's largest key < rank 1's smallest
    k0 = bench.cfg5_rank_keys(0, 3, 3000)
    k1 = bench.cfg5_rank_keys(1, 3, 3000)
    assert max(int(k[-1]) for k in k0) < min(int(k[0]) for k in k1)
