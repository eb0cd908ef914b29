#!/usr/bin/env python3
"""Compaction of 8 tables x 1 M records (cfg 5's shape: 16 B keys / 100 B
values, 25 % shared keys) through hg_compact_dev: sorted tables (the parallel
merge), one duplicate key late in table 3 and one inversion in every table
(the epochs of the reference loop), every table fully shuffled and half of
them shuffled (the rank path: dense key ranks, the loop in one wave), each
checked byte for byte against the oracle's compaction with --check; with
--serial the one-duplicate input also through the round-2 loop over entries
(HG_MERGE_SERIAL=exact).  Prints one JSON line per case (median of 3 wall ms)."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from horreum_amd import synth  # noqa: E402
from horreum_amd.engine import Engine  # noqa: E402
from horreum_amd import abi as _abi  # noqa: E402
_abi.knobs_from_env()  # the A/B scripts' HG_* knobs (the library reads no environment)


def tables(per_table, mode, rng_seed=5):
    rng = np.random.default_rng(rng_seed)
    shared = np.unique(rng.integers(0, 1 << 40, size=per_table // 4, dtype=np.uint64))
    out = []
    for t in range(8):
        own = rng.integers(0, 1 << 40, size=per_table - shared.size, dtype=np.uint64)
        k = np.unique(np.concatenate([shared, own]))
        if mode == "dup" and t == 3:
            j = int(k.size * 0.9)
            k = np.insert(k, j, k[j])
        elif mode == "every":
            j = int(rng.integers(1, k.size - 2))
            k = k.copy()
            k[j], k[j + 1] = k[j + 1], k[j]
        elif mode == "shuffle" or (mode == "half" and t % 2 == 1):
            k = rng.permutation(k)
        out.append(k)
    return out


def run(eng, keys, label, reps=3, check=False):
    dev = eng.device
    bufs = [synth.keyed_table(k, np.full(k.size, 100), seed=50 + t, device=dev)[0]
            for t, k in enumerate(keys)]
    sizes = [b.numel() for b in bufs]
    offs, total = [], 0
    for sz in sizes:
        offs.append(total)
        total += (sz + 7) & ~7
    arena = torch.zeros(total, dtype=torch.uint8, device=dev)
    for o, b in zip(offs, bufs):
        arena[o:o + b.numel()] = b
    hosts = [b.cpu().numpy() for b in bufs] if check else None
    del bufs
    out = eng.empty(total)
    c = eng.compact_dev(arena, offs, sizes, out)
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        c = eng.compact_dev(arena, offs, sizes, out)
        torch.cuda.synchronize(dev)
        ts.append((time.perf_counter() - t0) * 1e3)
    parity = None
    if check:
        from oracle import oracle
        want, _, wn = oracle.compacted_table(hosts)
        got = out[:c.data.numel()].cpu().numpy()
        parity = bool(wn == c.n and np.array_equal(got, want))
    print(json.dumps({"case": label, "records_in": int(sum(k.size for k in keys)),
                      "parity_vs_oracle": parity,
                      "records_out": int(c.n), "status": int(c.status), "table": int(c.table),
                      "epochs": int(c.index) if c.table == 2 else None,
                      "ms": round(sorted(ts)[reps // 2], 3),
                      "times_ms": [round(t, 3) for t in ts]}), flush=True)
    del arena, out
    torch.cuda.empty_cache()


def main():
    per = int(os.environ.get("PER_TABLE", 1_000_000))
    eng = Engine(0)
    run(eng, tables(per, "sorted"), "sorted (parallel merge)")
    run(eng, tables(per, "dup"), "one duplicate key at 0.9 of table 3 (epochs)")
    run(eng, tables(per, "every"), "one inversion in every table (epochs)")
    chk = "--check" in sys.argv
    run(eng, tables(per, "shuffle"), "every table shuffled (rank path)", check=chk)
    run(eng, tables(per, "half"), "tables 1, 3, 5, 7 shuffled (rank path)", check=chk)
    if "--serial" in sys.argv:
        os.environ["HG_MERGE_SERIAL"] = "exact"
        run(eng, tables(per, "dup"), "one duplicate key, serial reference loop (round-2 path)",
            reps=1)


if __name__ == "__main__":
    main()
