#!/usr/bin/env python3
"""BASELINE config 5 at full size, one GPU's share: the 8 sorted 8 GiB
SSTables of cfg 5 split by key range over 8 GPUs give each GPU 1 GiB of every
table, i.e. 8 tables x 1 GiB (16 B keys / 100 B values, 25 % of each table's
keys shared by all tables).  Decode all 8 -> newest-wins merge -> encode,
device resident (median of 3, two host syncs inside as in bench.py's
compaction leg), then the same through hg_compact_host from pageable host
memory (H2D of every table + D2H of the compacted table included).

Parity (size-independent, on the device): the compacted table must equal the
records of the key union, each taken from the first (newest) table holding
the key -- built here by a stable sort of (key, table) -- byte for byte.
Every record is 132 bytes, so the expected table is one gather of rows."""
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

GIB = float(1 << 30)
NTAB = 8
PER_TABLE = int(os.environ.get("CFG5_PER_TABLE", 8_134_407))  # 1 GiB of 132 B records
REC = 132


def main():
    eng = Engine(0)
    dev = eng.device
    rng = np.random.default_rng(5)
    t_gen = time.perf_counter()
    shared = np.unique(rng.integers(0, 1 << 40, size=PER_TABLE // 4, dtype=np.uint64))
    keys, bufs = [], []
    for t in range(NTAB):
        own = rng.integers(0, 1 << 40, size=PER_TABLE - shared.size, dtype=np.uint64)
        k = np.unique(np.concatenate([shared, own]))
        buf, _ = synth.keyed_table(k, np.full(k.size, 100), seed=50 + t, device=dev)
        keys.append(k)
        bufs.append(buf)
    sizes = [b.numel() for b in bufs]
    print(json.dumps({"generated_s": round(time.perf_counter() - t_gen, 1),
                      "table_bytes": sizes}), flush=True)

    # expected output rows: stable sort by key keeps the newest table first
    allk = np.concatenate(keys)
    tid = np.concatenate([np.full(k.size, t, np.int64) for t, k in enumerate(keys)])
    row = np.concatenate([np.arange(k.size, dtype=np.int64) for k in keys])
    order = np.argsort(allk, kind="stable")
    ks = allk[order]
    first = np.ones(ks.size, bool)
    first[1:] = ks[1:] != ks[:-1]
    base = np.zeros(NTAB + 1, np.int64)
    np.cumsum([k.size for k in keys], out=base[1:])
    want_rows = torch.from_numpy(base[tid[order][first]] + row[order][first]).to(dev)
    n_want = int(first.sum())
    del allk, tid, row, order, ks, first

    offs_b, total = [], 0
    for sz in sizes:
        offs_b.append(total)
        total += (sz + 7) & ~7
    arena = torch.zeros(total, dtype=torch.uint8, device=dev)
    for o, b in zip(offs_b, bufs):
        arena[o:o + b.numel()] = b
    hosts = [b.cpu().numpy() for b in bufs]
    caps = [sz // 16 for sz in sizes]
    span_t = [eng.empty(c * 16) for c in caps]
    nmax = sum(caps)
    pairs = eng.empty(nmax * 24)
    out = eng.empty(total)
    eng.reserve(max(sizes), nmax)
    tabs = [arena[o:o + sz] for o, sz in zip(offs_b, sizes)]
    dres = eng.empty(24 * NTAB)

    def run():
        eng.decode_batch_dev_async(tabs, sizes, span_t, caps, dres)
        r = dres.cpu().numpy()
        counts = [int(r[24 * i:24 * i + 8].view("<u8")[0]) for i in range(NTAB)]
        assert all(int(r[24 * i + 8:24 * i + 12].view("<i4")[0]) == 0 for i in range(NTAB))
        m = eng.merge_dev(arena, offs_b, span_t, counts, pairs, nmax)
        rc, out_len = eng.encode_dev(arena, pairs, m.n, out=out, cap=total)
        return m, out_len

    run()
    torch.cuda.synchronize(dev)
    times = []
    for _ in range(3):
        t0 = time.perf_counter()
        m, out_len = run()
        torch.cuda.synchronize(dev)
        times.append(time.perf_counter() - t0)
    wall = sorted(times)[1]
    in_bytes = sum(sizes)
    rows = torch.cat(bufs).view(-1, REC)
    want = rows.index_select(0, want_rows).view(-1)
    ok = (int(m.n) == n_want and out_len == n_want * REC
          and bool(torch.equal(out[:out_len], want)))
    del rows, want, arena, span_t, pairs, tabs, bufs
    torch.cuda.empty_cache()
    line = {"workload": "cfg5 full size, one GPU's share: 8 tables x 1 GiB, 16 B / 100 B, 25 % shared",
            "input_bytes": in_bytes, "merged_records": int(m.n), "merged_bytes": int(out_len),
            "device_ms": round(wall * 1e3, 3), "device_GiB_s": round(in_bytes / wall / GIB, 2),
            "device_times_ms": [round(t * 1e3, 3) for t in times], "parity": ok}
    print(json.dumps(line), flush=True)

    hout = np.empty(in_bytes, dtype=np.uint8)
    host_out = out[:out_len].cpu().numpy()
    del out
    torch.cuda.empty_cache()
    c = eng.compact_host(hosts, out=hout)  # warm-up (staging buffers, workspaces)
    ht = []
    for _ in range(3):
        t0 = time.perf_counter()
        c = eng.compact_host(hosts, out=hout)
        ht.append(time.perf_counter() - t0)
    t = sorted(ht)[1]
    hok = c.status == 0 and c.n == m.n and np.array_equal(c.data, host_out)
    line["host_inclusive"] = {"ms": round(t * 1e3, 1), "GiB_s": round(in_bytes / t / GIB, 2),
                              "times_ms": [round(x * 1e3, 1) for x in ht], "parity": bool(hok)}
    print(json.dumps(line), flush=True)
    return 0 if ok and hok else 1


if __name__ == "__main__":
    sys.exit(main())
