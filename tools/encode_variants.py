#!/usr/bin/env python3
"""Time hg_encode_dev_async on BASELINE cfg 3 (10 M pairs, 32 B keys / 256 B
values, contiguous arena) and on a mixed-size arena (16..48 B keys,
0..600 B values, shuffled pair order); median of 7 launches, outputs checked
(cfg 3: body bytes == arena rows and headers; mixed: against the oracle)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from horreum_amd import synth  # noqa: E402
from horreum_amd.engine import Engine  # noqa: E402
from horreum_amd import abi as _abi  # noqa: E402
_abi.knobs_from_env()  # the A/B scripts' HG_* knobs (the library reads no environment)
from oracle import oracle  # noqa: E402


def timed(eng, arena, pairs, n, out, total, res, reps=7):
    ts = []
    for i in range(reps + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        eng.encode_dev_async(arena, pairs, n, out, total, None, 0, None, res)
        e1.record()
        torch.cuda.synchronize()
        if i:
            ts.append(e0.elapsed_time(e1))
    return float(np.median(ts))


def main():
    eng = Engine(0)
    dev = eng.device
    res = eng.empty(64)
    n, k, v = 10_000_000, 32, 256
    arena, pairs = synth.fixed_arena(n, k, v, seed=3, device=dev)
    total = n * (16 + k + v)
    out = eng.empty(total)
    eng.reserve(0, n)
    ms = timed(eng, arena, pairs, n, out, total, res)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()  # back to back (the bench leg's timing): 10 calls in one event pair
    for _ in range(10):
        eng.encode_dev_async(arena, pairs, n, out, total, None, 0, None, res)
    e1.record()
    torch.cuda.synchronize()
    b2b = e0.elapsed_time(e1) / 10
    rr = out.view(n, 16 + k + v)
    ok = torch.equal(rr[:, 16:], arena.view(n, k + v)) and bool(
        (rr[:, :16].contiguous().view(torch.int64) == torch.tensor([k, v], device=dev)).all())
    alg = n * (k + v) + 24 * n + total
    print(json.dumps({"workload": "cfg3 32B/256B 10M", "ms": round(ms, 4), "b2b_ms": round(b2b, 4),
                      "GBps_alg": round(alg / ms / 1e6, 1), "parity": bool(ok)}), flush=True)
    # practical ceiling for this traffic: a device copy of the same output size
    src = torch.empty(total, dtype=torch.uint8, device=dev)
    ts = []
    for i in range(8):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out.copy_(src)
        e1.record()
        torch.cuda.synchronize()
        if i:
            ts.append(e0.elapsed_time(e1))
    cms = float(np.median(ts))
    print(json.dumps({"workload": "torch d2d copy, same bytes", "ms": round(cms, 4),
                      "GBps_rw": round(2 * total / cms / 1e6, 1)}), flush=True)
    del arena, pairs, out, rr, src
    torch.cuda.empty_cache()
    rng = np.random.default_rng(5)
    m = 2_000_000
    kl = rng.integers(16, 49, m)
    vl = rng.integers(0, 601, m)
    offs = np.concatenate([[0], np.cumsum(kl + vl)])
    ha = rng.integers(0, 256, int(offs[-1]), dtype=np.uint8)
    hp = np.zeros(m, dtype=oracle.PAIR_DTYPE)
    hp["key_off"], hp["val_off"], hp["klen"], hp["vlen"] = offs[:-1], offs[:-1] + kl, kl, vl
    hp = hp[rng.permutation(m)]
    want, _, _, _ = oracle.encode(ha, hp)
    arena, pairs = eng.to_device(ha), eng.to_device(hp.view(np.uint8))
    out = eng.empty(want.size)
    eng.reserve(0, m)
    ms = timed(eng, arena, pairs, m, out, want.size, res)
    ok = np.array_equal(out.cpu().numpy()[: want.size], want)
    alg = int((kl + vl).sum()) + 24 * m + want.size
    print(json.dumps({"workload": "mixed 16..48B/0..600B shuffled 2M", "bytes": int(want.size),
                      "ms": round(ms, 4), "GBps_alg": round(alg / ms / 1e6, 1), "parity": bool(ok)}),
          flush=True)


if __name__ == "__main__":
    main()
