#!/usr/bin/env python3
"""Time the batched multi-table decode (BASELINE cfg 4, one GPU's share:
32 tables of <= 64 MiB, 16 B keys, values uniform in [8, 4096] B, ~5 %
tombstones) and check every table against the oracle."""
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


def main():
    ntab = int(os.environ.get("NTAB", "32"))
    eng = Engine(0)
    dev = eng.device
    tabs = []
    for t in range(ntab):
        v = synth.mixed_table_vlens(64 << 20, 8, 4096, 0.05, seed=4 + t)
        keys = np.arange(v.size, dtype=np.uint64) * 7 + t
        buf, _ = synth.keyed_table(keys, v, seed=4 + t, device=dev)
        tabs.append((buf, v.size))
    bufs = [b for b, _ in tabs]
    lens = [b.numel() for b in bufs]
    caps = [n for _, n in tabs]
    spans = [eng.empty(n * 16) for n in caps]
    res = eng.empty(24 * ntab)
    for _ in range(2):
        eng.decode_batch_dev_async(bufs, lens, spans, caps, res)
    torch.cuda.synchronize()
    ts = []
    for _ in range(int(os.environ.get("REPS", "8"))):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        eng.decode_batch_dev_async(bufs, lens, spans, caps, res)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    # back to back (the bench leg's timing): 10 calls in one event pair
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        eng.decode_batch_dev_async(bufs, lens, spans, caps, res)
    e1.record()
    torch.cuda.synchronize()
    b2b = e0.elapsed_time(e1) / 10
    r = res.cpu().numpy()
    ok = True
    for i in range(min(ntab, int(os.environ.get("CHECK", "4")))):
        want, wn, wk, _, _ = oracle.decode(bufs[i].cpu().numpy())
        n = int(r[24 * i:24 * i + 8].view("<u8")[0])
        got = spans[i][: n * 16].cpu().numpy().view(oracle.SPAN_DTYPE)
        ok &= n == wn and np.array_equal(got, want)
    total = sum(lens)
    ms = float(np.median(ts))
    print(json.dumps({"tables": ntab, "bytes": total, "records": sum(caps), "ms": round(ms, 4),
                      "b2b_ms": round(b2b, 4),
                      "GiBps": round(total / ms / 1e6 / 1.073741824, 1),
                      "streams": os.environ.get("HG_DECODE_STREAMS", "4"), "parity": bool(ok)}),
          flush=True)


if __name__ == "__main__":
    main()
