#!/usr/bin/env python3
"""Decode time of small records whose values are zero bytes (the lane-walk
guesses' worst case: every 16 bytes of a value read as a header candidate),
checked against the oracle; A/B tool for the guess rules.  `--midlarge`:
400-1200 B zero values instead."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from horreum_amd.engine import Engine  # noqa: E402
from horreum_amd import abi as _abi  # noqa: E402
_abi.knobs_from_env()  # the A/B scripts' HG_* knobs (the library reads no environment)
from oracle import oracle  # noqa: E402


def main():
    rng = np.random.default_rng(9)
    if "--midlarge" in sys.argv:  # 16 B keys, 400-1200 B zero values (~816 MB)
        m = 1_000_000
        kl = np.full(m, 16)
        vl = rng.integers(400, 1201, m)
    else:
        m = 3_000_000
        kl = rng.integers(1, 24, m)
        vl = rng.integers(0, 64, m)
    offs = np.concatenate([[0], np.cumsum(16 + kl + vl)])
    buf = np.zeros(int(offs[-1]), np.uint8)
    hdr = np.stack([kl, vl], axis=1).astype("<u8").view(np.uint8).reshape(m, 16)
    for i in range(16):
        buf[offs[:-1] + i] = hdr[:, i]
    keys = rng.integers(1, 256, int(kl.sum()), dtype=np.uint8)  # non-zero key bytes
    kpos = np.repeat(offs[:-1] + 16, kl) + (np.arange(int(kl.sum())) - np.repeat(np.cumsum(kl) - kl, kl))
    buf[kpos] = keys
    eng = Engine(0)
    dev = eng.device
    d = torch.from_numpy(buf).to(dev)
    spans = eng.empty(buf.size // 16 * 16)
    res = eng.empty(64)
    for _ in range(3):
        eng.decode_dev_async(d, buf.size, spans, buf.size // 16, res)
    torch.cuda.synchronize()
    ts = []
    for _ in range(8):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        eng.decode_dev_async(d, buf.size, spans, buf.size // 16, res)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    n = int(res[:8].cpu().numpy().view("<u8")[0])
    want = oracle.decode(buf)[0]
    ok = n == m and np.array_equal(spans[: n * 16].cpu().numpy().view(oracle.SPAN_DTYPE), want)
    print(json.dumps({"workload": ("midlarge" if "--midlarge" in sys.argv else "small") + " records, zero-byte values", "bytes": int(buf.size),
                      "records": m, "ms": round(float(np.median(ts)), 4), "parity": bool(ok)}))


if __name__ == "__main__":
    main()
