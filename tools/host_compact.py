#!/usr/bin/env python3
"""Time hg_compact_host on the bench's cfg5-scaled tables (8 x 1 M records,
16 B / 100 B, 25 % shared keys) from pageable host memory; median of 5."""
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


def main():
    eng = Engine(0)
    rng = np.random.default_rng(5)
    shared = np.unique(rng.integers(0, 1 << 40, size=250_000, dtype=np.uint64))
    hosts = []
    for t in range(8):
        own = rng.integers(0, 1 << 40, size=1_000_000 - shared.size, dtype=np.uint64)
        keys = np.unique(np.concatenate([shared, own]))
        buf, _ = synth.keyed_table(keys, np.full(keys.size, 100), seed=50 + t, device=eng.device)
        hosts.append(buf.cpu().numpy())
    tot = sum(h.size for h in hosts)
    out = np.empty(tot, dtype=np.uint8)
    eng.compact_host(hosts, out=out)
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        c = eng.compact_host(hosts, out=out)
        ts.append(time.perf_counter() - t0)
    t = sorted(ts)[2]
    print(json.dumps({"ms": round(t * 1e3, 2), "all_ms": [round(x * 1e3, 1) for x in ts],
                      "GiB_s": round(tot / t / (1 << 30), 2), "n": int(c.n),
                      "status": int(c.status)}), flush=True)


if __name__ == "__main__":
    main()
