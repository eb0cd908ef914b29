#!/usr/bin/env python3
"""Wall time per cfg 2 decode step with and without per-step HIP events in
the timed loop (does the instrumentation cost the headline anything?)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from horreum_amd import synth  # noqa: E402
from horreum_amd.engine import Engine  # noqa: E402
from horreum_amd import abi as _abi  # noqa: E402
_abi.knobs_from_env()  # the A/B scripts' HG_* knobs (the library reads no environment)


def main():
    eng = Engine(0)
    dev = eng.device
    p = bench.shard_plan(0, 1)
    sst = synth.fixed_sst(p["n"], p["k"], p["v"], seed=p["seed"], device=dev)
    L = sst.numel()
    eng.reserve(L, 0)
    spans = eng.empty(p["n"] * 16)
    res = eng.empty(64)

    def step():
        eng.decode_dev_async(sst, L, spans, p["n"], res)

    out = {}
    for rep in range(3):
        wall, ms = bench.time_async(torch, step, 100, 20, 1, dev)
        out.setdefault("events_per_step_ms", []).append(round(wall / 100 * 1e3, 5))
        for _ in range(20):
            step()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        s.record()
        for _ in range(100):
            step()
        e.record()
        torch.cuda.synchronize()
        out.setdefault("bracket_only_ms", []).append(round((time.perf_counter() - t0) / 100 * 1e3, 5))
        out.setdefault("bracket_event_ms", []).append(round(s.elapsed_time(e) / 100, 5))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
