#!/usr/bin/env python3
"""Time the decode kernel on three workload shapes in one process.

cfg2 (fixed 16 B / 100 B records, 1 GiB), mixed 16 B / 8..4096 B values,
small mixed records, medium mixed records and large values up to 16 and 64 KiB.  Median launch time over 7 timed launches; every run's
spans are checked bit-exact against the oracle (test infrastructure)."""
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


KEYS = {"cfg2 16B/100B 1GiB": "cfg2", "mixed 16B/8..4096B": "mixed4k",
        "small mixed 0..24B/0..64B": "small", "medium 8..64B/64..512B": "medium",
        "large 16B/0..16KiB": "large", "huge 16B/0..64KiB": "huge",
        "midlarge 16B/400..1200B": "midlarge", "zero small 1..23B/0..63B": "zsmall",
        "zero midlarge 16B/400..1200B": "zmidlarge"}


def selected(label, words):
    """No words: every workload; a word equal to a workload's key (KEYS)
    selects that one; other words match label substrings."""
    if not words:
        return True
    return any(w == KEYS.get(label) or (w not in KEYS.values() and w in label) for w in words)


def workloads(dev):
    n = 8_134_407
    yield "cfg2 16B/100B 1GiB", synth.fixed_sst(n, 16, 100, seed=2, device=dev)
    rng = np.random.default_rng(4)
    for label, m, kr, vr in [("mixed 16B/8..4096B", 400_000, (16, 17), (8, 4097)),
                             ("small mixed 0..24B/0..64B", 4_000_000, (0, 24), (0, 64)),
                             ("medium 8..64B/64..512B", 1_500_000, (8, 65), (64, 513)),
                             ("large 16B/0..16KiB", 60_000, (16, 17), (0, 16385)),
                             ("huge 16B/0..64KiB", 15_000, (16, 17), (0, 65537)),
                             ("midlarge 16B/400..1200B", 1_000_000, (16, 17), (400, 1201))]:
        kl = rng.integers(*kr, m)
        vl = rng.integers(*vr, m)
        vl[rng.random(m) < 0.05] = 0
        offs = np.concatenate([[0], np.cumsum(16 + kl + vl)])
        buf = rng.integers(0, 256, int(offs[-1]), dtype=np.uint8)
        hdr = np.stack([kl, vl], axis=1).astype("<u8").view(np.uint8).reshape(m, 16)
        for i in range(16):
            buf[offs[:-1] + i] = hdr[:, i]
        yield label, torch.from_numpy(buf).to(dev)
    # zero-byte values (keys non-zero): every 16 value bytes read as a header candidate
    for label, m, kr, vr, seed in [("zero small 1..23B/0..63B", 3_000_000, (1, 24), (0, 64), 9),
                                   ("zero midlarge 16B/400..1200B", 1_000_000, (16, 17), (400, 1201), 9)]:
        yield label, torch.from_numpy(zero_valued(m, kr, vr, seed)).to(dev)


def zero_valued(m, kr, vr, seed):
    """Records with random non-zero key bytes and all-zero value bytes
    (tools/zero_values.py's shapes)."""
    rng = np.random.default_rng(seed)
    kl = np.full(m, kr[0]) if kr[1] - kr[0] == 1 else rng.integers(*kr, m)
    vl = rng.integers(*vr, m)
    offs = np.concatenate([[0], np.cumsum(16 + kl + vl)])
    buf = np.zeros(int(offs[-1]), np.uint8)
    hdr = np.stack([kl, vl], axis=1).astype("<u8").view(np.uint8).reshape(m, 16)
    for i in range(16):
        buf[offs[:-1] + i] = hdr[:, i]
    nk = int(kl.sum())
    kpos = np.repeat(offs[:-1] + 16, kl) + (np.arange(nk) - np.repeat(np.cumsum(kl) - kl, kl))
    buf[kpos] = rng.integers(1, 256, nk, dtype=np.uint8)
    return buf


def main():
    only = sys.argv[1:]  # label words (any match); none: every workload
    eng = Engine(0)
    eng.set_stream(torch.cuda.current_stream(eng.device))
    for label, sst in workloads(eng.device):
        if not selected(label, only):
            continue
        L = sst.numel()
        cap = L // 16
        spans = eng.empty(cap * 16)
        res = eng.empty(64)
        eng.reserve(L, 0)
        times = []
        for rnd in range(8):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            eng.decode_dev_async(sst, L, spans, cap, res)
            e1.record()
            torch.cuda.synchronize()
            if rnd > 0:
                times.append(e0.elapsed_time(e1))
        r = res[:24].cpu().numpy()
        n = int(r[:8].view("<u8")[0])
        kind = int(r[8:12].view("<i4")[0])
        host = sst.cpu().numpy()
        want, wn, wkind, _, _ = oracle.decode(host)
        got = spans[: n * 16].cpu().numpy().view(oracle.SPAN_DTYPE)
        ok = kind == wkind and n == wn and np.array_equal(got, want)
        ms = float(np.median(times))
        # back to back (the bench legs' timing): 20 calls in one event pair
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            eng.decode_dev_async(sst, L, spans, cap, res)
        e1.record()
        torch.cuda.synchronize()
        b2b = e0.elapsed_time(e1) / 20
        print(json.dumps({"workload": label, "bytes": L, "records": n, "ms": round(ms, 4),
                          "b2b_ms": round(b2b, 4),
                          "GBps_alg": round((L + 16 * n) / ms / 1e6, 1), "parity": bool(ok)}),
              flush=True)
        del spans, sst


if __name__ == "__main__":
    main()
