#!/usr/bin/env python3
"""CPU model of the lane-walk chunk check (hg_decode.hip lw_chunk_verify and
its gate in lw_chunk) on a decode_variants shape: per 4 KiB chunk entered at
its exact first record start, how many chunks pass, and why the others fail.
Test tooling (not part of the product).  Usage: verify_sim.py SHAPE [CHUNKS]
with SHAPE one of small medium zsmall zmidlarge."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

from oracle import oracle  # noqa: E402

CHUNK, SEG = 4096, 64


def table(shape):
    from decode_variants import zero_valued  # noqa: E402
    from tests.test_decode_gpu import _shape_table  # noqa: E402
    if shape == "small":
        return _shape_table(300_000, (0, 25), (0, 65), 7)
    if shape == "medium":
        return _shape_table(100_000, (8, 65), (64, 513), 7)
    if shape == "zsmall":
        return zero_valued(300_000, (1, 24), (0, 64), 9)
    if shape == "zmidlarge":
        return zero_valued(60_000, (16, 17), (400, 1201), 9)
    raise SystemExit("unknown shape " + shape)


def check(buf, starts, cb, zfilter):
    L = buf.size
    clen = min(CHUNK, L - cb)
    X = starts[np.searchsorted(starts, cb)] if np.searchsorted(starts, cb) < starts.size else L
    if X >= cb + clen:
        return "no start"
    xw = int(X - cb)
    je = xw // SEG
    z = np.zeros(CHUNK + 96, bool)
    seg = buf[cb:cb + CHUNK + 96]
    z[:seg.size] = seg == 0
    z4 = z[:-3] & z[1:-2] & z[2:-1] & z[3:]           # bytes j..j+3 zero
    cand = z4[4:4 + CHUNK + 64] & z4[12:12 + CHUNK + 64]
    lim = L - cb
    cand[max(0, lim - 16 + 1):] = False               # header past the file
    cand[clen:] = cand[clen:]                         # (halo bits stay for run ends)
    heavy = sum(1 for l in range(64) if l * SEG < clen and l >= je and z[l * SEG:l * SEG + 64].sum() >= 40)
    zh = heavy >= 16
    if zh and not zfilter:
        return "zero-heavy: not tried"
    prev_l1 = -1000
    m = 0
    lanes = []
    for l in range(64):
        s0 = l * SEG
        c = cand[s0:s0 + 64].copy()
        if s0 + 64 > clen:
            c[max(0, clen - s0):] = False
        nb = bool(cand[s0 + 64]) if s0 + 64 < clen else bool(cand[s0 + 64])
        re = c & ~np.concatenate([c[1:], [nb]])
        if zh:
            re &= ~z4[s0:s0 + 64]
        if l < je or s0 >= clen:
            re[:] = False
        elif l == je:
            re[:xw - s0] = False
        pos = np.flatnonzero(re)

        def greedy(last):
            kept = []
            for q in pos:
                if q - last >= 16:
                    kept.append(int(q))
                    last = q
            return kept, last
        k1, l1 = greedy(-64)
        kept, _ = greedy(-64 if l == je else prev_l1 - 64)
        prev_l1 = l1
        lanes.append((l, s0, kept))
    m = 0
    for l, s0, kept in lanes:
        if len(kept) > 4:
            return "more than 4 starts in a lane"
        nx = None
        first = None
        for q in kept:
            p = s0 + q
            k = int.from_bytes(buf[cb + p:cb + p + 8].tobytes(), "little")
            v = int.from_bytes(buf[cb + p + 8:cb + p + 16].tobytes(), "little")
            if k + v > lim - 16 - p:
                return "unreadable candidate"
            if first is None:
                first = p
            elif nx != p:
                return "within-lane successor mismatch"
            nx = p + 16 + k + v
        before = m
        if l == je:
            if first is None or first != xw:
                return "entry not a kept run end"
        elif first is not None and before != first:
            return "lane's first start != predecessors' successor"
        if first is not None:
            m = max(m, nx)
    if m < clen:
        return "a record starts after the last run end"
    return "pass"


def main():
    shape = sys.argv[1]
    nchunks = int(sys.argv[2]) if len(sys.argv) > 2 else 400
    buf = table(shape)
    want = oracle.decode(buf)[0]
    starts = want["off"].astype(np.int64)
    for zf in (False, True):
        res = {}
        for i in range(1, nchunks + 1):
            cb = i * CHUNK
            if cb + CHUNK > buf.size:
                break
            r = check(buf, starts, cb, zf)
            res[r] = res.get(r, 0) + 1
        tot = sum(res.values())
        print(shape, "klen-0 filter" if zf else "gate only", {k: round(v / tot, 3) for k, v in sorted(res.items())})


if __name__ == "__main__":
    main()
