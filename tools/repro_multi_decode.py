#!/usr/bin/env python3
"""Diagnostic (GPU box): the mixed 8..16 B key / 0..2048 B value tables of
tests/test_multi_gpu.py's pool test through every decode entry point, each
result printed against the oracle (no asserts, so one run shows them all)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import oracle  # noqa: E402
from tests import corpus  # noqa: E402


def main():
    from horreum_amd import abi
    from horreum_amd.engine import Engine
    from horreum_amd.multi import MultiEngine
    print("knobs", abi.knobs_from_env(), flush=True)  # HG_DEBUG_POISON=1: new buffers hold 0xA5
    tabs = []
    for t in range(9):
        arena, pairs = corpus.mixed(300 + 40 * t, 16, 2048, seed=60 + t, kmin=8, vmin=0)
        tabs.append(oracle.encode(arena, pairs)[0])
    want = [oracle.decode(d) for d in tabs]

    def report(tag, idx, outs):
        bad = []
        for i, o in zip(idx, outs):
            w, wn, wk, wo, _ = want[i]
            ok = (o.n, o.kind, o.offset) == (wn, wk, wo) and np.array_equal(o.spans[:wn], w[:wn])
            if not ok:
                bad.append((i, int(o.n), int(o.kind), int(o.offset), wn))
        print(f"{tag:40s} {'ok' if not bad else 'BAD ' + str(bad)}", flush=True)

    eng = Engine(0)
    for i in range(9):
        report(f"decode_host t{i}", [i], [eng.decode_host(tabs[i])])
    for i in range(9):
        report(f"decode_many_host [t{i}]", [i], eng.decode_many_host([tabs[i]]))
    report("decode_many_host [t1, t6]", [1, 6], eng.decode_many_host([tabs[1], tabs[6]]))
    report("decode_many_host [t1, t6] again", [1, 6], eng.decode_many_host([tabs[1], tabs[6]]))
    report("decode_many_host all 9", list(range(9)), eng.decode_many_host(tabs))
    for n in (2, 3, 5):
        m = MultiEngine([0] * n)
        report(f"MultiEngine x{n} decode_tables", list(range(9)), m.decode_tables(tabs))
        report(f"MultiEngine x{n} decode_tables again", list(range(9)), m.decode_tables(tabs))
        m.close()
    fresh = Engine(0)
    report("fresh decode_many_host [t1, t6]", [1, 6], fresh.decode_many_host([tabs[1], tabs[6]]))
    fresh2 = Engine(0)
    report("fresh decode_many_host [t1]", [1], fresh2.decode_many_host([tabs[1]]))
    # the pool test's order: a compaction on one context, then five contexts
    from tests.test_merge_gpu import encode_tables, sorted_tables
    datas = [d.tobytes() for d in encode_tables(sorted_tables(6, 12000, 0.4, 51))]
    single = eng.compact_host(datas, block_stride=5)
    print("compact_host status", single.status, single.n, flush=True)
    m5 = MultiEngine([0] * 5)
    report("after compact: MultiEngine x5 decode_tables", list(range(9)), m5.decode_tables(tabs))
    got = m5.compact(datas, block_stride=5)
    print("x5 compact", got.status, got.n, bool(np.array_equal(got.data, single.data)), flush=True)
    report("after compact: x5 decode_tables again", list(range(9)), m5.decode_tables(tabs))
    m5.close()


if __name__ == "__main__":
    main()
