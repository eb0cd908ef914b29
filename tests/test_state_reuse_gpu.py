"""One context, a seeded random sequence of every call kind on tables of
varying count and size -- single-table decode, batched decode, the host
batched decode, encode, compaction -- each result against the oracle
(src/format.rs:23-77, src/sstable/manager.rs:199-234).  A context carries
state from call to call (control regions cleared by the previous call,
argument staging halves whose copy is skipped when unchanged, encode group
sums cleared ahead, grown workspaces); round 5 found a staging bug that only
a larger call after a smaller one exposed, so this test mixes the call kinds
and sizes on purpose."""
import numpy as np
import pytest

from oracle import oracle
from tests import corpus
from tests.test_merge_gpu import encode_tables, sorted_tables

pytestmark = pytest.mark.gpu


def _pool():
    tabs = []
    for i, (n, kmax, vmax, kmin, vmin, zero) in enumerate([
            (400, 16, 2048, 8, 0, False), (3000, 24, 64, 0, 0, False), (1500, 64, 512, 8, 64, False),
            (900, 16, 1200, 16, 400, False), (2500, 23, 63, 1, 0, True), (120, 16, 4096, 16, 8, False)]):
        arena, pairs = corpus.mixed(n, kmax, vmax, seed=700 + i, kmin=kmin, vmin=vmin, zero_values=zero)
        tabs.append(oracle.encode(arena, pairs)[0])
    stride = oracle.encode(*corpus.fixed(20000, 16, 100, seed=710))[0] if hasattr(corpus, "fixed") else None
    if stride is not None:
        tabs.append(stride)
    tabs.append(tabs[0][:-9])            # truncated
    tabs.append(np.zeros(0, np.uint8))   # empty
    return tabs


def _compact_want(datas, stride):
    tabs = [(np.frombuffer(d, np.uint8), oracle.decode(np.frombuffer(d, np.uint8))[0]) for d in datas]
    refs, _ = oracle.compact(tabs)
    merged = [oracle.pairs_from_spans(tabs[t][0], tabs[t][1][r:r + 1])[0] for t, r in refs]
    arena, rec = oracle.pack_pairs(merged)
    want, _, wblocks, _ = oracle.encode(arena, rec, block_stride=stride)
    return want, wblocks


def test_mixed_call_sequence_on_one_context(engine):  # (engine: HG_TEST_POISON applies)
    import torch
    from horreum_amd.engine import Engine
    eng = Engine(0)
    try:
        tabs = _pool()
        want = [oracle.decode(t) for t in tabs]
        devs = [eng.to_device(t) if t.size else torch.zeros(0, dtype=torch.uint8, device="cuda:0")
                for t in tabs]
        comp_sets = [[d.tobytes() for d in encode_tables(sorted_tables(k, u, f, s))]
                     for k, u, f, s in ((2, 3000, 0.5, 720), (4, 6000, 0.4, 721), (3, 1500, 0.7, 722))]
        comp_want = {}
        rng = np.random.default_rng(7)

        def check_decode(i, n, kind, off, spans_np):
            w, wn, wk, wo, _ = want[i]
            assert (n, kind, off if kind else 0) == (wn, wk, wo if wk else 0), i
            assert np.array_equal(spans_np[:wn], w[:wn]), i

        for step in range(120):
            op = int(rng.integers(0, 5))
            if op == 0:  # single-table decode on the device
                i = int(rng.integers(0, len(tabs)))
                if not tabs[i].size:
                    continue
                o = eng.decode_dev(devs[i])
                torch.cuda.synchronize()
                check_decode(i, o.n, o.kind, o.offset, eng.spans_to_numpy(o.spans, min(o.n, tabs[i].size // 16)))
            elif op == 1:  # batched decode of 1..5 device tables
                idx = list(rng.choice(len(tabs), size=int(rng.integers(1, 6)), replace=False))
                caps = [max(tabs[i].size // 16, 1) for i in idx]
                spans = [eng.empty(c * 16) for c in caps]
                res = eng.empty(24 * len(idx))
                res.fill_(0xEE)
                eng.decode_batch_dev_async([devs[i] for i in idx], [tabs[i].size for i in idx], spans,
                                           caps, res)
                torch.cuda.synchronize()
                r = res.cpu().numpy()
                for j, i in enumerate(idx):
                    n = int(r[24 * j:24 * j + 8].view("<u8")[0])
                    kind = int(r[24 * j + 8:24 * j + 12].view("<i4")[0])
                    off = int(r[24 * j + 16:24 * j + 24].view("<u8")[0])
                    check_decode(i, n, kind, off, eng.spans_to_numpy(spans[j], min(n, caps[j])))
            elif op == 2:  # host tables, one batched launch chain
                idx = list(rng.choice(len(tabs), size=int(rng.integers(1, 6)), replace=False))
                for i, o in zip(idx, eng.decode_many_host([tabs[i] for i in idx])):
                    check_decode(i, o.n, o.kind, o.offset, o.spans)
            elif op == 3:  # encode
                n = int(rng.integers(1, 3000))
                arena, pairs = corpus.mixed(n, 24, int(rng.choice([64, 512, 2048])), seed=800 + step)
                stride = int(rng.choice([0, 1, 10]))
                got = eng.encode_host(arena, pairs, block_stride=stride)
                w, _, wblocks, _ = oracle.encode(arena, pairs, block_stride=stride)
                assert np.array_equal(got.data, w), step
                if stride:
                    assert np.array_equal(got.blocks, wblocks), step
            else:  # compaction
                c = int(rng.integers(0, len(comp_sets)))
                stride = int(rng.choice([0, 5]))
                got = eng.compact_host(comp_sets[c], block_stride=stride)
                if (c, stride) not in comp_want:
                    comp_want[(c, stride)] = _compact_want(comp_sets[c], stride)
                w, wblocks = comp_want[(c, stride)]
                assert got.status == 0 and np.array_equal(got.data, w), step
                if stride:
                    assert np.array_equal(got.blocks, wblocks), step
    finally:
        eng.close()
