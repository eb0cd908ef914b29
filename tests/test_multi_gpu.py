"""GPU parity of the multi-context paths (include/horreum_gpu.h
"several contexts"): range decode with an explicit entry, the speculative
range entry, a single table split over contexts with the host entry handoff,
many tables spread over contexts, and compaction split by key range -- all
against the oracle (src/format.rs:50-77, src/sstable/manager.rs:199-234) and
against the single-context engine, byte for byte.  The contexts are two or
three on device 0, each driven by its own host thread inside the library;
one test also drives two Engine contexts from two Python threads."""
import threading

import numpy as np
import pytest

from oracle import oracle
from tests import corpus
from tests.test_merge_gpu import encode_tables, sorted_tables

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def multi2():
    from horreum_amd.multi import MultiEngine
    m = MultiEngine([0, 0])
    yield m
    m.close()


@pytest.fixture(scope="module")
def multi3():
    from horreum_amd.multi import MultiEngine
    m = MultiEngine([0, 0, 0])
    yield m
    m.close()


# ---- range decode -----------------------------------------------------------------
@pytest.mark.parametrize("name", ["fixed_16_100", "mixed_small", "tiny", "zero_values",
                                  "mixed_4k", "large_values"])
def test_range_decode_chain(engine, name):
    """Cut a table at arbitrary byte offsets; decoding range after range from
    the previous range's exit reproduces the whole-table spans exactly."""
    _, _, data, _ = corpus.make(name)
    want, wn, wk, _, _ = oracle.decode(data)
    assert wk == 0
    d = engine.to_device(data)
    L = data.size
    rng = np.random.default_rng(L)
    cuts = sorted(set([0, L] + rng.integers(1, L, size=5).tolist() + [16384, 16400]))
    cuts = [c for c in cuts if c <= L]
    entry, got = 0, []
    for b, e in zip(cuts[:-1], cuts[1:]):
        out, ex = engine.decode_range_dev(d, L, b, e, entry)
        assert out.kind == 0, (b, e, out.kind, out.offset)
        got.append(engine.spans_to_numpy(out.spans, out.n))
        assert ex >= e or ex == L
        entry = ex
    got = np.concatenate(got) if got else np.zeros(0, oracle.SPAN_DTYPE)
    assert got.size == wn
    assert np.array_equal(got, want)


def test_range_decode_error_inside(engine):
    """A truncated table: the range holding the failing record reports the
    reference's error kind and absolute offset."""
    _, _, data, rec_off = corpus.make("mixed_small")
    bad = data[: int(rec_off[20000]) + 9]  # cut inside a header
    want, wn, wk, wo, _ = oracle.decode(bad)
    d = engine.to_device(bad)
    L = bad.size
    mid = (L // 2) & ~15
    out0, ex = engine.decode_range_dev(d, L, 0, mid, 0)
    assert out0.kind == 0
    out1, _ = engine.decode_range_dev(d, L, mid, L, ex)
    assert (out0.n + out1.n, out1.kind, out1.offset) == (wn, wk, wo)


@pytest.mark.parametrize("name", ["fixed_16_100", "mixed_small", "mixed_4k"])
def test_guess_entry(engine, name):
    """The speculative entry of a cut is (on these corpora) the exact first
    record start at or after it."""
    _, _, data, rec_off = corpus.make(name)
    d = engine.to_device(data)
    starts = np.asarray(rec_off, dtype=np.uint64)
    for cut in (16384, 50000, data.size // 2, data.size - 100):
        g = engine.guess_entry_dev(d, data.size, cut)
        i = np.searchsorted(starts, cut)
        exact = int(starts[i]) if i < starts.size else data.size
        assert g == exact, (cut, g, exact)
    assert engine.guess_entry_dev(d, data.size, data.size) == data.size


# ---- encoded size -----------------------------------------------------------------
def test_encoded_size(engine):
    arena, pairs, data, _ = corpus.make("mixed_4k")
    assert engine.encoded_size(pairs) == data.size
    dp = engine.to_device(pairs.view(np.uint8))
    assert engine.encoded_size(dp, pairs.size) == data.size
    assert engine.encoded_size(pairs[:0]) == 0


# ---- one table over several contexts ---------------------------------------------------
@pytest.mark.parametrize("name", ["fixed_16_100", "mixed_small", "tiny", "empty_keys_tombs",
                                  "zero_values", "mixed_4k", "large_values"])
def test_decode_file_split(multi3, name):
    _, _, data, _ = corpus.make(name)
    want, wn, wk, wo, _ = oracle.decode(data)
    out = multi3.decode_file(data)
    assert (out.n, out.kind, out.offset) == (wn, wk, wo)
    assert np.array_equal(out.spans, want)


def test_decode_file_split_errors(multi2):
    _, _, data, rec_off = corpus.make("mixed_small")
    for cut in (int(rec_off[25000]) + 3, int(rec_off[3000]) + 20, data.size - 1):
        bad = data[:cut]
        want, wn, wk, wo, _ = oracle.decode(bad)
        out = multi2.decode_file(bad)
        assert (out.n, out.kind, out.offset) == (wn, wk, wo), cut
        assert np.array_equal(out.spans[:wn], want[:wn])


def test_decode_file_split_large(multi2):
    """cfg 2 shape, 64 MiB, split over two contexts."""
    arena, pairs = corpus.fixed(500_000, 16, 100, seed=21)
    data = oracle.encode(arena, pairs)[0]
    want, wn, wk, _, _ = oracle.decode(data)
    out = multi2.decode_file(data)
    assert (out.n, out.kind) == (wn, wk) and np.array_equal(out.spans, want)


# ---- many tables over several contexts -------------------------------------------------
def test_decode_tables_round_robin(multi3):
    """cfg 4 shape in miniature: 7 tables of mixed 8 B..4 KiB values with
    tombstones (and one empty, one truncated) over three contexts."""
    tables = []
    for t in range(7):
        arena, pairs = corpus.mixed(400 + 50 * t, 16, 4096, seed=40 + t, kmin=16, vmin=8)
        tables.append(oracle.encode(arena, pairs)[0])
    tables[3] = np.zeros(0, np.uint8)
    tables[5] = tables[5][:-7]
    outs = multi3.decode_tables(tables)
    for d, o in zip(tables, outs):
        want, wn, wk, wo, _ = oracle.decode(d)
        assert (o.n, o.kind, o.offset) == (wn, wk, wo)
        assert np.array_equal(o.spans[:wn], want[:wn])


# ---- compaction split by key range ------------------------------------------------------
@pytest.mark.parametrize("k,n_universe,frac,seed,stride", [
    (8, 20000, 0.3, 31, 0),
    (8, 8000, 0.8, 32, 10),   # heavy overlap
    (3, 6000, 0.5, 33, 7),
    (5, 9000, 0.4, 34, 1),
])
def test_compact_split_by_key_range(engine, multi3, k, n_universe, frac, seed, stride):
    tables = sorted_tables(k, n_universe, frac, seed, long_prefix=seed % 2 == 0)
    datas = [d.tobytes() for d in encode_tables(tables)]
    single = engine.compact_host(datas, block_stride=stride)
    split = multi3.compact(datas, block_stride=stride)
    assert split.status == 0 and single.status == 0
    assert split.n == single.n
    assert np.array_equal(split.data, single.data)
    if stride:
        assert np.array_equal(split.blocks, single.blocks)
    # and the oracle: serialize_flatten(compact_inner(tables newest first))
    tabs = [(np.frombuffer(d, np.uint8), oracle.decode(np.frombuffer(d, np.uint8))[0])
            for d in datas]
    refs, _ = oracle.compact(tabs)
    merged = [oracle.pairs_from_spans(tabs[t][0], tabs[t][1][r:r + 1])[0] for t, r in refs]
    arena, rec = oracle.pack_pairs(merged)
    want, _, wblocks, _ = oracle.encode(arena, rec, block_stride=stride)
    assert np.array_equal(split.data, want)
    if stride:
        assert np.array_equal(split.blocks, wblocks)


def test_compact_split_unsorted_falls_back(engine, multi2):
    """Tables with duplicate / unordered keys are not range-separable: the
    split compaction hands them to one context's exact reference loop."""
    tables = sorted_tables(4, 3000, 0.5, 35)
    tables[1] = tables[1][::-1]
    tables[2] = tables[2] + tables[2][:30]
    datas = [d.tobytes() for d in encode_tables(tables)]
    single = engine.compact_host(datas, block_stride=3)
    split = multi2.compact(datas, block_stride=3)
    assert split.status == single.status == 0
    assert np.array_equal(split.data, single.data)
    assert np.array_equal(split.blocks, single.blocks)


def _compact_dev_case(engine, multi, tables, owner):
    import torch
    datas = [d for d in encode_tables(tables)]
    dev = [torch.from_numpy(d.copy()).to("cuda:0") if d.size else
           torch.zeros(0, dtype=torch.uint8, device="cuda:0") for d in datas]
    total = max(sum(d.size for d in datas), 1)
    outs = [torch.zeros(total, dtype=torch.uint8, device="cuda:0") for _ in range(multi.n)]
    torch.cuda.synchronize()
    rc, ol, orc, res = multi.compact_dev(dev, owner, outs)
    torch.cuda.synchronize()
    single = engine.compact_host([d.tobytes() for d in datas])
    got = np.concatenate([outs[g][:ol[g]].cpu().numpy() for g in range(multi.n)])
    return rc, got, sum(orc), res, single, ol


@pytest.mark.parametrize("k,n_universe,frac,seed", [(8, 20000, 0.3, 41), (5, 9000, 0.6, 42)])
def test_compact_dev_split_by_key_range(engine, multi3, k, n_universe, frac, seed):
    """hg_multi_compact_dev: tables resident on their owner contexts, key
    ranges gathered by device copies (no upload, no second decode), merged
    and encoded per context: the slices' concatenation is byte-identical to
    the single-context compaction and to the oracle."""
    tables = sorted_tables(k, n_universe, frac, seed, long_prefix=seed % 2 == 0)
    rc, got, nrec, res, single, ol = _compact_dev_case(engine, multi3, tables,
                                                       [t % 3 for t in range(k)])
    assert rc == 0 and single.status == 0
    assert nrec == single.n == res.n_out
    assert np.array_equal(got, single.data)
    assert sum(1 for x in ol if x) >= 2  # really split


def test_compact_dev_empty_slices(engine, multi3):
    """A table whose keys all fall in the lowest key range (its other slices
    are empty), an empty table, and owners that hold several tables."""
    tables = sorted_tables(4, 6000, 0.5, 43)
    tables.append([(b"\x00" + bytes([i]), b"low%d" % i) for i in range(40)])  # all in range 0
    tables.append([])
    rc, got, nrec, res, single, _ = _compact_dev_case(engine, multi3, tables, [0, 0, 1, 2, 1, 2])
    assert rc == 0 and single.status == 0
    assert np.array_equal(got, single.data) and nrec == single.n


def test_compact_dev_unsorted_falls_back(engine, multi2):
    """Not range-separable input: gathered on context 0, the reference loop
    there; the whole output in slice 0."""
    tables = sorted_tables(4, 3000, 0.5, 44)
    tables[1] = tables[1][::-1]
    tables[2] = tables[2] + tables[2][:30]
    rc, got, nrec, res, single, ol = _compact_dev_case(engine, multi2, tables, [1, 0, 1, 0])
    assert rc == single.status == 0
    assert ol[1] == 0
    assert np.array_equal(got, single.data) and nrec == single.n


# ---- contexts driven from separate Python threads ---------------------------------------
def test_two_contexts_two_threads():
    """include/horreum_gpu.h: distinct contexts may be used from distinct
    threads.  Two Engines on device 0, each decoding and encoding its own
    corpus repeatedly in its own thread, both bit-exact."""
    from horreum_amd.engine import Engine
    jobs = [corpus.make("mixed_small"), corpus.make("mixed_4k")]
    errors = []

    def work(i):
        try:
            eng = Engine(0, use_torch_stream=False)
            arena, pairs, data, _ = jobs[i]
            want = oracle.decode(data)[0]
            for _ in range(5):
                out = eng.decode_host(data)
                assert out.kind == 0 and np.array_equal(out.spans, want)
                enc = eng.encode_host(arena, pairs)
                assert np.array_equal(enc.data, data)
            eng.close()
        except Exception as e:  # noqa: BLE001 -- reported below
            errors.append((i, repr(e)))

    th = [threading.Thread(target=work, args=(i,)) for i in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors


def test_compact_dev_capacity_reports_slice_sizes(engine, multi2):
    """A slice that does not fit its caller buffer: HG_ERR_CAPACITY with every
    slice's size in out_lens (the overflowing one included), so the caller can
    resize and call again; the retry is byte-identical to one context's
    compaction."""
    import torch
    from horreum_amd.abi import Status
    tables = sorted_tables(4, 8000, 0.4, 47)
    datas = [d for d in encode_tables(tables)]
    dev = [torch.from_numpy(d.copy()).to("cuda:0") for d in datas]
    small = [torch.zeros(64, dtype=torch.uint8, device="cuda:0") for _ in range(2)]
    torch.cuda.synchronize()
    rc, ol, _, _ = multi2.compact_dev(dev, [0, 1, 0, 1], small)
    assert rc == Status.CAPACITY
    assert all(x > 64 for x in ol), ol  # both slices report what they need
    outs = [torch.zeros(int(x), dtype=torch.uint8, device="cuda:0") for x in ol]
    rc, ol2, orc, _ = multi2.compact_dev(dev, [0, 1, 0, 1], outs)
    torch.cuda.synchronize()
    assert rc == 0 and list(ol2) == list(ol)
    single = engine.compact_host([d.tobytes() for d in datas])
    got = np.concatenate([outs[g][:ol2[g]].cpu().numpy() for g in range(2)])
    assert np.array_equal(got, single.data) and sum(orc) == single.n


@pytest.mark.parametrize("k,n_universe,frac,seed", [(6, 20000, 0.3, 51), (8, 12000, 0.5, 52)])
def test_compact_dev_peer_copy_call_on_one_device(engine, multi3, knobs, k, n_universe, frac, seed):
    """The cross-GPU split's copy branch (hipMemcpyPeerAsync, hg_multi.hip
    copy_dev) run on one device (HG_MULTI_TEST_PEER_COPY=1: same-device
    contexts take the peer-copy call too): slices byte-identical to the
    single-context compaction, as with device-to-device copies."""
    knobs("HG_MULTI_TEST_PEER_COPY", 1)
    tables = sorted_tables(k, n_universe, frac, seed)
    rc, got, nrec, res, single, ol = _compact_dev_case(engine, multi3, tables,
                                                       [t % 3 for t in range(k)])
    assert rc == 0 and single.status == 0
    assert nrec == single.n == res.n_out
    assert np.array_equal(got, single.data)
    assert sum(1 for x in ol if x) >= 2


# ---- contexts on distinct devices (skipped on a one-GPU box) -----------------------------
@pytest.mark.skipif("not __import__('torch').cuda.device_count() >= 2",
                    reason="needs two GPUs: the peer-copy branch of the split")
@pytest.mark.parametrize("seed", [51, 52])
def test_compact_dev_across_devices(engine, seed):
    """hg_multi_compact_dev with contexts on devices 0 and 1: each table
    resident on its owner's GPU, key-range slices gathered by peer copies
    (hipMemcpyPeerAsync over xGMI), slice g written on device g; byte-identical
    to one context's compaction.  The caller's current device is unchanged."""
    import torch
    from horreum_amd.multi import MultiEngine
    m = MultiEngine([0, 1])
    try:
        tables = sorted_tables(6, 20000, 0.3, seed)
        datas = [d for d in encode_tables(tables)]
        owner = [t % 2 for t in range(len(datas))]
        dev = [torch.from_numpy(d.copy()).to("cuda:%d" % o) for d, o in zip(datas, owner)]
        total = sum(d.size for d in datas)
        outs = [torch.zeros(total, dtype=torch.uint8, device="cuda:%d" % g) for g in range(2)]
        torch.cuda.set_device(0)
        for g in range(2):
            torch.cuda.synchronize(g)
        rc, ol, orc, res = m.compact_dev(dev, owner, outs)
        assert torch.cuda.current_device() == 0
        for g in range(2):
            torch.cuda.synchronize(g)
        single = engine.compact_host([d.tobytes() for d in datas])
        got = np.concatenate([outs[g][:ol[g]].cpu().numpy() for g in range(2)])
        assert rc == 0 and np.array_equal(got, single.data) and sum(orc) == single.n
        assert all(ol)  # really split across the two GPUs
        split = m.compact([d.tobytes() for d in datas], block_stride=7)
        ref = engine.compact_host([d.tobytes() for d in datas], block_stride=7)
        assert split.status == 0 and np.array_equal(split.data, ref.data)
        assert np.array_equal(split.blocks, ref.blocks)
    finally:
        m.close()


@pytest.mark.skipif("not __import__('torch').cuda.device_count() >= 2",
                    reason="needs two GPUs")
def test_decode_tables_across_devices_keeps_caller_device():
    """Tables round-robin over contexts on devices 0 and 1 (cfg 4's split):
    every table's spans equal the oracle's, and the calling thread is left on
    the device it was on (the driver switches devices on the caller's thread)."""
    import torch
    from horreum_amd.multi import MultiEngine
    m = MultiEngine([1, 0])
    try:
        names = ["fixed_16_100", "mixed_small", "mixed_4k", "tiny"]
        datas = [corpus.make(nm)[2] for nm in names]
        torch.cuda.set_device(1)
        outs = m.decode_tables(datas)
        assert torch.cuda.current_device() == 1
        for d, o in zip(datas, outs):
            want, wn, wk, _, _ = oracle.decode(d)
            assert (o.n, o.kind) == (wn, wk) and np.array_equal(o.spans, want)
    finally:
        torch.cuda.set_device(0)
        m.close()


# ---- the library's host worker pool (hg_multi.hip FanPool) ---------------------------------
def _pool_case(engine):
    tables = sorted_tables(6, 12000, 0.4, 51)
    datas = [d.tobytes() for d in encode_tables(tables)]
    single = engine.compact_host(datas, block_stride=5)
    assert single.status == 0
    dec_tables = []
    for t in range(9):
        arena, pairs = corpus.mixed(300 + 40 * t, 16, 2048, seed=60 + t, kmin=8, vmin=0)
        dec_tables.append(oracle.encode(arena, pairs)[0])
    want = [oracle.decode(d) for d in dec_tables]

    def one_pass(m):
        outs = m.decode_tables(dec_tables)
        for (w, wn, wk, wo, _), o in zip(want, outs):
            assert (o.n, o.kind, o.offset) == (wn, wk, wo)
            assert np.array_equal(o.spans[:wn], w[:wn])
        got = m.compact(datas, block_stride=5)
        assert got.status == 0 and np.array_equal(got.data, single.data)
        assert np.array_equal(got.blocks, single.blocks)
    return one_pass


def test_worker_pool_growth_sequential(engine, multi2):
    """The multi-context driver runs its per-context steps on persistent host
    workers: a five-context driver grows the pool past the two- and
    three-context drivers' workers, then the two-context driver runs on the
    same pool again; decodes and compactions alternate on both, every result
    byte-identical to the oracle / the single-context engine."""
    from horreum_amd.multi import MultiEngine
    one_pass = _pool_case(engine)
    m5 = MultiEngine([0] * 5)
    try:
        for _ in range(2):
            one_pass(m5)
            one_pass(multi2)
    finally:
        m5.close()


def test_worker_pool_concurrent_drivers(engine, multi2):
    """Two multi-context drivers used at once from two Python threads: one
    holds the library's worker pool, the other runs its steps on threads of
    its own (include/horreum_gpu.h: distinct contexts may be used from
    distinct threads); both stay byte-identical throughout."""
    from horreum_amd.multi import MultiEngine
    one_pass = _pool_case(engine)
    m5 = MultiEngine([0] * 5)
    errors = []

    def run(m, reps):
        try:
            for _ in range(reps):
                one_pass(m)
        except Exception as e:  # noqa: BLE001 -- reported by the main thread
            errors.append(e)

    try:
        th = [threading.Thread(target=run, args=(m, 3)) for m in (m5, multi2)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert not errors, errors
    finally:
        m5.close()
