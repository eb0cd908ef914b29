"""GPU parity: batched point lookups (hg_keyindex_build / hg_lookup_*) vs the
oracle's restatement of SSTable::get (src/sstable/table.rs:54-70 with
Index::get, src/sstable/index.rs:72-78): same record for every key, absent
keys absent, tombstones found as tombstones."""
import numpy as np
import pytest

from horreum_amd.format import InternalPair
from horreum_amd.manager import SSTableManager
from horreum_amd.table import PersistedFile, SSTable
from oracle import oracle
from tests.test_merge_gpu import encode_tables, sorted_tables

pytestmark = pytest.mark.gpu


def _queries(table_pairs, rng, n_extra=400):
    keys = [k for k, _ in table_pairs]
    q = list(keys[::3])
    for k in keys[::7]:
        q.append(k + b"\x00")          # extension of a present key
        if k:
            q.append(k[:-1])           # prefix of a present key
    q += [rng.integers(0, 256, size=int(rng.integers(0, 30)), dtype=np.uint8).tobytes()
          for _ in range(n_extra)]
    q += [b"", b"\xff" * 40]
    return q


@pytest.mark.parametrize("seed,long_prefix", [(21, False), (22, True)])
def test_lookup_host_parity(engine, seed, long_prefix):
    rng = np.random.default_rng(seed)
    pairs = sorted_tables(1, 8000, 0.6, seed, long_prefix)[0]
    data = encode_tables([pairs])[0]
    spans = oracle.decode(data)[0]
    queries = _queries(pairs, rng)
    res = engine.lookup_host(data.tobytes(), queries)
    for q, r in zip(queries, res):
        want = oracle.table_get(data, spans, 10, q)
        if want is None:
            assert r["found"] == 0, q
        else:
            s = spans[want]
            assert r["found"] == 1 and r["rec"] == want, q
            assert r["val_off"] == s["off"] + 16 + s["klen"] and r["vlen"] == s["vlen"]


def test_lookup_device_batches(engine):
    """Key index built once, several query batches against it."""
    import torch
    rng = np.random.default_rng(23)
    pairs = sorted_tables(1, 20000, 0.5, 23, True)[0]
    data = encode_tables([pairs])[0]
    spans_h = oracle.decode(data)[0]
    dt = engine.to_device(data)
    dec = engine.decode_dev(dt, data.size)
    idx = engine.keyindex_build(dt, dec.spans, dec.n)
    for b in range(3):
        queries = _queries(pairs[b::3], rng, 200)
        karena, kdesc = engine.pack_keys(queries)
        dk = engine.to_device(karena)
        dq = engine.to_device(kdesc.view(np.uint8))
        out = engine.empty(24 * len(queries))
        engine.lookup_dev_async(dt, dec.spans, idx, dec.n, dk, dq, len(queries), out)
        torch.cuda.synchronize()
        res = out[: 24 * len(queries)].cpu().numpy().view(np.dtype(
            [("rec", "<u8"), ("val_off", "<u8"), ("vlen", "<u4"), ("found", "<i4")]))
        for q, r in zip(queries, res):
            want = oracle.table_get(data, spans_h, 10, q)
            assert (r["found"] == 1) == (want is not None), q
            if want is not None:
                assert r["rec"] == want


def test_sstable_get_many(engine, golden, tmp_path):
    """src/sstable/table.rs:110-144 through the batched path."""
    c = golden["table_search"]
    pairs = [InternalPair(bytes.fromhex(k), None if v is None else bytes.fromhex(v))
             for k, v in c["pairs"]]
    table = SSTable.new(PersistedFile.new(tmp_path / "t", pairs, engine), pairs, 113, c["stride"],
                        engine)
    keys = [bytes.fromhex(k) for k, _ in c["gets"]]
    got = table.get_many(keys, engine)
    for (key, want), g in zip(c["gets"], got):
        assert g == (None if want is None else
                     InternalPair(bytes.fromhex(want[0]),
                                  None if want[1] is None else bytes.fromhex(want[1])))
        assert g == table.get(bytes.fromhex(key), engine)


def test_manager_get_many(engine, golden, tmp_path):
    """Newest-first across tables (manager.rs:126-134), batched."""
    m = SSTableManager(tmp_path, 2, 100000, engine)
    for kvs, size in golden["payload_size"]["tables"]:
        m.create([InternalPair(bytes.fromhex(k), None if v is None else bytes.fromhex(v))
                  for k, v in kvs], size)
    keys = [b"abc00", b"abc01", b"abc02", b"xxx", b"zzz", b""]
    assert m.get_many(keys) == [m.get(k) for k in keys]


# ---- tables that are not strictly increasing (legal: src/sstable/table.rs:93-108) ------
def _unordered_pairs(seed, n):
    """Keys from a small alphabet: runs of duplicates, disorder, tombstones."""
    rng = np.random.default_rng(seed)
    pairs = []
    for _ in range(n):
        k = bytes(rng.choice(list(b"abc"), size=int(rng.integers(0, 4))).tolist())
        if rng.random() < 0.5 and pairs:
            k = pairs[-1][0]  # a duplicate of the previous key
        v = None if rng.random() < 0.3 else rng.integers(0, 256, int(rng.integers(1, 6)),
                                                          dtype=np.uint8).tobytes()
        pairs.append((k, v))
    return pairs


def _all_keys(depth=3):
    out = [b""]
    for d in range(1, depth + 2):
        out += [bytes(t) for t in np.array(np.meshgrid(*[list(b"abcd")] * d)).T.reshape(-1, d).tolist()]
    return out


@pytest.mark.parametrize("stride", [0, 1, 2, 3, 10])
def test_lookup_duplicate_and_unordered_keys(engine, golden, stride):
    """The record found is the reference's (Rust binary searches over the
    block first keys and in the block), on the table.rs:93-108 pairs and on
    random tables with duplicate runs and disorder."""
    tables = [[(b"abc", b"defg"), (b"abc", None), ("日本語💖".encode(), "ржавчина".encode())]]
    tables += [_unordered_pairs(seed, n) for seed, n in [(31, 50), (32, 300), (33, 2000)]]
    for pairs in tables:
        arena, recs = oracle.pack_pairs(pairs)
        data = oracle.encode(arena, recs)[0]
        spans = oracle.decode(data)[0]
        queries = sorted({k for k, _ in pairs}) + _all_keys() + ["日本語💖".encode()]
        res = engine.lookup_host(data.tobytes(), queries, stride)
        for q, r in zip(queries, res):
            want = oracle.table_get(data, spans, stride or max(len(pairs), 1), q)
            assert (r["found"] == 1) == (want is not None), (stride, q)
            if want is not None:
                assert r["rec"] == want, (stride, q)


@pytest.mark.parametrize("stride", [1, 3])
def test_get_many_equals_get_on_duplicates(engine, tmp_path, stride):
    """SSTable.get_many == SSTable.get key by key on the table.rs:93-108
    pairs (a live value and a tombstone under the same key), both equal to
    the oracle's record."""
    pairs = [InternalPair(b"abc", b"defg"), InternalPair(b"abc", None),
             InternalPair("日本語💖".encode(), "ржавчина".encode())]
    path = tmp_path / f"dup{stride}"
    table = SSTable.new(PersistedFile.new(path, pairs, engine), pairs, 39, stride, engine)
    keys = [b"abc", "日本語💖".encode(), b"ab", b"abd", b""]
    got = table.get_many(keys, engine)
    data = np.fromfile(path, dtype=np.uint8)
    spans = oracle.decode(data)[0]
    for k, g in zip(keys, got):
        assert g == table.get(k, engine), k
        want = oracle.table_get(data, spans, stride, k)
        assert (g is None) == (want is None), k
        if want is not None:
            assert g == pairs[want], k


def test_resident_tables_lru_budget(engine, tmp_path):
    """Resident lookup state is bounded per engine: past the byte budget the
    least recently used table is released (and rebuilt on its next batch);
    results never change."""
    from horreum_amd import table as tmod
    lru = tmod._lru(engine)
    old_budget = lru.budget
    tabs = []
    try:
        for i in range(3):
            pairs = [InternalPair(b"k%05d" % j + bytes([i]), b"v" * (j % 50 + 1)) for j in range(3000)]
            tabs.append((SSTable.new(PersistedFile.new(tmp_path / f"t{i}", pairs, engine), pairs,
                                     0, 10, engine), pairs))
        one = tabs[0][0].file.read_bytes(engine).size + 48 * 3000
        lru.budget = int(one * 1.5)  # room for one table
        for t, pairs in tabs + tabs[:1]:
            keys = [p.key for p in pairs[::97]] + [b"absent"]
            assert t.get_many(keys, engine) == [t.get(k, engine) for k in keys]
        assert tabs[0][0]._resident is not None       # the last one used
        assert tabs[1][0]._resident is None and tabs[2][0]._resident is None
        assert lru.total <= lru.budget
    finally:
        lru.budget = old_budget
        for t, _ in tabs:
            t.release()
