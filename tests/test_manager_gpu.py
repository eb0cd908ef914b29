"""SSTableManager byte paths on the engine (reference src/sstable/manager.rs):
directory open order, newest-first get, create, compaction through the device
merge, and the size accounting that drives the trigger."""
import os

import pytest

from horreum_amd.format import InternalPair
from horreum_amd.manager import SSTableManager
from oracle import oracle

pytestmark = pytest.mark.gpu


def _p(kv):
    k, v = kv
    return InternalPair(bytes.fromhex(k), None if v is None else bytes.fromhex(v))


def _oracle_bytes(pairs):
    arena, rec = oracle.pack_pairs([(p.key, p.value) for p in pairs])
    return oracle.encode(arena, rec)[0].tobytes()


def test_open_existing_files(engine, golden, tmp_path):
    """manager.rs:242-275: files table_0..2 written by the CPU oracle."""
    c = golden["manager_get_newest_first"]
    for i, t in enumerate(c["tables_oldest_first"]):
        (tmp_path / f"table_{i}").write_bytes(_oracle_bytes([_p(kv) for kv in t]))
    m = SSTableManager(tmp_path, c["stride"], 1000, engine)
    for key, want in c["gets"]:
        assert m.get(bytes.fromhex(key)) == _p(want)
    assert m.get(b"nope") is None


def test_get_pairs(engine, golden, tmp_path):
    """manager.rs:277-325: create four tables with their sizes, then get."""
    m = SSTableManager(tmp_path, 2, 1000, engine)
    for kvs, size in golden["payload_size"]["tables"]:
        m.create([_p(kv) for kv in kvs], size)
    assert sorted(os.listdir(tmp_path)) == [f"table_{i}" for i in range(4)]
    assert m.get(b"abc00") == InternalPair(b"abc00", b"xyz")
    assert m.get(b"abc01") == InternalPair(b"abc01", None)
    assert m.get(b"abc02") == InternalPair(b"abc02", b"def")
    assert m.get(b"xxx") == InternalPair(b"xxx", b"42")
    # reopening the directory: sizes recomputed from the files (table.rs:36-45)
    m2 = SSTableManager(tmp_path, 2, 1000, engine)
    assert [t.get_size() for t in m2.tables] == [s for _, s in golden["payload_size"]["tables"]]


def test_compaction_roundtrip(engine, tmp_path):
    """Flush three overlapping tables with a 50 % trigger: every flush after
    the first compacts; the result equals the oracle's compact_inner of the
    tables (newest first) and keeps tombstones."""
    m = SSTableManager(tmp_path, 3, 50, engine)
    batches = [
        [InternalPair(b"a%03d" % i, b"v0-%d" % i) for i in range(0, 300, 1)],
        [InternalPair(b"a%03d" % i, None if i % 7 == 0 else b"v1-%d" % i) for i in range(100, 400, 2)],
        [InternalPair(b"a%03d" % i, b"v2-%d" % i) for i in range(250, 500, 3)],
    ]
    history = []
    for b in batches:
        size = sum(len(p.key) + len(p.value or b"") for p in b)
        history.append(b)
        m.flush(b, size)
    assert len(m.tables) == 1 and os.listdir(tmp_path) == ["table_0"]
    # expected: fold the compactions the way the manager did (newest first each time)
    merged = None
    for b in history:
        tabs = [b] + ([merged] if merged is not None else [])
        datas = [_oracle_bytes(t) for t in tabs]
        dec = [(d, oracle.decode(d)[0]) for d in datas]
        refs, _ = oracle.compact(dec)
        merged = [InternalPair(*oracle.pairs_from_spans(dec[t][0], dec[t][1][r:r + 1])[0])
                  for t, r in refs]
    assert m.tables[0].get_all(engine) == merged
    assert open(tmp_path / "table_0", "rb").read() == _oracle_bytes(merged)
    # compacted size = sum of the inputs' sizes (manager.rs:138-158), not the payload
    assert m.tables[0].get_size() == sum(sum(len(p.key) + len(p.value or b"") for p in b)
                                         for b in batches)
    for p in merged[::17]:
        assert m.get(p.key) == p
    assert m.get(b"a007") == InternalPair(b"a007", b"v0-7")
    assert m.get(b"a112") == InternalPair(b"a112", None)  # tombstone kept


def test_no_compaction_below_trigger(engine, tmp_path):
    m = SSTableManager(tmp_path, 2, 1000, engine)
    m.flush([InternalPair(b"k1", b"aaaa")], 6)
    m.flush([InternalPair(b"k2", b"bb")], 4)
    assert len(m.tables) == 2 and m.should_compact() is None


def test_lexicographic_open_order(engine, tmp_path):
    """manager.rs:47-55 sorts paths as strings: after 12 tables, reopening
    ranks table_2 newer than table_11 (the reference's behaviour)."""
    m = SSTableManager(tmp_path, 2, 100000, engine)
    for i in range(12):
        m.create([InternalPair(b"key", b"v%d" % i)], 4)
    assert m.get(b"key") == InternalPair(b"key", b"v11")
    m2 = SSTableManager(tmp_path, 2, 100000, engine)
    assert [os.path.basename(t.file.path) for t in m2.tables][:4] == \
        ["table_0", "table_1", "table_10", "table_11"]
    assert m2.get(b"key") == InternalPair(b"key", b"v9")


def test_compaction_failure_keeps_tables(engine, tmp_path, monkeypatch):
    """a device failure inside compaction leaves every table and
    file in place (get() still answers, table_0 is not overwritten)."""
    from horreum_amd.abi import HorreumGpuError, Status
    m = SSTableManager(tmp_path, 2, 10, engine)
    m.create([InternalPair(b"k%02d" % i, b"old%d" % i) for i in range(20)], 100)
    before = open(tmp_path / "table_0", "rb").read()

    def boom(*a, **k):
        raise HorreumGpuError(Status.HIP, "injected")

    monkeypatch.setattr(engine, "compact_host", boom)
    with pytest.raises(HorreumGpuError):
        m.flush([InternalPair(b"k05", b"new")], 100)
    assert len(m.tables) == 2
    assert open(tmp_path / "table_0", "rb").read() == before
    assert m.get(b"k05") == InternalPair(b"k05", b"new")
    assert m.get(b"k06") == InternalPair(b"k06", b"old6")
    monkeypatch.undo()
    assert m.compact() is True and len(m.tables) == 1
    assert m.get(b"k05") == InternalPair(b"k05", b"new")


def test_compaction_of_duplicate_key_table(engine, golden, tmp_path):
    """create() accepts any pair list (the reference's create_table test
    writes 'abc' twice, src/sstable/table.rs:93-108); compaction then follows
    the reference loop exactly instead of failing."""
    c = golden["table_create"]
    dup = [_p(kv) for kv in c["pairs"]]
    m = SSTableManager(tmp_path, 1, 10, engine)
    m.create(dup, 39)
    m.flush([InternalPair(b"abc", b"zz"), InternalPair(b"b", None)], 5)
    assert len(m.tables) == 1
    tabs = [[(p.key, p.value) for p in [InternalPair(b"abc", b"zz"), InternalPair(b"b", None)]],
            [(p.key, p.value) for p in dup]]
    datas = []
    for t in tabs:
        arena, rec = oracle.pack_pairs(t)
        datas.append(oracle.encode(arena, rec)[0])
    dec = [(d, oracle.decode(d)[0]) for d in datas]
    refs, _ = oracle.compact(dec)
    merged = [InternalPair(*oracle.pairs_from_spans(dec[t][0], dec[t][1][r:r + 1])[0])
              for t, r in refs]
    assert m.tables[0].get_all(engine) == merged


def test_cold_open_over_the_byte_budget(engine, tmp_path, knobs):
    """A directory larger than the batched decode's device byte budget opens
    group by group (HG_DECODE_GROUP_BYTES set below one table's share, so
    every table is a group), spans identical to the oracle's; the context's
    work buffers are released afterwards (hg_ctx_trim)."""
    import numpy as np
    rng = np.random.default_rng(41)
    want = []
    for i in range(6):
        pairs = [(b"k%06d" % j + bytes([i]), rng.integers(0, 256, int(rng.integers(0, 200)),
                                                           dtype=np.uint8).tobytes())
                 for j in range(int(rng.integers(1000, 4000)))]
        arena, rec = oracle.pack_pairs(pairs)
        data = oracle.encode(arena, rec)[0]
        (tmp_path / f"table_{i}").write_bytes(data.tobytes())
        want.append(oracle.decode(data)[0])
    knobs("HG_DECODE_GROUP_BYTES", str(64 << 10))
    m = SSTableManager(tmp_path, 10, 1000, engine)
    assert len(m.tables) == 6
    for t, w in zip(m.tables, want):
        got = [p.key for p in t.get_all(engine)]
        assert len(got) == w.size
        data = np.fromfile(t.file.path, dtype=np.uint8)
        assert got == [data[int(s["off"]) + 16:int(s["off"]) + 16 + int(s["klen"])].tobytes()
                       for s in w]
    knobs("HG_DECODE_GROUP_BYTES", str(1 << 40))
    m2 = SSTableManager(tmp_path, 10, 1000, engine)  # one group: same tables
    assert [t.get_size() for t in m2.tables] == [t.get_size() for t in m.tables]
