"""The Python mirror of the reference API (horreum_amd.format / .index /
.table), tested the way the reference tests itself (src/format.rs:86-200,
src/sstable/index.rs:81-145, src/sstable/storage.rs:76-108,
src/sstable/table.rs:88-186), with the expected values from the golden
fixtures.  GPU-marked tests run the codec on the MI355X; the rest cover host
logic (ordering, index search, file quirks) and the loud failure without a
GPU."""
import os

import numpy as np
import pytest

from horreum_amd.format import DecodeError, InternalPair
from horreum_amd.index import Block, Index
from horreum_amd.table import PersistedFile, SSTable
from oracle import oracle


def _pairs(case):
    return [InternalPair(bytes.fromhex(k), None if v is None else bytes.fromhex(v))
            for k, v in case["pairs"]]


def _pair(kv):
    k, v = kv
    return InternalPair(bytes.fromhex(k), None if v is None else bytes.fromhex(v))


def _oracle_bytes(pairs):
    arena, rec = oracle.pack_pairs([(p.key, p.value) for p in pairs])
    data, _, _, _ = oracle.encode(arena, rec)
    return data.tobytes()


# ---- host logic (CPU) ----------------------------------------------------------------
def test_ordering(golden):
    """src/format.rs:177-183 (derived Ord: key, then None < Some)."""
    c = golden["ordering"]
    assert _pair(c["less"][0]) < _pair(c["greater"][0])
    assert InternalPair(b"a", None) < InternalPair(b"a", b"")
    assert InternalPair(b"a", b"x") < InternalPair(b"ab", None)
    assert InternalPair.default() == InternalPair(b"", None)


def test_index_get_host(golden):
    """src/sstable/index.rs:119-144 on the reference's block list."""
    pairs = _pairs(golden["index_creation"])
    idx = Index([Block(bytes.fromhex(k), p, n) for k, p, n in golden["index_creation"]["blocks"]])
    assert len(pairs) == 16
    for key, want in golden["index_get"]["lookups"]:
        got = idx.get(bytes.fromhex(key))
        assert got == (None if want is None else tuple(want))


def test_index_from_spans(golden):
    """Cold-open index (table.rs:46) from decode spans == the reference's
    Index::new blocks (index.rs:85-117), without a re-encode."""
    c = golden["index_creation"]
    data = _oracle_bytes(_pairs(c))
    spans, n, kind, _, _ = oracle.decode(data)
    assert kind == 0 and n == 16
    idx = Index.from_spans(data, spans, c["stride"])
    assert [(b.key.hex(), b.position, b.length) for b in idx.items] == \
        [tuple(b) for b in c["blocks"]]
    with pytest.raises(ValueError):
        Index.from_spans(data, spans, 0)


def test_persisted_file_no_truncate(tmp_path):
    """storage.rs:24-30 opens without truncate: a shorter write keeps the old tail."""
    path = tmp_path / "t"
    f = PersistedFile(path)
    f.write_bytes(b"A" * 40)
    f.write_bytes(b"B" * 10)
    assert open(path, "rb").read() == b"B" * 10 + b"A" * 30
    assert f.read_at(8, 4) == b"BBAA"
    with pytest.raises(EOFError):
        f.read_at(36, 8)
    with pytest.raises(FileNotFoundError):
        PersistedFile.open(tmp_path / "missing")


def test_pack_pairs_host():
    """The host packing of InternalPairs into the encode input (arena +
    descriptors) equals the oracle's, tombstones included (CPU only)."""
    from horreum_amd.format import pack_pairs
    rng = np.random.default_rng(3)
    pairs = [(rng.integers(0, 256, int(rng.integers(0, 20)), dtype=np.uint8).tobytes(),
              None if rng.random() < 0.2 else
              rng.integers(0, 256, int(rng.integers(0, 50)), dtype=np.uint8).tobytes())
             for _ in range(500)]
    arena, desc = pack_pairs([InternalPair(k, v) for k, v in pairs])
    warena, wdesc = oracle.pack_pairs(pairs)
    assert np.array_equal(desc, wdesc)
    assert arena[:warena.size].tobytes() == warena.tobytes()
    a0, d0 = pack_pairs([])
    assert d0.size == 0


def test_api_fails_loudly_without_gpu():
    """No CPU codec behind the API: without a HIP device the engine refuses."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    from horreum_amd import abi, format as fmt
    with pytest.raises(abi.HorreumGpuError):
        fmt.serialize_flatten([InternalPair(b"k", b"v")])


# ---- codec through the API (GPU) ---------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("case", ["serialize", "serialize_lacking_value", "serialize_non_ascii"])
def test_serialize(engine, golden, case):
    """src/format.rs:90-119."""
    c = golden[case]
    assert _pairs(c)[0].serialize(engine) == bytes.fromhex(c["bytes"])


@pytest.mark.gpu
def test_serialize_flatten(engine, golden):
    """src/format.rs:121-136."""
    c = golden["serialize_flatten"]
    assert InternalPair.serialize_flatten(_pairs(c), engine) == bytes.fromhex(c["bytes"])
    assert InternalPair.serialize_flatten([], engine) == b""


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["deserialize", "deserialize_lacking_value",
                                  "deserialize_non_ascii", "deserialize_from_bytes"])
def test_deserialize(engine, golden, case):
    """src/format.rs:138-200."""
    c = golden[case]
    data = bytes.fromhex(c["bytes"]) if "bytes" in c else _oracle_bytes(_pairs(c))
    assert InternalPair.deserialize_from_bytes(data, engine) == _pairs(c)


@pytest.mark.gpu
def test_deserialize_errors(engine, golden):
    """A trailing partial record: the reference returns Err(UnexpectedEof);
    here DecodeError with the kind and offset of the failing record."""
    data = bytes.fromhex(golden["storage_read"]["bytes"])
    with pytest.raises(DecodeError) as e:
        InternalPair.deserialize_from_bytes(data[:-1], engine)
    assert e.value.kind == 2 and e.value.offset == 24 and e.value.n_ok == 1
    with pytest.raises(DecodeError) as e:
        InternalPair.deserialize_from_bytes(data[:30], engine)
    assert e.value.kind == 1 and e.value.offset == 24


@pytest.mark.gpu
def test_storage_read(engine, golden, tmp_path):
    """src/sstable/storage.rs:78-107."""
    c = golden["storage_read"]
    f = PersistedFile.new(tmp_path / "s", _pairs(c), engine)
    assert bytes(f.read_bytes(engine)) == bytes.fromhex(c["bytes"])
    assert f.read_at(0, 24) == bytes.fromhex(c["bytes"])[:24]
    assert f.read_all(engine) == _pairs(c)
    pairs = _pairs(golden["storage_read_all"])
    assert PersistedFile.new(tmp_path / "a", pairs, engine).read_all(engine) == pairs


@pytest.mark.gpu
def test_index_creation(engine, golden):
    """src/sstable/index.rs:85-117: blocks from the same encode launch."""
    c = golden["index_creation"]
    idx = Index.new(_pairs(c), c["stride"], engine)
    assert [(b.key.hex(), b.position, b.length) for b in idx.items] == \
        [tuple(b) for b in c["blocks"]]
    for key, want in golden["index_get"]["lookups"]:
        assert idx.get(bytes.fromhex(key)) == (None if want is None else tuple(want))


@pytest.mark.gpu
def test_create_table(engine, golden, tmp_path):
    """src/sstable/table.rs:93-108."""
    c = golden["table_create"]
    pairs = _pairs(c)
    path = tmp_path / "test_create_table"
    f = PersistedFile.new(path, pairs, engine)
    table = SSTable.new(f, pairs, 39, c["stride"], engine)
    assert open(path, "rb").read() == InternalPair.serialize_flatten(pairs, engine)
    assert table.get_size() == 39


@pytest.mark.gpu
@pytest.mark.parametrize("via", ["new", "create", "open"])
def test_search_table(engine, golden, tmp_path, via):
    """src/sstable/table.rs:110-144, for a table made by new / create / open."""
    c = golden["table_search"]
    pairs = _pairs(c)
    path = tmp_path / "test_search_table"
    if via == "new":
        table = SSTable.new(PersistedFile.new(path, pairs, engine), pairs, 113, c["stride"], engine)
    elif via == "create":
        table = SSTable.create(path, pairs, 113, c["stride"], engine)
    else:
        PersistedFile.new(path, pairs, engine)
        table = SSTable.open(path, c["stride"], engine)
    assert table.get_size() == 113
    for key, want in c["gets"]:
        got = table.get(bytes.fromhex(key), engine)
        assert got == (None if want is None else _pair(want))


@pytest.mark.gpu
def test_iterate_table(engine, golden, tmp_path):
    """src/sstable/table.rs:146-168."""
    c = golden["table_iterate"]
    pairs = _pairs(c)
    f = PersistedFile.new(tmp_path / "i", pairs, engine)
    table = SSTable.new(f, pairs, 22, c["stride"], engine)
    assert table.get_all(engine) == pairs


@pytest.mark.gpu
def test_open_existing_file(engine, golden, tmp_path):
    """src/sstable/table.rs:170-185 (file written by the CPU oracle)."""
    c = golden["table_open_existing"]
    pairs = _pairs(c)
    path = tmp_path / "test_open_existing_file"
    path.write_bytes(_oracle_bytes(pairs))
    table = SSTable.open(path, c["stride"], engine)
    assert table.get_all(engine) == pairs
    assert table.get_size() == sum(len(p.key) + len(p.value or b"") for p in pairs)
    table.delete()
    assert not os.path.exists(path)


@pytest.mark.gpu
def test_payload_size(engine, golden, tmp_path):
    """table.rs:36-45 size accounting (manager.rs:283-306 expectations)."""
    for i, (kvs, want) in enumerate(golden["payload_size"]["tables"]):
        pairs = [_pair(kv) for kv in kvs]
        path = tmp_path / f"p{i}"
        PersistedFile.new(path, pairs, engine)
        assert SSTable.open(path, 3, engine).get_size() == want


@pytest.mark.gpu
def test_no_truncate_overwrite_fails_decode(engine, golden, tmp_path):
    """The no-truncate quirk end to end: a shorter table written over a
    longer file leaves a tail that no longer parses."""
    long_pairs = _pairs(golden["table_search"])
    short_pairs = _pairs(golden["table_iterate"])
    path = tmp_path / "q"
    PersistedFile.new(path, long_pairs, engine)
    f = PersistedFile.new(path, short_pairs, engine)
    data = bytes(f.read_bytes(engine))
    assert data.startswith(InternalPair.serialize_flatten(short_pairs, engine))
    want = oracle.decode(np.frombuffer(data, np.uint8))
    try:
        got = f.read_all(engine)
        assert want[2] == 0
        assert [(p.key, p.value) for p in got] == oracle.pairs_from_spans(data, want[0])
    except DecodeError as e:
        assert (e.kind, e.offset, e.n_ok) == (want[2], want[3], want[1])


@pytest.mark.gpu
def test_mapped_file_is_page_locked(engine, golden, tmp_path):
    """a table file is mmap'd once (pageable: staged
    transfers); PersistedFile.pin page-locks the same mapping so its bytes go
    to the device by direct DMA (hg_host_is_pinned); both read the same."""
    c = golden["storage_read"]
    f = PersistedFile.new(tmp_path / "m", _pairs(c), engine)
    arr = f.mapped(engine)
    assert bytes(arr) == bytes.fromhex(c["bytes"])
    assert not engine.host_is_pinned(arr)
    assert f.read_all(engine) == _pairs(c)
    assert f.pin(engine) is arr
    assert engine.host_is_pinned(arr)
    assert f.read_all(engine) == _pairs(c)
    f.delete()
    assert not (tmp_path / "m").exists()


@pytest.mark.gpu
def test_resident_lookups(engine, golden, tmp_path):
    """SSTable.get_many keeps the table resident in HBM: a second batch
    reuses it (no re-upload, no re-decode) and agrees with get()."""
    from horreum_amd.table import SSTable
    c = golden["table_search"]
    pairs = _pairs(c)
    t = SSTable.create(tmp_path / "r", pairs, 0, 3, engine)
    keys = [p.key for p in pairs] + [b"abc", b"zzz", b""]
    first = t.get_many(keys, engine)
    rt = t.resident(engine)
    second = t.get_many(list(reversed(keys)), engine)
    assert t.resident(engine) is rt
    assert first == [t.get(k, engine) for k in keys]
    assert second == list(reversed(first))


def test_rust_binary_search_two_level_matches_oracle():
    """index.rust_binary_search used as SSTable::get uses it (Index::get over
    block first keys, then the block; index.rs:72-78, table.rs:65-68) picks
    the oracle's record on tables with duplicate and unordered keys."""
    from horreum_amd.index import rust_binary_search
    rng = np.random.default_rng(5)
    for trial in range(40):
        n = int(rng.integers(1, 60))
        keys = [bytes(rng.choice(list(b"ab"), size=int(rng.integers(0, 3))).tolist()) for _ in range(n)]
        pairs = [(k, b"v") for k in keys]
        arena, recs = oracle.pack_pairs(pairs)
        data = oracle.encode(arena, recs)[0]
        spans = oracle.decode(data)[0]
        for stride in (1, 2, 3, 7):
            firsts = keys[::stride]
            for q in [b"", b"a", b"b", b"aa", b"ab", b"ba", b"bb", b"c", b"aaa"]:
                hit, b = rust_binary_search(firsts, q)
                got = None
                if hit or b > 0:
                    b = b if hit else b - 1
                    blk = keys[b * stride:(b + 1) * stride]
                    h2, j = rust_binary_search(blk, q)
                    got = b * stride + j if h2 else None
                assert got == oracle.table_get(data, spans, stride, q), (trial, stride, q)
    # Ok on the first probe that compares Equal, as Rust's std (1.52-1.81) does
    assert rust_binary_search([b"a", b"a", b"a", b"a"], b"a") == (True, 2)
    assert rust_binary_search([b"a", b"b"], b"c") == (False, 2)
