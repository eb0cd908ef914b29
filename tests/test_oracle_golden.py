"""CPU: pin the oracle restatement to the reference's own known-answer vectors
(tests/golden/format_vectors.json, transcribed from the reference tests)."""
import numpy as np
import pytest

from oracle import oracle


def _pairs(lst):
    return [(bytes.fromhex(k), None if v is None else bytes.fromhex(v)) for k, v in lst]


def _encode(lst, stride=0):
    arena, recs = oracle.pack_pairs(_pairs(lst))
    data, rec_off, blocks, rc = oracle.encode(arena, recs, stride)
    assert rc == 0
    return arena, recs, data, rec_off, blocks


def _decode_pairs(data):
    spans, n, kind, off, rc = oracle.decode(data)
    assert rc == 0 and kind == 0
    return oracle.pairs_from_spans(data, spans)


@pytest.mark.parametrize("case", ["serialize", "serialize_lacking_value", "serialize_non_ascii",
                                  "serialize_flatten", "storage_read"])
def test_serialize_vectors(golden, case):
    c = golden[case]
    _, _, data, _, _ = _encode(c["pairs"])
    assert data.tobytes().hex() == c["bytes"], c["ref"]


@pytest.mark.parametrize("case", ["deserialize", "deserialize_lacking_value",
                                  "deserialize_non_ascii", "storage_read"])
def test_deserialize_vectors(golden, case):
    c = golden[case]
    assert _decode_pairs(bytes.fromhex(c["bytes"])) == _pairs(c["pairs"]), c["ref"]


@pytest.mark.parametrize("case", ["deserialize_from_bytes", "storage_read_all", "table_iterate",
                                  "table_open_existing", "table_create"])
def test_round_trip_vectors(golden, case):
    c = golden[case]
    _, _, data, _, _ = _encode(c["pairs"])
    got = _decode_pairs(data)
    # decode yields None for an empty value (Some(b"") aliases None)
    want = [(k, v if v else None) for k, v in _pairs(c["pairs"])]
    assert got == want, c["ref"]


def test_ordering_vector(golden):
    c = golden["ordering"]
    (lk, lv), = _pairs(c["less"])
    (gk, gv), = _pairs(c["greater"])
    assert (lk, lv) < (gk, gv)  # derived Ord: key bytes, then value


def test_index_creation(golden):
    c = golden["index_creation"]
    arena, recs, _, _, blocks = _encode(c["pairs"], c["stride"])
    got = []
    for b in blocks:
        r = recs[int(b["first_rec"])]
        key = arena[int(r["key_off"]):int(r["key_off"]) + int(r["klen"])].tobytes().hex()
        got.append([key, int(b["position"]), int(b["length"])])
    assert got == c["blocks"], c["ref"]


def test_index_get(golden):
    c = golden["index_get"]
    arena, recs, _, _, blocks = _encode(c["pairs"], c["stride"])
    for key, want in c["lookups"]:
        got = oracle.index_get(blocks, arena, recs, bytes.fromhex(key))
        assert (list(got) if got else None) == want, (key, c["ref"])


def _table_get(arena, recs, data, blocks, key):
    """SSTable::get (src/sstable/table.rs:54-70) on the oracle."""
    hit = oracle.index_get(blocks, arena, recs, key)
    if hit is None:
        return None
    pos, ln = hit
    block = data[pos:pos + ln]
    pairs = _decode_pairs(block)
    keys = [k for k, _ in pairs]
    import bisect
    i = bisect.bisect_left(keys, key)
    return pairs[i] if i < len(keys) and keys[i] == key else None


def test_table_search(golden):
    c = golden["table_search"]
    arena, recs, data, _, blocks = _encode(c["pairs"], c["stride"])
    for key, want in c["gets"]:
        got = _table_get(arena, recs, data, blocks, bytes.fromhex(key))
        exp = None if want is None else (bytes.fromhex(want[0]),
                                         None if want[1] is None else bytes.fromhex(want[1]))
        assert got == exp, (key, c["ref"])


def test_manager_get_newest_first(golden):
    c = golden["manager_get_newest_first"]
    tables = [_encode(t, c["stride"]) for t in c["tables_oldest_first"]]
    for key, want in c["gets"]:
        got = None
        for arena, recs, data, _, blocks in reversed(tables):  # newest -> oldest (manager.rs:126-134)
            got = _table_get(arena, recs, data, blocks, bytes.fromhex(key))
            if got is not None:
                break
        assert got == (bytes.fromhex(want[0]), None if want[1] is None else bytes.fromhex(want[1]))


def test_compaction(golden):
    c = golden["compaction"]
    iters = []  # in the order the test passes them to compact_inner
    for lst in c["iterators"]:
        _, _, data, _, _ = _encode(lst)
        spans, n, kind, _, rc = oracle.decode(data)
        iters.append((data, spans))
    picks, rc = oracle.compact(iters)
    assert rc == 0
    got = []
    for t, r in picks:
        data, spans = iters[t]
        got.extend(oracle.pairs_from_spans(data, spans[r:r + 1]))
    assert got == _pairs(c["expected"]), c["ref"]


def test_compaction_empty_is_error():
    picks, rc = oracle.compact([(np.zeros(1, np.uint8), np.zeros(0, oracle.SPAN_DTYPE))])
    assert rc == -5 and picks == []


def test_payload_size(golden):
    for lst, want in golden["payload_size"]["tables"]:
        _, _, data, _, _ = _encode(lst)
        spans, *_ = oracle.decode(data)
        assert oracle.payload_size(spans) == want


def test_oracle_table_get(golden):
    """src/sstable/table.rs:110-144 through the oracle's SSTable::get."""
    c = golden["table_search"]
    pairs = [(bytes.fromhex(k), None if v is None else bytes.fromhex(v)) for k, v in c["pairs"]]
    arena, rec = oracle.pack_pairs(pairs)
    data = oracle.encode(arena, rec)[0]
    spans = oracle.decode(data)[0]
    for key, want in c["gets"]:
        r = oracle.table_get(data, spans, c["stride"], bytes.fromhex(key))
        if want is None:
            assert r is None
        else:
            got = oracle.pairs_from_spans(data, spans[r:r + 1])[0]
            assert got == (bytes.fromhex(want[0]), None if want[1] is None else bytes.fromhex(want[1]))


def test_compacted_table_matches_compact_then_encode():
    """oracle.compacted_table (used by the config-size GPU tests) equals
    compact() + serialize_flatten of the picked pairs, blocks included."""
    rng = np.random.default_rng(3)
    tabs = []
    for _ in range(4):
        keys = sorted(set(rng.integers(0, 500, 300).tolist()))
        pairs = [(b"k%05d" % k, None if rng.random() < .1 else
                  bytes(rng.integers(0, 256, rng.integers(1, 40), dtype=np.uint8))) for k in keys]
        arena, rec = oracle.pack_pairs(pairs)
        tabs.append(oracle.encode(arena, rec)[0])
    got, blocks, n = oracle.compacted_table(tabs, block_stride=7)
    decs = [(d, oracle.decode(d)[0]) for d in tabs]
    refs, _ = oracle.compact(decs)
    merged = [oracle.pairs_from_spans(decs[t][0], decs[t][1][r:r + 1])[0] for t, r in refs]
    arena, rec = oracle.pack_pairs(merged)
    want, _, wblocks, _ = oracle.encode(arena, rec, block_stride=7)
    assert n == len(merged)
    assert np.array_equal(got, want) and np.array_equal(blocks, wblocks)
