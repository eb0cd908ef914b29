"""GPU parity: hg_decode_* (HIP, gfx950) vs the oracle restatement of
InternalPair::deserialize_from_bytes (src/format.rs:50-77).  Integer/byte
work, so the bar is bit-exact: identical spans, record count, error kind and
error offset."""
import numpy as np
import pytest

from oracle import oracle
from tests import corpus

pytestmark = pytest.mark.gpu

CHUNK = 16384


def gpu_decode(engine, data, cap=None):
    buf = np.frombuffer(memoryview(data).cast("B"), dtype=np.uint8)
    d = engine.to_device(buf)
    out = engine.decode_dev(d, buf.size, cap=cap)
    cap_eff = buf.size // 16 if cap is None else cap
    spans = engine.spans_to_numpy(out.spans, min(out.n, cap_eff))
    return spans, out.n, out.kind, out.offset


def assert_same(engine, data, cap=None):
    ws, wn, wk, wo, _ = oracle.decode(data, cap)
    gs, gn, gk, go = gpu_decode(engine, data, cap)
    assert (gn, gk, go) == (wn, wk, wo)
    assert np.array_equal(gs, ws)


@pytest.mark.parametrize("case", ["deserialize", "deserialize_lacking_value",
                                  "deserialize_non_ascii", "storage_read"])
def test_golden_vectors(engine, golden, case):
    data = bytes.fromhex(golden[case]["bytes"])
    spans, n, kind, _ = gpu_decode(engine, data)
    assert kind == 0
    want = [(bytes.fromhex(k), None if v is None else bytes.fromhex(v))
            for k, v in golden[case]["pairs"]]
    assert oracle.pairs_from_spans(data, spans) == want


@pytest.mark.parametrize("name", sorted(corpus.CORPORA))
def test_corpus_parity(engine, name):
    _, _, data, _ = corpus.make(name)
    assert data.size > 0
    assert_same(engine, data)


@pytest.mark.parametrize("name", ["fixed_16_100", "mixed_small", "tiny", "large_values"])
def test_host_path_parity(engine, name):
    _, _, data, _ = corpus.make(name)
    ws, wn, wk, wo, _ = oracle.decode(data)
    out = engine.decode_host(data)
    assert (out.n, out.kind, out.offset) == (wn, wk, wo)
    assert np.array_equal(out.spans, ws)


def test_empty_and_tiny_inputs(engine):
    for data in [b"", b"\x00", bytes(15), bytes(16), bytes(17), bytes(32), bytes(33),
                 bytes([3] + [0] * 15)]:
        if len(data) == 0:
            out = engine.decode_dev(engine.empty(1), 0, cap=0)
            assert (out.n, out.kind) == (0, 0)
            continue
        assert_same(engine, data)


@pytest.mark.parametrize("name", ["fixed_16_100", "mixed_4k", "tiny", "large_values"])
def test_truncations(engine, name):
    """Every cut lands either on a boundary (ok), in a header
    (TRUNCATED_HEADER) or in a body (TRUNCATED_BODY) -- at chunk edges too."""
    _, _, data, rec_off = corpus.make(name)
    rng = np.random.default_rng(7)
    cuts = set(rng.integers(1, data.size, size=12).tolist())
    for k in range(1, min(data.size // CHUNK, 6) + 1):
        for d in (-17, -16, -1, 0, 1, 15, 16, 17):
            if 0 < k * CHUNK + d < data.size:
                cuts.add(k * CHUNK + d)
    cuts.update(int(x) + d for x in rec_off[1:6] for d in (0, 1, 8, 15, 16, 17))
    for cut in sorted(c for c in cuts if 0 < c < data.size):
        assert_same(engine, data[:cut])


def test_corrupt_lengths(engine):
    _, _, data, rec_off = corpus.make("mixed_small")
    rng = np.random.default_rng(9)
    for i in rng.integers(1, rec_off.size - 1, size=6):
        o = int(rec_off[i])
        for field, val in [(0, 1 << 40), (8, 1 << 33), (0, (1 << 64) - 1), (8, (1 << 63) + 5)]:
            bad = data.copy()
            bad[o + field:o + field + 8] = np.frombuffer(int(val).to_bytes(8, "little"), np.uint8)
            assert_same(engine, bad)
    # klen + vlen overflowing u64
    bad = data.copy()
    o = int(rec_off[3])
    bad[o:o + 8] = np.frombuffer(((1 << 63) + 1).to_bytes(8, "little"), np.uint8)
    bad[o + 8:o + 16] = np.frombuffer(((1 << 63) + 1).to_bytes(8, "little"), np.uint8)
    assert_same(engine, bad)


def test_random_garbage(engine):
    rng = np.random.default_rng(21)
    for size in [100, 5000, 70000]:
        assert_same(engine, rng.integers(0, 256, size=size, dtype=np.uint8))
        assert_same(engine, np.zeros(size, np.uint8))  # zero-length keys/values, 16 B apart


def test_capacity(engine):
    _, _, data, _ = corpus.make("fixed_16_100")
    for cap in [0, 1, 777, 19999]:
        ws, wn, wk, wo, rc = oracle.decode(data, cap)
        gs, gn, gk, go = gpu_decode(engine, data, cap)
        assert (gn, gk, go) == (wn, wk, wo) and rc == 5
        assert np.array_equal(gs, ws)


def test_many_chunks_mixed(engine):
    """~12 MiB of mixed records: thousands of chunks, look-back over many windows."""
    arena, pairs = corpus.mixed(200000, 24, 96, seed=31)
    data, _, _, _ = oracle.encode(arena, pairs)
    assert_same(engine, data)


def test_cfg2_full_size(engine):
    """BASELINE config 2 at full size (1 GiB of 16 B/100 B records, device
    resident): checked by size-independent properties -- every span is
    (132 i, 16, 100) -- plus exact parity on a 64 MiB prefix."""
    import torch
    from horreum_amd import synth
    n = 8_134_407
    sst = synth.fixed_sst(n, 16, 100, seed=2, device=engine.device)
    assert sst.numel() == 1_073_741_724
    out = engine.decode_dev(sst, sst.numel(), cap=n)
    assert (out.n, out.kind) == (n, 0)
    sp = out.spans[: n * 16].view(torch.int64).view(n, 2)
    idx = torch.arange(n, device=sst.device, dtype=torch.int64)
    assert torch.equal(sp[:, 0], idx * 132)
    assert torch.equal(sp[:, 1], torch.full_like(idx, 16 | (100 << 32)))
    pre = sst[: 64 << 20].cpu().numpy()
    assert_same(engine, pre)
