"""GPU parity: hg_decode_* (HIP, gfx950) vs the oracle restatement of
InternalPair::deserialize_from_bytes (src/format.rs:50-77).  Integer/byte
work, so the bar is bit-exact: identical spans, record count, error kind and
error offset."""
import numpy as np
import pytest

from oracle import oracle
from tests import corpus

pytestmark = pytest.mark.gpu

CHUNK = 16384          # bytes per piece staged in LDS
BATCH = 16 * CHUNK     # average bytes per workgroup ticket / look-back status
_BATCH_PRE = [0, 12, 25, 39, 54, 71, 89, 108]  # hg_decode.hip batch_pre(): varied batch sizes


def batch_edges(size):
    """Byte offsets where decode batches start (pieces 12..20 per batch)."""
    out, b = [], 1
    while True:
        e = ((b // 8) * 128 + _BATCH_PRE[b % 8]) * CHUNK
        if e >= size:
            return out
        out.append(e)
        b += 1


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


def test_host_path_pinned_registered_pageable(engine):
    """The three host-memory routes of hg_decode_host agree bit-exactly:
    pageable (threaded staging copies), registered (hipHostRegister) and
    pinned (torch pin_memory) -- on an ~80 MB table (two 64 MiB staging
    pieces, each copied by several host threads)."""
    import torch
    from horreum_amd.abi import SPAN_DTYPE
    data = corpus.make("mixed_4k")[2]
    data = np.tile(data, (80 << 20) // data.size + 1)
    ws, wn, wk, _, _ = oracle.decode(data)
    assert wk == 0
    out = engine.decode_host(data)
    assert (out.n, out.kind) == (wn, 0) and np.array_equal(out.spans, ws)
    assert not engine.host_is_pinned(data)
    reg = data.copy()
    engine.host_register(reg)
    try:
        assert engine.host_is_pinned(reg)
        out = engine.decode_host(reg)
        assert (out.n, out.kind) == (wn, 0) and np.array_equal(out.spans, ws)
    finally:
        engine.host_unregister(reg)
    pin = torch.from_numpy(data).pin_memory()
    spans_pin = torch.zeros(wn * 16, dtype=torch.uint8).pin_memory()
    sp = spans_pin.numpy().view(SPAN_DTYPE)
    out = engine.decode_host(pin.numpy(), out=sp)
    assert engine.host_is_pinned(pin.numpy()) and engine.host_is_pinned(sp)
    assert (out.n, out.kind) == (wn, 0) and np.array_equal(sp, ws)


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


def test_batch_edges(engine):
    """Cuts at look-back batch edges (128 KiB) and piece edges inside a batch."""
    arena, pairs = corpus.mixed(20000, 24, 96, seed=5)
    data, _, _, _ = oracle.encode(arena, pairs)
    assert data.size > 4 * BATCH
    cuts = set()
    for e in batch_edges(data.size):
        for d in (-17, -1, 0, 1, 16):
            cuts.add(e + d)
    for k in (1, 3, 7, 9, 15):
        for d in (-1, 0, 9):
            cuts.add(k * CHUNK + d)
    for cut in sorted(c for c in cuts if 0 < c < data.size):
        assert_same(engine, data[:cut])


def _fake_header_table(n, fake_at, fake_k, fake_v, seed):
    """16 B keys / 100 B values whose value bytes carry a plausible header
    (fake_k, fake_v) at value offset fake_at: a position whose header repeats
    one record length ahead, so entry guesses can lock onto the wrong phase."""
    rng = np.random.default_rng(seed)
    kl = np.full(n, 16, np.int64)
    vl = np.full(n, 100, np.int64)
    arena = rng.integers(0, 256, size=n * 116, dtype=np.uint8).reshape(n, 116)
    fake = np.frombuffer(int(fake_k).to_bytes(8, "little") + int(fake_v).to_bytes(8, "little"),
                         np.uint8)
    arena[:, 16 + fake_at:16 + fake_at + 16] = fake
    arena = arena.reshape(-1)
    pairs = np.zeros(n, dtype=oracle.PAIR_DTYPE)
    pairs["key_off"] = np.arange(n) * 116
    pairs["val_off"] = np.arange(n) * 116 + 16
    pairs["klen"] = kl
    pairs["vlen"] = vl
    data, _, _, _ = oracle.encode(arena, pairs)
    return data


def test_fake_headers_cfg2_size(engine):
    """The adversarial table at BASELINE cfg 2 size (8.13 M records, 1 GiB):
    every record's value carries a self-consistent fake header, so every
    pre-pass batch's entry guess can lock onto the wrong phase and chains of
    wrong-guess batches wait on each other's exact redo (the
    look-back budget must not turn a valid file into an error)."""
    data = _fake_header_table(8_134_407, 10, 4, 96, seed=12)
    assert data.size == 1_073_741_724
    assert_same(engine, data)


@pytest.mark.parametrize("zero", [False, True])
def test_midlarge_bench_size(engine, zero):
    """400-1200 B records at the size tools/decode_variants.py times (1 M
    records, ~816 MB): the pre-pass picks hop or lane-walk per batch here
    (DESIGN §3.1); zero-filled values add a header candidate every 16 bytes."""
    arena, pairs = corpus.mixed(1_000_000, 16, 1200, seed=81, kmin=16, vmin=400,
                                zero_values=zero)
    data = oracle.encode(arena, pairs)[0]
    del arena, pairs
    assert_same(engine, data)


@pytest.mark.parametrize("fake", [(10, 4, 96), (40, 0, 100), (2, 50, 50), (60, 1, 3)])
def test_fake_headers_in_values(engine, fake):
    """Adversarial phase: every record carries a self-consistent fake header.
    Wrong batch guesses must be redone exactly from the looked-back entry."""
    data = _fake_header_table(60000, *fake, seed=11)
    assert_same(engine, data)
    for cut in (BATCH * 3 + 5, BATCH * 17 - 1, data.size - 7):
        assert_same(engine, data[:cut])


@pytest.mark.parametrize("split_mb", [1, 3])
def test_stride_then_mixed(engine, split_mb):
    """Uniform 16/100 records, then mixed sizes: the stride pre-pass resolves
    (and predicts spans for) the head, the general engine the rest; spans the
    pre-pass wrote at predicted indices past the break must be repaired."""
    n1 = (split_mb << 20) // 132
    arena1, pairs1 = corpus.fixed(n1, 16, 100, seed=41)
    arena2, pairs2 = corpus.mixed(30000, 24, 300, seed=42)
    d1, _, _, _ = oracle.encode(arena1, pairs1)
    d2, _, _, _ = oracle.encode(arena2, pairs2)
    tail = oracle.encode(*corpus.fixed(20000, 8, 56, seed=43))[0]  # stride again, other R
    assert_same(engine, np.concatenate([d1, d2, tail]))
    assert_same(engine, np.concatenate([d2, d1]))


@pytest.mark.parametrize("mode", ["one_launch", "streams"])
def test_batch_decode(engine, knobs, mode):
    """hg_decode_batch_dev_async: several tables (incl. empty and broken ones)
    decoded in one launch chain (default) or on fanned-out streams; each
    equals its oracle.  Hop-mode (large record), stride and general-engine
    tables side by side."""
    import torch
    if mode == "streams":
        knobs("HG_DECODE_BATCH", "streams")
    names = ["fixed_16_100", "mixed_small", "tiny", "large_values", "mixed_4k", "zero_values"]
    datas = [corpus.make(nm)[2] for nm in names]
    datas.append(np.zeros(0, np.uint8))
    datas.append(datas[1][:-5])  # truncated
    big = oracle.encode(*_large_mixed(9000, seed=71))[0]
    datas += [big, big[:-3], np.zeros(0, np.uint8), big[: big.size // 3]]
    bad = big.copy()
    bad[int(oracle.decode(big)[0]["off"][4000]) + 3] = 0x7F  # klen ~2^30: body past the end
    datas.append(bad)
    dev = [engine.to_device(d) for d in datas]
    caps = [max(d.size // 16, 1) for d in datas]
    spans = [engine.empty(c * 16) for c in caps]
    res = engine.empty(24 * len(datas))
    engine.decode_batch_dev_async(dev, [d.size for d in datas], spans, caps, res)
    torch.cuda.synchronize()
    r = res.cpu().numpy()
    for i, d in enumerate(datas):
        ws, wn, wk, wo, _ = oracle.decode(d)
        n = int(r[24 * i:24 * i + 8].view("<u8")[0])
        kind = int(r[24 * i + 8:24 * i + 12].view("<i4")[0])
        off = int(r[24 * i + 16:24 * i + 24].view("<u8")[0])
        assert (n, kind, off if kind else 0) == (wn, wk, wo if wk else 0), names[i % len(names)]
        got = engine.spans_to_numpy(spans[i], min(n, caps[i]))
        assert np.array_equal(got, ws)


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


# ---- hop mode (large records: header-to-header walks through HBM) -----------------
@pytest.fixture
def hop_batches(knobs):
    """Force 64-piece pre-pass batches (16 hop segments per batch) on small tables."""
    knobs("HG_DECODE_BP", "64")
    knobs("HG_DECODE_SBP", "64")


def _large_mixed(n, seed, vmin=8, vmax=4096, tomb=0.05):
    arena, pairs = corpus.mixed(n, 16, vmax, seed=seed, kmin=16, vmin=vmin, tomb_frac=tomb)
    return arena, pairs


def _fake_chain_table(n, seed, fake_v=600, reps=4):
    """Values of 2-4 KiB that each carry a chain of `reps` self-consistent fake
    headers (klen 0, vlen fake_v) -- windows that start inside a value lock
    onto the fake chain, whose 3-hop span passes the large-record test."""
    rng = np.random.default_rng(seed)
    arena, pairs = _large_mixed(n, seed, vmin=2048, vmax=4096, tomb=0.0)
    hdr = np.frombuffer((0).to_bytes(8, "little") + int(fake_v).to_bytes(8, "little"), np.uint8)
    for i in range(n):
        vo = int(pairs["val_off"][i]) + int(rng.integers(0, 64))
        for r in range(reps):
            o = vo + r * (16 + fake_v)
            arena[o:o + 16] = hdr
    data, rec_off, _, _ = oracle.encode(arena, pairs)
    return data, rec_off


@pytest.mark.parametrize("batches", ["adaptive", "forced64"])
def test_hop_mode_mixed_4k(engine, request, batches):
    """cfg-4-shaped records (16 B keys, 8..4096 B values, 5 % tombstones):
    the pre-pass hops headers; spans bit-exact vs the oracle, whole table
    and cut inside / at the edges of 64 KiB hop segments."""
    if batches == "forced64":
        request.getfixturevalue("hop_batches")
    arena, pairs = _large_mixed(24000, seed=61)
    data, rec_off, _, _ = oracle.encode(arena, pairs)
    assert data.size > 40 << 20
    assert_same(engine, data)
    seg = 4 * CHUNK
    cuts = {data.size - 1, data.size - 17, int(rec_off[-1]) + 3}
    for k in (1, 5, 16, 17, 63, 64, 65):
        for d in (-16, -1, 0, 1, 15):
            cuts.add(k * seg + d)
    cuts.update(int(x) + d for x in rec_off[[100, 5000, 12345]] for d in (0, 1, 16, 17))
    for cut in sorted(c for c in cuts if 0 < c < data.size):
        assert_same(engine, data[:cut])


def test_hop_mode_corrupt_and_fake_chains(engine, hop_batches):
    """Hop batches with a corrupt length mid-table (exact error kind/offset)
    and values carrying fake header chains (wrong segment guesses are
    re-walked from the predecessor's exit)."""
    arena, pairs = _large_mixed(12000, seed=62)
    data, rec_off, _, _ = oracle.encode(arena, pairs)
    for i in (7, 3001, 9000):
        bad = data.copy()
        o = int(rec_off[i])
        bad[o + 8:o + 16] = np.frombuffer((1 << 41).to_bytes(8, "little"), np.uint8)
        assert_same(engine, bad)
    fake, _ = _fake_chain_table(8000, seed=63)
    assert_same(engine, fake)
    assert_same(engine, fake[: fake.size // 2 + 999])


def test_hop_mode_records_larger_than_window(engine, hop_batches):
    """Values of 5-70 KiB: many 64 KiB segments have no record start in
    their 4 KiB window (no guess) and are entered from the stitch."""
    arena, pairs = _large_mixed(1500, seed=64, vmin=5000, vmax=70000, tomb=0.02)
    data, _, _, _ = oracle.encode(arena, pairs)
    assert_same(engine, data)
    assert_same(engine, data[: data.size - 1000])


def test_hop_wide_segments_meeting_small_records(engine):
    """Tables past 64 MiB get pre-pass batches of >= 8 pieces; a batch whose
    piece 0 holds a few KiB-sized records walks 128 KiB hop segments
    (HOP_WIDE).  Islands of 100-byte records inside such segments pass a
    walk's record limit and send their batches to the general engine: spans,
    count and errors still equal the oracle's."""
    parts, rng = [], np.random.default_rng(77)
    for k in range(4):
        parts.append(_shape_table(10_500, (16, 17), (3000, 4096), seed=70 + k))
        if k < 3:
            parts.append(_shape_table(int(rng.integers(300, 9000)), (8, 17), (60, 100), seed=80 + k))
    data = np.concatenate(parts)
    assert data.size > 130 * (1 << 20)
    assert_same(engine, data)
    offs = oracle.decode(data)[0]["off"]
    bad = data.copy()
    o = int(offs[offs.size // 2])
    bad[o + 8:o + 16] = np.frombuffer(int(1 << 33).to_bytes(8, "little"), np.uint8)
    assert_same(engine, bad)


@pytest.mark.parametrize("shape", ["medium", "huge", "small_far"])
def test_guess_rules_shapes(engine, shape):
    """Tables that exercise the guess rules over many general batches:
    medium records (serial short walks of up to 64 records per piece),
    values up to 64 KiB (pieces without any record start are speculated
    empty), and small records whose shifted header reads decode as far
    candidates (>= 8 KiB, guesses only as a fallback).  Each whole, cut
    mid-record and cut at a piece edge, bit-exact vs the oracle."""
    if shape == "medium":
        arena, pairs = corpus.mixed(60000, 64, 512, seed=81, kmin=8, vmin=64)
    elif shape == "huge":
        arena, pairs = corpus.mixed(900, 16, 65536, seed=82, kmin=16, tomb_frac=0.02)
    else:
        arena, pairs = corpus.mixed(300000, 24, 64, seed=83)
    data, _, _, _ = oracle.encode(arena, pairs)
    assert data.size > 8 * (1 << 20)
    assert_same(engine, data)
    assert_same(engine, data[: data.size - 7])
    assert_same(engine, data[: (data.size // CHUNK - 3) * CHUNK])


def test_batch_decode_guess_shapes(engine):
    """One batched launch over tables of every shape the guess rules handle
    (stride, small, medium, 4 KiB, 64 KiB values) and truncated copies."""
    import torch
    specs = [corpus.fixed(30000, 16, 100, seed=91),
             corpus.mixed(150000, 24, 64, seed=92),
             corpus.mixed(30000, 64, 512, seed=93, kmin=8, vmin=64),
             corpus.mixed(4000, 16, 4096, seed=94, kmin=16, vmin=8),
             corpus.mixed(500, 16, 65536, seed=95, kmin=16)]
    datas = [oracle.encode(a, p)[0] for a, p in specs]
    datas += [d[: d.size - 11] for d in datas]
    dev = [engine.to_device(d) for d in datas]
    caps = [max(d.size // 16, 1) for d in datas]
    spans = [engine.empty(c * 16) for c in caps]
    res = engine.empty(24 * len(datas))
    engine.decode_batch_dev_async(dev, [d.size for d in datas], spans, caps, res)
    torch.cuda.synchronize()
    r = res.cpu().numpy()
    for i, d in enumerate(datas):
        ws, wn, wk, wo, _ = oracle.decode(d)
        n = int(r[24 * i:24 * i + 8].view("<u8")[0])
        kind = int(r[24 * i + 8:24 * i + 12].view("<i4")[0])
        off = int(r[24 * i + 16:24 * i + 24].view("<u8")[0])
        assert (n, kind, off if kind else 0) == (wn, wk, wo if wk else 0), i
        assert np.array_equal(engine.spans_to_numpy(spans[i], min(n, caps[i])), ws), i


def _shape_table(n, kr, vr, seed, zero_values=False):
    """decode_variants-style table built vectorised: n records, key lengths in
    [kr[0], kr[1]), value lengths in [vr[0], vr[1]) (5 % tombstones), random
    payload bytes (zero_values: every value byte 0)."""
    rng = np.random.default_rng(seed)
    kl = rng.integers(*kr, n)
    vl = rng.integers(*vr, n)
    vl[rng.random(n) < 0.05] = 0
    offs = np.concatenate([[0], np.cumsum(16 + kl + vl)])
    buf = rng.integers(0, 256, int(offs[-1]), dtype=np.uint8)
    if zero_values:  # value byte <=> inside [start + 16 + klen, next start)
        d = np.zeros(buf.size + 1, np.int32)
        np.add.at(d, offs[:-1] + 16 + kl, 1)
        np.add.at(d, offs[1:], -1)
        buf[np.cumsum(d[:-1]) > 0] = 0
    hdr = np.stack([kl, vl], axis=1).astype("<u8").view(np.uint8).reshape(n, 16)
    for i in range(16):
        buf[offs[:-1] + i] = hdr[:, i]
    return buf


_SB = np.dtype([("x0", "<u8"), ("exit", "<u8"), ("count", "<u4"), ("ok", "<u4"), ("pad", "<u8")])


def _prepass_codes(engine):
    """SpecBatch codes of the context's last decode (hg_decode.hip SB_*)."""
    import ctypes
    lib = engine.lib
    lib.hgk_ctx_workspace.restype = ctypes.c_void_p
    lib.hgk_ctx_workspace.argtypes = [ctypes.c_void_p]
    lib.hgk_debug_d2h.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
    lay = (ctypes.c_uint64 * 8)()
    lib.hgk_decode_last_layout(lay)
    sb_off, nspec = int(lay[0]), int(lay[2])
    sb = np.zeros(nspec, _SB)
    ws = lib.hgk_ctx_workspace(engine.ctx)
    lib.hgk_debug_d2h(sb.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(ws + sb_off), sb.nbytes)
    return sb["pad"] & 0xFFFFFFFF


@pytest.mark.parametrize("shape", [("small", 1_200_000, (0, 24), (0, 64)),
                                   ("medium", 220_000, (8, 65), (64, 513))])
def test_lane_walk_mode_at_scale(engine, shape):
    """Small / medium records over many pre-pass batches: the lane-walk mode
    (decode_spec_kernel, SB_LW) must resolve every batch itself -- its
    fallback to decode_kernel's engine is exact too, so parity alone would
    not notice a lane-walk regression -- and the spans must be bit-exact vs
    the oracle, whole and cut mid-record / at a piece edge."""
    _, n, kr, vr = shape
    data = _shape_table(n, kr, vr, seed=7)
    assert data.size > 48 * (1 << 20)
    assert_same(engine, data)
    codes = _prepass_codes(engine)
    assert np.mean(codes == 6) >= 0.99, np.unique(codes, return_counts=True)
    assert_same(engine, data[: data.size - 5])
    assert_same(engine, data[: (data.size // CHUNK - 5) * CHUNK + 3])


def _zero_valued(m, kr, vr, seed):
    """Random non-zero key bytes, all-zero value bytes (tools/decode_variants.py
    zero shapes): every 16 value bytes read as an empty record."""
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


def _decode_ms(engine, data, reps=3):
    import time
    import torch
    d = engine.to_device(data)
    spans = engine.empty(data.size // 16 * 16)
    res = engine.empty(64)
    engine.decode_dev_async(d, data.size, spans, data.size // 16, res)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        engine.decode_dev_async(d, data.size, spans, data.size // 16, res)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    return sorted(ts)[len(ts) // 2]


@pytest.mark.parametrize("shape", [("small", 1_500_000, (1, 24), (0, 64)),
                                   ("midlarge", 400_000, (16, 17), (400, 1201))])
def test_zero_valued_records_resolved_fast(engine, shape):
    """Zero-byte values (every position inside a value reads as an empty
    record): bit-exact vs the oracle, every pre-pass batch resolved by the
    lane walks (lw_guess_nz, the long lead-in), and no serial redo chain --
    round 2 took 984 ms on 832 MB of the midlarge shape; the bound here is
    loose (box noise) but three orders of magnitude below that."""
    _, m, kr, vr = shape
    data = _zero_valued(m, kr, vr, seed=9)
    assert_same(engine, data)
    codes = _prepass_codes(engine) & 0xFF
    assert np.mean(codes == 6) >= 0.99, np.unique(codes, return_counts=True)
    assert _decode_ms(engine, data) < 25.0
    assert_same(engine, data[: data.size - 3])


def test_one_lane_chunk_walk_errors(engine):
    """Chunks of at most HG_LW_SER records (zero-valued 400-1200 B records)
    are walked by one lane (lw_chunk_walk); a length it cannot follow -- past
    the file, a high word set, past 2^32 -- falls back to the exact serial
    walk: error kind and offset equal the oracle's, and the unbroken prefix
    before each corruption decodes bit-exact."""
    data = _zero_valued(60_000, (16, 17), (400, 1201), seed=11)
    offs = oracle.decode(data)[0]["off"]
    rng = np.random.default_rng(12)
    for i in rng.integers(200, offs.size - 200, size=4):
        o = int(offs[i])
        for field, val in [(8, 1 << 33), (8, (1 << 32) - 1), (0, 1 << 40), (8, data.size)]:
            bad = data.copy()
            bad[o + field:o + field + 8] = np.frombuffer(int(val).to_bytes(8, "little"), np.uint8)
            assert_same(engine, bad)
        assert_same(engine, data[:o + 7])


def _ctl_words(engine):
    """DecodeCtl of the last single-table decode (ticket, bad_rev, progress,
    repairs): its control region is one of two the context uses in turn."""
    import ctypes
    lib = engine.lib
    lib.hgk_ctx_decode_ctl.restype = ctypes.c_void_p
    lib.hgk_ctx_decode_ctl.argtypes = [ctypes.c_void_p]
    lib.hgk_debug_d2h.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
    ctl = np.zeros(4, np.uint32)
    lib.hgk_debug_d2h(ctl.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(lib.hgk_ctx_decode_ctl(engine.ctx)), 16)
    return ctl


def _ctl_repairs(engine):
    return int(_ctl_words(engine)[3])


@pytest.mark.parametrize("fake_every", [1, 3])
def test_splice_repair_of_wrong_batch_entries(engine, fake_every):
    """A pre-pass batch whose guessed entry is wrong but whose path joins the
    true one (a fake header planted inside the value that spans the batch's
    first byte, decoding as one record that lands on a later true header) is
    spliced onto its predecessor's exit (splice_repair) instead of decoded
    again: spans bit-exact vs the oracle, repairs counted."""
    arena, pairs = _large_mixed(30000, seed=71, vmin=1024, vmax=4096, tomb=0.0)
    data, rec_off, _, _ = oracle.encode(arena, pairs)
    starts = rec_off.astype(np.int64)
    assert_same(engine, data)  # learn the pre-pass geometry of this size
    import ctypes
    lay = (ctypes.c_uint64 * 8)()
    engine.lib.hgk_decode_last_layout(lay)
    sbp = int(lay[3])
    bsz = sbp * CHUNK
    planted = 0
    for b in range(1, data.size // bsz, fake_every):
        B = b * bsz
        i = int(np.searchsorted(starts, B, side="right")) - 1  # record spanning B
        if i + 3 >= starts.size:
            break
        vstart = int(starts[i]) + 16 + int(pairs["klen"][i])
        f = max(B + 5, vstart)
        if f + 16 > int(starts[i + 1]) - 16:
            continue  # no room inside this value before the next header
        h2 = int(starts[i + 2])  # the fake record jumps over starts[i + 1]
        body = h2 - f - 16
        hdr = (40).to_bytes(8, "little") + int(body - 40).to_bytes(8, "little")
        data[f:f + 16] = np.frombuffer(hdr, np.uint8)
        planted += 1
    assert planted > 10
    assert_same(engine, data)
    assert _ctl_repairs(engine) > 0


def _prepass_links(engine, sst):
    """Decode `sst` (device) and read back the pre-pass batch records
    (tools/spec_diag.py's view): (spans result, first_bad, link mismatches,
    splice repairs, pre-pass codes)."""
    import ctypes
    lib = engine.lib
    lib.hgk_ctx_workspace.restype = ctypes.c_void_p
    lib.hgk_ctx_workspace.argtypes = [ctypes.c_void_p]
    lib.hgk_debug_d2h.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
    out = engine.decode_dev(sst, sst.numel())
    lay = (ctypes.c_uint64 * 8)()
    lib.hgk_decode_last_layout(lay)
    sb_off, _, nspec = list(lay)[:3]
    ws = lib.hgk_ctx_workspace(engine.ctx)
    sbd = np.dtype([("x0", "<u8"), ("exit", "<u8"), ("count", "<u4"), ("ok", "<u4"), ("pad", "<u8")])
    sb = np.zeros(nspec, sbd)
    lib.hgk_debug_d2h(sb.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(ws + sb_off), sb.nbytes)
    ctl = _ctl_words(engine)
    links = int(np.sum(sb["x0"][1:] != sb["exit"][:-1]))
    return out, nspec - int(ctl[1]), links, int(ctl[3]), sb["pad"] & 0xFF, nspec


@pytest.mark.parametrize("seed", [4, 6])
def test_hop_entries_keep_tombstones(engine, knobs, seed):
    """Round-3 regression (cfg 4's batched decode 0.27 -> 0.48 ms): a hop
    segment's entry guess skipped a tombstone whose 16-byte key starts with
    zero bytes (header, zeros and key merged into one run of candidates whose
    end reads as an all-zero header), so the batch began one record late and
    every such batch was spliced behind a look-back chain.  At the batched
    geometry of cfg 4 (64-piece batches) every pre-pass batch of a cfg 4
    table must now link to its predecessor's exit: no repairs, nothing left
    to the general engine -- and the spans equal the generated layout."""
    from horreum_amd import synth
    knobs("HG_DECODE_BP", "64")
    knobs("HG_DECODE_SBP", "64")
    v = synth.mixed_table_vlens(64 << 20, 8, 4096, 0.05, seed=seed)
    keys = np.arange(v.size, dtype=np.uint64) * 7 + seed
    buf, offs = synth.keyed_table(keys, v, seed=seed, device=engine.device)
    out, first_bad, links, repairs, codes, nspec = _prepass_links(engine, buf)
    want = synth.span_rows(offs[:-1], np.full(v.size, 16), v)
    got = engine.spans_to_numpy(out.spans, out.n).view("<u8").reshape(-1, 2)
    assert out.kind == 0 and out.n == v.size and np.array_equal(got, want)
    assert (codes == 5).all(), codes  # every batch in hop mode
    assert (first_bad, links, repairs) == (nspec, 0, 0)



@pytest.mark.parametrize("kv", [(16, 100), (8, 56), (1, 0), (200, 3000)])
def test_uniform_stride_tables(engine, kv):
    """Fixed-size records of several sizes: bit-exact, at the capacity
    boundary too (cap = n, cap = n - 1: the capacity error), and torn last
    records."""
    n = (24 << 20) // (16 + sum(kv))
    data = oracle.encode(*corpus.fixed(n, kv[0], kv[1], seed=91))[0]
    assert_same(engine, data)
    assert_same(engine, data, cap=n)
    assert_same(engine, data, cap=n - 1)
    for cut in (BATCH * 5 + 3, data.size - 1):
        assert_same(engine, data[:cut])


@pytest.mark.parametrize("where", ["middle", "head", "tail"])
def test_broken_stride_lattice(engine, where):
    """One record of another size breaks the stride lattice: batches past it
    are stride runs whose positions are not (x0 - entry) / R."""
    n = (16 << 20) // 132
    arena, pairs = corpus.fixed(n, 16, 100, seed=92)
    i = {"middle": n // 2, "head": 3, "tail": n - 2}[where]
    pairs = pairs.copy()
    pairs["vlen"][i] = 37  # one shorter value (its bytes are the next ones in the arena)
    data = oracle.encode(arena, pairs)[0]
    assert_same(engine, data)


@pytest.mark.parametrize("split", ["halves", "every_batch"])
def test_one_stride_two_shapes(engine, split):
    """Records of one length R but two (klen, vlen) shapes: every pre-pass
    batch is a stride run on the one lattice entry + i * R, but the spans'
    lengths differ from piece to piece: bit-exact vs the oracle."""
    n = (24 << 20) // 132
    arena, pairs = corpus.fixed(n, 16, 100, seed=94)
    pairs = pairs.copy()
    sel = np.arange(n) >= n // 2 if split == "halves" else (np.arange(n) // 9000) % 2 == 1
    pairs["klen"][sel] = 20
    pairs["vlen"][sel] = 96
    data = oracle.encode(arena, pairs)[0]
    assert_same(engine, data)


def test_control_region_reuse(engine):
    """hg_decode_dev_async keeps two control regions and each call's pre-pass
    clears the next call's, so a call whose region is already clear skips the
    memset.  Calls of growing, shrinking and repeated sizes, a corrupt table
    and a stride table in between, on one context: every result bit-exact vs
    the oracle (a stale status, link or ticket would misplace spans)."""
    big = _shape_table(400_000, (0, 24), (0, 64), seed=11)
    small = _shape_table(30_000, (8, 65), (64, 513), seed=12)
    bad = big[: big.size // 2].copy()
    bad[bad.size // 3 + 8:bad.size // 3 + 16] = 0xFF  # a length field past the end
    stride = _shape_table(200_000, (16, 17), (100, 101), seed=13)
    tables = {"big": big, "small": small, "bad": bad, "stride": stride, "tiny": big[:100]}
    want = {k: oracle.decode(v) for k, v in tables.items()}
    dev = {k: engine.to_device(v) for k, v in tables.items()}
    for name in ["big", "big", "small", "big", "bad", "big", "small", "small", "stride",
                 "stride", "tiny", "big", "bad", "bad", "small", "big"]:
        ws, wn, wk, wo, _ = want[name]
        out = engine.decode_dev(dev[name], tables[name].size)
        spans = engine.spans_to_numpy(out.spans, min(out.n, tables[name].size // 16))
        assert (out.n, out.kind, out.offset) == (wn, wk, wo), name
        assert np.array_equal(spans, ws), name


def test_batch_control_region_reuse(engine):
    """hg_decode_batch_dev_async keeps its tables' control regions in two
    halves (each call's pre-pass clears the other) and skips the argument
    copy when the staged bytes are unchanged.  Repeated calls on the same
    buffers (also after their bytes changed in place: same arguments, new
    data), a different table set with an empty table in between, then the
    first set again: every table bit-exact vs the oracle."""
    import torch

    outs = {}  # output buffers per device-table list: repeated calls pass the same pointers

    def run(devs, datas):
        caps = [max(d.size // 16, 1) for d in datas]
        if id(devs) not in outs:
            outs[id(devs)] = ([engine.empty(c * 16) for c in caps], engine.empty(24 * len(datas)))
        spans, res = outs[id(devs)]
        for sp in spans:
            sp.fill_(0xEE)  # stale spans from the previous call must not survive
        engine.decode_batch_dev_async(devs, [d.size for d in datas], spans, caps, res)
        torch.cuda.synchronize()
        r = res.cpu().numpy()
        for i, d in enumerate(datas):
            ws, wn, wk, wo, _ = oracle.decode(d)
            n = int(r[24 * i:24 * i + 8].view("<u8")[0])
            kind = int(r[24 * i + 8:24 * i + 12].view("<i4")[0])
            off = int(r[24 * i + 16:24 * i + 24].view("<u8")[0])
            assert (n, kind, off if kind else 0) == (wn, wk, wo if wk else 0), i
            assert np.array_equal(engine.spans_to_numpy(spans[i], min(n, caps[i])), ws), i

    a = [oracle.encode(*_large_mixed(6000, seed=81))[0], _shape_table(100_000, (0, 24), (0, 64), seed=82),
         _shape_table(60_000, (16, 17), (100, 101), seed=83)]
    da = [engine.to_device(d) for d in a]
    run(da, a)
    run(da, a)
    # same buffers and sizes, other bytes: the arguments are unchanged
    other = _shape_table(100_000, (8, 20), (0, 40), seed=84)
    a1 = np.zeros_like(a[1])
    a1[:min(other.size, a1.size)] = other[:a1.size]
    da[1].copy_(engine.to_device(a1))
    a = [a[0], a1, a[2]]
    run(da, a)
    run(da, a)
    c = [a[2], np.zeros(0, np.uint8), oracle.encode(*_large_mixed(3000, seed=85))[0]]
    dc = [engine.to_device(d) for d in c]
    run(dc, c)
    run(dc, c)
    run(da, a)
    run(da, a)


def test_batch_staging_halves_with_varying_table_counts(engine):
    """The argument staging of hg_decode_batch_dev_async alternates between
    two halves of one device buffer, and a call whose staged bytes equal the
    half's last ones skips the copy.  Calls of different table counts in turn
    (3, 1, 3, 2, 3 ... tables): a half's place must not depend on the count,
    or a one-table call's second half overwrites the three-table arguments
    that the next identical call then reuses without a copy (found in round
    5: the next call decoded the previous tables).  Every result bit-exact."""
    import torch

    outs = {}

    def run(key, devs, datas):
        caps = [max(d.size // 16, 1) for d in datas]
        if key not in outs:
            outs[key] = ([engine.empty(c * 16) for c in caps], engine.empty(24 * len(datas)))
        spans, res = outs[key]
        res.fill_(0xEE)
        engine.decode_batch_dev_async(devs, [d.size for d in datas], spans, caps, res)
        torch.cuda.synchronize()
        r = res.cpu().numpy()
        for i, d in enumerate(datas):
            ws, wn, wk, wo, _ = oracle.decode(d)
            n = int(r[24 * i:24 * i + 8].view("<u8")[0])
            kind = int(r[24 * i + 8:24 * i + 12].view("<i4")[0])
            assert (n, kind) == (wn, wk), (key, i)
            assert np.array_equal(engine.spans_to_numpy(spans[i], min(n, caps[i])), ws), (key, i)

    sets = {}
    for key, seeds in (("three", (91, 92, 93)), ("one", (94,)), ("two", (95, 96))):
        datas = [oracle.encode(*_large_mixed(2000 + 300 * j, seed=s))[0] for j, s in enumerate(seeds)]
        sets[key] = ([engine.to_device(d) for d in datas], datas)
    for key in ("three", "one", "three", "two", "three", "one", "one", "three", "three", "two", "two",
                "three"):
        run(key, *sets[key])


@pytest.mark.parametrize("where", ["clean", "bad_header_in_tail", "stride_change_in_tail",
                                   "stride_change_at_tail", "tombstones"])
def test_stride_batch_tails(engine, where):
    """A 528 MB fixed-stride table (pre-pass batches of 32+ pieces) with the
    damage placed in the last pieces of full batches -- the region a tail-task
    scheme would hand to another workgroup (measured in round 5, not kept):
    clean, a broken header, a stride change inside the last eight pieces or
    exactly at their start, and tombstones (vlen 0: other record sizes) there;
    every result bit-exact vs the oracle."""
    import ctypes
    from horreum_amd import synth
    rec = 132
    host = synth.fixed_sst(4_000_000, 16, 100, seed=5, device="cpu").numpy().copy()
    assert_same(engine, host)
    lay = (ctypes.c_uint64 * 8)()
    engine.lib.hgk_decode_last_layout(lay)
    sbp = int(lay[3])
    assert sbp > 16, sbp  # long batches
    tails = 8
    for b in (3, 11, 40):
        t0 = (b * sbp + sbp - tails) * CHUNK  # first byte of batch b's tail task
        if where == "clean":
            continue
        if where == "bad_header_in_tail":
            r = (t0 + 3 * CHUNK + rec - 1) // rec * rec
            host[r + 8:r + 16] = np.frombuffer((1 << 33).to_bytes(8, "little"), np.uint8)
            break  # one error: the oracle stops there
        if where == "tombstones":
            for k in range(5):
                r = (t0 + k * CHUNK + 7 * rec) // rec * rec
                host[r + 8:r + 16] = 0  # vlen 0: a 32-byte record, then 100 bytes read as records
            continue
        cut = (t0 + (CHUNK * 2 + 50 if where == "stride_change_in_tail" else 0) + rec - 1) // rec * rec
        suffix = oracle.encode(*corpus.fixed((host.size - cut) // 76, 16, 44, seed=9))[0]
        host = np.concatenate([host[:cut], suffix])
        break
    assert_same(engine, host)


@pytest.mark.parametrize("shape", [
    ("tiny", 3_000_000, (0, 3), (0, 3)),      # 16-21 B records: up to 4 starts per 64-byte lane
    ("empty_mix", 2_500_000, (0, 2), (0, 40)),  # many klen 0 / vlen 0 records (run ends 8 apart)
    ("small_wide", 1_000_000, (0, 200), (0, 64)),
    # zero-byte values: zero-heavy chunks (the gate), mixed with checked ones
    ("zero_small", 1_500_000, (1, 24), (0, 64), True),
    ("zero_small_empty_keys", 1_500_000, (0, 24), (0, 64), True),
    ("zero_midlarge", 200_000, (16, 17), (400, 1200), True),
    ("zero_tiny", 2_000_000, (1, 3), (0, 24), True),
])
def test_lane_walk_chunk_verification_shapes(engine, shape):
    """Round 6's per-chunk discovery (lw_chunk_verify: run-end candidates
    kept >= 16 bytes apart, verified at once by DPP scans, the lane walks for
    chunks that fail it) on shapes that stress it: records of 16-21 bytes
    (four starts in one lane), empty keys and tombstones (false run ends 8
    bytes into a record), wider keys; bit-exact vs the oracle whole, cut
    mid-record, and with a corrupt length planted in the middle (the verified
    set fails, the exact walk reports the error the oracle reports).  Zero-
    valued shapes: their zero-heavy chunks skip the check (the gate) and
    take the walks, the other chunks the check."""
    n, kr, vr = shape[1:4]
    data = _shape_table(n, kr, vr, seed=11, zero_values=len(shape) > 4 and shape[4])
    assert_same(engine, data)
    assert_same(engine, data[: data.size - 7])
    bad = data.copy()
    want = oracle.decode(bad)[0]
    mid = int(want["off"][want.size // 2])
    bad[mid + 8: mid + 16] = np.frombuffer(np.uint64(1 << 40).tobytes(), np.uint8)  # vlen past the file
    assert_same(engine, bad)
