"""GPU parity: hg_encode_* (HIP, gfx950) vs the oracle restatement of
serialize/serialize_flatten (src/format.rs:23-42) and Index::new block
positions/lengths (src/sstable/index.rs:55-67).  Bit-exact bytes."""
import numpy as np
import pytest

from oracle import oracle
from tests import corpus

pytestmark = pytest.mark.gpu


def _pairs(lst):
    return [(bytes.fromhex(k), None if v is None else bytes.fromhex(v)) for k, v in lst]


def gpu_encode_dev(engine, arena, pairs, stride=0):
    import torch
    n = pairs.size
    total = int((16 + pairs["klen"].astype(np.uint64) + pairs["vlen"].astype(np.uint64)).sum())
    d_arena = engine.to_device(arena)
    d_pairs = engine.to_device(pairs.view(np.uint8))
    out = engine.empty(total)
    rec = torch.zeros(max(n, 1), dtype=torch.int64, device=engine.device)
    nb = (n + stride - 1) // stride if stride else 0
    blocks = engine.empty(max(nb, 1) * 24) if stride else None
    rc, out_len = engine.encode_dev(d_arena, d_pairs, n, out=out, cap=total, rec_off=rec,
                                    block_stride=stride, blocks=blocks)
    assert rc == 0 and out_len == total
    b = blocks[: nb * 24].cpu().numpy().view(oracle.BLOCK_DTYPE) if stride else None
    return out[:total].cpu().numpy(), rec[:n].cpu().numpy().astype(np.uint64), b


@pytest.mark.parametrize("case", ["serialize", "serialize_lacking_value", "serialize_non_ascii",
                                  "serialize_flatten", "storage_read"])
def test_golden_serialize(engine, golden, case):
    c = golden[case]
    arena, recs = oracle.pack_pairs(_pairs(c["pairs"]))
    out = engine.encode_host(arena, recs)
    assert out.data.tobytes().hex() == c["bytes"], c["ref"]
    data, _, _ = gpu_encode_dev(engine, arena, recs)
    assert data.tobytes().hex() == c["bytes"], c["ref"]


def test_golden_index(engine, golden):
    c = golden["index_creation"]
    arena, recs = oracle.pack_pairs(_pairs(c["pairs"]))
    out = engine.encode_host(arena, recs, block_stride=c["stride"])
    got = [[arena[int(recs[int(b["first_rec"])]["key_off"]):
                  int(recs[int(b["first_rec"])]["key_off"]) + int(recs[int(b["first_rec"])]["klen"])]
            .tobytes().hex(), int(b["position"]), int(b["length"])] for b in out.blocks]
    assert got == c["blocks"], c["ref"]


@pytest.mark.parametrize("name", sorted(corpus.CORPORA))
@pytest.mark.parametrize("stride", [0, 1, 10, 257])
def test_corpus_parity(engine, name, stride):
    arena, pairs = corpus.CORPORA[name][0](**corpus.CORPORA[name][1])
    want, wrec, wblk, _ = oracle.encode(arena, pairs, stride)
    data, rec, blk = gpu_encode_dev(engine, arena, pairs, stride)
    assert np.array_equal(data, want)
    assert np.array_equal(rec, wrec)
    if stride:
        assert np.array_equal(blk, wblk)


def test_unaligned_and_shuffled_sources(engine):
    """Descriptors pointing anywhere in the arena, in any order, overlapping."""
    rng = np.random.default_rng(5)
    arena = rng.integers(0, 256, size=1 << 16, dtype=np.uint8)
    n = 5000
    pairs = np.zeros(n, dtype=oracle.PAIR_DTYPE)
    pairs["klen"] = rng.integers(0, 40, n)
    pairs["vlen"] = rng.integers(0, 300, n)
    pairs["key_off"] = rng.integers(0, arena.size - 40, n)
    pairs["val_off"] = rng.integers(0, arena.size - 300, n)
    want, wrec, wblk, _ = oracle.encode(arena, pairs, 7)
    data, rec, blk = gpu_encode_dev(engine, arena, pairs, 7)
    assert np.array_equal(data, want) and np.array_equal(rec, wrec) and np.array_equal(blk, wblk)


def test_capacity(engine):
    arena, pairs = corpus.fixed(1000, 16, 100, seed=1)
    total = 1000 * 132
    d_arena = engine.to_device(arena)
    d_pairs = engine.to_device(pairs.view(np.uint8))
    out = engine.empty(total)
    out.fill_(0xAB)
    rc, out_len = engine.encode_dev(d_arena, d_pairs, 1000, out=out, cap=total - 5)
    assert rc == 5 and out_len == total
    assert int(out[total - 5:].cpu().numpy().min()) == 0xAB  # nothing past cap


def test_round_trip_encode_then_decode(engine):
    arena, pairs = corpus.mixed(50000, 40, 500, seed=8)
    data, _, _ = gpu_encode_dev(engine, arena, pairs)
    out = engine.decode_host(data)
    assert out.kind == 0 and out.n == pairs.size
    assert np.array_equal(out.spans["klen"], pairs["klen"])
    assert np.array_equal(out.spans["vlen"], pairs["vlen"])


def test_cfg3_full_size(engine):
    """BASELINE config 3 at full size: 10 M pairs of 32 B / 256 B -> 3.04 GB.
    Size-independent checks: total length, every header, record offsets,
    key/value bytes equal to the arena (compared on the device)."""
    import torch
    from horreum_amd import synth
    n, k, v = 10_000_000, 32, 256
    arena, pairs = synth.fixed_arena(n, k, v, seed=3, device=engine.device)
    total = n * (16 + k + v)
    out = engine.empty(total)
    rec = torch.empty(n, dtype=torch.int64, device=engine.device)
    rc, out_len = engine.encode_dev(arena, pairs, n, out=out, cap=total, rec_off=rec)
    assert rc == 0 and out_len == total == 3_040_000_000
    r = out.view(n, 16 + k + v)
    assert torch.equal(r[:, :16].contiguous().view(torch.int64),
                       torch.tensor([k, v], device=engine.device).expand(n, 2))
    assert torch.equal(r[:, 16:], arena.view(n, k + v))
    assert torch.equal(rec, torch.arange(n, device=engine.device, dtype=torch.int64) * (16 + k + v))


_EDGE_LENS = [0, 1, 7, 15, 16, 17, 31, 33]


def _edge_pairs(rng):
    """Uniform tiles (256 equal records: the division fast path) of every
    (klen, vlen) in _EDGE_LENS^2, then a tile mixing them all, in a shuffled
    arena: straddle pieces with sources shorter and longer than one 16-byte
    window, tails of 1..15 bytes, empty keys and tombstones."""
    combos = [(k, v) for k in _EDGE_LENS for v in _EDGE_LENS]
    kl, vl = [], []
    for k, v in combos[:12]:
        kl += [k] * 256
        vl += [v] * 256
    for _ in range(3):
        order = rng.permutation(len(combos))
        kl += [combos[i][0] for i in order]
        vl += [combos[i][1] for i in order]
    kl, vl = np.array(kl), np.array(vl)
    n = kl.size
    arena = rng.integers(0, 256, size=int((kl + vl).sum()) + 4096, dtype=np.uint8)
    pairs = np.zeros(n, dtype=oracle.PAIR_DTYPE)
    pairs["klen"], pairs["vlen"] = kl, vl
    # sources anywhere (unaligned), keys and values apart
    pairs["key_off"] = rng.integers(0, arena.size - 40, n)
    pairs["val_off"] = rng.integers(0, arena.size - 40, n)
    return arena, pairs


def test_piece_assembly_edges(engine):
    """Straddle/tail pieces assembled in registers and the uniform-tile path,
    bit-exact vs the oracle, with record offsets and blocks."""
    rng = np.random.default_rng(11)
    arena, pairs = _edge_pairs(rng)
    want, wrec, wblk, _ = oracle.encode(arena, pairs, 5)
    data, rec, blk = gpu_encode_dev(engine, arena, pairs, 5)
    assert np.array_equal(data, want)
    assert np.array_equal(rec, wrec) and np.array_equal(blk, wblk)


@pytest.mark.parametrize("cut", [1, 3, 8, 15, 16, 17, 31, 40, 77])
def test_capacity_cut_inside_pieces(engine, cut):
    """A capacity that ends inside a header, a straddle or a tail piece: every
    byte before it equals the oracle's, nothing at or past it is written."""
    rng = np.random.default_rng(12 + cut)
    arena, pairs = _edge_pairs(rng)
    want, _, _, _ = oracle.encode(arena, pairs)
    total = want.size
    cap = total - cut
    out = engine.empty(total)
    out.fill_(0xA5)
    rc, out_len = engine.encode_dev(engine.to_device(arena), engine.to_device(pairs.view(np.uint8)),
                                    pairs.size, out=out, cap=cap)
    got = out.cpu().numpy()
    assert rc == 5 and out_len == total
    assert np.array_equal(got[:cap], want[:cap])
    assert (got[cap:] == 0xA5).all()


@pytest.mark.parametrize("chunk_mb", ["16", None])
@pytest.mark.parametrize("shuffled", [False, True])
def test_host_encode_page_locked_chunks(engine, shuffled, chunk_mb, knobs):
    """hg_encode_host with page-locked arena, pairs and output takes the
    chunked path (upload of chunk i+1 overlapping the download of chunk i);
    > 64 MiB of output so several chunks run, with record offsets and blocks
    (global across chunks); shuffled pairs make every chunk reach far into
    the arena.  HG_ENC_CHUNK_MB=16 forces several chunks."""
    if chunk_mb:
        knobs("HG_ENC_CHUNK_MB", chunk_mb)
    rng = np.random.default_rng(21 + shuffled)
    n = 400_000
    kl = rng.integers(0, 48, n)
    vl = rng.integers(0, 400, n)
    vl[rng.random(n) < 0.05] = 0
    offs = np.concatenate([[0], np.cumsum(kl + vl)])
    arena = rng.integers(0, 256, int(offs[-1]), dtype=np.uint8)
    pairs = np.zeros(n, dtype=oracle.PAIR_DTYPE)
    pairs["key_off"], pairs["val_off"] = offs[:-1], offs[:-1] + kl
    pairs["klen"], pairs["vlen"] = kl, vl
    if shuffled:
        pairs = pairs[rng.permutation(n)]
    want, wrec, wblk, _ = oracle.encode(arena, pairs, 10)
    assert want.size > (64 << 20)  # > 4 chunks of 16 MiB
    out = np.empty(want.size, dtype=np.uint8)
    for a in (arena, pairs, out):
        engine.host_register(a)
    try:
        got = engine.encode_host(arena, pairs, block_stride=10, want_rec_off=True, out=out)
    finally:
        for a in (arena, pairs, out):
            engine.host_unregister(a)
    assert got.out_len == want.size
    assert np.array_equal(got.data, want)
    assert np.array_equal(got.rec_off, wrec) and np.array_equal(got.blocks, wblk)


def test_group_sums_reuse(engine):
    """hg_encode_dev keeps its group sums in two halves used in turn (each
    call's bases kernel clears the other, so a call no bigger than the last
    launches no memset): encodes of growing, shrinking and repeated sizes
    on one context, every output and record offset bit-exact vs the oracle
    (a stale group sum would shift a whole group of tiles)."""
    cases = {"big": corpus.mixed(300_000, 24, 96, seed=51), "small": corpus.mixed(3_000, 8, 40, seed=52),
             "mid": corpus.fixed(90_000, 16, 100, seed=53), "one": corpus.fixed(1, 4, 4, seed=54)}
    want = {k: oracle.encode(*v) for k, v in cases.items()}
    for name in ["big", "big", "small", "big", "mid", "mid", "one", "small", "big"]:
        arena, pairs = cases[name]
        data, rec_off, _, _ = want[name]
        got, rec, _ = gpu_encode_dev(engine, arena, pairs)
        assert np.array_equal(got, data), name
        assert np.array_equal(rec, rec_off.astype(np.uint64)), name
