"""GPU parity at BASELINE.json's config sizes (one GPU's share of each):

- config 4: 32 tables x 64 MiB (16 B keys, values uniform in 8 B..4 KiB, 5 %
  tombstones) decoded by one batched launch chain -- every span of every
  table against the oracle (src/format.rs:50-77);
- config 5 in miniature: 8 overlapping sorted tables, decode -> newest-wins
  merge -> encode on the device and through hg_compact_host, byte for byte
  against serialize_flatten(compact_inner(...)) built by the oracle
  (src/sstable/manager.rs:199-234, src/format.rs:40-42);
- config 5 at one GPU's full share (8 tables x 1 GiB, 65 M records): the
  compacted table must equal the key union with each key's record taken from
  the newest table holding it (a stable sort of (key, table) on the host),
  byte for byte -- a size-independent property the oracle does not need to
  replay record by record.
"""
import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu


def _device_tables(torch, eng, key_sets, vlens, seeds):
    from horreum_amd import synth
    return [synth.keyed_table(k, v, seed=s, device=eng.device)[0]
            for k, v, s in zip(key_sets, vlens, seeds)]


@pytest.mark.timeout(300)
def test_cfg4_batch_spans_vs_oracle(engine):
    import torch
    from horreum_amd import synth
    tabs, hosts = [], []
    for t in range(32):
        v = synth.mixed_table_vlens(64 << 20, 8, 4096, 0.05, seed=4 + t)
        keys = np.arange(v.size, dtype=np.uint64) * 7 + t
        buf, _ = synth.keyed_table(keys, v, seed=4 + t, device=engine.device)
        tabs.append(buf)
    lens = [b.numel() for b in tabs]
    caps = [n // 16 for n in lens]
    spans = [engine.empty(c * 16) for c in caps]
    res = engine.empty(24 * len(tabs))
    engine.decode_batch_dev_async(tabs, lens, spans, caps, res)
    torch.cuda.synchronize()
    r = res.cpu().numpy()
    for i, b in enumerate(tabs):
        host = b.cpu().numpy()
        want, wn, wk, _, _ = oracle.decode(host)
        n = int(r[24 * i:24 * i + 8].view("<u8")[0])
        kind = int(r[24 * i + 8:24 * i + 12].view("<i4")[0])
        assert (n, kind) == (wn, wk) == (wn, 0)
        got = spans[i][: n * 16].cpu().numpy().view(oracle.SPAN_DTYPE)
        assert np.array_equal(got, want), i
    assert sum(lens) > 2 * 10**9  # the whole per-GPU share was decoded


def _cfg5_tables(engine, ntab, per_table, seed):
    rng = np.random.default_rng(seed)
    shared = np.unique(rng.integers(0, 1 << 40, size=per_table // 4, dtype=np.uint64))
    keys = []
    for _ in range(ntab):
        own = rng.integers(0, 1 << 40, size=per_table - shared.size, dtype=np.uint64)
        keys.append(np.unique(np.concatenate([shared, own])))
    vl = [np.where(rng.random(k.size) < 0.05, 0, 100) for k in keys]
    bufs = _device_tables(None, engine, keys, vl, [50 + t for t in range(ntab)])
    return keys, vl, bufs


def _device_compact(engine, bufs):
    """Decode all (one batched chain) -> merge -> encode, all in HBM."""
    import torch
    sizes = [b.numel() for b in bufs]
    offs, total = [], 0
    for sz in sizes:
        offs.append(total)
        total += (sz + 7) & ~7
    arena = torch.zeros(max(total, 1), dtype=torch.uint8, device=engine.device)
    for o, b in zip(offs, bufs):
        arena[o:o + b.numel()] = b
    caps = [sz // 16 for sz in sizes]
    span_t = [engine.empty(c * 16) for c in caps]
    tabs = [arena[o:o + sz] for o, sz in zip(offs, sizes)]
    dres = engine.empty(24 * len(bufs))
    engine.decode_batch_dev_async(tabs, sizes, span_t, caps, dres)
    r = dres.cpu().numpy()
    counts = [int(r[24 * i:24 * i + 8].view("<u8")[0]) for i in range(len(bufs))]
    assert all(int(r[24 * i + 8:24 * i + 12].view("<i4")[0]) == 0 for i in range(len(bufs)))
    nmax = sum(counts)
    pairs = engine.empty(nmax * 24)
    m = engine.merge_dev(arena, offs, span_t, counts, pairs, nmax)
    assert m.status == 0
    out = engine.empty(total)
    rc, out_len = engine.encode_dev(arena, pairs, m.n, out=out, cap=total)
    assert rc == 0
    return out[:out_len], m.n


@pytest.mark.timeout(300)
@pytest.mark.parametrize("stride", [0, 10])
def test_cfg5_small_vs_oracle(engine, stride):
    """8 tables x 200 k records (26 MB each), 25 % shared keys, 5 % tombstones."""
    _, _, bufs = _cfg5_tables(engine, 8, 200_000, seed=5)
    hosts = [b.cpu().numpy() for b in bufs]
    want, wblocks, wn = oracle.compacted_table(hosts, block_stride=stride)
    got, n = _device_compact(engine, bufs)
    assert n == wn
    assert np.array_equal(got.cpu().numpy(), want)
    c = engine.compact_host(hosts, block_stride=stride)
    assert c.status == 0 and c.n == wn and np.array_equal(c.data, want)
    if stride:
        assert np.array_equal(c.blocks, wblocks)
    # hg_compact_dev (the bench leg's entry point) on the same device arena
    import torch
    offs, total = [], 0
    for b in bufs:
        offs.append(total)
        total += (b.numel() + 7) & ~7
    arena = torch.zeros(total, dtype=torch.uint8, device=engine.device)
    for o, b in zip(offs, bufs):
        arena[o:o + b.numel()] = b
    out = engine.empty(total)
    blocks = engine.empty(24 * (wn // stride + 2)) if stride else None
    d = engine.compact_dev(arena, offs, [b.numel() for b in bufs], out, stride, blocks)
    assert d.status == 0 and d.n == wn
    assert np.array_equal(d.data.cpu().numpy(), want)
    if stride:
        assert np.array_equal(d.blocks.cpu().numpy().view(wblocks.dtype), wblocks)


@pytest.mark.timeout(600)
def test_cfg5_full_share_property(engine):
    """8 x 1 GiB (8,134,407 records of 132 B each before dedup of the
    generator's keys): output == rows of the newest table per key."""
    import torch
    ntab, per = 8, 8_134_407
    rng = np.random.default_rng(55)
    shared = np.unique(rng.integers(0, 1 << 40, size=per // 4, dtype=np.uint64))
    keys, bufs = [], []
    from horreum_amd import synth
    for t in range(ntab):
        own = rng.integers(0, 1 << 40, size=per - shared.size, dtype=np.uint64)
        k = np.unique(np.concatenate([shared, own]))
        bufs.append(synth.keyed_table(k, np.full(k.size, 100), seed=60 + t,
                                      device=engine.device)[0])
        keys.append(k)
    assert sum(b.numel() for b in bufs) > 8 * 10**9
    allk = np.concatenate(keys)
    tid = np.concatenate([np.full(k.size, t, np.int64) for t, k in enumerate(keys)])
    row = np.concatenate([np.arange(k.size, dtype=np.int64) for k in keys])
    order = np.argsort(allk, kind="stable")
    ks = allk[order]
    first = np.ones(ks.size, bool)
    first[1:] = ks[1:] != ks[:-1]
    base = np.zeros(ntab + 1, np.int64)
    np.cumsum([k.size for k in keys], out=base[1:])
    want_rows = torch.from_numpy(base[tid[order][first]] + row[order][first]).to(engine.device)
    del allk, tid, row, order, ks
    got, n = _device_compact(engine, bufs)
    assert n == int(first.sum())
    rows = torch.cat(bufs).view(-1, 132)
    want = rows.index_select(0, want_rows).view(-1)
    assert got.numel() == want.numel()
    assert torch.equal(got, want)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("nctx", [1, 4])
def test_cfg4_all_256_tables_one_device(engine, nctx):
    """BASELINE config 4 at its FULL table count on one device: 256 tables x
    64 MiB (16 GiB; 16 B keys, values uniform in 8 B..4 KiB, 5 % tombstones)
    from host memory through hg_multi_decode_host (SSTableManager::new
    opening a directory, src/sstable/manager.rs:47-55) with `nctx` contexts
    sharing the GPU -- table i on context i % nctx, batched decode chains per
    group under the device byte budget.  Every span of every table against
    the oracle (src/format.rs:50-77).  (the largest batched decode
    tested had been 32 tables, and round 5's staging bug depended on the
    table count.)"""
    import torch
    from horreum_amd import synth
    from horreum_amd.multi import MultiEngine
    hosts = []
    for t in range(256):
        v = synth.mixed_table_vlens(64 << 20, 8, 4096, 0.05, seed=4 + t)
        keys = np.arange(v.size, dtype=np.uint64) * 7 + t
        buf, _ = synth.keyed_table(keys, v, seed=4 + t, device=engine.device)
        hosts.append(buf.cpu().numpy())
        del buf
    torch.cuda.empty_cache()
    assert sum(h.size for h in hosts) > 16 * 10**9
    m = MultiEngine([engine.device.index] * nctx)
    try:
        outs = m.decode_tables(hosts)
    finally:
        m.close()
    assert len(outs) == 256
    for i, (h, o) in enumerate(zip(hosts, outs)):
        want, wn, wk, _, _ = oracle.decode(h)
        assert (o.n, o.kind, wk) == (wn, 0, 0), i
        assert np.array_equal(o.spans, want), i
