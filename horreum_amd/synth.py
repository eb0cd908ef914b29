"""Synthetic, seeded SSTable workloads built directly in HBM (bench + tests).

BASELINE.json config 2: n records of 16-byte big-endian counter keys (sorted,
unique) and 100-byte uniform random values; config 3: 32 B / 256 B pairs in a
contiguous key||value arena with hg_pair descriptors.  Random bytes come from
torch's device generator (Philox) seeded per config; nothing is read from
disk or the network.
"""
import numpy as np


def _torch():
    import torch
    return torch


def be_counter_keys(n, k, device):
    """[n, k] uint8: big-endian counters 0..n-1."""
    torch = _torch()
    idx = torch.arange(n, device=device, dtype=torch.int64)
    cols = []
    for b in range(k - 1, -1, -1):
        cols.append(((idx >> (8 * b)) & 0xFF).to(torch.uint8) if b < 8
                    else torch.zeros(n, dtype=torch.uint8, device=device))
    return torch.stack(cols, dim=1)


def le64_rows(vals, device):
    """[n] int64 -> [n, 8] uint8 little-endian."""
    torch = _torch()
    return torch.stack([((vals >> (8 * b)) & 0xFF).to(torch.uint8) for b in range(8)], dim=1)


def fixed_sst(n, k, v, seed, device):
    """Encoded SSTable bytes of n fixed-size records, built on the device."""
    torch = _torch()
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    rec = torch.empty((n, 16 + k + v), dtype=torch.uint8, device=device)
    rec[:, 0:8] = le64_rows(torch.full((1,), k, dtype=torch.int64, device=device), device)
    rec[:, 8:16] = le64_rows(torch.full((1,), v, dtype=torch.int64, device=device), device)
    rec[:, 16:16 + k] = be_counter_keys(n, k, device)
    rec[:, 16 + k:] = torch.randint(0, 256, (n, v), dtype=torch.uint8, device=device, generator=g)
    return rec.view(-1)


def fixed_arena(n, k, v, seed, device):
    """(arena [n*(k+v)] uint8, pairs [n*24] uint8 as hg_pair) on the device."""
    torch = _torch()
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    arena = torch.empty((n, k + v), dtype=torch.uint8, device=device)
    arena[:, :k] = be_counter_keys(n, k, device)
    arena[:, k:] = torch.randint(0, 256, (n, v), dtype=torch.uint8, device=device, generator=g)
    idx = torch.arange(n, device=device, dtype=torch.int64)
    pairs = torch.empty((n, 3), dtype=torch.int64, device=device)
    pairs[:, 0] = idx * (k + v)
    pairs[:, 1] = idx * (k + v) + k
    pairs[:, 2] = k | (v << 32)
    return arena.view(-1), pairs.view(torch.uint8).view(-1)


def host_fixed_sst(n, k, v, seed):
    """numpy twin of fixed_sst for CPU baselines (same layout, numpy RNG)."""
    rng = np.random.default_rng(seed)
    rec = np.empty((n, 16 + k + v), dtype=np.uint8)
    rec[:, 0:8] = np.frombuffer(int(k).to_bytes(8, "little"), np.uint8)
    rec[:, 8:16] = np.frombuffer(int(v).to_bytes(8, "little"), np.uint8)
    idx = np.arange(n, dtype=np.uint64)
    for b in range(k):
        rec[:, 16 + k - 1 - b] = ((idx >> np.uint64(8 * b)) & np.uint64(0xFF)).astype(np.uint8) \
            if b < 8 else 0
    rec[:, 16 + k:] = rng.integers(0, 256, size=(n, v), dtype=np.uint8)
    return rec.reshape(-1)


def keyed_table(key_ids, vlens, seed, device):
    """Encoded SSTable with 16-byte big-endian keys `key_ids` (sorted uint64,
    host) and value lengths `vlens` (host; 0 = tombstone), random value bytes
    from the device generator.  Returns (bytes tensor, record offsets host)."""
    torch = _torch()
    key_ids = np.asarray(key_ids, dtype=np.uint64)
    vlens = np.asarray(vlens, dtype=np.int64)
    n = key_ids.size
    sizes = 32 + vlens
    offs = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(sizes, out=offs[1:])
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    buf = torch.randint(0, 256, (int(offs[-1]),), dtype=torch.uint8, device=device, generator=g)
    hdr = np.zeros((n, 32), dtype=np.uint8)
    hdr[:, 0] = 16
    hdr[:, 8:16] = vlens.astype("<u8").view(np.uint8).reshape(n, 8)
    hdr[:, 24:32] = key_ids.astype(">u8").view(np.uint8).reshape(n, 8)
    idx = torch.from_numpy(offs[:-1]).to(device)[:, None] + torch.arange(32, device=device)
    buf[idx.view(-1)] = torch.from_numpy(hdr).to(device).view(-1)
    return buf, offs


def mixed_table_vlens(max_bytes, vmin, vmax, tomb_frac, seed):
    """Value lengths of a table filled to <= max_bytes with 16-byte keys and
    values uniform in [vmin, vmax] (tomb_frac of them tombstones)."""
    rng = np.random.default_rng(seed)
    est = int(max_bytes / (32 + (vmin + vmax) / 2 * (1 - tomb_frac))) + 64
    v = rng.integers(vmin, vmax + 1, size=est)
    v[rng.random(est) < tomb_frac] = 0
    c = np.cumsum(32 + v)
    return v[: int(np.searchsorted(c, max_bytes, side="right"))]


def span_rows(offs, klens, vlens):
    """The spans a decode of a generated table must return (record offsets,
    key and value lengths as generated) as (n, 2) uint64 rows {off, klen |
    vlen << 32}: the hg_span layout, for checks by generator truth."""
    offs = np.asarray(offs, dtype=np.uint64)
    out = np.empty((offs.size, 2), dtype=np.uint64)
    out[:, 0] = offs
    out[:, 1] = np.asarray(klens, dtype=np.uint64) | (np.asarray(vlens, dtype=np.uint64) << np.uint64(32))
    return out


def mixed_sst_host(m, krange, vrange, tomb_frac, seed, layout=False, zero_values=False):
    """numpy SSTable of m records, key lengths uniform in krange = (lo, hi)
    and value lengths in vrange (hi exclusive), tomb_frac of the values
    tombstones, random key/value bytes (tools/decode_variants.py shapes);
    zero_values: non-zero key bytes and all-zero value bytes (every 16 value
    bytes then read as an empty record: the decode guesses' worst case).
    layout: also the generated (offsets, klens, vlens)."""
    rng = np.random.default_rng(seed)
    kl = rng.integers(*krange, m)
    vl = rng.integers(*vrange, m)
    vl[rng.random(m) < tomb_frac] = 0
    offs = np.concatenate([[0], np.cumsum(16 + kl + vl)])
    if zero_values:
        buf = np.zeros(int(offs[-1]), np.uint8)
        nk = int(kl.sum())
        kpos = np.repeat(offs[:-1] + 16, kl) + (np.arange(nk) - np.repeat(np.cumsum(kl) - kl, kl))
        buf[kpos] = rng.integers(1, 256, nk, dtype=np.uint8)
    else:
        buf = rng.integers(0, 256, int(offs[-1]), dtype=np.uint8)
    hdr = np.stack([kl, vl], axis=1).astype("<u8").view(np.uint8).reshape(m, 16)
    for i in range(16):
        buf[offs[:-1] + i] = hdr[:, i]
    return (buf, offs[:-1], kl, vl) if layout else buf
