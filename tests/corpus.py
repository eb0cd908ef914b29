"""Seeded synthetic SSTable corpora for parity tests (numpy; CPU side).

Every corpus is a list of (key, value | None) pairs plus its encoded bytes
(produced by the oracle restatement of src/format.rs:23-42, itself pinned by
the golden vectors).  Shapes cover what stresses boundary discovery: fixed
sizes, mixed sizes, tiny records (dense candidate headers), zero-filled
values (zero runs look like headers), values larger than a 16 KiB decode
chunk, tombstones and empty keys.
"""
import numpy as np

from oracle import oracle


def arena_pairs(keys_lens, vals_lens, rng, zero_values=False, key_fn=None):
    """Build (arena, PAIR_DTYPE) directly for large corpora (no Python lists)."""
    n = len(keys_lens)
    klen = np.asarray(keys_lens, dtype=np.uint64)
    vlen = np.asarray(vals_lens, dtype=np.uint64)
    sizes = klen + vlen
    offs = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(sizes, out=offs[1:])
    total = int(offs[-1])
    arena = (np.zeros(total, dtype=np.uint8) if zero_values
             else rng.integers(0, 256, size=total, dtype=np.uint8))
    pairs = np.zeros(n, dtype=oracle.PAIR_DTYPE)
    pairs["key_off"] = offs[:-1]
    pairs["val_off"] = offs[:-1] + klen
    pairs["klen"] = klen
    pairs["vlen"] = vlen
    if key_fn is not None:
        key_fn(arena, pairs)
    return arena, pairs


def be_counter_keys(arena, pairs):
    """Overwrite fixed-width keys with big-endian counters (sorted, unique)."""
    n = pairs.size
    if n == 0:
        return
    kl = int(pairs["klen"][0])
    idx = np.arange(n, dtype=np.uint64)
    ko = pairs["key_off"].astype(np.int64)
    for b in range(min(kl, 8)):
        arena[ko + (kl - 1 - b)] = ((idx >> np.uint64(8 * b)) & np.uint64(0xFF)).astype(np.uint8)
    for b in range(8, kl):
        arena[ko + (kl - 1 - b)] = 0


def fixed(n, k, v, seed, tomb_frac=0.0):
    rng = np.random.default_rng(seed)
    vl = np.full(n, v, dtype=np.uint64)
    if tomb_frac:
        vl[rng.random(n) < tomb_frac] = 0
    return arena_pairs(np.full(n, k), vl, rng, key_fn=be_counter_keys)


def mixed(n, kmax, vmax, seed, tomb_frac=0.05, zero_values=False, kmin=0, vmin=0):
    rng = np.random.default_rng(seed)
    kl = rng.integers(kmin, kmax + 1, size=n)
    vl = rng.integers(vmin, vmax + 1, size=n)
    if tomb_frac:
        vl[rng.random(n) < tomb_frac] = 0
    return arena_pairs(kl, vl, rng, zero_values=zero_values)


CORPORA = {
    # name: (generator, kwargs)
    "fixed_16_100": (fixed, dict(n=20000, k=16, v=100, seed=2)),
    "fixed_32_256": (fixed, dict(n=6000, k=32, v=256, seed=3)),
    "fixed_tomb": (fixed, dict(n=8000, k=16, v=100, seed=5, tomb_frac=0.3)),
    "mixed_small": (mixed, dict(n=30000, kmax=24, vmax=64, seed=11)),
    "tiny": (mixed, dict(n=40000, kmax=3, vmax=3, seed=12, tomb_frac=0.2)),
    "empty_keys_tombs": (mixed, dict(n=30000, kmax=0, vmax=2, seed=13, tomb_frac=0.5)),
    "zero_values": (mixed, dict(n=8000, kmax=16, vmax=200, seed=14, zero_values=True)),
    "mixed_4k": (mixed, dict(n=3000, kmax=32, vmax=4096, seed=15, kmin=8, vmin=8)),
    "large_values": (mixed, dict(n=120, kmax=64, vmax=70000, seed=16, tomb_frac=0.1)),
    "zero_large": (mixed, dict(n=60, kmax=8, vmax=50000, seed=17, zero_values=True)),
    # 400-1200 B records: the shape where the hop and lane-walk pre-passes
    # trade places; the zero-valued variant makes every value a
    # run of header candidates.
    "midlarge": (mixed, dict(n=4000, kmin=16, kmax=16, vmin=400, vmax=1200, seed=18)),
    "midlarge_zero": (mixed, dict(n=3000, kmin=16, kmax=16, vmin=400, vmax=1200, seed=19,
                                  zero_values=True)),
}


def make(name):
    gen, kw = CORPORA[name]
    arena, pairs = gen(**kw)
    data, rec_off, _, _ = oracle.encode(arena, pairs)
    return arena, pairs, data, rec_off
