"""MemTable bookkeeping and its flush path (reference src/memtable/mod.rs).

The reference snapshots its BTreeMap into a Vec<InternalPair> (one clone of
every key and value) and hands that to the SSTable writer, which serialises
it twice (once for the file, once more for the index).  Here a flush packs
the sorted entries straight into one contiguous key||value arena plus
hg_pair descriptors -- the engine's encode input -- so the table bytes and
the index blocks come from a single device encode.

Size accounting follows mod.rs:75-120 exactly, including its quirks:
`actual_size` is a usize (wrapping arithmetic), a re-put adds only the value
length difference, a put over a tombstone adds only the value length, a
delete subtracts only the value length (the key stays counted) and a delete
of an absent key counts nothing.  A flush happens after a put that leaves
the size above the limit (mod.rs:99-104), never after a delete.
"""
import numpy as np

from .abi import PAIR_DTYPE

_MASK = (1 << 64) - 1


class MemTable:
    def __init__(self, size_limit, on_flush=None):
        """on_flush(arena, pairs, size): receives every flush (e.g.
        SSTableManager.flush_arena)."""
        self.map = {}
        self.size_limit = size_limit
        self.actual_size = 0
        self.on_flush = on_flush

    def get(self, key):
        """mod.rs:68-72 (None for absent and deleted keys)."""
        return self.map.get(bytes(key))

    def put(self, key, value):
        """mod.rs:75-106; returns the previous value (None if absent/deleted)."""
        key, value = bytes(key), bytes(value)
        had = key in self.map
        prev = self.map.get(key)
        self.map[key] = value
        if had and prev is not None:
            self.actual_size = (self.actual_size + len(value) - len(prev)) & _MASK
        elif had:
            self.actual_size = (self.actual_size + len(value)) & _MASK
        else:
            self.actual_size = (self.actual_size + len(key) + len(value)) & _MASK
        if self.actual_size > self.size_limit:
            self.flush()
            self.actual_size = 0
        return prev

    def delete(self, key):
        """mod.rs:108-120."""
        key = bytes(key)
        prev = self.map.get(key)
        self.map[key] = None
        if prev is not None:
            self.actual_size = (self.actual_size - len(prev)) & _MASK
        return prev

    def snapshot(self):
        """The flush payload: (arena uint8, PAIR_DTYPE descriptors) of the
        entries in key order (BTreeMap iteration order, mod.rs:130-136);
        vlen 0 = tombstone."""
        keys = sorted(self.map)
        n = len(keys)
        desc = np.zeros(n, dtype=PAIR_DTYPE)
        if n == 0:
            return np.zeros(1, np.uint8), desc
        vals = [self.map[k] or b"" for k in keys]
        kl = np.fromiter((len(k) for k in keys), dtype=np.uint64, count=n)
        vl = np.fromiter((len(v) for v in vals), dtype=np.uint64, count=n)
        starts = np.zeros(n, dtype=np.uint64)
        np.cumsum((kl + vl)[:-1], out=starts[1:])
        desc["key_off"] = starts
        desc["val_off"] = starts + kl
        desc["klen"] = kl
        desc["vlen"] = vl
        blob = b"".join(k + v for k, v in zip(keys, vals))
        arena = np.frombuffer(blob, dtype=np.uint8) if blob else np.zeros(1, np.uint8)
        return arena, desc

    def flush(self):
        """mod.rs:123-158: hand the sorted snapshot and the size over, clear."""
        arena, desc = self.snapshot()
        if self.on_flush is not None:
            self.on_flush(arena, desc, self.actual_size)
        self.map.clear()
