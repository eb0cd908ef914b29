"""Python mirror of horreum's block index (reference src/sstable/index.rs).

`Index.new` takes the block positions and lengths from the SAME engine
launch that encodes the table (`hg_encode_*(..., block_stride, blocks)`),
replacing the reference's second full `serialize_flatten` per block
(src/sstable/index.rs:55-67).  `Index.from_spans` builds the same blocks
from a decode's spans (cold open, src/sstable/table.rs:46) without encoding
anything.  `get` is the reference's binary search (:72-78).
"""
from collections import namedtuple

import numpy as np

Block = namedtuple("Block", "key position length")  # src/sstable/index.rs:6-29


def rust_binary_search(keys, key):
    """Rust's slice::binary_search_by_key as the reference calls it
    (index.rs:74, table.rs:65), std 1.52-1.81: probe mid = left + (right -
    left) // 2 and return the first probe that compares Equal.  On keys that
    are not strictly increasing (legal, table.rs:93-108) this picks the same
    record the reference does, not just any record with the key.  Returns
    (True, i) for Ok(i), (False, i) for Err(i).  hg_lookup.hip runs the same
    search on the device."""
    left, right = 0, len(keys)
    while left < right:
        mid = left + (right - left) // 2
        k = keys[mid]
        if k == key:
            return True, mid
        if k < key:
            left = mid + 1
        else:
            right = mid
    return False, left


class Index:
    def __init__(self, items):
        self.items = list(items)
        self._keys = [b.key for b in self.items]

    @classmethod
    def new(cls, pairs, block_stride, engine=None):
        """src/sstable/index.rs:55-67 (pairs sorted; stride 0 is an error,
        the reference panics in `chunks(0)`)."""
        if block_stride <= 0:
            raise ValueError("block_stride must be positive (reference: chunks(0) panics)")
        from .format import serialize_flatten
        _, blocks = serialize_flatten(pairs, engine, block_stride=block_stride)
        return cls.from_blocks(pairs, blocks)

    @classmethod
    def from_blocks(cls, pairs, blocks):
        """hg_block records (first_rec, position, length) + the pairs."""
        return cls(Block(pairs[int(b["first_rec"])].key, int(b["position"]), int(b["length"]))
                   for b in blocks)

    @classmethod
    def from_spans(cls, data, spans, block_stride):
        """Blocks of a decoded table: block b starts at record b*stride; its
        length runs to the next block's start (or the last record's end)."""
        if block_stride <= 0:
            raise ValueError("block_stride must be positive (reference: chunks(0) panics)")
        n = spans.size
        if n == 0:
            return cls([])
        first = np.arange(0, n, block_stride)
        pos = spans["off"][first].astype(np.int64)
        last = spans[-1]
        end = int(last["off"]) + 16 + int(last["klen"]) + int(last["vlen"])
        lens = np.diff(np.append(pos, end))
        kl = spans["klen"][first].astype(np.int64)
        mv = memoryview(data).cast("B")
        # plain-int lists: no numpy scalar per field in the per-block loop
        return cls(Block(bytes(mv[p + 16:p + 16 + k]), p, ln)
                   for p, k, ln in zip(pos.tolist(), kl.tolist(), lens.tolist()))

    @classmethod
    def from_encoded(cls, data, blocks):
        """Blocks of freshly encoded table bytes (hg_block records): the first
        key of a block is read from the record at its position."""
        mv = memoryview(data).cast("B")
        items = []
        for b in blocks:
            pos, ln = int(b["position"]), int(b["length"])
            klen = int.from_bytes(mv[pos:pos + 8], "little")
            items.append(Block(bytes(mv[pos + 16:pos + 16 + klen]), pos, ln))
        return cls(items)

    def get(self, key):
        """src/sstable/index.rs:72-78: Ok(pos) of the binary search over the
        first keys -> that block; Err(pos) -> the block before it; None
        before the first block.  Returns (position, length)."""
        hit, pos = rust_binary_search(self._keys, bytes(key))
        if not hit:
            if pos == 0:
                return None
            pos -= 1
        b = self.items[pos]
        return (b.position, b.length)
