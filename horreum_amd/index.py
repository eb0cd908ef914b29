"""Python mirror of horreum's block index (reference src/sstable/index.rs).

`Index.new` takes the block positions and lengths from the SAME engine
launch that encodes the table (`hg_encode_*(..., block_stride, blocks)`),
replacing the reference's second full `serialize_flatten` per block
(src/sstable/index.rs:55-67).  `Index.from_spans` builds the same blocks
from a decode's spans (cold open, src/sstable/table.rs:46) without encoding
anything.  `get` is the reference's binary search (:72-78).
"""
import bisect
from collections import namedtuple

import numpy as np

Block = namedtuple("Block", "key position length")  # src/sstable/index.rs:6-29


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
        """src/sstable/index.rs:72-78: exact first-key match -> that block;
        otherwise the block before the insertion point; None before the
        first block.  Returns (position, length)."""
        key = bytes(key)
        i = bisect.bisect_left(self._keys, key)
        if i < len(self._keys) and self._keys[i] == key:
            pos = i
        elif i > 0:
            pos = i - 1
        else:
            return None
        b = self.items[pos]
        return (b.position, b.length)
