"""Python mirror of horreum's SSTable file layer (reference
src/sstable/storage.rs, src/sstable/table.rs) on the MI355X engine.

The byte work -- encoding on write, decoding on open / get / get_all, the
block index -- runs in libhorreum_gpu.so; this module does file I/O and the
reference's host logic (binary searches, size accounting) only.

Quirks kept from the reference:
- `PersistedFile.new` opens with create+write+read and NO truncate
  (storage.rs:24-30): writing a shorter table over a longer file leaves the
  old tail in place, and a later `read_all` then fails to decode it.
- `SSTable.size` is the payload Σ(klen + vlen), not the file size
  (table.rs:36-45); for a decoded table that is L - 16·n.
"""
import bisect
import os

from .format import decode_spans, pairs_from_spans, serialize_flatten
from .index import Index


class PersistedFile:
    """src/sstable/storage.rs:9-75."""

    def __init__(self, path):
        self.path = os.fspath(path)

    @classmethod
    def new(cls, path, pairs, engine=None):
        """storage.rs:21-38: encode `pairs` and write them at offset 0."""
        f = cls(path)
        f.write_bytes(serialize_flatten(pairs, engine))
        return f

    def write_bytes(self, data):
        fd = os.open(self.path, os.O_CREAT | os.O_RDWR, 0o644)  # no O_TRUNC (storage.rs:24-30)
        try:
            mv = memoryview(data)
            done = 0
            while done < len(mv):
                done += os.pwrite(fd, mv[done:], done)
        finally:
            os.close(fd)

    @classmethod
    def open(cls, path):
        """storage.rs:41-49 (the file must exist)."""
        if not os.path.isfile(path):
            raise FileNotFoundError(path)
        return cls(path)

    def read_bytes(self):
        with open(self.path, "rb") as fh:
            return fh.read()

    def read_at(self, position, length):
        """storage.rs:52-57: exactly `length` bytes at `position`
        (read_exact: a short read is an error)."""
        with open(self.path, "rb") as fh:
            fh.seek(position)
            data = fh.read(length)
        if len(data) != length:
            raise EOFError(f"read_at({position}, {length}): file has {len(data)} bytes there")
        return data

    def read_all(self, engine=None):
        """storage.rs:60-67 (decode errors raise DecodeError; the reference panics)."""
        data = self.read_bytes()
        return pairs_from_spans(data, decode_spans(data, engine))

    def delete(self):
        os.remove(self.path)


class SSTable:
    """src/sstable/table.rs:7-90."""

    def __init__(self, file, index, size):
        self.file = file
        self.index = index
        self.size = size

    @classmethod
    def create(cls, path, pairs, size, block_stride, engine=None):
        """manager.rs:68-74 + table.rs:22-31 in one engine launch: the file
        bytes and the block index come from the same encode."""
        if block_stride <= 0:
            raise ValueError("block_stride must be positive (reference: chunks(0) panics)")
        data, blocks = serialize_flatten(pairs, engine, block_stride=block_stride)
        f = PersistedFile(path)
        f.write_bytes(data)
        return cls(f, Index.from_blocks(pairs, blocks), size)

    @classmethod
    def new(cls, file, pairs, size, block_stride, engine=None):
        """table.rs:22-31: a table over an already written file."""
        return cls(file, Index.new(pairs, block_stride, engine), size)

    @classmethod
    def open(cls, path, block_stride, engine=None):
        """table.rs:33-49: decode the whole file once; size and index come
        from the spans (no re-encode)."""
        f = PersistedFile.open(path)
        data = f.read_bytes()
        spans = decode_spans(data, engine)
        size = len(data) - 16 * int(spans.size)
        return cls(f, Index.from_spans(data, spans, block_stride), size)

    def get(self, key, engine=None):
        """table.rs:54-70: index -> one block read -> decode -> binary search."""
        hit = self.index.get(key)
        if hit is None:
            return None
        position, length = hit
        block = self.file.read_at(position, length)
        pairs = pairs_from_spans(block, decode_spans(block, engine))
        keys = [p.key for p in pairs]
        key = bytes(key)
        i = bisect.bisect_left(keys, key)
        return pairs[i] if i < len(keys) and keys[i] == key else None

    def get_many(self, keys, engine=None):
        """SSTable::get for a batch of keys in one device launch (the table is
        read once, decoded, indexed and searched on the GPU).  Returns one
        InternalPair (tombstones included) or None per key."""
        from .engine import default_engine
        from .format import InternalPair
        eng = engine or default_engine()
        data = self.file.read_bytes()
        res = eng.lookup_host(data, keys)
        mv = memoryview(data)
        out = []
        for k, r in zip(keys, res):
            if not r["found"]:
                out.append(None)
                continue
            vo, vl = int(r["val_off"]), int(r["vlen"])
            out.append(InternalPair(k, mv[vo:vo + vl] if vl else None))
        return out

    def get_all(self, engine=None):
        """table.rs:73-75."""
        return self.file.read_all(engine)

    def get_size(self):
        return self.size

    def delete(self):
        self.file.delete()
