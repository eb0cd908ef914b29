"""Python mirror of horreum's SSTable file layer (reference
src/sstable/storage.rs, src/sstable/table.rs) on the MI355X engine.

The byte work -- encoding on write, decoding on open / get / get_all, the
block index -- runs in libhorreum_gpu.so; this module does file I/O and the
reference's host logic (binary searches, size accounting) only.

Host memory: a table file is mmap'd once (no read() copy);
its transfers go through the engine's pinned staging, the page faults and
copies split over host threads.  Page-locking the mapping with
hg_host_register (`PersistedFile.pin`, or `mapped(register=True)`) makes
every later transfer a direct DMA, but pinning runs at ~4-6 GB/s on the
MI355X box against ~45 GiB/s for the staged transfer (cold open of 32 x 64
MiB files: 370-600 ms to register vs ~50 ms to decode through staging), so
it pays only for a mapping moved many times and is off by default.  A
directory opens with one batched decode of all its tables (SSTableManager).
Batched lookups keep the table, its spans and its key index resident in HBM
after the first batch.

Quirks kept from the reference:
- `PersistedFile.new` opens with create+write+read and NO truncate
  (storage.rs:24-30): writing a shorter table over a longer file leaves the
  old tail in place, and a later `read_all` then fails to decode it.
- `SSTable.size` is the payload Σ(klen + vlen), not the file size
  (table.rs:36-45); for a decoded table that is L - 16·n.
"""
import mmap
import os
import weakref
from collections import OrderedDict

import numpy as np

from .format import DecodeError, decode_spans, pairs_from_spans, serialize_flatten
from .index import Index, rust_binary_search


class PersistedFile:
    """src/sstable/storage.rs:9-75."""

    def __init__(self, path):
        self.path = os.fspath(path)
        self._map = None      # (mmap, numpy view, registered engine or None)

    @classmethod
    def new(cls, path, pairs, engine=None):
        """storage.rs:21-38: encode `pairs` and write them at offset 0."""
        f = cls(path)
        f.write_bytes(serialize_flatten(pairs, engine))
        return f

    def write_bytes(self, data):
        self.unmap()
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

    def mapped(self, engine=None, register=False):
        """The whole file as a uint8 array over a private mmap of it; with
        `register`, page-locked with hg_host_register when the engine can (so
        transfers are direct DMA).  The mapping lives until delete() /
        unmap()."""
        if self._map is not None:
            if register and self._map[2] is None and self._map[0] is not None:
                self._register(engine)
            return self._map[1]
        size = os.path.getsize(self.path)
        if size == 0:
            self._map = (None, np.zeros(0, dtype=np.uint8), None)
            return self._map[1]
        with open(self.path, "rb") as fh:
            mm = mmap.mmap(fh.fileno(), size, access=mmap.ACCESS_COPY)
        arr = np.frombuffer(mm, dtype=np.uint8)
        self._map = (mm, arr, None)
        if register:
            self._register(engine)
        return arr

    def _register(self, engine=None):
        mm, arr, _ = self._map
        try:
            from .engine import default_engine
            eng = engine or default_engine()
            eng.host_register(arr)
            self._map = (mm, arr, eng)
        except Exception:  # noqa: BLE001 -- pageable (staged copies) stays
            pass

    def pin(self, engine=None):
        """Map and page-lock the file for repeated direct-DMA transfers."""
        return self.mapped(engine, register=True)

    def unmap(self):
        if self._map is None:
            return
        mm, arr, reg = self._map
        self._map = None
        if reg is not None:
            try:
                reg.host_unregister(arr)
            except Exception:  # noqa: BLE001
                pass
        del arr
        if mm is not None:
            try:
                mm.close()
            except BufferError:  # views still exported: the mapping goes with them
                pass

    def __del__(self):
        # a registration must end before its pages are unmapped: a stale one
        # would make a later mapping at the same address look page-locked
        try:
            self.unmap()
        except Exception:  # noqa: BLE001 -- interpreter shutdown
            pass

    def read_bytes(self, engine=None):
        return self.mapped(engine)

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
        data = self.read_bytes(engine)
        return pairs_from_spans(data, decode_spans(data, engine))

    def delete(self):
        self.unmap()
        os.remove(self.path)


class _ResidentLRU:
    """Tables kept resident in HBM for batched lookups, per engine, least
    recently used first: once their bytes (table + spans + key index) pass
    the budget (HG_RESIDENT_BYTES, default 32 GiB) the oldest are released
    (their next get_many uploads them again)."""

    def __init__(self, budget):
        self.budget = budget
        self.items = OrderedDict()  # id(table) -> (weakref(table), bytes)
        self.total = 0

    def _forget(self, key, ref):
        """Weakref callback: a table collected without release() leaves."""
        item = self.items.get(key)
        if item is not None and item[0] is ref:
            del self.items[key]
            self.total -= item[1]

    def touch(self, table, nbytes):
        key = id(table)
        item = self.items.get(key)
        if item is not None and item[0]() is table:
            self.items.move_to_end(key)
            return
        if item is not None:  # a dead table's id reused: its entry is stale
            del self.items[key]
            self.total -= item[1]
        self.items[key] = (weakref.ref(table, lambda r, k=key: self._forget(k, r)), nbytes)
        self.total += nbytes
        while self.total > self.budget and len(self.items) > 1:
            _, (ref, b) = self.items.popitem(last=False)
            self.total -= b
            old = ref()
            # only the state this engine holds: a table that moved to another
            # engine keeps that engine's resident copy
            if old is not None and old._resident is not None and _LRUS.get(old._resident[0]) is self:
                old._resident = None

    def drop(self, table):
        item = self.items.get(id(table))
        if item is not None and item[0]() is table:
            del self.items[id(table)]
            self.total -= item[1]


_LRUS = weakref.WeakKeyDictionary()  # engine -> _ResidentLRU


def _lru(engine):
    lru = _LRUS.get(engine)
    if lru is None:
        lru = _LRUS[engine] = _ResidentLRU(int(os.environ.get("HG_RESIDENT_BYTES", 32 << 30)))
    return lru


class SSTable:
    """src/sstable/table.rs:7-90."""

    def __init__(self, file, index, size, block_stride=0):
        self.file = file
        self.index = index
        self.size = size
        self.block_stride = block_stride  # records per index block (batched lookups)
        self._resident = None  # (engine, ResidentTable): lookups stay in HBM

    @classmethod
    def create(cls, path, pairs, size, block_stride, engine=None):
        """manager.rs:68-74 + table.rs:22-31 in one engine launch: the file
        bytes and the block index come from the same encode."""
        if block_stride <= 0:
            raise ValueError("block_stride must be positive (reference: chunks(0) panics)")
        data, blocks = serialize_flatten(pairs, engine, block_stride=block_stride)
        f = PersistedFile(path)
        f.write_bytes(data)
        return cls(f, Index.from_blocks(pairs, blocks), size, block_stride)

    @classmethod
    def new(cls, file, pairs, size, block_stride, engine=None):
        """table.rs:22-31: a table over an already written file."""
        return cls(file, Index.new(pairs, block_stride, engine), size, block_stride)

    @classmethod
    def open(cls, path, block_stride, engine=None):
        """table.rs:33-49: decode the whole file once; size and index come
        from the spans (no re-encode)."""
        f = PersistedFile.open(path)
        data = f.read_bytes(engine)
        return cls.from_decoded(f, data, decode_spans(data, engine), block_stride)

    @classmethod
    def from_decoded(cls, f, data, spans, block_stride):
        """An opened table from its bytes and spans (table.rs:36-49)."""
        if block_stride <= 0:
            raise ValueError("block_stride must be positive (reference: chunks(0) panics)")
        size = len(data) - 16 * int(spans.size)
        return cls(f, Index.from_spans(data, spans, block_stride), size, block_stride)

    def get(self, key, engine=None):
        """table.rs:54-70: index -> one block read -> decode -> binary search."""
        hit = self.index.get(key)
        if hit is None:
            return None
        position, length = hit
        block = self.file.read_at(position, length)
        pairs = pairs_from_spans(block, decode_spans(block, engine))
        hit, i = rust_binary_search([p.key for p in pairs], bytes(key))
        return pairs[i] if hit else None

    def resident(self, engine=None):
        """The table in HBM for batched lookups: uploaded, decoded and
        indexed by the first call, reused by later ones while it stays within
        the engine's resident budget (least recently used tables go first)."""
        from .engine import default_engine
        eng = engine or default_engine()
        if self._resident is None or self._resident[0] is not eng:
            if self._resident is not None:  # an engine switch: leave the old engine's LRU
                _lru(self._resident[0]).drop(self)
                self._resident = None
            data = self.file.read_bytes(eng)
            rt = eng.resident_table(data)
            if rt.kind != 0:
                raise DecodeError(rt.kind, rt.offset, rt.n)
            self._resident = (eng, rt)
            _lru(eng).touch(self, len(data) + 48 * int(rt.n))  # bytes + spans + key index
        else:
            _lru(eng).touch(self, 0)
        return self._resident[1]

    def release(self):
        """Free the table's resident HBM state (it is rebuilt on demand)."""
        if self._resident is not None:
            _lru(self._resident[0]).drop(self)
        self._resident = None

    def get_many(self, keys, engine=None):
        """SSTable::get for a batch of keys in one device launch against the
        resident table (only the keys go up): the same block search and
        in-block search as `get`, so `get_many(ks)[i] == get(ks[i])` on any
        table, duplicate or unordered keys included.  Returns one
        InternalPair (tombstones included) or None per key."""
        from .engine import default_engine
        from .format import InternalPair
        eng = engine or default_engine()
        rt = self.resident(eng)
        res = eng.lookup_resident(rt, keys, self.block_stride)
        data = self.file.read_bytes(eng)
        mv = memoryview(data).cast("B")
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
        self.release()
        self.file.delete()
