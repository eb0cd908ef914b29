"""Python mirror of horreum's SSTableManager byte paths (reference
src/sstable/manager.rs) on the MI355X engine: opening a table directory,
creating tables, newest-first lookups, and compaction.

Compaction's byte work -- decode every table, k-way merge (newest wins,
tombstones kept), encode the merged table and its index -- is one engine call
(`hg_compact_host`, manager.rs:137-159 + :199-234).  The control plane stays
out (the mpsc command loop, manager.rs:85-123): callers invoke `create`,
`get`, `compact` and `flush` directly.

Reference quirks kept on purpose:
- tables are opened in lexicographic path order (manager.rs:47-55), so
  `table_10` sorts before `table_2`;
- a new table is named `table_{len(tables)}` (manager.rs:77-81);
- a compacted table's size is the sum of its inputs' sizes
  (manager.rs:138-158 passes should_compact's total), not its payload;
- the trigger is (sum of newer sizes) / (oldest size) > ratio_percent / 100
  (manager.rs:170-194).
"""
import os

from .engine import default_engine
from .format import DecodeError
from .index import Index
from .table import PersistedFile, SSTable


class CompactionError(Exception):
    def __init__(self, out):
        super().__init__(f"compaction failed: status {out.status} (kind {out.kind}, "
                         f"table {out.table}, index {out.index})")
        self.out = out


class SSTableManager:
    def __init__(self, directory, block_stride, compaction_trigger_ratio, engine=None):
        """manager.rs:38-65 (compaction_trigger_ratio in percent)."""
        self.table_directory = os.fspath(directory)
        self.block_stride = block_stride
        self.engine = engine
        paths = sorted(os.path.join(self.table_directory, f)
                       for f in os.listdir(self.table_directory))
        self.tables = self._open_all(paths)
        self.compaction_trigger_ratio = compaction_trigger_ratio / 100.0

    def _open_all(self, paths):
        """manager.rs:47-55 as batched decodes of the tables (the files
        mmap'd pageable -- staged through pinned buffers, see table.py --
        and decoded by one launch chain per group of tables under the
        engine's byte budget); a table that does not decode raises
        DecodeError like SSTable.open."""
        if not paths:
            return []
        eng = self.engine or default_engine()
        files = [PersistedFile.open(p) for p in paths]
        datas = [f.read_bytes(eng) for f in files]
        outs = eng.decode_many_host(datas)
        eng.trim()  # the batched decode sized the context's buffers for the whole directory
        tables = []
        for f, d, o in zip(files, datas, outs):
            if o.kind != 0:
                raise DecodeError(o.kind, o.offset, o.n)
            tables.append(SSTable.from_decoded(f, d, o.spans, self.block_stride))
        return tables

    def _new_table_path(self):
        return os.path.join(self.table_directory, f"table_{len(self.tables)}")

    def create(self, pairs, size):
        """manager.rs:68-74: one encode writes the file and yields the index."""
        self.tables.append(SSTable.create(self._new_table_path(), pairs, size, self.block_stride,
                                          self.engine))

    def get(self, key):
        """manager.rs:126-134: newest table first."""
        for table in reversed(self.tables):
            pair = table.get(key, self.engine)
            if pair is not None:
                return pair
        return None

    def get_many(self, keys):
        """get() for a batch of keys: one device lookup launch per table,
        newest table first; a key stops at the first table that holds it
        (tombstones included, as manager.rs:126-134)."""
        keys = [bytes(k) for k in keys]
        out = [None] * len(keys)
        todo = list(range(len(keys)))
        for table in reversed(self.tables):
            if not todo:
                break
            got = table.get_many([keys[i] for i in todo], self.engine)
            left = []
            for i, g in zip(todo, got):
                if g is None:
                    left.append(i)
                else:
                    out[i] = g
            todo = left
        return out

    def should_compact(self):
        """manager.rs:170-194: the compacted size, or None."""
        if not self.tables:
            return None
        oldest = self.tables[0].get_size()
        total = sum(t.get_size() for t in self.tables)
        newer = total - oldest
        ratio = newer / oldest if oldest else (float("inf") if newer else float("nan"))
        return total if ratio > self.compaction_trigger_ratio else None

    def compact(self):
        """manager.rs:137-159 with the byte work on the GPU.  The table list
        and the files stay untouched until the compacted bytes exist: a read
        error, a device error (HIP, out of memory) or a format error leaves
        every table readable (the reference moves the list out first, :146,
        but its CPU codec has no device failures to survive)."""
        size = self.should_compact()
        if size is None:
            return False
        eng = self.engine or default_engine()
        datas = [t.file.read_bytes(eng) for t in reversed(self.tables)]  # newest first (:148)
        out = eng.compact_host(datas, block_stride=self.block_stride)
        if out.status != 0:
            raise CompactionError(out)
        data = out.data.tobytes()
        tables, self.tables = self.tables, []  # :146
        for t in tables:
            t.delete()
        f = PersistedFile(self._new_table_path())  # table_0 (:77-81 on the emptied list)
        f.write_bytes(data)
        self.tables.append(SSTable(f, Index.from_encoded(data, out.blocks), size, self.block_stride))
        return True

    def flush_arena(self, arena, desc, size):
        """The Flush command fed by MemTable.flush: one encode writes the new
        table and its index straight from the memtable arena, then maybe
        compact (manager.rs:104-114)."""
        eng = self.engine or default_engine()
        out = eng.encode_host(arena, desc, block_stride=self.block_stride)
        data = out.data.tobytes()
        f = PersistedFile(self._new_table_path())
        f.write_bytes(data)
        self.tables.append(SSTable(f, Index.from_encoded(data, out.blocks), size, self.block_stride))
        self.compact()

    def flush(self, pairs, size):
        """The Flush command (manager.rs:104-114): create, then maybe compact."""
        self.create(pairs, size)
        self.compact()
