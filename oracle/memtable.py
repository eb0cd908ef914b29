"""Test infrastructure: restatement of horreum's MemTable bookkeeping
(reference src/memtable/mod.rs) -- the size accounting that decides when a
memtable flushes, and what a flush hands to the SSTable writer.  Pure Python
(small cases only).  `actual_size` is a usize: Rust release builds wrap, so
arithmetic here is modulo 2**64.
"""
MASK = (1 << 64) - 1


class RefMemTable:
    def __init__(self, size_limit):
        self.map = {}          # BTreeMap<Vec<u8>, Option<Vec<u8>>> (ordered at flush)
        self.size_limit = size_limit
        self.actual_size = 0
        self.flushes = []      # [(sorted [(key, value|None)], size)]

    def get(self, key):
        """mod.rs:68-72: map.get(key).cloned().flatten()."""
        return self.map.get(bytes(key))

    def put(self, key, value):
        """mod.rs:75-106."""
        key, value = bytes(key), bytes(value)
        had = key in self.map
        prev = self.map.get(key)
        self.map[key] = value
        if had and prev is not None:        # :84-87 Some(Some(v)): += new - old (wrapping)
            self.actual_size = (self.actual_size + len(value) - len(prev)) & MASK
        elif had:                           # :88-90 Some(None): += new value length
            self.actual_size = (self.actual_size + len(value)) & MASK
        else:                               # :91-94 None: += key + value
            self.actual_size = (self.actual_size + len(key) + len(value)) & MASK
        if self.actual_size > self.size_limit:   # :99-104
            self.flush()
            self.actual_size = 0
        return prev

    def delete(self, key):
        """mod.rs:108-120: insert None; subtract the old value's length."""
        key = bytes(key)
        prev = self.map.get(key)
        self.map[key] = None
        if prev is not None:
            self.actual_size = (self.actual_size - len(prev)) & MASK
        return prev

    def flush(self):
        """mod.rs:123-158: the sorted pairs and the current size; then clear."""
        pairs = sorted(self.map.items())
        self.flushes.append((pairs, self.actual_size))
        self.map.clear()
