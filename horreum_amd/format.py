"""Python mirror of horreum's record codec API (reference src/format.rs) on
the MI355X engine.

`InternalPair` keeps the reference's value semantics (src/format.rs:6-20):
owned `key` bytes, `value` bytes or `None` for a deletion, ordered by key and
then value with `None < Some` (the derived `Ord`, :5).  Encoding and decoding
run in libhorreum_gpu.so (`hg_encode_host` / `hg_decode_host`); there is no
CPU codec here.  Where the reference panics (`unwrap()` on a decode error,
src/sstable/storage.rs:64-66) this module raises `DecodeError` carrying the
engine's error kind and the failing record's offset.

Wire format (src/format.rs:23-37): `[u64 LE klen][u64 LE vlen][key][value]`;
`vlen == 0` <=> `None`, so `Some(b"")` is written as a deletion and decodes
as `None` -- exactly as in the reference.
"""
import functools

import numpy as np

from .abi import BLOCK_DTYPE, PAIR_DTYPE, SPAN_DTYPE, Status
from .engine import default_engine


class DecodeError(Exception):
    """bincode::Error equivalent: kind (abi.Status) and record offset."""

    def __init__(self, kind, offset, n_ok):
        try:
            name = Status(kind).name
        except ValueError:
            name = str(kind)
        super().__init__(f"decode failed: {name} at byte {offset} "
                         f"after {n_ok} records")
        self.kind = kind
        self.offset = offset
        self.n_ok = n_ok


@functools.total_ordering
class InternalPair:
    """src/format.rs:6-11."""

    __slots__ = ("key", "value")

    def __init__(self, key, value=None):
        self.key = bytes(key)
        self.value = None if value is None else bytes(value)

    @classmethod
    def default(cls):
        """src/format.rs:80-84: empty key, no value (16 zero bytes on the wire)."""
        return cls(b"", None)

    def _order(self):
        return (self.key, self.value is not None, self.value or b"")

    def __eq__(self, other):
        return isinstance(other, InternalPair) and self._order() == other._order()

    def __lt__(self, other):
        return self._order() < other._order()

    def __hash__(self):
        return hash(self._order())

    def __repr__(self):
        return f"InternalPair({self.key!r}, {self.value!r})"

    # ---- codec (src/format.rs:23-77) ------------------------------------------------
    def serialize(self, engine=None):
        """src/format.rs:23-37."""
        return serialize_flatten([self], engine)

    @staticmethod
    def serialize_flatten(pairs, engine=None):
        return serialize_flatten(pairs, engine)

    @staticmethod
    def deserialize_from_bytes(data, engine=None):
        return deserialize_from_bytes(data, engine)


def pack_pairs(pairs):
    """Pairs -> (arena uint8, PAIR_DTYPE descriptors): the contiguous
    key||value arena the engine encodes from (the memtable buffer of
    SURVEY.md §8 f3).  Host packing only; no record bytes are produced here.
    Offsets come from one cumulative sum over the lengths (no per-record
    descriptor writes)."""
    n = len(pairs)
    desc = np.zeros(n, dtype=PAIR_DTYPE)
    if n == 0:
        return np.zeros(1, np.uint8), desc
    keys = [bytes(p.key) for p in pairs]
    vals = [bytes(p.value) if p.value is not None else b"" for p in pairs]
    kl = np.fromiter(map(len, keys), dtype=np.uint64, count=n)
    vl = np.fromiter(map(len, vals), dtype=np.uint64, count=n)
    starts = np.zeros(n, dtype=np.uint64)
    np.cumsum((kl + vl)[:-1], out=starts[1:])
    desc["key_off"] = starts
    desc["val_off"] = starts + kl
    desc["klen"] = kl
    desc["vlen"] = vl
    blob = b"".join([b for kv in zip(keys, vals) for b in kv])
    arena = np.frombuffer(blob, dtype=np.uint8) if blob else np.zeros(1, np.uint8)
    return arena, desc


def serialize_flatten(pairs, engine=None, block_stride=0):
    """src/format.rs:40-42: records concatenated in the given order (no
    sortedness assumed).  With block_stride > 0 also returns the index blocks
    of src/sstable/index.rs:55-67 from the same launch: (bytes, blocks)."""
    if len(pairs) == 0:
        return (b"", np.zeros(0, dtype=BLOCK_DTYPE)) if block_stride else b""
    eng = engine or default_engine()
    arena, desc = pack_pairs(pairs)
    out = eng.encode_host(arena, desc, block_stride=block_stride)
    data = out.data.tobytes()
    return (data, out.blocks) if block_stride else data


def decode_spans(data, engine=None):
    """Bytes -> SPAN_DTYPE array (zero-copy record view), raising DecodeError
    where the reference's deserialize_from_bytes returns Err."""
    buf = np.frombuffer(memoryview(data).cast("B"), dtype=np.uint8)
    if buf.size == 0:
        return np.zeros(0, dtype=SPAN_DTYPE)
    eng = engine or default_engine()
    out = eng.decode_host(buf)
    if out.kind != Status.OK:
        raise DecodeError(out.kind, out.offset, out.n)
    return out.spans


def pairs_from_spans(data, spans):
    """Materialise owned InternalPairs from spans (src/format.rs:70-75):
    value is Some iff vlen > 0."""
    mv = memoryview(data).cast("B")
    out = []
    for off, kl, vl in zip(spans["off"].tolist(), spans["klen"].tolist(), spans["vlen"].tolist()):
        k0 = off + 16
        out.append(InternalPair(mv[k0:k0 + kl], mv[k0 + kl:k0 + kl + vl] if vl else None))
    return out


def deserialize_from_bytes(data, engine=None):
    """src/format.rs:50-59: every record of `data`, in order."""
    return pairs_from_spans(data, decode_spans(data, engine))
