"""TEST INFRASTRUCTURE ONLY — ctypes binding of the CPU oracle (liboracle.so).

Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the
checker / CPU baseline.  The product (horreum_amd/, libhorreum_gpu.so) never
imports this module.  See horreum_oracle.c for the reference lines each
function restates.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.environ.get("HGO_LIBRARY") or os.path.join(HERE, "liboracle.so")

SPAN_DTYPE = np.dtype([("off", "<u8"), ("klen", "<u4"), ("vlen", "<u4")])
PAIR_DTYPE = np.dtype([("key_off", "<u8"), ("val_off", "<u8"), ("klen", "<u4"), ("vlen", "<u4")])
BLOCK_DTYPE = np.dtype([("first_rec", "<u8"), ("position", "<u8"), ("length", "<u8")])


class _Err(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("reserved", ctypes.c_uint32), ("offset", ctypes.c_uint64)]


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        vp, u64, u32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32
        L.hgo_decode.argtypes = [vp, u64, vp, u64, ctypes.POINTER(u64), ctypes.POINTER(_Err)]
        L.hgo_encode.argtypes = [vp, vp, u64, vp, u64, vp, u32, vp, ctypes.POINTER(u64)]
        L.hgo_index_get.argtypes = [vp, u64, vp, vp, vp, u64, ctypes.POINTER(u64),
                                    ctypes.POINTER(u64)]
        L.hgo_compact.argtypes = [u32, vp, vp, vp, vp, vp, u64, ctypes.POINTER(u64)]
        L.hgo_payload_size.argtypes = [vp, u64]
        L.hgo_payload_size.restype = u64
        L.hgo_table_get.argtypes = [vp, vp, u64, ctypes.c_uint32, vp, u64,
                                    ctypes.POINTER(u64)]
        L.hgo_table_get.restype = ctypes.c_int
        L.hgo_bench_decode_owned.argtypes = [vp, u64, ctypes.POINTER(ctypes.c_double)]
        L.hgo_bench_decode_owned.restype = u64
        L.hgo_bench_encode_owned.argtypes = [vp, vp, u64, ctypes.POINTER(ctypes.c_double)]
        L.hgo_bench_encode_owned.restype = u64
        L.hgo_mt_decode.argtypes = [vp, u64, vp, u64, vp, u32, ctypes.POINTER(ctypes.c_double)]
        L.hgo_mt_decode.restype = u64
        L.hgo_mt_encode.argtypes = [vp, vp, u64, vp, u32, ctypes.POINTER(ctypes.c_double)]
        L.hgo_mt_encode.restype = u64
        L.hgo_mt_memcpy.argtypes = [vp, vp, u64, u32, ctypes.POINTER(ctypes.c_double)]
        L.hgo_mt_memcpy.restype = None
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else ctypes.c_void_p(0)


def _u8(data):
    return np.ascontiguousarray(np.frombuffer(memoryview(data).cast("B"), dtype=np.uint8))


def pack_pairs(pairs):
    """[(key bytes, value bytes | None)] -> (arena uint8, PAIR_DTYPE records)."""
    keys = [bytes(k) for k, _ in pairs]
    vals = [b"" if v is None else bytes(v) for _, v in pairs]
    arena = np.frombuffer(b"".join(k + v for k, v in zip(keys, vals)), dtype=np.uint8).copy()
    rec = np.zeros(len(pairs), dtype=PAIR_DTYPE)
    off = 0
    for i, (k, v) in enumerate(zip(keys, vals)):
        rec[i] = (off, off + len(k), len(k), len(v))
        off += len(k) + len(v)
    return arena, rec


def encode(arena, pairs, block_stride=0):
    """-> (bytes uint8, rec_off uint64, blocks | None, status)."""
    arena = np.ascontiguousarray(arena, dtype=np.uint8)
    pairs = np.ascontiguousarray(pairs, dtype=PAIR_DTYPE)
    n = pairs.size
    total = int((16 + pairs["klen"].astype(np.uint64) + pairs["vlen"].astype(np.uint64)).sum())
    out = np.zeros(max(total, 1), dtype=np.uint8)
    rec = np.zeros(max(n, 1), dtype=np.uint64)
    nb = (n + block_stride - 1) // block_stride if block_stride else 0
    blocks = np.zeros(max(nb, 1), dtype=BLOCK_DTYPE) if block_stride else None
    out_len = ctypes.c_uint64()
    rc = lib().hgo_encode(_p(arena), _p(pairs), n, _p(out), total, _p(rec), block_stride,
                          _p(blocks), ctypes.byref(out_len))
    assert out_len.value == total
    return out[:total], rec[:n], (blocks[:nb] if blocks is not None else None), rc


def decode(data, cap=None):
    """-> (spans SPAN_DTYPE[:min(n,cap)], n, kind, offset, status)."""
    buf = _u8(data)
    cap = buf.size // 16 if cap is None else int(cap)
    spans = np.zeros(max(cap, 1), dtype=SPAN_DTYPE)
    n = ctypes.c_uint64()
    err = _Err()
    rc = lib().hgo_decode(_p(buf), buf.size, _p(spans), cap, ctypes.byref(n), ctypes.byref(err))
    return spans[: min(n.value, cap)], n.value, err.kind, err.offset, rc


def pairs_from_spans(data, spans):
    """Materialise InternalPair-like tuples (key, value | None) from spans."""
    buf = _u8(data)
    out = []
    for s in spans:
        o, k, v = int(s["off"]), int(s["klen"]), int(s["vlen"])
        key = buf[o + 16:o + 16 + k].tobytes()
        val = buf[o + 16 + k:o + 16 + k + v].tobytes() if v else None
        out.append((key, val))
    return out


def index_get(blocks, arena, pairs, key):
    pos = ctypes.c_uint64()
    ln = ctypes.c_uint64()
    kb = np.frombuffer(bytes(key) or b"\0", dtype=np.uint8)
    hit = lib().hgo_index_get(_p(blocks), blocks.size, _p(arena), _p(pairs), _p(kb), len(key),
                              ctypes.byref(pos), ctypes.byref(ln))
    return (pos.value, ln.value) if hit else None


def compact(tables_newest_first):
    """tables: [(data uint8, spans)] newest first -> [(table, rec)], status."""
    ot, orr, rc = compact_arrays(tables_newest_first)
    return list(zip(ot.tolist(), orr.tolist())), rc


def compact_arrays(tables_newest_first):
    """compact() as arrays: (table index uint32[n], record index uint64[n], status)."""
    T = len(tables_newest_first)
    datas = [_u8(d) for d, _ in tables_newest_first]
    spans = [np.ascontiguousarray(s, dtype=SPAN_DTYPE) for _, s in tables_newest_first]
    counts = np.array([s.size for s in spans], dtype=np.uint64)
    dptr = (ctypes.c_void_p * max(T, 1))(*[d.ctypes.data for d in datas])
    sptr = (ctypes.c_void_p * max(T, 1))(*[s.ctypes.data for s in spans])
    cap = int(counts.sum())
    ot = np.zeros(max(cap, 1), dtype=np.uint32)
    orr = np.zeros(max(cap, 1), dtype=np.uint64)
    n = ctypes.c_uint64()
    rc = lib().hgo_compact(T, ctypes.cast(dptr, ctypes.c_void_p), ctypes.cast(sptr, ctypes.c_void_p),
                           _p(counts), _p(ot), _p(orr), cap, ctypes.byref(n))
    return ot[: n.value], orr[: n.value], rc


def compacted_table(tables_newest_first, block_stride=0):
    """serialize_flatten(compact_inner(decode(t) for t in tables)) -- the bytes
    SSTableManager::compact writes (src/sstable/manager.rs:137-159, 199-234;
    src/format.rs:40-42) -> (bytes uint8, blocks | None, records)."""
    datas = [_u8(d) for d in tables_newest_first]
    decs = []
    for d in datas:
        spans, n, kind, _, _ = decode(d)
        assert kind == 0, "input table does not decode"
        decs.append((d, spans[:n]))
    ot, orr, rc = compact_arrays(decs)
    assert rc == 0
    base = np.zeros(len(datas) + 1, dtype=np.uint64)
    np.cumsum([d.size for d in datas], out=base[1:])
    arena = np.concatenate(datas) if datas else np.zeros(1, np.uint8)
    pairs = np.zeros(ot.size, dtype=PAIR_DTYPE)
    for t, (_, spans) in enumerate(decs):
        sel = ot == t
        s = spans[orr[sel]]
        ko = base[t] + s["off"] + np.uint64(16)
        pairs["key_off"][sel] = ko
        pairs["val_off"][sel] = ko + s["klen"].astype(np.uint64)
        pairs["klen"][sel] = s["klen"]
        pairs["vlen"][sel] = s["vlen"]
    data, _, blocks, rc = encode(arena, pairs, block_stride=block_stride)
    assert rc == 0
    return data, blocks, int(ot.size)


def table_get(data, spans, stride, key):
    """SSTable::get (src/sstable/table.rs:54-70) on a decoded table: the
    record index holding `key`, or None."""
    buf = _u8(data)
    spans = np.ascontiguousarray(spans, dtype=SPAN_DTYPE)
    kb = np.frombuffer(bytes(key) or b"\0", dtype=np.uint8)
    rec = ctypes.c_uint64()
    hit = lib().hgo_table_get(_p(buf), _p(spans), spans.size, stride, _p(kb), len(key),
                              ctypes.byref(rec))
    return rec.value if hit else None


def payload_size(spans):
    spans = np.ascontiguousarray(spans, dtype=SPAN_DTYPE)
    return int(lib().hgo_payload_size(_p(spans), spans.size))


def bench_decode_owned(data):
    buf = _u8(data)
    t = ctypes.c_double()
    n = lib().hgo_bench_decode_owned(_p(buf), buf.size, ctypes.byref(t))
    return n, t.value


def bench_encode_owned(arena, pairs):
    t = ctypes.c_double()
    n = lib().hgo_bench_encode_owned(_p(arena), _p(pairs), pairs.size, ctypes.byref(t))
    return n, t.value


def mt_decode(data, nthreads, spans=None, scratch=None):
    """Optimised multi-threaded CPU decode (cpu_opt.c) -> (spans, n, seconds)."""
    buf = _u8(data)
    if spans is None:
        spans = np.zeros(max(buf.size // 16, 1), dtype=SPAN_DTYPE)
    if scratch is None:
        scratch = np.empty(buf.size // 16 + 2 * nthreads + 2, dtype=SPAN_DTYPE)
    t = ctypes.c_double()
    n = lib().hgo_mt_decode(_p(buf), buf.size, _p(spans), spans.size, _p(scratch), nthreads,
                            ctypes.byref(t))
    return spans, n, t.value


def mt_memcpy(dst, src, nthreads):
    """Multi-threaded host memcpy (the CPU roofline row) -> seconds."""
    t = ctypes.c_double()
    lib().hgo_mt_memcpy(_p(dst), _p(src), min(dst.size, src.size), nthreads, ctypes.byref(t))
    return t.value


def mt_encode(arena, pairs, nthreads, out=None):
    """Optimised multi-threaded CPU encode (cpu_opt.c) -> (bytes, seconds)."""
    total = int((16 + pairs["klen"].astype(np.uint64) + pairs["vlen"].astype(np.uint64)).sum())
    if out is None:
        out = np.empty(max(total, 1), dtype=np.uint8)
    t = ctypes.c_double()
    n = lib().hgo_mt_encode(_p(arena), _p(pairs), pairs.size, _p(out), nthreads, ctypes.byref(t))
    return out[:n], t.value
