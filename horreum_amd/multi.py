"""Several contexts driven by one host thread each (hg_multi_* in
libhorreum_gpu.so): a table directory decoded table-per-context,
one huge table decoded range-per-context with the entry handed over by the
host, and compaction split by key range.  No collectives: the only thing that
crosses between contexts is one u64 entry per split (and the splitter keys).

The contexts may sit on different devices (one per GPU of a node) or several
on one device (the tests drive two contexts on device 0 from two threads).
"""
import ctypes

import numpy as np

from .abi import (BLOCK_DTYPE, SPAN_DTYPE, HgErr, HgMergeResult, HorreumGpuError, Status, check,
                  load_library)
from .engine import CompactOut, DecodeOut, Engine


def _u8(data):
    return np.ascontiguousarray(np.frombuffer(memoryview(data).cast("B"), dtype=np.uint8))


class MultiEngine:
    """Contexts on `devices` (a list of device ids; repeats allowed), each
    with its own stream."""

    def __init__(self, devices):
        self.lib = load_library()
        self.engines = [Engine(int(d), use_torch_stream=False) for d in devices]
        n = len(self.engines)
        self._ctxs = (ctypes.c_void_p * n)(*[e.ctx.value for e in self.engines])

    @property
    def n(self):
        return len(self.engines)

    def close(self):
        for e in self.engines:
            e.close()
        self.engines = []

    def _args(self):
        return ctypes.cast(self._ctxs, ctypes.c_void_p), len(self.engines)

    def decode_tables(self, tables):
        """hg_multi_decode_host: every table (bytes-like) -> DecodeOut with a
        numpy SPAN_DTYPE array; table i runs on context i % n."""
        bufs = [_u8(t) for t in tables]
        k = len(bufs)
        spans = [np.zeros(max(b.size // 16, 1), dtype=SPAN_DTYPE) for b in bufs]
        tp = (ctypes.c_void_p * max(k, 1))(*[b.ctypes.data if b.size else 0 for b in bufs])
        ln = (ctypes.c_uint64 * max(k, 1))(*[b.size for b in bufs])
        sp = (ctypes.c_void_p * max(k, 1))(*[s.ctypes.data for s in spans])
        cp = (ctypes.c_uint64 * max(k, 1))(*[b.size // 16 for b in bufs])
        n_out = (ctypes.c_uint64 * max(k, 1))()
        errs = (HgErr * max(k, 1))()
        ctxs, nctx = self._args()
        check(self.lib.hg_multi_decode_host(ctxs, nctx, k, ctypes.cast(tp, ctypes.c_void_p),
                                            ctypes.cast(ln, ctypes.c_void_p),
                                            ctypes.cast(sp, ctypes.c_void_p),
                                            ctypes.cast(cp, ctypes.c_void_p),
                                            ctypes.cast(n_out, ctypes.c_void_p),
                                            ctypes.cast(errs, ctypes.c_void_p)),
              "hg_multi_decode_host")
        return [DecodeOut(spans[i][:min(n_out[i], bufs[i].size // 16)], n_out[i], errs[i].kind,
                          errs[i].offset) for i in range(k)]

    def decode_file(self, data, cap=None):
        """hg_multi_decode_file_host: one table cut into one byte range per
        context -> DecodeOut (numpy spans)."""
        buf = _u8(data)
        cap = buf.size // 16 if cap is None else int(cap)
        spans = np.zeros(max(cap, 1), dtype=SPAN_DTYPE)
        n, err = ctypes.c_uint64(), HgErr()
        ctxs, nctx = self._args()
        rc = self.lib.hg_multi_decode_file_host(ctxs, nctx, buf.ctypes.data_as(ctypes.c_void_p),
                                                buf.size, spans.ctypes.data_as(ctypes.c_void_p),
                                                cap, ctypes.byref(n), ctypes.byref(err))
        if rc < 0:
            raise HorreumGpuError(rc, "hg_multi_decode_file_host")
        return DecodeOut(spans[:min(n.value, cap)], n.value, err.kind, err.offset)

    def compact_dev(self, tables, owner, outs):
        """hg_multi_compact_dev: `tables` are device uint8 tensors (newest
        first), table t on context owner[t]'s device; slice g of the
        compacted table goes to outs[g] (a device uint8 tensor on context g's
        device).  -> (status, [slice bytes], [slice records], HgMergeResult)."""
        k, n = len(tables), self.n
        tp = (ctypes.c_void_p * max(k, 1))(*[t.data_ptr() if t.numel() else 0 for t in tables])
        ln = (ctypes.c_uint64 * max(k, 1))(*[t.numel() for t in tables])
        ow = (ctypes.c_uint32 * max(k, 1))(*[int(o) for o in owner])
        op = (ctypes.c_void_p * n)(*[o.data_ptr() for o in outs])
        cp = (ctypes.c_uint64 * n)(*[o.numel() for o in outs])
        ol = (ctypes.c_uint64 * n)()
        orc = (ctypes.c_uint64 * n)()
        res = HgMergeResult()
        ctxs, nctx = self._args()
        rc = self.lib.hg_multi_compact_dev(ctxs, nctx, k, ctypes.cast(ow, ctypes.c_void_p),
                                           ctypes.cast(tp, ctypes.c_void_p),
                                           ctypes.cast(ln, ctypes.c_void_p),
                                           ctypes.cast(op, ctypes.c_void_p),
                                           ctypes.cast(cp, ctypes.c_void_p),
                                           ctypes.cast(ol, ctypes.c_void_p),
                                           ctypes.cast(orc, ctypes.c_void_p), ctypes.byref(res))
        if rc in (Status.HIP, Status.INVALID_ARG, Status.INTERNAL, Status.TOO_LARGE):
            raise HorreumGpuError(rc, "hg_multi_compact_dev")
        return rc, list(ol), list(orc), res

    PHASES = ("decode_ms", "sample_cut_ms", "copies_ms", "merge_ms", "encode_ms")

    def last_phases(self):
        """Per context, the phase times of the last compact_dev that split by
        key range (diagnostics export hgk_multi_last_phases): its decode of
        the tables it owns, the sample / splitter / cut steps, and for its key
        range the slice copies, the merge and the encode (ms; -1 unknown)."""
        fn = getattr(self.lib, "hgk_multi_last_phases", None)
        if fn is None:
            return []
        fn.restype = ctypes.c_uint32
        fn.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
        out = (ctypes.c_double * (5 * self.n))()
        m = fn(ctypes.cast(out, ctypes.c_void_p), self.n)
        return [dict(zip(self.PHASES, [round(out[5 * g + k], 4) for k in range(5)])) for g in range(m)]

    def compact(self, tables, block_stride=0, out=None):
        """hg_multi_compact_host: SSTableManager::compact's byte work split by
        key range over the contexts (`tables` newest first) -> CompactOut."""
        bufs = [_u8(t) for t in tables]
        k = len(bufs)
        cap = max(sum(b.size for b in bufs), 1)
        if out is None:
            out = np.empty(cap, dtype=np.uint8)
        ptrs = (ctypes.c_void_p * max(k, 1))(*[b.ctypes.data if b.size else 0 for b in bufs])
        lens = (ctypes.c_uint64 * max(k, 1))(*[b.size for b in bufs])
        n_hint = sum(b.size for b in bufs) // 16
        nb = int(self.lib.hg_block_count(n_hint, block_stride)) if block_stride else 0
        blocks = np.empty(max(nb, 1), dtype=BLOCK_DTYPE) if block_stride else None
        out_len, res = ctypes.c_uint64(), HgMergeResult()
        ctxs, nctx = self._args()
        rc = self.lib.hg_multi_compact_host(
            ctxs, nctx, k, ctypes.cast(ptrs, ctypes.c_void_p), ctypes.cast(lens, ctypes.c_void_p),
            out.ctypes.data_as(ctypes.c_void_p), cap, ctypes.byref(out_len), int(block_stride),
            blocks.ctypes.data_as(ctypes.c_void_p) if blocks is not None else ctypes.c_void_p(0),
            ctypes.byref(res))
        if rc in (Status.HIP, Status.INVALID_ARG, Status.INTERNAL, Status.TOO_LARGE):
            raise HorreumGpuError(rc, "hg_multi_compact_host")
        nbo = int(self.lib.hg_block_count(res.n_out, block_stride)) if block_stride else 0
        return CompactOut(rc, out[:out_len.value], blocks[:nbo] if blocks is not None else None,
                          res.n_out, res.kind, res.table, res.index)
