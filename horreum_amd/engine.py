"""Device engine: one HIP context (GPU + stream) and its buffers.

PyTorch is used only as plumbing: HBM allocations (`torch.empty(..., device=
"cuda")`) and the stream the C ABI launches on (torch's current stream by
default, so torch/HIP events time exactly the launched kernels).  All compute
happens in libhorreum_gpu.so; there is no CPU fallback.
"""
import ctypes
from collections import namedtuple

import numpy as np

from .abi import (BLOCK_DTYPE, KEY_DTYPE, LOOKUP_DTYPE, PAIR_DTYPE, SPAN_DTYPE, HgErr,
                  HgMergeResult, HorreumGpuError, Status, check, load_library)

DecodeOut = namedtuple("DecodeOut", "spans n kind offset")
EncodeOut = namedtuple("EncodeOut", "data rec_off blocks out_len")
MergeOut = namedtuple("MergeOut", "status n kind table index")
CompactOut = namedtuple("CompactOut", "status data blocks n kind table index")
ResidentTable = namedtuple("ResidentTable", "table spans index n kind offset")


def _torch():
    import torch  # noqa: WPS433 (deferred: importing torch is slow)
    return torch


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


class Engine:
    """A context on `device`.  Not thread-safe; use one Engine per thread."""

    def __init__(self, device=0, use_torch_stream=True):
        self.lib = load_library()
        torch = _torch()
        if not torch.cuda.is_available():
            raise HorreumGpuError(Status.HIP, "no HIP device visible")
        self.device = torch.device("cuda", device)
        ctx = ctypes.c_void_p()
        check(self.lib.hg_ctx_create(device, ctypes.byref(ctx)), "hg_ctx_create")
        self.ctx = ctx
        if use_torch_stream:
            self.set_stream(torch.cuda.current_stream(self.device))

    # ---- context --------------------------------------------------------------
    def set_stream(self, stream):
        """Launch on a torch stream (its handle may be 0: the null stream);
        None selects the context's own stream."""
        if stream is None:
            check(self.lib.hg_ctx_use_own_stream(self.ctx), "hg_ctx_use_own_stream")
            return
        check(self.lib.hg_ctx_set_stream(self.ctx, ctypes.c_void_p(stream.cuda_stream)),
              "hg_ctx_set_stream")

    def reserve(self, max_sst_bytes=0, max_pairs=0):
        check(self.lib.hg_ctx_reserve(self.ctx, max_sst_bytes, max_pairs), "hg_ctx_reserve")

    def synchronize(self):
        check(self.lib.hg_ctx_synchronize(self.ctx), "hg_ctx_synchronize")

    def close(self):
        if getattr(self, "ctx", None):
            self.lib.hg_ctx_destroy(self.ctx)
            self.ctx = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    # ---- device buffers ---------------------------------------------------------
    def empty(self, nbytes):
        torch = _torch()
        return torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=self.device)

    def to_device(self, array):
        torch = _torch()
        a = np.ascontiguousarray(np.frombuffer(memoryview(array).cast("B"), dtype=np.uint8))
        return torch.from_numpy(a.copy()).to(self.device) if a.size else self.empty(1)

    # ---- decode -------------------------------------------------------------------
    def decode_dev(self, sst, length=None, spans=None, cap=None):
        """Decode `length` bytes of the uint8 device tensor `sst`.

        Returns DecodeOut(spans=device uint8 tensor [cap*16], n, kind, offset);
        raises HorreumGpuError on runtime failures only (format errors are
        returned in `kind`, as the ABI does)."""
        length = sst.numel() if length is None else int(length)
        if cap is None:
            cap = length // 16 if spans is None else spans.numel() // SPAN_DTYPE.itemsize
        if spans is None:
            spans = self.empty(cap * SPAN_DTYPE.itemsize)
        n = ctypes.c_uint64()
        err = HgErr()
        rc = self.lib.hg_decode_dev(self.ctx, _ptr(sst), length, _ptr(spans), cap,
                                    ctypes.byref(n), ctypes.byref(err))
        if rc < 0:
            raise HorreumGpuError(rc, "hg_decode_dev")
        return DecodeOut(spans, n.value, err.kind, err.offset)

    def decode_dev_async(self, sst, length, spans, cap, result):
        check(self.lib.hg_decode_dev_async(self.ctx, _ptr(sst), int(length), _ptr(spans),
                                           int(cap), _ptr(result)), "hg_decode_dev_async")

    def decode_batch_dev_async(self, tables, lens, spans, caps, results):
        """Decode many device tables in one launch chain on the context
        stream (every table keeps its own workspace slice).  `results`:
        device tensor of at least len(tables) * 24 bytes (hg_decode_result
        records)."""
        k = len(tables)
        tp = (ctypes.c_void_p * max(k, 1))(*[t.data_ptr() for t in tables])
        ln = (ctypes.c_uint64 * max(k, 1))(*[int(x) for x in lens])
        sp = (ctypes.c_void_p * max(k, 1))(*[s.data_ptr() for s in spans])
        cp = (ctypes.c_uint64 * max(k, 1))(*[int(x) for x in caps])
        check(self.lib.hg_decode_batch_dev_async(self.ctx, k, ctypes.cast(tp, ctypes.c_void_p),
                                                 ctypes.cast(ln, ctypes.c_void_p),
                                                 ctypes.cast(sp, ctypes.c_void_p),
                                                 ctypes.cast(cp, ctypes.c_void_p), _ptr(results)),
              "hg_decode_batch_dev_async")

    def decode_host(self, data, cap=None, out=None):
        """Host bytes in, numpy SPAN_DTYPE array out.  Page-locked buffers
        (pinned, or registered with host_register) are DMA'd directly;
        pageable ones go through the pinned staging pipeline.  `out`: an
        optional preallocated SPAN_DTYPE array (e.g. a pinned one)."""
        buf = np.ascontiguousarray(np.frombuffer(memoryview(data).cast("B"), dtype=np.uint8))
        if out is not None:
            spans = out
            cap = spans.size if cap is None else min(int(cap), spans.size)
        else:
            cap = buf.size // 16 if cap is None else int(cap)
            spans = np.zeros(max(cap, 1), dtype=SPAN_DTYPE)
        n = ctypes.c_uint64()
        err = HgErr()
        rc = self.lib.hg_decode_host(self.ctx, buf.ctypes.data_as(ctypes.c_void_p), buf.size,
                                     spans.ctypes.data_as(ctypes.c_void_p), cap, ctypes.byref(n),
                                     ctypes.byref(err))
        if rc < 0:
            raise HorreumGpuError(rc, "hg_decode_host")
        return DecodeOut(spans[: min(n.value, cap)], n.value, err.kind, err.offset)

    def decode_range_dev(self, sst, length, begin, stop, entry, spans=None, cap=None):
        """Range decode (hg_decode_range_dev): the records of the device
        table `sst` (length bytes) that start in [entry, stop), entry an exact
        record start.  Returns (DecodeOut, exit)."""
        if cap is None:
            cap = max(int(stop) - int(begin), 0) // 16 + 2 if spans is None \
                else spans.numel() // SPAN_DTYPE.itemsize
        if spans is None:
            spans = self.empty(max(int(cap), 1) * SPAN_DTYPE.itemsize)
        n, ex, err = ctypes.c_uint64(), ctypes.c_uint64(), HgErr()
        rc = self.lib.hg_decode_range_dev(self.ctx, _ptr(sst), int(length), int(begin), int(stop),
                                          int(entry), _ptr(spans), int(cap), ctypes.byref(n),
                                          ctypes.byref(ex), ctypes.byref(err))
        if rc < 0:
            raise HorreumGpuError(rc, "hg_decode_range_dev")
        return DecodeOut(spans, n.value, err.kind, err.offset), ex.value

    def guess_entry_dev(self, sst, length, stop):
        """Speculative first record start at or after `stop` (a guess)."""
        e = ctypes.c_uint64()
        check(self.lib.hg_decode_guess_entry_dev(self.ctx, _ptr(sst), int(length), int(stop),
                                                 ctypes.byref(e)), "hg_decode_guess_entry_dev")
        return e.value

    def encoded_size(self, pairs, n=None):
        """sum(16 + klen + vlen) of hg_pair records: a numpy PAIR_DTYPE array
        (summed on the host) or a uint8 device tensor (reduced on the device)."""
        out = ctypes.c_uint64()
        if isinstance(pairs, np.ndarray):
            pairs = np.ascontiguousarray(pairs, dtype=PAIR_DTYPE)
            ptr, n = pairs.ctypes.data_as(ctypes.c_void_p), pairs.size
        else:
            ptr = _ptr(pairs)
            n = pairs.numel() // PAIR_DTYPE.itemsize if n is None else int(n)
        check(self.lib.hg_encoded_size(self.ctx, ptr, n, ctypes.byref(out)), "hg_encoded_size")
        return out.value

    def trim(self):
        """Free this context's device work buffers (hg_ctx_trim): they grow
        again on demand."""
        check(self.lib.hg_ctx_trim(self.ctx), "hg_ctx_trim")

    def decode_many_host(self, tables):
        """Many host tables (bytes-like) decoded by ONE batched launch chain on
        this context (hg_multi_decode_host with one context; the cold open of
        a table directory, src/sstable/manager.rs:47-55) -> [DecodeOut]."""
        bufs = [np.ascontiguousarray(np.frombuffer(memoryview(t).cast("B"), dtype=np.uint8))
                for t in tables]
        k = len(bufs)
        if k == 0:
            return []
        spans = [np.zeros(max(b.size // 16, 1), dtype=SPAN_DTYPE) for b in bufs]
        tp = (ctypes.c_void_p * k)(*[b.ctypes.data if b.size else 0 for b in bufs])
        ln = (ctypes.c_uint64 * k)(*[b.size for b in bufs])
        sp = (ctypes.c_void_p * k)(*[x.ctypes.data for x in spans])
        cp = (ctypes.c_uint64 * k)(*[b.size // 16 for b in bufs])
        n_out = (ctypes.c_uint64 * k)()
        errs = (HgErr * k)()
        ctxs = (ctypes.c_void_p * 1)(self.ctx.value)
        check(self.lib.hg_multi_decode_host(ctypes.cast(ctxs, ctypes.c_void_p), 1, k,
                                            ctypes.cast(tp, ctypes.c_void_p),
                                            ctypes.cast(ln, ctypes.c_void_p),
                                            ctypes.cast(sp, ctypes.c_void_p),
                                            ctypes.cast(cp, ctypes.c_void_p),
                                            ctypes.cast(n_out, ctypes.c_void_p),
                                            ctypes.cast(errs, ctypes.c_void_p)),
              "hg_multi_decode_host")
        return [DecodeOut(spans[i][:min(n_out[i], bufs[i].size // 16)], n_out[i], errs[i].kind,
                          errs[i].offset) for i in range(k)]

    # ---- host memory ---------------------------------------------------------------
    def host_register(self, array):
        """Page-lock a host numpy buffer for direct DMA (hipHostRegister)."""
        check(self.lib.hg_host_register(ctypes.c_void_p(array.ctypes.data), array.nbytes),
              "hg_host_register")

    def host_unregister(self, array):
        check(self.lib.hg_host_unregister(ctypes.c_void_p(array.ctypes.data)),
              "hg_host_unregister")

    def host_is_pinned(self, array):
        return bool(self.lib.hg_host_is_pinned(ctypes.c_void_p(array.ctypes.data)))

    @staticmethod
    def spans_to_numpy(spans, n):
        return spans[: n * SPAN_DTYPE.itemsize].cpu().numpy().view(SPAN_DTYPE)

    # ---- encode -------------------------------------------------------------------
    def encode_dev(self, arena, pairs, n, out=None, cap=None, rec_off=None, block_stride=0,
                   blocks=None):
        """Encode `n` hg_pair records (uint8 device tensor `pairs`) whose bytes
        live in device tensor `arena`.  Returns the encoded length."""
        if out is None:
            raise ValueError("out buffer required")
        cap = out.numel() if cap is None else int(cap)
        out_len = ctypes.c_uint64()
        rc = self.lib.hg_encode_dev(self.ctx, _ptr(arena), _ptr(pairs), int(n), _ptr(out), cap,
                                    _ptr(rec_off), int(block_stride), _ptr(blocks),
                                    ctypes.byref(out_len))
        if rc not in (Status.OK, Status.CAPACITY):
            raise HorreumGpuError(rc, "hg_encode_dev")
        return rc, out_len.value

    def encode_dev_async(self, arena, pairs, n, out, cap, rec_off, block_stride, blocks, result):
        check(self.lib.hg_encode_dev_async(self.ctx, _ptr(arena), _ptr(pairs), int(n), _ptr(out),
                                           int(cap), _ptr(rec_off), int(block_stride),
                                           _ptr(blocks), _ptr(result)), "hg_encode_dev_async")

    def encode_host(self, arena, pairs, block_stride=0, want_rec_off=False, out=None):
        """numpy arena (uint8) + PAIR_DTYPE records -> EncodeOut (numpy).
        `out`: optional caller-owned uint8 buffer of >= the encoded size (e.g.
        page-locked with host_register: with arena, pairs and out all
        page-locked the upload and download overlap in chunks)."""
        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        pairs = np.ascontiguousarray(pairs, dtype=PAIR_DTYPE)
        n = pairs.size
        total = int((16 + pairs["klen"].astype(np.uint64) + pairs["vlen"].astype(np.uint64)).sum())
        if out is None:
            out = np.empty(max(total, 1), dtype=np.uint8)
        elif out.dtype != np.uint8 or out.size < total or not out.flags.c_contiguous:
            raise ValueError("out must be a contiguous uint8 array of >= %d bytes" % total)
        rec_off = np.empty(max(n, 1), dtype=np.uint64) if want_rec_off else None
        nb = int(self.lib.hg_block_count(n, block_stride)) if block_stride else 0
        blocks = np.empty(max(nb, 1), dtype=BLOCK_DTYPE) if block_stride else None
        out_len = ctypes.c_uint64()

        def vp(a):
            return a.ctypes.data_as(ctypes.c_void_p) if a is not None else ctypes.c_void_p(0)

        rc = self.lib.hg_encode_host(self.ctx, vp(arena), arena.size, vp(pairs), n, vp(out),
                                     total, vp(rec_off), int(block_stride), vp(blocks),
                                     ctypes.byref(out_len))
        check(rc, "hg_encode_host")
        return EncodeOut(out[:total], rec_off[:n] if rec_off is not None else None,
                         blocks[:nb] if blocks is not None else None, out_len.value)


    # ---- point lookups ----------------------------------------------------------------
    @staticmethod
    def pack_keys(keys):
        """[bytes] -> (key arena uint8, KEY_DTYPE descriptors)."""
        keys = [bytes(k) for k in keys]
        desc = np.zeros(len(keys), dtype=KEY_DTYPE)
        off = 0
        for i, k in enumerate(keys):
            desc[i] = (off, len(k), 0)
            off += len(k)
        arena = np.frombuffer(b"".join(keys), dtype=np.uint8) if off else np.zeros(1, np.uint8)
        return arena, desc

    def lookup_host(self, table, keys, block_stride=0):
        """SSTable::get for many keys (src/sstable/table.rs:54-70) on host
        table bytes with blocks of `block_stride` records (0: one block) ->
        LOOKUP_DTYPE results (found, rec, val_off, vlen)."""
        buf = np.ascontiguousarray(np.frombuffer(memoryview(table).cast("B"), dtype=np.uint8))
        arena, desc = self.pack_keys(keys)
        out = np.zeros(max(len(desc), 1), dtype=LOOKUP_DTYPE)
        check(self.lib.hg_lookup_host(self.ctx, buf.ctypes.data_as(ctypes.c_void_p), buf.size,
                                      int(block_stride), arena.ctypes.data_as(ctypes.c_void_p),
                                      int(desc["len"].sum()) if desc.size else 0,
                                      desc.ctypes.data_as(ctypes.c_void_p), desc.size,
                                      out.ctypes.data_as(ctypes.c_void_p)), "hg_lookup_host")
        return out[: desc.size]

    def resident_table(self, data):
        """Upload host table bytes once and keep what lookups need in HBM:
        the bytes, their spans and the key index (SSTable::get's state,
        src/sstable/table.rs:54-70).  Raises DecodeError-like HorreumGpuError
        via the caller if the table does not decode."""
        buf = np.ascontiguousarray(np.frombuffer(memoryview(data).cast("B"), dtype=np.uint8))
        dev = self.to_device(buf)
        out = self.decode_dev(dev, buf.size)
        idx = self.keyindex_build(dev, out.spans, out.n) if out.kind == 0 else None
        return ResidentTable(dev, out.spans, idx, out.n, out.kind, out.offset)

    def lookup_resident(self, rt, keys, block_stride=0):
        """Batched point lookups against a ResidentTable (blocks of
        `block_stride` records, 0: one block): only the query keys go up and
        the results come back (LOOKUP_DTYPE)."""
        torch = _torch()
        arena, desc = self.pack_keys(keys)
        nq = desc.size
        res = torch.empty(max(nq, 1) * LOOKUP_DTYPE.itemsize, dtype=torch.uint8,
                          device=self.device)
        if nq:
            kd = self.to_device(arena)
            qd = self.to_device(desc.view(np.uint8))
            self.lookup_dev_async(rt.table, rt.spans, rt.index, rt.n, kd, qd, nq, res,
                                  block_stride)
        out = res[: nq * LOOKUP_DTYPE.itemsize].cpu().numpy().view(LOOKUP_DTYPE)
        return out

    def keyindex_build(self, table, spans, n):
        """Device key index (32 B per record) of a decoded device table."""
        idx = self.empty(max(int(self.lib.hg_keyindex_bytes(n)), 1))
        check(self.lib.hg_keyindex_build_dev_async(self.ctx, _ptr(table), table.numel(),
                                                   _ptr(spans), int(n), _ptr(idx)),
              "hg_keyindex_build_dev_async")
        return idx

    def lookup_dev_async(self, table, spans, index, n, keys, queries, nq, results, block_stride=0):
        check(self.lib.hg_lookup_dev_async(self.ctx, _ptr(table), _ptr(spans), _ptr(index), int(n),
                                           int(block_stride), _ptr(keys), _ptr(queries), int(nq),
                                           _ptr(results)),
              "hg_lookup_dev_async")

    # ---- merge / compaction -----------------------------------------------------------
    def merge_dev(self, arena, table_off, spans, counts, out, cap):
        """k-way merge of decoded tables living in device tensor `arena`.
        table_off: byte offset of each table in the arena; spans: device
        tensors of hg_span records (offsets relative to each table); counts:
        records per table.  Priority order: index 0 wins equal keys.  Writes
        hg_pair records (offsets into the arena) to device tensor `out`."""
        k = len(counts)
        toff = (ctypes.c_uint64 * max(k, 1))(*[int(x) for x in table_off])
        sp = (ctypes.c_void_p * max(k, 1))(*[s.data_ptr() if s is not None else 0 for s in spans])
        cnt = (ctypes.c_uint64 * max(k, 1))(*[int(x) for x in counts])
        res = HgMergeResult()
        rc = self.lib.hg_merge_dev(self.ctx, k, _ptr(arena), arena.numel() if arena is not None
                                   else 0, ctypes.cast(toff, ctypes.c_void_p),
                                   ctypes.cast(sp, ctypes.c_void_p),
                                   ctypes.cast(cnt, ctypes.c_void_p), _ptr(out), int(cap),
                                   ctypes.byref(res))
        if rc in (Status.HIP, Status.INVALID_ARG, Status.INTERNAL):
            raise HorreumGpuError(rc, "hg_merge_dev")
        return MergeOut(rc, res.n_out, res.kind, res.table, res.index)

    def compact_host(self, tables, block_stride=0, out=None):
        """SSTableManager::compact's byte work (src/sstable/manager.rs:137-159)
        on host bytes: `tables` (bytes-like, priority order: newest first) ->
        the compacted SSTable bytes (+ index blocks).  `out`: optional
        caller-owned uint8 buffer of at least the total input size (the
        result is a view of it), so repeated calls do not fault in fresh
        pages."""
        bufs = [np.ascontiguousarray(np.frombuffer(memoryview(t).cast("B"), dtype=np.uint8))
                for t in tables]
        k = len(bufs)
        ptrs = (ctypes.c_void_p * max(k, 1))(*[b.ctypes.data if b.size else 0 for b in bufs])
        lens = (ctypes.c_uint64 * max(k, 1))(*[b.size for b in bufs])
        cap = max(sum(b.size for b in bufs), 1)
        if out is None:
            out = np.empty(cap, dtype=np.uint8)
        elif out.dtype != np.uint8 or out.size < cap or not out.flags.c_contiguous:
            raise ValueError("out must be a contiguous uint8 array of >= %d bytes" % cap)
        n_hint = sum(b.size for b in bufs) // 16
        nb = int(self.lib.hg_block_count(n_hint, block_stride)) if block_stride else 0
        blocks = np.empty(max(nb, 1), dtype=BLOCK_DTYPE) if block_stride else None
        out_len = ctypes.c_uint64()
        res = HgMergeResult()
        rc = self.lib.hg_compact_host(self.ctx, k, ctypes.cast(ptrs, ctypes.c_void_p),
                                      ctypes.cast(lens, ctypes.c_void_p),
                                      out.ctypes.data_as(ctypes.c_void_p), cap,
                                      ctypes.byref(out_len), int(block_stride),
                                      blocks.ctypes.data_as(ctypes.c_void_p)
                                      if blocks is not None else ctypes.c_void_p(0),
                                      ctypes.byref(res))
        if rc in (Status.HIP, Status.INVALID_ARG, Status.INTERNAL, Status.TOO_LARGE):
            raise HorreumGpuError(rc, "hg_compact_host")
        nbo = int(self.lib.hg_block_count(res.n_out, block_stride)) if block_stride else 0
        return CompactOut(rc, out[:out_len.value], blocks[:nbo] if blocks is not None else None,
                          res.n_out, res.kind, res.table, res.index)

    def compact_dev(self, arena, table_off, lens, out, block_stride=0, blocks=None):
        """compact_host on tables already in device tensor `arena` (table t =
        arena[table_off[t], +lens[t]), priority order: newest first).  Writes
        the compacted SSTable to device tensor `out` (and, with block_stride,
        its index blocks to device tensor `blocks`); returns CompactOut whose
        `data` is the written prefix of `out` (blocks: the written prefix of
        `blocks`, as hg_block records in a uint8 tensor)."""
        k = len(lens)
        toff = (ctypes.c_uint64 * max(k, 1))(*[int(x) for x in table_off])
        ln = (ctypes.c_uint64 * max(k, 1))(*[int(x) for x in lens])
        out_len = ctypes.c_uint64()
        res = HgMergeResult()
        rc = self.lib.hg_compact_dev(self.ctx, k, _ptr(arena),
                                     arena.numel() if arena is not None else 0,
                                     ctypes.cast(toff, ctypes.c_void_p),
                                     ctypes.cast(ln, ctypes.c_void_p), _ptr(out),
                                     out.numel() if out is not None else 0, ctypes.byref(out_len),
                                     int(block_stride), _ptr(blocks), ctypes.byref(res))
        if rc in (Status.HIP, Status.INVALID_ARG, Status.INTERNAL, Status.TOO_LARGE):
            raise HorreumGpuError(rc, "hg_compact_dev")
        nbo = int(self.lib.hg_block_count(res.n_out, block_stride)) if block_stride else 0
        return CompactOut(rc, out[:out_len.value] if out is not None else None,
                          blocks[:nbo * 24] if blocks is not None else None,
                          res.n_out, res.kind, res.table, res.index)


_default = None


def default_engine():
    """Process-wide engine on cuda:0 (created on first use)."""
    global _default
    if _default is None:
        _default = Engine(0)
    return _default
