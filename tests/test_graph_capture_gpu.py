"""the single-table decode and the encode keep per-context
state between calls (which control half the previous call's kernels left
clear), which a HIP-graph replay would not follow.  Capture is therefore
refused by every stream-ordered entry point (HG_ERR_INVALID_ARG, nothing
enqueued).  ADVICE r5 (medium): after hg_ctx_reserve the first encode and a
one-table batched decode allocate nothing."""
import ctypes

import numpy as np
import pytest

from oracle import oracle
from tests import corpus

pytestmark = pytest.mark.gpu


def _table(n, seed):
    arena, pairs = corpus.mixed(n, 24, 600, seed=seed)
    return arena, pairs, oracle.encode(arena, pairs)[0]


def test_every_stream_ordered_entry_point_refuses_capture():
    """Graph capture is not supported (a context carries state between calls
    that a replay would not follow; round 6 saw a captured decode fault on
    its first replay): on a capturing stream every stream-ordered entry point
    returns HG_ERR_INVALID_ARG and enqueues nothing -- the capture holds only
    the caller's own work, and the context works normally afterwards."""
    import torch
    from horreum_amd.engine import Engine
    arena, pairs, table = _table(2_000, 903)
    want = oracle.decode(table)
    eng = Engine(0)
    try:
        d = eng.to_device(table)
        da, dp = eng.to_device(arena), eng.to_device(pairs.view(np.uint8))
        cap = table.size // 16
        spans, res, out = eng.empty(table.size), eng.empty(128), eng.empty(table.size)
        idx = eng.empty(64)
        lib = eng.lib
        vp = ctypes.c_void_p
        tp = (ctypes.c_void_p * 1)(d.data_ptr())
        ln = (ctypes.c_uint64 * 1)(table.size)
        sp = (ctypes.c_void_p * 1)(spans.data_ptr())
        cp = (ctypes.c_uint64 * 1)(cap)
        toff = (ctypes.c_uint64 * 1)(0)
        cnt = (ctypes.c_uint64 * 1)(10)
        s = torch.cuda.Stream()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        rcs = {}
        with torch.cuda.graph(g, stream=s, capture_error_mode="relaxed"):
            eng.set_stream(torch.cuda.current_stream())
            ctx = eng.ctx
            rcs["decode"] = lib.hg_decode_dev_async(ctx, vp(d.data_ptr()), table.size,
                                                    vp(spans.data_ptr()), cap, vp(res.data_ptr()))
            rcs["range"] = lib.hg_decode_range_dev_async(ctx, vp(d.data_ptr()), table.size, 0,
                                                         table.size, 0, vp(spans.data_ptr()), cap,
                                                         vp(res.data_ptr()))
            rcs["encode"] = lib.hg_encode_dev_async(ctx, vp(da.data_ptr()), vp(dp.data_ptr()),
                                                    pairs.size, vp(out.data_ptr()), table.size,
                                                    None, 0, None, vp(res.data_ptr()))
            rcs["batch"] = lib.hg_decode_batch_dev_async(ctx, 1, ctypes.cast(tp, vp),
                                                         ctypes.cast(ln, vp), ctypes.cast(sp, vp),
                                                         ctypes.cast(cp, vp), vp(res.data_ptr()))
            rcs["merge"] = lib.hg_merge_dev_async(ctx, 1, vp(d.data_ptr()), table.size,
                                                  ctypes.cast(toff, vp), ctypes.cast(sp, vp),
                                                  ctypes.cast(cnt, vp), vp(out.data_ptr()), 10,
                                                  vp(res.data_ptr()))
            rcs["keyindex"] = lib.hg_keyindex_build_dev_async(ctx, vp(d.data_ptr()), table.size,
                                                              vp(spans.data_ptr()), 1,
                                                              vp(idx.data_ptr()))
            rcs["lookup"] = lib.hg_lookup_dev_async(ctx, vp(d.data_ptr()), vp(spans.data_ptr()),
                                                    vp(idx.data_ptr()), 1, 0, vp(d.data_ptr()),
                                                    vp(idx.data_ptr()), 1, vp(res.data_ptr()))
            res.zero_()  # the caller's own work: all the graph holds
        eng.set_stream(torch.cuda.current_stream())
        assert rcs == {k: -1 for k in rcs}, rcs
        g.replay()
        torch.cuda.synchronize()
        del g
        # the context is usable after the refused capture
        out_d = eng.decode_dev(d, table.size)
        assert (out_d.n, out_d.kind) == (want[1], 0)
        assert np.array_equal(eng.spans_to_numpy(out_d.spans, out_d.n), want[0])
    finally:
        eng.close()


def test_reserve_then_first_calls_do_not_grow():
    """after hg_ctx_reserve the first encode (its group
    sums) and a one-table batched decode grow none of the context's work
    buffers (hgk_ctx_device_bytes, a diagnostics export)."""
    import torch
    from horreum_amd.engine import Engine
    arena, pairs, table = _table(40_000, 904)
    eng = Engine(0)
    try:
        n = pairs.size
        d = eng.to_device(table)
        da, dp = eng.to_device(arena), eng.to_device(pairs.view(np.uint8))
        out, spans, res = eng.empty(table.size), eng.empty(table.size), eng.empty(128)
        eng.reserve(table.size, n)
        held = eng.lib.hgk_ctx_device_bytes
        held.restype, held.argtypes = ctypes.c_uint64, [ctypes.c_void_p]
        b0 = held(eng.ctx)
        eng.encode_dev_async(da, dp, n, out, table.size, None, 0, None, res)
        eng.decode_batch_dev_async([d], [table.size], [spans], [table.size // 16], res[64:])
        eng.decode_dev_async(d, table.size, spans, table.size // 16, res[64:])
        torch.cuda.synchronize()
        assert held(eng.ctx) == b0, (b0, held(eng.ctx))  # no work buffer grew
        assert np.array_equal(out.cpu().numpy(), table)
    finally:
        eng.close()
