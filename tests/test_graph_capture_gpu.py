"""the single-table decode and the encode keep per-context
state between calls (which control half the previous call left clean).  A
call captured into a HIP graph must not lean on it: every replay reuses the
half captured.  Each entry point captured once and replayed several times,
with eager calls on the same context in between (they flip the halves), every
result against the oracle (src/format.rs:23-77).  Also: the entry points
that stage arguments through pinned memory refuse a capturing stream, and
hg_ctx_reserve leaves nothing for the first calls to allocate."""
import ctypes

import numpy as np
import pytest

from oracle import oracle
from tests import corpus

pytestmark = pytest.mark.gpu


def _table(n, seed):
    arena, pairs = corpus.mixed(n, 24, 600, seed=seed)
    return arena, pairs, oracle.encode(arena, pairs)[0]


def _check_decode(eng, spans, res, want):
    ws, wn, wk, _, _ = want
    r = res[:24].cpu().numpy()
    assert int(r[:8].view("<u8")[0]) == wn and int(r[8:12].view("<i4")[0]) == wk == 0
    assert np.array_equal(eng.spans_to_numpy(spans, wn), ws)


def test_decode_capture_replay(knobs):
    import torch
    from horreum_amd.engine import Engine
    _, _, table = _table(60_000, 901)  # ~20 MB: many pre-pass batches, look-back across them
    want = oracle.decode(table)
    eng = Engine(0)
    try:
        eng.reserve(table.size, 0)
        d = eng.to_device(table)
        cap = table.size // 16
        spans, res = eng.empty(cap * 16), eng.empty(64)
        s = torch.cuda.Stream()
        # an eager warm-up call on the capture stream
        with torch.cuda.stream(s):
            eng.set_stream(s)
            eng.decode_dev_async(d, table.size, spans, cap, res)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s, capture_error_mode="relaxed"):
            eng.set_stream(torch.cuda.current_stream())
            eng.decode_dev_async(d, table.size, spans, cap, res)
        eng.set_stream(s)
        for i in range(4):
            spans.fill_(0xEE)
            res.fill_(0xEE)
            g.replay()
            torch.cuda.synchronize()
            _check_decode(eng, spans, res, want)
            if i % 2 == 0:  # an eager call between replays flips the halves
                spans.fill_(0xEE)
                with torch.cuda.stream(s):
                    eng.decode_dev_async(d, table.size, spans, cap, res)
                torch.cuda.synchronize()
                _check_decode(eng, spans, res, want)
        del g
    finally:
        eng.close()


def test_encode_capture_replay():
    import torch
    from horreum_amd.engine import Engine
    arena, pairs, want = _table(80_000, 902)
    _, _, wblocks, _ = oracle.encode(arena, pairs, block_stride=7)
    eng = Engine(0)
    try:
        n = pairs.size
        eng.reserve(0, n)
        da = eng.to_device(arena)
        dp = eng.to_device(pairs.view(np.uint8))
        out = eng.empty(want.size)
        nb = (n + 6) // 7
        blocks = eng.empty(nb * 24)
        res = eng.empty(64)
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            eng.set_stream(s)
            eng.encode_dev_async(da, dp, n, out, want.size, None, 7, blocks, res)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s, capture_error_mode="relaxed"):
            eng.set_stream(torch.cuda.current_stream())
            eng.encode_dev_async(da, dp, n, out, want.size, None, 7, blocks, res)
        eng.set_stream(s)
        for i in range(4):
            out.fill_(0)
            blocks.fill_(0)
            g.replay()
            torch.cuda.synchronize()
            r = res[:16].cpu().numpy()
            assert int(r[:8].view("<u8")[0]) == want.size and int(r[8:12].view("<i4")[0]) == 0
            assert np.array_equal(out.cpu().numpy(), want), i
            assert np.array_equal(blocks.cpu().numpy().view("<u8").reshape(-1, 3),
                                  wblocks.view("<u8").reshape(-1, 3)), i
            if i % 2 == 0:
                out.fill_(0)
                with torch.cuda.stream(s):
                    eng.encode_dev_async(da, dp, n, out, want.size, None, 7, blocks, res)
                torch.cuda.synchronize()
                assert np.array_equal(out.cpu().numpy(), want), i
        del g
    finally:
        eng.close()


def test_staged_entry_points_refuse_capture():
    """hg_decode_batch_dev_async and hg_merge_dev_async stage their
    arguments through pinned host memory (re-read at a replay): they return
    HG_ERR_INVALID_ARG on a capturing stream and enqueue nothing."""
    import torch
    from horreum_amd.engine import Engine
    _, _, table = _table(2_000, 903)
    eng = Engine(0)
    try:
        d = eng.to_device(table)
        spans, res = eng.empty(table.size), eng.empty(64)
        lib = eng.lib
        tp = (ctypes.c_void_p * 1)(d.data_ptr())
        ln = (ctypes.c_uint64 * 1)(table.size)
        sp = (ctypes.c_void_p * 1)(spans.data_ptr())
        cp = (ctypes.c_uint64 * 1)(table.size // 16)
        s = torch.cuda.Stream()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s, capture_error_mode="relaxed"):
            eng.set_stream(torch.cuda.current_stream())
            rc_b = lib.hg_decode_batch_dev_async(eng.ctx, 1, ctypes.cast(tp, ctypes.c_void_p),
                                                 ctypes.cast(ln, ctypes.c_void_p),
                                                 ctypes.cast(sp, ctypes.c_void_p),
                                                 ctypes.cast(cp, ctypes.c_void_p),
                                                 ctypes.c_void_p(res.data_ptr()))
            toff = (ctypes.c_uint64 * 1)(0)
            cnt = (ctypes.c_uint64 * 1)(10)
            rc_m = lib.hg_merge_dev_async(eng.ctx, 1, ctypes.c_void_p(d.data_ptr()), table.size,
                                          ctypes.cast(toff, ctypes.c_void_p),
                                          ctypes.cast(sp, ctypes.c_void_p),
                                          ctypes.cast(cnt, ctypes.c_void_p),
                                          ctypes.c_void_p(spans.data_ptr()), 10,
                                          ctypes.c_void_p(res.data_ptr()))
            res.zero_()  # something to capture
        eng.set_stream(None)
        assert (rc_b, rc_m) == (-1, -1)
        del g
    finally:
        eng.close()


def test_reserve_then_first_calls_do_not_grow():
    """after hg_ctx_reserve the first encode (its group
    sums) and a one-table batched decode allocate nothing: the device memory
    the allocator reports does not move across them."""
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
        torch.cuda.synchronize()
        free0 = torch.cuda.mem_get_info()[0]
        eng.encode_dev_async(da, dp, n, out, table.size, None, 0, None, res)
        eng.decode_batch_dev_async([d], [table.size], [spans], [table.size // 16], res[64:])
        eng.decode_dev_async(d, table.size, spans, table.size // 16, res[64:])
        torch.cuda.synchronize()
        free1 = torch.cuda.mem_get_info()[0]
        assert free1 == free0, (free0, free1)
        assert np.array_equal(out.cpu().numpy(), table)
    finally:
        eng.close()
