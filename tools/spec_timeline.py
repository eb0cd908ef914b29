#!/usr/bin/env python3
"""Pre-pass timeline on cfg 2 (diagnostics; needs a library built with
-DHG_SPEC_TIMELINE, passed as HG_LIBRARY): per pre-pass workgroup the
realtime clock (100 MHz) at its start, after its first piece and at its
end, read back from the span scratch of each batch's first piece.  Prints
the spread of start times, first-piece times, streaming times and end
times over the workgroups, in microseconds."""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from horreum_amd import synth  # noqa: E402
from horreum_amd.engine import Engine  # noqa: E402
from horreum_amd import abi as _abi  # noqa: E402
_abi.knobs_from_env()  # the A/B scripts' HG_* knobs (the library reads no environment)

MAX_REC_PIECE = 1024


def main():
    eng = Engine(0)
    eng.set_stream(torch.cuda.current_stream(eng.device))
    sst = synth.fixed_sst(8_134_407, 16, 100, seed=2, device=eng.device)
    L = sst.numel()
    lib = eng.lib
    lib.hgk_ctx_workspace.restype = ctypes.c_void_p
    lib.hgk_ctx_workspace.argtypes = [ctypes.c_void_p]
    lib.hgk_debug_d2h.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
    so, po, to = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
    lib.hgk_decode_ws_layout(ctypes.c_uint64(L), ctypes.byref(so), ctypes.byref(po), ctypes.byref(to))
    for rep in range(int(os.environ.get("REPS", 4))):
        out = eng.decode_dev(sst, L)
        torch.cuda.synchronize()
        lay = (ctypes.c_uint64 * 8)()
        lib.hgk_decode_last_layout(lay)
        nspec, sbp = int(lay[2]), int(lay[3])
        ws = lib.hgk_ctx_workspace(eng.ctx)
        t = np.zeros((nspec, 5), np.uint64)
        row = np.zeros(5, np.uint64)
        for b in range(nspec):
            lib.hgk_debug_d2h(row.ctypes.data_as(ctypes.c_void_p),
                              ctypes.c_void_p(ws + so.value + b * sbp * MAX_REC_PIECE * 16), 40)
            t[b] = row
        t0 = t[:, 0].min()
        us = (t.astype(np.int64) - int(t0)) / 100.0  # 100 MHz
        q = lambda v: [round(float(x), 1) for x in np.percentile(v, [0, 10, 50, 90, 100])]
        print(json.dumps({"rep": rep, "records": out.n, "nspec": nspec, "sbp": sbp,
                          "start_us_pct_0_10_50_90_100": q(us[:, 0]),
                          "first_piece_us": q(us[:, 1] - us[:, 0]),
                          "piece0_landed_us": q(us[:, 3] - us[:, 0]),
                          "guess_done_us (b > 0)": q((us[1:, 4] - us[1:, 0])),
                          "rest_us": q(us[:, 2] - us[:, 1]),
                          "end_us": q(us[:, 2])}), flush=True)
        x = np.arange(nspec) % 8  # the XCD a workgroup lands on (round-robin dispatch)
        if os.environ.get("SWAP_PAIRS"):  # batch b ran on workgroup b ^ 1
            x = (np.arange(nspec) ^ 1) % 8
        print(json.dumps({"rep": rep, "by_blockIdx_mod_8": {
            "first_piece_us": [round(float(np.mean((us[:, 1] - us[:, 0])[x == k])), 1) for k in range(8)],
            "rest_us": [round(float(np.mean((us[:, 2] - us[:, 1])[x == k])), 1) for k in range(8)],
            "end_us_max": [round(float(np.max(us[:, 2][x == k])), 1) for k in range(8)]}}), flush=True)


if __name__ == "__main__":
    main()
