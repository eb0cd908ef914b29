#!/usr/bin/env python3
"""Lane-walk pre-pass phase cycles (decode_spec_kernel, LW_STAMP): per pre-pass
batch, s_memtime cycles per phase as thread 0 of the workgroup sees them
(0 staging, 1 masks + guesses + walks, 2 chain marks, 3 relaxation rounds,
4 count scan, 5 span stores, 6 lead-in probe, 7 rounds run), for the
decode_variants workloads named on the command line (default small medium).
The instrumented launch goes through hgk_decode_launch_diag; its timing is
not quoted anywhere.  The phase clock is compiled in only by
`tools/build_variant.sh diag "-DHG_LW_DIAG=1"` (run with HG_LIBRARY pointing at
build_exp/diag/libhorreum_gpu.so); the default build records nothing."""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from decode_variants import workloads  # noqa: E402
from horreum_amd import abi  # noqa: E402
from horreum_amd.engine import Engine  # noqa: E402
from horreum_amd import abi as _abi  # noqa: E402
_abi.knobs_from_env()  # the A/B scripts' HG_* knobs (the library reads no environment)

PIECE, BATCH_MIN, SPEC_BP_MIN, DIAG_WORDS, LW_PROF = 16384, 16, 4, 24, 8
NAMES = ["fetch_masks", "guess_walk", "chain", "relax", "store", "stitch", "leadin", "nrounds"]


def main():
    only = sys.argv[1:] or ["small", "medium"]
    eng = Engine(0)
    lib = abi.load_library()
    lib.hgk_decode_launch_diag.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                           ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_void_p]
    lib.hgk_decode_workspace_bytes.argtypes = [ctypes.c_uint64]
    lib.hgk_decode_workspace_bytes.restype = ctypes.c_uint64
    lay = (ctypes.c_uint64 * 8)()
    for label, sst in workloads(eng.device):
        if not any(w in label for w in only):
            continue
        L = sst.numel()
        npieces = (L + PIECE - 1) // PIECE
        nch = (npieces + BATCH_MIN - 1) // BATCH_MIN
        nspec_max = (npieces + SPEC_BP_MIN - 1) // SPEC_BP_MIN
        ws = torch.zeros(int(lib.hgk_decode_workspace_bytes(L)), dtype=torch.uint8, device=eng.device)
        spans = eng.empty((L // 16) * 16)
        res = eng.empty(64)
        diag = torch.zeros(nch * DIAG_WORDS + nspec_max * LW_PROF, dtype=torch.int32,
                           device=eng.device)
        stream = torch.cuda.current_stream(eng.device).cuda_stream
        for _ in range(2):
            diag.zero_()
            rc = lib.hgk_decode_launch_diag(ctypes.c_void_p(sst.data_ptr()), L,
                                            ctypes.c_void_p(spans.data_ptr()), L // 16,
                                            ctypes.c_void_p(res.data_ptr()),
                                            ctypes.c_void_p(ws.data_ptr()),
                                            ctypes.c_void_p(diag.data_ptr()), ctypes.c_void_p(stream))
            assert rc == 0
            torch.cuda.synchronize()
        lib.hgk_decode_last_layout(lay)
        nspec, sbp = int(lay[2]), int(lay[3])
        d = diag[nch * DIAG_WORDS:].cpu().numpy().astype(np.uint32).reshape(-1, LW_PROF)[:nspec]
        d = d[d[:, 0] > 0]
        out = {"label": label, "batches": int(d.shape[0]), "pieces_per_batch": sbp}
        for k, n in enumerate(NAMES):
            col = d[:, k].astype(np.float64)
            per = col / sbp if k < 6 else col
            out[n] = {"p50_per_piece" if k < 6 else "p50": round(float(np.median(per)), 1),
                      "p90": round(float(np.percentile(per, 90)), 1)}
        tot = d[:, :7].sum(axis=1).astype(np.float64)
        out["total_cycles_per_batch_p50"] = float(np.median(tot))
        print(json.dumps(out), flush=True)
        del ws, spans, diag, sst


if __name__ == "__main__":
    main()
