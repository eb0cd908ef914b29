#!/usr/bin/env python3
"""Per-chunk decode diagnostics (DIAG build of decode_kernel).

Prints phase durations (s_memtime cycles, relative to each chunk's start),
survivor counts, lifting levels, how the entry guess was made and whether it
held, and look-back spin counts, for the cfg2 table and a mixed-size table.
Timing of the DIAG build is not quoted anywhere: it exists for shares.
"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from horreum_amd import abi, synth  # noqa: E402
from horreum_amd.engine import Engine  # noqa: E402
from horreum_amd import abi as _abi  # noqa: E402
_abi.knobs_from_env()  # the A/B scripts' HG_* knobs (the library reads no environment)

NAMES = ["t_spec", "t_agg", "t_lb", "t_end", "n_stride", "n_general", "n_serial", "guess",
         "spins", "count", "flags", "redo", "c_prep", "c_relax", "rounds", "n_short",
         "p_filter", "p_cand", "p_walk", "p_seed", "p_rounds", "p_emit", "p_stage", "p_stride"]
W = len(NAMES)
PIECE = 16384
BATCH_MIN = 16  # hg_decode.hip: at most npieces / BATCH_MIN batches per launch


def n_batches(L):
    return ((L + PIECE - 1) // PIECE + BATCH_MIN - 1) // BATCH_MIN


def run(eng, sst, L, label):
    lib = abi.load_library()
    lib.hgk_decode_launch_diag.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                           ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_void_p]
    lib.hgk_decode_workspace_bytes.argtypes = [ctypes.c_uint64]
    lib.hgk_decode_workspace_bytes.restype = ctypes.c_uint64
    nch = n_batches(L)
    ws = torch.zeros(int(lib.hgk_decode_workspace_bytes(L)), dtype=torch.uint8, device=eng.device)
    cap = L // 16
    spans = eng.empty(cap * 16)
    res = eng.empty(64)
    diag = torch.zeros(nch * W, dtype=torch.int32, device=eng.device)
    stream = torch.cuda.current_stream(eng.device).cuda_stream
    eng.set_stream(torch.cuda.current_stream(eng.device))
    out = {}
    for mode in ("plain", "diag"):
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        times = []
        for _ in range(6):
            ev0.record()
            rc = lib.hgk_decode_launch_diag(
                ctypes.c_void_p(sst.data_ptr()), L, ctypes.c_void_p(spans.data_ptr()), cap,
                ctypes.c_void_p(res.data_ptr()), ctypes.c_void_p(ws.data_ptr()),
                ctypes.c_void_p(diag.data_ptr() if mode == "diag" else 0), ctypes.c_void_p(stream))
            ev1.record()
            torch.cuda.synchronize()
            assert rc == 0
            times.append(ev0.elapsed_time(ev1))
        out[mode + "_ms"] = sorted(times)[len(times) // 2]
    r = res[:24].cpu().numpy()
    out["n"] = int(r[:8].view("<u8")[0])
    out["kind"] = int(r[8:12].view("<i4")[0])
    d = diag.cpu().numpy().astype(np.uint32).reshape(nch, W)
    d = d[d[:, 3] != 0]  # rows of batches that ran (t_end stamped)
    out["batches"] = int(d.shape[0])
    out["label"] = label
    if d.shape[0] == 0:  # the pre-pass resolved the whole table: no general batches ran
        print(json.dumps(out), flush=True)
        return out
    stats = {}
    for i, nm in enumerate(NAMES):
        col = d[:, i].astype(np.float64)
        stats[nm] = {"p10": float(np.percentile(col, 10)), "p50": float(np.median(col)),
                     "p90": float(np.percentile(col, 90)), "max": float(col.max())}
    g = d[:, 7]
    out["guess_have"] = float(((g & 1) != 0).mean())
    out["guess_from_pred"] = float(((g & 2) != 0).mean())
    out["guess_ok"] = float(((g & 4) != 0).mean())
    out["spec_ok"] = float(((d[:, 10] & 8) != 0).mean())
    out["redo"] = float((d[:, 11] != 0).mean())
    pieces = d[:, [4, 5, 6, 15]].sum(axis=0).astype(np.float64)
    out["pieces_stride_general_serial_short"] = (pieces / max(pieces.sum(), 1)).round(4).tolist()
    out["stats"] = stats
    out["label"] = label
    print(json.dumps(out), flush=True)
    return out


def main():
    """Diagnostics for the decode_variants.py workloads whose label contains
    one of the command-line words (all of them without arguments)."""
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from decode_variants import workloads
    only = sys.argv[1:]
    eng = Engine(0)
    for label, sst in workloads(eng.device):
        if only and not any(w in label for w in only):
            continue
        run(eng, sst, sst.numel(), label)
        del sst


if __name__ == "__main__":
    main()
