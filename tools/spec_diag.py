#!/usr/bin/env python3
"""Pre-pass diagnostics: how each decode_spec_kernel batch went (SpecBatch.pad:
1 stride, 2 stride broke, 3 hop: small records, 4 hop: unreadable record,
5 hop ok, 6 lane walks ok, 7 lane walks: unresolved) and the resolved prefix, for the decode_variants workloads."""
import ctypes
import os
import sys
from collections import Counter

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from decode_variants import workloads as _workloads  # noqa: E402
from horreum_amd import synth  # noqa: E402
from horreum_amd.engine import Engine  # noqa: E402
from horreum_amd import abi as _abi  # noqa: E402
_abi.knobs_from_env()  # the A/B scripts' HG_* knobs (the library reads no environment)


def workloads(dev):
    yield from _workloads(dev)
    # BASELINE cfg-4 tables (64 MiB, keyed, 8..4096 B values): two, or
    # CFG4_TABLES of them (with HG_DECODE_BP=64 HG_DECODE_SBP=64 each single-table
    # decode has the batched decode's geometry for cfg 4's 32 tables per GPU)
    for t in range(int(os.environ.get("CFG4_TABLES", "2"))):
        v = synth.mixed_table_vlens(64 << 20, 8, 4096, 0.05, seed=4 + t)
        keys = np.arange(v.size, dtype=np.uint64) * 7 + t
        buf, _ = synth.keyed_table(keys, v, seed=4 + t, device=dev)
        yield f"cfg4 table {t}", buf

SB = np.dtype([("x0", "<u8"), ("exit", "<u8"), ("count", "<u4"), ("ok", "<u4"), ("pad", "<u8")])


def main():
    args = [x for x in sys.argv[1:] if not x.startswith("--")]
    only = args[0] if args else None
    eng = Engine(0)
    lib = eng.lib
    lib.hgk_ctx_workspace.restype = ctypes.c_void_p
    lib.hgk_ctx_workspace.argtypes = [ctypes.c_void_p]
    lib.hgk_debug_d2h.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
    for label, sst in workloads(eng.device):
        if only and only not in label:
            continue
        L = sst.numel()
        out = eng.decode_dev(sst, L)
        lay = (ctypes.c_uint64 * 8)()
        lib.hgk_decode_last_layout(lay)
        sb_off, sp_off, nspec, sbp, bp, nb, st_off = list(lay)[:7]
        ws = lib.hgk_ctx_workspace(eng.ctx)
        sb = np.zeros(nspec, SB)
        lib.hgk_debug_d2h(sb.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(ws + sb_off),
                          sb.nbytes)
        ctl = np.zeros(4, np.uint32)  # the last call's control region (one of two in turn)
        lib.hgk_ctx_decode_ctl.restype = ctypes.c_void_p
        lib.hgk_ctx_decode_ctl.argtypes = [ctypes.c_void_p]
        lib.hgk_debug_d2h(ctl.ctypes.data_as(ctypes.c_void_p),
                          ctypes.c_void_p(lib.hgk_ctx_decode_ctl(eng.ctx)), 16)
        fb = nspec - int(ctl[1])
        codes = Counter(int(c) & 0xFF for c in sb["pad"])
        why = Counter((int(c) >> 8) & 0xFF for c in sb["pad"] if (int(c) >> 8) & 0xFF)
        links = int(np.sum(sb["x0"][1:] != sb["exit"][:-1]))
        print(f"{label}: n={out.n} kind={out.kind} nspec={nspec} sbp={sbp} bp={bp} "
              f"first_bad={fb} codes={dict(sorted(codes.items()))} dead_why={dict(why)} link_mismatch={links} "
              f"ok={int(sb['ok'].sum())} lw_serial={int((sb['pad'] >> 32).sum())} repairs={int(ctl[3])}", flush=True)
        if "--truth" in sys.argv:  # are the guessed entries / exits true record starts?
            from oracle import oracle
            starts = oracle.decode(sst.cpu().numpy())[0]["off"]
            okm = sb["ok"] != 0
            x_in = np.isin(sb["x0"][okm], starts) | (sb["x0"][okm] == L)
            e_in = np.isin(sb["exit"][okm], starts) | (sb["exit"][okm] == L)
            print(f"   ok batches {int(okm.sum())}: entry true {int(x_in.sum())}, exit true {int(e_in.sum())}")
        bad = np.nonzero(sb["x0"][1:] != sb["exit"][:-1])[0][:5]
        for j in bad:
            print(f"   link {j}->{j+1}: exit {sb['exit'][j]} x0 {sb['x0'][j+1]} "
                  f"codes {sb['pad'][j]},{sb['pad'][j+1]}")
        del sst


if __name__ == "__main__":
    main()
