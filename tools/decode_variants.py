#!/usr/bin/env python3
"""A/B the decode kernel geometries (bytes per workgroup) in one process.

For each workload, every variant is run interleaved (rounds x variants) and
the median launch time is reported, with a parity check of every run's
result against the 16 KiB variant's spans (bit-exact)."""
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

VARIANTS = [4096, 8192, 16384]


def workloads(dev):
    n = 8_134_407
    yield "cfg2 16B/100B 1GiB", synth.fixed_sst(n, 16, 100, seed=2, device=dev)
    rng = np.random.default_rng(4)
    for label, m, kr, vr in [("mixed 16B/8..4096B", 400_000, (16, 17), (8, 4097)),
                             ("small mixed 0..24B/0..64B", 4_000_000, (0, 24), (0, 64))]:
        kl = rng.integers(*kr, m)
        vl = rng.integers(*vr, m)
        vl[rng.random(m) < 0.05] = 0
        offs = np.concatenate([[0], np.cumsum(16 + kl + vl)])
        buf = rng.integers(0, 256, int(offs[-1]), dtype=np.uint8)
        hdr = np.stack([kl, vl], axis=1).astype("<u8").view(np.uint8).reshape(m, 16)
        for i in range(16):
            buf[offs[:-1] + i] = hdr[:, i]
        yield label, torch.from_numpy(buf).to(dev)


def main():
    lib = abi.load_library()
    f = lib.hgk_decode_launch_variant
    f.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                  ctypes.c_void_p]
    lib.hgk_decode_workspace_bytes.argtypes = [ctypes.c_uint64]
    lib.hgk_decode_workspace_bytes.restype = ctypes.c_uint64
    eng = Engine(0)
    stream = torch.cuda.current_stream(eng.device).cuda_stream
    for label, sst in workloads(eng.device):
        L = sst.numel()
        cap = L // 16
        ws = torch.zeros(int(lib.hgk_decode_workspace_bytes(L)), dtype=torch.uint8,
                         device=eng.device)
        spans = {c: eng.empty(cap * 16) for c in VARIANTS}
        res = {c: eng.empty(64) for c in VARIANTS}
        times = {c: [] for c in VARIANTS}
        for rnd in range(8):
            for c in VARIANTS:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                rc = f(ctypes.c_void_p(sst.data_ptr()), L, ctypes.c_void_p(spans[c].data_ptr()),
                       cap, ctypes.c_void_p(res[c].data_ptr()), ctypes.c_void_p(ws.data_ptr()),
                       None, c, ctypes.c_void_p(stream))
                e1.record()
                torch.cuda.synchronize()
                assert rc == 0
                if rnd > 0:
                    times[c].append(e0.elapsed_time(e1))
        out = {"workload": label, "bytes": L}
        ref = None
        for c in VARIANTS[::-1]:
            r = res[c][:24].cpu().numpy()
            n = int(r[:8].view("<u8")[0])
            kind = int(r[8:12].view("<i4")[0])
            sp = spans[c][: n * 16]
            if ref is None:
                ref = (n, kind, sp)
            same = (n, kind) == ref[:2] and torch.equal(sp, ref[2])
            ms = float(np.median(times[c]))
            out[str(c)] = {"ms": round(ms, 4), "GBps": round(L / ms / 1e6, 1), "n": n,
                           "kind": kind, "same_as_16k": bool(same)}
        print(json.dumps(out), flush=True)
        del sst, spans


if __name__ == "__main__":
    main()
