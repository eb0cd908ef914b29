#!/usr/bin/env python3
"""Time hg_encode_host on BASELINE cfg 3 (10 M pairs, 32 B / 256 B) from
page-locked (torch pin_memory) buffers; median of 3.  HG_ENCODE_HOST_SERIAL=1
selects the upload-all / encode / download-all path."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from horreum_amd import synth  # noqa: E402
from horreum_amd.engine import Engine  # noqa: E402
from horreum_amd import abi as _abi  # noqa: E402
_abi.knobs_from_env()  # the A/B scripts' HG_* knobs (the library reads no environment)


def main():
    eng = Engine(0)
    n, k, v = 10_000_000, 32, 256
    a_d, p_d = synth.fixed_arena(n, k, v, seed=3, device=eng.device)
    total = n * (16 + k + v)
    a_t = torch.empty(a_d.numel(), dtype=torch.uint8).pin_memory()
    a_t.copy_(a_d)
    p_t = torch.empty(p_d.numel(), dtype=torch.uint8).pin_memory()
    p_t.copy_(p_d)
    o_t = torch.empty(total, dtype=torch.uint8).pin_memory()
    ha, hp, ho = a_t.numpy(), p_t.numpy(), o_t.numpy()
    ol = ctypes.c_uint64()

    def vp(x):
        return ctypes.c_void_p(x.ctypes.data)

    def enc():
        rc = eng.lib.hg_encode_host(eng.ctx, vp(ha), ha.size, vp(hp), n, vp(ho), total,
                                    ctypes.c_void_p(0), 0, ctypes.c_void_p(0), ctypes.byref(ol))
        assert rc == 0 and ol.value == total

    enc()
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        enc()
        ts.append(time.perf_counter() - t0)
    ok = bool((o_t[16:16 + k + v] == a_t[:k + v]).all()) and bool(
        (o_t[-(k + v):] == a_t[-(k + v):]).all())
    print(json.dumps({"serial": bool(os.environ.get("HG_ENCODE_HOST_SERIAL")),
                      "ms": round(sorted(ts)[1] * 1e3, 2), "all": [round(x * 1e3, 1) for x in ts],
                      "GiB_s": round(total / sorted(ts)[1] / (1 << 30), 2), "ok": ok}), flush=True)


if __name__ == "__main__":
    main()
