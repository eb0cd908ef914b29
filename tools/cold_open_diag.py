#!/usr/bin/env python3
"""Where the cold open of 32 cfg 4 table files goes (bench
multi_table_decode_cfg4.cold_open): mmap, hg_host_register, the batched
decode, the block indexes -- timed one step at a time."""
import json
import os
import shutil
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from horreum_amd import synth  # noqa: E402
from horreum_amd.engine import Engine  # noqa: E402
from horreum_amd.index import Index  # noqa: E402
from horreum_amd.table import PersistedFile  # noqa: E402
from horreum_amd import abi as _abi  # noqa: E402
_abi.knobs_from_env()  # the A/B scripts' HG_* knobs (the library reads no environment)


def main():
    eng = Engine(0)
    dev = eng.device
    d = tempfile.mkdtemp(prefix="hg_cold_diag_")
    try:
        for t in range(32):
            v = synth.mixed_table_vlens(64 << 20, 8, 4096, 0.05, seed=4 + t)
            keys = np.arange(v.size, dtype=np.uint64) * 7 + t
            buf, _ = synth.keyed_table(keys, v, seed=4 + t, device=dev)
            buf.cpu().numpy().tofile(os.path.join(d, f"table_{t:03d}"))
        torch.cuda.synchronize()
        for rep in range(3):
            out = {}
            t0 = time.perf_counter()
            paths = sorted(os.path.join(d, f) for f in os.listdir(d))
            files = [PersistedFile.open(p) for p in paths]
            t1 = time.perf_counter()
            datas = [f.read_bytes(eng) for f in files]
            t2 = time.perf_counter()
            outs = eng.decode_many_host(datas)
            t3 = time.perf_counter()
            idx = [Index.from_spans(dd, o.spans, 64) for dd, o in zip(datas, outs)]
            t4 = time.perf_counter()
            out.update(rep=rep, list_open_ms=round((t1 - t0) * 1e3, 2),
                       mmap_register_ms=round((t2 - t1) * 1e3, 2),
                       decode_many_host_ms=round((t3 - t2) * 1e3, 2),
                       index_ms=round((t4 - t3) * 1e3, 2), blocks=sum(len(i.items) for i in idx))
            for f in files:
                f.unmap()
            print(json.dumps(out), flush=True)
    finally:
        shutil.rmtree(d, ignore_errors=True)


if __name__ == "__main__":
    main()
