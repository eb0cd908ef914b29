#!/usr/bin/env python3
"""Which host mappings can hg_host_register page-lock for direct DMA?
Tries a file mmap (copy-on-write, shared read-only), an anonymous mmap
filled by readinto, and numpy memory; registers, decodes through
hg_decode_host, and prints what worked."""
import mmap
import os
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from horreum_amd.engine import Engine  # noqa: E402
from oracle import oracle  # noqa: E402
from tests import corpus  # noqa: E402

eng = Engine(0)
_, _, data, _ = corpus.make("mixed_small")
want = oracle.decode(data)[0]
for size in tuple(int(x) for x in sys.argv[1:]) or (data.size,):
    d = data[:size]
    path = os.path.join(tempfile.mkdtemp(), "t")
    open(path, "wb").write(d.tobytes())
    for mode in ("file_copy", "file_shared_read", "anon_readinto", "numpy"):
        try:
            with open(path, "rb") as fh:
                if mode == "file_copy":
                    mm = mmap.mmap(fh.fileno(), size, access=mmap.ACCESS_COPY)
                    arr = np.frombuffer(mm, np.uint8)
                elif mode == "file_shared_read":
                    mm = mmap.mmap(fh.fileno(), size, access=mmap.ACCESS_READ)
                    arr = np.frombuffer(mm, np.uint8)
                elif mode == "anon_readinto":
                    mm = mmap.mmap(-1, (size + 4095) // 4096 * 4096)
                    arr = np.frombuffer(mm, np.uint8)[:size]
                    fh.readinto(memoryview(arr))
                else:
                    mm = None
                    arr = np.fromfile(fh, np.uint8)
            reg = "ok"
            try:
                eng.host_register(arr)
            except Exception as e:  # noqa: BLE001
                reg = repr(e)[:80]
            pinned = eng.host_is_pinned(arr)
            try:
                out = eng.decode_host(arr)
                dec = "ok" if out.kind == 0 else f"kind {out.kind}"
            except Exception as e:  # noqa: BLE001
                dec = repr(e)[:80]
            print(f"size {size} {mode:18s} register={reg} pinned={pinned} decode={dec}", flush=True)
            if reg == "ok":
                eng.host_unregister(arr)
        except Exception as e:  # noqa: BLE001
            print(f"size {size} {mode:18s} FAILED {e!r}"[:160], flush=True)
