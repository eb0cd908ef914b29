#!/usr/bin/env python3
"""PCIe duplex probe (not part of the product): 1 GiB pinned H2D and 1 GiB
pinned D2H, one after the other vs concurrently on two streams, and the
same in 64 MiB pieces."""
import json
import time

import torch

G = 1 << 30
h_up = torch.empty(G, dtype=torch.uint8).pin_memory()
h_dn = torch.empty(G, dtype=torch.uint8).pin_memory()
d_up = torch.empty(G, dtype=torch.uint8, device="cuda")
d_dn = torch.empty(G, dtype=torch.uint8, device="cuda")
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def t(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return sorted(ts)[reps // 2] * 1e3


def serial():
    d_up.copy_(h_up, non_blocking=True)
    h_dn.copy_(d_dn, non_blocking=True)


def concurrent(piece=G):
    for o in range(0, G, piece):
        with torch.cuda.stream(s1):
            d_up[o:o + piece].copy_(h_up[o:o + piece], non_blocking=True)
        with torch.cuda.stream(s2):
            h_dn[o:o + piece].copy_(d_dn[o:o + piece], non_blocking=True)


out = {"h2d_ms": t(lambda: d_up.copy_(h_up, non_blocking=True)),
       "d2h_ms": t(lambda: h_dn.copy_(d_dn, non_blocking=True)),
       "serial_ms": t(serial), "concurrent_ms": t(concurrent),
       "concurrent_64MiB_pieces_ms": t(lambda: concurrent(64 << 20))}
print(json.dumps({k: round(v, 2) for k, v in out.items()}), flush=True)
