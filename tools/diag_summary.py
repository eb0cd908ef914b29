#!/usr/bin/env python3
"""Condense gpurun_out/diag.log (tools/decode_diag.py output) to p50 phase costs."""
import json
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/diag.log"
for line in open(path):
    if not line.startswith("{"):
        continue
    d = json.loads(line)
    st = d.pop("stats")
    print(d["label"], "plain_ms", round(d["plain_ms"], 4), "guess_ok", round(d["guess_ok"], 4),
          "redo", round(d["redo"], 4), d.get("pieces_stride_general_serial_short"))
    print("   ", {k: v["p50"] for k, v in st.items()})
