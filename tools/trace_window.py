#!/usr/bin/env python3
"""Ops of a rocprofv3 trace in time order (kernel trace, plus the memory-copy
trace when given): start relative to the first op of the window, duration,
gap since the previous op's end.  Usage:
  trace_window.py <kernel_trace.csv> [memory_copy_trace.csv] --around NAME --nth N --span K
prints K ops starting at the N-th launch of the kernel whose name contains NAME."""
import argparse
import csv

ap = argparse.ArgumentParser()
ap.add_argument("files", nargs="+")
ap.add_argument("--around", default="decode_spec")
ap.add_argument("--nth", type=int, default=4)
ap.add_argument("--span", type=int, default=12)
ap.add_argument("--before", type=int, default=3)
args = ap.parse_args()
rows = []
for f in args.files:
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name") or (f"copy {r.get('Direction', '')} {r.get('Size', r.get('Bytes', ''))}")
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name.split("(")[0]))
rows.sort()
hits = [i for i, r in enumerate(rows) if args.around in r[2]]
i0 = max(0, hits[min(args.nth, len(hits) - 1)] - args.before)
t0, prev_end = rows[i0][0], None
for s, e, n in rows[i0:i0 + args.span]:
    gap = "" if prev_end is None else f"gap {(s - prev_end) / 1e3:7.1f}"
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {gap:12s} {n[-60:]}")
    prev_end = e if prev_end is None else max(prev_end, e)
