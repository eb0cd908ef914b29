#!/usr/bin/env python3
"""Per-call timeline of the decode launches in a rocprofv3 kernel trace:
for each decode_spec_kernel, its duration, the gap to the next hg kernel on
the queue, that kernel's duration, and the span from the first op of the
call (any op since the previous call's last hg kernel) to the last.
Usage: trace_gaps.py <kernel_trace.csv> [N: also print the ops around call N]"""
import csv
import sys

rows = []
for r in csv.DictReader(open(sys.argv[1])):
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0],
                 r.get("Grid_Size_X") or r.get("Grid_Size")))
rows.sort()
calls = []
for i, (s, e, n, g) in enumerate(rows):
    if "decode_spec_kernel" not in n:
        continue
    nxt = rows[i + 1] if i + 1 < len(rows) else None
    prev = rows[i - 1] if i else None
    calls.append({
        "grid": g,
        "spec_us": (e - s) / 1e3,
        "prev": prev[2][-28:] if prev else None,
        "gap_before_us": (s - prev[1]) / 1e3 if prev else None,
        "gap_us": (nxt[0] - e) / 1e3 if nxt else None,
        "next": nxt[2][-28:] if nxt else None,
        "next_us": (nxt[1] - nxt[0]) / 1e3 if nxt else None,
    })
by = {}
for c in calls:
    by.setdefault(c["grid"], []).append(c)
if len(sys.argv) > 2:  # print the ops around call N of the first grid
    n = int(sys.argv[2])
    idx = [i for i, r in enumerate(rows) if "decode_spec_kernel" in r[2]]
    i = idx[min(n, len(idx) - 1)]
    t0 = rows[i][0]
    for s, e, nm, g in rows[max(0, i - 4):i + 6]:
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {nm[-40:]} grid {g}")
for g, cs in by.items():
    cs = cs[2:] or cs  # skip warm-up calls
    med = lambda k: sorted(x[k] for x in cs if x[k] is not None)[len(cs) // 2]
    print(f"grid {g}: calls {len(cs)} spec {med('spec_us'):.1f} us, gap {med('gap_us'):.1f}, "
          f"next {cs[0]['next']} {med('next_us'):.1f} us, before: {cs[0]['prev']} gap {med('gap_before_us'):.1f}")
