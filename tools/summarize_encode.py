#!/usr/bin/env python3
"""Summarise the encode evidence passes of tools/evidence_r5a.sh (ENCODE_PMC=1:
gpurun_out/<tag>_enc_{trace,fetch,write,sq}/, each its own run of
tools/encode_variants.py) into profiles/<tag>_pmc_encode.json: per kernel and
grid (the grid names the workload), dispatches, average duration, HBM bytes
per dispatch (FETCH_SIZE doubled per MI355X_MICROARCH.md's gfx950 note, KB ->
bytes; WRITE_SIZE KB -> bytes) and the SQ counters per dispatch.

Usage: summarize_encode.py <gpurun_out> <tag>"""
import csv
import glob
import hashlib
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKLOADS = {2000128: "mixed 2M shuffled", 10000128: "cfg3 10M 32B/256B"}


def rows(d, name):
    out = []
    for f in sorted(glob.glob(os.path.join(d, "**", name), recursive=True)):
        with open(f, newline="") as fh:
            out.extend(csv.DictReader(fh))
    return out


def key(name, grid):
    return f"{name.split('(')[0]} grid={grid}"


def ours(name):
    return "hgk::" in name


def main():
    out_dir, tag = sys.argv[1], sys.argv[2]
    base = os.path.join(out_dir, f"{tag}_enc_")
    kern = {}
    durs = defaultdict(list)
    for r in rows(base + "trace", "*kernel_trace.csv"):
        if not ours(r["Kernel_Name"]):
            continue
        k = key(r["Kernel_Name"], int(r["Grid_Size_X"]))
        durs[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k, v in durs.items():
        grid = int(k.rsplit("=", 1)[1])
        kern[k] = {"workload": WORKLOADS.get(grid, "?"), "grid": grid, "dispatches": len(v),
                   "avg_us": round(sum(v) / len(v), 2)}
    ctr = defaultdict(lambda: defaultdict(list))
    for sub in ("fetch", "write", "sq"):
        for r in rows(base + sub, "*counter_collection.csv"):
            if not ours(r["Kernel_Name"]):
                continue
            k = key(r["Kernel_Name"], int(r["Grid_Size"]))
            ctr[k][(r["Dispatch_Id"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    for k, per in ctr.items():
        acc = defaultdict(list)
        for (_, cname), vals in per.items():
            acc[cname].append(sum(vals))  # (a counter's instances summed per dispatch)
        e = kern.setdefault(k, {"grid": int(k.rsplit("=", 1)[1])})
        for cname, vals in sorted(acc.items()):
            avg = sum(vals) / len(vals)
            if cname == "FETCH_SIZE":
                e["hbm_read_bytes"] = int(round(2 * avg * 1024))
            elif cname == "WRITE_SIZE":
                e["hbm_write_bytes"] = int(round(avg * 1024))
            else:
                e[cname] = int(round(avg))
    src = os.path.join(ROOT, "horreum_amd", "csrc", "hg_encode.hip")
    doc = {
        "tag": tag,
        "what": "encode (tools/encode_variants.py): rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE / "
                "SQ passes, each its own run; FETCH_SIZE doubled per the MI355X guide (gfx950), "
                "KB units -> bytes",
        "kernels": dict(sorted(kern.items())),
        "_source": {"sha256": {"hg_encode.hip": hashlib.sha256(open(src, "rb").read()).hexdigest()}},
        "cfg3_algorithmic_bytes": 6160000000,
    }
    path = os.path.join(ROOT, "profiles", f"{tag}_pmc_encode.json")
    with open(path, "w") as f:
        json.dump(doc, f, indent=1)
    print(path)
    for k, e in doc["kernels"].items():
        print(k, e.get("avg_us"), e.get("hbm_read_bytes"), e.get("hbm_write_bytes"))


if __name__ == "__main__":
    main()
