#!/usr/bin/env python3
"""Summarise tools/pmc_compaction.sh output (gpurun_out/<tag>_c*) into
profiles/<tag>_pmc_compaction.json: per kernel of the compaction leg, the
average duration and HBM bytes per leg call (FETCH_SIZE doubled per
MI355X_MICROARCH.md's gfx950 note -- exact for wide coalesced streaming reads,
an upper bound for the merge's 16-byte gathers -- WRITE_SIZE as is), and the
totals against the leg's algorithmic bytes.

Usage: summarize_compaction.py <gpurun_out> <tag>"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CALLS = 4  # tools/compact_leg.py: one warm-up + three timed leg calls
OURS = ("hgk::", "hgm::", "void hgk::", "void hgm::")


def short(name):
    return name.split("(")[0].replace("void ", "")


def newest_run(files):
    """The files of the newest rocprofv3 run among `files` (gpurun_out/ keeps
    earlier runs' <pid>_*.csv next to the new ones)."""
    if not files:
        return []
    top = max(files, key=os.path.getmtime)
    pid = os.path.basename(top).split("_")[0]
    return [f for f in files if os.path.dirname(f) == os.path.dirname(top)
            and os.path.basename(f).split("_")[0] == pid]


def main():
    out, tag = sys.argv[1], sys.argv[2]
    dest = sys.argv[3] if len(sys.argv) > 3 else f"{tag}_pmc_compaction.json"
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from summarize_pmc import source_stamp
    res = {"tag": tag, "calls_per_run": CALLS, "kernels": {}, "_source": source_stamp()}
    stats = newest_run(glob.glob(os.path.join(out, f"{tag}_ctrace", "**", "*kernel_stats.csv"),
                                 recursive=True))
    for r in csv.DictReader(open(stats[0])):
        if not r["Name"].startswith(OURS):
            continue
        k = res["kernels"].setdefault(short(r["Name"]), {})
        k["avg_us"] = round(float(r["AverageNs"]) / 1e3, 2)
        k["dispatches_per_call"] = int(r["Calls"]) // CALLS
    # the three timed calls alone (the warm-up call's first dispatches pay
    # first-use costs: decode_multi 131 us there against 26 us after)
    trace = newest_run(glob.glob(os.path.join(out, f"{tag}_ctrace", "**", "*kernel_trace.csv"),
                                 recursive=True))
    durs = defaultdict(list)
    for r in (csv.DictReader(open(trace[0])) if trace else []):
        if r["Kernel_Name"].startswith(OURS):
            durs[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for name, d in durs.items():
        per = len(d) // CALLS
        if name in res["kernels"] and per:
            res["kernels"][name]["timed_avg_us"] = round(sum(d[per:]) / len(d[per:]), 2)
    for cnt, sub, scale, key in (("FETCH_SIZE", "cfetch", 2.0, "hbm_read_bytes"),
                                 ("WRITE_SIZE", "cwrite", 1.0, "hbm_write_bytes")):
        tot = defaultdict(float)
        for f in newest_run(glob.glob(os.path.join(out, f"{tag}_{sub}", "**",
                                                "*counter_collection.csv"), recursive=True)):
            for r in csv.DictReader(open(f)):
                if r["Counter_Name"] == cnt and r["Kernel_Name"].startswith(OURS):
                    tot[short(r["Kernel_Name"])] += float(r["Counter_Value"]) * 1024 * scale
        for k, v in tot.items():
            res["kernels"].setdefault(k, {})[key] = round(v / CALLS)
    rd = sum(k.get("hbm_read_bytes", 0) for k in res["kernels"].values())
    wr = sum(k.get("hbm_write_bytes", 0) for k in res["kernels"].values())
    log = os.path.join(out, f"{tag}_ctrace.log")
    leg = [json.loads(x) for x in open(log) if x.startswith("{")] if os.path.exists(log) else []
    if leg:
        L, O, n = leg[-1]["input_bytes_per_gpu"], leg[-1]["merged_bytes"], leg[-1]["merged_records"]
        # read the tables, write the compacted table; spans (16 B per input
        # record) and pairs (24 B per output record) each written and read once
        nin = leg[-1]["input_records"]
        alg = L + O + 2 * 16 * nin + 2 * 24 * n
        res["algorithmic_bytes"] = alg
        res["algorithmic_note"] = "tables + output + 2 x spans + 2 x pairs"
        res["leg"] = leg[-1]
    res["traffic_bytes_per_call"] = rd + wr
    if res.get("algorithmic_bytes"):
        res["traffic_over_algorithmic"] = round((rd + wr) / res["algorithmic_bytes"], 3)
    path = os.path.join(ROOT, "profiles", dest)
    with open(path, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
