#!/usr/bin/env python3
"""Summarise tools/pmc_general.sh output into profiles/<tag>_pmc_<shape>.json.

Per shape and kernel: average duration (kernel-trace stats), HBM bytes per
dispatch (FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM for wide streaming
reads, WRITE_SIZE as is; both KiB in rocprofv3) and the median per-dispatch
SQ counters (summed over the rows rocprofv3 writes per dispatch).
Usage: summarize_pmc.py <gpurun_out> <tag> <shape>...
"""
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    return name.split("(")[0].replace("void ", "").strip()


def newest(d, pat):
    files = glob.glob(os.path.join(d, "**", pat), recursive=True)
    return max(files, key=os.path.getmtime) if files else None


def counters(d):
    f = newest(d, "*counter_collection.csv")
    per = defaultdict(float)
    if not f:
        return {}
    for r in csv.DictReader(open(f)):
        per[(short(r["Kernel_Name"]), r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    out = defaultdict(lambda: defaultdict(list))
    for (k, _, c), v in per.items():
        out[k][c].append(v)
    return {k: {c: statistics.median(v) for c, v in cs.items()} for k, cs in out.items()}


def source_stamp():
    """sha256 of the kernel sources and the commit the profile was taken at
    (bench.py compares them with the sources it runs: current_source)."""
    import hashlib
    import subprocess
    sha = {}
    for f in ("hg_decode.hip", "hg_encode.hip", "hg_merge.hip"):
        p = os.path.join(ROOT, "horreum_amd", "csrc", f)
        sha[f] = hashlib.sha256(open(p, "rb").read()).hexdigest() if os.path.exists(p) else None
    try:
        commit = subprocess.run(["git", "-C", ROOT, "rev-parse", "--short", "HEAD"],
                                capture_output=True, text=True).stdout.strip() or None
    except OSError:
        commit = None
    return {"sha256": sha, "commit": commit or os.environ.get("GIT_COMMIT")}


def main():
    out_dir, tag, shapes = sys.argv[1], sys.argv[2], sys.argv[3:]
    for s in shapes:
        res = {"shape": s, "kernels": {}, "_source": source_stamp()}
        st = newest(os.path.join(out_dir, f"{tag}_trace_{s}"), "*kernel_stats.csv")
        if st:
            for r in csv.DictReader(open(st)):
                res["kernels"].setdefault(short(r["Name"]), {})["avg_us"] = \
                    round(float(r["AverageNs"]) / 1e3, 2)
                res["kernels"][short(r["Name"])]["calls"] = int(r["Calls"])
        for part in ("fetch", "write", "sqa", "sqb"):
            for k, cs in counters(os.path.join(out_dir, f"{tag}_{part}_{s}")).items():
                d = res["kernels"].setdefault(k, {})
                for c, v in cs.items():
                    if c == "FETCH_SIZE":
                        d["hbm_read_bytes"] = 2 * v * 1024
                    elif c == "WRITE_SIZE":
                        d["hbm_write_bytes"] = v * 1024
                    else:
                        d[c] = v
        log = os.path.join(out_dir, f"{tag}_trace_{s}.log")
        if os.path.exists(log):
            res["workload"] = [json.loads(x) for x in open(log) if x.startswith("{")]
        path = os.path.join(ROOT, "profiles", f"{tag}_pmc_{s}.json")
        with open(path, "w") as f:
            json.dump(res, f, indent=1)
        print(json.dumps(res))


if __name__ == "__main__":
    main()
