#!/bin/bash
# FETCH_SIZE / WRITE_SIZE (separate --pmc passes) of the bench's extra legs;
# prints per-kernel medians (KiB per launch) for kernels matching KERN.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  d=gpurun_out/pmc_legs_$c; rm -rf $d
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $d -- python3 bench.py --steps 2 \
    --warmup 1 --cpu-sample-mb 0 --no-encode --no-host > $d.log 2>&1 || exit $?
  f=$(find $d -name "*counter_collection.csv" | head -1)
  python3 - "$f" "$c" "${KERN:-hg}" <<'PY'
import csv, sys, statistics, collections
v = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if sys.argv[3] in r["Kernel_Name"]:
        v[(r["Kernel_Name"].split("(")[0], r["Dispatch_Id"])].append(float(r["Counter_Value"]))
per = collections.defaultdict(list)
for (k, _), xs in v.items():
    per[k].append(sum(xs))
for k, xs in per.items():
    print(f"{sys.argv[2]:10s} {k[:40]:40s} n={len(xs):3d} median_KiB={statistics.median(xs):12.0f}")
PY
done
