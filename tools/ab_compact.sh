#!/bin/bash
# A/B of the cfg 5-scaled compaction leg: kernel stats per variant.
# Variants: base (in-tree library), kway (HG_MERGE_KWAY=1: the one-pass k-way merge),
# noprebuild (HG_COMPACT_PREBUILD=0: merge entries built after the host has the counts),
# encpairs, nokent, or a build_exp/NAME.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
for round in 1 2; do for n in "$@"; do
  d=gpurun_out/cl_${n}_$round; rm -rf $d
  unset HG_LIBRARY HG_MERGE_KWAY HG_COMPACT_ENCODE HG_MERGE_KENT HG_COMPACT_PREBUILD HG_COMPACT_RECORDS
  case $n in base) ;; pairs) export HG_COMPACT_RECORDS=0 ;; kway) export HG_MERGE_KWAY=1 ;; noprebuild) export HG_COMPACT_PREBUILD=0 ;; encpairs) export HG_COMPACT_ENCODE=pairs ;; nokent) export HG_MERGE_KENT=0 ;; *) export HG_LIBRARY=build_exp/$n/libhorreum_gpu.so ;; esac
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $d -- python3 tools/compact_leg.py > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  echo "== $n round $round: $(grep "^{" $d.log | tail -1 | python3 -c "import json,sys; l=json.loads(sys.stdin.read()); print(l['ms'], l['status'], l.get('merged_records'))")"
  f=$(find $d -name "*kernel_stats.csv" | head -1)
  python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "hg" in r["Name"]:
        print(f'  {r["Name"].split("(")[0][:44]:44s} calls={r["Calls"]:>4s} avg_us={float(r["AverageNs"])/1e3:8.2f}')
PY
done; done
