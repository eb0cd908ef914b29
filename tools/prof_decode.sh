#!/bin/bash
# Per-kernel rocprofv3 stats of the cfg2 decode (tools/decode_variants.py cfg2).
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pt -- python3 tools/decode_variants.py ${1:-cfg2} > gpurun_out/pt.log 2>&1 || exit $?
grep workload gpurun_out/pt.log
f=$(find gpurun_out/pt -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "hgk" in r["Name"] or "rocclr" in r["Name"]:
        print(f'{r["Name"].split("(")[0]:40s} calls={r["Calls"]:>5s} avg_us={float(r["AverageNs"])/1e3:9.2f} min_us={float(r["MinNs"])/1e3:9.2f}')
PY
