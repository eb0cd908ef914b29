#!/bin/bash
# A/B kernel stats of one decode workload under environment settings:
#   tools/ab_env.sh "HG_X=0" "HG_X=1" ...   (WL=cfg2 by default)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
i=0
for round in 1 2; do for setting in "$@"; do
  i=$((i + 1))
  d=gpurun_out/abenv_${i}
  export $setting
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d \
    -- python3 tools/decode_variants.py ${WL:-cfg2} > $d.log 2>&1 || exit $?
  echo "== $setting round $round: $(grep -o '"ms": [0-9.]*' $d.log | tr '\n' ' ')"
  f=$(find $d -name "*kernel_stats.csv" | head -1)
  python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "hgk" in r["Name"]:
        print(f'  {r["Name"].split("(")[0]:36s} calls={r["Calls"]:>4s} avg_us={float(r["AverageNs"])/1e3:8.2f} min_us={float(r["MinNs"])/1e3:8.2f}')
PY
done; done
