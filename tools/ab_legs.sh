#!/bin/bash
# A/B kernel stats of the bench's extra legs (cfg4 batched decode, cfg5-scaled
# compaction) for experimental builds: tools/ab_legs.sh NAME...
# (build_exp/NAME/libhorreum_gpu.so via HG_LIBRARY; KERN filters the kernels shown)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
for round in 1 2; do for n in "$@"; do
  d=gpurun_out/legs_${n}_$round
  rm -rf $d
  HG_LIBRARY=build_exp/$n/libhorreum_gpu.so timeout -k 10 300 rocprofv3 --kernel-trace --stats \
    --output-format csv -d $d -- python3 bench.py --steps 4 --warmup 1 --cpu-sample-mb 0 \
    --no-encode --no-host > $d.log 2>&1 || exit $?
  echo "== $n round $round: $(python3 -c "import json,sys; l=json.loads(open('$d.log').read().strip().splitlines()[-1]); x=l['extra']; print({k: x[k].get('ms_per_step', x[k]) for k in x})")"
  f=$(find $d -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "${KERN:-hg}" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if sys.argv[2] in r["Name"]:
        print(f'  {r["Name"].split("(")[0][:40]:40s} calls={r["Calls"]:>4s} avg_us={float(r["AverageNs"])/1e3:8.2f} min_us={float(r["MinNs"])/1e3:8.2f}')
PY
done; done
