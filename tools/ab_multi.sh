#!/bin/bash
# A/B of the batched multi-table decode (cfg 4, tools/multi_table.py) and the
# cfg 5 compaction leg (tools/compact_leg.py) between the in-tree library
# ("base") and build_exp/NAME libraries, alternating, ROUNDS rounds.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
for round in $(seq 1 ${ROUNDS:-2}); do for n in "$@"; do
  if [ "$n" = base ]; then unset HG_LIBRARY; else export HG_LIBRARY=$PWD/build_exp/$n/libhorreum_gpu.so; fi
  timeout -k 10 200 python3 tools/multi_table.py > gpurun_out/abm_$n.log 2>&1 || { tail -3 gpurun_out/abm_$n.log; exit 1; }
  timeout -k 10 200 python3 tools/compact_leg.py > gpurun_out/abc_$n.log 2>&1 || { tail -3 gpurun_out/abc_$n.log; exit 1; }
  echo "== $n round $round: cfg4 $(grep '^{' gpurun_out/abm_$n.log | tail -1 | python3 -c 'import json,sys; l=json.loads(sys.stdin.read()); print(l["ms"], "b2b", l["b2b_ms"], l.get("parity"))') compact $(grep '^{' gpurun_out/abc_$n.log | tail -1 | python3 -c 'import json,sys; l=json.loads(sys.stdin.read()); print(l["ms"], l["status"])')"
done; done
