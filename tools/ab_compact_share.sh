#!/bin/bash
# A/B of the cfg 5 per-GPU share compaction leg (8 x 1 GiB): wall ms per
# variant, alternating (variants as tools/ab_compact.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
for round in 1 2; do for n in "$@"; do
  unset HG_LIBRARY HG_COMPACT_RECORDS
  case $n in base) ;; pairs) export HG_COMPACT_RECORDS=0 ;; records) export HG_COMPACT_RECORDS=1 ;; *) export HG_LIBRARY=build_exp/$n/libhorreum_gpu.so ;; esac
  PER_TABLE=8134407 timeout -k 10 300 python3 tools/compact_leg.py > gpurun_out/cs_$n.log 2>&1 || { tail -5 gpurun_out/cs_$n.log; exit 1; }
  echo "== $n round $round share: $(grep "^{" gpurun_out/cs_$n.log | tail -1 | python3 -c "import json,sys; l=json.loads(sys.stdin.read()); print(l['ms'], l['times_ms'], l['status'])")"
  timeout -k 10 300 python3 tools/compact_leg.py > gpurun_out/cs_s_$n.log 2>&1 || { tail -5 gpurun_out/cs_s_$n.log; exit 1; }
  echo "== $n round $round scaled: $(grep "^{" gpurun_out/cs_s_$n.log | tail -1 | python3 -c "import json,sys; l=json.loads(sys.stdin.read()); print(l['ms'], l['times_ms'], l['status'])")"
done; done
