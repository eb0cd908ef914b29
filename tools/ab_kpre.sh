#!/bin/bash
# A/B of compaction-mode key prefixes (HG_COMPACT_KPRE=0: the entry builder
# reads every key line): the cfg 5-scaled and per-GPU-share legs, alternating.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
for round in 1 2; do for k in 1 0; do
  HG_COMPACT_KPRE=$k timeout -k 10 200 python3 tools/compact_leg.py > gpurun_out/abk_$k.log 2>&1 || { tail -3 gpurun_out/abk_$k.log; exit 1; }
  echo "kpre=$k scaled $(grep -o '"ms": [0-9.]*' gpurun_out/abk_$k.log | head -1) $(grep -o '"parity_count_ok": [a-z]*' gpurun_out/abk_$k.log)"
done; done
for k in 1 0; do
  HG_COMPACT_KPRE=$k PER_TABLE=8134407 timeout -k 10 300 python3 tools/compact_leg.py > gpurun_out/abk_share_$k.log 2>&1 || { tail -3 gpurun_out/abk_share_$k.log; exit 1; }
  echo "kpre=$k share $(grep -o '"ms": [0-9.]*' gpurun_out/abk_share_$k.log | head -1) $(grep -o '"parity_[a-z]*_ok": [a-z]*' gpurun_out/abk_share_$k.log | tr '\n' ' ')"
done
