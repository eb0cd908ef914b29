#!/bin/bash
# Pre-pass batch size A/B (knob HG_DECODE_SBP via the environment, forwarded by
# tools/decode_variants.py) on the lane-walk shapes: default, 8 and 32 pieces.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
for r in 1 2; do for v in 0 8 32; do
  if [ $v = 0 ]; then unset HG_DECODE_SBP; else export HG_DECODE_SBP=$v; fi
  timeout -k 10 300 python3 tools/decode_variants.py small medium zero > gpurun_out/sbp_$v.log 2>&1 || { tail -3 gpurun_out/sbp_$v.log; exit 1; }
  echo "== sbp=$v round $r"; grep -o '"workload": "[^"]*".*"b2b_ms": [0-9.]*' gpurun_out/sbp_$v.log | sed 's/"bytes.*"ms"/ms/'
  grep -c '"parity": true' gpurun_out/sbp_$v.log
done; done
