#!/bin/bash
# Round GPU check: parity tests, decode workload timings, diagnostics, bench.
# Every GPU step has its own time limit; a fault/timeout (rc >= 124) stops.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -${TAILN:-6} "gpurun_out/$name.log"
  if [ $rc -ge 124 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
TAILN=4 step pytest_gpu 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider
[ -n "$VARIANTS" ] && step variants 400 python tools/decode_variants.py
[ -n "$DIAG" ] && step diag 300 python tools/decode_diag.py
step bench 400 python bench.py
