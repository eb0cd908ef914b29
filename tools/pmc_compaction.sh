#!/bin/bash
# rocprofv3 evidence for the cfg 5-scaled compaction leg (run on the GPU box):
# kernel trace + stats, FETCH_SIZE and WRITE_SIZE, each pass its own run of
# tools/compact_leg.py (4 leg calls: 1 warm-up + 3 timed).  Summarised here
# by tools/summarize_compaction.py into profiles/<TAG>_pmc_compaction.json.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${TAG:-r2}
run() {  # run <name> <seconds> <args...>
  local name=$1 secs=$2; shift 2
  timeout -s KILL "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
rm -rf gpurun_out/${TAG}_ctrace gpurun_out/${TAG}_cfetch gpurun_out/${TAG}_cwrite
run ${TAG}_ctrace ${T_TRACE:-200} rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_ctrace -- python3 tools/compact_leg.py
run ${TAG}_cfetch ${T_PMC:-120} rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_cfetch -- python3 tools/compact_leg.py
run ${TAG}_cwrite ${T_PMC:-120} rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_cwrite -- python3 tools/compact_leg.py
