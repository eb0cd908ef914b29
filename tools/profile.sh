#!/bin/bash
# rocprofv3 evidence for the bench's kernels (run on the GPU box):
#  1. kernel trace + stats of a bench run (per-kernel average durations);
#  2. FETCH_SIZE and WRITE_SIZE in separate --pmc passes (no other tracing).
# Output: gpurun_out/prof_*; summarised by tools/summarize_prof.py.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
# Headline passes run the cfg2 decode leg alone, so per-kernel averages and
# PMC medians are of that workload only; one more trace covers every leg.
BENCH="bench.py --steps ${STEPS:-20} --warmup 5 --cpu-sample-mb 0 --no-encode --no-extra --no-host"
run() {  # run <name> <seconds> <args...>
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
run prof_trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_trace -- python3 $BENCH
run prof_fetch 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch -- python3 bench.py --steps 5 --warmup 2 --cpu-sample-mb 0 --no-encode --no-extra --no-host
run prof_write 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write -- python3 bench.py --steps 5 --warmup 2 --cpu-sample-mb 0 --no-encode --no-extra --no-host
run prof_legs 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_legs -- python3 bench.py --steps 5 --warmup 2 --cpu-sample-mb 0
python3 tools/summarize_prof.py gpurun_out "${TAG:-r1}" > gpurun_out/prof_summary.log 2>&1; tail -20 gpurun_out/prof_summary.log
