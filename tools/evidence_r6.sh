#!/bin/bash
# Round 6 evidence (GPU box), every pass at the final sources and each its own
# run (no counter pass shares a run with tracing):
#   smoke, the GPU tests, the bench (its JSON line),
#   the headline's kernel stats and FETCH / WRITE passes (tools/profile.sh),
#   per-shape decode PMC (tools/pmc_general.sh),
#   the compaction legs' trace + PMC, 8 x 1 M and 8 x 1 GiB (tools/pmc_compaction.sh),
#   the encode's trace / FETCH / WRITE / SQ passes and the copy probe.
# Stops at the first failing step; summaries are made on the CPU side
# (tools/summarize_*.py) into profiles/r6_*.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r6}
run() {  # run <name> <seconds> <args...>
  local name=$1 secs=$2; shift 2
  timeout -s KILL "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
[ -z "$SKIP_TESTS" ] && { TAG=$T bash tools/run.sh smoke tests || exit 1; }
[ -z "$SKIP_BENCH" ] && { TAG=$T bash tools/run.sh bench || exit 1; }
[ -z "$SKIP_PROF" ] && { TAG=$T STEPS=20 bash tools/profile.sh || exit 1; }
[ -z "$SKIP_GENERAL" ] && { TAG=$T SHAPES="small medium midlarge zsmall zmidlarge" bash tools/pmc_general.sh || exit 1; }
if [ -z "$SKIP_COMPACT" ]; then
  TAG=$T bash tools/pmc_compaction.sh || exit 1
  PER_TABLE=8134407 T_TRACE=400 T_PMC=300 TAG=${T}share bash tools/pmc_compaction.sh || exit 1
fi
if [ -z "$SKIP_ENCODE" ]; then
  run ${T}_enc_trace 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_enc_trace -- python3 tools/encode_variants.py
  run ${T}_enc_fetch 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${T}_enc_fetch -- python3 tools/encode_variants.py
  run ${T}_enc_write 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${T}_enc_write -- python3 tools/encode_variants.py
  run ${T}_enc_sq 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d gpurun_out/${T}_enc_sq -- python3 tools/encode_variants.py
  run ${T}_copy_probe 120 ./tools/probes/copy_probe
fi
