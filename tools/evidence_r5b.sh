#!/bin/bash
# Round 5 evidence, call B (GPU box): the GPU tests, the bench, then the
# rocprofv3 evidence at the current sources -- the headline's kernel stats and
# FETCH/WRITE passes (tools/profile.sh), per-shape decode PMC
# (tools/pmc_general.sh) and the compaction legs (tools/pmc_compaction.sh);
# summarised on the CPU side into profiles/ (tools/summarize_*.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r5}
[ -z "$SKIP_TESTS" ] && { TAG=$T tools/run.sh smoke tests || exit 1; }
[ -z "$SKIP_BENCH" ] && { TAG=$T tools/run.sh bench || exit 1; }
TAG=$T STEPS=20 bash tools/profile.sh || exit 1
TAG=$T SHAPES="small medium midlarge zsmall zmidlarge" bash tools/pmc_general.sh || exit 1
TAG=$T bash tools/pmc_compaction.sh || exit 1
PER_TABLE=8134407 T_TRACE=400 T_PMC=300 TAG=${T}share bash tools/pmc_compaction.sh || exit 1
