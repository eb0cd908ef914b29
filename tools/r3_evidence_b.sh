# Round-3 evidence, part B (GPU box): the compaction legs' kernel stats and
# PMC bytes (8 x 1 M records; the per-GPU share 8 x 1 GiB), the headline's
# (tools/profile.sh), then smoke + GPU tests + bench (tools/r3_full.sh).
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=r3 bash tools/pmc_compaction.sh || exit 1
PER_TABLE=8134407 T_TRACE=400 T_PMC=300 TAG=r3share bash tools/pmc_compaction.sh || exit 1
TAG=r3 STEPS=20 bash tools/profile.sh || exit 1
TAG=r3_final bash tools/r3_full.sh
