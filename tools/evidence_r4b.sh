# Round-4 evidence, part B (GPU box): the compaction legs' kernel stats and PMC
# bytes (8 x 1 M records; the per-GPU share 8 x 1 GiB); summarised on the CPU
# side by tools/summarize_compaction.py.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=r4 bash tools/pmc_compaction.sh || exit 1
PER_TABLE=8134407 T_TRACE=400 T_PMC=300 TAG=r4share bash tools/pmc_compaction.sh || exit 1
