# Round-3 evidence, part A (GPU box): rocprofv3 kernel stats, FETCH_SIZE /
# WRITE_SIZE and SQ counters of the decode on the bench's variable-size shapes
# (tools/pmc_general.sh); summarised here by tools/summarize_pmc.py into
# profiles/r3_pmc_<shape>.json.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=r3 SHAPES="small medium midlarge zsmall zmidlarge" bash tools/pmc_general.sh
