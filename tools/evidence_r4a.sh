# Round-4 evidence, part A (GPU box): decode PMC per variable-size shape and
# the headline's kernel stats + FETCH/WRITE passes (summarised on the CPU side
# by tools/summarize_pmc.py / summarize_prof.py into profiles/).
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=r4 SHAPES="small medium midlarge zsmall zmidlarge" bash tools/pmc_general.sh || exit 1
TAG=r4 STEPS=20 bash tools/profile.sh || exit 1
