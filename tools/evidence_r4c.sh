# Round-4 evidence, part C (GPU box): smoke, every GPU test, the bench, and the
# N = 2 / 4 shared-card rehearsals of the multi-rank bench.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=r4_final tools/run.sh smoke tests bench rehearsal
