# Round-3 session-2 GPU step: compaction A/B (merge entries from the decode
# workspace vs merge_prep_kernel), then smoke + GPU tests + bench.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 bash tools/ab_compact.sh base nokent > gpurun_out/ab_kent.log 2>&1; rc=$?; cat gpurun_out/ab_kent.log; [ $rc -eq 0 ] || exit $rc
TAG=r3s2 bash tools/r3_full.sh
