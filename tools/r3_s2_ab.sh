# Round-3 session-2 GPU step: compaction-mode key prefix stores, default
# policy vs nontemporal (build_exp/kprent), cfg 5 leg kernel stats.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 bash tools/ab_compact.sh base kprent > gpurun_out/ab_kprent.log 2>&1; rc=$?; cat gpurun_out/ab_kprent.log; [ $rc -eq 0 ] || exit $rc
