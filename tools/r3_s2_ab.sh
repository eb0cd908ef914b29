# Round-3 session-2 GPU step: lane-walk chunk DMA cache policy A/B, then the
# decode PMC evidence of the bench's variable-size shapes (r3_evidence_a.sh).
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
ROUNDS=2 WL="small medium zsmall mixed4k" timeout -k 10 400 bash tools/ab_variants.sh base lwnt > gpurun_out/ab_lwnt.log 2>&1; rc=$?; cat gpurun_out/ab_lwnt.log; [ $rc -eq 0 ] || exit $rc
bash tools/r3_evidence_a.sh
