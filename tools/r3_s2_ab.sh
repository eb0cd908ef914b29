# Round-3 session-2 GPU step: pre-pass batch size A/B on the lane-walk shapes
# (environment overrides of the batch geometry; no rebuild).
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
for round in 1 2; do for setting in "X=0" "HG_DECODE_SBP=8" "HG_DECODE_BP=32 HG_DECODE_SBP=32"; do
  ( export $setting
    timeout -k 10 300 python3 tools/decode_variants.py small medium zsmall zmidlarge > gpurun_out/absbp.log 2>&1 ) || { tail -5 gpurun_out/absbp.log; exit 1; }
  echo "== $setting round $round: $(grep -o '"ms": [0-9.]*' gpurun_out/absbp.log | tr '\n' ' ') parity $(grep -c '"parity": true' gpurun_out/absbp.log)"
done; done
