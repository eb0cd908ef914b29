cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python3 tools/spec_diag.py zero > gpurun_out/r3_ab3_specdiag.log 2>&1 || { tail -5 gpurun_out/r3_ab3_specdiag.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r3_ab3_specdiag.log | grep -v "  link"
WL="cfg2 small medium zero" bash tools/ab_variants.sh base nozero
