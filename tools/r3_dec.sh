cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r3_dec}
timeout -k 10 600 python3 -u -m pytest tests/test_decode_gpu.py tests/test_lookup_gpu.py tests/test_manager_gpu.py tests/test_api.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
timeout -k 10 300 python3 tools/spec_diag.py zero --truth > gpurun_out/${T}_specdiag.log 2>&1 || { tail -5 gpurun_out/${T}_specdiag.log; exit 1; }
timeout -k 10 300 python3 tools/spec_diag.py midlarge --truth >> gpurun_out/${T}_specdiag.log 2>&1 || { tail -5 gpurun_out/${T}_specdiag.log; exit 1; }
timeout -k 10 400 python3 tools/decode_variants.py > gpurun_out/${T}_variants.log 2>&1 || { tail -5 gpurun_out/${T}_variants.log; exit 1; }
cat gpurun_out/${T}_specdiag.log | grep -v amdgpu.ids; cat gpurun_out/${T}_variants.log | grep -v amdgpu.ids
