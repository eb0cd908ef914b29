# Round-3: kernel trace of cfg 4's batched decode (tools/multi_table.py).
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3_cfg4 -o run -- python3 tools/multi_table.py > gpurun_out/r3_cfg4.log 2>&1 || { tail -5 gpurun_out/r3_cfg4.log; exit 1; }
grep -o '"ms[^,]*' gpurun_out/r3_cfg4.log | head -2
