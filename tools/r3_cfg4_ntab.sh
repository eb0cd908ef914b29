# Round-3: cfg 4's batched decode kernels at 1, 8 and 32 tables (kernel trace).
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
for n in 1 8 32; do
  NTAB=$n CHECK=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3_cfg4_n$n -o run -- python3 tools/multi_table.py > gpurun_out/r3_cfg4_n$n.log 2>&1 || { tail -5 gpurun_out/r3_cfg4_n$n.log; exit 1; }
  grep '^{' gpurun_out/r3_cfg4_n$n.log
done
