#!/bin/bash
# Kernel trace of the bench's extra legs (cfg4 batched decode, cfg5-scaled compaction).
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pl -- python3 bench.py --steps 4 --warmup 1 --cpu-sample-mb 0 --no-encode > gpurun_out/pl.log 2>&1 || exit $?
f=$(find gpurun_out/pl -name "*kernel_trace.csv" | head -1)
cp "$f" gpurun_out/pl_trace.csv
echo "$f"
