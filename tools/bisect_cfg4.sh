#!/bin/bash
# cfg 4 batched-decode timing of several builds on one box (each build_exp/bisect/<sha>
# is `git archive <sha>` built in-tree on the CPU side). Usage: tools/bisect_cfg4.sh sha...
set -e
mkdir -p gpurun_out
root=$(pwd)
for c in "$@"; do
  cd "$root/build_exp/bisect/$c"
  echo -n "$c " | tee -a "$root/gpurun_out/bisect_cfg4.log"
  CHECK=${CHECK:-1} REPS=${REPS:-10} timeout -k 10 170 python -u tools/multi_table.py 2>&1 | tee -a "$root/gpurun_out/bisect_cfg4.log"
done
