#!/bin/bash
# Kernel-trace the cfg 2 decode under experimental libraries (build_exp/NAME,
# "base" = in-tree): per-kernel averages into gpurun_out/eutr_NAME/.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
for n in "$@"; do
  if [ "$n" = base ]; then unset HG_LIBRARY; else export HG_LIBRARY=$PWD/build_exp/$n/libhorreum_gpu.so; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/eutr_$n -- python3 tools/decode_variants.py ${WL:-cfg2} > gpurun_out/eutr_$n.log 2>&1 || exit 1
  f=$(ls -t gpurun_out/eutr_$n/*/*kernel_stats.csv | head -1)
  echo "== $n"; grep -E "decode_kernel|decode_spec_kernel" "$f" | cut -d, -f1-8
done
