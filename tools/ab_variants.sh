#!/bin/bash
# Time decode_variants.py workloads (WL words) under experimental libraries
# built by tools/build_variant.sh: tools/ab_variants.sh NAME...  ("base" = the in-tree library)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
for round in $(seq 1 ${ROUNDS:-2}); do for name in "$@"; do
  if [ "$name" = base ]; then unset HG_LIBRARY; else export HG_LIBRARY=$PWD/build_exp/$name/libhorreum_gpu.so; fi
  timeout -k 10 300 python3 tools/decode_variants.py ${WL:-} > gpurun_out/abv_$name.log 2>&1 || { tail -3 gpurun_out/abv_$name.log; exit 1; }
  echo "== $name round $round"; grep -o '"workload": "[^"]*".*"b2b_ms": [0-9.]*' gpurun_out/abv_$name.log | sed 's/"bytes.*"ms"/ms/'
done; done
