cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for round in 1 2; do for n in "$@"; do
  if [ "$n" = base ]; then unset HG_LIBRARY; else export HG_LIBRARY=$PWD/build_exp/$n/libhorreum_gpu.so; fi
  timeout -k 10 300 python3 tools/encode_variants.py > gpurun_out/abe_$n.log 2>&1 || { tail -3 gpurun_out/abe_$n.log; exit 1; }
  echo "== $n round $round: $(grep -o '"ms": [0-9.]*\|"b2b_ms": [0-9.]*' gpurun_out/abe_$n.log | tr '\n' ' ') $(grep -c 'true' gpurun_out/abe_$n.log)"
done; done
