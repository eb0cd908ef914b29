cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for round in 1 2; do for name in ${NAMES:-base hop384 lean0}; do
  if [ "$name" = base ]; then unset HG_LIBRARY; else export HG_LIBRARY=$PWD/build_exp/$name/libhorreum_gpu.so; fi
  timeout -k 10 200 python3 tools/multi_table.py > gpurun_out/ab_mt_$name.log 2>&1 || { tail -3 gpurun_out/ab_mt_$name.log; exit 1; }
  timeout -k 10 200 python3 tools/decode_variants.py ${WL:-cfg2 mixed} > gpurun_out/ab_dv_$name.log 2>&1 || exit 1
  echo "== $name $round: $(grep -o '"ms": [0-9.]*' gpurun_out/ab_mt_$name.log | tr '\n' ' ') | $(grep -o '"ms": [0-9.]*' gpurun_out/ab_dv_$name.log | tr '\n' ' ')"
done; done
