# Round-3 A/B: the batched pre-pass (decode_spec_multi) at 6 waves/SIMD
# (80 VGPRs, build_exp/w6) against the in-tree 5 (89 VGPRs) on cfg 4.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
for round in 1 2 3; do for name in base w6; do
  if [ "$name" = base ]; then unset HG_LIBRARY; else export HG_LIBRARY=$PWD/build_exp/$name/libhorreum_gpu.so; fi
  timeout -k 10 300 python3 tools/multi_table.py > gpurun_out/abo_mt_$name.log 2>&1 || { tail -5 gpurun_out/abo_mt_$name.log; exit 1; }
  echo "== $name round $round: cfg4 $(grep -o '"ms[^,]*' gpurun_out/abo_mt_$name.log | head -2 | tr '\n' ' ') $(grep -o '"parity": [a-z]*' gpurun_out/abo_mt_$name.log)"
done; done
