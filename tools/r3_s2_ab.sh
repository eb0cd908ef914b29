# Round-3 session-2 GPU step: 256 KiB hop segments for the sparsest batches
# (x8: <= 8 candidate run ends in piece 0, x12: <= 12) on cfg 4 and the
# single-table large-record shapes.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
for round in 1 2; do for name in base x8 x12; do
  if [ "$name" = base ]; then unset HG_LIBRARY; else export HG_LIBRARY=$PWD/build_exp/$name/libhorreum_gpu.so; fi
  timeout -k 10 300 python3 tools/multi_table.py > gpurun_out/abh_mt_$name.log 2>&1 || { tail -5 gpurun_out/abh_mt_$name.log; exit 1; }
  echo "== $name round $round: cfg4 $(grep -o '"ms[^,]*' gpurun_out/abh_mt_$name.log | head -2 | tr '\n' ' ') $(grep -o '"parity": [a-z]*' gpurun_out/abh_mt_$name.log)"
done; done
ROUNDS=2 WL="mixed4k midlarge large huge" timeout -k 10 400 bash tools/ab_variants.sh base x8 x12
