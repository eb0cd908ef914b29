cd "$GRAFT_REPO_ROOT"
for r in 1 2 3; do for n in ${VARIANTS:-base}; do
  if [ $n = base ]; then unset HG_LIBRARY; else export HG_LIBRARY=$PWD/build_exp/$n/libhorreum_gpu.so; fi
  echo "$n $(timeout -k 10 300 python3 tools/multi_table.py 2>/dev/null | tail -1) $(timeout -k 10 200 python3 tools/decode_variants.py 8..4096 0..16 2>/dev/null | grep -o '"ms": [0-9.]*\|"parity": [a-z]*' | tr '\n' ' ')"
done; done
