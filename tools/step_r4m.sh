# Round 4: the pre-pass's first piece -- raw barriers for the guess
# broadcast and the stride OR (HG_SPEC_RAWSYNC) vs __syncthreads, and the
# guess's cost (noguess: cfg 2's entries computed, timing only).
set -e
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=r4m PYT="tests/test_decode_gpu.py tests/test_configs_gpu.py" tools/run.sh tests
ROUNDS=3 WL="cfg2 small medium zsmall midlarge" timeout -k 10 700 bash tools/ab_variants.sh base norawsync
for v in base norawsync noguess; do
  if [ $v = base ]; then unset HG_LIBRARY; else export HG_LIBRARY=$PWD/build_exp/$v/libhorreum_gpu.so; fi
  rm -rf gpurun_out/r4m_$v
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4m_$v -o run \
    -- python3 tools/decode_variants.py cfg2 > gpurun_out/r4m_$v.log 2>&1
  echo "== $v"; grep -h -E "decode_spec" gpurun_out/r4m_$v/run_kernel_stats.csv
done
