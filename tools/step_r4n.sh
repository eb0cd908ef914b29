# Round 4: pre-pass halos by DMA (HG_SPEC_HALO_DMA) -- decode GPU tests, then
# a same-box A/B and the pre-pass kernel time.
set -e
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=r4n PYT="tests/test_decode_gpu.py tests/test_configs_gpu.py tests/test_merge_gpu.py" tools/run.sh tests
ROUNDS=3 WL="cfg2 small medium" timeout -k 10 700 bash tools/ab_variants.sh base nohalo
for v in base nohalo; do
  if [ $v = base ]; then unset HG_LIBRARY; else export HG_LIBRARY=$PWD/build_exp/$v/libhorreum_gpu.so; fi
  rm -rf gpurun_out/r4n_$v
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4n_$v -o run \
    -- python3 tools/decode_variants.py cfg2 > gpurun_out/r4n_$v.log 2>&1
  echo "== $v"; grep -h -E "decode_spec" gpurun_out/r4n_$v/run_kernel_stats.csv
done
