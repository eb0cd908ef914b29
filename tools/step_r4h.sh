# Round 4: pre-pass staging floor -- the stream-only build (no per-piece
# checks after piece 0; results invalid, timing only) vs the in-tree library.
set -e
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
run() {  # name, env...
  local name=$1; shift
  rm -rf gpurun_out/r4h_$name
  env "$@" timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4h_$name -o run \
    -- python3 tools/decode_variants.py cfg2 > gpurun_out/r4h_$name.log 2>&1
  echo "== $name"; grep -h -E "decode_spec|decode_kernel" gpurun_out/r4h_$name/run_kernel_stats.csv
}
run base X=1
run stream1 HG_LIBRARY=$PWD/build_exp/stream1/libhorreum_gpu.so
run stream1b HG_LIBRARY=$PWD/build_exp/stream1/libhorreum_gpu.so
run stream2 HG_LIBRARY=$PWD/build_exp/stream2/libhorreum_gpu.so
echo "== probe"; SWEEP_GLDS_ONLY=1 timeout -k 10 120 tools/probes/sweep_probe 2>&1 | grep -E "glds x2|flat"
