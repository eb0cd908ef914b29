# Round 4: pre-pass staging floor -- the stream-only build (no per-piece
# checks after piece 0; results invalid, timing only) vs the in-tree library.
set -e
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4h_$name -o run \
    -- python3 tools/decode_variants.py cfg2 > gpurun_out/r4h_$name.log 2>&1
  echo "== $name"; grep -h -E "decode_spec" gpurun_out/r4h_$name/run_kernel_stats.csv
}
run base X=1
run stream HG_LIBRARY=$PWD/build_exp/stream/libhorreum_gpu.so
ROUNDS=3 WL="cfg2 small medium" timeout -k 10 600 bash tools/ab_variants.sh base fuse | grep "^==\|cfg2\|small\|medium"
