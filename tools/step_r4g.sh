# Round 4: pre-pass kernel durations on cfg 2 under rocprofv3 (kernel trace
# only): the in-tree library (LDS-DMA staging), the register-staged build
# (old), the fused lane walks (fuse), and the in-tree one at 32-piece batches.
set -e
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4g_$name -o run \
    -- python3 tools/decode_variants.py cfg2 > gpurun_out/r4g_$name.log 2>&1
  echo "== $name"; grep -h -E "decode_spec|decode_kernel|decode_lw" gpurun_out/r4g_$name/*/run_kernel_stats.csv 2>/dev/null ||
    find gpurun_out/r4g_$name -name "*kernel_stats.csv" -exec grep -h -E "decode_spec|decode_kernel|decode_lw" {} \;
}
run base X=1
run old HG_LIBRARY=$PWD/build_exp/old/libhorreum_gpu.so
run fuse HG_LIBRARY=$PWD/build_exp/fuse/libhorreum_gpu.so
run sbp32 HG_DECODE_SBP=32
