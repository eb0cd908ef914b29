# Round 4: speculative spans in the pre-pass (HG_SPEC_EMIT): decode GPU tests
# on the new library, then a same-box A/B against noemit / fuse, and the
# kernel durations on cfg 2.
set -e
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=r4i_merge PYT=tests/test_merge_gpu.py tools/run.sh tests
TAG=r4i tools/run.sh tests
ROUNDS=3 WL="cfg2 small medium zsmall midlarge" timeout -k 10 700 bash tools/ab_variants.sh base noemit fuse
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4i_prof -o run \
  -- python3 tools/decode_variants.py cfg2 > gpurun_out/r4i_prof.log 2>&1
grep -h -E "decode_" gpurun_out/r4i_prof/run_kernel_stats.csv
timeout -k 10 600 bash tools/ab_compact.sh base rounds kwnopass
