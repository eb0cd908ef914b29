# Round 4: store ordering in the pre-pass (HG_SPEC_ST_AFTER) and the fused
# lane walks, same-box A/B on the decode shapes; merge + decode GPU tests.
set -e
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=r4j PYT="tests/test_merge_gpu.py tests/test_decode_gpu.py" tools/run.sh tests
ROUNDS=3 WL="cfg2 small medium zsmall midlarge zmidlarge" timeout -k 10 700 bash tools/ab_variants.sh base stafter fuse
timeout -k 10 300 bash tools/ab_compact.sh base stafter | grep "^=="
