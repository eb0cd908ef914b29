# Round 4: compaction without the look-back-status and group-sum memsets and
# with the merge error word in the staging copy, against HEAD (build_exp/prev);
# cfg 3 encode both ways; the merge / encode / manager GPU tests.
set -e
timeout -k 10 400 bash tools/ab_compact.sh base prev | grep "^=="
for r in 1 2; do
  echo "== encode base round $r"; timeout -k 10 200 python3 tools/encode_variants.py 2>&1 | grep '^{' | head -1
  echo "== encode prev round $r"; HG_LIBRARY=$PWD/build_exp/prev/libhorreum_gpu.so timeout -k 10 200 python3 tools/encode_variants.py 2>&1 | grep '^{' | head -1
done
TAG=r4i PYT="tests/test_merge_gpu.py tests/test_encode_gpu.py tests/test_manager_gpu.py tests/test_multi_gpu.py tests/test_configs_gpu.py" tools/run.sh tests
