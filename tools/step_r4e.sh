# Round 4: same-box A/Bs -- rank loop (templated vs first version), cfg 3
# encode (HEAD vs round 2's 0b3b8ac, each with its own tools), compaction
# gather variants, lane-guess rule -- then the merge and decode GPU tests.
set -e
TAG=r4d tools/run.sh merge
HG_LIBRARY=$PWD/build_exp/rank0/horreum_amd/libhorreum_gpu.so TAG=r4d_old tools/run.sh merge
for r in 1 2 3; do
  echo "== encode HEAD round $r"; timeout -k 10 200 python3 tools/encode_variants.py 2>&1 | grep '^{'
  echo "== encode 0b3b8ac round $r"; (cd build_exp/bisect/0b3b8ac && timeout -k 10 200 python3 tools/encode_variants.py 2>&1 | grep '^{')
done
timeout -k 10 400 bash tools/ab_compact.sh base rpt2 recu4 recu1 | grep "^=="
WL="cfg2 small medium midlarge zero" VARIANTS="nonz1" TAG=r4e tools/run.sh ab
TAG=r4e PYT="tests/test_merge_gpu.py tests/test_decode_gpu.py" tools/run.sh tests
