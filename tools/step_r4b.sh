set -e
L=$PWD/build_exp
for r in 1 2; do
  TAG=r4b tools/run.sh cfg4
  HG_LIBRARY=$L/noz16/libhorreum_gpu.so TAG=r4b_noz16 tools/run.sh cfg4
done
TAG=r4b tools/run.sh cfg4diag | grep "^cfg4 table" | head -8
ROUNDS=1 WL="cfg2 mixed small medium large huge midlarge zero" VARIANTS="noz16" TAG=r4b tools/run.sh ab
bash tools/ab_compact.sh base noxcd
