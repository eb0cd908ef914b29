# Round 4: the narrowed zero-first-byte lane-guess rule against the round-3
# rule (nonz1), every decode shape, then the decode GPU tests.
set -e
ROUNDS=2 WL="cfg2 mixed small medium large huge midlarge zero" VARIANTS="nonz1" TAG=r4g tools/run.sh ab
TAG=r4g PYT="tests/test_decode_gpu.py tests/test_configs_gpu.py" tools/run.sh tests
