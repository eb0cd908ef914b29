# Round 4: lane-walk relaxation shift by DPP wave_shr vs __shfl_up (noshr).
set -e
ROUNDS=2 WL="small medium mixed midlarge zero" VARIANTS="noshr" TAG=r4j tools/run.sh ab
TAG=r4j PYT="tests/test_decode_gpu.py" tools/run.sh tests
