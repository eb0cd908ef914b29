# Round 4: rank loop (single pending read, packed keys), lane-guess rule
# with the zero bits from the masks, then the merge and decode GPU tests.
set -e
TAG=r4f tools/run.sh merge
WL="cfg2 small medium midlarge zero" VARIANTS="nonz1" TAG=r4f tools/run.sh ab
TAG=r4f PYT="tests/test_merge_gpu.py tests/test_decode_gpu.py" tools/run.sh tests
