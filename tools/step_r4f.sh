# Round 4: LDS-DMA pre-pass staging + DMA issued from asm (no compiler
# vmcnt(0) before LDS reads): decode GPU tests on the new library, then a
# same-box A/B against the register-staged / builtin-DMA build (old) and the
# asm DMA for the lane walks only (lwasm).
set -e
TAG=r4f PYT="tests/test_decode_gpu.py" tools/run.sh tests
WL="cfg2 small medium mixed4k zsmall midlarge zmidlarge" VARIANTS="old lwasm fuse" TAG=r4f tools/run.sh ab
HG_LIBRARY=$PWD/build_exp/fuse/libhorreum_gpu.so TAG=r4f_fuse PYT="tests/test_decode_gpu.py" tools/run.sh tests
