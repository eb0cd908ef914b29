#!/bin/bash
# The round-4 same-box A/B experiments, one case each; every profiles/r4_ab_*
# log names its case.  Variant libraries are built on the CPU side first
# (tools/ab_round4.sh --build CASE runs tools/build_variant.sh for them), then
# the case runs on the GPU box: gpurun -- 'bash tools/ab_round4.sh CASE'.
# "base" is always the in-tree library.  Cases whose variant is an older
# commit (rank0, the encode bisect) say which; build those from that commit.
#
#   hopz16     hop guesses without 16-zero-byte starts (noz16: -DHG_HOP_Z16=0):
#              cfg 4, every decode shape, the cfg 4 pre-pass codes
#   lw_nz1     the paired zero-first-byte lane-guess rule (nonz1: -DHG_LW_NZ1=0)
#   lw_wshr    relaxation shift by DPP wave_shr (noshr: -DHG_LW_WSHR=0)
#   rank_enc   the merge cases (the rank loop's first version was build rank0,
#              the commit before 8cc5f5a), cfg 3 encode (round 2's build was
#              0b3b8ac), record-gather unrolls (recu4/recu1: -DHG_ENC_REC_U=4/1;
#              rpt2, two pieces per thread, was reverted code)
#   compact_gaps / gather_adj  compaction against an older build (prev: the
#              commit before 6c06271) or reverted code (adj2/adj4, f2c4303)
#   dma_asm    LDS-DMA from asm (old: -DHG_SPEC_GLDS=0 -DHG_DMA_ASM=0 -DHG_LW_FUSE=0;
#              lwasm: -DHG_SPEC_GLDS=0 -DHG_LW_FUSE=0; fuse: the default)
#   staging    pre-pass kernel times under rocprofv3 (old as above; sbp32 by env)
#   floor      staging-only builds (stream1/stream2: -DHG_SPEC_STREAM_ONLY=1/2,
#              results invalid) and tools/probes/sweep_probe
#   spec_emit  speculative pre-pass spans (emit: -DHG_SPEC_EMIT=1
#              -DHG_SPEC_ST_AFTER=1) and the one-pass k-way merge (HG_MERGE_KWAY=1;
#              kwnopass: -DHG_KW_NOPASS=1, results invalid)
#   fuse       stores behind the DMA (stafter: -DHG_SPEC_ST_AFTER=1), fused lane
#              walks (nofuse: -DHG_LW_FUSE=0)
#   glds_cfg4  compaction leg and cfg 4 (nofuse: -DHG_LW_FUSE=0; noglds:
#              -DHG_SPEC_GLDS=0 -DHG_LW_FUSE=0)
#   span8      lane-walk spans as 8-byte scratch entries (reverted code: the
#              variant built from it was base; span16 = -DHG_LW_SPAN8=0)
set -e
root=$(cd "$(dirname "$0")/.." && pwd)
variants() {  # name:defines per case (build side)
  case $1 in
    hopz16) echo "noz16:-DHG_HOP_Z16=0" ;;
    lw_nz1) echo "nonz1:-DHG_LW_NZ1=0" ;;
    lw_wshr) echo "noshr:-DHG_LW_WSHR=0" ;;
    rank_enc) echo "recu4:-DHG_ENC_REC_U=4 recu1:-DHG_ENC_REC_U=1" ;;
    dma_asm) echo "old:-DHG_SPEC_GLDS=0_-DHG_DMA_ASM=0_-DHG_LW_FUSE=0 lwasm:-DHG_SPEC_GLDS=0_-DHG_LW_FUSE=0 nofuse:-DHG_LW_FUSE=0" ;;
    staging) echo "old:-DHG_SPEC_GLDS=0_-DHG_DMA_ASM=0_-DHG_LW_FUSE=0" ;;
    floor) echo "stream1:-DHG_SPEC_STREAM_ONLY=1 stream2:-DHG_SPEC_STREAM_ONLY=2" ;;
    spec_emit) echo "emit:-DHG_SPEC_EMIT=1_-DHG_SPEC_ST_AFTER=1 kwnopass:-DHG_KW_NOPASS=1" ;;
    fuse) echo "stafter:-DHG_SPEC_ST_AFTER=1 nofuse:-DHG_LW_FUSE=0" ;;
    glds_cfg4) echo "nofuse:-DHG_LW_FUSE=0 noglds:-DHG_SPEC_GLDS=0_-DHG_LW_FUSE=0" ;;
    span8) echo "span16:-DHG_LW_SPAN8=0" ;;
  esac
}
if [ "$1" = --build ]; then
  for v in $(variants "$2"); do
    "$root/tools/build_variant.sh" "${v%%:*}" "$(echo "${v#*:}" | tr _ ' ')"
  done
  exit 0
fi
cd "${GRAFT_REPO_ROOT:-$root}" && mkdir -p gpurun_out && export TMPDIR=/tmp
names() { for v in $(variants "$1"); do printf '%s ' "${v%%:*}"; done; }
use() {  # select a variant library for the following commands
  if [ "$1" = base ]; then unset HG_LIBRARY; else export HG_LIBRARY=$PWD/build_exp/$1/libhorreum_gpu.so; fi
}
kstats() {  # rocprofv3 kernel stats of decode_variants.py $WL under variant $1
  rm -rf gpurun_out/ab4_$1
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab4_$1 -o run \
    -- python3 tools/decode_variants.py ${WL:-cfg2} > gpurun_out/ab4_$1.log 2>&1
  echo "== $1"; grep -h -E "hgk::|hgm::" gpurun_out/ab4_$1/run_kernel_stats.csv
}
case $1 in
  hopz16)
    for r in 1 2; do for v in base noz16; do use $v; TAG=ab4_$v tools/run.sh cfg4; done; done; use base
    TAG=ab4 tools/run.sh cfg4diag | grep "^cfg4 table" | head -8
    ROUNDS=1 WL="cfg2 mixed small medium large huge midlarge zero" bash tools/ab_variants.sh base noz16 ;;
  lw_nz1|lw_wshr)
    ROUNDS=2 WL="cfg2 mixed small medium large huge midlarge zero" bash tools/ab_variants.sh base $(names $1)
    TAG=ab4 PYT="tests/test_decode_gpu.py" tools/run.sh tests ;;
  rank_enc)
    TAG=ab4 tools/run.sh merge
    for r in 1 2 3; do echo "== encode base round $r"; timeout -k 10 200 python3 tools/encode_variants.py 2>&1 | grep '^{'; done
    timeout -k 10 400 bash tools/ab_compact.sh base $(names $1) | grep "^==" ;;
  compact_gaps|gather_adj)  # VARIANTS: the older / reverted builds, placed in build_exp/
    timeout -k 10 500 bash tools/ab_compact.sh base ${VARIANTS:?} | grep "^==\|encode_records" ;;
  span8)
    TAG=ab4 PYT="tests/test_decode_gpu.py tests/test_merge_gpu.py tests/test_configs_gpu.py" tools/run.sh tests
    ROUNDS=3 WL="cfg2 small medium zsmall midlarge zmidlarge mixed4k" timeout -k 10 700 bash tools/ab_variants.sh base span16
    for v in base span16; do use $v; WL="small" kstats $v; done; use base ;;
  dma_asm|fuse)
    TAG=ab4 PYT="tests/test_decode_gpu.py tests/test_merge_gpu.py" tools/run.sh tests
    ROUNDS=3 WL="cfg2 small medium zsmall midlarge zmidlarge" timeout -k 10 700 bash tools/ab_variants.sh base $(names $1) ;;
  staging)
    for v in base old; do use $v; kstats $v; done; use base; HG_DECODE_SBP=32 kstats sbp32 ;;
  floor)
    for v in base stream1 stream2; do use $v; kstats $v; done; use base
    echo "== probe"; SWEEP_GLDS_ONLY=1 timeout -k 10 120 tools/probes/sweep_probe 2>&1 | grep -E "glds x2|flat" ;;
  spec_emit)
    ROUNDS=3 WL="cfg2 small medium zsmall midlarge" timeout -k 10 700 bash tools/ab_variants.sh base emit
    use emit; kstats emit; use base
    timeout -k 10 600 bash tools/ab_compact.sh base kway kwnopass ;;
  glds_cfg4)
    timeout -k 10 600 bash tools/ab_compact.sh base $(names $1)
    for r in 1 2; do for v in base $(names $1); do use $v
      echo "== cfg4 $v round $r: $(timeout -k 10 200 python3 tools/multi_table.py 2>/dev/null | grep '^{')"
    done; done ;;
  *) echo "unknown case $1 (see the header)"; exit 2 ;;
esac
