#!/bin/bash
# Round 5 evidence, call A (GPU box): hop-segment geometry A/B on the hop
# shapes and cfg 4, then the encode kernel's counters at the current sources
#  and the plain device-copy ceiling for cfg 3's traffic.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
run() {  # run <name> <seconds> <args...>
  local name=$1 secs=$2; shift 2
  timeout -s KILL "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
if [ -n "$HOP_VARIANTS" ]; then
  ROUNDS=2 WL="midlarge mixed4k large huge zmidlarge" bash tools/ab_variants.sh base $HOP_VARIANTS || exit 1
  for r in 1 2; do for v in base $HOP_VARIANTS; do
    if [ $v = base ]; then unset HG_LIBRARY; else export HG_LIBRARY=$PWD/build_exp/$v/libhorreum_gpu.so; fi
    timeout -k 10 300 python3 tools/multi_table.py > gpurun_out/abh_cfg4_$v.log 2>&1 || { tail -3 gpurun_out/abh_cfg4_$v.log; exit 1; }
    echo "== cfg4 $v round $r: $(grep '^{' gpurun_out/abh_cfg4_$v.log | tail -1 | cut -c1-200)"
  done; done
  unset HG_LIBRARY
fi
if [ -n "$ENCODE_PMC" ]; then
  run r5_enc_trace 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5_enc_trace -- python3 tools/encode_variants.py
  run r5_enc_fetch 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r5_enc_fetch -- python3 tools/encode_variants.py
  run r5_enc_write 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r5_enc_write -- python3 tools/encode_variants.py
  run r5_enc_sq 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d gpurun_out/r5_enc_sq -- python3 tools/encode_variants.py
  run r5_copy_probe 120 ./tools/probes/copy_probe
fi
