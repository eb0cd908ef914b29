#!/bin/bash
# rocprofv3 evidence for the decode engine on variable-size records (run on
# the GPU box): kernel stats, FETCH_SIZE / WRITE_SIZE and SQ counter passes
# (each in its own run, no other tracing) for the workload shapes named in
# $SHAPES (substrings of tools/decode_variants.py labels).
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${TAG:-r2}
SHAPES=${SHAPES:-"small medium"}
run() {  # run <name> <seconds> <args...>
  local name=$1 secs=$2; shift 2
  timeout -s KILL "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
run ${TAG}_counters_list 60 rocprofv3 -L
for s in $SHAPES; do
  run ${TAG}_trace_$s 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_trace_$s -- python3 tools/decode_variants.py $s
  run ${TAG}_fetch_$s 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_fetch_$s -- python3 tools/decode_variants.py $s
  run ${TAG}_write_$s 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_write_$s -- python3 tools/decode_variants.py $s
  run ${TAG}_sqa_$s 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d gpurun_out/${TAG}_sqa_$s -- python3 tools/decode_variants.py $s
  run ${TAG}_sqb_$s 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM --output-format csv -d gpurun_out/${TAG}_sqb_$s -- python3 tools/decode_variants.py $s
done
python3 tools/summarize_pmc.py gpurun_out "$TAG" $SHAPES > gpurun_out/${TAG}_pmc_summary.log 2>&1
tail -40 gpurun_out/${TAG}_pmc_summary.log
