#!/bin/bash
# One launcher for the GPU-box steps (under gpurun, from the repo root); each
# step has its own time limit and the script stops at the first failure.
#   TAG=r4 tools/run.sh smoke tests bench      logs: gpurun_out/${TAG}_<step>.*
# Steps:
#   smoke       __graft_entry__.smoke()
#   tests       pytest -m gpu (extra pytest arguments in $PYT, e.g. a file list)
#   bench       python bench.py (arguments in $BENCH_ARGS)
#   rehearsal   the N > 1 bench with N ranks sharing the card, N in $NS ("2 4")
#   cfg4        tools/multi_table.py (batched decode, cfg 4 per-GPU share)
#   cfg4trace   rocprofv3 kernel trace of it at $NTABS tables ("1 8 32")
#   variants    tools/decode_variants.py on $WL shapes (default: all)
#   ab          tools/ab_variants.sh base $VARIANTS on $WL (build_exp/<variant>/)
#   merge       tools/merge_epochs.py (sorted / epochs / rank-path timings)
#   compact     tools/compact_leg.py (the bench's cfg 5 scaled leg alone)
#   cfg4diag    tools/spec_diag.py on cfg 4's tables at the batched geometry
#   two         tools/two_share.sh base (two share-leg compactions at once)
#   probes      tools/probes/copy_probe and sweep_probe (SWEEP_RING=1)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-run}
fail() { echo "== $1 failed"; tail -${2:-20} "$3"; exit 1; }
for step in "$@"; do
  case $step in
    smoke)
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 ||
        fail smoke 5 gpurun_out/${T}_smoke.log
      tail -1 gpurun_out/${T}_smoke.log ;;
    tests)
      timeout -k 10 1100 python3 -u -m pytest ${PYT:-tests} -m gpu -x -v --timeout 300 --timeout-method thread \
        -p no:cacheprovider > gpurun_out/${T}_pytest.log 2>&1 || fail tests 30 gpurun_out/${T}_pytest.log
      tail -2 gpurun_out/${T}_pytest.log ;;
    bench)
      timeout -k 10 900 python3 bench.py ${BENCH_ARGS:-} > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err ||
        fail bench 5 gpurun_out/${T}_bench.err
      tail -c 600 gpurun_out/${T}_bench.json ;;
    rehearsal)
      for N in ${NS:-2 4}; do
        HG_BENCH_SHARE_GPU=1 timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
          --master-addr 127.0.0.1 --master-port $((29500 + N)) bench.py --gpus $N --steps 20 --warmup 5 \
          > gpurun_out/${T}_rehearsal_n$N.json 2> gpurun_out/${T}_rehearsal_n$N.err ||
          fail "rehearsal n$N" 20 gpurun_out/${T}_rehearsal_n$N.err
        tail -c 300 gpurun_out/${T}_rehearsal_n$N.json
      done ;;
    cfg4)
      timeout -k 10 300 python3 tools/multi_table.py > gpurun_out/${T}_cfg4.log 2>&1 || fail cfg4 5 gpurun_out/${T}_cfg4.log
      grep '^{' gpurun_out/${T}_cfg4.log ;;
    cfg4trace)
      for n in ${NTABS:-1 8 32}; do
        NTAB=$n CHECK=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
          -d gpurun_out/${T}_cfg4_n$n -o run -- python3 tools/multi_table.py > gpurun_out/${T}_cfg4_n$n.log 2>&1 ||
          fail "cfg4trace n$n" 5 gpurun_out/${T}_cfg4_n$n.log
        grep '^{' gpurun_out/${T}_cfg4_n$n.log
      done ;;
    variants)
      timeout -k 10 500 python3 tools/decode_variants.py ${WL:-} > gpurun_out/${T}_variants.log 2>&1 ||
        fail variants 5 gpurun_out/${T}_variants.log
      grep -v amdgpu.ids gpurun_out/${T}_variants.log ;;
    ab)
      WL="${WL:-small medium mixed4k zsmall midlarge}" timeout -k 10 900 bash tools/ab_variants.sh base ${VARIANTS:?} ||
        exit 1 ;;
    merge)
      timeout -k 10 600 python3 tools/merge_epochs.py ${MERGE_ARGS:-} > gpurun_out/${T}_merge.log 2>&1 || fail merge 5 gpurun_out/${T}_merge.log
      grep -v amdgpu.ids gpurun_out/${T}_merge.log ;;
    compact)
      timeout -k 10 300 python3 tools/compact_leg.py > gpurun_out/${T}_compact.log 2>&1 ||
        fail compact 5 gpurun_out/${T}_compact.log
      grep -v amdgpu.ids gpurun_out/${T}_compact.log | tail -5 ;;
    cfg4diag)  # per-table pre-pass codes at the batched decode's geometry (64-piece batches)
      CFG4_TABLES=${CFG4_TABLES:-32} HG_DECODE_BP=64 HG_DECODE_SBP=64 timeout -k 10 400 \
        python3 tools/spec_diag.py cfg4 > gpurun_out/${T}_cfg4diag.log 2>&1 || fail cfg4diag 5 gpurun_out/${T}_cfg4diag.log
      grep -v amdgpu.ids gpurun_out/${T}_cfg4diag.log ;;
    two)  # two processes compacting the cfg 5 share at once on one GPU
      timeout -k 10 600 bash tools/two_share.sh base > gpurun_out/${T}_two.log 2>&1 || fail two 20 gpurun_out/${T}_two.log
      cat gpurun_out/${T}_two.log ;;
    probes)  # copy ceiling (encode) and the pre-pass stream geometry
      timeout -k 10 300 tools/probes/copy_probe > gpurun_out/${T}_copy_probe.log 2>&1 || fail probes 5 gpurun_out/${T}_copy_probe.log
      SWEEP_RING=1 timeout -k 10 300 tools/probes/sweep_probe > gpurun_out/${T}_sweep_ring.log 2>&1 ||
        fail probes 5 gpurun_out/${T}_sweep_ring.log
      cat gpurun_out/${T}_copy_probe.log gpurun_out/${T}_sweep_ring.log ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
