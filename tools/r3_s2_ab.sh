# Round-3 session-2 GPU step: lane-walk serial-walk A/B (decode_variants),
# FETCH_SIZE calibration probe, compaction A/B (per-piece entries vs
# merge_prep), then smoke + GPU tests + bench (tools/r3_full.sh).
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
ROUNDS=1 WL="small medium midlarge zsmall zmidlarge mixed4k large" timeout -k 10 600 bash tools/ab_variants.sh base ser12 ser24 ser40 ser999 > gpurun_out/ab_ser.log 2>&1; rc=$?; cat gpurun_out/ab_ser.log; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/fetch_cal -- ./tools/probes/fetch_cal > gpurun_out/fetch_cal.log 2>&1 || { tail -5 gpurun_out/fetch_cal.log; exit 1; }
tail -5 gpurun_out/fetch_cal.log
timeout -k 10 400 bash tools/ab_compact.sh base nokent > gpurun_out/ab_kent.log 2>&1; rc=$?; cat gpurun_out/ab_kent.log; [ $rc -eq 0 ] || exit $rc
TAG=r3s2 bash tools/r3_full.sh
