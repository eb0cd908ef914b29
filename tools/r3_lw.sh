# Lane-walk A/B: the VALU probe, then decode_variants under the variant libraries.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 120 ./tools/probes/valu_rate > gpurun_out/valu_rate.log 2>&1 || { tail -3 gpurun_out/valu_rate.log; exit 1; }
cat gpurun_out/valu_rate.log
WL="${WL:-small medium mixed4k zsmall midlarge}" bash tools/ab_variants.sh ${VARIANTS:-base old zdot lean}
