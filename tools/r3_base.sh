cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_smoke0.log 2>&1 || { tail -5 gpurun_out/r3_smoke0.log; exit 1; }
timeout -k 10 400 python3 bench.py > gpurun_out/r3_bench0.json 2> gpurun_out/r3_bench0.err || { tail -5 gpurun_out/r3_bench0.err; exit 1; }
timeout -k 10 300 python3 tools/spec_diag.py zero --truth > gpurun_out/r3_specdiag0.log 2>&1 || { tail -5 gpurun_out/r3_specdiag0.log; exit 1; }
timeout -k 10 300 python3 tools/spec_diag.py midlarge --truth >> gpurun_out/r3_specdiag0.log 2>&1 || { tail -5 gpurun_out/r3_specdiag0.log; exit 1; }
timeout -k 10 400 python3 tools/decode_variants.py > gpurun_out/r3_variants0.log 2>&1 || { tail -5 gpurun_out/r3_variants0.log; exit 1; }
cat gpurun_out/r3_specdiag0.log; cat gpurun_out/r3_variants0.log
