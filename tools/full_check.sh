cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_v13.log 2>&1 || { tail -5 gpurun_out/smoke_v13.log; exit 1; }
tail -1 gpurun_out/smoke_v13.log
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_v13.log 2>&1 || { tail -15 gpurun_out/pytest_gpu_v13.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_v13.log
timeout -k 10 400 python3 bench.py > gpurun_out/bench_v13.json 2> gpurun_out/bench_v13.err || { tail -5 gpurun_out/bench_v13.err; exit 1; }
tail -c 600 gpurun_out/bench_v13.json
TAG=r1_v13 bash tools/profile.sh
