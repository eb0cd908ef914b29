cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_decode_gpu.py -x -q -k "host_path" -p no:cacheprovider > gpurun_out/host_tests.log 2>&1; rc=$?; tail -3 gpurun_out/host_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --cpu-sample-mb 0 --no-encode --no-extra > gpurun_out/bench_host.log 2>&1; rc=$?; tail -2 gpurun_out/bench_host.log; exit $rc
