#!/bin/bash
# Round-end style check on the GPU box: smoke, every GPU test, the bench, the
# rocprofv3 evidence for the headline (tools/profile.sh) and for the general
# decode engine (tools/pmc_general.sh).  TAG names the files under profiles/.
# Run as: GIT_COMMIT=<sha> TAG=r2_vN bash tools/full_check.sh
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${TAG:-r2}
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -5 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 1200 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -15 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 600 python3 bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -5 gpurun_out/bench_$TAG.err; exit 1; }
tail -c 400 gpurun_out/bench_$TAG.json
[ -n "$NO_PROFILE" ] && exit 0
TAG=$TAG bash tools/profile.sh || exit 1
TAG=$TAG bash tools/pmc_general.sh > gpurun_out/pmc_general_$TAG.log 2>&1 || { tail -5 gpurun_out/pmc_general_$TAG.log; exit 1; }
