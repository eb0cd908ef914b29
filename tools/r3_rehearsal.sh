# Rehearsal of the driver's N > 1 bench on a one-GPU box: N ranks share the
# card (HG_BENCH_SHARE_GPU=1: gloo for the timing collectives).  The rates are
# those of ranks sharing one HBM, not scaling points; every leg checks its
# parity on every rank.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
for N in 2 4; do
  HG_BENCH_SHARE_GPU=1 timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
    --master-addr 127.0.0.1 --master-port $((29500 + N)) bench.py --gpus $N --steps 20 --warmup 5 \
    > gpurun_out/r3_rehearsal_n$N.json 2> gpurun_out/r3_rehearsal_n$N.err || { tail -20 gpurun_out/r3_rehearsal_n$N.err; exit 1; }
  tail -c 300 gpurun_out/r3_rehearsal_n$N.json
done
