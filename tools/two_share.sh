#!/bin/bash
# Two processes running the cfg 5 share compaction leg at once on one GPU
# (the N = 2 shared-card rehearsal's shape), per library: base (in-tree) and
# build_exp/NAME.  Prints each process's leg line.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
for n in "$@"; do
  if [ "$n" = base ]; then unset HG_LIBRARY; else export HG_LIBRARY=$PWD/build_exp/$n/libhorreum_gpu.so; fi
  PER_TABLE=8134407 timeout -k 10 240 python3 tools/compact_leg.py > gpurun_out/two_${n}_a.log 2>&1 &
  A=$!
  PER_TABLE=8134407 timeout -k 10 240 python3 tools/compact_leg.py > gpurun_out/two_${n}_b.log 2>&1 &
  B=$!
  wait $A; ra=$?; wait $B; rb=$?
  for x in a b; do
    echo "== $n $x: $(grep '^{' gpurun_out/two_${n}_$x.log | tail -1 | python3 -c 'import json,sys; l=json.loads(sys.stdin.read()); print(l["ms"], l["times_ms"], l["status"], l.get("parity_bytes_ok"), l.get("merge_paths"))')"
  done
  [ $ra -eq 0 ] && [ $rb -eq 0 ] || exit 1
done
