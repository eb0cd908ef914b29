# Round 4: the LDS-DMA pre-pass in compaction (KPRE) and batched (cfg 4)
# mode: same-box A/B of the in-tree library (LDS-DMA + fused lane walks),
# nofuse (LDS-DMA only) and noglds (register-staged, separate lane walks).
set -e
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 bash tools/ab_compact.sh base nofuse noglds
for r in 1 2; do for v in base nofuse noglds; do
  if [ $v = base ]; then unset HG_LIBRARY; else export HG_LIBRARY=$PWD/build_exp/$v/libhorreum_gpu.so; fi
  echo "== cfg4 $v round $r: $(timeout -k 10 200 python3 tools/multi_table.py 2>/dev/null | grep '^{')"
done; done
