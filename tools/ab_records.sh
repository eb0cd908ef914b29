#!/bin/bash
# Round 5: compaction in records mode (the merge's last round writes the
# records) vs pairs + encode (HG_COMPACT_RECORDS=0), the bench's two cfg 5
# legs, same box, alternating; then a rocprofv3 kernel trace of each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
for r in 1 2; do for m in 1 0; do
  HG_COMPACT_RECORDS=$m timeout -k 10 200 python3 tools/compact_leg.py > gpurun_out/abr_$m.log 2>&1 ||
    { tail -5 gpurun_out/abr_$m.log; exit 1; }
  echo "== records=$m round $r scaled: $(grep -o '"ms_per_step": [0-9.]*\|"exact": [a-z]*\|"parity[a-z_]*": [a-z]*' gpurun_out/abr_$m.log | tr '\n' ' ')"
  HG_COMPACT_RECORDS=$m PER_TABLE=8134407 timeout -k 10 300 python3 tools/compact_leg.py > gpurun_out/abr_share_$m.log 2>&1 ||
    { tail -5 gpurun_out/abr_share_$m.log; exit 1; }
  echo "== records=$m round $r share: $(grep -o '"ms_per_step": [0-9.]*\|"exact": [a-z]*\|"parity[a-z_]*": [a-z]*' gpurun_out/abr_share_$m.log | tr '\n' ' ')"
done; done
for m in 1 0; do
  rm -rf gpurun_out/abr_prof_$m
  HG_COMPACT_RECORDS=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abr_prof_$m -o run \
    -- python3 tools/compact_leg.py > gpurun_out/abr_prof_$m.log 2>&1 || { tail -5 gpurun_out/abr_prof_$m.log; exit 1; }
  echo "== records=$m kernels"; grep -h -E "hgk::|hgm::" gpurun_out/abr_prof_$m/run_kernel_stats.csv | cut -d, -f1-4
done
