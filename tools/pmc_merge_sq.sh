#!/bin/bash
# SQ counters of the cfg 5-scaled compaction leg's kernels (tools/compact_leg.py),
# two passes of 8 SQ counters each, each pass its own run; kernel averages
# printed per pass (merge / decode-entries / encode kernels).
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-msq}
pass() {  # pass <name> <counters...>
  local name=$1; shift
  rm -rf gpurun_out/${T}_$name
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/${T}_$name -- python3 tools/compact_leg.py \
    > gpurun_out/${T}_$name.log 2>&1 || { echo "== $name failed"; tail -3 gpurun_out/${T}_$name.log; exit 1; }
  f=$(find gpurun_out/${T}_$name -name "*counter_collection.csv" | head -1)
  python3 - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].split("(")[0]
    if "hg" not in k:
        continue
    acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    print(k[:40].ljust(40), " ".join("%s=%.3g" % (c.replace("SQ_", ""), sorted(v)[len(v) // 2]) for c, v in cs.items()))
PY
}
pass sqa SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS
pass sqb SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM
