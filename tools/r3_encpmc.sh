# SQ counters of the compaction leg's kernels (encode gather in particular).
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d gpurun_out/encsq -- python3 tools/compact_leg.py > gpurun_out/encsq.log 2>&1 || { tail -3 gpurun_out/encsq.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM TA_BUSY_avr TA_BUSY_max --output-format csv -d gpurun_out/encsq2 -- python3 tools/compact_leg.py > gpurun_out/encsq2.log 2>&1 || { tail -3 gpurun_out/encsq2.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
for d in ("encsq", "encsq2"):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"gpurun_out/{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            acc[r["Kernel_Name"].split("(")[0][:40]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in sorted(acc.items()):
        if "hg" not in k: continue
        print(d, k, {c: round(sum(v) / len(v)) for c, v in sorted(cs.items())})
PY
