# Lane-walk A/B round 2: variants, then SQ instruction counts (base vs old).
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
WL="${WL:-small medium mixed4k}" bash tools/ab_variants.sh ${VARIANTS:-base nomlf occ3 occ2 old} || exit 1
for v in base old; do
  if [ "$v" = base ]; then unset HG_LIBRARY; else export HG_LIBRARY=$PWD/build_exp/$v/libhorreum_gpu.so; fi
  for s in small medium; do
    timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d gpurun_out/lwsq_${v}_$s -- python3 tools/decode_variants.py $s > gpurun_out/lwsq_${v}_$s.log 2>&1 || { echo "pmc $v $s failed"; tail -3 gpurun_out/lwsq_${v}_$s.log; exit 1; }
  done
done
unset HG_LIBRARY
python3 - <<'PY'
import csv, glob, collections
for v in ("base", "old"):
    for s in ("small", "medium"):
        fs = glob.glob(f"gpurun_out/lwsq_{v}_{s}/**/*counter_collection.csv", recursive=True)
        acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
        for f in fs:
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"]
                if "decode_lw" not in k: continue
                acc[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
        out = {c: sum(d.values()) / max(1, len(d)) for c, d in acc.items()}
        print(v, s, {c: round(x) for c, x in sorted(out.items())})
PY
