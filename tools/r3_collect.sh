#!/bin/bash
# After tools/r3_evidence.sh: summaries and logs into profiles/ (run here).
set -e
cd "$(dirname "$0")/.."
python3 tools/summarize_pmc.py gpurun_out r3 small medium midlarge zsmall zmidlarge > /dev/null
python3 tools/summarize_compaction.py gpurun_out r3 > /dev/null
python3 tools/summarize_compaction.py gpurun_out r3share r3_pmc_compaction_share.json > /dev/null
python3 tools/summarize_prof.py gpurun_out r3 | tail -5
cp gpurun_out/r3_final_bench.json profiles/r3_bench_final.json
cp gpurun_out/r3_final_pytest.log profiles/r3_pytest_gpu_final.log
cp gpurun_out/r3_final_smoke.log profiles/r3_smoke_final.log
ls -la profiles | grep "r3_\|pmc_summary"
