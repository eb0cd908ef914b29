#!/usr/bin/env python3
"""Time bench.py's config-5-scaled compaction leg alone (decode -> merge ->
encode of 8 x 1 M-record tables in HBM) and print its JSON line; with
--kernels also prints the merge's per-kernel split (hipEvents around the
merge call are not split per kernel: use rocprofv3 for that)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from horreum_amd.engine import Engine  # noqa: E402
from horreum_amd import abi as _abi  # noqa: E402
_abi.knobs_from_env()  # the A/B scripts' HG_* knobs (the library reads no environment)


def main():
    eng = Engine(0)
    dev = eng.device
    eng.set_stream(torch.cuda.current_stream(dev))
    per = int(os.environ.get("PER_TABLE", 1_000_000))  # 8_134_407: the per-GPU share of cfg 5
    line = bench.compaction_leg(torch, eng, dev, 1, 0, per_table=per)
    line["merge_path"] = "one-pass k-way" if os.environ.get("HG_MERGE_KWAY") == "1" else "pairwise rounds"
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
