#!/bin/bash
# Per-kernel VGPRs / spills / occupancy / LDS of one .hip file (gfx950), compact.
# Usage: tools/resusage.sh horreum_amd/csrc/hg_decode.hip [extra hipcc flags]
f=$1; shift
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I"$(dirname "$0")/../include" "$@" -c "$f" -o /dev/null \
  -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c '
import re, sys
cur = None
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}; continue
    for key in ("VGPRs", "VGPRs Spill", "SGPRs Spill", "Occupancy \\[waves/SIMD\\]", "LDS Size \\[bytes/block\\]"):
        m = re.search(r"remark:\s+" + key + r": (\d+)", line)
        if m and cur is not None:
            cur[key.split()[0] + ("_spill" if "Spill" in key else "")] = int(m.group(1))
            if key.startswith("LDS"):
                print("%-70s vgpr %3d vspill %3d sspill %3d occ %d lds %d" % (cur["name"][:70], cur.get("VGPRs", 0), cur.get("VGPRs_spill", 0), cur.get("SGPRs_spill", 0), cur.get("Occupancy", 0), cur["LDS"]))
'
