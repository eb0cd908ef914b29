#!/usr/bin/env python3
"""Static instruction counts of one kernel in a hipcc -S listing:
tools/isa_count.py file.s kernel_substring.  (A/B aid for code-size and
VALU changes; dynamic counts come from rocprofv3 --pmc SQ_INSTS_VALU.)"""
import re
import sys
from collections import Counter

lines = open(sys.argv[1]).read().split("\n")
pat = sys.argv[2]
start = next(i for i, l in enumerate(lines) if re.match(r"^\S*" + re.escape(pat) + r"\S*:", l))
end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
body = [l.strip() for l in lines[start:end] if l.startswith("\t") and not l.startswith("\t.")]
body = [l for l in body if l and not l.startswith(";")]
kind = Counter(l.split("_")[0] for l in body)
print(f"{pat}: {len(body)} instructions; " + ", ".join(f"{k} {v}" for k, v in kind.most_common(8)))
