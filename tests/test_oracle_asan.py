"""CPU: the oracle's ASan/UBSan build (oracle/Makefile `asan`) runs the
golden-vector checks and the multi-threaded CPU codec in a child process with
the ASan runtime preloaded; any sanitizer report fails the test."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import sys
sys.path.insert(0, sys.argv[1])
import numpy as np
from oracle import oracle
from tests import corpus
assert oracle.LIB.endswith("liboracle_asan.so"), oracle.LIB
for name in ("mixed_small", "tiny", "zero_values", "mixed_4k", "large_values"):
    arena, pairs, data, _ = corpus.make(name)
    want, wn, wk, _, _ = oracle.decode(data)
    for t in (1, 4):
        spans, n, _ = oracle.mt_decode(data, t)
        assert n == wn and np.array_equal(spans[:n], want)
        out, _ = oracle.mt_encode(arena, pairs, t)
        assert np.array_equal(out, data)
    oracle.decode(data[: data.size // 2 + 3])
    tabs = [(data, want)]
    oracle.compact(tabs)
print("asan-ok")
'''


def test_oracle_under_asan():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"], check=True)
    lib = os.path.join(ROOT, "oracle", "liboracle_asan.so")
    asan_rt = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True,
                             text=True).stdout.strip()
    if not asan_rt or not os.path.exists(asan_rt):
        pytest.skip("no libasan runtime")
    env = dict(os.environ, HGO_LIBRARY=lib, LD_PRELOAD=asan_rt,
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT], env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0 and "asan-ok" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
