"""CPU: the optimised multi-threaded CPU codec (oracle/cpu_opt.c, the
cpu_baseline's all-cores row) produces exactly the oracle's spans and bytes:
byte ranges with guessed entries handed over in order, for 1..8 threads."""
import numpy as np
import pytest

from oracle import oracle
from tests import corpus


@pytest.mark.parametrize("name", ["fixed_16_100", "mixed_small", "tiny", "empty_keys_tombs",
                                  "zero_values", "mixed_4k", "large_values", "midlarge",
                                  "midlarge_zero"])
@pytest.mark.parametrize("threads", [1, 3, 8])
def test_mt_decode_matches_oracle(name, threads):
    _, _, data, _ = corpus.make(name)
    want, wn, wk, _, _ = oracle.decode(data)
    spans, n, secs = oracle.mt_decode(data, threads)
    assert n == wn and secs >= 0
    assert np.array_equal(spans[:n], want)


def test_mt_decode_reports_errors():
    _, _, data, rec_off = corpus.make("mixed_small")
    bad = data[: int(rec_off[1000]) + 5]
    _, n, _ = oracle.mt_decode(bad, 4)
    assert n == 2**64 - 1


@pytest.mark.parametrize("name", ["fixed_32_256", "mixed_small", "mixed_4k", "empty_keys_tombs"])
@pytest.mark.parametrize("threads", [1, 5])
def test_mt_encode_matches_oracle(name, threads):
    arena, pairs, data, _ = corpus.make(name)
    out, secs = oracle.mt_encode(arena, pairs, threads)
    assert np.array_equal(out, data)
