"""The generator-truth span layouts the bench legs check against
(synth.span_rows) agree with the oracle's decode of the same bytes (CPU)."""
import numpy as np

from horreum_amd import synth
from oracle import oracle


def test_mixed_sst_layout_matches_oracle():
    for kr, vr in (((0, 24), (0, 64)), ((8, 65), (64, 513))):
        buf, off, kl, vl = synth.mixed_sst_host(5000, kr, vr, 0.05, 7, layout=True)
        want, n, kind, _, _ = oracle.decode(buf)
        assert kind == 0 and n == 5000
        rows = synth.span_rows(off, kl, vl)
        assert np.array_equal(want.view("<u8").reshape(-1, 2), rows)
        assert np.array_equal(buf, synth.mixed_sst_host(5000, kr, vr, 0.05, 7))
