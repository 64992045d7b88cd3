"""CPU: the §8f oracles (oracle/next_oracle.c) against the reference's golden vectors
(tests/golden/make_golden_next.py) -- bit-exact."""
import os

import numpy as np
import pytest

import oracle

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def splat():
    return np.load(os.path.join(GOLD, "next_splat.npz"))


def _cases(z, prefix, key):
    return sorted(k.split("/")[0] for k in z.files if k.startswith(prefix) and k.endswith("/" + key))


def test_forward_interpolate_oracle_bit_exact(splat):
    names = _cases(splat, "fi_", "flow")
    assert len(names) >= 6
    for k in names:
        got = oracle.forward_interpolate(splat[f"{k}/flow"])
        assert oracle.same_bits(got, splat[f"{k}/out"]), k


def test_grid_sample_values_oracle_bit_exact(splat):
    for k in _cases(splat, "gsv_", "input"):
        h, w = (int(v) for v in splat[f"{k}/hw"])
        values, valid = oracle.grid_sample_values(splat[f"{k}/input"], h, w)
        assert oracle.same_bits(values, splat[f"{k}/values"]), k
        assert np.array_equal(valid, splat[f"{k}/valid"]), k
