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


@pytest.fixture(scope="module")
def flowz():
    return np.load(os.path.join(GOLD, "next_flow.npz"))


def upsample_inputs(z, k):
    import prng
    N, H, W, seed = (int(v) for v in z[f"{k}/shape"])
    return (prng.normal(seed, (N, 2, H, W), 4.0),
            prng.normal(seed + 1, (N, 576, H, W), float(z[f"{k}/mscale"])))


def test_upsample_oracle_vs_reference(flowz):
    # libm expf vs ATen's vectorized exp: a few ulp, never more (tolerance in units of the output rms)
    for k in _cases(flowz, "up_", "out"):
        flow, mask = upsample_inputs(flowz, k)
        ref = flowz[f"{k}/out"]
        got = oracle.upsample_flow(flow, mask)
        assert oracle.normwise_err(got, ref) <= 2e-6, k


def test_png16_codec_oracle_bit_exact(flowz):
    for k in ("enc_rand", "enc_small"):
        assert np.array_equal(oracle.flow_to_png16(flowz[f"{k}/flow"]), flowz[f"{k}/png"]), k
    flow, valid, bad = oracle.flow_16bit_to_float(flowz["dec/png"])
    assert bad == 0
    assert np.array_equal(valid, flowz["dec/valid"])
    assert np.array_equal(flow.astype(np.float64), flowz["dec/flow"])   # exact in float32
    assert bool(flowz["dec_bad/raises"]) and oracle.flow_16bit_to_float(flowz["dec_bad/png"])[2] == 1


@pytest.fixture(scope="module")
def voxz():
    return np.load(os.path.join(GOLD, "next_voxel.npz"))


def test_voxel_oracle_vs_reference(voxz):
    """Accumulated grids bit-exact (serial fold); normalized within 2 ulp-ish (reduction order)."""
    from voxel_cases import DSEC_VOXEL, MVSEC_VOXEL, dsec_case, mvsec_case
    for k, (n, C, H, W, seed) in DSEC_VOXEL.items():
        p, t, x, y = dsec_case(k, n, H, W, seed)
        assert oracle.same_bits(oracle.voxel_dsec(p, t, x, y, C, H, W, False), voxz[f"{k}/norm0"]), k
        got = oracle.voxel_dsec(p, t, x, y, C, H, W, True)
        np.testing.assert_allclose(got, voxz[f"{k}/norm1"], rtol=1e-6, atol=1e-6, err_msg=k)
    for k, (n, C, H, W, seed) in MVSEC_VOXEL.items():
        ev = mvsec_case(k, n, H, W, seed)
        g0, bad = oracle.voxel_mvsec(ev, C, H, W, False)
        if f"{k}/raises" in voxz.files:
            assert bad, k
            continue
        assert not bad and oracle.same_bits(g0, voxz[f"{k}/norm0"]), k
        g1, _ = oracle.voxel_mvsec(ev, C, H, W, True)
        np.testing.assert_allclose(g1, voxz[f"{k}/norm1"], rtol=1e-6, atol=1e-6, err_msg=k)
