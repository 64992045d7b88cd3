"""GPU parity of lookup + convc1 + ReLU (CorrBlock.lookup_conv1x1_relu) in both
modes: "fused" (ecorr_lookup_conv1x1_relu[_packed], one kernel, fp32 MFMA) and "split" (the
default: ecorr_lookup, then ecorr_conv1x1_relu_split on the f16 matrix cores) against the unfused
path.  Split-mode specifics (scales, NaN, ragged O / Q): test_conv_split_gpu.py.

Bars: with one-hot weights (each output channel copies one correlation channel, times 1, plus a
bias) the fused-mode output is BIT-EXACT relu(corr + bias), because an fmaf chain over exact zeros and
one exact 1.0 reproduces its input -- this pins the sampling, the channel order and the epilogue;
with dense weights either mode's output agrees normwise (max|d| / rms <= 1e-5) with an fp64 conv of our own
(bit-exact, oracle-checked) lookup output; e2e flow with the fused path stays within the 1e-3 px
EPE bar of the reference goldens (test_e2e_gpu.py cases).
"""
import glob
import os

import numpy as np
import pytest
import torch

import oracle
import prng
from conftest import GOLDEN

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module")
def ea():
    if not torch.cuda.is_available():
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    import eraft_amd
    eraft_amd.lib()
    return eraft_amd


def _block(ea, B, D, H, W, seed, L=4):
    f1 = torch.from_numpy(prng.normal(seed, (B, D, H, W))).to(DEV)
    f2 = torch.from_numpy(prng.normal(seed + 1, (B, D, H, W))).to(DEV)
    return ea.CorrBlock(f1, f2, num_levels=L)


@pytest.mark.parametrize("shape", [(2, 64, 16, 24, 4), (1, 32, 60, 80, 4), (2, 32, 17, 20, 3), (1, 16, 9, 13, 2)],
                         ids=lambda s: "b%d_d%d_%dx%d_l%d" % s)
def test_one_hot_weights_bit_exact(ea, shape):
    B, D, H, W, L = shape
    C, O = L * 81, 128
    with torch.no_grad():
        blk = _block(ea, B, D, H, W, 31, L)
        coords = torch.from_numpy(prng.coords_with_flow(32, B, H, W, 3.0)).to(DEV)
        coords[0, :, 0, :3] = torch.tensor([float("nan"), 1e9, -7.0e5], device=DEV)   # direct path
        corr = blk(coords)
        pick = torch.arange(O, device=DEV) * 7 % C
        wgt = torch.zeros(O, C, 1, 1, device=DEV)
        wgt[torch.arange(O), pick] = 1.0
        bias = torch.from_numpy(prng.normal(33, (O,))).to(DEV)
        out = blk.lookup_conv1x1_relu(coords, wgt, bias, mode="fused")
        ref = torch.relu(corr[:, pick] + bias.view(1, O, 1, 1))
    assert oracle.same_bits(out.cpu().numpy(), ref.cpu().numpy())
    # no bias: pure copy through relu
    with torch.no_grad():
        out0 = blk.lookup_conv1x1_relu(coords, wgt[:, :, 0, 0], mode="fused")
    assert oracle.same_bits(out0.cpu().numpy(), torch.relu(corr[:, pick]).cpu().numpy())


@pytest.mark.parametrize("mode", ["fused", "split"])
@pytest.mark.parametrize("shape", [(2, 64, 16, 24), (16, 256, 60, 80)], ids=["small", "dsec_b16"])
def test_dense_weights_normwise(ea, shape, mode):
    B, D, H, W = shape
    with torch.no_grad():
        blk = _block(ea, B, D, H, W, 41)
        coords_np = prng.coords_with_flow(42, B, H, W, 3.0)
        coords = torch.from_numpy(coords_np).to(DEV)
        corr = blk(coords)
        wgt = torch.from_numpy(prng.normal(43, (256, 324, 1, 1)) * 0.05).to(DEV)
        bias = torch.from_numpy(prng.normal(44, (256,)) * 0.1).to(DEV)
        out = blk.lookup_conv1x1_relu(coords, wgt, bias, mode=mode)
    # our lookup is bit-exact vs the oracle (checked elsewhere); conv it in fp64 here
    c64 = corr.double().cpu()
    ref = torch.relu(torch.einsum("oc,bchw->bohw", wgt[:, :, 0, 0].double().cpu(), c64)
                     + bias.double().cpu().view(1, -1, 1, 1)).numpy()
    got = out.cpu().numpy().astype(np.float64)
    err = np.max(np.abs(got - ref)) / np.sqrt(np.mean(ref * ref))
    assert err <= 1e-5, err
    if B * H * W <= 800:
        levels = [lv[:, 0].cpu().numpy() for lv in blk.corr_pyramid]
        assert oracle.same_bits(corr.cpu().numpy(), oracle.lookup(levels, coords_np, 4))


def test_fused_rejects_unsupported(ea):
    with torch.no_grad():
        blk = ea.CorrBlock(torch.zeros(1, 8, 16, 16, device=DEV), torch.zeros(1, 8, 16, 16, device=DEV),
                           radius=3)
        with pytest.raises(ValueError):   # the fused kernel is radius 4 only
            blk.lookup_conv1x1_relu(torch.zeros(1, 2, 16, 16, device=DEV), torch.zeros(64, 196, device=DEV),
                                    mode="fused")
        with pytest.raises(ValueError):
            blk.lookup_conv1x1_relu(torch.zeros(1, 2, 16, 16, device=DEV), torch.zeros(64, 196, device=DEV),
                                    mode="fp32")
        blk = ea.CorrBlock(torch.zeros(1, 8, 16, 16, device=DEV), torch.zeros(1, 8, 16, 16, device=DEV))
        with pytest.raises(RuntimeError):   # weight does not map 324 channels
            blk.lookup_conv1x1_relu(torch.zeros(1, 2, 16, 16, device=DEV), torch.zeros(64, 300, device=DEV))


@pytest.mark.parametrize("shape", [(2, 64, 16, 24, 4, 256), (1, 32, 23, 40, 3, 128)], ids=["l4_o256", "l3_o128"])
def test_packed_weight_matches_weight_as_stored(ea, shape):
    """ecorr_lookup_conv1x1_relu_packed (the weight in MFMA fragment order, what CorrBlock uses) is
    bitwise ecorr_lookup_conv1x1_relu with the weight as stored; an in-place weight update re-packs."""
    from eraft_amd import _lib
    B, D, H, W, L, O = shape
    C = L * 81
    with torch.no_grad():
        blk = _block(ea, B, D, H, W, 51, L)
        coords = torch.from_numpy(prng.coords_with_flow(52, B, H, W, 3.0)).to(DEV)
        wgt = torch.from_numpy(prng.normal(53, (O, C, 1, 1)) * 0.05).to(DEV)
        bias = torch.from_numpy(prng.normal(54, (O,)) * 0.1).to(DEV)
        got = blk.lookup_conv1x1_relu(coords, wgt, bias, mode="fused")
        ref = torch.empty_like(got)
        _lib.check(_lib.lib().ecorr_lookup_conv1x1_relu(
            blk._pyramid.data_ptr(), coords.data_ptr(), B, H, W, H * W, L, 4, wgt.data_ptr(), bias.data_ptr(), O,
            ref.data_ptr(), _lib.stream_of(coords)), "unpacked")
        torch.cuda.synchronize()
        assert torch.equal(got, ref)
        wgt.mul_(-1.0)   # in place: the cached packed weight must not be reused
        got2 = blk.lookup_conv1x1_relu(coords, wgt, bias, mode="fused")
        _lib.check(_lib.lib().ecorr_lookup_conv1x1_relu(
            blk._pyramid.data_ptr(), coords.data_ptr(), B, H, W, H * W, L, 4, wgt.data_ptr(), bias.data_ptr(), O,
            ref.data_ptr(), _lib.stream_of(coords)), "unpacked")
        torch.cuda.synchronize()
        assert torch.equal(got2, ref) and not torch.equal(got2, got)
        # changes through .data keep the version counter -- the packed weight is scoped
        # to the block (one ERAFT forward), so the next block packs the weight as it is now ...
        wgt.data.mul_(2.0)
        blk2 = _block(ea, B, D, H, W, 51, L)
        got3 = blk2.lookup_conv1x1_relu(coords, wgt, bias, mode="fused")
        _lib.check(_lib.lib().ecorr_lookup_conv1x1_relu(
            blk2._pyramid.data_ptr(), coords.data_ptr(), B, H, W, H * W, L, 4, wgt.data_ptr(), bias.data_ptr(), O,
            ref.data_ptr(), _lib.stream_of(coords)), "unpacked")
        torch.cuda.synchronize()
        assert torch.equal(got3, ref) and not torch.equal(got3, got2)
        # ... and a new storage behind the same tensor (.data = t) re-packs within the block
        wgt.data = wgt.data * -0.5
        got4 = blk2.lookup_conv1x1_relu(coords, wgt, bias, mode="fused")
        _lib.check(_lib.lib().ecorr_lookup_conv1x1_relu(
            blk2._pyramid.data_ptr(), coords.data_ptr(), B, H, W, H * W, L, 4, wgt.data_ptr(), bias.data_ptr(), O,
            ref.data_ptr(), _lib.stream_of(coords)), "unpacked")
        torch.cuda.synchronize()
        assert torch.equal(got4, ref) and not torch.equal(got4, got3)
