"""The two level-0 GEMMs of include/ecorr.h against the fp64 oracle.

ecorr_build       fp32 MFMA: every element an exact k-ordered fmaf chain.
ecorr_build_split f16 matrix cores on per-pixel power-of-two-scaled hi + lo halves of each fp32
                  operand (lo*hi + hi*lo + hi*hi, fp32 accumulation).

Bar (north star): level 0 within 1e-5 normwise (max|d| / rms) of the reference's fp32 GEMM; the
fp64 oracle stands in for it here (the reference's own values are checked in test_corr_gpu).  The
split build must also be at least as accurate as the fp32 one on every case, including operands
scaled far from 1 (the per-pixel scales) and ragged shapes (the non-vector staging path, D not a
multiple of the 16-deep K chunk).  Pooled levels stay bit-exact from either level 0.
"""
import numpy as np
import pytest
import torch

import oracle
import prng

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
GEMM_TOL = 1e-5

CASES = [  # (B, D, H, W, operand scale, seed)
    (2, 256, 16, 24, 1.0, 1),
    (1, 256, 60, 80, 1.0, 2),
    (2, 256, 32, 32, 1e-3, 3),
    (2, 256, 32, 32, 3e4, 4),
    (1, 100, 17, 22, 1.0, 5),      # ragged: non-vector loads, D % 16 != 0
    (3, 64, 9, 13, 0.25, 6),
]


@pytest.fixture(scope="module")
def ea():
    if not torch.cuda.is_available():
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    import eraft_amd
    eraft_amd.lib()
    return eraft_amd


def _build(ea, f1, f2, mode, levels=4):
    from eraft_amd import _lib
    B, D, H, W = f1.shape
    _, _, off = _lib.layout(B * H * W, H, W, levels)
    pyr = _lib.build_pyramid(f1, f2, B, D, H, W, H * W, levels, off, "test build", mode=mode)
    torch.cuda.synchronize()
    from eraft_amd.layout import formats, untile
    h, w, _ = _lib.layout(B * H * W, H, W, levels)
    ntx = formats(H, W, levels)
    return [untile(pyr[off[i]:off[i + 1]], B * H * W, h[i], w[i], ntx[i])[:, 0].cpu().numpy()
            for i in range(levels)]


@pytest.mark.parametrize("case", CASES, ids=lambda c: "b%d_d%d_%dx%d_s%g" % c[:5])
def test_split_vs_fp32_vs_fp64(ea, case):
    B, D, H, W, scale, seed = case
    f1n = (prng.normal(10 * seed, (B, D, H, W)) * np.float32(scale)).astype(np.float32)
    f2n = (prng.normal(10 * seed + 1, (B, D, H, W)) * np.float32(scale)).astype(np.float32)
    f1, f2 = torch.from_numpy(f1n).to(DEV), torch.from_numpy(f2n).to(DEV)
    truth = oracle.corr_level0(f1n, f2n)
    errs = {}
    with torch.no_grad():
        for mode in ("fp32", "split"):
            lv = _build(ea, f1, f2, mode, levels=3 if min(H, W) < 16 else 4)
            errs[mode] = oracle.normwise_err(lv[0], truth)
            ref_levels = oracle.pyramid_from_level0(lv[0], len(lv))
            for i in range(1, len(lv)):
                assert oracle.same_bits(lv[i], ref_levels[i]), f"{mode}: level {i}"
    print(f"normwise vs fp64: fp32 {errs['fp32']:.2e}  split {errs['split']:.2e}")
    assert errs["fp32"] <= GEMM_TOL and errs["split"] <= GEMM_TOL
    assert errs["split"] <= max(errs["fp32"], 1e-6)


def test_split_query_slab_matches_whole(ea):
    """Per-pixel scales: a query-row slab build (row sharding) is bitwise the whole build's rows."""
    from eraft_amd import _lib
    B, D, H, W = 2, 256, 30, 40
    f1n = prng.normal(71, (B, D, H, W))
    f1n[:, :, 7:9] *= np.float32(1e-4)   # rows with a very different magnitude
    f2n = prng.normal(72, (B, D, H, W))
    f1, f2 = torch.from_numpy(f1n).to(DEV), torch.from_numpy(f2n).to(DEV)
    with torch.no_grad():
        whole = _build(ea, f1, f2, "split")
        r0, rr = 6, 5
        slab = f1[:, :, r0:r0 + rr].contiguous()
        q = rr * W
        _, _, off = _lib.layout(B * q, H, W, 4)
        pyr = _lib.build_pyramid(slab, f2, B, D, H, W, q, 4, off, "slab", mode="split")
        torch.cuda.synchronize()
    from eraft_amd.layout import formats, untile
    h, w, _ = _lib.layout(B * q, H, W, 4)
    ntx = formats(H, W, 4)
    for i in range(4):
        got = untile(pyr[off[i]:off[i + 1]], B * q, h[i], w[i], ntx[i])[:, 0].cpu().numpy()
        want = whole[i].reshape(B, H * W, h[i], w[i])[:, r0 * W:(r0 + rr) * W].reshape(B * q, h[i], w[i])
        assert oracle.same_bits(got, want), f"level {i}"



@pytest.mark.parametrize("case", [(2, 256, 16, 24, 1.0, 7), (1, 100, 17, 22, 1e-3, 8)],
                         ids=lambda c: "b%d_d%d_%dx%d_s%g" % c[:5])
def test_split_inloop_fallback(ea, case, monkeypatch):
    """The split build's fallback (panels too large for one buffer range: the operands split in
    the K loop instead of by pack_kernel; forced here with ECORR_BUILD_PK=0, read per launch)
    meets the same bar on the vector and the ragged (register-staged) loops."""
    B, D, H, W, scale, seed = case
    f1n = (prng.normal(10 * seed, (B, D, H, W)) * np.float32(scale)).astype(np.float32)
    f2n = (prng.normal(10 * seed + 1, (B, D, H, W)) * np.float32(scale)).astype(np.float32)
    f1, f2 = torch.from_numpy(f1n).to(DEV), torch.from_numpy(f2n).to(DEV)
    truth = oracle.corr_level0(f1n, f2n)
    monkeypatch.setenv("ECORR_BUILD_PK", "0")
    with torch.no_grad():
        lv = _build(ea, f1, f2, "split", levels=3)
    err = oracle.normwise_err(lv[0], truth)
    print(f"in-loop split normwise vs fp64 {err:.2e}")
    assert err <= GEMM_TOL
    ref_levels = oracle.pyramid_from_level0(lv[0], 3)
    for i in range(1, 3):
        assert oracle.same_bits(lv[i], ref_levels[i]), f"level {i}"


@pytest.mark.parametrize("case", [(2, 256, 16, 24, 1.0, 9), (3, 100, 17, 22, 1e-3, 10), (1, 256, 60, 80, 1.0, 11),
                                  (2, 64, 5, 300, 3e4, 12)],
                         ids=lambda c: "b%d_d%d_%dx%d_s%g" % c[:5])
def test_split_single_pack_launch_matches_two(ea, case, monkeypatch):
    """Both operand passes run as ONE launch (pack_both_kernel, grid z = operand, surplus x blocks
    of the shorter pass return at once).  Shapes with n_mt != n_nt (ragged 17x22, the band tiles of
    a 5-row map, DSEC 60x80) must give the pyramid bit for bit as one launch per operand
    (ECORR_BUILD_PACK2=1, read per launch)."""
    B, D, H, W, scale, seed = case
    f1 = torch.from_numpy((prng.normal(10 * seed, (B, D, H, W)) * np.float32(scale)).astype(np.float32)).to(DEV)
    f2 = torch.from_numpy((prng.normal(10 * seed + 1, (B, D, H, W)) * np.float32(scale)).astype(np.float32)).to(DEV)
    with torch.no_grad():
        one = _build(ea, f1, f2, "split", levels=3)
        monkeypatch.setenv("ECORR_BUILD_PACK2", "1")
        two = _build(ea, f1, f2, "split", levels=3)
    for i in range(3):
        assert oracle.same_bits(one[i], two[i]), f"level {i}"
