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
    (2, 256, 45, 68, 1.0, 7),      # fp32 mode: build_f32_kernel with ragged query/target tiles
    (1, 256, 19, 30, 1.0, 8),      # fp32 mode: W % 4 != 0 falls back to the generic kernel
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
    return [untile(pyr[off[i]:off[i + 1]], B * H * W, h[i], w[i], ntx[i], i)[:, 0].cpu().numpy()
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
        got = untile(pyr[off[i]:off[i + 1]], B * q, h[i], w[i], ntx[i], i)[:, 0].cpu().numpy()
        want = whole[i].reshape(B, H * W, h[i], w[i])[:, r0 * W:(r0 + rr) * W].reshape(B * q, h[i], w[i])
        assert oracle.same_bits(got, want), f"level {i}"



def _heavy_cases():
    """Operands at the split's documented precision limit (build.hip: lo keeps 11 bits down to
    2^-17 of a pixel's maximum, f16 subnormals below): per-pixel dynamic range 2^17 and 2^24,
    ReLU-sparse channels (half and 90% exact zeros), log-normal heavy tails, one dominant channel."""
    B, D, H, W = 2, 256, 24, 32
    out = []
    for k, (name, gen) in enumerate([
            ("range2^17", lambda s: prng.normal(s, (B, D, H, W)) * np.exp2(-17.0 * prng.uniform(s + 7, (B, D, H, W), 0, 1))),
            ("range2^24", lambda s: prng.normal(s, (B, D, H, W)) * np.exp2(-24.0 * prng.uniform(s + 7, (B, D, H, W), 0, 1))),
            ("relu50", lambda s: np.maximum(prng.normal(s, (B, D, H, W)), 0)),
            ("relu90", lambda s: np.maximum(prng.normal(s, (B, D, H, W)) - 1.2816, 0)),
            ("lognormal", lambda s: prng.normal(s, (B, D, H, W)) * np.exp(2.0 * prng.normal(s + 7, (B, D, H, W)))),
            ("dominant", lambda s: prng.normal(s, (B, D, H, W)) * np.where(np.arange(D)[None, :, None, None] == 3, 1e5, 1.0)),
    ]):
        out.append((name, gen(100 + 10 * k).astype(np.float32), gen(101 + 10 * k).astype(np.float32)))
    return out


@pytest.mark.parametrize("case", _heavy_cases(), ids=lambda c: c[0])
def test_split_precision_limits(ea, case):
    """Normwise <= 1e-5 vs fp64 and no worse than the fp32-MFMA GEMM where features have a wide
    within-pixel dynamic range, exact zeros or heavy tails."""
    name, f1n, f2n = case
    f1, f2 = torch.from_numpy(f1n).to(DEV), torch.from_numpy(f2n).to(DEV)
    truth = oracle.corr_level0(f1n, f2n)
    errs = {}
    with torch.no_grad():
        for mode in ("fp32", "split"):
            lv = _build(ea, f1, f2, mode, levels=3)
            errs[mode] = oracle.normwise_err(lv[0], truth)
    print(f"{name}: normwise vs fp64 fp32 {errs['fp32']:.2e} split {errs['split']:.2e}")
    if name != "lognormal":
        assert errs["fp32"] <= GEMM_TOL and errs["split"] <= GEMM_TOL
    # log-normal tails (e^{2 N(0,1)} scales) make the products cancel: sum |a_k b_k| is far above
    # |sum a_k b_k|, so no fp32-accumulating GEMM meets 1e-5 normwise vs fp64 there (the fp32-MFMA
    # chain measures 3.3e-5; the reference's sgemm accumulates in fp32 too).  The bar for that
    # case is the reference-faithful one: no worse than the fp32 GEMM.  Where ONE product dominates
    # each dot product ("dominant", a channel 1e5 x the rest) nothing averages out and the split's
    # per-product error (2^-22 relative: lo*lo is dropped) exceeds the fp32 chain's (one rounding,
    # 2^-24): 1.6e-6 vs 4e-7 measured, still 6x under the bar; hence the 2e-6 floor.
    assert errs["split"] <= max(errs["fp32"], 2e-6)


def test_split_precision_real_fnet_features(ea):
    """The same bar on real feature maps: E-RAFT's fnet (PRNG weights at the reference's init
    scales, tests/e2e_weights.py) applied to PRNG event volumes, 256 x 320 input -> 32 x 40."""
    import eraft_amd.network as nw
    from e2e_weights import make_state_dict
    net = nw.ERAFT({"subtype": "standard"}, n_first_channels=15)
    net.load_state_dict(make_state_dict(net.state_dict()))
    net = net.eval().to(DEV)
    im1 = torch.from_numpy(prng.normal(41, (1, 15, 256, 320))).to(DEV)
    im2 = torch.from_numpy(prng.normal(42, (1, 15, 256, 320))).to(DEV)
    with torch.no_grad():
        f1, f2 = net.fnet([im1, im2])
        f1, f2 = f1.float().contiguous(), f2.float().contiguous()
        assert f1.shape == (1, 256, 32, 40)
        f1n, f2n = f1.cpu().numpy(), f2.cpu().numpy()
        truth = oracle.corr_level0(f1n, f2n)
        errs = {m: oracle.normwise_err(_build(ea, f1, f2, m)[0], truth) for m in ("fp32", "split")}
    frac0 = float((f1n == 0).mean())
    print(f"fnet features (zeros {frac0:.1%}): fp32 {errs['fp32']:.2e} split {errs['split']:.2e}")
    assert errs["fp32"] <= GEMM_TOL and errs["split"] <= GEMM_TOL
    assert errs["split"] <= max(errs["fp32"], 1e-6)


def test_stray_dev_env_vars_change_nothing(ea, monkeypatch):
    """Round 1 read A/B knobs with getenv on every launch (ECORR_BUILD_SKIP_EPILOGUE dropped pyramid
    stores with status ECORR_OK).  The library reads no environment: setting every old knob must
    leave the pyramid, the lookup and the fused lookup bit for bit unchanged."""
    import eraft_amd
    B, D, H, W = 2, 256, 23, 40
    f1 = torch.from_numpy(prng.normal(61, (B, D, H, W))).to(DEV)
    f2 = torch.from_numpy(prng.normal(62, (B, D, H, W))).to(DEV)
    coords = torch.from_numpy(prng.coords_with_flow(63, B, H, W, 3.0)).to(DEV)
    wt = torch.from_numpy(prng.normal(64, (256, 324)) * np.float32(0.05)).to(DEV)

    def run():
        with torch.no_grad():
            blk = eraft_amd.CorrBlock(f1, f2)
            outs = [lv.clone() for lv in blk.corr_pyramid] + [blk(coords), blk.lookup_conv1x1_relu(coords, wt)]
            torch.cuda.synchronize()
        return outs

    clean = run()
    for k, v in {"ECORR_BUILD_SKIP_EPILOGUE": "1", "ECORR_BUILD_PK": "0", "ECORR_BUILD_PACK2": "1",
                 "ECORR_BUILD_ABL": "5", "ECORR_BUILD_GM": "2", "ECORR_BUILD_KB32": "1", "ECORR_BUILD_GLDS": "0",
                 "ECORR_BUILD_NOBAND": "1", "ECORR_BUILD_PKPIPE": "0", "ECORR_LOOKUP_SKIP": "15",
                 "ECORR_LOOKUP_QB": "16", "ECORR_LOOKUP_V": "4", "ECORR_FUSED_PHASE": "1",
                 "ECORR_SPLAT_STOP": "0"}.items():
        monkeypatch.setenv(k, v)
    dirty = run()
    for a, b in zip(clean, dirty):
        assert torch.equal(a, b)


def test_split_two_stage_calls_match_one(ea):
    """ecorr_build_split_pack + ecorr_build_split_gemm (what CorrBlock issues) == ecorr_build_split."""
    import ctypes
    from eraft_amd import _lib
    B, D, H, W = 2, 256, 23, 40
    f1 = torch.from_numpy(prng.normal(81, (B, D, H, W))).to(DEV)
    f2 = torch.from_numpy(prng.normal(82, (B, D, H, W))).to(DEV)
    _, _, off = _lib.layout(B * H * W, H, W, 4)
    with torch.no_grad():
        two = _lib.build_pyramid(f1, f2, B, D, H, W, H * W, 4, off, "two-stage", mode="split")
        one = torch.empty_like(two)
        nb = ctypes.c_int64()
        _lib.check(_lib.lib().ecorr_build_split_workspace_size(B, D, H, W, H * W, ctypes.byref(nb)), "ws")
        ws = torch.empty(nb.value, dtype=torch.uint8, device=DEV)
        _lib.check(_lib.lib().ecorr_build_split(f1.data_ptr(), f2.data_ptr(), B, D, H, W, H * W, 4, one.data_ptr(),
                                                ws.data_ptr(), _lib.stream_of(f1)), "one call")
        torch.cuda.synchronize()
    from eraft_amd.layout import formats, untile
    h, w, _ = _lib.layout(B * H * W, H, W, 4)
    ntx = formats(H, W, 4)
    for i in range(4):
        a = untile(one[off[i]:off[i + 1]], B * H * W, h[i], w[i], ntx[i], i)
        b = untile(two[off[i]:off[i + 1]], B * H * W, h[i], w[i], ntx[i], i)
        assert torch.equal(a, b), f"level {i}"


def test_nonfinite_fmap_entries(ea):
    """fmaps with +-inf and NaN entries against the reference (tests/golden/nonfinite_corr.npz,
    corr.py:58-60).  fp32 mode (ecorr_build) reproduces the reference's +inf / -inf / NaN pattern
    exactly.  The split build's documented deviation: every level-0 element whose
    query or target pixel holds a non-finite entry is NaN (the lo half of an inf is inf - inf), i.e.
    NaN exactly where the reference is non-finite; every other element finite and normwise within
    the bar.  Both modes: levels 1-3 bit-exact from their own level 0, non-finite exactly where the
    reference's are; the lookup non-finite exactly where the reference's is."""
    from test_oracle_golden import _load, _nonfinite_fmaps, finite_pattern_equal
    import os
    from conftest import GOLDEN
    z = _load(os.path.join(GOLDEN, "nonfinite_corr.npz"))
    f1n, f2n = _nonfinite_fmaps(z)
    L, r = int(z["L"]), int(z["r"])
    ref0 = z["level0"]
    fin = np.isfinite(ref0)
    f1, f2 = torch.from_numpy(f1n).to(DEV), torch.from_numpy(f2n).to(DEV)
    coords = torch.from_numpy(z["coords_s3"]).to(DEV)
    for mode in ("fp32", "split"):
        lv = _build(ea, f1, f2, mode, levels=L)
        if mode == "fp32":
            assert finite_pattern_equal(lv[0], ref0), "fp32: non-finite pattern"
        else:
            assert np.array_equal(np.isnan(lv[0]), ~fin) and np.isfinite(lv[0][fin]).all(), "split: NaN pattern"
        assert oracle.normwise_err(lv[0][fin], ref0[fin]) <= GEMM_TOL, mode
        pooled = oracle.pyramid_from_level0(lv[0], L)
        for i in range(1, L):
            assert oracle.same_bits(lv[i], pooled[i]), f"{mode}: level {i}"
            assert np.array_equal(np.isfinite(lv[i]), np.isfinite(z[f"level{i}"])), f"{mode}: level {i} pattern"
        prev = ea._lib.build_mode()
        ea._lib.set_build_mode(mode)
        try:
            with torch.no_grad():
                out = ea.CorrBlock(f1, f2, num_levels=L, radius=r)(coords).cpu().numpy()
        finally:
            ea._lib.set_build_mode(prev)
        assert np.array_equal(np.isfinite(out), np.isfinite(z["out_s3"])), f"{mode}: lookup pattern"
        assert oracle.same_bits(out, oracle.lookup(lv, z["coords_s3"], r)), f"{mode}: lookup vs oracle"
