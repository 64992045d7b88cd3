"""Pin the CPU oracle (oracle/ecorr_oracle.c) against golden vectors from the reference.

CPU-only.  Goldens: tests/golden/make_golden.py (imports /root/reference read-only, torch CPU,
AVX512).  Bars: pooling and lookup BIT-EXACT given the reference's own level 0; level 0 within the
normwise GEMM tolerance max|d|/rms <= 1e-5.
"""
import glob
import hashlib
import json
import os

import numpy as np
import pytest

import oracle
import prng
from conftest import GOLDEN

CORR_CASES = sorted(glob.glob(os.path.join(GOLDEN, "corr_*.npz")))
GEMM_TOL = 1e-5


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _load(path):
    z = np.load(path)  # allow_pickle=False (default): fixtures are plain arrays
    return {k: z[k] for k in z.files}


def _names(path):
    return os.path.basename(path)[:-4]


@pytest.fixture(scope="module", params=CORR_CASES, ids=_names)
def case(request):
    return _load(request.param)


def test_prng_regenerates_fixture_inputs(case):
    B, D, H, W, seed = (int(case[k]) for k in ("B", "D", "H", "W", "seed"))
    assert _sha(prng.normal(seed, (B, D, H, W))) == str(case["sha_fmap1"])
    assert _sha(prng.normal(seed + 1, (B, D, H, W))) == str(case["sha_fmap2"])


def test_level0_normwise(case):
    B, D, H, W, seed = (int(case[k]) for k in ("B", "D", "H", "W", "seed"))
    f1, f2 = prng.normal(seed, (B, D, H, W)), prng.normal(seed + 1, (B, D, H, W))
    got = oracle.corr_level0(f1, f2)
    assert got.shape == case["level0"].shape
    assert oracle.normwise_err(got, case["level0"]) <= GEMM_TOL


def test_pool_bit_exact(case):
    L = int(case["L"])
    levels = oracle.pyramid_from_level0(case["level0"], L)
    for i in range(1, L):
        assert oracle.same_bits(levels[i], case[f"level{i}"]), f"level {i}"


def test_lookup_bit_exact(case):
    L, r = int(case["L"]), int(case["r"])
    levels = [case[f"level{i}"] for i in range(L)]
    sets = [k[len("coords_"):] for k in case if k.startswith("coords_")]
    assert sets
    for s in sets:
        got = oracle.lookup(levels, case[f"coords_{s}"], r)
        ref = case[f"out_{s}"]
        assert got.shape == ref.shape
        assert oracle.same_bits(got, ref), f"coords set {s}: " + \
            f"{int(np.sum(got.view(np.uint32) != ref.view(np.uint32)))} mismatching words"


def test_lookup_nan_level_reproduced():
    """A 1-pixel level gives W-1 = 0 and NaN samples in the reference (SURVEY §7 hard part 7)."""
    c = _load(os.path.join(GOLDEN, "corr_b2_8x12.npz"))
    ref = c["out_s0p5"]
    assert np.isnan(ref[:, 243:]).all() and not np.isnan(ref[:, :243]).any()
    got = oracle.lookup([c[f"level{i}"] for i in range(4)], c["coords_s0p5"], 4)
    assert oracle.same_bits(got, ref)


def test_round_trip_flips_are_exercised():
    """The nearint set must actually contain floor() flips, or the bit-exact claim is weak."""
    c = _load(os.path.join(GOLDEN, "corr_t16x24.npz"))
    x = c["coords_nearint"][:, 0].astype(np.float32).reshape(-1)
    W = np.float32(c["W"])
    g = (np.float32(2) * x) / (W - np.float32(1)) - np.float32(1)
    ix = (g + np.float32(1)) * ((W - np.float32(1)) / np.float32(2))
    assert np.sum(np.floor(ix) != np.floor(x)) > 0


def test_sampler_and_coords_grid():
    z = _load(os.path.join(GOLDEN, "sampler.npz"))
    out, mask = oracle.bilinear_sampler(z["img"], z["grid"], mask=True)
    assert oracle.same_bits(out, z["out"])
    assert oracle.same_bits(mask, z["mask"])
    assert oracle.same_bits(oracle.bilinear_sampler(z["img"], z["grid"]), z["out_nomask"])
    assert oracle.same_bits(oracle.coords_grid(2, 3, 5), z["coords_grid_2_3_5"])


@pytest.mark.parametrize("name", ["dsec60x80", "mvsec32x32"])
def test_large_level0_samples(name):
    z = _load(os.path.join(GOLDEN, f"large_{name}.npz"))
    B, D, H, W, seed = (int(z[k]) for k in ("B", "D", "H", "W", "seed"))
    f1, f2 = prng.normal(seed, (B, D, H, W)), prng.normal(seed + 1, (B, D, H, W))
    assert _sha(f1) == str(z["sha_fmap1"])
    rows, cols = z["l0_rows"], z["l0_cols"]
    # only the sampled query rows are computed (keeps the CPU suite fast)
    uq = np.unique(rows)
    Q = H * W
    got = np.empty(rows.shape, dtype=np.float32)
    for qb in np.array_split(uq, max(1, uq.size // 512)):
        for q in qb:
            b, p = divmod(int(q), Q)
            row = oracle.corr_level0(f1[b:b + 1], f2[b:b + 1], p, 1)[0].reshape(-1)
            sel = rows == q
            got[sel] = row[cols[sel]]
    err = np.max(np.abs(got.astype(np.float64) - z["l0_vals"])) / float(z["l0_rms"])
    assert err <= GEMM_TOL


def test_reference_raise_shapes_recorded():
    with open(os.path.join(GOLDEN, "errors.json")) as fh:
        errs = json.load(fh)
    assert errs == {"2x40": "RuntimeError", "4x4": "RuntimeError", "6x6": "RuntimeError"}
    for k in errs:
        h, w = map(int, k.split("x"))
        with pytest.raises(RuntimeError):
            oracle.pyramid_from_level0(np.zeros((1, h, w), np.float32), 4)


def _nonfinite_fmaps(z):
    """fmaps of tests/golden/nonfinite_corr.npz: the PRNG fmaps with `entries` written in."""
    B, D, H, W, seed = (int(z[k]) for k in ("B", "D", "H", "W", "seed"))
    f1, f2 = prng.normal(seed, (B, D, H, W)), prng.normal(seed + 1, (B, D, H, W))
    for t, b, d, y, x, v in z["entries"]:
        (f1 if t == 0 else f2)[int(b), int(d), int(y), int(x)] = np.float32(v)
    assert _sha(f1) == str(z["sha_fmap1"]) and _sha(f2) == str(z["sha_fmap2"])   # (with the entries)
    return f1, f2


def finite_pattern_equal(got, ref):
    """Same +inf / -inf / NaN positions (no payload or sign-of-NaN comparison)."""
    return (np.array_equal(np.isnan(got), np.isnan(ref)) and np.array_equal(np.isposinf(got), np.isposinf(ref))
            and np.array_equal(np.isneginf(got), np.isneginf(ref)))


def test_nonfinite_oracle():
    """fmaps with +-inf and NaN entries (corr.py:58's fp32 GEMM: +-inf rows / columns, inf * 0 and
    inf - inf = NaN): the fp64 oracle reproduces the reference's non-finite pattern exactly and its
    finite values normwise; pooling and the lookup stay bit-exact on the reference's level 0."""
    z = _load(os.path.join(GOLDEN, "nonfinite_corr.npz"))
    f1, f2 = _nonfinite_fmaps(z)
    got = oracle.corr_level0(f1, f2)
    ref = z["level0"]
    assert np.isposinf(ref).any() and np.isneginf(ref).any() and np.isnan(ref).any()
    assert finite_pattern_equal(got, ref)
    fin = np.isfinite(ref)
    assert oracle.normwise_err(got[fin], ref[fin]) <= GEMM_TOL
    L, r = int(z["L"]), int(z["r"])
    levels = oracle.pyramid_from_level0(ref, L)
    for i in range(1, L):
        assert oracle.same_bits(levels[i], z[f"level{i}"]), f"level {i}"
    assert oracle.same_bits(oracle.lookup([z[f"level{i}"] for i in range(L)], z["coords_s3"], r), z["out_s3"])
