"""GPU parity of the HIP CorrBlock path against the oracle and the reference goldens.

Bars (BASELINE.json north_star):
  * level 0 (GEMM): normwise, max|d| / rms(ref) <= 1e-5 against the fp64 oracle and the
    reference's own values;
  * pyramid levels 1..L-1: bit-exact against the oracle pooling OUR level 0;
  * lookup: bit-exact (NaN-payload aside) against the reference outputs when fed the REFERENCE
    pyramid, and against the oracle on our own pyramid;
  * bilinear_sampler / coords_grid: bit-exact against the reference.
All calls go through libecorr.so (ctypes, C ABI); nothing here can fall back to ATen.
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

CORR_CASES = sorted(glob.glob(os.path.join(GOLDEN, "corr_*.npz")))
GEMM_TOL = 1e-5
DEV = "cuda:0"


def _load(path):
    z = np.load(path)
    return {k: z[k] for k in z.files}


@pytest.fixture(scope="module")
def ea():
    if not torch.cuda.is_available():
        pytest.fail("no HIP device visible: GPU tests must run on the MI355X box")
    import eraft_amd
    eraft_amd.lib()
    return eraft_amd


def _lookup_on(ea, levels, coords, radius):
    """ecorr_lookup on an externally supplied pyramid (list of [N, h, w] numpy levels)."""
    from eraft_amd import _lib
    from eraft_amd.layout import pack
    B, _, H, W = coords.shape
    flat = pack([torch.from_numpy(np.ascontiguousarray(lv)) for lv in levels], H, W).to(DEV)
    c = torch.from_numpy(np.ascontiguousarray(coords)).to(DEV)
    K = 2 * radius + 1
    out = torch.empty((B, len(levels) * K * K, H, W), dtype=torch.float32, device=DEV)
    _lib.check(_lib.lib().ecorr_lookup(flat.data_ptr(), c.data_ptr(), B, H, W, H * W, len(levels),
                                       radius, out.data_ptr(), _lib.stream_of(out)), "lookup")
    torch.cuda.synchronize()
    return out.cpu().numpy()


@pytest.mark.parametrize("path", CORR_CASES, ids=lambda p: os.path.basename(p)[:-4])
def test_golden_case(ea, path):
    z = _load(path)
    B, D, H, W, L, r, seed = (int(z[k]) for k in ("B", "D", "H", "W", "L", "r", "seed"))
    f1, f2 = prng.normal(seed, (B, D, H, W)), prng.normal(seed + 1, (B, D, H, W))
    with torch.no_grad():
        blk = ea.CorrBlock(torch.from_numpy(f1).to(DEV), torch.from_numpy(f2).to(DEV),
                           num_levels=L, radius=r)
        torch.cuda.synchronize()
    ours = [lv[:, 0].cpu().numpy() for lv in blk.corr_pyramid]
    assert [o.shape for o in ours] == [z[f"level{i}"].shape for i in range(L)]
    # GEMM: normwise against the reference and against the fp64 oracle
    assert oracle.normwise_err(ours[0], z["level0"]) <= GEMM_TOL
    assert oracle.normwise_err(ours[0], oracle.corr_level0(f1, f2)) <= GEMM_TOL
    # pooling bit-exact on our own level 0
    ref_levels = oracle.pyramid_from_level0(ours[0], L)
    for i in range(1, L):
        assert oracle.same_bits(ours[i], ref_levels[i]), f"level {i}"
    golden_levels = [z[f"level{i}"] for i in range(L)]
    for s in [k[len("coords_"):] for k in z if k.startswith("coords_")]:
        c = z[f"coords_{s}"]
        # bit-exact vs the reference when fed the reference's pyramid
        got = _lookup_on(ea, golden_levels, c, r)
        assert oracle.same_bits(got, z[f"out_{s}"]), f"{s}: vs reference"
        # full HIP path (our pyramid) bit-exact vs the oracle on that pyramid
        with torch.no_grad():
            o = blk(torch.from_numpy(c).to(DEV)).cpu().numpy()
        assert oracle.same_bits(o, oracle.lookup(ours, c, r)), f"{s}: vs oracle"


def test_static_corr(ea):
    f1, f2 = prng.normal(5, (2, 64, 6, 10)), prng.normal(6, (2, 64, 6, 10))
    with torch.no_grad():
        v = ea.CorrBlock.corr(torch.from_numpy(f1).to(DEV), torch.from_numpy(f2).to(DEV))
    assert tuple(v.shape) == (2, 6, 10, 1, 6, 10)
    ref = oracle.corr_level0(f1, f2).reshape(2, 6, 10, 1, 6, 10)
    assert oracle.normwise_err(v.cpu().numpy(), ref) <= GEMM_TOL


def test_sampler_and_coords_grid(ea):
    z = _load(os.path.join(GOLDEN, "sampler.npz"))
    img = torch.from_numpy(z["img"]).to(DEV)
    g = torch.from_numpy(z["grid"]).to(DEV)
    with torch.no_grad():
        out, mask = ea.bilinear_sampler(img, g, mask=True)
        out2 = ea.bilinear_sampler(img, g)
        cg = ea.coords_grid(2, 3, 5, device=DEV)
    assert oracle.same_bits(out.cpu().numpy(), z["out"])
    assert oracle.same_bits(mask.cpu().numpy(), z["mask"])
    assert oracle.same_bits(out2.cpu().numpy(), z["out_nomask"])
    assert oracle.same_bits(cg.cpu().numpy(), z["coords_grid_2_3_5"])
    assert oracle.same_bits(ea.coords_grid(2, 3, 5).numpy(), z["coords_grid_2_3_5"])


@pytest.mark.parametrize("name", ["dsec60x80", "mvsec32x32"])
def test_large_against_reference_samples(ea, name):
    z = _load(os.path.join(GOLDEN, f"large_{name}.npz"))
    B, D, H, W, seed = (int(z[k]) for k in ("B", "D", "H", "W", "seed"))
    f1, f2 = prng.normal(seed, (B, D, H, W)), prng.normal(seed + 1, (B, D, H, W))
    coords = prng.coords_with_flow(int(z["coords_seed"]), B, H, W, 3.0)
    with torch.no_grad():
        blk = ea.CorrBlock(torch.from_numpy(f1).to(DEV), torch.from_numpy(f2).to(DEV))
        out = blk(torch.from_numpy(coords).to(DEV)).cpu().numpy()
    l0 = blk.corr_pyramid[0].reshape(B * H * W, H * W)
    vals = l0[torch.from_numpy(z["l0_rows"]).to(DEV), torch.from_numpy(z["l0_cols"]).to(DEV)].cpu().numpy()
    assert np.max(np.abs(vals.astype(np.float64) - z["l0_vals"])) / float(z["l0_rms"]) <= GEMM_TOL
    # lookup samples differ from the reference only through level-0 rounding: normwise too
    got = out.reshape(-1)[z["out_idx"]]
    assert np.max(np.abs(got.astype(np.float64) - z["out_vals"])) / float(z["out_rms"]) <= GEMM_TOL
    # and the lookup is bit-exact against the oracle on our own pyramid
    levels = [lv[:, 0].cpu().numpy() for lv in blk.corr_pyramid]
    assert oracle.same_bits(out, oracle.lookup(levels, coords, 4))


# BASELINE configs at their per-GPU batch: configs[1] DSEC B=16 (the bench line), configs[2] MVSEC
# 32 x 32 at B=64, configs[3]'s per-GPU slice (DSEC B=256 over 8 GPUs = B=32), configs[4]'s whole
# 1280 x 720 job (fmap 92 x 160 after the 736-row pad, B=4; the row-sharded ranks build slabs of it,
# bitwise its rows: tests/test_rowshard_gpu.py)
BATCH_CONFIGS = [(16, 60, 80, 11, 2), (64, 32, 32, 31, 2), (32, 60, 80, 41, 2), (4, 92, 160, 61, 16)]


@pytest.mark.parametrize("cfg", BATCH_CONFIGS, ids=["c2_dsec_b16", "c3_mvsec_b64", "c4_slice_dsec_b32",
                                                   "c5_92x160_b4"])
def test_bench_config_full_size(ea, cfg):
    """Pooling and the full lookup bit-exact vs the oracle at the config's full size (D = 256, the
    split build's <true, 16> K loop), GEMM normwise on sampled query rows of every batch item,
    lookups on two coordinate fields (coords_grid + i.i.d. N(0, 3 px) flow, and the
    bench's smooth warm-start field), repeat calls bitwise deterministic."""
    B, H, W, seed, per_b = cfg
    D = 256
    f1 = torch.from_numpy(prng.normal(seed, (B, D, H, W))).to(DEV)
    f2 = torch.from_numpy(prng.normal(seed + 1, (B, D, H, W))).to(DEV)
    fields = {"iid3": prng.coords_with_flow(seed + 2, B, H, W, 3.0),
              "smooth": prng.coords_smooth(seed + 3, B, H, W)}
    outs = {}
    with torch.no_grad():
        blk = ea.CorrBlock(f1, f2)
        for name, c in fields.items():
            ct = torch.from_numpy(c).to(DEV)
            outs[name] = blk(ct)
            assert torch.equal(outs[name], blk(ct)), name
        torch.cuda.synchronize()
    levels = [lv[:, 0].cpu().numpy() for lv in blk.corr_pyramid]
    ref_levels = oracle.pyramid_from_level0(levels[0], 4)
    for i in range(1, 4):
        assert oracle.same_bits(levels[i], ref_levels[i]), f"level {i}"
    del ref_levels
    # sampled rows: per_b per batch item (spread through the map, first and last query included)
    Q = H * W
    rows = [b * Q + p for b in range(B) for p in
            sorted({0, Q - 1 - b} | {(b * 997 + k * 7919) % Q for k in range(per_b - 2)})]
    f1n, f2n = f1.cpu().numpy(), f2.cpu().numpy()
    for rw in rows:
        b, p = divmod(int(rw), Q)
        ref = oracle.corr_level0(f1n[b:b + 1], f2n[b:b + 1], p, 1)[0]
        assert oracle.normwise_err(levels[0][rw], ref) <= GEMM_TOL, f"row {rw}"
    for name, c in fields.items():
        assert oracle.same_bits(outs[name].cpu().numpy(), oracle.lookup(levels, c, 4)), name


def test_errors_match_reference(ea):
    with torch.no_grad():
        for (h, w) in [(4, 4), (2, 40), (6, 6)]:   # tests/golden/errors.json: RuntimeError
            f = torch.zeros(1, 16, h, w, device=DEV)
            with pytest.raises(RuntimeError):
                ea.CorrBlock(f, f)
        f = torch.zeros(1, 16, 8, 8, device=DEV)
        with pytest.raises(RuntimeError):   # non-contiguous: the reference's .view raises
            ea.CorrBlock(f.transpose(2, 3), f.transpose(2, 3))
        with pytest.raises(RuntimeError):   # CPU tensors: no CPU fallback
            ea.CorrBlock(f.cpu(), f.cpu())
        blk = ea.CorrBlock(f, f)
        with pytest.raises(RuntimeError):
            blk(torch.zeros(1, 2, 8, 9, device=DEV))
    g = torch.zeros(1, 16, 8, 8, device=DEV, requires_grad=True)
    with pytest.raises(RuntimeError):
        ea.CorrBlock(g, g)


# Tile-geometry sweep: H % 8 = 0..7 (regular 8 x 16 tiles, 4 x 32 band tiles for remainders 1-4,
# padded tile rows for 5-7), widths that are / are not multiples of 4, 16 and 32 (vector and
# scalar loaders, partial band tiles), 1..5 levels (levels >= 4 pooled by pool2_kernel), tiled
# and compact level formats.
GEOMETRY = [(1, 32, 60, 80, 4), (1, 16, 17, 20, 4), (2, 16, 19, 24, 3), (1, 8, 20, 36, 4),
            (1, 8, 21, 40, 2), (1, 16, 22, 18, 4), (1, 8, 23, 16, 1), (1, 16, 24, 44, 4),
            (1, 8, 25, 33, 4), (2, 16, 36, 52, 5), (1, 8, 12, 100, 4), (1, 16, 92, 160, 4)]


@pytest.mark.parametrize("geom", GEOMETRY, ids=lambda g: "b%d_d%d_%dx%d_l%d" % g)
def test_geometry_vs_oracle(ea, geom):
    B, D, H, W, L = geom
    f1, f2 = prng.normal(21, (B, D, H, W)), prng.normal(22, (B, D, H, W))
    coords = prng.coords_with_flow(23, B, H, W, 2.5)
    with torch.no_grad():
        blk = ea.CorrBlock(torch.from_numpy(f1).to(DEV), torch.from_numpy(f2).to(DEV), num_levels=L)
        out = blk(torch.from_numpy(coords).to(DEV)).cpu().numpy()
    levels = [lv[:, 0].cpu().numpy() for lv in blk.corr_pyramid]
    if H * W <= 2500:
        assert oracle.normwise_err(levels[0], oracle.corr_level0(f1, f2)) <= GEMM_TOL
    else:   # sampled query rows at the larger shapes
        for rw in range(0, B * H * W, 613):
            b, p = divmod(rw, H * W)
            ref = oracle.corr_level0(f1[b:b + 1], f2[b:b + 1], p, 1)[0]
            assert oracle.normwise_err(levels[0][rw], ref) <= GEMM_TOL
    ref_levels = oracle.pyramid_from_level0(levels[0], L)
    for i in range(1, L):
        assert oracle.same_bits(levels[i], ref_levels[i]), f"level {i}"
    assert oracle.same_bits(out, oracle.lookup(levels, coords, 4))


# Column-pair window staging (every level width even, lookup_stage.h) vs single columns (some level
# width odd): floor flips of integer coordinates, half-pixel shifts, windows hanging over every
# image edge, and NaN / inf / huge coordinates (the direct path), bit-exact vs the oracle.
@pytest.mark.parametrize("shape", [(2, 32, 24, 32, 4), (1, 32, 20, 36, 4), (1, 16, 60, 80, 4)],
                         ids=["pairs_24x32", "single_20x36", "pairs_60x80"])
def test_lookup_adversarial_coords(ea, shape):
    B, D, H, W, L = shape
    f1, f2 = prng.normal(51, (B, D, H, W)), prng.normal(52, (B, D, H, W))
    ys, xs = np.meshgrid(np.arange(H, dtype=np.float32), np.arange(W, dtype=np.float32), indexing="ij")
    grid = np.broadcast_to(np.stack([xs, ys])[None], (B, 2, H, W)).astype(np.float32)
    edge = grid.copy()
    edge[:, 0, :, :4] = np.float32(-4.5) - edge[:, 0, :, :4]              # left of the image
    edge[:, 0, :, -4:] += np.float32(3.7)                                  # right of it
    edge[:, 1, :2] = np.float32(-0.999)                                    # just above
    edge[:, 1, -2:] = np.float32(H - 1) + np.float32(2.25)                 # below
    odd = prng.coords_with_flow(53, B, H, W, 6.0).astype(np.float32)   # 6-px random flow
    odd[0, :, 0, :6] = np.array([[np.nan, np.inf, -np.inf, 1e9, -7.0e5, 3.0e7]] * 2, dtype=np.float32)
    sets = {"int": grid, "half": grid + np.float32(0.5), "edge": edge, "odd": odd}
    with torch.no_grad():
        blk = ea.CorrBlock(torch.from_numpy(f1).to(DEV), torch.from_numpy(f2).to(DEV), num_levels=L)
        levels = [lv[:, 0].cpu().numpy() for lv in blk.corr_pyramid]
        for name, c in sets.items():
            c = np.ascontiguousarray(c, dtype=np.float32)
            out = blk(torch.from_numpy(c).to(DEV)).cpu().numpy()
            assert oracle.same_bits(out, oracle.lookup(levels, c, 4)), name


# The reference's own outputs through the column-pair staging: the golden cases' leading levels whose
# widths are all even (t16x24: 24, 12, 6; b2_8x12: 12, 6) looked up alone give the reference's
# leading channels, bit-exact, for every golden coordinate set (integer, near-integer, special).
@pytest.mark.parametrize("name,L", [("corr_t16x24", 3), ("corr_b2_8x12", 2)])
def test_golden_pair_staging(ea, name, L):
    z = _load(os.path.join(GOLDEN, name + ".npz"))
    r, W = int(z["r"]), int(z["W"])
    assert all((W >> i) % 2 == 0 for i in range(L))   # the column-pair path
    K = 2 * r + 1
    levels = [z[f"level{i}"] for i in range(L)]
    for s in [k[len("coords_"):] for k in z if k.startswith("coords_")]:
        got = _lookup_on(ea, levels, z[f"coords_{s}"], r)
        assert oracle.same_bits(got, z[f"out_{s}"][:, :L * K * K]), s


def test_degenerate_shapes_as_reference(ea):
    """tests/golden/degenerate.npz (make_golden_degenerate.py): D = 0 features -> the reference's
    NaN volumes, sampled bit for bit (NaN where a corner lies inside a level, 0 where none does);
    an empty batch or map raises RuntimeError as the reference's reshape / avg_pool2d do."""
    z = np.load(os.path.join(GOLDEN, "degenerate.npz"))
    coords = torch.from_numpy(z["d0/coords"]).to(DEV)
    B, _, H, W = coords.shape
    f = torch.zeros((B, 0, H, W), device=DEV)
    with torch.no_grad():
        got = ea.CorrBlock(f, f.clone(), num_levels=2, radius=1)(coords).cpu().numpy()
    assert oracle.same_bits(got, z["d0/out"])
    for shape in ((0, 8, H, W), (2, 8, 0, W)):
        with pytest.raises(RuntimeError):
            ea.CorrBlock(torch.zeros(shape, device=DEV), torch.zeros(shape, device=DEV), num_levels=2, radius=1)
