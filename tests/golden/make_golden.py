#!/usr/bin/env python3
"""Capture golden vectors from the imported reference (wzygzlm/E-RAFT at /root/reference).

Run ONLY in the build container (the reference does not exist on the GPU box):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

The reference is imported read-only (sys.dont_write_bytecode, sys.path insert) and exercised on
torch-CPU with ATen capability AVX512 (recorded in each fixture).  Inputs come from tests/prng.py
(bit-reproducible), so fixtures store seeds plus sha256 of the regenerated inputs, and the
reference's OUTPUTS.  What each fixture pins:

  corr_<case>.npz   CorrBlock build (corr.py:13-27) and lookups (corr.py:29-50) at small shapes:
                    full pyramid levels + full lookup outputs for several coordinate sets.
  large_<case>.npz  DSEC 60x80 and MVSEC 32x32: sampled level-0 entries (normwise GEMM parity) and
                    sampled lookup outputs plus output rms.
  sampler.npz       bilinear_sampler (utils.py:7-21) incl. mask=True; coords_grid (utils.py:24-27).
  e2e_<case>.npz    ERAFT.forward (eraft.py:88-145) with PRNG weights: final low-res flow and
                    (subsampled) final upsampled flow, standard and warm-start.
  errors.json       shapes on which the reference raises.
  nonfinite_corr.npz  the pyramid and a lookup from fmaps with +-inf / NaN entries (NONFINITE).
"""
import hashlib
import json
import os
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))          # tests/ (prng)
sys.path.insert(0, "/root/reference")

import numpy as np  # noqa: E402
import torch  # noqa: E402

import prng  # noqa: E402
from model.corr import CorrBlock  # noqa: E402  (reference)
from model.utils import bilinear_sampler, coords_grid  # noqa: E402  (reference)

torch.set_num_threads(8)
META = {"torch": torch.__version__, "cpu_capability": torch.backends.cpu.get_cpu_capability(),
        "reference": "/root/reference (wzygzlm/E-RAFT)"}


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def fmaps(seed, B, D, H, W):
    return prng.normal(seed, (B, D, H, W)), prng.normal(seed + 1, (B, D, H, W))


def coord_sets(B, H, W, seed):
    """Coordinate distributions exercising interior, zero padding and floor() flips."""
    sets = {
        "s0p5": prng.coords_with_flow(seed, B, H, W, 0.5),
        "s6": prng.coords_with_flow(seed + 1, B, H, W, 6.0),
        "s40": prng.coords_with_flow(seed + 2, B, H, W, 40.0),   # mostly out of bounds
        "int": prng.coords_with_flow(0, B, H, W, 0.0),          # standard mode, iteration 0
    }
    # integers nudged by a few ulps-worth: the unnormalize round trip flips floor() here
    base = prng.coords_with_flow(0, B, H, W, 0.0)
    pick = prng.uniform(seed + 3, (B, 2, H, W), 0.0, 8.0).astype(np.int64)
    eps = np.array([0.0, 1e-6, -1e-6, 2e-6, -2e-6, 5e-7, -5e-7, 0.5], dtype=np.float32)
    sets["nearint"] = (base + eps[pick]).astype(np.float32)
    return sets


def special_coords(B, H, W, seed):
    c = prng.coords_with_flow(seed, B, H, W, 3.0)
    flat = c.reshape(-1)
    specials = np.array([np.nan, np.inf, -np.inf, 1e6, -1e6, 3e38, -0.0, 0.0, -0.5, -1.0,
                         W - 1, W, H - 1, H, 1e-30, 8388608.0, 16777217.0, -4.0, 4.0],
                        dtype=np.float32)
    idx = (np.arange(specials.size) * 37 + 5) % flat.size
    flat[idx] = specials
    flat[(idx + 11) % flat.size] = specials[::-1]
    return c


def run_corr_case(name, B, D, H, W, L, r, seed, extra_coords=None):
    f1, f2 = fmaps(seed, B, D, H, W)
    blk = CorrBlock(torch.from_numpy(f1), torch.from_numpy(f2), num_levels=L, radius=r)
    out = {"B": B, "D": D, "H": H, "W": W, "L": L, "r": r, "seed": seed,
           "sha_fmap1": sha(f1), "sha_fmap2": sha(f2)}
    for i, lv in enumerate(blk.corr_pyramid):
        out[f"level{i}"] = lv.numpy()[:, 0].copy()
    sets = coord_sets(B, H, W, seed + 100)
    if extra_coords is not None:
        sets.update(extra_coords)
    for cname, c in sets.items():
        o = blk(torch.from_numpy(c)).numpy()
        out[f"coords_{cname}"] = c
        out[f"out_{cname}"] = o
    np.savez_compressed(os.path.join(HERE, f"corr_{name}.npz"), **{
        k: (np.asarray(v) if not isinstance(v, str) else np.asarray(v)) for k, v in out.items()})
    print(f"corr_{name}: levels {[out[f'level{i}'].shape for i in range(L)]} sets {list(sets)}")


# non-finite fmap entries: (tensor, batch, channel, row, col, value); chosen so that the reference's
# fp32 GEMM (corr.py:58) yields +-inf rows / columns, inf * 0 = NaN, +inf + -inf = NaN and NaN
NONFINITE = [("f1", 0, 5, 2, 3, np.inf), ("f1", 0, 9, 7, 10, np.nan), ("f2", 0, 17, 4, 14, -np.inf),
             ("f2", 0, 33, 9, 5, np.inf), ("f1", 0, 33, 11, 1, 0.0), ("f2", 0, 40, 10, 12, np.nan),
             ("f1", 0, 60, 0, 0, np.inf), ("f2", 0, 60, 1, 1, np.inf), ("f1", 0, 61, 0, 0, np.inf),
             ("f2", 0, 61, 1, 1, -2.0), ("f1", 1, 7, 8, 15, -np.inf), ("f2", 1, 100, 3, 3, np.inf)]


def run_nonfinite():
    """nonfinite_corr.npz: the pyramid and one lookup from fmaps holding +-inf and NaN entries
    (fmaps = fmaps(seed) with `entries` [tensor 0/1, b, d, y, x, value] written in)."""
    B, D, H, W, L, r, seed = 2, 256, 12, 16, 4, 4, 90
    f1, f2 = fmaps(seed, B, D, H, W)
    for which, b, d, y, x, v in NONFINITE:
        (f1 if which == "f1" else f2)[b, d, y, x] = np.float32(v)
    blk = CorrBlock(torch.from_numpy(f1), torch.from_numpy(f2), num_levels=L, radius=r)
    ent = np.array([[0 if w == "f1" else 1, b, d, y, x, v] for w, b, d, y, x, v in NONFINITE], dtype=np.float64)
    out = {"B": B, "D": D, "H": H, "W": W, "L": L, "r": r, "seed": seed, "entries": ent,
           "sha_fmap1": sha(f1), "sha_fmap2": sha(f2)}
    for i, lv in enumerate(blk.corr_pyramid):
        out[f"level{i}"] = lv.numpy()[:, 0].copy()
    c = prng.coords_with_flow(seed + 100, B, H, W, 3.0)
    out["coords_s3"] = c
    out["out_s3"] = blk(torch.from_numpy(c)).numpy()
    np.savez_compressed(os.path.join(HERE, "nonfinite_corr.npz"), **out)
    l0 = out["level0"]
    print(f"nonfinite_corr: level0 +inf {int(np.isposinf(l0).sum())} -inf {int(np.isneginf(l0).sum())} "
          f"NaN {int(np.isnan(l0).sum())}")


def run_large_case(name, B, H, W, seed, n_samples=16384):
    D = 256
    f1, f2 = fmaps(seed, B, D, H, W)
    blk = CorrBlock(torch.from_numpy(f1), torch.from_numpy(f2), num_levels=4, radius=4)
    lv0 = blk.corr_pyramid[0].numpy().reshape(B * H * W, H * W)
    rng = np.random.default_rng(seed)
    rows = rng.integers(0, lv0.shape[0], n_samples)
    cols = rng.integers(0, lv0.shape[1], n_samples)
    coords = prng.coords_with_flow(seed + 7, B, H, W, 3.0)
    o = blk(torch.from_numpy(coords)).numpy()
    oi = rng.integers(0, o.size, n_samples)
    np.savez_compressed(
        os.path.join(HERE, f"large_{name}.npz"), B=B, D=D, H=H, W=W, seed=seed,
        sha_fmap1=sha(f1), sha_fmap2=sha(f2),
        l0_rows=rows, l0_cols=cols, l0_vals=lv0[rows, cols], l0_rms=np.sqrt(np.mean(
            lv0.astype(np.float64) ** 2)),
        coords_seed=seed + 7, sha_coords=sha(coords),
        out_idx=oi, out_vals=o.reshape(-1)[oi],
        out_rms=np.sqrt(np.mean(o.astype(np.float64) ** 2)),
        level_rms=np.array([np.sqrt(np.mean(lv.numpy().astype(np.float64) ** 2))
                            for lv in blk.corr_pyramid]))
    print(f"large_{name}: level0 rms {np.sqrt(np.mean(lv0.astype(np.float64)**2)):.4f}")


def run_sampler():
    img = prng.normal(900, (2, 3, 7, 9))
    g = prng.uniform(901, (2, 5, 6, 2), -3.0, 11.0)
    out, mask = bilinear_sampler(torch.from_numpy(img), torch.from_numpy(g), mask=True)
    out2 = bilinear_sampler(torch.from_numpy(img), torch.from_numpy(g))
    cg = coords_grid(2, 3, 5).numpy()
    np.savez_compressed(os.path.join(HERE, "sampler.npz"), img=img, grid=g, out=out.numpy(),
                        mask=mask.numpy(), out_nomask=out2.numpy(), coords_grid_2_3_5=cg)
    print("sampler: out", tuple(out.shape), "mask", tuple(mask.shape))


def run_errors():
    errs = {}
    for (H, W) in [(4, 4), (2, 40), (6, 6)]:
        f1, f2 = fmaps(5, 1, 16, H, W)
        try:
            CorrBlock(torch.from_numpy(f1), torch.from_numpy(f2))
            errs[f"{H}x{W}"] = None
        except Exception as e:  # noqa: BLE001 - record the reference's exception type
            errs[f"{H}x{W}"] = type(e).__name__
    with open(os.path.join(HERE, "errors.json"), "w") as fh:
        json.dump(errs, fh, indent=1, sort_keys=True)
    print("errors:", errs)


# ---------------------------------------------------------------- e2e (eraft.py:88-145)
def prng_state_dict(template):
    """Deterministic weights for every state_dict entry (same recipe in tests/e2e_weights)."""
    sys.path.insert(0, os.path.dirname(HERE))
    from e2e_weights import make_state_dict  # noqa: E402
    return make_state_dict(template)


def run_e2e(name, H, W, bins, subtype, seed, warm, up_stride):
    from model.eraft import ERAFT  # reference
    torch.manual_seed(0)
    net = ERAFT({"subtype": subtype}, n_first_channels=bins)
    net.load_state_dict(prng_state_dict(net.state_dict()))
    net.eval()
    im1 = prng.normal(seed, (1, bins, H, W))
    im2 = prng.normal(seed + 1, (1, bins, H, W))
    flow_init = None
    if warm:
        fi = prng.normal(seed + 2, (1, 2, H // 8, W // 8), 1.5)
        flow_init = torch.from_numpy(fi)
    with torch.no_grad():
        low, ups = net(torch.from_numpy(im1), torch.from_numpy(im2), iters=12, flow_init=flow_init)
    up = ups[-1].numpy()
    rec = dict(H=H, W=W, bins=bins, subtype=subtype, seed=seed, warm=warm, up_stride=up_stride,
               sha_im1=sha(im1), sha_im2=sha(im2), flow_low=low.numpy(),
               flow_up=up[:, :, ::up_stride, ::up_stride].copy(),
               flow_up_first=ups[0].numpy()[:, :, ::up_stride, ::up_stride].copy())
    if warm:
        rec["flow_init"] = fi
    np.savez_compressed(os.path.join(HERE, f"e2e_{name}.npz"), **rec)
    print(f"e2e_{name}: |flow_low| mean {np.abs(low.numpy()).mean():.3f}")


def main():
    if "--e2e-only" in sys.argv:
        return run_all_e2e()
    if "--nonfinite-only" in sys.argv:
        return run_nonfinite()
    with open(os.path.join(HERE, "meta.json"), "w") as fh:
        json.dump(META, fh, indent=1)
    run_corr_case("t16x24", 1, 256, 16, 24, 4, 4, 10,
                  extra_coords={"special": special_coords(1, 16, 24, 77)})
    run_corr_case("b2_8x12", 2, 256, 8, 12, 4, 4, 20)         # level 3 is 1x1 -> NaN
    run_corr_case("odd18x22", 1, 256, 18, 22, 4, 4, 30)       # odd level dims, floor pooling
    run_corr_case("l3r2_d64", 1, 64, 12, 16, 3, 2, 40)        # num_levels=3, radius=2
    run_corr_case("d100_l2r3", 1, 100, 8, 16, 2, 3, 50)       # 1/sqrt(D) with sqrt exact, not 2^k
    run_corr_case("d3_l3r1", 2, 3, 8, 8, 3, 1, 60)            # sqrt(3) inexact
    run_corr_case("l1r0_d256", 1, 256, 6, 10, 1, 0, 70)       # single level, radius 0
    run_large_case("dsec60x80", 1, 60, 80, 1000)
    run_large_case("mvsec32x32", 2, 32, 32, 2000)
    run_nonfinite()
    run_sampler()
    run_errors()
    run_all_e2e()


def run_all_e2e():
    run_e2e("small_standard", 128, 160, 15, "standard", 3000, False, 1)
    run_e2e("small_warm", 128, 160, 15, "warm_start", 3100, True, 1)
    run_e2e("dsec_standard", 480, 640, 15, "standard", 3200, False, 4)
    run_e2e("mvsec_warm", 256, 256, 5, "warm_start", 3300, True, 1)


if __name__ == "__main__":
    main()
