"""Pin the torch-CPU restatement (bench.py's cpu_baseline) bit-for-bit to the reference goldens."""
import glob
import os

import numpy as np
import pytest
import torch

import oracle
import prng
from conftest import GOLDEN
from torch_ref import TorchCpuCorrBlock

CASES = sorted(glob.glob(os.path.join(GOLDEN, "corr_*.npz")))


@pytest.mark.parametrize("path", CASES, ids=lambda p: os.path.basename(p)[:-4])
def test_torch_ref_matches_reference(path):
    z = np.load(path)
    B, D, H, W, L, r, seed = (int(z[k]) for k in ("B", "D", "H", "W", "L", "r", "seed"))
    f1, f2 = prng.normal(seed, (B, D, H, W)), prng.normal(seed + 1, (B, D, H, W))
    blk = TorchCpuCorrBlock(torch.from_numpy(f1), torch.from_numpy(f2), num_levels=L, radius=r)
    for i in range(L):   # same ATen sgemm as the reference on this host -> identical bits
        assert oracle.same_bits(blk.corr_pyramid[i][:, 0].numpy(), z[f"level{i}"])
    for k in z.files:
        if k.startswith("coords_"):
            s = k[len("coords_"):]
            assert oracle.same_bits(blk(torch.from_numpy(z[k])).numpy(), z[f"out_{s}"]), s


def test_torch_ref_splat_matches_reference():
    import torch_ref
    z = np.load(os.path.join(GOLDEN, "next_splat.npz"))
    for k in sorted(f.split("/")[0] for f in z.files if f.startswith("fi_") and f.endswith("/flow")):
        got = torch_ref.forward_interpolate_pytorch(torch.from_numpy(z[f"{k}/flow"])).numpy()
        assert oracle.same_bits(got, z[f"{k}/out"]), k


def test_torch_ref_voxel_matches_reference():
    from voxel_cases import DSEC_VOXEL, dsec_case
    import torch_ref
    z = np.load(os.path.join(GOLDEN, "next_voxel.npz"))
    torch.set_num_threads(1)
    try:
        for k, (n, C, H, W, seed) in DSEC_VOXEL.items():
            ev = {c: torch.from_numpy(v) for c, v in zip("ptxy", dsec_case(k, n, H, W, seed))}
            for norm in (0, 1):
                got = torch_ref.voxel_grid_dsec(ev, C, H, W, bool(norm)).numpy()
                assert oracle.same_bits(got, z[f"{k}/norm{norm}"]), (k, norm)
    finally:
        torch.set_num_threads(os.cpu_count() or 1)


def test_torch_ref_voxel_mvsec_matches_reference():
    """oracle/torch_ref.voxel_grid_mvsec (the bench's MVSEC reference leg) against the reference's
    own outputs: bit-exact accumulated and normalized grids; the out-of-range event raises."""
    from voxel_cases import MVSEC_VOXEL, mvsec_case
    import torch_ref
    z = np.load(os.path.join(GOLDEN, "next_voxel.npz"))
    torch.set_num_threads(1)
    try:
        for k, (n, C, H, W, seed) in MVSEC_VOXEL.items():
            ev = torch.from_numpy(mvsec_case(k, n, H, W, seed))
            if f"{k}/raises" in z.files:
                with pytest.raises((IndexError, RuntimeError)):
                    torch_ref.voxel_grid_mvsec(ev, C, H, W, True)
                continue
            for norm in (0, 1):
                got = torch_ref.voxel_grid_mvsec(ev, C, H, W, bool(norm)).numpy()
                assert oracle.same_bits(got, z[f"{k}/norm{norm}"]), (k, norm)
    finally:
        torch.set_num_threads(os.cpu_count() or 1)
