#!/usr/bin/env python3
"""Capture golden vectors for the SURVEY §8f "next" rows from the imported reference.

Run ONLY in the build container (the reference does not exist on the GPU box):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_next.py

Like make_golden.py: the reference (/root/reference, wzygzlm/E-RAFT) is imported read-only and run
on torch-CPU; inputs are drawn from tests/prng.py and stored alongside the reference's outputs.

  next_splat.npz    utils/image_utils.py forward_interpolate_pytorch (:50-83) on several flow
                    fields (sub-pixel, large/out-of-image, converging = many collisions, integer =
                    floor == ceil, NaN/inf, 3-D input) and grid_sample_values (:10-47) on scattered
                    points incl. the empty set.
"""
import os
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))          # tests/ (prng)
sys.path.insert(0, "/root/reference")

import numpy as np  # noqa: E402
import torch  # noqa: E402

import prng  # noqa: E402
from utils.image_utils import forward_interpolate_pytorch, grid_sample_values  # noqa: E402  (reference)

torch.set_num_threads(8)


def splat_cases():
    cases = {}
    cases["fi_dsec_s3"] = prng.normal(100, (2, 2, 60, 80), 3.0)
    cases["fi_s30"] = prng.normal(101, (1, 2, 24, 32), 30.0)
    h, w = 36, 44
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    conv = np.stack([(21.3 - xx) * 0.93, (17.6 - yy) * 0.93])[None]
    cases["fi_converge"] = (conv + prng.normal(102, (1, 2, h, w), 0.05)).astype(np.float32)
    cases["fi_int"] = np.round(prng.normal(103, (2, 2, 20, 28), 2.0)).astype(np.float32)
    f = prng.normal(104, (1, 2, 16, 24), 2.0)
    f[0, 0, 3, 5] = np.nan
    f[0, 1, 7, 9] = np.inf
    f[0, 0, 10, 2] = -np.inf
    f[0, 1, 0, 0] = 1e30
    cases["fi_special"] = f
    cases["fi_3d"] = prng.normal(105, (2, 12, 17), 1.5)   # [2, H, W] input -> [1, 2, H, W]
    cases["fi_mvsec"] = prng.normal(106, (4, 2, 32, 32), 1.5)
    out = {}
    for k, flow in cases.items():
        ref = forward_interpolate_pytorch(torch.from_numpy(flow.copy())).numpy()
        out[f"{k}/flow"] = flow
        out[f"{k}/out"] = ref
    # grid_sample_values on scattered points (n != h*w, some outside)
    for k, (n, h, w, seed) in {"gsv_scatter": (5000, 30, 40, 110), "gsv_dense": (20000, 9, 11, 111),
                               "gsv_empty": (0, 5, 7, 112)}.items():
        x = prng.uniform(seed, (n,), -3.0, w + 2.0)
        y = prng.uniform(seed + 1, (n,), -3.0, h + 2.0)
        z = prng.normal(seed + 2, (n,))
        inp = np.stack([x, y, z]).astype(np.float32).reshape(3, n)
        v, m = grid_sample_values(torch.from_numpy(inp.copy()), h, w)
        out[f"{k}/input"] = inp
        out[f"{k}/hw"] = np.array([h, w], dtype=np.int64)
        out[f"{k}/values"] = v.numpy()
        out[f"{k}/valid"] = m.numpy()
    return out


def main():
    np.savez_compressed(os.path.join(HERE, "next_splat.npz"), **splat_cases())
    print("wrote next_splat.npz")


if __name__ == "__main__":
    main()
