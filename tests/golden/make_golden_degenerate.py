#!/usr/bin/env python3
"""Capture the reference CorrBlock's behaviour on degenerate shapes (model/corr.py:12-60).

Run ONLY in the build container (the reference does not exist on the GPU box):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_degenerate.py

  degenerate.npz   D = 0 feature channels: the reference builds 0 / sqrt(0) = NaN volumes and its
                   lookup returns NaN where a bilinear corner lies inside a level, 0 where all four
                   lie outside (zero padding) -- stored with its coords (PRNG, some far outside);
                   B = 0 and H = 0: the reference raises RuntimeError (recorded as the error text).
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
from model.corr import CorrBlock  # noqa: E402  (reference)
from model.utils import coords_grid  # noqa: E402  (reference)

torch.set_num_threads(1)
out = {}
B, H, W, L, R = 2, 6, 7, 2, 1
coords = coords_grid(B, H, W) + torch.from_numpy(prng.normal(801, (B, 2, H, W)) * np.float32(4.0))
f = torch.zeros((B, 0, H, W))
blk = CorrBlock(f, f.clone(), num_levels=L, radius=R)
out["d0/coords"] = coords.numpy()
out["d0/out"] = blk(coords).numpy()
for name, shape in (("b0", (0, 8, H, W)), ("h0", (2, 8, 0, W))):
    try:
        CorrBlock(torch.zeros(shape), torch.zeros(shape), num_levels=L, radius=R)(torch.zeros((shape[0], 2) + shape[2:]))
        out[f"{name}/raises"] = np.array("")
    except RuntimeError as e:
        out[f"{name}/raises"] = np.array(str(e)[:200])
np.savez_compressed(os.path.join(HERE, "degenerate.npz"), **out)
print({k: (v.shape, v.dtype) for k, v in out.items()})
