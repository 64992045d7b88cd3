#!/usr/bin/env python3
"""Role timeline of the warp-specialized fused lookup + convc1 kernel from the mo_wsst lab build:
per workgroup, cycles its producer wave 0 spends producing / waiting at the tile barrier and its
consumer wave 4 consuming / waiting, and the steps.  usage: tools/mostamps.py LIB"""
import ctypes
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import eraft_amd  # noqa: E402
from eraft_amd import _lib  # noqa: E402

L = ctypes.CDLL(os.path.join(ROOT, sys.argv[1]))
for name, (res, args) in _lib.SYMBOLS.items():
    if hasattr(L, name):
        getattr(L, name).restype = res
        getattr(L, name).argtypes = args
_lib._lib = L
B, H, W = 16, 60, 80
g = torch.Generator(device="cuda").manual_seed(0)
with torch.no_grad():
    f1 = torch.randn((B, 256, H, W), generator=g, device="cuda")
    f2 = torch.randn((B, 256, H, W), generator=g, device="cuda")
    blk = eraft_amd.CorrBlock(f1, f2)
    c = (eraft_amd.coords_grid(B, H, W, device="cuda") + 2.0 * torch.randn((B, 2, H, W), generator=g, device="cuda")).contiguous()
    wgt = torch.randn((256, 324, 1, 1), generator=g, device="cuda") * 0.05
    t0 = time.time()
    while time.time() - t0 < 2.0:
        for _ in range(20):
            blk.lookup_conv1x1_relu(c, wgt)
        torch.cuda.synchronize()
n = 256
buf = (ctypes.c_uint64 * (8 * n))()
assert L.ecorr_lab_mostamps(buf, n) == 0
a = np.frombuffer(buf, dtype=np.uint64).reshape(n, 8).astype(np.float64)
pb, pw, ps, cb, cwt, cs, tot = a[:, 0], a[:, 1], a[:, 2], a[:, 3], a[:, 4], a[:, 5], a[:, 6]
print(f"steps median {np.median(ps):.0f}; total cycles median {np.median(tot):.0f}")
print(f"producer: busy {np.median(pb / ps):.0f} cyc/step, barrier wait {np.median(pw / ps):.0f}")
print(f"consumer: busy {np.median(cb / cs):.0f} cyc/step, barrier wait {np.median(cwt / cs):.0f}")
