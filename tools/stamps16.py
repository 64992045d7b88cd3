#!/usr/bin/env python3
"""Per-block timing of build_split16_kernel from the st16 lab build (tools/lab_build.py st16):
prologue / K loop / epilogue durations, in-loop and epilogue clocks, mid-barrier cycles.  The
builds run back to back for ~2 s first (MI355X_MICROARCH.md: clock under load).
  python tools/stamps16.py tools/st16_lab/e-raft_amd/libecorr.so"""
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
    getattr(L, name).restype = res
    getattr(L, name).argtypes = args
_lib._lib = L
B, H, W = 16, 60, 80
g = torch.Generator(device="cuda").manual_seed(0)
with torch.no_grad():
    f1 = torch.randn((B, 256, H, W), generator=g, device="cuda")
    f2 = torch.randn((B, 256, H, W), generator=g, device="cuda")
    t0 = time.time()
    while time.time() - t0 < 2.0:
        for _ in range(50):
            eraft_amd.CorrBlock(f1, f2)
        torch.cuda.synchronize()
n = B * 19 * 38
buf = (ctypes.c_uint64 * (8 * n))()
assert L.ecorr_lab_stamps16(buf, n) == 0
a = np.frombuffer(buf, dtype=np.uint64).reshape(n, 8).astype(np.float64)
med = lambda x: float(np.median(x))
print(f"blocks {n}")
print(f"prologue us        median {med(a[:, 0]) / 100:.2f}")
print(f"K loop us          median {med(a[:, 2]) / 100:.2f}  cycles {med(a[:, 1]):.0f}  clock {med(a[:, 1] / (a[:, 2] * 10e-9)) / 1e9:.3f} GHz")
print(f"epilogue us        median {med(a[:, 4]) / 100:.2f}  cycles {med(a[:, 3]):.0f}  clock {med(a[:, 3] / np.maximum(a[:, 4], 1) / 10e-9) / 1e9:.3f} GHz")
print(f"mid wait+barrier   median cycles {med(a[:, 5]):.0f} (7 per block)")
print(f"MFMA cycles per wave per tile: {768 * 16}")
