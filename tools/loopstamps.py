#!/usr/bin/env python3
"""K-loop breakdown from the loopstamps lab build: per block, cycles (s_memtime) in the DMA wait,
the barrier and the whole loop (wave 0), and wave 3's DMA wait.  usage: loopstamps.py LIB [N]"""
import ctypes, os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import eraft_amd  # noqa
from eraft_amd import _lib  # noqa
L = ctypes.CDLL(os.path.join(ROOT, sys.argv[1]))
for name, (res, args) in _lib.SYMBOLS.items():
    getattr(L, name).restype = res
    getattr(L, name).argtypes = args
_lib._lib = L
g = torch.Generator(device="cuda").manual_seed(0)
with torch.no_grad():
    f1 = torch.randn((16, 256, 60, 80), generator=g, device="cuda")
    f2 = torch.randn((16, 256, 60, 80), generator=g, device="cuda")
    for _ in range(3):
        eraft_amd.CorrBlock(f1, f2)
    torch.cuda.synchronize()
n = 11552
buf = (ctypes.c_uint64 * (5 * n))()   # ecorr_lab_stamps copies 5 words per block
assert L.ecorr_lab_stamps(buf, n) == 0
a = np.frombuffer(buf, dtype=np.uint64).reshape(n, 5).astype(np.float64)
for k, nm in enumerate(["wave0 dma wait", "wave0 barrier", "wave0 loop total", "loop realtime (10ns)", "wave0 q wait (qwait)"]):
    print(f"{nm:18s} cycles/block: median {np.median(a[:, k]):9.0f}  p10 {np.percentile(a[:, k], 10):9.0f}  p90 {np.percentile(a[:, k], 90):9.0f}")
print(f"MFMA cycles per wave per tile (384 x 32): {384 * 32}")
print(f"in-loop clock: {np.median(a[:, 2] / (a[:, 3] * 10e-9)) / 1e9:.3f} GHz (s_memtime / s_memrealtime)")
