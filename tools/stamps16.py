#!/usr/bin/env python3
"""Per-block timeline of build_split16_kernel from the st16 lab build (tools/lab_build.py st16):
prologue / K loop / epilogue durations and clocks, per-CU concurrency, and the K loop's fitted
duration beside another block's loop, beside its epilogue, or alone (least squares over every
block).  The builds run back to back for ~2 s first (MI355X_MICROARCH.md: the clock under load).
  python tools/stamps16.py tools/st16_lab/e-raft_amd/libecorr.so [B H W]"""
import collections
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
    if hasattr(L, name):   # (a lab build of an older ABI lacks later symbols)
        getattr(L, name).restype = res
        getattr(L, name).argtypes = args
_lib._lib = L
B, H, W = (int(x) for x in sys.argv[2:5]) if len(sys.argv) > 4 else (16, 60, 80)
g = torch.Generator(device="cuda").manual_seed(0)
with torch.no_grad():
    f1 = torch.randn((B, 256, H, W), generator=g, device="cuda")
    f2 = torch.randn((B, 256, H, W), generator=g, device="cuda")
    t0 = time.time()
    while time.time() - t0 < 2.0:
        for _ in range(50):
            eraft_amd.CorrBlock(f1, f2)
        torch.cuda.synchronize()
nq = (H * W + 255) // 256
rem = H % 8
nreg = ((W + 15) // 16) * (H // 8 if 0 < rem <= 4 else (H + 7) // 8)
n = B * nq * (nreg + ((W + 31) // 32 if 0 < rem <= 4 else 0))
buf = (ctypes.c_uint64 * (8 * n))()
assert L.ecorr_lab_stamps16(buf, n) == 0
a = np.frombuffer(buf, dtype=np.uint64).reshape(n, 8).astype(np.int64)
ts, tl0, tl1, te = a[:, 0], a[:, 1], a[:, 2], a[:, 3]
cl, ce = a[:, 4].astype(np.float64), a[:, 5].astype(np.float64)
hw, xcc = a[:, 6], a[:, 7] & 0xF
cu = (hw >> 8) & 0xFF
us = lambda x: x / 100.0
med = lambda x: float(np.median(x))
print(f"blocks {n}, kernel span {us(te.max() - ts.min()):.1f} us")
print(f"prologue us  median {us(med(tl0 - ts)):.2f}")
print(f"K loop us    median {us(med(tl1 - tl0)):.2f}  cycles {med(cl):.0f}  clock {med(cl / ((tl1 - tl0) * 10e-9)) / 1e9:.3f} GHz "
      f"(MFMA per wave {768 * 16})")
print(f"epilogue us  median {us(med(te - tl1)):.2f}  cycles {med(ce):.0f}  clock {med(ce / np.maximum(te - tl1, 1) / 10e-9) / 1e9:.3f} GHz")
cus = collections.defaultdict(list)
for i in range(n):
    cus[(int(xcc[i]), int(cu[i]))].append(i)
rows, gaps = [], []
busy2 = epi_loop = epi_epi = idle = 0.0
base, span = ts.min(), te.max() - ts.min()
for k, idx in cus.items():
    for i in idx:
        tl = te_ = 0.0
        for j in idx:
            if j == i:
                continue
            tl += max(0, min(tl1[i], tl1[j]) - max(tl0[i], tl0[j]))
            te_ += max(0, min(tl1[i], te[j]) - max(tl0[i], tl1[j]))
        rows.append((us(tl), us(te_), us(max(0, tl1[i] - tl0[i] - tl - te_))))
    st = sorted(idx, key=lambda i: ts[i])
    for i in st[2:]:
        prev = [te[j] for j in idx if te[j] <= ts[i]]
        if prev:
            gaps.append(us(ts[i] - max(prev)))
for k, idx in list(cus.items())[:64]:
    grid = np.arange(base, te.max(), 10)
    sl = np.zeros(len(grid), np.int32)
    se = np.zeros(len(grid), np.int32)
    for i in idx:
        sl[(grid >= ts[i]) & (grid < tl1[i])] += 1
        se[(grid >= tl1[i]) & (grid < te[i])] += 1
    tot = sl + se
    idle += np.mean(tot == 0)
    busy2 += np.mean(tot >= 2)
    epi_loop += np.mean((se >= 1) & (sl >= 1))
    epi_epi += np.mean(se >= 2)
m = min(64, len(cus))
print(f"per-CU time fractions: 2 blocks resident {busy2 / m:.2f}, epilogue beside a loop {epi_loop / m:.2f}, "
      f"two epilogues {epi_epi / m:.2f}, idle {idle / m:.3f}; next block starts median {med(gaps):.2f} us after a block ends")
A = np.array(rows)
sol, *_ = np.linalg.lstsq(A, np.ones(len(A)), rcond=None)
print("loop time split (median us): beside a loop {:.2f}, beside an epilogue {:.2f}, alone {:.2f}".format(*np.median(A, 0)))
print("fitted loop time (us): beside a loop {:.2f}, beside an epilogue {:.2f}, alone {:.2f}".format(*(1 / sol)))
