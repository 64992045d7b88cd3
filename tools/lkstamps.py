#!/usr/bin/env python3
"""Per-workgroup timeline of the radius-4 lookup (lookup_cols_reg) from the lkstamps lab build
(tools/lab_build.py lkstamps): phase 0 (coordinate chains + origins), phase 1 (window staging),
phase 2 (blend + output stores, until the wave's stores retired), per level; per-CU residency.
Lookups run back to back for ~2 s first (clock under load), then one stamped call is read.
  python tools/lkstamps.py tools/lkstamps_lab/e-raft_amd/libecorr.so [smooth|iid]"""
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
field = sys.argv[2] if len(sys.argv) > 2 else "smooth"
B, H, W = 16, 60, 80
g = torch.Generator(device="cuda").manual_seed(0)
with torch.no_grad():
    f1 = torch.randn((B, 256, H, W), generator=g, device="cuda")
    f2 = torch.randn((B, 256, H, W), generator=g, device="cuda")
    blk = eraft_amd.CorrBlock(f1, f2)
    base = eraft_amd.coords_grid(B, H, W, device="cuda")
    if field == "iid":
        c = base + 3.0 * torch.randn((B, 2, H, W), generator=g, device="cuda")
    else:
        yy, xx = torch.meshgrid(torch.arange(H, device="cuda"), torch.arange(W, device="cuda"), indexing="ij")
        c = base + torch.stack([2.0 * torch.sin(yy / 9.0), 1.5 * torch.cos(xx / 11.0)]).float()
    c = c.contiguous()
    t0 = time.time()
    while time.time() - t0 < 2.0:
        for _ in range(100):
            blk(c)
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    blk(c)
    e1.record()
    torch.cuda.synchronize()
    print(f"stamped call {e0.elapsed_time(e1) * 1e3:.1f} us ({field})")
gx, gy = (H * W + 63) // 64, 4
n = gx * gy * B
buf = (ctypes.c_uint64 * (8 * n))()
assert L.ecorr_lab_lkstamps(buf, n) == 0
a = np.frombuffer(buf, dtype=np.uint64).reshape(n, 8).astype(np.int64)
t0, t1, t2 = a[:, 0], a[:, 1], a[:, 2]
te = a[:, 3:6].max(1)
lvl = (np.arange(n) // gx) % gy
hw, xcc = a[:, 6], a[:, 7] & 0xF
cu = (hw >> 8) & 0xFF
us = lambda x: x / 100.0   # s_memrealtime: 100 MHz
print(f"workgroups {n}, kernel span {us(te.max() - t0.min()):.1f} us")
for lv in range(gy):
    m = lvl == lv
    print(f"level {lv}: phase0 {us(np.median(t1[m] - t0[m])):.2f}  phase1 {us(np.median(t2[m] - t1[m])):.2f}  "
          f"phase2 {us(np.median(te[m] - t2[m])):.2f}  life {us(np.median(te[m] - t0[m])):.2f} us (median)  "
          f"wave ends spread {us(np.median(a[m, 3:6].max(1) - a[m, 3:6].min(1))):.2f}")
cus = collections.defaultdict(list)
for i in range(n):
    cus[(int(xcc[i]), int(cu[i]))].append(i)
base_t, end_t = t0.min(), te.max()
grid = np.arange(base_t, end_t, 5)
occ = []
for k, idx in cus.items():
    res = np.zeros(len(grid), np.int32)
    for i in idx:
        res[(grid >= t0[i]) & (grid < te[i])] += 1
    occ.append(res)
occ = np.array(occ)
print(f"CUs {len(cus)}, workgroups per CU {n / len(cus):.2f}; resident workgroups per CU over the span: "
      + ", ".join(f"{k}: {np.mean(occ == k):.2f}" for k in range(0, int(occ.max()) + 1)))
q = np.linspace(0, 1, 11)
starts = np.quantile(us(t0 - base_t), q)
ends = np.quantile(us(te - base_t), q)
print("start deciles (us): " + " ".join(f"{x:.1f}" for x in starts))
print("end deciles (us):   " + " ".join(f"{x:.1f}" for x in ends))
first = np.array([min(t0[i] for i in idx) for idx in cus.values()])
last = np.array([max(te[i] for i in idx) for idx in cus.values()])
print(f"per-CU first start median {us(np.median(first - base_t)):.2f} us, last end spread "
      f"{us(np.quantile(last - base_t, 0.05)):.1f}..{us(np.quantile(last - base_t, 0.95)):.1f} us")
