#!/usr/bin/env python3
"""Per-phase timeline of the banded splat (lab build sp_stamps): median phase lengths over the
workgroups of one DSEC B=16 forward_interpolate launch after warm-up.  usage: spstamps.py LIB"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from ab_lib_loader import load  # noqa: E402
import eraft_amd  # noqa: E402
from eraft_amd import _lib  # noqa: E402

L = load(os.path.join(ROOT, sys.argv[1]))
_lib._lib = L
for B, H, W in ((16, 60, 80), (4, 92, 160)):
    g = torch.Generator(device="cuda").manual_seed(5)
    flow = torch.nn.functional.avg_pool2d(torch.randn((B, 2, H, W), generator=g, device="cuda") * 9.0, 5, stride=1,
                                          padding=2).contiguous()
    for _ in range(5):
        eraft_amd.forward_interpolate_pytorch(flow)
    torch.cuda.synchronize()
    nwg = 256 if B == 16 else 256
    st = np.zeros((65536, 6), dtype=np.uint64)
    L.ecorr_lab_spstamps(st.ctypes.data_as(ctypes.c_void_p), 65536)
    n = int((st[:, 0] > 0).sum())
    s = st[:n].astype(np.int64)
    t0 = s[:, 0].min()
    ph = np.diff(s, axis=1) / 100.0   # us
    names = ["stage", "count", "scan", "bucket", "fold"]
    print(f"B={B} {H}x{W}: {n} workgroups, span {(s[:, 5].max() - t0) / 100:.1f} us, start spread {(s[:, 0].max() - t0) / 100:.1f} us")
    print("   median us: " + ", ".join(f"{k} {np.median(ph[:, i]):.2f}" for i, k in enumerate(names)),
          " | max: " + ", ".join(f"{k} {ph[:, i].max():.2f}" for i, k in enumerate(names)))
