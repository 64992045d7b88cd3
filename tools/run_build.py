#!/usr/bin/env python3
"""Run N CorrBlock builds (split mode, DSEC B=16 by default) through a chosen libecorr.so -- the
program that tools/prof_build.sh profiles.  usage: run_build.py [LIB|tree] [N] [B H W]"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import eraft_amd  # noqa: E402
from eraft_amd import _lib  # noqa: E402

lib = sys.argv[1] if len(sys.argv) > 1 else "tree"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 10
B, H, W = (int(x) for x in sys.argv[3:6]) if len(sys.argv) > 5 else (16, 60, 80)
if lib != "tree":
    L = ctypes.CDLL(os.path.join(ROOT, lib))
    for name, (res, args) in _lib.SYMBOLS.items():
        if hasattr(L, name):   # (a lab build of an older ABI lacks later symbols)
            getattr(L, name).restype = res
            getattr(L, name).argtypes = args
    _lib._lib = L
g = torch.Generator(device="cuda").manual_seed(0)
with torch.no_grad():
    f1 = torch.randn((B, 256, H, W), generator=g, device="cuda")
    f2 = torch.randn((B, 256, H, W), generator=g, device="cuda")
    for _ in range(n):
        eraft_amd.CorrBlock(f1, f2)
    torch.cuda.synchronize()
print("ok", lib, n)
