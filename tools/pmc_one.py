#!/usr/bin/env python3
"""Run the DSEC B=16 CorrBlock build N times with a given libecorr.so (tree or lab build), for a
rocprofv3 --pmc pass over one library.  usage: tools/pmc_one.py LIB [N]
Summarize with: tools/pmc_one.py --summary <rocprof dir> <kernel prefix>"""
import csv
import ctypes
import glob
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if sys.argv[1] == "--summary":
    acc = {}
    for f in glob.glob(os.path.join(sys.argv[2], "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if sys.argv[3] in r["Kernel_Name"]:
                acc.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    for k, v in sorted(acc.items()):
        print(f"{k:28s} mean {sum(v) / len(v):16.1f}  n={len(v)}")
    sys.exit(0)
import torch  # noqa: E402
sys.path.insert(0, ROOT)
import eraft_amd  # noqa: E402
from eraft_amd import _lib  # noqa: E402
L = ctypes.CDLL(os.path.join(ROOT, sys.argv[1]))
for name, (res, args) in _lib.SYMBOLS.items():
    getattr(L, name).restype = res
    getattr(L, name).argtypes = args
_lib._lib = L
n = int(sys.argv[2]) if len(sys.argv) > 2 else 5
g = torch.Generator(device="cuda").manual_seed(0)
with torch.no_grad():
    shape = tuple(int(v) for v in os.environ.get("PMC_SHAPE", "16,256,60,80").split(","))   # B,D,H,W
    f1 = torch.randn(shape, generator=g, device="cuda")
    f2 = torch.randn(shape, generator=g, device="cuda")
    for _ in range(n):
        eraft_amd.CorrBlock(f1, f2)
    torch.cuda.synchronize()
print("ok")
