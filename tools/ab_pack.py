#!/usr/bin/env python3
"""The split build's operand pass alone (ecorr_build_split_pack) per library (tree + AB_ALT_LIB
name=path,...), DSEC B = 16: 20 back-to-back launches between two HIP events, median of rotated
rounds.  Lab variants whose panels differ are fine here (the GEMM does not run).  One JSON line."""
import ctypes
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import eraft_amd  # noqa: E402,F401
from eraft_amd import _lib  # noqa: E402

LIBS = {"tree": _lib.lib()}
for k, item in enumerate(filter(None, os.environ.get("AB_ALT_LIB", "").split(","))):
    name, _, path = item.rpartition("=")
    L = ctypes.CDLL(os.path.join(ROOT, path))
    for sym, (rt, args) in _lib.SYMBOLS.items():
        if hasattr(L, sym):
            getattr(L, sym).restype = rt
            getattr(L, sym).argtypes = args
    LIBS[name or f"alt{k}"] = L
B, D, H, W = 16, 256, 60, 80
g = torch.Generator(device="cuda").manual_seed(3)
f1 = torch.randn((B, D, H, W), generator=g, device="cuda")
f2 = torch.randn((B, D, H, W), generator=g, device="cuda")
n = ctypes.c_int64()
_lib.check(_lib.lib().ecorr_build_split_workspace_size(B, D, H, W, H * W, ctypes.byref(n)), "ws")
ws = torch.empty(n.value, dtype=torch.uint8, device="cuda")
st = _lib.stream_of(f1)
times = {k: [] for k in LIBS}
names = list(LIBS)
for rnd in range(12):
    for name in names[rnd % len(names):] + names[:rnd % len(names)]:
        L = LIBS[name]
        for _ in range(3):
            L.ecorr_build_split_pack(f1.data_ptr(), f2.data_ptr(), B, D, H, W, H * W, ws.data_ptr(), st)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            L.ecorr_build_split_pack(f1.data_ptr(), f2.data_ptr(), B, D, H, W, H * W, ws.data_ptr(), st)
        e1.record()
        torch.cuda.synchronize()
        times[name].append(e0.elapsed_time(e1) / 20 * 1e3)
print(json.dumps({"probe": "operand pass alone, DSEC B=16", "us": {k: round(statistics.median(v), 1) for k, v in times.items()}}))
