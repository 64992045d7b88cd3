#!/usr/bin/env python3
"""Interleaved A/B of the convex upsampling kernel (ecorr_upsample_flow) between the tree's
libecorr.so and AB_ALT_LIB lab builds (name=path,...) in one process, DSEC B=16 60x80.  Reports each
library's normwise error (max|d| / rms) against an fp64 evaluation of the reference's expression
(eraft.py:74-85) and the median time of 20 calls per round over rotated rounds."""
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
    for sym, (res, args) in _lib.SYMBOLS.items():
        if hasattr(L, sym):
            getattr(L, sym).restype = res
            getattr(L, sym).argtypes = args
    LIBS[name or f"alt{k}"] = L
N, H, W = 16, 60, 80
g = torch.Generator(device="cuda").manual_seed(0)
flow = torch.randn((N, 2, H, W), generator=g, device="cuda") * 3.0
mask = torch.randn((N, 576, H, W), generator=g, device="cuda")
out = torch.empty((N, 2, 8 * H, 8 * W), device="cuda")
st = _lib.stream_of(flow)


def run(L):
    _lib.check(L.ecorr_upsample_flow(flow.data_ptr(), mask.data_ptr(), N, H, W, out.data_ptr(), st), "upsample")


with torch.no_grad():
    m = torch.softmax(mask.double().view(N, 1, 9, 8, 8, H, W), dim=2)
    up = torch.nn.functional.unfold(8 * flow.double(), [3, 3], padding=1).view(N, 2, 9, 1, 1, H, W)
    ref = torch.sum(m * up, dim=2).permute(0, 1, 4, 2, 5, 3).reshape(N, 2, 8 * H, 8 * W)
    rms = float(ref.pow(2).mean().sqrt())
    for name, L in LIBS.items():
        run(L)
        torch.cuda.synchronize()
        print(f"normwise {name}: {float((out.double() - ref).abs().max()) / rms:.2e}", flush=True)
    times = {k: [] for k in LIBS}
    names = list(LIBS)
    for rnd in range(10):
        for name in names[rnd % len(names):] + names[:rnd % len(names)]:
            run(LIBS[name])
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                run(LIBS[name])
            e1.record()
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) / 20 * 1e3)
res = {k: round(statistics.median(v), 1) for k, v in times.items()}
for k, v in res.items():
    print(f"upsample B={N} {k:10s} median {v:.1f} us", flush=True)
print(json.dumps({"ab_upsample_us": res}))
