#!/usr/bin/env python3
"""Interleaved A/B of the fused lookup + convc1 + ReLU kernel (ecorr_lookup_conv1x1_relu) between
the tree's libecorr.so and AB_ALT_LIB lab builds (name=path,...) in ONE process, at the bench shape
(DSEC B=16 60x80, one pyramid built by the tree library).  Checks first that every library's output
is bitwise the tree's (AB_NOCHECK=1 skips), then times 12 calls per round in rotated order.
  AB_ALT_LIB=v=tools/v_lab/e-raft_amd/libecorr.so python tools/ab_motion.py
"""
import ctypes
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import eraft_amd  # noqa: E402
from eraft_amd import _lib  # noqa: E402


def load(path):
    L = ctypes.CDLL(path)
    for name, (res, args) in _lib.SYMBOLS.items():
        if hasattr(L, name):
            getattr(L, name).restype = res
            getattr(L, name).argtypes = args
    return L


LIBS = {"tree": load(_lib.LIB_PATH)}
for k, item in enumerate(filter(None, os.environ.get("AB_ALT_LIB", "").split(","))):
    name, _, path = item.rpartition("=")
    LIBS[name or f"alt{k}"] = load(os.path.join(ROOT, path))
B, H, W, D = 16, 60, 80, 256
g = torch.Generator(device="cuda").manual_seed(0)
with torch.no_grad():
    _lib._lib = LIBS["tree"]
    f1 = torch.randn((B, D, H, W), generator=g, device="cuda")
    f2 = torch.randn((B, D, H, W), generator=g, device="cuda")
    blk = eraft_amd.CorrBlock(f1, f2)
    base = eraft_amd.coords_grid(B, H, W, device="cuda")
    coords = [(base + 2.0 * torch.randn((B, 2, H, W), generator=g, device="cuda")).contiguous() for _ in range(12)]
    wgt = torch.randn((256, 324, 1, 1), generator=g, device="cuda") * 0.05
    bias = torch.randn((256,), generator=g, device="cuda") * 0.1

    def call(c):
        return blk.lookup_conv1x1_relu(c, wgt, bias, mode="fused")

    if not os.environ.get("AB_NOCHECK"):
        ref = call(coords[0])
        for name, L in LIBS.items():
            _lib._lib = L
            same = torch.equal(call(coords[0]), ref)
            print(f"bitwise {name}: {'same' if same else 'DIFFERENT'}", flush=True)
            if not same:
                raise SystemExit(f"{name}: fused lookup differs")
    times = {k: [] for k in LIBS}
    names = list(LIBS)
    for rnd in range(int(os.environ.get("AB_ROUNDS", "10"))):
        for name in names[rnd % len(names):] + names[:rnd % len(names)]:
            _lib._lib = LIBS[name]
            call(coords[0])
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for c in coords:
                call(c)
            e1.record()
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) / len(coords) * 1e3)
    res = {}
    for name, ts in times.items():
        med = statistics.median(ts)
        print(f"fused lookup+convc1 B={B} {name:10s} median {med:.1f} us  min {min(ts):.1f}", flush=True)
        res[name] = round(med, 1)
    print(json.dumps({"ab_motion_us": res}))
