#!/usr/bin/env python3
"""Interleaved timing of ecorr_lookup vs ecorr_lookup_qmax (the lookup + per-query partial maxima
the split convc1 uses) on the same pyramid and coordinates, DSEC B=16, smooth field; and of the
split path's two launches back to back vs each alone (where the conv reads a freshly written corr)."""
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import eraft_amd  # noqa: E402
from eraft_amd import _lib  # noqa: E402

B, D, H, W, Q = 16, 256, 60, 80, 4800
g = torch.Generator(device="cuda").manual_seed(0)
with torch.no_grad():
    blk = eraft_amd.CorrBlock(torch.randn((B, D, H, W), generator=g, device="cuda"),
                              torch.randn((B, D, H, W), generator=g, device="cuda"))
    coords = (eraft_amd.coords_grid(B, H, W, device="cuda")
              + torch.nn.functional.avg_pool2d(torch.randn((B, 2, H, W), generator=g, device="cuda") * 9, 5, 1, 2))
    coords = coords.contiguous()
    out = torch.empty((B, 324, H, W), device="cuda")
    qmax = torch.empty((B, 12, Q), device="cuda")
    wgt = torch.randn((256, 324), generator=g, device="cuda") * 0.05
    bias = torch.randn((256,), generator=g, device="cuda") * 0.1
    pk = _lib.packed_conv1x1_weight(wgt, 256, 324, "split", _lib.stream_of(wgt), {})
    res = torch.empty((B, 256, H, W), device="cuda")
import ctypes  # noqa: E402
LIBS = {"tree": _lib.lib()}
for k, item in enumerate(filter(None, os.environ.get("AB_ALT_LIB", "").split(","))):
    name, _, path = item.rpartition("=")
    Lx = ctypes.CDLL(os.path.join(ROOT, path))
    for sym, (restype, args) in _lib.SYMBOLS.items():
        if hasattr(Lx, sym):
            getattr(Lx, sym).restype = restype
            getattr(Lx, sym).argtypes = args
    LIBS[name or f"alt{k}"] = Lx
L = LIBS["tree"]
st = _lib.stream_of(out)
P = blk._pyramid.data_ptr()


def lookup():
    _lib.check(L.ecorr_lookup(P, coords.data_ptr(), B, H, W, Q, 4, 4, out.data_ptr(), st), "lookup")


def lookup_qmax():
    _lib.check(L.ecorr_lookup_qmax(P, coords.data_ptr(), B, H, W, Q, 4, 4, out.data_ptr(), qmax.data_ptr(), st), "qmax")


def conv():
    _lib.check(L.ecorr_conv1x1_relu_split(out.data_ptr(), B, 324, Q, qmax.data_ptr(), 12, pk.data_ptr(),
                                          bias.data_ptr(), 256, res.data_ptr(), st), "conv")


def both():
    lookup_qmax()
    conv()


fns = {"lookup": lookup, "lookup_qmax": lookup_qmax, "conv": conv, "lookup_qmax+conv": both}
for lname, Lx in list(LIBS.items())[1:]:   # lab builds: the split path's two launches back to back
    def both_x(Lx=Lx):
        _lib.check(Lx.ecorr_lookup_qmax(P, coords.data_ptr(), B, H, W, Q, 4, 4, out.data_ptr(), qmax.data_ptr(), st),
                   "qmax")
        _lib.check(Lx.ecorr_conv1x1_relu_split(out.data_ptr(), B, 324, Q, qmax.data_ptr(), 12, pk.data_ptr(),
                                               bias.data_ptr(), 256, res.data_ptr(), st), "conv")
    fns[f"{lname}: lookup_qmax+conv"] = both_x
times = {k: [] for k in fns}
names = list(fns)
both()
torch.cuda.synchronize()
for rnd in range(12):
    for name in names[rnd % len(names):] + names[:rnd % len(names)]:
        fns[name]()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(12):
            fns[name]()
        e1.record()
        torch.cuda.synchronize()
        times[name].append(e0.elapsed_time(e1) / 12 * 1e3)
for k, v in times.items():
    print(f"{k:18s} median {statistics.median(v):7.1f} us  min {min(v):7.1f}", flush=True)
