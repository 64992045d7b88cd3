#!/usr/bin/env python3
"""Interleaved A/B of the split-f16 convc1 + ReLU (ecorr_conv1x1_relu_split, conv.hip) between the
tree's libecorr.so and AB_ALT_LIB lab builds (name=path,...) in one process, at DSEC B=16 60x80 on
a materialized lookup (C = 324 -> O = 256).  Reports each library's normwise error (max|d| / rms)
against an fp64 conv, whether its output is bitwise the tree's, and the median time of 20 calls per
round over rotated rounds.  AB_CONV_IID=1: an i.i.d. normal input instead of a real lookup;
AB_CONV_PRE=1: no per-query maxima passed (the kernel's own max pre-pass)."""
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

LIBS = {"tree": _lib.lib()}
for k, item in enumerate(filter(None, os.environ.get("AB_ALT_LIB", "").split(","))):
    name, _, path = item.rpartition("=")
    L = ctypes.CDLL(os.path.join(ROOT, path))
    for sym, (res, args) in _lib.SYMBOLS.items():
        if hasattr(L, sym):
            getattr(L, sym).restype = res
            getattr(L, sym).argtypes = args
    LIBS[name or f"alt{k}"] = L
B, D, H, W, C, O = 16, 256, 60, 80, 324, 256
Q = H * W
g = torch.Generator(device="cuda").manual_seed(0)
with torch.no_grad():
    if os.environ.get("AB_CONV_IID"):
        x = torch.randn((B, C, Q), generator=g, device="cuda")
    else:
        f1 = torch.randn((B, D, H, W), generator=g, device="cuda")
        f2 = torch.randn((B, D, H, W), generator=g, device="cuda")
        blk = eraft_amd.CorrBlock(f1, f2)
        coords = eraft_amd.coords_grid(B, H, W, device="cuda") + torch.randn((B, 2, H, W), generator=g,
                                                                              device="cuda") * 3.0
        x = blk(coords).view(B, C, Q)
    w = torch.randn((O, C), generator=g, device="cuda") * 0.05
    bias = torch.randn((O,), generator=g, device="cuda") * 0.1
out = torch.empty((B, O, Q), device="cuda")
st = _lib.stream_of(out)
packed = {}
for name, L in LIBS.items():
    n = ctypes.c_int64()
    _lib.check(L.ecorr_conv1x1_split_size(O, C, ctypes.byref(n)), "size")
    pk = torch.empty(n.value, dtype=torch.uint8, device="cuda")
    _lib.check(L.ecorr_conv1x1_split_pack(w.data_ptr(), O, C, pk.data_ptr(), st), "pack")
    packed[name] = pk


# per-query partial maxima as ecorr_lookup_qmax leaves them (G = 12 groups; here one group holds the
# max, the rest 0) unless AB_CONV_PRE=1 (the kernel's own pre-pass)
G = 12
qmax = None
if not os.environ.get("AB_CONV_PRE"):
    qmax = torch.zeros((B, G, Q), device="cuda")
    qmax[:, 0] = x.abs().nan_to_num(nan=0.0).amax(dim=1)


def run(name):
    _lib.check(LIBS[name].ecorr_conv1x1_relu_split(x.data_ptr(), B, C, Q, None if qmax is None else qmax.data_ptr(), G,
                                                   packed[name].data_ptr(), bias.data_ptr(), O, out.data_ptr(), st),
               "conv")


with torch.no_grad():
    ref = torch.relu(torch.einsum("oc,bcq->boq", w.double(), x.double()) + bias.double().view(1, -1, 1))
    rms = float(ref.pow(2).mean().sqrt())
    base = None
    for name in LIBS:
        out.fill_(float("nan"))
        run(name)
        torch.cuda.synchronize()
        err = float((out.double() - ref).abs().max()) / rms
        same = "" if base is None else ("  bitwise tree: " + ("same" if torch.equal(out, base) else "DIFFERENT"))
        if base is None:
            base = out.clone()
        print(f"normwise {name}: {err:.2e}{same}", flush=True)
    times = {k: [] for k in LIBS}
    names = list(LIBS)
    for rnd in range(10):
        for name in names[rnd % len(names):] + names[:rnd % len(names)]:
            run(name)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                run(name)
            e1.record()
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) / 20 * 1e3)
res = {k: round(statistics.median(v), 1) for k, v in times.items()}
for k, v in res.items():
    print(f"conv split B={B} {k:10s} median {v:.1f} us", flush=True)
print(json.dumps({"ab_conv_us": res}))
