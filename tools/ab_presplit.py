#!/usr/bin/env python3
"""Lookup + convc1 + ReLU per iteration at DSEC B = 16 (60 x 80, D = 256, O = 256), the split mode
(ecorr_lookup_qmax + ecorr_conv1x1_relu_split) against the presplit mode (ecorr_lookup_presplit +
ecorr_conv1x1_relu_presplit, ABI 16) and the fused one: 12 iterations per timing (the bench's
smooth coordinate fields), median of rounds, HIP events on the launch stream; then each mode's
normwise error against the fp64 conv of the exact lookup, and the two conv kernels alone on one
materialized input.  Prints one JSON line."""
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

B, D, H, W, O = 16, 256, 60, 80, 256
Q = H * W
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(11)
f1 = torch.randn((B, D, H, W), generator=g, device=dev)
f2 = torch.randn((B, D, H, W), generator=g, device=dev)
base = eraft_amd.coords_grid(B, H, W, device=dev)
coords = []
for i in range(12):
    fl = torch.nn.functional.avg_pool2d(torch.randn((B, 2, H, W), generator=g, device=dev) * 6.0, 7, stride=1,
                                        padding=3)
    coords.append((base + fl).contiguous())
wgt = torch.randn((O, 324, 1, 1), generator=g, device=dev) * 0.05
bias = torch.randn((O,), generator=g, device=dev) * 0.1
stream = torch.cuda.current_stream(dev)


def run(fn, rounds=7):
    ts = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for c in coords:
            fn(c)
        e1.record(stream)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / len(coords) * 1e3)
    return round(statistics.median(ts[1:]), 1)


res = {}
with torch.no_grad():
    blk = eraft_amd.CorrBlock(f1, f2)
    modes = ("split", "presplit", "fused")
    for m in modes:
        blk.lookup_conv1x1_relu(coords[0], wgt, bias, mode=m)
    assert blk._colscale is not None
    for rnd in range(2):
        for m in (modes if rnd == 0 else modes[::-1]):
            res.setdefault(m, {}).setdefault("us_per_iter", []).append(
                run(lambda c, m=m: blk.lookup_conv1x1_relu(c, wgt, bias, mode=m)))
    corr = blk(coords[3]).double()
    ref = torch.relu(torch.einsum("oc,bchw->bohw", wgt.view(O, 324).double(), corr) + bias.double()[None, :, None, None])
    rms = float(ref.pow(2).mean().sqrt())
    for m in modes:
        got = blk.lookup_conv1x1_relu(coords[3], wgt, bias, mode=m).double()
        res[m]["normwise_vs_fp64"] = float((got - ref).abs().max()) / rms
    # the conv kernels alone on one materialized input each
    st = _lib.stream_of(f1)
    qmax = torch.empty((B, 12, Q), device=dev)
    cin = torch.empty((B, 324, Q), device=dev)
    _lib.check(_lib.lib().ecorr_lookup_qmax(blk._pyramid.data_ptr(), coords[0].data_ptr(), B, H, W, Q, 4, 4,
                                            cin.data_ptr(), qmax.data_ptr(), st), "qmax")
    nb = ctypes.c_int64()
    _lib.check(_lib.lib().ecorr_presplit_size(B, 4, Q, ctypes.byref(nb)), "size")
    pin = torch.empty(nb.value, dtype=torch.uint8, device=dev)
    sc = blk._colscale
    _lib.check(_lib.lib().ecorr_lookup_presplit(blk._pyramid.data_ptr(), coords[0].data_ptr(), B, H, W, Q, 4, 4,
                                                sc.data_ptr(), pin.data_ptr(), st), "presplit lookup")
    pk = _lib.packed_conv1x1_weight(wgt, O, 324, "split", st, {})
    pkp = _lib.packed_conv1x1_weight(wgt, O, 324, "presplit", st, {})
    out = torch.empty((B, O, Q), device=dev)
    res["conv_split_us"] = run(lambda c: _lib.lib().ecorr_conv1x1_relu_split(
        cin.data_ptr(), B, 324, Q, qmax.data_ptr(), 12, pk.data_ptr(), bias.data_ptr(), O, out.data_ptr(), st))
    res["conv_presplit_us"] = run(lambda c: _lib.lib().ecorr_conv1x1_relu_presplit(
        pin.data_ptr(), B, 4, Q, sc.data_ptr(), pkp.data_ptr(), bias.data_ptr(), O, out.data_ptr(), st))
    res["lookup_qmax_us"] = run(lambda c: _lib.lib().ecorr_lookup_qmax(
        blk._pyramid.data_ptr(), c.data_ptr(), B, H, W, Q, 4, 4, cin.data_ptr(), qmax.data_ptr(), st))
    res["lookup_presplit_us"] = run(lambda c: _lib.lib().ecorr_lookup_presplit(
        blk._pyramid.data_ptr(), c.data_ptr(), B, H, W, Q, 4, 4, sc.data_ptr(), pin.data_ptr(), st))
    # lab builds (AB_ALT_LIB=name=path,...): their presplit lookup and conv on the same inputs
    for k, item in enumerate(filter(None, os.environ.get("AB_ALT_LIB", "").split(","))):
        name, _, path = item.rpartition("=")
        L = ctypes.CDLL(os.path.join(ROOT, path))
        for sym, (rt, args) in _lib.SYMBOLS.items():
            if hasattr(L, sym):
                getattr(L, sym).restype = rt
                getattr(L, sym).argtypes = args
        pin2 = torch.empty_like(pin)
        n2 = ctypes.c_int64()
        _lib.check(L.ecorr_conv1x1_presplit_size(O, 4, ctypes.byref(n2)), "size")
        pk2 = torch.empty(n2.value, dtype=torch.uint8, device=dev)
        _lib.check(L.ecorr_conv1x1_split_pack_presplit(wgt.data_ptr(), O, 4, pk2.data_ptr(), st), "pack")
        out2 = torch.empty_like(out)
        res.setdefault("alt", {})[name or f"alt{k}"] = {
            "lookup_presplit_us": run(lambda c: L.ecorr_lookup_presplit(
                blk._pyramid.data_ptr(), c.data_ptr(), B, H, W, Q, 4, 4, sc.data_ptr(), pin2.data_ptr(), st)),
            "conv_presplit_us": run(lambda c: L.ecorr_conv1x1_relu_presplit(
                pin2.data_ptr(), B, 4, Q, sc.data_ptr(), pk2.data_ptr(), bias.data_ptr(), O, out2.data_ptr(), st))}
    blk2 = eraft_amd.CorrBlock(f1, f2)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    blk2._column_scale(st)
    e1.record(stream)
    torch.cuda.synchronize()
    res["column_scale_us_once_per_block"] = round(e0.elapsed_time(e1) * 1e3, 1)
print(json.dumps({"probe": "lookup + convc1 + relu per iteration, DSEC B=16 60x80", "modes": res}))
