#!/usr/bin/env python3
"""Interleaved A/B of two builds of libecorr.so in ONE process: the tree's own library against
AB_ALT_LIB (a .so built from another revision, e.g. `git stash; make; cp libecorr.so
libecorr_alt.so; git stash pop; make`).  For changes a runtime knob cannot select (data layouts,
template constants).  Times the 12-call lookup and the fused lookup + convc1 on DSEC B=16; both
libraries must produce bitwise-identical outputs."""
import ctypes
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
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    assert L.ecorr_abi_version() == _lib.ABI_VERSION, path
    return L


LIBS = {"tree": load(_lib.LIB_PATH), "alt": load(os.path.join(ROOT, os.environ["AB_ALT_LIB"]))}
B, H, W, D = int(os.environ.get("AB_BATCH", "16")), 60, 80, 256
g = torch.Generator(device="cuda").manual_seed(0)
with torch.no_grad():
    f1 = torch.randn((B, D, H, W), generator=g, device="cuda")
    f2 = torch.randn((B, D, H, W), generator=g, device="cuda")
    _lib._lib = LIBS["tree"]
    blk = eraft_amd.CorrBlock(f1, f2)
    base = eraft_amd.coords_grid(B, H, W, device="cuda")
    init = torch.nn.functional.avg_pool2d(torch.randn((B, 2, H, W), generator=g, device="cuda") * 9.0, 5, 1, 2)
    coords = [(base + init + 0.5 * torch.randn((B, 2, H, W), generator=g, device="cuda")).contiguous()
              for _ in range(12)]
    wt = torch.randn((256, 324), generator=g, device="cuda") * 0.05
    bias = torch.randn((256,), generator=g, device="cuda") * 0.1
    fused = hasattr(blk, "lookup_conv1x1_relu")
    algo = B * H * W * 2904
    # integer coordinates (zero flow: the first iteration without warm start) exercise the
    # floor-flip cases of the normalize/unnormalize round trip
    coords_int = [base.contiguous() for _ in range(12)]
    times = {(k, op): [] for k in LIBS for op in ("build", "lookup", "lookup_int", "fused")}
    ref = {}
    names = list(LIBS)
    for rnd in range(int(os.environ.get("AB_ROUNDS", "8"))):
        for name in names[rnd % 2:] + names[:rnd % 2]:
            _lib._lib = LIBS[name]
            outs = {"build": eraft_amd.CorrBlock(f1, f2)._pyramid, "lookup": blk(coords[0]),
                    "lookup_int": blk(coords_int[0])}
            if fused:
                outs["fused"] = blk.lookup_conv1x1_relu(coords[0], wt, bias)
            torch.cuda.synchronize()
            if rnd < 2:
                for op, o in outs.items():
                    if op in ref:
                        if os.environ.get("AB_ALLOW_DIFF"):   # numerically different variants
                            d = (o - ref[op]).abs().max().item() if o.shape == ref[op].shape else float("nan")
                            print(f"{name} {op}: max |diff| vs first {d:.3g}", flush=True)
                        else:
                            assert torch.equal(o, ref[op]), f"{name} {op} output differs"
                    else:
                        ref[op] = o.clone()
            for op in outs:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                if op == "build":
                    for _ in range(3):
                        eraft_amd.CorrBlock(f1, f2)
                else:
                    for c in (coords_int if op == "lookup_int" else coords):
                        blk(c) if op.startswith("lookup") else blk.lookup_conv1x1_relu(c, wt, bias)
                e1.record()
                torch.cuda.synchronize()
                times[(name, op)].append(e0.elapsed_time(e1) / (3 if op == "build" else len(coords)))
for (name, op), ts in times.items():
    if not ts:
        continue
    med = statistics.median(ts)
    extra = f"  -> {algo / med / 1e6:.0f} GB/s algorithmic" if op.startswith("lookup") else ""
    print(f"{op:10s} {name:5s} median {med * 1e3:.1f} us/call  min {min(ts) * 1e3:.1f}{extra}")
