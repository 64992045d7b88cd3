#!/usr/bin/env python3
"""Interleaved A/B of the radius-4 lookup between the tree's libecorr.so and AB_ALT_LIB lab builds
(name=path,...) in ONE process, on one pyramid built by the tree library (DSEC B=16 60x80;
coordinates AB_COORDS=smooth (default), int (zero flow) or rough (i.i.d. 12-px flow)).
Checks first that every library's lookup is bitwise identical to the tree's (AB_NOCHECK=1 skips:
ablation builds), then times 12 lookups per round in rotated order.
  AB_ALT_LIB=v=tools/v_lab/e-raft_amd/libecorr.so python tools/ab_lookup.py
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
        try:
            fn = getattr(L, name)
        except AttributeError:
            continue
        fn.restype = res
        fn.argtypes = args
    return L


LIBS = {"tree": load(_lib.LIB_PATH)}
for k, item in enumerate(filter(None, os.environ.get("AB_ALT_LIB", "").split(","))):
    name, _, path = item.rpartition("=")
    LIBS[name or f"alt{k}"] = load(os.path.join(ROOT, path))
B, H, W, D = int(os.environ.get("AB_BATCH", "16")), 60, 80, 256
g = torch.Generator(device="cuda").manual_seed(0)
with torch.no_grad():
    _lib._lib = LIBS["tree"]
    f1 = torch.randn((B, D, H, W), generator=g, device="cuda")
    f2 = torch.randn((B, D, H, W), generator=g, device="cuda")
    blk = eraft_amd.CorrBlock(f1, f2)
    base = eraft_amd.coords_grid(B, H, W, device="cuda")
    init = torch.nn.functional.avg_pool2d(torch.randn((B, 2, H, W), generator=g, device="cuda") * 9.0, 5, 1, 2)
    mode = os.environ.get("AB_COORDS", "smooth")   # smooth | int (zero flow) | rough (i.i.d. flow)
    if mode == "int":
        coords = [base.clone() for _ in range(12)]
    elif mode.startswith("iid"):   # iid<sigma>: SURVEY 8(d)'s i.i.d. N(0, sigma^2) flow (iid3, iid40)
        coords = [(base + float(mode[3:]) * torch.randn((B, 2, H, W), generator=g, device="cuda")).contiguous()
                  for _ in range(12)]
    elif mode == "rough":
        coords = [(base + 12.0 * torch.randn((B, 2, H, W), generator=g, device="cuda")).contiguous()
                  for _ in range(12)]
    else:
        coords = [(base + init + 0.5 * torch.randn((B, 2, H, W), generator=g, device="cuda")).contiguous()
                  for _ in range(12)]
    if not os.environ.get("AB_NOCHECK"):
        checks = [coords[0], coords[0] + 0.3]   # + a non-integer shift (the int mode's floors flip)
        refs = [blk(c) for c in checks]
        for name, L in LIBS.items():
            _lib._lib = L
            same = all(torch.equal(blk(c), r) for c, r in zip(checks, refs))
            print(f"bitwise {name}: {'same' if same else 'DIFFERENT'}", flush=True)
            if not same:
                raise SystemExit(f"{name}: lookup differs")
    times = {k: [] for k in LIBS}
    names = list(LIBS)
    for rnd in range(int(os.environ.get("AB_ROUNDS", "10"))):
        for name in names[rnd % len(names):] + names[:rnd % len(names)]:
            _lib._lib = LIBS[name]
            for c in coords[:2]:
                blk(c)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for c in coords:
                blk(c)
            e1.record()
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) / len(coords) * 1e3)
    res = {}
    for name, ts in times.items():
        med = statistics.median(ts)
        print(f"lookup B={B} {mode} {name:10s} median {med:.1f} us  min {min(ts):.1f}", flush=True)
        res[name] = round(med, 1)
    print(json.dumps({"ab_lookup_us": res}))
