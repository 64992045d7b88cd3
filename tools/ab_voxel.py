#!/usr/bin/env python3
"""Interleaved A/B of the DSEC event -> voxel conversion (ecorr_voxel_grid_dsec, voxel.hip) between
the tree's libecorr.so and AB_ALT_LIB lab builds (name=path,...) in one process, on the window
bench.py's next_rows.voxel_grid_dsec times (1M events, 15 x 480 x 640; seed 8).  Reports whether
each library's grid is bitwise the tree's, and per arm (normalize 1 / 0) the median device time of
20 calls per round over rotated rounds (HIP events on the call's stream: the whole call)."""
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

n, C, H, W = 1_000_000, 15, 480, 640
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(8)
t = torch.sort(torch.rand((n,), generator=g, device=dev) * 1e5).values
p = (torch.rand((n,), generator=g, device=dev) < 0.5).float()
t = t - t[0]
x = torch.rand((n,), generator=g, device=dev) * (W + 2) - 1.5
y = torch.rand((n,), generator=g, device=dev) * (H + 2) - 1.5
out = torch.empty((C, H, W), device=dev)
st = _lib.stream_of(out)
ws = {}
for name, L in LIBS.items():
    b = ctypes.c_int64()
    _lib.check(L.ecorr_voxel_workspace_size(1, n, C, H, W, ctypes.byref(b)), "ws")
    ws[name] = torch.empty(b.value, dtype=torch.uint8, device=dev)


def run(name, norm):
    _lib.check(LIBS[name].ecorr_voxel_grid_dsec(p.data_ptr(), t.data_ptr(), x.data_ptr(), y.data_ptr(), n, C, H, W,
                                                norm, out.data_ptr(), ws[name].data_ptr(), st), "voxel")


res = {}
with torch.no_grad():
    base = {}
    for name in LIBS:
        for norm in (1, 0):
            out.fill_(float("nan"))
            run(name, norm)
            torch.cuda.synchronize()
            if name == "tree":
                base[norm] = out.clone()
            else:
                res.setdefault(name, {})[f"bitwise_norm{norm}"] = bool(torch.equal(out, base[norm]))
    times = {(nm, nr): [] for nm in LIBS for nr in (1, 0)}
    names = list(LIBS)
    for rnd in range(6):
        for nm in names[rnd % len(names):] + names[:rnd % len(names)]:
            for nr in (1, 0):
                for _ in range(3):
                    run(nm, nr)
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(21)]
                ev[0].record()
                for i in range(20):
                    run(nm, nr)
                    ev[i + 1].record()
                torch.cuda.synchronize()
                times[(nm, nr)] += [ev[i].elapsed_time(ev[i + 1]) * 1e3 for i in range(20)]
    for (nm, nr), ts in times.items():
        res.setdefault(nm, {})[f"us_norm{nr}"] = round(statistics.median(ts), 1)
print(json.dumps({"probe": "ab_voxel dsec 1M events 15x480x640", "libs": res}))
