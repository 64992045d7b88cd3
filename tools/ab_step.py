#!/usr/bin/env python3
"""Interleaved A/B of the whole bench step -- split build (ecorr_build_split: operand pass + GEMM) then
12 lookups (ecorr_lookup) on the smooth warm-start fields -- between the tree's libecorr.so and the
AB_ALT_LIB lab builds (name=path,...) in one process, at DSEC B = 16.  For variants whose effect
crosses the kernel boundary (a store policy in the build that changes what the lookups find in the
caches), which tools/ab_build.py and tools/ab_lookup.py time apart.  Each library builds its own
pyramid; the first lookup output is checked bitwise against the tree's.  Reports the median time of
STEPS back-to-back steps per round over rotated rounds."""
import ctypes
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import eraft_amd  # noqa: E402
from eraft_amd import _lib  # noqa: E402
import ab_lib_loader  # noqa: E402

LIBS = ab_lib_loader.load_libs()
B, D, H, W, LV, R, ITERS, STEPS = 16, 256, 60, 80, 4, 4, 12, 10
Q = H * W
g = torch.Generator(device="cuda").manual_seed(0)
f1 = torch.randn((B, D, H, W), generator=g, device="cuda")
f2 = torch.randn((B, D, H, W), generator=g, device="cuda")
base = eraft_amd.coords_grid(B, H, W, device="cuda")
smooth = torch.nn.functional.avg_pool2d(torch.randn((B, 2, H, W), generator=g, device="cuda") * 6.0, 9, stride=1,
                                        padding=4)
coords = [(base + smooth + 0.3 * torch.randn((B, 2, H, W), generator=g, device="cuda")).contiguous()
          for _ in range(ITERS)]
st = _lib.stream_of(f1)
C = LV * (2 * R + 1) ** 2
out = torch.empty((B, C, H, W), device="cuda")

state = {}
for name, L in LIBS.items():
    h, w = (ctypes.c_int * LV)(), (ctypes.c_int * LV)()
    off = (ctypes.c_int64 * (LV + 1))()
    _lib.check(L.ecorr_pyramid_layout(B * Q, H, W, LV, h, w, off), "layout")
    n = ctypes.c_int64()
    _lib.check(L.ecorr_build_split_workspace_size(B, D, H, W, Q, ctypes.byref(n)), "ws")
    state[name] = (torch.empty(off[LV], device="cuda"), torch.empty(n.value, dtype=torch.uint8, device="cuda"))


def step(name):
    L = LIBS[name]
    pyr, ws = state[name]
    _lib.check(L.ecorr_build_split(f1.data_ptr(), f2.data_ptr(), B, D, H, W, Q, LV, pyr.data_ptr(), ws.data_ptr(), st),
               "build")
    for c in coords:
        _lib.check(L.ecorr_lookup(pyr.data_ptr(), c.data_ptr(), B, H, W, Q, LV, R, out.data_ptr(), st), "lookup")


with torch.no_grad():
    ref = None
    for name in LIBS:
        step(name)
        torch.cuda.synchronize()
        if ref is None:
            ref = out.clone()
            print("tree: reference output", flush=True)
        else:
            print(f"{name}: last lookup bitwise the tree's: {torch.equal(out.view(torch.int32), ref.view(torch.int32))}",
                  flush=True)
    times = {k: [] for k in LIBS}
    names = list(LIBS)
    for rnd in range(8):
        for name in names[rnd % len(names):] + names[:rnd % len(names)]:
            step(name)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(STEPS):
                step(name)
            e1.record()
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) / STEPS * 1e3)
res = {k: round(statistics.median(v), 1) for k, v in times.items()}
for k, v in res.items():
    print(f"step B={B} {k:14s} median {v:.1f} us", flush=True)
print(json.dumps({"ab_step_us": res}))
