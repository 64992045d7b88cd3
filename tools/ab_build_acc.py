#!/usr/bin/env python3
"""Level-0 accuracy of the CorrBlock build per library (tree + AB_ALT_LIB name=path,...): normwise
max|L0 - fp64| / rms(fp64) on i.i.d. fmaps (B = 2, 60 x 80, D = 256) and on fmaps with per-pixel
scales 2^-20..2^20 (per-row error relative to the row's own rms).  Lab probe for numerics variants
of the split (tools/lab_build.py lo8 / lo6).  One JSON line."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import ab_build  # noqa: E402

res = {}
g = torch.Generator(device="cuda").manual_seed(5)
B, D, H, W = 2, 256, 60, 80
f1 = torch.randn((B, D, H, W), generator=g, device="cuda")
f2 = torch.randn((B, D, H, W), generator=g, device="cuda")
s1 = torch.exp2(torch.linspace(-20, 20, H * W, device="cuda")).view(1, 1, H, W)
cases = {"iid": (f1, f2), "scaled": (f1 * s1, f2)}
with torch.no_grad():
    for cname, (a, b) in cases.items():
        ref = torch.einsum("bdq,bdt->bqt", a.view(B, D, -1).double(), b.view(B, D, -1).double()) / 16.0
        ref = ref.reshape(B * H * W, H * W)
        for name, L in ab_build.LIBS.items():
            l0 = ab_build.levels_of(L, a, b, 4)[0].reshape(B * H * W, H * W).double()
            d = (l0 - ref).abs()
            glob = float(d.max() / ref.pow(2).mean().sqrt())
            row = float((d.amax(dim=1) / ref.pow(2).mean(dim=1).sqrt()).max())
            res.setdefault(name, {})[cname] = {"normwise": glob, "max_row_normwise": row}
print(json.dumps({"probe": "level-0 accuracy vs fp64", "libs": res}))
