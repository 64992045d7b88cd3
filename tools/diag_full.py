#!/usr/bin/env python3
"""Where do two libraries' pyramids differ? (dev tool) Builds DSEC B=1 60x80 D=256 with the tree's
libecorr.so and AB_ALT_LIB, and per level prints the mismatch fraction and its distribution over
query row mod 64 / mod 16, target row / column."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import ab_build  # noqa: E402  (loads the libraries named in AB_ALT_LIB)

g = torch.Generator(device="cuda").manual_seed(0)
B, D, H, W = int(os.environ.get("DIAG_B", "1")), 256, 60, 80
f1 = torch.randn((B, D, H, W), generator=g, device="cuda")
f2 = torch.randn((B, D, H, W), generator=g, device="cuda")
libs = list(ab_build.LIBS.items())
with torch.no_grad():
    pa = [x.cpu().numpy() for x in ab_build.levels_of(libs[0][1], f1, f2)]
    pb = [x.cpu().numpy() for x in ab_build.levels_of(libs[1][1], f1, f2)]
for i, (a, b) in enumerate(zip(pa, pb)):
    a = a.reshape(B * H * W, a.shape[-2], a.shape[-1]); b = b.reshape(a.shape)
    bad = ~((a == b) | (np.isnan(a) & np.isnan(b)))
    print(f"level {i}: shape {a.shape} mismatch {bad.mean():.4f}")
    if bad.any():
        q = np.nonzero(bad.any(axis=(1, 2)))[0]
        print("  query rows bad:", len(q), "first", q[:20], "mod64 hist", np.bincount(q % 64, minlength=64)[:64].tolist())
        t = bad.any(axis=0)
        print("  target rows bad:", np.nonzero(t.any(axis=1))[0][:40].tolist())
        print("  target cols bad:", np.nonzero(t.any(axis=0))[0][:40].tolist())
        r = np.nonzero(bad)
        print("  sample", [(int(r[0][k]), int(r[1][k]), int(r[2][k]), float(a[r[0][k], r[1][k], r[2][k]]), float(b[r[0][k], r[1][k], r[2][k]])) for k in range(min(8, len(r[0])))])
