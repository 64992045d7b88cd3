#!/usr/bin/env python3
"""Level-0 mismatch pattern between the tree library and AB_ALT_LIB at a small shape (dev tool):
for a few query rows prints both 8 x 16 target blocks, NaN counts, and whether the alternative's
values occur elsewhere in the tree's row (a permutation) or at a power-of-two scale."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import ab_build  # noqa: E402

B, D, H, W = (int(x) for x in os.environ.get("DIAG_SHAPE", "1,256,16,32").split(","))
g = torch.Generator(device="cuda").manual_seed(0)
f1 = torch.randn((B, D, H, W), generator=g, device="cuda")
f2 = torch.randn((B, D, H, W), generator=g, device="cuda")
libs = list(ab_build.LIBS.items())
with torch.no_grad():
    pa = [x.cpu().numpy() for x in ab_build.levels_of(libs[0][1], f1, f2)]
    pb = [x.cpu().numpy() for x in ab_build.levels_of(libs[1][1], f1, f2)]
np.set_printoptions(precision=3, linewidth=200, suppress=True)
a0 = pa[0].reshape(B * H * W, H, W)
b0 = pb[0].reshape(B * H * W, H, W)
print("level 0 nan in alt:", np.isnan(b0).mean(), "equal:", (a0 == b0).mean())
for q in [0, 1, 17, 64, 255, 256]:
    if q >= a0.shape[0]:
        continue
    print(f"query {q} tree block rows 0-7 cols 0-15:\n{a0[q, :8, :16]}\n alt:\n{b0[q, :8, :16]}")
    bv = b0[q].ravel()
    av = a0[q].ravel()
    found = sum(1 for x in bv[:64] if np.isfinite(x) and np.any(np.isclose(av, x, rtol=0, atol=0)))
    print(f" alt's first 64 values found in tree row: {found}/64")
    ratio = bv / np.where(av == 0, 1, av)
    print(" ratio sample", ratio[:8])
for i in range(1, 4):
    a = pa[i]; b = pb[i]
    print(f"level {i}: equal {(a == b).mean():.4f} nan {np.isnan(b).mean():.4f}")
# where do the alternative's wrong level-0 values come from?  For a sample of mismatches, the
# tree's (query, y, x) holding the closest value (relative 1e-5), as offsets from the right place
bad = np.argwhere((a0 != b0) & np.isfinite(b0))
print("mismatches:", len(bad), "by target half (x >> 3 & 1):", np.bincount((bad[:, 2] >> 3) & 1, minlength=2),
      "by target row y:", np.bincount(bad[:, 1], minlength=H)[:8], "by query % 64 // 16:", np.bincount(bad[:, 0] % 64 // 16, minlength=4))
flat = a0.ravel()
order = np.argsort(flat)
srt = flat[order]
rs = np.random.default_rng(0)
for q, y, x in bad[rs.choice(len(bad), size=min(12, len(bad)), replace=False)]:
    val = b0[q, y, x]
    i = np.searchsorted(srt, val)
    cands = []
    for j in range(max(0, i - 3), min(len(srt), i + 3)):
        if abs(srt[j] - val) <= 1e-5 * max(1.0, abs(val)):
            qq, yy, xx = np.unravel_index(order[j], a0.shape)
            cands.append((int(qq) - q, int(yy) - y, int(xx) - x))
    print(f" q {q} y {y} x {x}: alt {val:.5f} tree {a0[q, y, x]:.5f}; tree matches at (dq, dy, dx) {cands}")
