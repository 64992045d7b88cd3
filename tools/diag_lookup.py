#!/usr/bin/env python3
"""Diagnose lookup mismatches vs a golden case: per level / coordinate set, count differing
outputs and print a few with their coordinates.  usage: python tools/diag_lookup.py [case]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)
import eraft_amd  # noqa: E402
from eraft_amd import _lib  # noqa: E402

case = sys.argv[1] if len(sys.argv) > 1 else "b2_8x12"
z = np.load(os.path.join(ROOT, "tests", "golden", f"corr_{case}.npz"))
L, r = int(z["L"]), int(z["r"])
levels = [z[f"level{i}"] for i in range(L)]
from eraft_amd.layout import tile  # noqa: E402
flat = torch.cat([tile(torch.from_numpy(lv)) for lv in levels]).cuda()
K = 2 * r + 1
for k in z.files:
    if not k.startswith("coords_"):
        continue
    s = k[7:]
    c = z[k]
    B, _, H, W = c.shape
    out = torch.empty((B, L * K * K, H, W), device="cuda")
    ct = torch.from_numpy(c).cuda()
    _lib.check(_lib.lib().ecorr_lookup(flat.data_ptr(), ct.data_ptr(), B, H, W, H * W, L, r,
                                       out.data_ptr(), _lib.stream_of(out)), "lookup")
    got = out.cpu().numpy()
    ref = z[f"out_{s}"]
    bad = ~((got == ref) | (np.isnan(got) & np.isnan(ref)))
    print(f"{s}: {bad.sum()} / {bad.size} differ; per level:",
          [int(bad[:, i * K * K:(i + 1) * K * K].sum()) for i in range(L)])
    idx = np.argwhere(bad)[:6]
    for b, ch, y, x in idx:
        print(f"   b={b} ch={ch} (lvl {ch // (K*K)}, a={ch % (K*K) // K}, b={ch % K}) q=({y},{x}) "
              f"coords=({c[b,0,y,x]:.6f},{c[b,1,y,x]:.6f}) got={got[b,ch,y,x]:.6g} ref={ref[b,ch,y,x]:.6g}")
