#!/usr/bin/env python3
"""does a FULL-epilogue store whose wave-uniform term rides in the scalar soffset
get lost?  (dev tool)  Builds DSEC 60x80 D=256 pyramids (B from SOFF_B, default 16) with each library
named in AB_ALT_LIB (plus the tree) into NaN-prefilled buffers, SOFF_REPS times, and reports the
elements never written per level, with their query rows (mod 256 = position in the 256-query block
tile, mod 64) and target tiles.
  AB_ALT_LIB=soff=tools/soff_full_lab/e-raft_amd/libecorr.so python tools/soff_repro.py"""
import collections
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from ab_lib_loader import load_libs  # noqa: E402
import eraft_amd  # noqa: E402
from eraft_amd import _lib  # noqa: E402
from eraft_amd.layout import formats, untile  # noqa: E402

B, D, H, W = int(os.environ.get("SOFF_B", "16")), 256, 60, 80
LV = 4
g = torch.Generator(device="cuda").manual_seed(0)
libs = load_libs()
with torch.no_grad():
    f1 = torch.randn((B, D, H, W), generator=g, device="cuda")
    f2 = torch.randn((B, D, H, W), generator=g, device="cuda")
    Q = H * W
    hs, ws, off = _lib.layout(B * Q, H, W, LV)
    ntx = formats(H, W, LV)
    ref = None
    for name, L in libs.items():
        _lib._lib = L
        tot = collections.Counter()
        rows = collections.Counter()
        for rep in range(int(os.environ.get("SOFF_REPS", "5"))):
            pyr = torch.full((off[-1],), float("nan"), device="cuda")
            ws_n = _lib._i64()
            _lib.check(L.ecorr_build_split_workspace_size(B, D, H, W, Q, ctypes.byref(ws_n)), "ws")
            wsb = torch.empty(ws_n.value, dtype=torch.uint8, device="cuda")
            st = _lib.stream_of(f1)
            _lib.check(L.ecorr_build_split(f1.data_ptr(), f2.data_ptr(), B, D, H, W, Q, LV, pyr.data_ptr(), wsb.data_ptr(), st), "build")
            torch.cuda.synchronize()
            if ref is None:
                ref = pyr.clone()
            elif rep == 0:
                same = torch.equal(pyr.view(torch.int32), ref.view(torch.int32))
                print(f"  {name}: pyramid bitwise {'same as' if same else 'DIFFERENT from'} the tree's", flush=True)
                for i in range(LV):
                    a = untile(pyr[off[i]:off[i + 1]], B * Q, hs[i], ws[i], ntx[i], i).view(B * Q, hs[i], ws[i])
                    t = untile(ref[off[i]:off[i + 1]], B * Q, hs[i], ws[i], ntx[i], i).view(B * Q, hs[i], ws[i])
                    d = a.view(torch.int32) != t.view(torch.int32)
                    nd = int(d.sum())
                    if not nd:
                        continue
                    r = d.any(dim=2).any(dim=1).nonzero().flatten()
                    print(f"    level {i}: {nd} elements differ in {r.numel()} rows; rows {r[:12].tolist()}", flush=True)
                    for q in r[:4].tolist():
                        yx = d[q].nonzero()
                        j = yx[0].tolist()
                        print(f"      row {q} (b {q // Q}, q {q % Q}, tile pos {q % Q % 256}, mod64 {q % 64}): {yx.shape[0]} px, "
                              f"rows {sorted(set(yx[:, 0].tolist()))[:10]} cols {sorted(set(yx[:, 1].tolist()))[:12]}; "
                              f"got {float(a[q][j[0], j[1]])} want {float(t[q][j[0], j[1]])}", flush=True)
            for i in range(LV):
                lv = untile(pyr[off[i]:off[i + 1]], B * Q, hs[i], ws[i], ntx[i], i).view(B * Q, hs[i], ws[i])
                bad = torch.isnan(lv)
                n = int(bad.sum())
                tot[i] += n
                if n and i == 0:
                    r = bad.any(dim=2).any(dim=1).nonzero().flatten().cpu().numpy()
                    for q in r[:64]:
                        rows[int(q)] += 1
                    if rep == 0:
                        qq = r[:6]
                        for q in qq:
                            yx = bad[q].nonzero().cpu().numpy()
                            print(f"  {name} rep0 level0 row {q} (b {q // Q}, q {q % Q}, in-tile {q % Q % 256}, mod64 {q % 64}): "
                                  f"{len(yx)} px, target rows {sorted(set((yx[:, 0] // 4).tolist()))} cols/8 {sorted(set((yx[:, 1] // 8).tolist()))}")
        print(f"{name}: unwritten elements per level over reps {dict(tot)}; distinct level-0 rows {len(rows)}", flush=True)
