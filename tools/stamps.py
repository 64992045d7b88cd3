#!/usr/bin/env python3
"""Per-block timeline of the split build from the stamps lab build (tools/lab_build.py stamps):
s_memrealtime (100 MHz) at block start, after the K loop, after the epilogue, and the block's
HW_ID / XCC_ID.  Prints loop / epilogue durations, per-CU concurrency and the idle gaps.
  python tools/stamps.py tools/stamps_lab/e-raft_amd/libecorr.so [B H W]"""
import collections
import ctypes
import os
import statistics
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import eraft_amd  # noqa: E402
from eraft_amd import _lib  # noqa: E402

path = os.path.join(ROOT, sys.argv[1])
B, H, W = (int(x) for x in sys.argv[2:5]) if len(sys.argv) > 4 else (16, 60, 80)
L = ctypes.CDLL(path)
for name, (res, args) in _lib.SYMBOLS.items():
    getattr(L, name).restype = res
    getattr(L, name).argtypes = args
_lib._lib = L
g = torch.Generator(device="cuda").manual_seed(0)
with torch.no_grad():
    f1 = torch.randn((B, 256, H, W), generator=g, device="cuda")
    f2 = torch.randn((B, 256, H, W), generator=g, device="cuda")
    for _ in range(3):
        eraft_amd.CorrBlock(f1, f2)
    torch.cuda.synchronize()
nq = (H * W + 255) // 256
rem = H % 8
nreg = ((W + 15) // 16) * (H // 8 if 0 < rem <= 4 else (H + 7) // 8)
nnt = nreg + ((W + 31) // 32 if 0 < rem <= 4 else 0)
n = B * nq * nnt
buf = (ctypes.c_uint64 * (5 * n))()
assert L.ecorr_lab_stamps(buf, n) == 0
a = np.frombuffer(buf, dtype=np.uint64).reshape(n, 5).astype(np.int64)
t0, t1, t2, t3 = a[:, 0], a[:, 1], a[:, 2], a[:, 3]
hw = a[:, 4] >> 32
xcc = a[:, 4] & 0xF
cu = (hw >> 8) & 0xFF
base = t0.min()
us = lambda x: x / 100.0  # 100 MHz ticks -> us
loop, epi = us(t1 - t0), us(t2 - t1)
print(f"blocks {n}, kernel span {us(t2.max() - base):.1f} us")
print(f"loop  us: median {np.median(loop):.2f} p10 {np.percentile(loop, 10):.2f} p90 {np.percentile(loop, 90):.2f}")
iss = us(t3 - t1)
print(f"epilogue issue (all waves' stores issued) us: median {np.median(iss):.2f} p10 {np.percentile(iss, 10):.2f} p90 {np.percentile(iss, 90):.2f}")
print(f"epi   us: median {np.median(epi):.2f} p10 {np.percentile(epi, 10):.2f} p90 {np.percentile(epi, 90):.2f}")
if os.environ.get("STAMPS_PROLOGUE"):   # stamps4: slot 3 = prologue done (first barrier, t(0) landed)
    pro = us(t3 - t0)
    core = us(t1 - t3)
    print(f"prologue us: median {np.median(pro):.2f} p10 {np.percentile(pro, 10):.2f} p90 {np.percentile(pro, 90):.2f}")
    print(f"K loop (after prologue) us: median {np.median(core):.2f} p10 {np.percentile(core, 10):.2f} p90 {np.percentile(core, 90):.2f}")
    # dispatch gap: on each CU slot, the time from one block's end to the next block's start
    gaps = []
    for idx in [v for v in [[i for i in range(n) if (int(xcc[i]), int(cu[i])) == k] for k in list({(int(xcc[i]), int(cu[i])) for i in range(0, n, 97)})[:32]]]:
        ends = sorted(t2[idx])
        starts = sorted(t0[idx])
        for s0 in starts[2:]:
            prev = [e for e in ends if e <= s0]
            if prev:
                gaps.append(us(s0 - prev[-1]))
    if gaps:
        print(f"block start after the previous block end on the CU (us): median {np.median(gaps):.2f} p90 {np.percentile(gaps, 90):.2f}")
# per CU: slots, busy fraction, overlap of one block's epilogue with another's loop
cus = collections.defaultdict(list)
for i in range(n):
    cus[(int(xcc[i]), int(cu[i]))].append(i)
print(f"CUs seen {len(cus)}, blocks per CU median {statistics.median(len(v) for v in cus.values())}")
span = t2.max() - base
busy2, epi_vs_loop, epi_vs_epi, idle = 0, 0, 0, 0
grid = np.arange(base, t2.max(), 10)   # 0.1 us resolution
for k, idx in list(cus.items())[:64]:
    state_loop = np.zeros(len(grid), np.int32)
    state_epi = np.zeros(len(grid), np.int32)
    for i in idx:
        state_loop[(grid >= t0[i]) & (grid < t1[i])] += 1
        state_epi[(grid >= t1[i]) & (grid < t2[i])] += 1
    tot = state_loop + state_epi
    idle += np.mean(tot == 0)
    busy2 += np.mean(tot >= 2)
    epi_vs_loop += np.mean((state_epi >= 1) & (state_loop >= 1))
    epi_vs_epi += np.mean(state_epi >= 2)
m = min(64, len(cus))
print(f"per-CU time fractions (64 CUs): 2 blocks resident {busy2 / m:.2f}, epilogue beside a loop "
      f"{epi_vs_loop / m:.2f}, two epilogues {epi_vs_epi / m:.2f}, CU idle {idle / m:.3f}")
first = sorted(cus.items())[0]
print("first CU timeline (us from kernel start): " +
      " ".join(f"[{us(t0[i] - base):.1f} {us(t1[i] - base):.1f} {us(t2[i] - base):.1f}]" for i in sorted(first[1], key=lambda i: t0[i])[:12]))

# Loop progress rates by what the CU's other resident blocks are doing: per block, the time its K
# loop spent beside another block's loop (tL), beside another's epilogue (tE) or alone (t0);
# least squares for 1 loop = rL tL + rE tE + r0 t0 (rates in loops per us).
rows = []
for idx in cus.values():
    for i in idx:
        tl = te = 0.0
        for j in idx:
            if j == i:
                continue
            tl += max(0, min(t1[i], t1[j]) - max(t0[i], t0[j]))
            te += max(0, min(t1[i], t2[j]) - max(t0[i], t1[j]))
        tot = t1[i] - t0[i]
        rows.append((us(tl), us(te), us(max(0, tot - tl - te))))
A = np.array(rows)
sol, *_ = np.linalg.lstsq(A, np.ones(len(A)), rcond=None)
print("loop time split (median us): beside a loop {:.2f}, beside an epilogue {:.2f}, alone {:.2f}".format(*np.median(A, 0)))
print("fitted loop time at each rate (us): beside a loop {:.2f}, beside an epilogue {:.2f}, alone {:.2f}".format(*(1 / sol)))
