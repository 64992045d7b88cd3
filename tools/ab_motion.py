#!/usr/bin/env python3
"""A/B timing of the fused lookup + convc1 kernel's phases (dev knob ECORR_FUSED_PHASE) at the
bench shape, next to the unfused path; interleaved in one process."""
import os
import statistics
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import eraft_amd  # noqa: E402

B, H, W, D = 16, 60, 80, 256
g = torch.Generator(device="cuda").manual_seed(0)
VARIANTS = {"fused": "0", "lookup_phase": "1", "gemm_phase": "2"}
with torch.no_grad():
    f1 = torch.randn((B, D, H, W), generator=g, device="cuda")
    f2 = torch.randn((B, D, H, W), generator=g, device="cuda")
    blk = eraft_amd.CorrBlock(f1, f2)
    base = eraft_amd.coords_grid(B, H, W, device="cuda")
    coords = [(base + 2.0 * torch.randn((B, 2, H, W), generator=g, device="cuda")).contiguous() for _ in range(12)]
    wgt = torch.randn((256, 324, 1, 1), generator=g, device="cuda") * 0.05
    bias = torch.randn((256,), generator=g, device="cuda") * 0.1
    times = {k: [] for k in list(VARIANTS) + ["lookup", "unfused"]}

    def timed(fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for c in coords:
            fn(c)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / len(coords) * 1e3

    for rnd in range(6):
        for name, ph in VARIANTS.items():
            os.environ["ECORR_FUSED_PHASE"] = ph
            times[name].append(timed(lambda c: blk.lookup_conv1x1_relu(c, wgt, bias)))
        os.environ.pop("ECORR_FUSED_PHASE")
        times["lookup"].append(timed(lambda c: blk(c)))
        times["unfused"].append(timed(lambda c: torch.relu(F.conv2d(blk(c), wgt, bias))))
for name, ts in times.items():
    print(f"{name:14s} median {statistics.median(ts[1:]):8.1f} us/iter  min {min(ts[1:]):8.1f}")
