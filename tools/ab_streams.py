#!/usr/bin/env python3
"""A/B: one batch of pairs as one stream vs split into sub-batches pipelined on S streams (the
lookups of one sub-batch overlap the MFMA-bound build of the next).  Same total work per step."""
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import eraft_amd  # noqa: E402

B, D, H, W, IT = int(os.environ.get("AB_BATCH", "16")), 256, 60, 80, 12
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
f1 = torch.randn((B, D, H, W), generator=g, device=dev)
f2 = torch.randn((B, D, H, W), generator=g, device=dev)
base = eraft_amd.coords_grid(B, H, W, device=dev)
init = torch.nn.functional.avg_pool2d(torch.randn((B, 2, H, W), generator=g, device=dev) * 9.0, 5, 1, 2)
coords = [(base + init + 0.5 * torch.randn((B, 2, H, W), generator=g, device=dev)).contiguous() for _ in range(IT)]


def make_plan(S):
    n = B // S
    parts = []
    for s in range(S):
        sl = slice(s * n, (s + 1) * n)
        parts.append((f1[sl].contiguous(), f2[sl].contiguous(), [c[sl].contiguous() for c in coords]))
    streams = [torch.cuda.Stream(dev) for _ in range(S)]
    return parts, streams


def step(plan):
    parts, streams = plan
    main = torch.cuda.current_stream(dev)
    prev_build = None
    for (a, b, cs), st in zip(parts, streams):
        st.wait_stream(main)
        if prev_build is not None:
            st.wait_event(prev_build)   # stagger: this build starts when the previous one ends
        with torch.cuda.stream(st):
            blk = eraft_amd.CorrBlock(a, b)
            ev = torch.cuda.Event()
            ev.record(st)
            prev_build = ev
            for c in cs:
                blk(c)
    for st in streams:
        main.wait_stream(st)


plans = {f"s{S}": make_plan(S) for S in (1, 2, 4)}
times = {k: [] for k in plans}
with torch.no_grad():
    for _ in range(3):
        for p in plans.values():
            step(p)
    torch.cuda.synchronize()
    for rnd in range(7):
        for k, p in plans.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                step(p)
            e1.record()
            torch.cuda.synchronize()
            times[k].append(e0.elapsed_time(e1) / 5)
for k, ts in times.items():
    med = statistics.median(ts)
    print(f"{k}: median {med:.3f} ms/step  min {min(ts):.3f}  -> {B / med * 1e3:.0f} pairs/s")
