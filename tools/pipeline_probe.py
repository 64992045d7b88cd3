#!/usr/bin/env python3
"""Throughput of the bench step (CorrBlock build + 12 lookups, DSEC B=16) run back to back on one
stream vs pipelined over two streams (batch s + 1's build beside batch s's lookups).
  python tools/pipeline_probe.py [steps]"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import eraft_amd  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
B, D, H, W = 16, 256, 60, 80
g = torch.Generator(device="cuda").manual_seed(0)
with torch.no_grad():
    f1 = [torch.randn((B, D, H, W), generator=g, device="cuda") for _ in range(2)]
    f2 = [torch.randn((B, D, H, W), generator=g, device="cuda") for _ in range(2)]
    base = eraft_amd.coords_grid(B, H, W, device="cuda")
    coords = [(base + torch.randn((B, 2, H, W), generator=g, device="cuda")).contiguous() for _ in range(12)]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]

    def step(s, st):
        with torch.cuda.stream(st):
            blk = eraft_amd.CorrBlock(f1[s % 2], f2[s % 2])
            for c in coords:
                out = blk(c)
        return blk, out

    def run(pipelined):
        keep = []
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for s in range(steps):
            keep.append(step(s, streams[s % 2] if pipelined else streams[0]))
            if len(keep) > 2:
                keep.pop(0)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps * 1e3

    for mode in (False, True, False, True):
        run(mode)
    res = {m: min(run(m) for _ in range(3)) for m in (False, True)}
    for m, ms in res.items():
        print(f"{'pipelined 2 streams' if m else 'one stream         '}: {ms:.3f} ms/step  {B / ms * 1e3:.0f} pairs/s")
