#!/usr/bin/env python3
"""Interleaved A/B timing of lookup variants (dev env knobs) in ONE process; outputs must be
bitwise identical across variants."""
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import eraft_amd  # noqa: E402

VARIANTS = {"cols3reg": {}, "cols3": {"ECORR_LOOKUP_V": "3"}, "staged4": {"ECORR_LOOKUP_V": "4"}}
if os.environ.get("AB_VARIANTS"):   # '{"name": {"KNOB": "v", ...}, ...}'
    import json
    VARIANTS = json.loads(os.environ["AB_VARIANTS"])
KNOBS = ("ECORR_LOOKUP_QB", "ECORR_LOOKUP_V", "ECORR_LOOKUP_SKIP")
B, H, W, D = int(os.environ.get("AB_BATCH", "16")), 60, 80, 256
g = torch.Generator(device="cuda").manual_seed(0)
with torch.no_grad():
    f1 = torch.randn((B, D, H, W), generator=g, device="cuda")
    f2 = torch.randn((B, D, H, W), generator=g, device="cuda")
    blk = eraft_amd.CorrBlock(f1, f2)
    base = eraft_amd.coords_grid(B, H, W, device="cuda")
    init = torch.nn.functional.avg_pool2d(torch.randn((B, 2, H, W), generator=g, device="cuda") * 9.0, 5, 1, 2)
    coords = [(base + init + 0.5 * torch.randn((B, 2, H, W), generator=g, device="cuda")).contiguous()
              for _ in range(12)]
    algo = B * H * W * 2904
    times = {k: [] for k in VARIANTS}
    ref = None
    names = list(VARIANTS)
    for rnd in range(int(os.environ.get("AB_ROUNDS", "6"))):
        # rotate the order every round: the first variant of a round runs measurably slower
        for name in names[rnd % len(names):] + names[:rnd % len(names)]:
            env = VARIANTS[name]
            for k in KNOBS:
                os.environ.pop(k, None)
            os.environ.update(env)
            out = blk(coords[0])
            torch.cuda.synchronize()
            if ref is None:
                ref = out.clone()
            elif rnd == 0 and "skip" not in name:
                assert torch.equal(out, ref), f"{name} output differs"
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for c in coords:
                blk(c)
            e1.record()
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) / len(coords))
for name, ts in times.items():
    med = statistics.median(ts)
    print(f"{name:8s} median {med * 1e3:.1f} us/call  min {min(ts) * 1e3:.1f}  -> {algo / med / 1e6:.0f} GB/s "
          f"algorithmic ({algo / med / 1e6 / 8000 * 100:.1f}% of 8 TB/s)")
