"""Lookup-only probe (DSEC B=16, 12 calls) for rocprofv3 PMC passes."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import eraft_amd  # noqa: E402

B, H, W, D = 16, 60, 80, 256
g = torch.Generator(device="cuda").manual_seed(0)
with torch.no_grad():
    f1 = torch.randn((B, D, H, W), generator=g, device="cuda")
    f2 = torch.randn((B, D, H, W), generator=g, device="cuda")
    blk = eraft_amd.CorrBlock(f1, f2)
    base = eraft_amd.coords_grid(B, H, W, device="cuda")
    init = torch.nn.functional.avg_pool2d(torch.randn((B, 2, H, W), generator=g, device="cuda") * 9.0, 5, 1, 2)
    coords = [(base + init + 0.5 * torch.randn((B, 2, H, W), generator=g, device="cuda")).contiguous() for _ in range(12)]
    for c in coords:
        blk(c)
    torch.cuda.synchronize()
print("ok")
