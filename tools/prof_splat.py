"""Kernel-time probe for the warm-start splat (run under rocprofv3 --kernel-trace --stats)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import eraft_amd  # noqa: E402

B, H, W = (int(v) for v in (sys.argv[1:4] if len(sys.argv) > 3 else (16, 60, 80)))
g = torch.Generator(device="cuda").manual_seed(5)
flow = torch.nn.functional.avg_pool2d(torch.randn((B, 2, H, W), generator=g, device="cuda") * 9.0,
                                      5, stride=1, padding=2).contiguous()
for _ in range(20):
    eraft_amd.forward_interpolate_pytorch(flow)
torch.cuda.synchronize()
print("ok")
