"""Kernel-time probe for the SURVEY §8f kernels at the bench shapes (run under rocprofv3
--kernel-trace --stats): splat, upsample, PNG codec, voxel grid (DSEC, 1M events)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import eraft_amd  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(5)
B, H, W = 16, 60, 80
flow = torch.nn.functional.avg_pool2d(torch.randn((B, 2, H, W), generator=g, device=dev) * 9.0, 5, 1, 2).contiguous()
mask = torch.randn((B, 576, H, W), generator=g, device=dev) * 0.25
n = 1_000_000
t = torch.sort(torch.rand((n,), generator=g, device=dev) * 1e5).values
ev = {"p": (torch.rand((n,), generator=g, device=dev) < 0.5).float(), "t": t - t[0],
      "x": torch.rand((n,), generator=g, device=dev) * 642 - 1.5, "y": torch.rand((n,), generator=g, device=dev) * 482 - 1.5}
vg = eraft_amd.VoxelGrid((15, 480, 640), normalize=True)
up = eraft_amd.upsample_flow(flow, mask)
for _ in range(20):
    eraft_amd.forward_interpolate_pytorch(flow)
    eraft_amd.upsample_flow(flow, mask)
    eraft_amd.flow_to_png16(up)
    vg.convert(ev)
torch.cuda.synchronize()
print("ok")
