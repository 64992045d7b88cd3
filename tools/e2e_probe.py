#!/usr/bin/env python3
"""End-to-end ERAFT.forward throughput on one GPU (DSEC 480x640, 15 bins, 12 iterations, random
weights at the reference's init scales): the same network with (a) the reference's CorrBlock op
sequence on the GPU (oracle/torch_ref.py = ATen bmm / avg_pool2d / grid_sample), (b) eraft_amd's
CorrBlock, (c) + the fused lookup/convc1 and HIP convex upsampling.  Usage: e2e_probe.py [B]."""
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import eraft_amd.network as nw  # noqa: E402
from e2e_weights import make_state_dict  # noqa: E402
from torch_ref import TorchCpuCorrBlock  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4
dev = torch.device("cuda", 0)
torch.backends.cudnn.benchmark = True
g = torch.Generator(device=dev).manual_seed(0)
im1 = torch.randn((B, 15, 480, 640), generator=g, device=dev)
im2 = torch.randn((B, 15, 480, 640), generator=g, device=dev)


def build(fuse=False, hip_up=False):
    net = nw.ERAFT({"subtype": "standard"}, n_first_channels=15, fuse_motion_corr=fuse, hip_upsample=hip_up)
    net.load_state_dict(make_state_dict(net.state_dict()))
    return net.eval().to(dev)


def run(net, corr_cls=None, reps=5):
    saved = nw.CorrBlock
    if corr_cls is not None:
        nw.CorrBlock = corr_cls
    try:
        with torch.no_grad():
            net(im1, im2, iters=12)
            torch.cuda.synchronize()
            ts = []
            for _ in range(reps):
                t0 = time.perf_counter()
                net(im1, im2, iters=12)
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
    finally:
        nw.CorrBlock = saved
    return statistics.median(ts)


net = build()
t_ref = run(net, TorchCpuCorrBlock)
t_ours = run(net)
t_all = run(build(fuse=True, hip_up=True))
for name, t in (("reference CorrBlock ops on GPU", t_ref), ("eraft_amd CorrBlock", t_ours),
                ("eraft_amd CorrBlock + fused convc1 + HIP upsample", t_all)):
    print(f"B={B} {name:52s} {t * 1e3:8.1f} ms/forward  {B / t:7.1f} pairs/s")
