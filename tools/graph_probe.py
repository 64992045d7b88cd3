#!/usr/bin/env python3
"""Launch-bound regime (BASELINE configs[2]-like, small volumes): CorrBlock build + 12 lookups and
the full ERAFT.forward, eager vs captured into one HIP graph (torch.cuda.CUDAGraph; the C-ABI
launches ride the capturing stream).  Prints per-step times and checks replay == eager bitwise."""
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import eraft_amd  # noqa: E402
import eraft_amd.network as nw  # noqa: E402
from e2e_weights import make_state_dict  # noqa: E402

dev = torch.device("cuda", 0)


def timeit(fn, reps=50):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts) * 1e3


def corr_case(B, H, W):
    g = torch.Generator(device=dev).manual_seed(1)
    f1 = torch.randn((B, 256, H, W), generator=g, device=dev)
    f2 = torch.randn((B, 256, H, W), generator=g, device=dev)
    base = eraft_amd.coords_grid(B, H, W, device=dev)
    coords = [(base + torch.randn((B, 2, H, W), generator=g, device=dev)).contiguous() for _ in range(12)]
    outs = []

    def step():
        blk = eraft_amd.CorrBlock(f1, f2)
        outs.clear()
        for c in coords:
            outs.append(blk(c))
    with torch.no_grad():
        step()
        eager = [o.clone() for o in outs]
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            step()
        torch.cuda.current_stream(dev).wait_stream(s)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            step()
        graph.replay()
        torch.cuda.synchronize()
        same = all(torch.equal(a, b) for a, b in zip(eager, outs))
        te, tg = timeit(step), timeit(graph.replay)
    print(f"CorrBlock B={B} {H}x{W}: eager {te:.3f} ms, graph {tg:.3f} ms ({te / tg:.2f}x), replay==eager {same}")


def eraft_case(B, H, W, bins):
    net = nw.ERAFT({"subtype": "warm_start"}, n_first_channels=bins, fuse_motion_corr=True, hip_upsample=True)
    net.load_state_dict(make_state_dict(net.state_dict()))
    net = net.eval().to(dev)
    g = torch.Generator(device=dev).manual_seed(2)
    im1 = torch.randn((B, bins, H, W), generator=g, device=dev)
    im2 = torch.randn((B, bins, H, W), generator=g, device=dev)
    init = torch.randn((B, 2, H // 8, W // 8), generator=g, device=dev)
    res = {}

    def step():
        low, ups = net(im1, im2, iters=12, flow_init=init)
        res["low"], res["up"] = low, ups[-1]
    with torch.no_grad():
        step()
        eager = (res["low"].clone(), res["up"].clone())
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            step()
        torch.cuda.current_stream(dev).wait_stream(s)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            step()
        graph.replay()
        torch.cuda.synchronize()
        same = torch.equal(eager[0], res["low"]) and torch.equal(eager[1], res["up"])
        te, tg = timeit(step, 20), timeit(graph.replay, 20)
    print(f"ERAFT warm start B={B} {bins}x{H}x{W}: eager {te:.2f} ms, graph {tg:.2f} ms ({te / tg:.2f}x), "
          f"replay==eager {same}")


corr_case(1, 32, 32)
corr_case(64, 32, 32)
corr_case(1, 60, 80)
eraft_case(1, 256, 256, 5)
