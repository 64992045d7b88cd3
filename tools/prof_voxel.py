#!/usr/bin/env python3
"""Event -> voxel grid probe for rocprofv3 kernel-trace / PMC passes: the DSEC
window bench.py's next_rows.voxel_grid_dsec times (1M events, 15 x 480 x 640, normalized), N calls.
  python tools/prof_voxel.py [N]
Summarize a PMC pass per call:  python tools/prof_voxel.py --summary <rocprof dir>"""
import collections
import csv
import glob
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VOXEL_KERNELS = ("VoxelArgs", "VTileArgs", "norm_finalize", "norm_apply", "scan_reduce", "scan_sums", "scan_apply")

if len(sys.argv) > 1 and sys.argv[1] == "--summary":
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    calls = collections.defaultdict(set)   # counter -> (file, dispatch) of each call's first kernel
    for f in glob.glob(os.path.join(sys.argv[2], "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "ecorr::" not in k or not any(v in k for v in VOXEL_KERNELS):
                continue
            short = k.replace("(anonymous namespace)", "").split("(")[0].split("::")[-1]   # ecorr::(anon)::gather<true>(...)
            per[r["Counter_Name"]][short] += float(r["Counter_Value"])
            if short.startswith(("prep", "vb_count")):
                calls[r["Counter_Name"]].add((f, r["Dispatch_Id"]))
    for name, ks in sorted(per.items()):
        n = max(1, len(calls[name]))
        tot = sum(ks.values()) / n
        print(f"{name}: {tot / 1e3:.2f} MB per call (KB counter / 1e3), {n} calls")
        for k, v in sorted(ks.items(), key=lambda t: -t[1]):
            print(f"    {k:24s} {v / n / 1e3:9.2f} MB")
    sys.exit(0)

import torch  # noqa: E402
sys.path.insert(0, ROOT)
import eraft_amd  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 5
n, C, H, W = 1_000_000, 15, 480, 640
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(8)   # bench.py measure_voxel's events
t = torch.sort(torch.rand((n,), generator=g, device=dev) * 1e5).values
ev = {"p": (torch.rand((n,), generator=g, device=dev) < 0.5).float(), "t": t - t[0],
      "x": torch.rand((n,), generator=g, device=dev) * (W + 2) - 1.5,
      "y": torch.rand((n,), generator=g, device=dev) * (H + 2) - 1.5}
vg = eraft_amd.VoxelGrid((C, H, W), normalize=True)
with torch.no_grad():
    for _ in range(N):
        vg.convert(ev)
    torch.cuda.synchronize()
print("ok")
