#!/usr/bin/env python3
"""Device time of the banded splat's overflow paths: forward_interpolate on the
collision map of tests/test_splat_gpu.py (every pixel within a few pixels of one point: buckets of
~1,000 keys, sub-range re-evaluation) and on the one-target map (19,200 contributions in one bucket:
the single-thread ordered walk), against a DSEC warm-start field of the same size.  Median of 20
HIP-event-timed calls each.  Prints one JSON line."""
import json
import os
import statistics
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import eraft_amd  # noqa: E402

h, w = 60, 80
yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
maps = {
    "smooth_b16": (np.random.default_rng(0).standard_normal((16, 2, h, w)) * 1.5).astype(np.float32),
    "collisions_b3": np.repeat(np.stack([(40.25 - xx) * 0.99, (30.5 - yy) * 0.99])[None], 3, axis=0),
    "one_target_b2": np.repeat(np.stack([40.0 - xx, 30.0 - yy])[None], 2, axis=0),
}
out = {}
with torch.no_grad():
    for name, m in maps.items():
        flow = torch.from_numpy(np.ascontiguousarray(m, dtype=np.float32)).cuda()
        for _ in range(3):
            eraft_amd.forward_interpolate_pytorch(flow)
        ts = []
        for _ in range(20):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            eraft_amd.forward_interpolate_pytorch(flow)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        out[name] = {"batch": int(m.shape[0]), "us_per_call_median": round(statistics.median(ts), 1)}
print(json.dumps({"probe": "splat overflow paths (eager call incl. the Python wrapper)", "maps": out}))
