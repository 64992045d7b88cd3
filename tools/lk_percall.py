#!/usr/bin/env python3
"""Per-call timing of the 12 lookups of a bench step: is call 1 (right after
the build, whose 1.96 GB pyramid store has cycled the Infinity Cache) slower than calls 2-12, whose
smooth-flow windows are mostly the lines call 1 fetched?

Arms (DSEC B=16, bench.py's make_inputs, seed 1234), per-call fence-free HIP events:
  step      build, then the 12 lookups of the bench's 12 coordinate fields (the bench step)
  again     the same block's 12 lookups once more right after `step` (no build in between)
  same      build, then coords[0] 12 times (identical windows every call)
  flushed   build, then per call a 512 MiB device write (evicts the Infinity Cache) before it
  iid       build, then 12 i.i.d. N(0, 3 px) fields
LK_PMC=1: only the `step` arm, a few steps, for a rocprofv3 --pmc pass (dispatch order = call
index).  Prints one JSON line."""
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import eraft_amd  # noqa: E402

B, D, H, W, IT = 16, 256, 60, 80, 12
dev = torch.device("cuda", 0)
steps = int(os.environ.get("LK_STEPS", "12"))
with torch.no_grad():
    f1, f2, coords = bench.make_inputs(B, D, H, W, IT, dev, seed=1234)
    g = torch.Generator(device=dev).manual_seed(7)
    base = eraft_amd.coords_grid(B, H, W, device=dev)
    iid = [(base + 3.0 * torch.randn((B, 2, H, W), generator=g, device=dev)).contiguous() for _ in range(IT)]
    flush = torch.empty(512 << 18, dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(dev)
    ev = [bench.timing_event() for _ in range(2 * IT)]

    def calls(blk, fields, flush_each=False):
        for k, c in enumerate(fields):
            if flush_each:
                flush.fill_(float(k))
            ev[2 * k].record(stream)
            blk(c)
            ev[2 * k + 1].record(stream)
        torch.cuda.synchronize()
        return [ev[2 * k].elapsed_time(ev[2 * k + 1]) * 1e3 for k in range(IT)]

    arms = {} if os.environ.get("LK_PMC") else {"step": [], "again": [], "same": [], "flushed": [], "iid": []}
    if os.environ.get("LK_PMC"):
        for _ in range(steps):
            blk = eraft_amd.CorrBlock(f1, f2)
            for c in coords:
                blk(c)
        torch.cuda.synchronize()
        print("ok")
        raise SystemExit(0)
    for _ in range(3):   # warm-up
        blk = eraft_amd.CorrBlock(f1, f2)
        calls(blk, coords)
    for s in range(steps):
        blk = eraft_amd.CorrBlock(f1, f2)
        arms["step"].append(calls(blk, coords))
        arms["again"].append(calls(blk, coords))
        blk = eraft_amd.CorrBlock(f1, f2)
        arms["same"].append(calls(blk, [coords[0]] * IT))
        blk = eraft_amd.CorrBlock(f1, f2)
        arms["flushed"].append(calls(blk, coords, flush_each=True))
        blk = eraft_amd.CorrBlock(f1, f2)
        arms["iid"].append(calls(blk, iid))
    out = {}
    for name, rows in arms.items():
        per = [round(statistics.median(r[k] for r in rows), 2) for k in range(IT)]
        out[name] = {"us_per_call_median": per, "call1": per[0],
                     "calls2_12_mean": round(sum(per[1:]) / (IT - 1), 2)}
    print(json.dumps({"probe": "lookup per call", "steps": steps, "arms": out}))
