#!/usr/bin/env python3
"""Per-kernel durations from a rocprofv3 kernel trace (run_kernel_trace.csv), over all dispatches
and past the clock ramp: the chip settles its clock over the first ~15 steps of sustained load
(DESIGN.md §5), so `steady` averages each kernel's dispatches from ordinal SKIP on (default 16).
  python tools/kt_steady.py path/to/kernel_trace.csv [SKIP]   -> a table and one JSON line"""
import collections
import csv
import json
import statistics
import sys


def main():
    path = sys.argv[1]
    skip = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    durs = collections.defaultdict(list)
    with open(path) as fh:
        for row in csv.DictReader(fh):
            name = row.get("Kernel_Name") or row.get("KernelName")
            t0, t1 = int(row["Start_Timestamp"]), int(row["End_Timestamp"])
            durs[name].append((t0, (t1 - t0) / 1e3))   # ns -> us
    res = {}
    for name, v in durs.items():
        v.sort()
        d = [x[1] for x in v]
        tail = d[skip:] if len(d) > skip else []
        res[name] = {"dispatches": len(d), "avg_us": round(statistics.mean(d), 2), "min_us": round(min(d), 2),
                     "max_us": round(max(d), 2),
                     "steady_avg_us": round(statistics.mean(tail), 2) if tail else None,
                     "steady_from_dispatch": skip if tail else None}
    width = max(len(n) for n in res) if res else 10
    print(f"{'kernel':{min(width, 70)}s} {'n':>5s} {'avg':>9s} {'steady':>9s} {'min':>9s} {'max':>9s}  (us)")
    for name, r in sorted(res.items(), key=lambda kv: -kv[1]["avg_us"] * kv[1]["dispatches"]):
        st = f"{r['steady_avg_us']:9.2f}" if r["steady_avg_us"] is not None else f"{'-':>9s}"
        print(f"{name[:70]:{min(width, 70)}s} {r['dispatches']:5d} {r['avg_us']:9.2f} {st} {r['min_us']:9.2f} {r['max_us']:9.2f}")
    print(json.dumps({"kernel_trace": path, "steady_from_dispatch": skip, "kernels": res}))


if __name__ == "__main__":
    main()
