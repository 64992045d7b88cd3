#!/usr/bin/env python3
"""Summarize rocprofv3 --pmc CSVs (one dir per pass) into per-kernel averages per dispatch.
usage: tools/pmc_summary.py gpurun_out/<tag> > profiles/<tag>/pmc_summary.txt"""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, "pmc*", "*counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        if "ecorr" not in name:
            continue
        name = name.replace("void ", "").replace("ecorr::(anonymous namespace)::", "")
        name = name.split("(ecorr")[0].split("(int")[0]
        agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
print("# per-dispatch averages (FETCH_SIZE / WRITE_SIZE in KB as reported; gfx950 FETCH_SIZE reads")
print("# ~1/2 of wide streaming bytes, MI355X_MICROARCH.md §HBM)")
for k, d in sorted(agg.items()):
    print(k)
    for c, v in sorted(d.items()):
        print(f"  {c:28s} {sum(v) / len(v):16.1f}   (n={len(v)})")
