#!/usr/bin/env python3
"""Per-kernel SQ counter medians (build_split16 vs build_qs) from tools/gpu_qssq.sh's passes.
usage: tools/qssq_parse.py LAB [LAB ...]"""
import collections
import csv
import glob
import sys

for lab in sys.argv[1:]:
    res = collections.defaultdict(dict)
    for i in (1, 2):
        for f in glob.glob(f"gpurun_out/qssq/{lab}{i}/**/*counter_collection.csv", recursive=True):
            acc = collections.defaultdict(lambda: collections.defaultdict(float))
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"]
                if "build_split16" in k or "build_qs" in k:
                    kk = "split16" if "build_split16" in k else "qs"
                    acc[(kk, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
            per = collections.defaultdict(lambda: collections.defaultdict(list))
            for (k, d), cs in acc.items():
                for c, v in cs.items():
                    per[k][c].append(v)
            for k, cs in per.items():
                for c, v in cs.items():
                    res[k][c] = sorted(v)[len(v) // 2]
    print(lab)
    print(f"   {'counter':24s} {'split16':>10s} {'qs':>10s}")
    for c in sorted(set(c for k in res for c in res[k])):
        print(f"   {c:24s} {res['split16'].get(c, 0):10.4g} {res['qs'].get(c, 0):10.4g}")
