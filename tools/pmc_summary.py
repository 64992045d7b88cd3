#!/usr/bin/env python3
"""Summarize rocprofv3 --pmc CSVs (one dir per pass) into per-kernel averages per dispatch.

usage: tools/pmc_summary.py gpurun_out/<tag> [profiles/<tag>]
Every pmc* pass directory under <tag> (any depth) is keyed by the launch shape its bench run
printed (roofline.shape_key in <pass dir>.log); bench.py uses only a record of its own shape.
Writes <out>/pmc_summary.txt (human) and <out>/pmc_summary.json (bench.py reads the HBM traffic
of its dominant kernel from profiles/latest_pmc.json, a copy of the newest summary).

HBM traffic per dispatch, corrected as MI355X_MICROARCH.md §HBM prescribes: FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide (16 B/lane)
coalesced read, so read bytes = 2 * FETCH_SIZE * 1024 for kernels whose loads are 16-byte
vectors (the build).  The lookup's 8-byte buffer loads are an uncalibrated width: its read bytes
are reported uncorrected (1 * FETCH_SIZE) and flagged.  Infinity-Cache hits count as fabric
traffic (the counters sit at the L2's memory side).
"""
import collections
import csv
import glob
import json
import os
import sys

def source_digest():
    """Same digest as eraft_amd._lib.source_digest() (kept torch-free here): which kernel sources
    this summary measured; bench.py refuses a summary of other sources."""
    import hashlib
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    csrc = os.path.join(repo, "e-raft_amd", "csrc")
    files = sorted(os.path.join(csrc, f) for f in os.listdir(csrc)
                   if f.endswith((".hip", ".h")) or f == "Makefile")   # the Makefile: compile flags
    files.append(os.path.join(repo, "include", "ecorr.h"))
    h = hashlib.sha256()
    for f in files:
        h.update(os.path.basename(f).encode())
        h.update(open(f, "rb").read())
    return h.hexdigest()[:16]


root = sys.argv[1]
out = sys.argv[2] if len(sys.argv) > 2 else None


def shape_of(pmc_dir):
    """The launch shape of one PMC pass: roofline.shape_key of the bench JSON line in its log
    (<pass dir>.log, written by tools/profile.sh beside the pass directory)."""
    try:
        for ln in open(pmc_dir.rstrip("/") + ".log"):
            if ln.startswith("{"):
                return json.loads(ln)["roofline"]["shape_key"]
    except (OSError, ValueError, KeyError):
        pass
    return None


agg = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(list)))
for d in sorted(glob.glob(os.path.join(root, "**", "pmc*"), recursive=True)):
    if not os.path.isdir(d):
        continue
    key = shape_of(d)
    if key is None:
        print(f"# skipped {d}: no bench JSON with roofline.shape_key in {d}.log")
        continue
    for f in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if "ecorr" not in name:
                continue
            name = name.replace("void ", "").replace("ecorr::(anonymous namespace)::", "")
            name = name.split("(ecorr")[0].split("(int")[0].split("(float")[0].split("(LookupParams")[0]
            agg[key][name][r["Counter_Name"]].append(float(r["Counter_Value"]))
lines = ["# per-dispatch averages per launch shape (FETCH_SIZE / WRITE_SIZE in KiB as reported; gfx950",
         "# FETCH_SIZE reads ~1/2 of wide streaming bytes, MI355X_MICROARCH.md §HBM)"]
shapes = {}
for key in sorted(agg):
    lines.append(f"== {key}")
    js = {}
    for k, d in sorted(agg[key].items()):
        lines.append(k)
        avg = {c: sum(v) / len(v) for c, v in d.items()}
        for c, v in sorted(avg.items()):
            lines.append(f"  {c:28s} {v:16.1f}   (n={len(d[c])})")
        wide = k.startswith(("build_kernel", "build_split_kernel", "build_split16_kernel", "build_f32_kernel"))
        rec = {"counters": avg}
        if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
            rd = avg["FETCH_SIZE"] * 1024 * (2 if wide else 1)
            wr = avg["WRITE_SIZE"] * 1024
            rec.update(read_bytes=rd, write_bytes=wr, hbm_bytes=rd + wr,
                       read_correction="x2 (16-B/lane loads)" if wide else "none (dword loads, uncalibrated)")
            lines.append(f"  => HBM bytes/dispatch {rd + wr:.4g} (read {rd:.4g} {rec['read_correction']}, write {wr:.4g})")
        if "GRBM_GUI_ACTIVE" in avg:
            rec["grbm_gui_active"] = avg["GRBM_GUI_ACTIVE"]
        js[k] = rec
    shapes[key] = {"kernels": js}
txt = "\n".join(lines)
print(txt)
if out:
    os.makedirs(out, exist_ok=True)
    open(os.path.join(out, "pmc_summary.txt"), "w").write(txt + "\n")
    json.dump({"source": root, "source_digest": source_digest(), "shapes": shapes},
              open(os.path.join(out, "pmc_summary.json"), "w"), indent=1)
