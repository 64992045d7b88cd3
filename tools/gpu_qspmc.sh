#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of build_qs_kernel vs build_split16_kernel (one ab_build round each),
# one PMC pass per counter.  usage: tools/gpu_qspmc.sh
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/qspmc; mkdir -p $OUT
export AB_NOCHECK=1 AB_ROUNDS=2 AB_ALT_LIB=qs=tools/qs_lab/e-raft_amd/libecorr.so
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 120 rocprofv3 --pmc $c -d $OUT/$c -o run --output-format csv -- python3 tools/ab_build.py > $OUT/$c.log 2>&1
  rc=$?; echo "pass $c rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $OUT/$c.log; exit $rc; fi
done
python3 - <<'PY'
import csv, glob, collections
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob(f"gpurun_out/qspmc/{c}/**/*counter_collection.csv", recursive=True):
        acc = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "build_" in k or "pack_" in k:
                acc[(k[:60], r["Dispatch_Id"])].append(float(r["Counter_Value"]))
        per = collections.defaultdict(list)
        for (k, d), v in acc.items():
            per[k].append(sum(v))
        for k, v in per.items():
            print(c, k, "dispatches", len(v), "median KB", sorted(v)[len(v) // 2])
PY
