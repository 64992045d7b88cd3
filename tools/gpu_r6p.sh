#!/bin/bash
# Round 6: the MVSEC voxel line (bench.measure_voxel_mvsec) and its kernel trace.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/r6p; mkdir -p $OUT
timeout -k 10 300 python3 -c "import bench, torch, json; print(json.dumps(bench.measure_voxel_mvsec(torch.device('cuda', 0))))" > $OUT/mvsec.json 2> $OUT/mvsec.err || { echo "mvsec failed"; tail -20 $OUT/mvsec.err; exit 1; }
cat $OUT/mvsec.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 -c "import bench, torch, json; print(json.dumps(bench.measure_voxel_mvsec(torch.device('cuda', 0))))" > $OUT/kt.log 2>&1 || { echo "kt failed"; tail -5 $OUT/kt.log; exit 1; }
python3 - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/r6p/kt/run_kernel_stats.csv')):
    print(f"{r['Name'][:90]:90s} calls {int(r['Calls']):5d} avg {float(r['AverageNs'])/1e3:9.2f} us")
PY
find $OUT -name '*kernel_trace.csv' -delete
