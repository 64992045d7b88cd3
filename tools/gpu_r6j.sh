#!/bin/bash
# Round 6: tiled voxel path -- parity tests, kernel trace, A/B against lab builds (AB_ALT_LIB).
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/r6j; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_voxel_gpu.py > $OUT/pytest_voxel.txt 2>&1 || { echo "voxel tests failed"; tail -40 $OUT/pytest_voxel.txt; exit 1; }
tail -2 $OUT/pytest_voxel.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/voxkt -o run --output-format csv -- python3 tools/prof_voxel.py 10 > $OUT/voxkt.log 2>&1 || { echo "voxel kt failed"; tail -5 $OUT/voxkt.log; exit 1; }
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/r6j/voxkt/run_kernel_stats.csv')))
tot=0
for r in rows:
    if 'ecorr::' in r['Name'] or 'fillBuffer' in r['Name']:
        us=float(r['AverageNs'])/1e3; n=int(r['Calls'])
        if n==10: tot+=us
        print(f"{r['Name'][:80]:80s} calls {n:4d} avg {us:8.2f} us")
print("per call (10-call kernels):", round(tot,1), "us")
PY
if [ -n "$AB_ALT_LIB" ]; then
  timeout -k 10 200 python3 tools/ab_voxel.py > $OUT/ab_voxel.json 2> $OUT/ab_voxel.err || { echo "ab failed"; tail -5 $OUT/ab_voxel.err; exit 1; }
  cat $OUT/ab_voxel.json
fi
echo DONE
