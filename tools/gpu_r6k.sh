#!/bin/bash
# Round 6: presplit convc1 (ABI 16) -- conv / lookup GPU tests, then the A/B probe and a kernel trace.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/r6k; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_conv_split_gpu.py tests/test_motion_gpu.py tests/test_corr_gpu.py > $OUT/pytest.txt 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error|assert" $OUT/pytest.txt | head -30; tail -30 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
timeout -k 10 300 python3 tools/ab_presplit.py > $OUT/ab_presplit.json 2> $OUT/ab_presplit.err || { echo "ab failed"; tail -20 $OUT/ab_presplit.err; exit 1; }
cat $OUT/ab_presplit.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 tools/ab_presplit.py > $OUT/kt.log 2>&1 || { echo "kt failed"; tail -5 $OUT/kt.log; exit 1; }
python3 - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/r6k/kt/run_kernel_stats.csv')):
    if any(k in r['Name'] for k in ('lookup_cols_reg', 'conv1x1_split', 'colscale', 'split_pack')):
        print(f"{r['Name'][:100]:100s} calls {int(r['Calls']):5d} avg {float(r['AverageNs'])/1e3:8.2f} us")
PY
find $OUT -name '*kernel_trace.csv' -delete
echo DONE
