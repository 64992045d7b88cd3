#!/bin/bash
# Round 6: 16-byte-load operand pass -- build parity tests, the build A/B (bitwise pyramids + time),
# a kernel trace of a short bench.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/r6n; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_corr_gpu.py tests/test_level0_full_gpu.py tests/test_build_modes_gpu.py tests/test_rowshard_gpu.py > $OUT/pytest.txt 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $OUT/pytest.txt | head -30; tail -5 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
timeout -k 10 300 python3 tools/ab_build.py > $OUT/ab_build.txt 2>&1 || { echo "ab failed"; tail -20 $OUT/ab_build.txt; exit 1; }
tail -4 $OUT/ab_build.txt
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-next --no-e2e > $OUT/kt.log 2>&1 || { echo "kt failed"; tail -5 $OUT/kt.log; exit 1; }
grep '^{' $OUT/kt.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print(d['value'], d['corrblock_frac'], k['build']['ms_per_launch'], k['pack']['ms_per_launch'], k['lookup']['ms_per_launch'])"
python3 tools/kt_steady.py $OUT/kt/run_kernel_trace.csv | head -5
find $OUT -name '*kernel_trace.csv' -delete
echo DONE
