#!/bin/bash
# Round 6: splat overflow paths -- parity tests, then their device time.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/r6f; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_splat_gpu.py > $OUT/pytest_splat.txt 2>&1 || { echo "splat tests failed"; tail -30 $OUT/pytest_splat.txt; exit 1; }
tail -2 $OUT/pytest_splat.txt
timeout -k 10 120 python -u tools/prof_splat_overflow.py > $OUT/splat_overflow.json 2> $OUT/splat_overflow.err || { echo "probe failed"; tail $OUT/splat_overflow.err; exit 1; }
cat $OUT/splat_overflow.json
