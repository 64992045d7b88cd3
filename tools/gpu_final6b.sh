#!/bin/bash
# Round 6 closing check after test-only / bench-only changes (the kernel sources and their PMC record
# unchanged): the GPU suite, smoke, the default bench line.
cd "$GRAFT_REPO_ROOT"; TAG=${1:-r6final4}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E 'FAILED|ERROR|passed|failed' $OUT/pytest_gpu.log | tail -5; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $OUT/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py > $OUT/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && { tail -20 $OUT/bench.log; exit $rc; }
grep '^{' $OUT/bench.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['corrblock_frac'], d['roofline'].get('traffic'), json.dumps(d['next_rows']['voxel_grid_mvsec'])[:200])"
