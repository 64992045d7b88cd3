#!/bin/bash
# Round-3 check: GPU tests, smoke, headline bench (+ optional C5 line).  usage: tools/gpu_r3.sh TAG
cd "$GRAFT_REPO_ROOT"; TAG=${1:-r3}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E 'FAILED|ERROR|passed|failed' $OUT/pytest_gpu.log | tail -20
[ $rc -gt 1 ] && exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $OUT/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py > $OUT/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 3000 $OUT/bench.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u bench.py --mode rowshard --steps 10 --warmup 3 --no-cpu-baseline --no-next > $OUT/bench_c5.log 2>&1
rc=$?; echo "c5 rc=$rc"; tail -c 600 $OUT/bench_c5.log
exit $rc
