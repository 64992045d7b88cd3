#!/bin/bash
# GPU parity of the splat + a bench line.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_splat_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_splat.log 2>&1
rc=$?; echo "pytest splat rc=$rc"; grep -E "PASSED|FAILED|Error|assert|passed|failed" gpurun_out/pytest_splat.log | tail -30
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_splat.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_splat.log
exit $rc
