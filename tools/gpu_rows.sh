#!/bin/bash
# GPU parity of the SURVEY §8f rows 2 and 4 + e2e + a bench line.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_splat_gpu.py tests/test_flow_gpu.py tests/test_e2e_gpu.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_rows.log 2>&1
rc=$?; echo "pytest rows rc=$rc"; grep -E "PASSED|FAILED|Error|assert|passed|failed|all-native" gpurun_out/pytest_rows.log | tail -40
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_rows.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_rows.log
exit $rc
