#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_voxel_gpu.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_voxel.log 2>&1
rc=$?; echo "pytest voxel rc=$rc"; grep -E "PASSED|FAILED|Error|assert|passed|failed" gpurun_out/pytest_voxel.log | tail -30
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_voxel.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_voxel.log | cut -c1-300
exit $rc
