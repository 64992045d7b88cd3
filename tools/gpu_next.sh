#!/bin/bash
# GPU parity of the SURVEY §8f kernels + the full GPU suite + bench.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_motion_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_next.log 2>&1
rc=$?; echo "pytest next rc=$rc"; grep -E "PASSED|FAILED|Error|assert|passed|failed" gpurun_out/pytest_next.log | tail -20
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_check.sh
