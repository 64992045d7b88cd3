#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_e2e_gpu.py tests/test_rowshard_gpu.py -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_e2e.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E 'EPE|PASSED|FAILED|passed|failed|Error' gpurun_out/pytest_e2e.log | tail -20
exit $rc
