#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_corr_gpu.py tests/test_rowshard_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_ab.log
[ $rc -gt 1 ] && exit $rc
ECORR_BUILD_KB32=1 timeout -k 10 300 python -u -m pytest tests/test_corr_gpu.py -x -q --timeout 200 --timeout-method thread -k "golden_case or bench_config" > gpurun_out/pytest_ab32.log 2>&1
rc=$?; echo "pytest kb32 rc=$rc"; tail -1 gpurun_out/pytest_ab32.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u tools/ab_build.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/ab_build.log
