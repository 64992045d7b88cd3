#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_corr_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_ab.log
[ $rc -gt 1 ] && exit $rc
ECORR_LOOKUP_QB=16 timeout -k 10 300 python -u -m pytest tests/test_corr_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_ab16.log 2>&1
rc=$?; echo "pytest qb16 rc=$rc"; tail -2 gpurun_out/pytest_ab16.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u tools/ab_lookup.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/ab_lookup.log
