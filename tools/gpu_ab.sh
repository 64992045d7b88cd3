#!/bin/bash
# Build-kernel A/B on the GPU: parity of the default and the MF16 variant, then interleaved timing.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_corr_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_ab.log
[ $rc -ne 0 ] && exit $rc
ECORR_BUILD_NOBAND=1 timeout -k 10 300 python -u -m pytest tests/test_corr_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_ab_mf16.log 2>&1
rc=$?; echo "pytest noband rc=$rc"; tail -2 gpurun_out/pytest_ab_mf16.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/ab_build.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/ab_build.log
