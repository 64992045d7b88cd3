#!/bin/bash
# Operand-pass A/B: parity of the build tests on the single-launch pack, then interleaved timing of
# one launch (4-wave cap / uncapped) vs one launch per operand.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_corr_gpu.py tests/test_build_modes_gpu.py tests/test_rowshard_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_pack.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_pack.log
[ $rc -ne 0 ] && exit $rc
AB_ROUNDS=12 AB_VARIANTS='{"pack1": {}, "pack1_nocap": {"ECORR_BUILD_PACK2": "2"}, "pack2": {"ECORR_BUILD_PACK2": "1"}}' \
  timeout -k 10 300 python -u tools/ab_build.py > gpurun_out/ab_pack.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/ab_pack.log | tail -20; exit $rc
