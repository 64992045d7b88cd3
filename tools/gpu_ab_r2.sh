#!/bin/bash
# Round-2 build A/B on the GPU: parity of the tree, then interleaved timing against lab builds.
#   AB_ALT_LIB list in $1 (checked against the tree bit for bit: first entry), ablations in $2
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_corr_gpu.py tests/test_build_modes_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_ab.log
[ $rc -ne 0 ] && exit $rc
AB_ALT_LIB="$1" AB_ROUNDS=12 timeout -k 10 300 python -u tools/ab_build.py > gpurun_out/ab_build.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/ab_build.log | tail -8
[ $rc -ne 0 ] && exit $rc
if [ -n "$2" ]; then
  AB_NOCHECK=1 AB_ALT_LIB="$2" AB_ROUNDS=12 timeout -k 10 300 python -u tools/ab_build.py > gpurun_out/ab_build_abl.log 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/ab_build_abl.log | tail -8
fi
exit $rc
