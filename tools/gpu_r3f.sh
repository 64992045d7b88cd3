#!/bin/bash
# split16 epilogue rework: parity tests of the build, A/B vs the previous split16, stamps.
cd "$GRAFT_REPO_ROOT"; TAG=${1:-r3e}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_corr_gpu.py tests/test_build_modes_gpu.py tests/test_rowshard_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest_build.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_build.log; [ $rc -ne 0 ] && exit $rc
AB_NOCHECK=1 AB_ROUNDS=12 AB_ALT_LIB=cur16=tools/cur16_lab/e-raft_amd/libecorr.so,ploop=tools/prio_loop_lab/e-raft_amd/libecorr.so,pepi=tools/prio_epi_lab/e-raft_amd/libecorr.so timeout -k 10 300 python -u tools/ab_build.py > $OUT/ab_build.log 2>&1
rc=$?; echo "ab_build rc=$rc"; grep -v amdgpu.ids $OUT/ab_build.log | tail -4; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/stamps16.py tools/st16_lab/e-raft_amd/libecorr.so > $OUT/stamps16.log 2>&1
rc=$?; echo "stamps16 rc=$rc"; grep -v amdgpu.ids $OUT/stamps16.log | tail -8
exit $rc
