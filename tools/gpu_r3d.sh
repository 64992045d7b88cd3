#!/bin/bash
# split16: stamps (tree, epilogue stores out of range) + A/B.  usage: tools/gpu_r3d.sh TAG
cd "$GRAFT_REPO_ROOT"; TAG=${1:-r3d}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 200 python -u tools/stamps16.py tools/st16_lab/e-raft_amd/libecorr.so > $OUT/stamps16.log 2>&1
rc=$?; echo "stamps16 rc=$rc"; grep -v amdgpu.ids $OUT/stamps16.log | tail -8; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/stamps16.py tools/st16_e16oob_lab/e-raft_amd/libecorr.so > $OUT/stamps16_e16oob.log 2>&1
rc=$?; echo "stamps16 e16oob rc=$rc"; grep -v amdgpu.ids $OUT/stamps16_e16oob.log | tail -8; [ $rc -ne 0 ] && exit $rc
AB_NOCHECK=1 AB_ROUNDS=12 AB_ALT_LIB=e16oob=tools/e16oob_lab/e-raft_amd/libecorr.so,prev=tools/prevbuild_lab/e-raft_amd/libecorr.so timeout -k 10 300 python -u tools/ab_build.py > $OUT/ab_build.log 2>&1
rc=$?; echo "ab_build rc=$rc"; grep -v amdgpu.ids $OUT/ab_build.log | tail -4
exit $rc
