#!/bin/bash
# split16 ablations: K loop alone (2 blocks / 1 block per CU), epilogue without its LDS transpose,
# loop priority stamps.  usage: tools/gpu_r3g.sh TAG
cd "$GRAFT_REPO_ROOT"; TAG=${1:-r3g}; OUT=gpurun_out/$TAG; mkdir -p $OUT
AB_NOCHECK=1 AB_ROUNDS=10 AB_ALT_LIB=noepi=tools/noepi16_lab/e-raft_amd/libecorr.so,noepi1cu=tools/noepi16_1cu_lab/e-raft_amd/libecorr.so,nolds=tools/e16nolds_lab/e-raft_amd/libecorr.so timeout -k 10 300 python -u tools/ab_build.py > $OUT/ab_build.log 2>&1
rc=$?; echo "ab_build rc=$rc"; grep -v amdgpu.ids $OUT/ab_build.log | tail -5; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/stamps16.py tools/st16_e16nolds_lab/e-raft_amd/libecorr.so > $OUT/stamps16_nolds.log 2>&1
rc=$?; echo "stamps16 nolds rc=$rc"; grep -v amdgpu.ids $OUT/stamps16_nolds.log | tail -8; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/stamps16.py tools/st16_prio_loop_lab/e-raft_amd/libecorr.so > $OUT/stamps16_ploop.log 2>&1
rc=$?; echo "stamps16 ploop rc=$rc"; grep -v amdgpu.ids $OUT/stamps16_ploop.log | tail -8
exit $rc
