#!/bin/bash
# split16 vs 32x32 build A/B, split16 stamps, lookup ablations.  usage: tools/gpu_r3c.sh TAG
cd "$GRAFT_REPO_ROOT"; TAG=${1:-r3c}; OUT=gpurun_out/$TAG; mkdir -p $OUT
AB_NOCHECK=1 AB_ROUNDS=12 AB_ALT_LIB=s32=tools/s32_lab/e-raft_amd/libecorr.so,prev=tools/prevbuild_lab/e-raft_amd/libecorr.so timeout -k 10 300 python -u tools/ab_build.py > $OUT/ab_build.log 2>&1
rc=$?; echo "ab_build rc=$rc"; grep -v amdgpu.ids $OUT/ab_build.log | tail -4; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/stamps16.py tools/st16_lab/e-raft_amd/libecorr.so > $OUT/stamps16.log 2>&1
rc=$?; echo "stamps16 rc=$rc"; grep -v amdgpu.ids $OUT/stamps16.log | tail -8; [ $rc -ne 0 ] && exit $rc
AB_NOCHECK=1 AB_COORDS=smooth AB_ALT_LIB=noblend=tools/lk_noblend_lab/e-raft_amd/libecorr.so,nostore=tools/lk_nostore_lab/e-raft_amd/libecorr.so timeout -k 10 200 python -u tools/ab_lookup.py > $OUT/ab_lookup_abl.log 2>&1
rc=$?; echo "ab_lookup ablations rc=$rc"; grep -v amdgpu.ids $OUT/ab_lookup_abl.log | tail -4
exit $rc
