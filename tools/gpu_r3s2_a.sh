#!/bin/bash
# Round-3 session-2 lab call: lookup variants on all three coordinate fields, split16 MFMA-order
# variants (timing; level 0 moves by roundings), store-pattern rates.  usage: tools/gpu_r3s2_a.sh TAG
cd "$GRAFT_REPO_ROOT"; TAG=${1:-r3s2a}; OUT=gpurun_out/$TAG; mkdir -p $OUT
AB_ALT_LIB=occ5=tools/lkocc5_lab/e-raft_amd/libecorr.so,pipe=tools/lkpipe_lab/e-raft_amd/libecorr.so,pipe2=tools/lkpipe2_lab/e-raft_amd/libecorr.so bash tools/gpu_ab_lookup_modes.sh $TAG/lk || exit $?
AB_NOCHECK=1 AB_ALT_LIB=bpair=tools/mo_bpair_lab/e-raft_amd/libecorr.so,a8=tools/mo_a8_lab/e-raft_amd/libecorr.so timeout -k 10 300 python -u tools/ab_build.py > $OUT/ab_build_mo.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/ab_build_mo.log | tail -5; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 ./tools/store_lab 10 > $OUT/store_lab.txt 2>&1
rc=$?; cat $OUT/store_lab.txt; exit $rc
