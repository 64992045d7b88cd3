#!/bin/bash
# Round-3 session-2: GPU suite on the tree (11-slot lookup rows, FULL split16 epilogue), then A/B
# against HEAD's library (tools/head_lab) for the build and the lookup, the bpair MFMA order, and
# the gather roofline probe.  usage: tools/gpu_r3s2_b.sh TAG
cd "$GRAFT_REPO_ROOT"; TAG=${1:-r3s2b}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
AB_ALT_LIB=head=tools/head_lab/e-raft_amd/libecorr.so timeout -k 10 300 python -u tools/ab_build.py > $OUT/ab_build_head.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/ab_build_head.log | tail -4; [ $rc -ne 0 ] && exit $rc
AB_NOCHECK=1 AB_ROUNDS=16 AB_ALT_LIB=bpair=tools/mo_bpair_lab/e-raft_amd/libecorr.so timeout -k 10 300 python -u tools/ab_build.py > $OUT/ab_build_bpair.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/ab_build_bpair.log | tail -3; [ $rc -ne 0 ] && exit $rc
AB_ALT_LIB=head=tools/head_lab/e-raft_amd/libecorr.so bash tools/gpu_ab_lookup_modes.sh $TAG/lk || exit $?
timeout -k 10 120 ./tools/gather_lab 10 > $OUT/gather_lab.txt 2>&1
rc=$?; cat $OUT/gather_lab.txt; exit $rc
