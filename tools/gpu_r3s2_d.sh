#!/bin/bash
# Gray-order MFMA (tree) vs HEAD (bpair) A/B, and per-block stamps of the current split16 kernel.
cd "$GRAFT_REPO_ROOT"; TAG=${1:-r3s2d}; OUT=gpurun_out/$TAG; mkdir -p $OUT
AB_NOCHECK=1 AB_ROUNDS=16 AB_ALT_LIB=head=tools/head_lab/e-raft_amd/libecorr.so timeout -k 10 300 python -u tools/ab_build.py > $OUT/ab_build_gray.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/ab_build_gray.log | tail -3; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/stamps16.py tools/st16_lab/e-raft_amd/libecorr.so > $OUT/stamps16.txt 2>&1
rc=$?; grep -v amdgpu.ids $OUT/stamps16.txt | tail -30; exit $rc
