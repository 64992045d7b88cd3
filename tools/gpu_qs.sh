#!/bin/bash
# build_qs_kernel vs the tree: pyramid bitwise at every ab_build shape + DSEC B=16 timing, then
# the B=16 per-level diff if the check fails.  usage: tools/gpu_qs.sh TAG [lab]
cd "$GRAFT_REPO_ROOT"; TAG=${1:-qs}; LAB=${2:-qs}; OUT=gpurun_out/$TAG; mkdir -p $OUT
AB_ROUNDS=10 AB_ALT_LIB=$LAB=tools/${LAB}_lab/e-raft_amd/libecorr.so timeout -k 10 300 python -u tools/ab_build.py > $OUT/ab_build.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/ab_build.log | tail -12
if [ $rc -ne 0 ]; then
  DIAG_B=16 AB_ALT_LIB=$LAB=tools/${LAB}_lab/e-raft_amd/libecorr.so timeout -k 10 200 python -u tools/diag_full.py > $OUT/diag.txt 2>&1
  grep -v amdgpu.ids $OUT/diag.txt | head -40
fi
exit $rc
