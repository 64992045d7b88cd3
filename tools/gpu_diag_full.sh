#!/bin/bash
# Where does the tree's pyramid differ from HEAD's (tools/head_lab)? DSEC B=16.
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/diag_full; mkdir -p $OUT
DIAG_B=16 AB_ALT_LIB=head=tools/head_lab/e-raft_amd/libecorr.so timeout -k 10 200 python -u tools/diag_full.py > $OUT/tree_vs_head.txt 2>&1; rc=$?
grep -v amdgpu.ids $OUT/tree_vs_head.txt; exit $rc
