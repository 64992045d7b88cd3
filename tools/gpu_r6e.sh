#!/bin/bash
# Round 6: GEMM level-0 store locality (timing only, AB_NOCHECK).
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/r6e; mkdir -p $OUT
AB_NOCHECK=1 AB_ROUNDS=14 AB_ALT_LIB=l0contig=tools/l0contig_lab/e-raft_amd/libecorr.so,l0c1k=tools/l0c1k_lab/e-raft_amd/libecorr.so timeout -k 10 400 python -u tools/ab_build.py > $OUT/ab_l0c.txt 2>&1 || { echo "ab failed"; tail $OUT/ab_l0c.txt; exit 1; }
grep median $OUT/ab_l0c.txt
echo DONE
