#!/bin/bash
# Round 6: split16 accumulators in AGPRs -- bitwise A/B of the whole build at the checked shapes, time.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/r6h; mkdir -p $OUT
AB_ROUNDS=12 AB_ALT_LIB=s16_rd8=tools/s16_rd8_lab/e-raft_amd/libecorr.so timeout -k 10 400 python -u tools/ab_build.py > $OUT/ab_rd8.txt 2>&1 || { echo "ab failed"; tail $OUT/ab_rd8.txt; exit 1; }
grep -E "DIFFERENT|median" $OUT/ab_rd8.txt; grep -c "same" $OUT/ab_rd8.txt
