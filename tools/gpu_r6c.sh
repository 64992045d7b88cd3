#!/bin/bash
# Round 6: split convc1 variants (soffset column loads, prefetch distance 3), A/B in one process.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/r6c; mkdir -p $OUT
L=""; for n in ${CVS:-cv_mixasm}; do L="$L,$n=tools/${n}_lab/e-raft_amd/libecorr.so"; done
AB_ALT_LIB=${L#,} timeout -k 10 300 python -u tools/ab_conv.py > $OUT/cv.txt 2>&1 || { echo "cv failed"; tail -20 $OUT/cv.txt; exit 1; }
grep -E "normwise|median" $OUT/cv.txt
AB_CONV_IID=1 AB_ALT_LIB=${L#,} timeout -k 10 300 python -u tools/ab_conv.py > $OUT/cv_iid.txt 2>&1 || { echo "cv iid failed"; tail -20 $OUT/cv_iid.txt; exit 1; }
grep -E "normwise|median" $OUT/cv_iid.txt
echo DONE
