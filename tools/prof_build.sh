#!/bin/bash
# rocprofv3 kernel trace + HBM PMC passes over tools/run_build.py for each LIB given.
# usage: tools/prof_build.sh TAG LIB [LIB...]   (LIB = tree or a path to a libecorr.so)
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=$1; shift
for LIB in "$@"; do
  N=$(echo $LIB | tr '/.' '__')
  OUT=gpurun_out/$TAG/$N; mkdir -p $OUT
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 tools/run_build.py $LIB 10 > $OUT/kt.log 2>&1 || { echo "kt failed $LIB"; tail -5 $OUT/kt.log; exit 1; }
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES"; do
    i=$((i+1))
    timeout -k 10 90 rocprofv3 --pmc $grp -d $OUT/pmc$i -o run --output-format csv -- python3 tools/run_build.py $LIB 3 > $OUT/pmc$i.log 2>&1 || { echo "pmc $i failed $LIB"; tail -5 $OUT/pmc$i.log; exit 1; }
  done
  echo "== $LIB"
  f=$(find $OUT/kt -name '*kernel_stats.csv' | head -1); grep -E "build|pack" $f | cut -d, -f1-8
  python3 tools/pmc_summary.py $OUT | grep -E "^[a-z]|HBM|TCC|MFMA|GRBM"
done
