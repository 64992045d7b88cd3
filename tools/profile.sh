#!/bin/bash
# rocprofv3 passes over a short bench run: kernel trace + stats, then one PMC group per pass
# (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE cannot share a pass).  Usage: tools/profile.sh TAG [bench args]
cd "$GRAFT_REPO_ROOT"
TAG=${1:-prof}; shift
ARGS=${@:---steps 3 --warmup 1 --no-cpu-baseline --no-next}
KT_ARGS=${KT_ARGS:---steps 20 --warmup 5 --no-cpu-baseline --no-next}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 bench.py $KT_ARGS > $OUT/kt.log 2>&1 || { echo "kernel-trace pass failed rc=$?"; tail -20 $OUT/kt.log; exit 1; }
echo "kt ok"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES" "TCC_HIT_sum TCC_MISS_sum" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp -d $OUT/pmc$i -o run --output-format csv -- python3 bench.py $ARGS > $OUT/pmc$i.log 2>&1
  rc=$?
  echo "pmc pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/pmc$i.log; exit $rc; fi
done
# HBM traffic of the other BASELINE configs (bench.py's roofline.traffic is keyed by launch shape)
for cfg in "c3:--batch 64 --height 32 --width 32" "c5:--mode rowshard"; do
  name=${cfg%%:*}; cargs=${cfg#*:}
  mkdir -p $OUT/$name
  j=0
  for grp in FETCH_SIZE WRITE_SIZE; do
    j=$((j+1))
    timeout -k 10 120 rocprofv3 --pmc $grp -d $OUT/$name/pmc$j -o run --output-format csv -- python3 bench.py $cargs --steps 3 --warmup 1 --no-cpu-baseline --no-next > $OUT/$name/pmc$j.log 2>&1
    rc=$?
    echo "$name pmc pass $j ($grp) rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 $OUT/$name/pmc$j.log; exit $rc; fi
  done
done
find $OUT -name '*.csv' | head -50
