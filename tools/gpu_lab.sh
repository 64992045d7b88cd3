#!/bin/bash
# One lab call: optional GPU suite / bench, then A/Bs of lab builds against the tree.
#   RUN_TESTS=1 RUN_BENCH=1 AB="name1 name2" ABT="timing-only names" LK="lookup lab names" tools/gpu_lab.sh TAG
# AB: bitwise-checked build A/Bs (each alone vs the tree); ABT: timing-only build A/Bs (no check);
# LK: lookup A/Bs (tools/ab_lookup.py, bitwise-checked); STAMPS: build stamps labs (st16*);
# Every step under its own time limit,
# chained: the first failure ends the call.
cd "$GRAFT_REPO_ROOT"; TAG=${1:-lab}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
if [ -n "$LISTCTR" ]; then   # the PMC counters this box offers
  timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1; echo "counters rc=$?"
fi
if [ -n "$RUN_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E 'FAILED|ERROR|passed|failed' $OUT/pytest_gpu.log | tail -5; [ $rc -ne 0 ] && exit $rc
fi
if [ -n "$RUN_BENCH" ]; then
  timeout -k 10 400 python -u bench.py $BENCH_ARGS > $OUT/bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -c 600 $OUT/bench.log; echo; [ $rc -ne 0 ] && exit $rc
fi
for n in $AB; do
  AB_ALT_LIB=$n=tools/${n}_lab/e-raft_amd/libecorr.so timeout -k 10 300 python -u tools/ab_build.py > $OUT/ab_$n.log 2>&1
  rc=$?; echo "ab $n rc=$rc"; grep -E "DIFFERENT|differs|median" $OUT/ab_$n.log | tail -4; [ $rc -ne 0 ] && exit $rc
done
if [ -n "$ABT" ]; then
  L=""; for n in $ABT; do L="$L,$n=tools/${n}_lab/e-raft_amd/libecorr.so"; done
  AB_NOCHECK=1 AB_ALT_LIB=${L#,} timeout -k 10 400 python -u tools/ab_build.py > $OUT/abt.log 2>&1
  rc=$?; echo "abt rc=$rc"; grep median $OUT/abt.log; [ $rc -ne 0 ] && exit $rc
fi
if [ -n "$LK" ]; then   # all lookup labs in one process per coordinate field (smooth, i.i.d. sigma 3)
  L=""; for n in $LK; do L="$L,$n=tools/${n}_lab/e-raft_amd/libecorr.so"; done
  for f in smooth iid3; do
    AB_COORDS=$f AB_ALT_LIB=${L#,} timeout -k 10 300 python -u tools/ab_lookup.py > $OUT/lk_$f.log 2>&1
    rc=$?; echo "lk $f rc=$rc"; grep -E "DIFFERENT|differs|median" $OUT/lk_$f.log | tail -8; [ $rc -ne 0 ] && exit $rc
  done
fi
if [ -n "$MO" ]; then   # fused lookup + convc1 labs, one process
  L=""; for n in $MO; do L="$L,$n=tools/${n}_lab/e-raft_amd/libecorr.so"; done
  AB_ALT_LIB=${L#,} timeout -k 10 300 python -u tools/ab_motion.py > $OUT/mo.log 2>&1
  rc=$?; echo "mo rc=$rc"; grep -E "DIFFERENT|differs|median" $OUT/mo.log | tail -8; [ $rc -ne 0 ] && exit $rc
fi
if [ -n "$UP" ]; then   # convex upsampling labs, one process
  L=""; for n in $UP; do L="$L,$n=tools/${n}_lab/e-raft_amd/libecorr.so"; done
  AB_ALT_LIB=${L#,} timeout -k 10 300 python -u tools/ab_upsample.py > $OUT/up.log 2>&1
  rc=$?; echo "up rc=$rc"; grep -E "normwise|median" $OUT/up.log | tail -8; [ $rc -ne 0 ] && exit $rc
fi
if [ -n "$CV" ]; then   # split convc1 labs, one process
  L=""; for n in $CV; do L="$L,$n=tools/${n}_lab/e-raft_amd/libecorr.so"; done
  AB_ALT_LIB=${L#,} timeout -k 10 300 python -u tools/ab_conv.py > $OUT/cv.log 2>&1
  rc=$?; echo "cv rc=$rc"; grep -E "normwise|median" $OUT/cv.log | tail -8; [ $rc -ne 0 ] && exit $rc
fi
if [ -n "$STEP" ]; then   # whole-step labs (build + 12 lookups), one process
  L=""; for n in $STEP; do L="$L,$n=tools/${n}_lab/e-raft_amd/libecorr.so"; done
  AB_ALT_LIB=${L#,} timeout -k 10 300 python -u tools/ab_step.py > $OUT/step.log 2>&1
  rc=$?; echo "step rc=$rc"; grep -E "bitwise|median" $OUT/step.log | tail -10; [ $rc -ne 0 ] && exit $rc
fi
for n in $MOSTAMPS; do
  timeout -k 10 120 python -u tools/mostamps.py tools/${n}_lab/e-raft_amd/libecorr.so > $OUT/mostamps_$n.log 2>&1
  rc=$?; echo "mostamps $n rc=$rc"; tail -4 $OUT/mostamps_$n.log; [ $rc -ne 0 ] && exit $rc
done
for n in $STAMPS; do   # build stamps labs (tools/stamps16.py)
  timeout -k 10 120 python -u tools/stamps16.py tools/${n}_lab/e-raft_amd/libecorr.so > $OUT/stamps_$n.log 2>&1
  rc=$?; echo "stamps $n rc=$rc"; cat $OUT/stamps_$n.log | tail -7; [ $rc -ne 0 ] && exit $rc
done
exit 0
