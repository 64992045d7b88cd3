#!/bin/bash
# Round-3 check + lookup A/B (column-pair staging shifted to the true origin vs the round-2 staging)
# + per-block build stamps.  usage: tools/gpu_r3b.sh TAG
cd "$GRAFT_REPO_ROOT"; TAG=${1:-r3}; OUT=gpurun_out/$TAG; mkdir -p $OUT
bash tools/gpu_r3.sh $TAG || exit $?
for c in smooth iid3 iid40 int; do
  AB_COORDS=$c AB_ALT_LIB=prev=tools/prevlk_lab/e-raft_amd/libecorr.so timeout -k 10 200 python -u tools/ab_lookup.py > $OUT/ab_lookup_$c.log 2>&1
  rc=$?; echo "ab_lookup $c rc=$rc"; grep -v amdgpu.ids $OUT/ab_lookup_$c.log | tail -4; [ $rc -ne 0 ] && exit $rc
done
AB_NOCHECK=1 AB_ROUNDS=12 AB_ALT_LIB=prev=tools/prevbuild_lab/e-raft_amd/libecorr.so timeout -k 10 300 python -u tools/ab_build.py > $OUT/ab_build.log 2>&1
rc=$?; echo "ab_build rc=$rc"; grep -v amdgpu.ids $OUT/ab_build.log | tail -3; [ $rc -ne 0 ] && exit $rc
STAMPS_PROLOGUE=1 timeout -k 10 200 python -u tools/stamps.py tools/stamps4_lab/e-raft_amd/libecorr.so > $OUT/stamps4.log 2>&1
rc=$?; echo "stamps4 rc=$rc"; grep -v amdgpu.ids $OUT/stamps4.log | tail -14
exit $rc
