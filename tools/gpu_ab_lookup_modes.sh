#!/bin/bash
# Lookup A/B (tools/ab_lookup.py) on every coordinate field of SURVEY 8(d): smooth, i.i.d. sigma 3,
# sigma 40.  usage: AB_ALT_LIB=name=path tools/gpu_ab_lookup_modes.sh TAG
cd "$GRAFT_REPO_ROOT"; TAG=${1:-ablk}; OUT=gpurun_out/$TAG; mkdir -p $OUT
for m in smooth iid3 iid40; do
  AB_COORDS=$m timeout -k 10 240 python -u tools/ab_lookup.py > $OUT/ab_lookup_$m.log 2>&1
  rc=$?; grep -v amdgpu.ids $OUT/ab_lookup_$m.log | tail -4; [ $rc -ne 0 ] && exit $rc
done
exit 0
