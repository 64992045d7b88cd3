#!/bin/bash
# Round-3 profile: rocprof kernel trace + the PMC passes (tools/profile.sh), then the headline bench
# once more on the same box.  usage: tools/gpu_prof3.sh TAG
cd "$GRAFT_REPO_ROOT"; TAG=${1:-r3prof}; OUT=gpurun_out/$TAG; mkdir -p $OUT
bash tools/profile.sh $TAG || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; exit $rc
