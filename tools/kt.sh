#!/bin/bash
# rocprofv3 kernel trace + stats (csv) of a python script.  usage: tools/kt.sh TAG script.py [args]
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 "$@" > $OUT/kt.log 2>&1
rc=$?; echo "kt rc=$rc"
f=$(find $OUT -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cut -d, -f1-8 "$f" | head -20
exit $rc
