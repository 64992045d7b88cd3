#!/bin/bash
# Queue one gpurun call; re-queue ONLY when gpurun reports exit 3 (no box: nothing ran, nothing
# charged), at most GQ_TRIES (20) attempts.  Any other exit code is final.  usage: tools/gpurun_q.sh LOG TIMEOUT CMD
LOG=$1; TO=$2; shift 2
for i in $(seq 1 ${GQ_TRIES:-20}); do
  timeout $((TO + 900)) /usr/local/graft/bin/gpurun --timeout $TO -- "$@" > $LOG 2>&1
  rc=$?
  echo "attempt $i exit=$rc" >> $LOG.attempts
  [ $rc -ne 3 ] && break
  sleep 120
done
echo "exit=$rc" >> $LOG
