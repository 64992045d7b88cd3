#!/bin/bash
# K-loop breakdowns (tools/loopstamps.py) of the named loopstamps lab builds.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in $1; do
  echo "== $v"
  timeout -k 10 120 python -u tools/loopstamps.py tools/${v}_lab/e-raft_amd/libecorr.so > gpurun_out/loopstamps_$v.log 2>&1 || { cat gpurun_out/loopstamps_$v.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/loopstamps_$v.log
done
