#!/bin/bash
# Per-block timelines of the split build (stamps lab builds) + a timing A/B of a variant.
# usage: tools/gpu_stamps.sh "lab1 lab2 ..." [AB_ALT_LIB spec]
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in $1; do
  echo "== $v"
  timeout -k 10 120 python -u tools/stamps.py tools/${v}_lab/e-raft_amd/libecorr.so > gpurun_out/stamps_$v.log 2>&1 || { cat gpurun_out/stamps_$v.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/stamps_$v.log
done
if [ -n "$2" ]; then
  AB_ALT_LIB=$2 timeout -k 10 300 python -u tools/ab_build.py > gpurun_out/ab_stamps.log 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/ab_stamps.log | grep -v bitwise | tail -8; exit $rc
fi
