#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for c in b2_8x12 t16x24 odd18x22; do
  timeout -k 10 120 python -u tools/diag_lookup.py $c > gpurun_out/diag_$c.log 2>&1 || { echo "diag $c rc=$?"; tail -5 gpurun_out/diag_$c.log; exit 1; }
  cat gpurun_out/diag_$c.log | grep -v amdgpu.ids
done
