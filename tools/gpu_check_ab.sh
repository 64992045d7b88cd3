#!/bin/bash
# Full GPU check (tests, smoke, bench) then an interleaved build A/B without the bitwise check
# (AB_ALT_LIB in $1: lab builds of another pyramid layout cannot be compared level by level).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
bash tools/gpu_check.sh || exit $?
AB_NOCHECK=1 AB_ALT_LIB="$1" AB_ROUNDS=12 timeout -k 10 300 python -u tools/ab_build.py > gpurun_out/ab_build.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/ab_build.log | tail -6
exit $rc
