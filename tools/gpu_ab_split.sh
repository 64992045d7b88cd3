#!/bin/bash
# Interleaved build A/B (tools/ab_build.py) with the variants in $AB_VARIANTS.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ab_build.py > gpurun_out/ab_split.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/ab_split.log | tail -20; exit $rc
