#!/bin/bash
# Interleaved lookup A/B (tools/ab_lookup.py) against the lab builds named in AB_ALT_LIB.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ab_lookup.py > gpurun_out/ab_lookup.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/ab_lookup.log | tail -12; exit $rc
