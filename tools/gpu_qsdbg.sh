#!/bin/bash
# QS debug variants: level-0 equality vs the tree at a small shape (diag_qs), then the tree's split16 tests
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/qsdbg
for v in qsord qsseq; do
  AB_ALT_LIB=qs=tools/${v}_lab/e-raft_amd/libecorr.so timeout -k 10 120 python -u tools/diag_qs.py 2>&1 | grep -v amdgpu.ids > gpurun_out/qsdbg/$v.txt
  echo "== $v"; head -1 gpurun_out/qsdbg/$v.txt; tail -3 gpurun_out/qsdbg/$v.txt
done
timeout -k 10 400 python -u -m pytest tests/test_corr_gpu.py tests/test_build_modes_gpu.py -x -q --timeout 300 > gpurun_out/qsdbg/pytest_gray.log 2>&1
echo "pytest rc=$?"; tail -3 gpurun_out/qsdbg/pytest_gray.log
