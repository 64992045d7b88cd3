#!/bin/bash
# PK build: parity (mode tests + corr + rowshard), interleaved build A/B, rocprof kernel trace.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/$1
TAG=${1:-pk}
timeout -k 10 400 python -u -m pytest tests/test_build_modes_gpu.py tests/test_corr_gpu.py tests/test_rowshard_gpu.py -x -q -s --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E 'normwise|FAILED|ERROR|passed|failed|Error' gpurun_out/pytest_$TAG.log | tail -12
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/ab_build.py > gpurun_out/ab_$TAG.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/ab_$TAG.log | tail -8
[ $rc -ne 0 ] && exit $rc
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/kt -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-next > gpurun_out/$TAG/kt.log 2>&1
rc=$?; echo "rocprof rc=$rc"; grep -o '"value": [0-9.]*' gpurun_out/$TAG/kt.log
f=$(find gpurun_out/$TAG/kt -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cut -d, -f1-4 "$f" | head -6 | cut -c1-60,200-
exit $rc
