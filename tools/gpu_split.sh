#!/bin/bash
# Split-build check: mode tests + corr parity + row-shard, then bench in both build modes.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_build_modes_gpu.py tests/test_corr_gpu.py tests/test_rowshard_gpu.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_split.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E 'normwise|PASSED|FAILED|ERROR|passed|failed|Error' gpurun_out/pytest_split.log | tail -40
[ $rc -ne 0 ] && exit $rc
for m in split fp32; do
  ECORR_BUILD_MODE=$m timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-next > gpurun_out/bench_$m.log 2>&1
  rc=$?; echo "bench $m rc=$rc"; tail -1 gpurun_out/bench_$m.log | cut -c1-200; grep -o '"kernels".*' gpurun_out/bench_$m.log | cut -c1-700
  [ $rc -ne 0 ] && exit $rc
done
exit 0
