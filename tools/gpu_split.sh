#!/bin/bash
# Split-build check: mode tests + corr parity + row-shard, then bench per build variant and a
# rocprof kernel trace of the default.  usage: tools/gpu_split.sh TAG
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-split}
timeout -k 10 400 python -u -m pytest tests/test_build_modes_gpu.py tests/test_corr_gpu.py tests/test_rowshard_gpu.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E 'normwise|FAILED|ERROR|passed|failed|Error' gpurun_out/pytest_$TAG.log | tail -20
[ $rc -ne 0 ] && exit $rc
for v in "split" "split ECORR_BUILD_PK=0" "fp32"; do
  set -- $v; m=$1; shift
  env ECORR_BUILD_MODE=$m $@ timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-next > gpurun_out/bench_$TAG.log 2>&1
  rc=$?; echo "bench $v rc=$rc"; grep -o '"value": [0-9.]*' gpurun_out/bench_$TAG.log; grep -o '"kernels".*' gpurun_out/bench_$TAG.log | cut -c1-420
  [ $rc -ne 0 ] && exit $rc
done
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/kt -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-next > gpurun_out/$TAG/kt.log 2>&1
rc=$?; echo "rocprof rc=$rc"
f=$(find gpurun_out/$TAG/kt -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cut -d, -f1-4 "$f" | head -12
exit $rc
