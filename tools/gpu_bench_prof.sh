#!/bin/bash
# GPU parity (corr only) + bench + profile passes.  usage: tools/gpu_bench_prof.sh TAG
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-prof}
timeout -k 10 300 python -u -m pytest tests/test_corr_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_corr.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_corr.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_$TAG.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_$TAG.log
[ $rc -ne 0 ] && exit $rc
bash tools/profile.sh $TAG
