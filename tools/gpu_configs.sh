#!/bin/bash
# bench lines for the other BASELINE configs on one GPU: C3 (MVSEC 32x32 fmap, batch 64) and C5
# (1280x720 -> 92x160 fmap, batch 4, row-shard mode with one rank)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 200 python -u bench.py --batch 64 --height 32 --width 32 --steps 20 --warmup 5 --no-cpu-baseline --no-next > gpurun_out/bench_c3.log 2>&1
rc=$?; echo "c3 rc=$rc"; tail -1 gpurun_out/bench_c3.log | cut -c1-600
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u bench.py --mode rowshard --steps 10 --warmup 3 --no-cpu-baseline --no-next > gpurun_out/bench_c5.log 2>&1
rc=$?; echo "c5 rc=$rc"; tail -1 gpurun_out/bench_c5.log | cut -c1-600
exit $rc
