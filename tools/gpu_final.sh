#!/bin/bash
# Round-end check: every GPU test, smoke, the headline bench, C3/C5 lines, a 2-rank batch-sharded
# rehearsal on one GPU (gloo), then the rocprof kernel trace + PMC passes.  usage: tools/gpu_final.sh TAG
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-final}
bash tools/gpu_check.sh || exit $?
bash tools/gpu_configs.sh || exit $?
BENCH_SINGLE_DEVICE=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --no-next > gpurun_out/bench_2rank.log 2>&1
rc=$?; echo "2-rank rehearsal rc=$rc"; grep -o '"value": [0-9.]*, "unit": "pairs/s", "n_gpus": 2' gpurun_out/bench_2rank.log
[ $rc -ne 0 ] && exit $rc
bash tools/profile.sh $TAG
