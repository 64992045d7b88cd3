#!/bin/bash
# Layout change A/B: GPU tests on the tree, build A/B (no bitwise check: the layouts differ), then
# the bench on the tree and on tools/prev_lab's library (the previous layout) on the same box.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
AB_NOCHECK=1 AB_ALT_LIB=prev=tools/prev_lab/e-raft_amd/libecorr.so AB_ROUNDS=12 timeout -k 10 300 python -u tools/ab_build.py > gpurun_out/ab_build.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/ab_build.log | tail -3; [ $rc -ne 0 ] && exit $rc
for k in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-next > gpurun_out/bench_tree$k.log 2>&1 || exit $?
  cp e-raft_amd/libecorr.so /tmp/tree.so && cp tools/prev_lab/e-raft_amd/libecorr.so e-raft_amd/libecorr.so
  sed -i 's/ABI_VERSION = 13/ABI_VERSION = 12/' e-raft_amd/_lib.py
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-next > gpurun_out/bench_prev$k.log 2>&1; rc=$?
  cp /tmp/tree.so e-raft_amd/libecorr.so; sed -i 's/ABI_VERSION = 12/ABI_VERSION = 13/' e-raft_amd/_lib.py
  [ $rc -ne 0 ] && exit $rc
done
python3 - <<'PY'
import json
for n in ("tree1", "prev1", "tree2", "prev2"):
    d = json.loads([x for x in open(f"gpurun_out/bench_{n}.log") if x.startswith("{")][-1])
    k = d["kernels"]
    print(n, d["value"], "gemm", k["build"]["ms_per_launch"], "pack", k["pack"]["ms_per_launch"], "lookup", k["lookup"]["ms_per_launch"])
PY
