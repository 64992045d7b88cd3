#!/bin/bash
# Round 6: the spawn-first bench tests (batch shard in both launcher forms, row shard self-launched).
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/r6i; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_batch_shard_gpu.py > $OUT/pytest_spawn.txt 2>&1 || { echo "spawn tests failed"; tail -40 $OUT/pytest_spawn.txt; exit 1; }
tail -6 $OUT/pytest_spawn.txt
