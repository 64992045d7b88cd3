#!/bin/bash
# Round 6, first call: the --gpus self-launch tests, per-call lookup timing + PMC, counter list,
# a short bench line.  Every GPU step under its own timeout, chained so that a failure ends the call.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/r6a; mkdir -p $OUT
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_batch_shard_gpu.py > $OUT/pytest_spawn.txt 2>&1 || { echo "spawn tests failed"; tail -30 $OUT/pytest_spawn.txt; exit 1; }
tail -3 $OUT/pytest_spawn.txt
timeout -k 10 300 python -u tools/lk_percall.py > $OUT/lk_percall.json 2> $OUT/lk_percall.err || { echo "percall failed"; tail -20 $OUT/lk_percall.err; exit 1; }
cat $OUT/lk_percall.json
timeout -k 10 120 rocprofv3 --list-avail > $OUT/counters.txt 2>&1 || echo "list-avail rc=$?"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  LK_PMC=1 LK_STEPS=3 timeout -s KILL 90 rocprofv3 --pmc $grp -d $OUT/pmc$i -o run --output-format csv -- python3 tools/lk_percall.py > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/pmc$i.log; exit 1; }
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-next --no-e2e > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
python3 -c "import json; r=json.load(open('$OUT/bench.json')); print(r['value'], r['ms_per_step'], r['corrblock_frac'], r['kernels']['build']['ms_per_launch'], r['kernels']['lookup']['ms_per_launch'])"
echo DONE
