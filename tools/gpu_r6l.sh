#!/bin/bash
# Round 6: presplit convc1 -- its tests, the A/B probe, the bench's next_rows conv leg.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/r6l; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_conv_split_gpu.py tests/test_e2e_gpu.py > $OUT/pytest.txt 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $OUT/pytest.txt | head -30; exit 1; }
tail -2 $OUT/pytest.txt
timeout -k 10 300 python3 tools/ab_presplit.py > $OUT/ab_presplit.json 2> $OUT/ab_presplit.err || { echo "ab failed"; tail -20 $OUT/ab_presplit.err; exit 1; }
cat $OUT/ab_presplit.json
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench.log; exit 1; }
python3 - <<'PY'
import json
d = json.loads([l for l in open('gpurun_out/r6l/bench.log') if l.startswith('{')][-1])
print(json.dumps(d["next_rows"]["lookup_conv1x1_relu"]))
print(json.dumps(d["next_rows"].get("voxel_grid_dsec")))
PY
echo DONE
