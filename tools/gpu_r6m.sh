#!/bin/bash
# Round 6: presplit lookup store ablations (timing only) via tools/ab_presplit.py's AB_ALT_LIB arm.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/r6m; mkdir -p $OUT
timeout -k 10 300 python3 tools/ab_presplit.py > $OUT/ab.json 2> $OUT/ab.err || { echo "ab failed"; tail -20 $OUT/ab.err; exit 1; }
cat $OUT/ab.json
