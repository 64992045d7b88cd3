#!/bin/bash
cd "$GRAFT_REPO_ROOT"
for k in 0 1 2 3 99; do
  ECORR_SPLAT_STOP=$k bash tools/kt.sh kt_splat_$k tools/prof_splat.py 16 60 80 | grep splat_kernel | cut -d, -f1-4
done
