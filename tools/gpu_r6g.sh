#!/bin/bash
# Round 6: re-measure the GEMM and lookup bounds DESIGN.md states (timing-only ablations, one box).
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/r6g; mkdir -p $OUT
L=""; for n in s16_noepi s16_stoob noscale; do L="$L,$n=tools/${n}_lab/e-raft_amd/libecorr.so"; done
AB_NOCHECK=1 AB_ROUNDS=12 AB_ALT_LIB=${L#,} timeout -k 10 400 python -u tools/ab_build.py > $OUT/ab_build_bounds.txt 2>&1 || { echo "ab failed"; tail $OUT/ab_build_bounds.txt; exit 1; }
grep median $OUT/ab_build_bounds.txt
for n in st16 st16_s16stoob; do
  timeout -k 10 120 python -u tools/stamps16.py tools/${n}_lab/e-raft_amd/libecorr.so > $OUT/stamps_$n.txt 2>&1 || { echo "stamps $n failed"; tail $OUT/stamps_$n.txt; exit 1; }
  echo "== $n"; tail -8 $OUT/stamps_$n.txt
done
L=""; for n in lk_ldoob lk_stoob lk_bothoob; do L="$L,$n=tools/${n}_lab/e-raft_amd/libecorr.so"; done
AB_NOCHECK=1 AB_COORDS=smooth AB_ALT_LIB=${L#,} timeout -k 10 300 python -u tools/ab_lookup.py > $OUT/lk_oob_smooth.txt 2>&1 || { echo "lk failed"; tail $OUT/lk_oob_smooth.txt; exit 1; }
grep median $OUT/lk_oob_smooth.txt
echo DONE
