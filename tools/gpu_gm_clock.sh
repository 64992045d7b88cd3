#!/bin/bash
# GEMM tile-group (decode_tile GM) arms: whole-build A/B in one process, per-block clock stamps, and
# L2 PMC per dispatch.  usage: ARMS="gm9 gm10" STAMPS="st16 st16_gm10" tools/gpu_gm_clock.sh TAG
cd "$GRAFT_REPO_ROOT"; TAG=${1:-gm}; OUT=gpurun_out/$TAG; mkdir -p $OUT
ABT="$ARMS" STAMPS="$STAMPS" bash tools/gpu_lab.sh $TAG || exit $?
for n in tree $ARMS; do
  if [ $n = tree ]; then LIB=e-raft_amd/libecorr.so; else LIB=tools/${n}_lab/e-raft_amd/libecorr.so; fi
  bash tools/pmc_kernel.sh $TAG/pmc_$n build_split16 "tools/pmc_one.py $LIB 20" "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES" > $OUT/pmc_$n.txt 2>&1 || exit $?
  echo "== $n"; grep -E "TCC_MISS|FETCH|GRBM" $OUT/pmc_$n.txt
done
