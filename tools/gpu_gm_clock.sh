cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r5gm2; mkdir -p $OUT
STAMPS="st16 st16_gm2 st16_gm4 st16_gm16" bash tools/gpu_lab.sh r5gm2 || exit $?
for n in tree gm2 gm4 gm16; do
  if [ $n = tree ]; then LIB=e-raft_amd/libecorr.so; else LIB=tools/${n}_lab/e-raft_amd/libecorr.so; fi
  bash tools/pmc_kernel.sh r5gm2/pmc_$n build_split16 "tools/pmc_one.py $LIB 20" "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES" > $OUT/pmc_$n.txt 2>&1 || exit $?
  echo "== $n"; cat $OUT/pmc_$n.txt
done
