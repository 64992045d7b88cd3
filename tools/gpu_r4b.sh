#!/bin/bash
# Round-4 diagnosis: build / lookup per-block stamps, then PMC passes (TLB, TA/TCP stalls, SQ waits,
# TCC stalls) on the lookup probe and the build probe.
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r4b; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 120 python -u tools/stamps16.py tools/st16_lab/e-raft_amd/libecorr.so > $OUT/stamps_st16.log 2>&1
rc=$?; echo "stamps rc=$rc"; tail -7 $OUT/stamps_st16.log; [ $rc -ne 0 ] && exit $rc
for f in smooth iid; do
  timeout -k 10 120 python -u tools/lkstamps.py tools/lkstamps_lab/e-raft_amd/libecorr.so $f > $OUT/lkstamps_$f.log 2>&1
  rc=$?; echo "lkstamps $f rc=$rc"; tail -12 $OUT/lkstamps_$f.log; [ $rc -ne 0 ] && exit $rc
done
G1="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_PENDING_STALL_CYCLES_sum TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE"
G2="TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum"
G3="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_LEVEL_VMEM"
G4="TCC_EA0_WRREQ_STALL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum TCC_BUSY_avr"
bash tools/pmc_kernel.sh r4b/pmc_lookup lookup_cols "tools/prof_lookup.py" "$G1" "$G2" "$G3" "$G4" > $OUT/pmc_lookup.txt 2>&1
rc=$?; echo "pmc lookup rc=$rc"; cat $OUT/pmc_lookup.txt; [ $rc -ne 0 ] && exit $rc
bash tools/pmc_kernel.sh r4b/pmc_build build_split16 "tools/run_build.py tree 10" "$G1" "$G2" "$G3" "$G4" > $OUT/pmc_build.txt 2>&1
rc=$?; echo "pmc build rc=$rc"; cat $OUT/pmc_build.txt; exit $rc
