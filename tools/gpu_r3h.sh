#!/bin/bash
# split16 level-0 stores without the LDS transpose: bitwise A/B, stamps, PMC write bytes.
cd "$GRAFT_REPO_ROOT"; TAG=${1:-r3h}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
AB_ROUNDS=12 AB_ALT_LIB=l0direct=tools/l0direct_lab/e-raft_amd/libecorr.so timeout -k 10 300 python -u tools/ab_build.py > $OUT/ab_build.log 2>&1
rc=$?; echo "ab_build rc=$rc"; grep -v amdgpu.ids $OUT/ab_build.log | grep -v "bitwise.*same" | tail -4; [ $rc -ne 0 ] && exit $rc
for lib in st16 st16_l0direct; do
  timeout -k 10 200 python -u tools/stamps16.py tools/${lib}_lab/e-raft_amd/libecorr.so > $OUT/stamps_$lib.log 2>&1
  rc=$?; echo "stamps $lib rc=$rc"; grep -v amdgpu.ids $OUT/stamps_$lib.log | tail -7; [ $rc -ne 0 ] && exit $rc
done
for lib in e-raft_amd/libecorr.so tools/l0direct_lab/e-raft_amd/libecorr.so; do
  nm=$(echo $lib | tr '/' '_')
  for grp in WRITE_SIZE FETCH_SIZE; do
    timeout -s KILL 90 rocprofv3 --pmc $grp -d $OUT/pmc_${nm}_$grp -o run --output-format csv -- python3 tools/pmc_one.py $lib 5 > $OUT/pmc_${nm}_$grp.log 2>&1
    rc=$?; echo "pmc $nm $grp rc=$rc"; [ $rc -ne 0 ] && exit $rc
    python3 tools/pmc_one.py --summary $OUT/pmc_${nm}_$grp build_split16
  done
done
