#!/bin/bash
# Round 6, second call: the splat batch test, the GEMM L2-read arm, the C5 tile
# group size (item 3: time + FETCH), next-row PMC incl. the voxel kernels (item 6), voxel kernel trace.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/r6b; mkdir -p $OUT
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_splat_gpu.py > $OUT/pytest_splat.txt 2>&1 || { echo "splat tests failed"; tail -30 $OUT/pytest_splat.txt; exit 1; }
tail -2 $OUT/pytest_splat.txt
AB_NOCHECK=1 AB_ROUNDS=12 AB_ALT_LIB=l2rd=tools/l2rd_lab/e-raft_amd/libecorr.so timeout -k 10 300 python -u tools/ab_build.py > $OUT/ab_l2rd.txt 2>&1 || { echo "l2rd failed"; tail $OUT/ab_l2rd.txt; exit 1; }
grep median $OUT/ab_l2rd.txt
AB_SHAPES='[[4,256,92,160],[16,256,60,80]]' AB_ALT_LIB=gm8=tools/gm8_lab/e-raft_amd/libecorr.so,gm12=tools/gm12_lab/e-raft_amd/libecorr.so,gm16=tools/gm16_lab/e-raft_amd/libecorr.so timeout -k 10 400 python -u tools/ab_build.py > $OUT/ab_gm_c5.txt 2>&1 || { echo "gm c5 failed"; tail $OUT/ab_gm_c5.txt; exit 1; }
grep -E "DIFFERENT|median" $OUT/ab_gm_c5.txt
for v in tree gm8 gm12 gm16; do
  lib=e-raft_amd/libecorr.so; [ $v != tree ] && lib=tools/${v}_lab/e-raft_amd/libecorr.so
  PMC_SHAPE=4,256,92,160 timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $OUT/c5f_$v -o run --output-format csv -- python3 tools/pmc_one.py $lib 5 > $OUT/c5f_$v.log 2>&1 || { echo "c5 pmc $v failed"; tail -5 $OUT/c5f_$v.log; exit 1; }
  echo "C5 FETCH $v:"; python3 tools/pmc_one.py --summary $OUT/c5f_$v build_split16_kernel
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/voxkt -o run --output-format csv -- python3 tools/prof_voxel.py 10 > $OUT/voxkt.log 2>&1 || { echo "voxel kt failed"; tail -5 $OUT/voxkt.log; exit 1; }
bash tools/pmc_next.sh r6b/pmcnext > $OUT/pmc_next.txt 2>&1 || { echo "pmc_next failed"; tail -20 $OUT/pmc_next.txt; exit 1; }
tail -30 $OUT/pmc_next.txt
echo DONE
