#!/bin/bash
# HBM traffic (FETCH_SIZE / WRITE_SIZE, one pass each) of the SURVEY §8f kernels that bench.py's
# next_rows leg runs (split / fused convc1, convex upsampling, splat, voxel grid), summarized per
# kernel by tools/pmc_one.py --summary.  usage: tools/pmc_next.sh TAG
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; TAG=${1:-pmcnext}; OUT=gpurun_out/$TAG; mkdir -p $OUT
i=0
for grp in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp -d $OUT/pmc$i -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e > $OUT/pmc$i.log 2>&1
  rc=$?; echo "pmc pass $i ($grp) rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/pmc$i.log; exit $rc; }
done
for k in conv1x1_split_kernel lookup_conv_kernel upsample_kernel splat_band_kernel lookup_cols_reg; do
  echo "== $k"; python3 tools/pmc_one.py --summary $OUT $k
done
# the voxel grid's kernels (their names carry no "voxel": vb_count, vb_gather, ... for DSEC),
# from a probe that runs only them
for grp in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $grp -d $OUT/vox_$grp -o run --output-format csv -- python3 tools/prof_voxel.py 5 > $OUT/vox_$grp.log 2>&1
  rc=$?; echo "voxel pmc $grp rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/vox_$grp.log; exit $rc; }
done
echo "== voxel (per convert call)"; python3 tools/prof_voxel.py --summary $OUT
