#!/bin/bash
# Round-6 final, in two calls (each within gpurun's 20-minute limit):
#   PART=1: every GPU test, smoke, then the rocprof kernel trace and the PMC passes (C2 full set,
#           C3 / C5 traffic) summarized on the box (tools/pmc_summary.py) -- copy
#           gpurun_out/TAG/prof/pmc_summary.json to profiles/latest_pmc.json before PART=2, so
#           the bench lines carry the measured traffic of these sources;
#   PART=2: the headline bench + C3 / C5 lines, a 2-rank batch-sharded rehearsal on one GPU (gloo),
#           then a kernel trace of the SURVEY §8f rows.
# usage: PART=1|2 tools/gpu_final6.sh TAG
cd "$GRAFT_REPO_ROOT"; TAG=${1:-r6final}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
if [ "${PART:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E 'FAILED|ERROR|passed|failed' $OUT/pytest_gpu.log | tail -8; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -1 $OUT/smoke.log; [ $rc -ne 0 ] && exit $rc
  bash tools/profile.sh $TAG/prof
  rc=$?; [ $rc -ne 0 ] && exit $rc
  python3 tools/pmc_summary.py $OUT/prof $OUT/prof > $OUT/prof/pmc_summary.log 2>&1
  rc=$?; echo "pmc_summary rc=$rc"; exit $rc
fi
timeout -k 10 400 python -u bench.py > $OUT/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u bench.py --batch 64 --height 32 --width 32 --steps 20 --warmup 5 --no-cpu-baseline --no-next > $OUT/bench_c3.log 2>&1
rc=$?; echo "c3 rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u bench.py --mode rowshard --steps 10 --warmup 3 --no-cpu-baseline --no-next > $OUT/bench_c5.log 2>&1
rc=$?; echo "c5 rc=$rc"; [ $rc -ne 0 ] && exit $rc
# `bench.py --gpus 2` with no launcher: it starts the 2 ranks itself (both on cuda:0 over gloo here)
BENCH_SINGLE_DEVICE=1 timeout -k 10 200 python bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --no-next > $OUT/bench_2rank.log 2>&1
rc=$?; echo "2-rank rc=$rc"; [ $rc -ne 0 ] && exit $rc
python3 - $OUT <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/bench*.log")):
    ln = [l for l in open(f) if l.startswith("{")]
    if not ln:
        print(f, "no JSON"); continue
    d = json.loads(ln[-1]); k = d["kernels"]
    print(f.split("/")[-1], d["value"], "pairs/s", d["ms_per_step"], "ms/step frac", d["corrblock_frac"],
          "gemm", k["build"]["ms_per_launch"], "pack", k.get("pack", {}).get("ms_per_launch"), "lookup",
          k["lookup"]["ms_per_launch"], "traffic", d["roofline"].get("traffic"))
PY
# the SURVEY §8f rows (split / fused convc1, upsampling, splat, voxel) under the kernel trace, no e2e
mkdir -p $OUT/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof/kt_next -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $OUT/prof/kt_next.log 2>&1
rc=$?; echo "kt next rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u tools/prof_splat_overflow.py > $OUT/splat_overflow.json 2> $OUT/splat_overflow.err
rc=$?; echo "splat overflow rc=$rc"; cat $OUT/splat_overflow.json; [ $rc -ne 0 ] && exit $rc
bash tools/pmc_next.sh $TAG/pmcnext > $OUT/pmc_next.txt 2>&1
rc=$?; echo "pmc next rc=$rc"; tail -25 $OUT/pmc_next.txt
# keep what comes back under gpurun's 64 MiB: the summaries stay, the raw per-dispatch CSVs go
find $OUT -name '*counter_collection.csv' -delete; find $OUT -name '*kernel_trace.csv' -delete
exit $rc
