#!/bin/bash
# PMC passes over one probe program, one counter group per pass (rocprofv3 does not split groups),
# then the per-dispatch average of every counter over the kernels whose name matches MATCH.
#   tools/pmc_kernel.sh TAG MATCH "probe.py args" "GROUP1" ["GROUP2" ...]
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=$1; MATCH=$2; PROBE=$3; shift 3
OUT=gpurun_out/$TAG; mkdir -p $OUT
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp -d $OUT/pmc$i -o run --output-format csv -- python3 $PROBE > $OUT/pmc$i.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "pmc pass $i ($grp) rc=$rc"; tail -3 $OUT/pmc$i.log; exit $rc; }
done
python3 - "$OUT" "$MATCH" <<'PY'
import collections, csv, glob, sys
out, match = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(list)
for f in glob.glob(out + "/pmc*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if match in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(f"{k:40s} {sum(v) / len(v):18.1f}  (dispatches {len(v)})")
PY
