#!/bin/bash
# SQ counters of build_qs_kernel (lab builds given as args) beside build_split16_kernel, two PMC
# passes per build.  usage: tools/gpu_qssq.sh qs qsnomf ...
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/qssq; mkdir -p $OUT
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA"
B="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_MISC"
export AB_NOCHECK=1 AB_ROUNDS=2
for lab in "$@"; do
  i=0
  for grp in "$A" "$B"; do
    i=$((i+1))
    AB_ALT_LIB=x=tools/${lab}_lab/e-raft_amd/libecorr.so timeout -k 10 120 rocprofv3 --pmc $grp -d $OUT/$lab$i -o run --output-format csv -- python3 tools/ab_build.py > $OUT/$lab$i.log 2>&1
    rc=$?; echo "$lab pass $i rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $OUT/$lab$i.log; exit $rc; fi
  done
done
python3 - "$@" <<'PY'
import csv, glob, collections, sys
for lab in sys.argv[1:]:
    res = collections.defaultdict(dict)
    for i in (1, 2):
        for f in glob.glob(f"gpurun_out/qssq/{lab}{i}/**/*counter_collection.csv", recursive=True):
            acc = collections.defaultdict(lambda: collections.defaultdict(float))
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"]
                if "build_split16" in k or "build_qs" in k:
                    acc[(k[:40], r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
            per = collections.defaultdict(lambda: collections.defaultdict(list))
            for (k, d), cs in acc.items():
                for c, v in cs.items():
                    per[k][c].append(v)
            for k, cs in per.items():
                for c, v in cs.items():
                    res[k][c] = sorted(v)[len(v) // 2]
    for k, cs in res.items():
        print(lab, k)
        for c in sorted(cs):
            print(f"   {c:24s} {cs[c]:.4g}")
PY
