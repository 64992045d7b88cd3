#!/usr/bin/env python3
"""Static instruction mix of one kernel in a hipcc -S listing, split at the last MFMA (K loop +
prologue vs epilogue).  usage: tools/isa_count.py build.s build_split_kernelILb1EE"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
m = re.search(r"^(_Z\S*" + re.escape(sys.argv[2]) + r"\S*):", s, re.M)
start = m.start()
end = s.find(".Lfunc_end", start)
ins = [l.strip() for l in s[start:end].splitlines() if l.startswith("\t") and not l.strip().startswith((".", ";"))]
last = max(i for i, l in enumerate(ins) if l.startswith("v_mfma"))


def mix(seq):
    c = collections.Counter()
    for l in seq:
        op = l.split()[0]
        if op.startswith("v_mfma"):
            c["mfma"] += 1
        elif op.startswith("v_"):
            c["valu"] += 1
            c["v:" + op] += 1
        elif op.startswith("ds_"):
            c["ds"] += 1
        elif op.startswith(("buffer_", "global_")):
            c["vmem"] += 1
        elif op.startswith("s_"):
            c["salu"] += 1
    return c


for name, seq in (("loop+prologue", ins[: last + 1]), ("epilogue", ins[last + 1 :])):
    c = mix(seq)
    top = sorted(((v, k) for k, v in c.items() if k.startswith("v:")), reverse=True)[:14]
    print(f"{name}: {len(seq)} instr, mfma {c['mfma']} valu {c['valu']} ds {c['ds']} vmem {c['vmem']} salu {c['salu']}")
    print("   " + ", ".join(f"{k[2:]} {v}" for v, k in top))
meta = s[end:end + 4000]
for k in ("vgpr_count", "agpr_count", "sgpr_count", "private_segment_fixed_size", "spill_count"):
    for mm in re.finditer(r"\.?" + k + r":\s*(\d+)", meta):
        print(k, mm.group(1))
        break
