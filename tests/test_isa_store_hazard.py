"""CPU guard of the store-data hazard behind round 3's lost level-0 stores (VERDICT r4 item 3,
DESIGN.md §3.1 "Stores and soffset").

Root cause (round 5, tools/soff_repro.py + tools/soff_lab.hip on the GPU): a buffer store of more
than 8 bytes reads its data VGPRs after it issues; a VALU that overwrites them in the next cycle
needs one wait state.  hipcc (LLVM's GCNHazardRecognizer) inserts it only when the store's soffset is
NOT a register -- with the wave-uniform row term in an SGPR soffset it emitted
`buffer_store_dwordx4 v[174:177], ..., s65 offen nt` followed at once by `v_cndmask_b32 v174, 0, 1`,
and that store wrote the integer 1 (1.4e-45) instead of the value: 192 elements of 20 query rows of a
B = 16 build, every element still written (the round-3 diagnosis read it as unwritten rows).  With the
term in the voffset (soffset = 0) the pad is there and every build is bitwise.  The range check
(tools/soff_lab.hip): an access happens iff voffset < num_records and voffset + soffset <
num_records, so soffset itself is safe wherever both stay in range (the split16 / conv LDS-DMA and
query loads) -- the hazard is the store-data one only.

This test compiles every kernel source for gfx950 and requires that no wide (dwordx3/x4) buffer
store takes its soffset from an SGPR; the detector itself is checked on the round-3 variant
(tools/lab_build.py soff_full), where it must find the hazard."""
import concurrent.futures
import os
import re
import shutil
import subprocess
import sys
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "e-raft_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"
SOURCES = ["abi", "build", "conv", "lookup", "motion", "rows", "splat", "upsample", "voxel"]
WIDE = re.compile(r"buffer_store_(?:dwordx3|dwordx4|b96|b128)\s+v\[(\d+):(\d+)\],\s*\S+,\s*s\[\d+:\d+\],\s*(\S+)")
VDST = re.compile(r"v_\S+\s+v(?:\[(\d+):(\d+)\]|(\d+))\b")


def _asm(src_dir, name, out_dir):
    out = os.path.join(out_dir, name + ".s")
    flags = ["-fno-slp-vectorize"] if name == "build" else []
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", *flags,
                    "-I" + os.path.join(ROOT, "include"), "--cuda-device-only", "-S",
                    os.path.join(src_dir, name + ".hip"), "-o", out], check=True, capture_output=True)
    return [l.strip() for l in open(out) if l.startswith("\t") and not l.strip().startswith((".", ";"))]


def scan(ins):
    """(wide stores with an SGPR soffset, of which immediately followed by a VALU writing their data)."""
    sgpr, hazards = [], []
    for i, l in enumerate(ins):
        m = WIDE.match(l)
        if not m or not re.fullmatch(r"s\d+", m.group(3)):
            continue
        sgpr.append(l)
        lo, hi = int(m.group(1)), int(m.group(2))
        w = VDST.match(ins[i + 1]) if i + 1 < len(ins) else None
        if w:
            a = int(w.group(1) or w.group(3))
            b = int(w.group(2) or w.group(3))
            if not (b < lo or a > hi):
                hazards.append(l + " || " + ins[i + 1])
    return sgpr, hazards


@pytest.fixture(scope="module")
def compiled():
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not installed")
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import lab_build
    d = tempfile.mkdtemp()
    try:
        bad = os.path.join(d, "e-raft_amd", "csrc")   # the tree's layout: the sources include ../../include
        shutil.copytree(CSRC, bad, ignore=shutil.ignore_patterns("build"))
        shutil.copytree(os.path.join(ROOT, "include"), os.path.join(d, "include"))
        p = os.path.join(bad, "build.hip")
        s = open(p).read()
        for _, old, new in lab_build.PATCHES["soff_full"]:
            assert old in s
            s = s.replace(old, new)
        open(p, "w").write(s)
        with concurrent.futures.ThreadPoolExecutor(8) as ex:
            jobs = {n: ex.submit(_asm, CSRC, n, d) for n in SOURCES}
            jobs["soff_full"] = ex.submit(_asm, bad, "build", bad)
            yield {n: j.result() for n, j in jobs.items()}
    finally:
        shutil.rmtree(d, ignore_errors=True)


def test_no_wide_store_with_sgpr_soffset(compiled):
    for n in SOURCES:
        sgpr, hazards = scan(compiled[n])
        assert not sgpr, f"{n}.hip: wide buffer stores with an SGPR soffset: {sgpr[:3]}"


def test_detector_finds_round3_variant(compiled):
    sgpr, hazards = scan(compiled["soff_full"])
    assert sgpr and hazards, "the soffset FULL epilogue should show the unpadded store-data hazard"
