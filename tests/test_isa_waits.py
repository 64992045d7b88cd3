"""CPU guard of the build K loops' hand-counted waits.

build_split16_kernel<true> (the D = 256 split build) and build_f32_kernel<true>
(e-raft_amd/csrc/build.hip) stage the shared target panel into LDS by LDS-DMA
(`buffer_load_dwordx4 ... lds`) through NBUF buffers and wait for chunk (pair) k with a STATIC
`s_waitcnt vmcnt(N)` before barrier k: N counts the VMEM instructions the source issues after
chunk k's DMA pieces.  That count is right only while hipcc
keeps the source's issue order (sched_barrier fences hold it today; DESIGN.md §3.1 records the
hoisted q(0) load that once made barrier 0 release a wave before t(0) landed).

This test compiles build.hip for gfx950 (`hipcc --cuda-device-only -S`), replays each kernel's
instruction stream up to its K loop's closing barrier and checks, in the order the assembler
actually emits:
  * RAW: at barrier k (k < NK) every DMA piece of chunk k has retired under the waits issued so far
    (vmcnt(N) retires all but the N youngest VMEM instructions; loads, stores and LDS-DMA count
    together, in issue order);
  * WAR: chunk m >= NBUF (which overwrites chunk m - NBUF's buffer) is issued only after barrier
    m - NBUF + SPAN (chunk j is read between barriers j and j + SPAN: the split16 loop reads a
    pair's last target group after the next pair's barrier), and every barrier is preceded by an
    lgkmcnt(0) after the wave's last LDS read;
  * split16 kernel: the LDS reads between barrier k and k + 1 address buffers k % NBUF (or
    (k - 1) % NBUF, SPAN 2) only (their offset field, one base register).
A deliberately swapped issue order (q(0) hoisted over t(0)) must be flagged.
"""
import os
import re
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "e-raft_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"

# kernel -> (LDS buffers, DMA pieces per chunk, K chunks, bytes per buffer, query loads per chunk,
# barriers a chunk's reads span, barriers up to the loop's closing one)
KERNELS = {
    "build_split16_kernelILb1EE": dict(nbuf=4, copies=4, nk=8, chunk=16384, qloads=8, span=2, barriers=9),
    "build_f32_kernelILb1EE": dict(nbuf=3, copies=2, nk=16, chunk=8192, qloads=16, span=1, barriers=18),
}
SPLIT = "build_split16_kernelILb1EE"


@pytest.fixture(scope="module")
def asm():
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not installed")
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "build.s")
        subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-slp-vectorize",
                        "-I" + os.path.join(ROOT, "include"), "--cuda-device-only", "-S",
                        os.path.join(CSRC, "build.hip"), "-o", out],
                       check=True, capture_output=True)
        return open(out).read()


def kernel_loop(s, name):
    """The kernel's instructions up to and including the first s_barrier after its last MFMA."""
    m = re.search(r"^(_Z\S*" + re.escape(name) + r"\S*):", s, re.M)
    assert m, f"{name} not in the listing"
    end = s.find(".Lfunc_end", m.start())
    ins = [ln.strip() for ln in s[m.start():end].splitlines()
           if ln.startswith("\t") and not ln.strip().startswith((".", ";"))]
    last = max(i for i, ln in enumerate(ins) if ln.startswith("v_mfma"))
    close = next(i for i in range(last, len(ins)) if ins[i] == "s_barrier")
    return ins[:close + 1]


def is_vmem(ln):
    return ln.startswith(("buffer_", "global_", "scratch_", "flat_"))


def is_dma(ln):
    return ln.startswith("buffer_load") and ln.split()[-1] == "lds"


def check_loop(ins, nbuf, copies, nk, chunk, check_offsets, span=1):
    """Violations of the RAW / WAR rules above (empty list = the waits hold)."""
    errs = []
    issued = done = 0        # VMEM instructions issued / retired (a prefix, in issue order)
    dma = []                 # (issue index, barriers passed before it) per DMA piece
    nbar = 0
    lds_pending = False      # an LDS read issued after the last lgkmcnt(0)
    reads = []               # (barrier region, ds_read line)
    for ln in ins:
        op = ln.split()[0]
        if is_vmem(ln):
            if op.startswith("flat_"):
                errs.append(f"flat VMEM op (retires out of order): {ln}")
            if is_dma(ln):
                dma.append((issued, nbar))
            issued += 1
        elif op == "s_waitcnt":
            m = re.search(r"vmcnt\((\d+)\)", ln)
            if m:
                done = max(done, issued - int(m.group(1)))
            if re.search(r"lgkmcnt\(0\)", ln):
                lds_pending = False
        elif op.startswith("ds_read"):
            lds_pending = True
            reads.append((nbar - 1, ln))
        elif op == "s_barrier":
            if lds_pending and nbar > 0:
                errs.append(f"barrier {nbar}: an LDS read of the previous chunk may still be in flight")
            if nbar < nk:
                last = copies * (nbar + 1) - 1
                if last >= len(dma):
                    errs.append(f"barrier {nbar}: chunk {nbar}'s DMA not issued yet")
                elif done <= dma[last][0]:
                    errs.append(f"barrier {nbar}: chunk {nbar}'s DMA may be in flight "
                                f"({issued - done} VMEM ops outstanding, piece #{dma[last][0]} of {issued})")
            nbar += 1
    if len(dma) % copies:
        errs.append(f"{len(dma)} DMA pieces, not a multiple of {copies}")
    for p, (_, before) in enumerate(dma):
        m = p // copies
        if m >= nbuf and before < m - nbuf + span + 1:
            errs.append(f"chunk {m}'s DMA issued after barrier {before - 1}, before barrier {m - nbuf + span} "
                        f"retired the reads of chunk {m - nbuf}")
    if check_offsets:
        bases = {re.match(r"ds_read\S*\s+\S+,\s*(\S+)", r).group(1) for _, r in reads}
        if len(bases) != 1:
            errs.append(f"LDS reads on several base registers {sorted(bases)}: offsets not checkable")
        else:
            for region, r in reads:
                m = re.search(r"offset:(\d+)", r)
                buf = (int(m.group(1)) if m else 0) // chunk
                if region < 0 or buf not in {(region - d) % nbuf for d in range(span)}:
                    errs.append(f"read in barrier region {region} addresses buffer {buf}: {r}")
    return errs


@pytest.mark.parametrize("name", sorted(KERNELS))
def test_static_waits_match_issue_order(asm, name):
    k = KERNELS[name]
    ins = kernel_loop(asm, name)
    assert sum(1 for ln in ins if ln == "s_barrier") == k["barriers"]
    assert sum(1 for ln in ins if is_dma(ln)) >= k["copies"] * k["nk"]
    # the query fragment loads (buffer loads to VGPRs; the exponent loads are global_load_dword)
    assert sum(1 for ln in ins if ln.startswith("buffer_load") and not is_dma(ln)) == k["qloads"] * k["nk"]
    errs = check_loop(ins, k["nbuf"], k["copies"], k["nk"], k["chunk"], name == SPLIT, k["span"])
    assert not errs, "\n".join(errs)


def test_checker_flags_a_hoisted_query_load(asm):
    """q(0) moved in front of t(0) -- the race DESIGN.md §3.1 records -- is caught at barrier 0."""
    k = KERNELS[SPLIT]
    ins = kernel_loop(asm, SPLIT)
    first = next(i for i, ln in enumerate(ins) if is_dma(ln))
    q = [i for i, ln in enumerate(ins) if i > first and is_vmem(ln) and not is_dma(ln)][:k["qloads"]]
    swapped = ins[:first] + [ins[i] for i in q] + [ln for i, ln in enumerate(ins[first:], first) if i not in q]
    errs = check_loop(swapped, k["nbuf"], k["copies"], k["nk"], k["chunk"], True, k["span"])
    assert any(e.startswith("barrier 0:") for e in errs), errs
    # and a DMA refill issued one barrier early (WAR on a buffer still being read)
    dmas = [i for i, ln in enumerate(ins) if is_dma(ln)]
    p = dmas[k["copies"] * k["nbuf"]]           # first piece of chunk NBUF
    bar = max(i for i, ln in enumerate(ins[:p]) if ln == "s_barrier")
    early = ins[:bar] + [ins[p]] + [ln for i, ln in enumerate(ins[bar:], bar) if i != p]
    errs = check_loop(early, k["nbuf"], k["copies"], k["nk"], k["chunk"], True, k["span"])
    assert any("before barrier" in e for e in errs), errs


# ---- conv.hip: conv1x1_split_kernel<2> (the split convc1, query columns 2 chunks ahead) stages its weight chunks by LDS-DMA
# through 3 buffers, two chunks ahead, and waits for chunk c + 1 at the end of step c with a static
# vmcnt(12) (step c's 8 query-column loads + 4 DMA pieces are the only newer VMEM ops; vmcnt(4) in
# the remainder steps, whose dead query-column loads the compiler drops -- this replay caught that
# race when the remainder still waited vmcnt(12)).  Its K loop is
# rolled (3 steps per trip) with a 0-2 step remainder, so the straight-line stream replayed here is
# prologue + two trips of the loop body + both remainder steps: barriers 0 (prologue) .. 8.
# The presplit instantiation (PRE = true, ABI 16) loads 2 16-byte pieces per chunk: vmcnt(6) at the
# step barriers (2 loads + 4 DMA pieces newer than chunk c + 1's).
CONVS = {"conv1x1_split_kernelILi2ELb0EE": 12, "conv1x1_split_kernelILi2ELb1EE": 6}


@pytest.fixture(scope="module")
def conv_asm():
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not installed")
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "conv.s")
        subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                        "-I" + os.path.join(ROOT, "include"), "--cuda-device-only", "-S",
                        os.path.join(CSRC, "conv.hip"), "-o", out],
                       check=True, capture_output=True)
        return open(out).read()


def conv_stream(s, name):
    """Straight-line replay of the conv kernel: prologue, loop body twice, the remainder steps."""
    m = re.search(r"^(_Z\S*" + re.escape(name) + r"\S*):", s, re.M)
    assert m, f"{name} not in the listing"
    end = s.find(".Lfunc_end", m.start())
    lines = s[m.start():end].splitlines()
    # the K loop: the loop header whose body holds the MFMAs
    heads = [i for i, ln in enumerate(lines) if "Inner Loop Header" in ln]
    head = next(h for h in heads if any("v_mfma" in ln for ln in lines[h:h + 200]))
    label = lines[head].split(":")[0]
    back = next(i for i in range(head, len(lines)) if re.search(r"s_cbranch\S*\s+" + re.escape(label) + r"$",
                                                                 lines[i].strip()))
    last_bar = max(i for i, ln in enumerate(lines) if ln.strip() == "s_barrier")

    def ins(a, b):
        return [ln.strip() for ln in lines[a:b]
                if ln.startswith("\t") and not ln.strip().startswith((".", ";"))]
    return ins(0, head) + ins(head, back + 1) * 2 + ins(back + 1, last_bar + 1)


@pytest.mark.parametrize("name", sorted(CONVS))
def test_conv_static_waits_match_issue_order(conv_asm, name):
    ins = conv_stream(conv_asm, name)
    assert sum(1 for ln in ins if ln == "s_barrier") == 9
    assert sum(1 for ln in ins if is_dma(ln)) == 4 * 10   # chunks 0 .. 9, 4 pieces per wave each
    assert any(f"vmcnt({CONVS[name]})" in ln for ln in ins)
    errs = check_loop(ins, nbuf=3, copies=4, nk=9, chunk=16384, check_offsets=False, span=1)
    assert not errs, "\n".join(errs)


@pytest.mark.parametrize("name", sorted(CONVS))
def test_conv_checker_flags_a_short_wait(conv_asm, name):
    """vmcnt(N) -> vmcnt(N + 4) at the step barriers would let chunk c + 1's pieces be in flight."""
    n = CONVS[name]
    ins = [ln.replace(f"vmcnt({n})", f"vmcnt({n + 4})") for ln in conv_stream(conv_asm, name)]
    errs = check_loop(ins, nbuf=3, copies=4, nk=9, chunk=16384, check_offsets=False, span=1)
    assert any("DMA may be in flight" in e for e in errs), errs
