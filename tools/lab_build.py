#!/usr/bin/env python3
"""Lab builds of libecorr.so for A/B and ablation (dev tool; the product has no runtime knobs).

Copies e-raft_amd/csrc + include to tools/<name>_lab/, applies the named source patches (exact
string replacements, each must match) and builds tools/<name>_lab/e-raft_amd/libecorr.so, which
tools/ab_build.py loads as AB_ALT_LIB.  Ablation variants produce invalid pyramids (AB_NOCHECK=1).
  python tools/lab_build.py noepi nomfma ...
"""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EPI = "    // ---------------- epilogue (per wave, from registers) ----------------\n"

# name -> list of (file, old, new)
PATCHES = {
    # epilogue replaced by one store per lane of the accumulator sum
    "noepi": [("build.hip", EPI, EPI + """    {
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) s += acc[i][j][r];
        P.lvl[0][(int64_t)blockIdx.x * 256 + tid] = s;
        return;
    }
""")],
}
# epilogue pieces: level 0 only (scaling + LDS line transposes + stores); no level-2/3 pixel stores
PATCHES["l0only"] = [("build.hip", "    const int L = P.fused_levels;\n    const int64_t rows0", "    const int L = 1;\n    const int64_t rows0")]
PATCHES["prio"] = [("build.hip", "    // ---------------- epilogue (per wave, from registers) ----------------\n",
                     "    // ---------------- epilogue (per wave, from registers) ----------------\n    __builtin_amdgcn_s_setprio(2);\n")]
PATCHES["prio3"] = [("build.hip", "    // ---------------- epilogue (per wave, from registers) ----------------\n",
                     "    // ---------------- epilogue (per wave, from registers) ----------------\n    __builtin_amdgcn_s_setprio(3);\n")]
# the K loop at issue priority 1, the epilogue back at 0: a block's MFMA stream ahead of the
# co-resident block's epilogue VALU (which is older, so wins at equal priority)
PATCHES["loopprio"] = [("build.hip", "    TFrags fa, fb;\n", "    __builtin_amdgcn_s_setprio(1);\n    TFrags fa, fb;\n"),
                       ("build.hip", EPI, EPI + "    __builtin_amdgcn_s_setprio(0);\n")]
PATCHES["loopprio3"] = [("build.hip", "    TFrags fa, fb;\n", "    __builtin_amdgcn_s_setprio(3);\n    TFrags fa, fb;\n"),
                        ("build.hip", EPI, EPI + "    __builtin_amdgcn_s_setprio(0);\n")]
PATCHES["lk_noblend"] = [("lookup.hip", "                const float v = blend(c[0], c[1], c[SW], c[SW + 1], wx[ai], wy[bb]);",
                          "                const float v = c[0];")]
# tile order: m-tiles per group of the grouped order (tree: 8)
# split16 tile-group bound (balanced groups since round 5; the round-4/5 records of gm2/4/16 were
# taken with full groups + a remainder, gm9/10/12 are the same either way at DSEC's 19 query tiles)
for _gm in (2, 3, 4, 6, 8, 9, 12, 16):
    PATCHES[f"gm{_gm}"] = [("build.hip", "constexpr int kGM16 = 10;", f"constexpr int kGM16 = {_gm};")]
# timing only: each v_mfma_f32_32x32x16_f16 replaced by two v_mfma_f32_16x16x32_f16 on the same
# fragments (the same MAC count, garbage sums): does the 16x16 shape hold a higher clock here?
def _m16(x, y):
    return ("build.hip", f"acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16({x}, {y}, acc[i][j], 0, 0, 0);",
            "{ floatx4 c0 = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]}, "
            "c1 = {acc[i][j][4], acc[i][j][5], acc[i][j][6], acc[i][j][7]}; "
            f"c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16({x}, {y}, c0, 0, 0, 0); "
            f"c1 = __builtin_amdgcn_mfma_f32_16x16x32_f16({x}, {y}, c1, 0, 0, 0); "
            "acc[i][j][0] = c0[0]; acc[i][j][1] = c0[1]; acc[i][j][2] = c0[2]; acc[i][j][3] = c0[3]; "
            "acc[i][j][4] = c1[0]; acc[i][j][5] = c1[1]; acc[i][j][6] = c1[2]; acc[i][j][7] = c1[3]; }")
PATCHES["mfma16"] = [_m16("f.th[j]", "q.ql[i]"), _m16("f.tl[j]", "q.qh[i]"), _m16("f.th[j]", "q.qh[i]")]
PATCHES["epi_nolds"] = [("build.hip", "        for (int s = 0; s < 4; ++s) pc[s] = *reinterpret_cast<const floatx4*>(xp + ro + s * XS);",
                         "        for (int s = 0; s < 4; ++s) pc[s] = floatx4{(float)(ro + s), (float)ql, (float)lo, 1.0f};"),
                        ("build.hip", """                    *reinterpret_cast<floatx4*>(xp + wo + 32 * g4 + 16 * arow) =
                        floatx4{v[jl][g4][0], v[jl][g4][1], v[jl][g4][2], v[jl][g4][3]};""",
                         """                    asm volatile("" :: "v"(floatx4{v[jl][g4][0], v[jl][g4][1], v[jl][g4][2], v[jl][g4][3]}));""")]
# split16 kernel: the 32x32 build_split_kernel launched instead (same late exponent loads), for A/B
PATCHES["s32"] = [("build.hip", "        const bool s16 = (P.D + 15) / 16 == 2 * NCP;", "        const bool s16 = false;")]
# split16 per-block timing, lane 0 of wave 0 -> g_st16[block] = {start, loop start, loop end, block end
# (s_memrealtime), loop cycles, epilogue cycles (s_memtime), HW_ID, XCC_ID}
# (s_memtime cycles, s_memrealtime 10 ns ticks); tools/stamps16.py
ST16_DECL = """
__device__ unsigned long long g_st16[65536][8];
"""
ST16_EXPORT = """
extern "C" __attribute__((visibility("default"))) int ecorr_lab_stamps16(void* dst, int n) {
    return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(ecorr::g_st16), (size_t)n * 64, 0, hipMemcpyDeviceToHost);
}
"""
PATCHES["st16"] = [
    ("build.hip", "constexpr int SQ = 256; ", ST16_DECL + "constexpr int SQ = 256; "),
    ("build.hip", """    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    int b, qt, nt;
    decode_tile<kGM16, true>(P, xcd_remap(blockIdx.x, gridDim.x), P.n_qt, b, qt, nt);
    const NTile tc = ntile_of(P, nt);
    const int q0 = qt * SQ;
    const int H = P.H, W = P.W;
    const int64_t Q = (int64_t)H * W;

    // per-pixel exponents: loaded behind the K loop's last static wait (only the epilogue reads them)""",
     """    const unsigned long long r_start = __builtin_amdgcn_s_memrealtime();
    unsigned long long c_mid = 0;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    int b, qt, nt;
    decode_tile<kGM16, true>(P, xcd_remap(blockIdx.x, gridDim.x), P.n_qt, b, qt, nt);
    const NTile tc = ntile_of(P, nt);
    const int q0 = qt * SQ;
    const int H = P.H, W = P.W;
    const int64_t Q = (int64_t)H * W;

    // per-pixel exponents: loaded behind the K loop's last static wait (only the epilogue reads them)"""),
    ("build.hip", """    wait_vm_n<true>(s16_vm_after(0));   // t(0) landed
    __builtin_amdgcn_s_barrier();
    PHASE;""", """    wait_vm_n<true>(s16_vm_after(0));   // t(0) landed
    __builtin_amdgcn_s_barrier();
    PHASE;
    const unsigned long long c_loop0 = __builtin_amdgcn_s_memtime(), r_loop0 = __builtin_amdgcn_s_memrealtime();
    PHASE;"""),
    ("build.hip", """            if (tg == 6 && cp + 1 < NCP) {   // mid(cp): publish t(cp + 1), retire the reads of t(cp - 1)
                wait_vm_n<true>(s16_vm_after(cp + 1));
                __builtin_amdgcn_s_barrier();
                PHASE;""", """            if (tg == 6 && cp + 1 < NCP) {   // mid(cp): publish t(cp + 1), retire the reads of t(cp - 1)
                const unsigned long long cm = __builtin_amdgcn_s_memtime();
                wait_vm_n<true>(s16_vm_after(cp + 1));
                __builtin_amdgcn_s_barrier();
                c_mid += __builtin_amdgcn_s_memtime() - cm;
                PHASE;"""),
    ("build.hip", """    __syncthreads();      // ... in every wave: the panel buffers are the epilogue's scratch""",
     """    __syncthreads();      // ... in every wave: the panel buffers are the epilogue's scratch
    const unsigned long long c_loop1 = __builtin_amdgcn_s_memtime(), r_loop1 = __builtin_amdgcn_s_memrealtime();"""),
    ("build.hip", """        split16_epilogue<MUL, false>(P, acc, smem + wave * (2 * 64 * S16LS), wave * 64, exq, ext, fst, tc, b, q0, lane);
}""", """        split16_epilogue<MUL, false>(P, acc, smem + wave * (2 * 64 * S16LS), wave * 64, exq, ext, fst, tc, b, q0, lane);
    __syncthreads();
    if (tid == 0 && blockIdx.x < 65536) {
        unsigned long long* g = g_st16[blockIdx.x];
        g[0] = r_start;
        g[1] = r_loop0;
        g[2] = r_loop1;
        g[3] = __builtin_amdgcn_s_memrealtime();
        g[4] = c_loop1 - c_loop0;
        g[5] = __builtin_amdgcn_s_memtime() - c_loop1;
        (void)c_mid;
        g[6] = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);
        g[7] = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20);
    }
}"""),
    ("build.hip", "}  // namespace ecorr\n", "}  // namespace ecorr\n" + ST16_EXPORT),
]
# split16 wave priority: the K loop at s_setprio 1 over the partner block's epilogue (the older wave
# otherwise wins the SIMD's issue arbitration) / the epilogue at 1
PATCHES["prio_loop"] = [("build.hip", """    read_a(0, 0, af[0]);
    PHASE;
#pragma unroll
    for (int cp = 0; cp < NCP; ++cp) {""", """    read_a(0, 0, af[0]);
    __builtin_amdgcn_s_setprio(1);
    PHASE;
#pragma unroll
    for (int cp = 0; cp < NCP; ++cp) {"""),
    ("build.hip", """    wait_vm<0, true>();   // the exponents have landed and this wave's reads are done ...""",
     """    __builtin_amdgcn_s_setprio(0);
    wait_vm<0, true>();   // the exponents have landed and this wave's reads are done ...""")]
PATCHES["prio_epi"] = [("build.hip", """    wait_vm<0, true>();   // the exponents have landed and this wave's reads are done ...""",
     """    __builtin_amdgcn_s_setprio(1);
    wait_vm<0, true>();   // the exponents have landed and this wave's reads are done ...""")]
PATCHES["onecu16"] = [("build.hip", """__global__ __launch_bounds__(256, 2) void build_split16_kernel(BuildParams P) {
    // ALL LDS in this one array (cdna_hip_programming.md trap 4(a), see build_split_kernel)
    __shared__ __attribute__((aligned(16))) char smem[SLDS + (SQ + 256) * 4];""", """__global__ __launch_bounds__(256, 1) void build_split16_kernel(BuildParams P) {
    // ALL LDS in this one array (cdna_hip_programming.md trap 4(a), see build_split_kernel)
    __shared__ __attribute__((aligned(16))) char smem[SLDS + (SQ + 256) * 4 + 16384];""")]
# (round 3: split16 level-0 lines stored straight from their lanes, no LDS transpose -- the source
# option is gone: 4.8 ms and 5.4 GB written, profiles/r03_lab/r3h_*)
# the query-stationary persistent build (build_qs_kernel) in place of build_split16_kernel
PATCHES["qs"] = [("build.hip", "constexpr bool kBuildQS = false;", "constexpr bool kBuildQS = true;")]
PATCHES["qsnomf"] = PATCHES["qs"] + [
    ("build.hip", '''        asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+v"(c) : "v"(a), "a"(b));''',
     '''        asm volatile("" : "+v"(c) : "v"(a), "a"(b));'''),
    ("build.hip", '''        asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, 0" : "=&v"(c) : "v"(a), "a"(b));''',
     '''        asm volatile("v_mov_b32 %0, 0" : "=v"(c[0]) : "v"(a), "a"(b));'''),
]
# QS epilogue stores with the default cache policy (write-back L2) instead of nt | sc1
PATCHES["qsst0"] = PATCHES["qs"] + [("build.hip", "constexpr int QS_ST = 18;", "constexpr int QS_ST = 0;")]
PATCHES["qsnomfst0"] = PATCHES["qsnomf"] + PATCHES["qsst0"][1:]
# QS timing probes: no wait for the panel past the first unit (races: timing only); the previous
# half's whole epilogue before this half's MFMAs (its stores get the whole half to complete)
PATCHES["qsnowait"] = PATCHES["qs"] + [("build.hip", "    using WN = std::integral_constant<int, QS_NST>;",
                                        "    using WN = std::integral_constant<int, 63>;")]
# split16 level-0/1 stores as nt | sc1 instead of nt
PATCHES["st18"] = [("build.hip", "constexpr int ST_L01 = 2; ", "constexpr int ST_L01 = 18;")]
# QS scheduling freedom: no scheduling barrier between the interleaved steps / one per two steps
PATCHES["qsnosb"] = PATCHES["qs"] + [("build.hip", "            if constexpr (EPI) epi_step(AE, kc, fast_c);\n            __builtin_amdgcn_sched_barrier(0);",
                                      "            if constexpr (EPI) epi_step(AE, kc, fast_c);")]
PATCHES["qssb2"] = PATCHES["qs"] + [("build.hip", "            if constexpr (EPI) epi_step(AE, kc, fast_c);\n            __builtin_amdgcn_sched_barrier(0);",
                                     "            if constexpr (EPI) epi_step(AE, kc, fast_c);\n            if constexpr ((decltype(kc)::value & 1) == 1) __builtin_amdgcn_sched_barrier(0);")]
# QS timing probe: every pyramid store out of range (same instructions, no store traffic)
PATCHES["qsnost"] = PATCHES["qs"] + [
    ("build.hip", "P.lvl[0] + (int64_t)C.rows0 * P.lsz[0], 0, C.nq * l0stride, 0x00020000);",
     "P.lvl[0] + (int64_t)C.rows0 * P.lsz[0], 0, 0, 0x00020000);"),
    ("build.hip", "return __builtin_amdgcn_make_buffer_rsrc(P.lvl[L] + (int64_t)g0 * G, 0, gspan * G * 4, 0x00020000);",
     "return __builtin_amdgcn_make_buffer_rsrc(P.lvl[L] + (int64_t)g0 * G, 0, 0 * gspan, 0x00020000);"),
]
# lookup output store cache policy (tree: nt = 2)
# the tree as it is (the baseline of an A/B against an edited tree)
PATCHES["base"] = []
# lookup windows staged one column per work item (b32 loads) instead of 8-byte column pairs
PATCHES["nopair"] = [("lookup.hip", "        bool pair = true;", "        bool pair = false;")]
# timing only: no window loads for one level (what does each level's staging cost?)
for _lv in range(4):
    PATCHES[f"lk_skip{_lv}"] = [("lookup_stage.h", "            const bool need = (unsigned)(ry - rlo) < (unsigned)(rhi - rlo);",
                                 f"            const bool need = lv != {_lv} && (unsigned)(ry - rlo) < (unsigned)(rhi - rlo);")]
PATCHES["lk_prio2"] = [("lookup.hip", "    if (md == 0) {\n        int yo[K];", "    __builtin_amdgcn_s_setprio(2);\n    if (md == 0) {\n        int yo[K];")]
PATCHES["nopairm"] = [("motion.hip", "    bool pair = true;", "    bool pair = false;")]
# fused lookup + convc1 ablations (timing only, AB_NOCHECK=1): no GEMM phase / no lookup phase
PATCHES["mo_nogemm"] = [("motion.hip", "    for (int oc = 0; oc < O; oc += OB) {", "    for (int oc = 0; oc < 0; oc += OB) {")]
PATCHES["mo_nolookup"] = [("motion.hip", "    for (int lv = 0; lv < P.levels; ++lv) {\n        stage_level",
                           "    for (int lv = 0; lv < 0; ++lv) {\n        stage_level")]
# every lane reads the same 32 bytes of W (weight traffic ~0, same instructions)
PATCHES["mo_samew"] = [("motion.hip", "        const int r0 = (ob + col) * C, r1 = (ob + 32 + col) * C;",
                        "        const int r0 = 0 * (ob + col) * C, r1 = 0 * (ob + 32 + col) * C;")]
PATCHES["mo_nolookup_samew"] = PATCHES["mo_nolookup"] + PATCHES["mo_samew"]
# ... and without the MFMAs (fragments kept alive): is the matrix pipe what bounds the GEMM phase?
PATCHES["mo_nolookup_nomfma"] = PATCHES["mo_nolookup"] + [("motion.hip", """                acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(wc[j >> 2][j & 3], bq[j], acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(wc[2 + (j >> 2)][j & 3], bq[j], acc1, 0, 0, 0);""",
    """                asm volatile("" :: "v"(wc[j >> 2][j & 3]), "v"(wc[2 + (j >> 2)][j & 3]), "v"(bq[j]));""")]
# ... and without the output stores (the epilogue's bias loads kept)
PATCHES["mo_nolookup_nomfma_nost"] = PATCHES["mo_nolookup_nomfma"] + [("motion.hip", "                        out[((int64_t)b * O + o) * P.q_count + q] = v < 0.0f ? 0.0f : v;   // NaN stays NaN",
    "                        if (v == 1234.5f) out[((int64_t)b * O + o) * P.q_count + q] = v;")]
PATCHES["mo_nolookup_nost"] = PATCHES["mo_nolookup"] + PATCHES["mo_nolookup_nomfma_nost"][-1:]
PATCHES["l01oob"] = [("build.hip", "ok ? base + (int)(s * lsz * 4) : SOOB, 0, ST_L01);", "ok ? SOOB : SOOB, 0, ST_L01);")]
PATCHES["dmaoob"] = [("build.hip", "in ? kc * PANEL + c * 1024 + lane * 16 : SOOB, 0, 0, 0);", "in ? SOOB : SOOB, 0, 0, 0);")]
PATCHES["qoob"] = [("build.hip", "rq, in ? qgo + kc * PANEL + i * 2048 : SOOB, 0, 0));", "rq, in ? SOOB : SOOB, 0, 0));"),
                   ("build.hip", "rq, in ? qgo + kc * PANEL + i * 2048 + 1024 : SOOB, 0, 0));", "rq, in ? SOOB : SOOB, 0, 0));")]
# split-loop prefetch depth of the target panel (tree: 4 chunks / buffers)
for _dt in (3, 5, 6):
    PATCHES[f"dt{_dt}"] = [("build.hip", "constexpr int SDT = 4; ", f"constexpr int SDT = {_dt}; ")]
# timing only: every block reads the same query / target panels (all L2 hits, same traffic to the CUs)
PATCHES["sameq"] = [("build.hip", "P.pk1 + ((int64_t)b * P.n_mt + qp) * pstride", "P.pk1")]
PATCHES["samet"] = [("build.hip", "P.pk2 + ((int64_t)b * P.n_nt + nt) * pstride", "P.pk2")]
# epilogue pacing: s_sleep after each level-0 line's four stores (timing A/B; bitwise the same)
for _sl in (2, 6, 16):
    PATCHES[f"pace{_sl}"] = [("build.hip", "ok ? base + (int)(s * lsz * 4) : SOOB, 0, ST_L01);\n",
                              f"ok ? base + (int)(s * lsz * 4) : SOOB, 0, ST_L01);\n        __builtin_amdgcn_s_sleep({_sl});\n")]
COMBOS = {}
COMBOS.update({"sameqt": ["sameq", "samet"]})
# round 6, timing only: the store stream kept, every panel AND per-pixel exponent
# read from batch item 0's first tiles (L2-resident), so the K loop's reads never leave the L2
PATCHES["sameex"] = [("build.hip", "eq = q0 + tid < P.q_count ? P.ex1[(int64_t)b * P.q_count + q0 + tid] : 0;",
                      "eq = q0 + tid < P.q_count ? P.ex1[tid] : 0;"),
                     ("build.hip", "et = (y < H && x < W) ? P.ex2[(int64_t)b * Q + (int64_t)y * W + x] : 0;",
                      "et = (y < H && x < W) ? P.ex2[tid] : 0;")]
COMBOS.update({"l2rd": ["sameq", "samet", "sameex"]})
# round 6, timing only: the level-0 stores of FULL tiles into one contiguous 128-KB region per block
# (l0contig: a wave's 8 stores of a query group fill 8 KB; l0c1k: each store instruction writes 1 KB
# contiguous) instead of 2 x 256 B per query image -- is the scattered write stream's DRAM page
# locality (row activations, power) part of the GEMM's clock loss?  The pyramid is wrong (AB_NOCHECK).
_L0C_DECL = ("build.hip", "    const int grpw = qwu >> 6;   // FULL: the wave's interleaved group (block-relative)\n",
             "    const int grpw = qwu >> 6;   // FULL: the wave's interleaved group (block-relative)\n"
             "    const __amdgpu_buffer_rsrc_t r0c = __builtin_amdgcn_make_buffer_rsrc(P.lvl[0], 0, 0x7ffffff0, 0x00020000);\n"
             "    const int c0 = (int)(blockIdx.x * 131072u) + (qwu >> 6) * 4 * 8192 + L0C_LANE;\n")
PATCHES["l0contig"] = [("build.hip", "constexpr int SQ = 256; ", "#define L0C_LANE ((8 * jl) * 128 + 16 * pc)\nconstexpr int SQ = 256; "), _L0C_DECL,
                       ("build.hip", "            if (FULL) fst4(r0, v0, (qwu + 16 * qg + s) * l0stride, x);",
                        "            if (FULL) fst4(r0c, c0 + qg * 8192 + s * 128, 0, x);")]
PATCHES["l0c1k"] = [("build.hip", "constexpr int SQ = 256; ", "#define L0C_LANE (jl * 128 + 16 * pc)\nconstexpr int SQ = 256; "), _L0C_DECL,
                    ("build.hip", "            if (FULL) fst4(r0, v0, (qwu + 16 * qg + s) * l0stride, x);",
                     "            if (FULL) fst4(r0c, c0 + qg * 8192 + s * 1024, 0, x);")]
COMBOS.update({"dmaqoob": ["dmaoob", "qoob"], "noepi_r2": ["noepi"]})
COMBOS.update({"st16_prio_loop": ["st16", "prio_loop"]})
COMBOS.update({"noepi_mfma16": ["noepi", "mfma16"]})
COMBOS.update({"st16_sscale": ["st16", "sscale"], "st16_noscale": ["st16", "noscale"]})
# round 6: the round-3 split16 ablations, rebuilt on today's kernel (their recipes were retired; the
# older noepi / l01oob patch the 32x32 build_split_kernel, not split16): every epilogue store out of
# range (same instructions, no store traffic), and the epilogue replaced by one store per lane
PATCHES["s16_stoob"] = [
    ("build.hip", "__builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(uint4v, v), rs, ok ? off : SOOB, 0, ST_L01);",
     "__builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(uint4v, v), rs, (ok ? off : SOOB) | 0x70000000, 0, ST_L01);"),
    ("build.hip", "__builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(uint2v, v), rs, ok ? off : SOOB, 0, ST_L01);",
     "__builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(uint2v, v), rs, (ok ? off : SOOB) | 0x70000000, 0, ST_L01);"),
    ("build.hip", "__builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(uint4v, v), rs, voff + uoff, 0, ST_L01);",
     "__builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(uint4v, v), rs, (voff + uoff) | 0x70000000, 0, ST_L01);"),
    ("build.hip", "__builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(uint2v, v), rs, voff + uoff, 0, ST_L01);",
     "__builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(uint2v, v), rs, (voff + uoff) | 0x70000000, 0, ST_L01);")]
PATCHES["s16_noepi"] = [("build.hip", """    if (q0 + SQ <= P.q_count && (((int64_t)b * P.q_count + q0) & (kGroup - 1)) == 0)
        split16_epilogue<MUL, true>(P, acc, smem + wave * (2 * 64 * S16LS), wave * 64, exq, ext, fst, tc, b, q0, lane);
    else
        split16_epilogue<MUL, false>(P, acc, smem + wave * (2 * 64 * S16LS), wave * 64, exq, ext, fst, tc, b, q0, lane);
}""", """    {
        float s = 0.f;
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
            for (int t = 0; t < 8; ++t)
#pragma unroll
                for (int i = 0; i < 4; ++i) s += acc[g][t][i];
        P.lvl[0][(int64_t)blockIdx.x * 256 + tid] = s;
    }
}""")]
COMBOS.update({"st16_s16stoob": ["st16", "s16_stoob"]})
# round 6: the level-0 LDS transpose reads of a query group issued back to back (eight in flight)
# before its eight stores; the emitted code read two ahead with a wait per store (bitwise the same)
PATCHES["s16_rd8"] = [("build.hip", """#pragma unroll
        for (int s = 0; s < 8; ++s) {
            const floatx4 x = *reinterpret_cast<const floatx4*>(xr + (s + 8 * jl) * S16LS + 16 * pc);
            if (FULL) fst4(r0, v0, (qwu + 16 * qg + s) * l0stride, x);
            else st4(r0, l0off + (16 * qg + s) * l0stride, l0ok && l0q + 16 * qg + s < nq, x);
        }""", """        floatx4 xs8[8];
#pragma unroll
        for (int s = 0; s < 8; ++s) xs8[s] = *reinterpret_cast<const floatx4*>(xr + (s + 8 * jl) * S16LS + 16 * pc);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            if (FULL) fst4(r0, v0, (qwu + 16 * qg + s) * l0stride, xs8[s]);
            else st4(r0, l0off + (16 * qg + s) * l0stride, l0ok && l0q + 16 * qg + s < nq, xs8[s]);
        }""")]
# round 6, timing only (what bounds the split conv's instruction floor?): the split VALU replaced
# by one conversion per value (lo = 0), and the A-fragment LDS reads replaced by register values
PATCHES["cv_nosplit"] = [("conv.hip", """        const float x = v[j] * s;
        const _Float16 h = (_Float16)x;
        hi[j] = h;
        lo[j] = (_Float16)(x - (float)h);""", """        hi[j] = (_Float16)v[j];
        lo[j] = (_Float16)s;""")]
PATCHES["cv_nolds"] = [("conv.hip", """            ah[i] = *reinterpret_cast<const halfx8*>(wb + ((4 * oh + i) * 2 + 0) * 1024);
            al[i] = *reinterpret_cast<const halfx8*>(wb + ((4 * oh + i) * 2 + 1) * 1024);""",
                        """            ah[i] = bh * (_Float16)(i + 1);
            al[i] = bl * (_Float16)(i + 2);"""),
                       ("conv.hip", """                ah[s] = *reinterpret_cast<const halfx8*>(wb + ((4 * oh + i + 2) * 2 + 0) * 1024);
                al[s] = *reinterpret_cast<const halfx8*>(wb + ((4 * oh + i + 2) * 2 + 1) * 1024);""",
                        """                ah[s] = bl * (_Float16)(i + 3);
                al[s] = bh * (_Float16)(i + 4);""")]
# round 6: the split's lo half as one fused op, f16(fma(hi, -1, x)) -- v_fma_mix (hi extended from f16
# in the fma, one rounding to f16: bitwise (_Float16)(x - (float)hi), x - hi being exact)
PATCHES["cv_fmix"] = [("conv.hip", """        lo[j] = (_Float16)(x - (float)h);""", """        lo[j] = (_Float16)__builtin_fmaf((float)h, -1.0f, x);""")]
# round 6: the split with v_fma_mixlo/hi_f16 (inline asm; the compiler turns fma(hi, -1, x) back into
# sub + converts): lo pair = f16(x0 - hi0), f16(x1 - hi1) from the packed hi register, 2 ops per pair
PATCHES["cv_mixasm"] = [("conv.hip", """__device__ __forceinline__ void split8(const float (&v)[8], float s, halfx8& hi, halfx8& lo) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const float x = v[j] * s;
        const _Float16 h = (_Float16)x;
        hi[j] = h;
        lo[j] = (_Float16)(x - (float)h);
    }
}""", """__device__ __forceinline__ void split8(const float (&v)[8], float s, halfx8& hi, halfx8& lo) {
    typedef _Float16 half2v __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
        const float x0 = v[j] * s, x1 = v[j + 1] * s;
        const half2v h = {(_Float16)x0, (_Float16)x1};
        const unsigned hp = __builtin_bit_cast(unsigned, h);
        unsigned lp;
        asm volatile("v_fma_mixlo_f16 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(lp) : "v"(hp), "v"(x0));
        asm volatile("v_fma_mixhi_f16 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(lp) : "v"(hp), "v"(x1));
        const half2v l = __builtin_bit_cast(half2v, lp);
        hi[j] = h[0];
        hi[j + 1] = h[1];
        lo[j] = l[0];
        lo[j + 1] = l[1];
    }
}""")]
# round 6: the accumulators in AGPRs ("+a"): the partner block's epilogue VALU then shares no
# register-file traffic with the MFMAs' accumulator reads / writes; the epilogue pays one
# v_accvgpr_read per accumulator (bitwise the same pyramid)
PATCHES["s16_agpr"] = [
    ("build.hip", """        for (int t = 0; t < 8; ++t) asm volatile("" : "+v"(acc[g][t]));

    // query fragments""", """        for (int t = 0; t < 8; ++t) asm volatile("" : "+a"(acc[g][t]));

    // query fragments"""),
    ("build.hip", """asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(bq));""",
     """asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(bq));"""),
    ("build.hip", """        for (int t = 0; t < 8; ++t) asm volatile("" : "+v"(acc[g][t]));
    // FULL""", """        for (int t = 0; t < 8; ++t) asm volatile("" : "+a"(acc[g][t]));
    // FULL""")]

# ---- round 4: the split16 epilogue's scaling (bitwise-equal variants unless marked timing only)
_S16_PK = """                for (int h = 0; h < 2; ++h) {
                    const floatx2 x = floatx2{acc[qg][tg][2 * h], acc[qg][tg][2 * h + 1]} *
                                      (sq2 * floatx2{s4[2 * h], s4[2 * h + 1]});
                    v[tg][2 * h] = MUL ? x[0] : __fdiv_rn(x[0], P.scale);
                    v[tg][2 * h + 1] = MUL ? x[1] : __fdiv_rn(x[1], P.scale);
                }"""
# scalar v_mul_f32 instead of v_pk_mul_f32 (MI355X_MICROARCH.md: packed f32 VALU beside MFMAs is
# an anti-lever), same products in the same order
PATCHES["sscale"] = [("build.hip", _S16_PK, """                for (int t = 0; t < 4; ++t) {
                    const float x = __fmul_rn(acc[qg][tg][t], __fmul_rn(sq, s4[t]));
                    v[tg][t] = MUL ? x : __fdiv_rn(x, P.scale);
                }""")]
# timing only: no scaling at all (v = acc): what the scaling costs
PATCHES["noscale"] = [("build.hip", _S16_PK, """                for (int t = 0; t < 4; ++t) v[tg][t] = acc[qg][tg][t] + s4[t] * 0.0f;""")]


# ---- round 4: fused lookup + convc1, second resident workgroup of each CU in the first dispatch
# round (linear ids 256..511: CU-breadth-first placement) started late by ~N x 4 us, so one
# workgroup's lookup phase runs beside the other's GEMM phase instead of in step with it
for _n in (1, 3, 6):
    PATCHES[f"mo_stag{_n}"] = [("motion.hip", """    const int tid = threadIdx.x, g = tid % QBM, part = tid / QBM, lane = tid & 63, wave = tid >> 6;
    const int half = part & 1;""", f"""    {{
        const unsigned lin = blockIdx.x + gridDim.x * blockIdx.y;
        if (lin >= 256 && lin < 512)
            for (int z = 0; z < {_n}; ++z) __builtin_amdgcn_s_sleep(127);
    }}
    const int tid = threadIdx.x, g = tid % QBM, part = tid / QBM, lane = tid & 63, wave = tid >> 6;
    const int half = part & 1;""")]

# ---- round 4: persistent split16 build -- 512 blocks (two per CU) walk the tiles, one barrier
# between a block's tiles; would measure what the per-block dispatch gaps cost (bitwise the same).
# Not run: the tile loop pushes the kernel to 256 VGPRs + 204 B/lane of scratch spills.
PATCHES["s16_pers"] = [
    ("build.hip", """template <bool MUL>
__global__ __launch_bounds__(256, 2) void build_split16_kernel(BuildParams P) {
    // ALL LDS in this one array (cdna_hip_programming.md trap 4(a), see build_split_kernel)
    __shared__ __attribute__((aligned(16))) char smem[SLDS + (SQ + 256) * 4];
    int* exq""", """template <bool MUL>
__device__ __forceinline__ void split16_tile(const BuildParams& P, char* smem, int tile) {
    int* exq"""),
    ("build.hip", """    decode_tile<kGM16, true>(P, xcd_remap(blockIdx.x, gridDim.x), P.n_qt, b, qt, nt);
    const NTile tc = ntile_of(P, nt);
    const int q0 = qt * SQ;
    const int H = P.H, W = P.W;
    const int64_t Q = (int64_t)H * W;

    // per-pixel exponents: loaded behind the K loop's last static wait (only the epilogue reads them)""",
     """    decode_tile(P, tile, P.n_qt, b, qt, nt);
    const NTile tc = ntile_of(P, nt);
    const int q0 = qt * SQ;
    const int H = P.H, W = P.W;
    const int64_t Q = (int64_t)H * W;

    // per-pixel exponents: loaded behind the K loop's last static wait (only the epilogue reads them)"""),
    ("build.hip", """        split16_epilogue<MUL, false>(P, acc, smem + wave * (2 * 64 * S16LS), wave * 64, exq, ext, fst, tc, b, q0, lane);
}
""", """        split16_epilogue<MUL, false>(P, acc, smem + wave * (2 * 64 * S16LS), wave * 64, exq, ext, fst, tc, b, q0, lane);
}

template <bool MUL>
__global__ __launch_bounds__(256, 2) void build_split16_kernel(BuildParams P, int ntiles) {
    __shared__ __attribute__((aligned(16))) char smem[SLDS + (SQ + 256) * 4];
    for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
        split16_tile<MUL>(P, smem, xcd_remap(t, ntiles));
        __syncthreads();   // every wave's epilogue is done with the panel buffers
    }
}
"""),
    ("build.hip", """            if (P.scale_is_mul) hipLaunchKernelGGL((build_split16_kernel<true>), grid, dim3(256), 0, stream, P);
            else hipLaunchKernelGGL((build_split16_kernel<false>), grid, dim3(256), 0, stream, P);""",
     """            const dim3 pg((unsigned)(ntiles < 512 ? ntiles : 512));
            if (P.scale_is_mul) hipLaunchKernelGGL((build_split16_kernel<true>), pg, dim3(256), 0, stream, P, (int)ntiles);
            else hipLaunchKernelGGL((build_split16_kernel<false>), pg, dim3(256), 0, stream, P, (int)ntiles);"""),
]


# ---- round 4: the fused lookup + convc1 as the two-workgroup kernel (the tree: warp-specialized)
# (mo_2wg: the two-workgroup fused kernel -- the tree since round 5; the WS kernel is lab_patches/lookup_conv_ws.diff)

# ---- round 4: stamps of the warp-specialized fused kernel: per workgroup, the cycles its producer
# wave 0 spends in produce(), its consumer wave 4 in consume(), both in the barrier, and the steps
MO_DECL = """
__device__ unsigned long long g_mo[4096][8];
"""
MO_EXPORT = """
extern "C" __attribute__((visibility("default"))) int ecorr_lab_mostamps(void* dst, int n) {
    return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(ecorr::g_mo), (size_t)n * 64, 0, hipMemcpyDeviceToHost);
}
"""
PATCHES["mo_wsst"] = [
    ("motion.hip", "constexpr int KC = 16;     // channels per weight chunk", "constexpr int KC = 16;     // channels per weight chunk" + MO_DECL),
    ("motion.hip", """    const int t0 = (int)blockIdx.x;
    if (wave < 4) load_coords(t0);
    for (int k = 0; t0 + (k - 1) * G < ntiles; ++k) {
        const int t = t0 + k * G;
        if (wave < 4) {
            if (t < ntiles) produce(t, k & 1);
        } else if (k > 0) {
            consume(t - G, (k - 1) & 1);
        }
        __syncthreads();   // the buffers swap roles
    }
}""", """    const int t0 = (int)blockIdx.x;
    if (wave < 4) load_coords(t0);
    unsigned long long busy = 0, waitc = 0, steps = 0;
    const unsigned long long tstart = __builtin_amdgcn_s_memtime();
    for (int k = 0; t0 + (k - 1) * G < ntiles; ++k) {
        const int t = t0 + k * G;
        const unsigned long long a0 = __builtin_amdgcn_s_memtime();
        if (wave < 4) {
            if (t < ntiles) produce(t, k & 1);
        } else if (k > 0) {
            consume(t - G, (k - 1) & 1);
        }
        __builtin_amdgcn_s_waitcnt(0);
        const unsigned long long a1 = __builtin_amdgcn_s_memtime();
        __syncthreads();   // the buffers swap roles
        const unsigned long long a2 = __builtin_amdgcn_s_memtime();
        busy += a1 - a0;
        waitc += a2 - a1;
        ++steps;
    }
    if (lane == 0 && (wave == 0 || wave == 4) && blockIdx.x < 4096) {
        const int o = wave == 0 ? 0 : 3;
        g_mo[blockIdx.x][o + 0] = busy;
        g_mo[blockIdx.x][o + 1] = waitc;
        g_mo[blockIdx.x][o + 2] = steps;
        if (wave == 0) g_mo[blockIdx.x][6] = __builtin_amdgcn_s_memtime() - tstart;
    }
}"""),
    ("motion.hip", "}  // namespace ecorr\n", "}  // namespace ecorr\n" + MO_EXPORT),
]


# split convc1: non-temporal query-column loads (read once)
PATCHES["cv_bnt"] = [("conv.hip", "v[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(csrc, off + j * qs, 0, 0));",
                      "v[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(csrc, off + j * qs, 0, 2));")]
# the QMAX lookup's output stores with sc1 (16) / nt | sc1 (18) instead of the default policy
PATCHES["lk_qsc1"] = [("lookup.hip", "constexpr int kOutAux = QMAX ? 0 : 2;", "constexpr int kOutAux = QMAX ? 16 : 2;")]
PATCHES["lk_qntsc1"] = [("lookup.hip", "constexpr int kOutAux = QMAX ? 0 : 2;", "constexpr int kOutAux = QMAX ? 18 : 2;")]
# lookup_cols_reg dispatch order: all level-0 workgroups first (the longest: the largest image),
# then levels 1..3 fill the last round (LPT for the drain tail) -- or the reverse
_LK_OLD = """    const int lv = blockIdx.y, b = blockIdx.z;
    const int q0 = blockIdx.x * QB;
    const int p = q0 + g;"""
def _lk_lvmajor(rev):
    return [("lookup.hip", _LK_OLD, """    const int lin = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    const int per = gridDim.x * gridDim.z;
    const int lvo = lin / per, rr = lin - lvo * per;
    const int lv = %s, b = rr / gridDim.x;
    const int q0 = (rr - b * gridDim.x) * QB;
    const int p = q0 + g;""" % ("gridDim.y - 1 - lvo" if rev else "lvo"))]
# ... or the level fastest: a query group's four level workgroups dispatched back to back
PATCHES["lk_lvminor"] = [("lookup.hip", _LK_OLD, """    const int lin = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    const int lv = lin % gridDim.y, xb = lin / gridDim.y;
    const int b = xb / gridDim.x;
    const int q0 = (xb - b * gridDim.x) * QB;
    const int p = q0 + g;""")]
PATCHES["lk_lvmajor"] = _lk_lvmajor(False)
PATCHES["lk_lvmajor_rev"] = _lk_lvmajor(True)
PATCHES["cv_pf3"] = [("conv.hip", "constexpr int kConvPD = 2;", "constexpr int kConvPD = 3;")]
# round 6: the query-column loads with the channel row in the scalar soffset (one address VGPR for
# all 8 loads of a chunk instead of a v_add each); the range rule (an access iff voffset < records
# and voffset + soffset < records) keeps lanes past Q and channels past C reading 0
PATCHES["cv_soff"] = [("conv.hip", """        const int off = cbase + (c * SKC + 8 * kh) * qs;
#pragma unroll
        for (int j = 0; j < 8; ++j)
            v[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(csrc, off + j * qs, 0, 0));""",
                       """#pragma unroll
        for (int j = 0; j < 8; ++j)
            v[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(csrc, cvo, (c * SKC + j) * qs, 0));"""),
                      ("conv.hip", "    const int cbase = (qok ? q : C * Q) * 4, qs = Q * 4;\n",
                       "    const int cbase = (qok ? q : C * Q) * 4, qs = Q * 4;\n    const int cvo = cbase + 8 * kh * qs;\n")]
COMBOS["cv_soff_pf3"] = ["cv_soff", "cv_pf3"]
PATCHES["cv_pf4"] = [("conv.hip", "constexpr int kConvPD = 2;", "constexpr int kConvPD = 4;")]

# ---- round 5: is the lookup concurrency-bound?  LDS padded so that 4 / 3 workgroups fit a CU
# instead of 5 (timing only, bitwise the same); and de-phased first rounds (a share of the first
# 1280 workgroups sleeps ~3.8 / ~1.9 us before its coordinate loads)
def _lk_pad(nf):
    return [("lookup.hip", """    __shared__ WB st;
    const int tid = threadIdx.x, g = tid % QB;
    const int part = __builtin_amdgcn_readfirstlane(tid / QB);   // wave-uniform""", """    __shared__ WB st;
    __shared__ float lk_pad[%d];
    const int tid = threadIdx.x, g = tid %% QB;
    if (P.q_count == -12345) { lk_pad[tid] = 1.0f; __syncthreads(); P.out[tid] = lk_pad[(tid + 1) %% 192]; }
    const int part = __builtin_amdgcn_readfirstlane(tid / QB);   // wave-uniform""" % nf)]
PATCHES["lk_occ4"] = _lk_pad(2048)
PATCHES["lk_occ3"] = _lk_pad(5000)
def _lk_sleep(n, mod):
    return [("lookup.hip", """    __shared__ WB st;
    const int tid = threadIdx.x, g = tid % QB;
    const int part = __builtin_amdgcn_readfirstlane(tid / QB);   // wave-uniform""", """    __shared__ WB st;
    {
        const int lin = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
        if (lin < 1280 && (lin >> 8) %% %d == 1) __builtin_amdgcn_s_sleep(%d);
    }
    const int tid = threadIdx.x, g = tid %% QB;
    const int part = __builtin_amdgcn_readfirstlane(tid / QB);   // wave-uniform""" % (mod, n))]
PATCHES["lk_sleep127"] = _lk_sleep(127, 2)
PATCHES["lk_sleep64"] = _lk_sleep(64, 2)

# ---- round 5: where the lookup's time goes -- the same instructions with the window loads and / or
# the output stores out of range (no memory traffic; timing only)
PATCHES["lk_ldoob"] = [("lookup_stage.h", "__builtin_amdgcn_raw_buffer_load_b64(rsrc, need ? off : OOB, 0, 0);",
                        "__builtin_amdgcn_raw_buffer_load_b64(rsrc, need ? OOB : OOB + (off & 4), 0, 0);")]
PATCHES["lk_stoob"] = [("lookup.hip", "P.out + (int64_t)b * P.C * P.q_count, 0, P.C * P.q_count * 4, 0x00020000);",
                        "P.out + (int64_t)b * P.C * P.q_count, 0, P.q_count == -1 ? 4 : 0, 0x00020000);")]
COMBOS["lk_bothoob"] = ["lk_ldoob", "lk_stoob"]

# the same on lookup_win (round 5)
PATCHES["lkw_ldoob"] = [("lookup.hip", "(rsrc, (need ? off : OOB) + ry * WK::STEP, 0, 0);", "(rsrc, OOB + ry * WK::STEP + (need ? 0 : 4), 0, 0);")]
COMBOS["lkw_bothoob"] = ["lkw_ldoob", "lk_stoob"]

# lookup_win output store policy (aux bits: 1 sc0, 2 nt, 16 sc1) and window-load policy
for _a in (1, 3, 16, 17, 19):
    PATCHES[f"lkw_st{_a}"] = [("lookup.hip", "constexpr int kOutAux = QMAX ? 0 : 2;\n    auto store", f"constexpr int kOutAux = QMAX ? 0 : {_a};\n    auto store")]
for _a in (1, 16, 17):
    PATCHES[f"lkw_ld{_a}"] = [("lookup.hip", "(rsrc, (need ? off : OOB) + ry * WK::STEP, 0, 0);", f"(rsrc, (need ? off : OOB) + ry * WK::STEP, 0, {_a});")]
# round 5, VERDICT r4 item 3: the FULL epilogue's wave-uniform store term in the scalar soffset
# instead of the voffset (the round-3 variant that lost ~0.03% of level-0 stores): tools/soff_repro.py
PATCHES["soff_full"] = [
    ("build.hip", "__builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(uint4v, v), rs, voff + uoff, 0, ST_L01);",
     "__builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(uint4v, v), rs, voff, uoff, ST_L01);"),
    ("build.hip", "__builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(uint2v, v), rs, voff + uoff, 0, ST_L01);",
     "__builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(uint2v, v), rs, voff, uoff, ST_L01);")]

# round 5: the split16 GEMM's grouped tile order -- GM m-tiles x all n-tiles per group (tree: 8)
# (GM = 10 in two balanced groups at DSEC -- kept, build.hip decode_tile; gm_clock_l2_b.txt)
#  the in-kernel clock of each tile-group arm: per-block stamps (tools/stamps16.py)
for _gm in (2, 4, 8, 9, 12, 16):
    COMBOS[f"st16_gm{_gm}"] = ["st16", f"gm{_gm}"]

# round 5: per-phase stamps of the banded splat (thread 0 of each workgroup, s_memrealtime 100 MHz)
# -> g_sps[block][0..5] = start, staged, counted, scanned, bucketed, end; ecorr_lab_spstamps()
SPS_DECL = """
__device__ unsigned long long g_sps[65536][6];
__device__ __forceinline__ void sps(int k) {
    const int id = blockIdx.x + gridDim.x * blockIdx.y;
    if (threadIdx.x == 0 && id < 65536) g_sps[id][k] = __builtin_amdgcn_s_memrealtime();
}
"""
SPS_EXPORT = """
extern "C" __attribute__((visibility("default"))) int ecorr_lab_spstamps(void* dst, int n) {
    return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(ecorr::g_sps), (size_t)n * 48, 0, hipMemcpyDeviceToHost);
}
"""
PATCHES["sp_stamps"] = [
    ("splat.hip", "constexpr int NTB = 1024;", SPS_DECL + "constexpr int NTB = 1024;"),
    ("splat.hip", "    const int tid = threadIdx.x, band = (int)(blockIdx.x % (unsigned)G), b = (int)(blockIdx.x / (unsigned)G);\n",
     "    sps(0);\n    const int tid = threadIdx.x, band = (int)(blockIdx.x % (unsigned)G), b = (int)(blockIdx.x / (unsigned)G);\n"),
    ("splat.hip", "    __syncthreads();\n    const float* src = staged ? spts : gpts;\n",
     "    __syncthreads();\n    sps(1);\n    const float* src = staged ? spts : gpts;\n"),
    ("splat.hip", "    __syncthreads();\n\n    // 2. exclusive scan of cnt[0 .. nb)", "    __syncthreads();\n    sps(2);\n\n    // 2. exclusive scan of cnt[0 .. nb)"),
    ("splat.hip", "    __syncthreads();\n    // cnt[t] = start of target t's bucket", "    __syncthreads();\n    sps(3);\n    // cnt[t] = start of target t's bucket"),
    ("splat.hip", "            lkey[lo + r] = k;\n        }\n        __syncthreads();\n",
     "            lkey[lo + r] = k;\n        }\n        __syncthreads();\n        sps(4);\n"),
    ("splat.hip", "        for (int t = tid; t < nb; t += NTB) fold_sorted(lkey, t, t > 0 ? cnt[t - 1] : 0, cnt[t]);\n        return;\n",
     "        for (int t = tid; t < nb; t += NTB) fold_sorted(lkey, t, t > 0 ? cnt[t - 1] : 0, cnt[t]);\n        __syncthreads();\n        sps(5);\n        return;\n"),
    ("splat.hip", "}  // namespace ecorr\n", "}  // namespace ecorr\n" + SPS_EXPORT),
]

# round 5 diagnostics (timing only): output stores concentrated on 307 KB (the channel term dropped:
# all 81 channels of a level write one 256-B piece per workgroup) -- do the output writes cost the
# window reads their cache hits?  And window loads all from the first query group's slab (every
# workgroup reads the same lines: L2 hits)
PATCHES["lk_stsmall"] = [("lookup.hip", "sbase + (a * K + bb) * P.q_count * 4, kOutAux);", "sbase * 0 + ((a * K + bb) & 0), kOutAux);")]
PATCHES["lk_ldsmall"] = [("lookup_stage.h", "    const int64_t R0 = (int64_t)b * P.q_count + q0;   // first query row of the group",
                          "    const int64_t R0 = 0 * ((int64_t)b * P.q_count + q0);   // (lab: every group reads group 0)")]
COMBOS["lk_bothsmall"] = ["lk_stsmall", "lk_ldsmall"]

# timing only: each workgroup's 81 channels x 64 queries written as one contiguous 20.7 KB piece
# (same bytes, same store instructions, a wrong layout) -- does the NCHW output's 256-B-per-row
# scatter cost the write stream?
PATCHES["lk_stblock"] = [
    ("lookup.hip", "    const int voff = p * 4;\n    const int sbase = lv * KK * P.q_count * 4;",
     "    const int voff = g * 4;\n    const int sbase = (blockIdx.x + gridDim.x * lv) * KK * 256;"),
    ("lookup.hip", "sbase + (a * K + bb) * P.q_count * 4, kOutAux);", "sbase + (a * K + bb) * 256, kOutAux);"),
    ("lookup.hip", "sbase + ((part * AP + ai) * K + bb) * P.q_count * 4, kOutAux);", "sbase + ((part * AP + ai) * K + bb) * 256, kOutAux);")]

# ---- round 5, split convc1: what bounds conv1x1_split_kernel (timing only)?  Every workgroup reads
# batch item 0's first 64 query columns (the corr stream served by L2), and / or every output store
# out of range (no write stream)
PATCHES["cv_l2ld"] = [("conv.hip", "const_cast<float*>(in + (int64_t)b * C * Q), 0, C * Q * 4, 0x00020000);",
                       "const_cast<float*>(in + (int64_t)0 * b * C * Q), 0, C * Q * 4, 0x00020000);"),
                      ("conv.hip", "const int cbase = (qok ? q : C * Q) * 4, qs = Q * 4;",
                       "const int cbase = (qok ? qi : C * Q) * 4, qs = Q * 4;")]
PATCHES["cv_stoob"] = [("conv.hip", "const int obase = (qok ? q : O * Q) * 4;", "const int obase = (O * Q + 0 * q) * 4;")]
COMBOS["cv_bothoob"] = ["cv_l2ld", "cv_stoob"]
# (the ring form -- column chunks by LDS-DMA from a producer wave that waits only for its own loads
#  -- was measured from a tree copy and dropped: profiles/r05_lab/cv_ab_ring_oob.txt)
# query blocks per workgroup (QB: 2 = 64 queries, 4 = 128 queries sharing each weight chunk) and
# the column prefetch distance; cvq4n: QB 4 without the 4-waves-per-SIMD register cap (1 workgroup/CU)
for _qb, _pd in [(4, 1), (2, 1), (4, 2)]:
    PATCHES[f"cvq{_qb}p{_pd}"] = [("conv.hip", "constexpr int kConvQB = 2;", f"constexpr int kConvQB = {_qb};"),
                                  ("conv.hip", "constexpr int kConvPD = 2;", f"constexpr int kConvPD = {_pd};")]
# (A fragments double-buffered -- cv_adb, profiles/r05_lab/cv_ab_adb.txt -- is in the tree since round 5)
# timing only: no step barrier (LDS buffers race), or no MFMAs (the A / B
# operands still read and split, one add each keeps them live)
PATCHES["cv_nobar_"] = [("conv.hip", """        __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };""", """        __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)
        __builtin_amdgcn_sched_barrier(0);
    };""")]
PATCHES["cv_nomfma_"] = [("conv.hip", x, y) for x, y in [
    ("acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[s], bl, acc[i], 0, 0, 0);",
     "acc[i][0] += (float)ah[s][0] * (float)bl[0] + (float)al[s][1] * (float)bh[1];"),
    ("acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[s], bh, acc[i], 0, 0, 0);", ""),
    ("acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[s], bh, acc[i], 0, 0, 0);", "")]]
COMBOS["cv_adb_nobar"] = ["cv_nobar_"]
COMBOS["cv_adb_nomfma"] = ["cv_nomfma_"]
# 2 tiles per wave: a workgroup covers 128 output channels (half the weight chunk, 2 pieces per
# wave), 4 workgroups per CU; the halves of a query tile back to back on one XCD
PATCHES["cvt2"] = [("conv.hip", "constexpr int kConvTPW = 4;", "constexpr int kConvTPW = 2;")]
PATCHES["cvt2p3"] = PATCHES["cvt2"] + [("conv.hip", "constexpr int kConvPD = 2;", "constexpr int kConvPD = 3;")]
# convex upsampling (upsample.hip): two sub-rows i, i + 4 per thread (the 3x3 flow window loaded once,
# half the workgroups: one dispatch round at DSEC B = 16); mask loads with the default policy
PATCHES["up_i2"] = [("upsample.hip", """    const int i = blockIdx.y, n = blockIdx.z;
    if (p >= HW) return;""", """    const int n = blockIdx.z;
    if (p >= HW) return;"""),
                    ("upsample.hip", """    const float* mrow = mask + ((int64_t)n * 576 + i * 8) * HW + p;""",
                     """#pragma unroll 1
    for (int i = blockIdx.y; i < 8; i += 4) {
    const float* mrow = mask + ((int64_t)n * 576 + i * 8) * HW + p;"""),
                    ("upsample.hip", """        __builtin_nontemporal_store(floatx4{res[c][4], res[c][5], res[c][6], res[c][7]}, (floatx4*)(o + 4));
    }
}""", """        __builtin_nontemporal_store(floatx4{res[c][4], res[c][5], res[c][6], res[c][7]}, (floatx4*)(o + 4));
    }
    }
}"""),
                    ("upsample.hip", "const dim3 grid((unsigned)((H * W + NTU - 1) / NTU), 8, (unsigned)N);",
                     "const dim3 grid((unsigned)((H * W + NTU - 1) / NTU), 4, (unsigned)N);")]
# convex upsampling: output stores with the default policy instead of non-temporal
PATCHES["up_stplain"] = [("upsample.hip", """        __builtin_nontemporal_store(floatx4{res[c][0], res[c][1], res[c][2], res[c][3]}, (floatx4*)o);
        __builtin_nontemporal_store(floatx4{res[c][4], res[c][5], res[c][6], res[c][7]}, (floatx4*)(o + 4));""",
                          """        *(floatx4*)o = floatx4{res[c][0], res[c][1], res[c][2], res[c][3]};
        *(floatx4*)(o + 4) = floatx4{res[c][4], res[c][5], res[c][6], res[c][7]};""")]
# lookup: window loads non-temporal (aux 2) -- the upsampling's lesson checked the other way
PATCHES["lk_ldnt"] = [("lookup_stage.h", "const uint2v u = __builtin_amdgcn_raw_buffer_load_b64(rsrc, need ? off : OOB, 0, 0);",
                       "const uint2v u = __builtin_amdgcn_raw_buffer_load_b64(rsrc, need ? off : OOB, 0, 2);"),
                      ("lookup_stage.h", "vals[c][ry][0] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsrc, need ? off : OOB, 0, 0));",
                       "vals[c][ry][0] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsrc, need ? off : OOB, 0, 2));")]
# split16 epilogue: levels 2 and 3 (92 + 23 MB at DSEC B = 16, what the 12 lookups re-read most
# densely) stored with the default policy (or only level 3), so that they may stay in the Infinity
# Cache for the lookups; levels 0-1 stay nt.  Step-level A/B: tools/ab_step.py
def _st23(aux, levels):
    rep = [("build.hip", """    auto fst2 = [&](__amdgpu_buffer_rsrc_t rs, int voff, int uoff, floatx2 v) {
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(uint2v, v), rs, voff + uoff, 0, ST_L01);
    };""", """    auto fst2 = [&](__amdgpu_buffer_rsrc_t rs, int voff, int uoff, floatx2 v) {
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(uint2v, v), rs, voff + uoff, 0, ST_L01);
    };
    auto fst2p = [&](__amdgpu_buffer_rsrc_t rs, int voff, int uoff, floatx2 v) {
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(uint2v, v), rs, voff + uoff, 0, %d);
    };
    auto st2p = [&](__amdgpu_buffer_rsrc_t rs, int off, bool ok, floatx2 v) {
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(uint2v, v), rs, ok ? off : SOOB, 0, %d);
    };""" % (aux, aux))]
    for lv in levels:
        rep += [("build.hip", f"if (FULL) fst2(r{lv}, v{lv},", f"if (FULL) fst2p(r{lv}, v{lv},"),
                ("build.hip", f"else st2(r{lv}, (grp * G{lv}", f"else st2p(r{lv}, (grp * G{lv}")]
    return rep
PATCHES["st23_plain"] = _st23(0, (2, 3))
PATCHES["st3_plain"] = _st23(0, (3,))
PATCHES["st23_sc1"] = _st23(16, (2, 3))
# timing only (phase-1 conflicts): every staging ds_write at a lane-linear,
# conflict-free address (same instruction count; the windows then hold the wrong values)
PATCHES["lk_wrlin"] = [("lookup_stage.h",
    "                    st.win[sr.skip[c] == v ? DUMMY : sr.dst[c] + ry * SW + v] = sr.vals[c][ry][v];",
    "                    st.win[(((c * SR::S + ry) * SR::V + v) * NTQ + (int)threadIdx.x % NTQ) % DUMMY] = sr.vals[c][ry][v];")]
# timing only: no weight DMA inside the K loop (every chunk multiplies the prologue's stale weights)
PATCHES["cv_nowdma"] = [("conv.hip", "        issue_w(min(c + 2, nkc - 1), (c + 2) % NB);   // past the last chunk a harmless repeat\n", "")]


# recipe-name prefix -> the lab_patches diff it applies on top of
# voxel tiled gather (timing only unless noted): phases skipped / LDS capacity
_VX_FOLD = "    if (yc < A.H && xc < A.W && tc0 < tc1) {"
PATCHES["vx_nofold_"] = [("voxel.hip", _VX_FOLD, "    if (yc < 0) {")]
PATCHES["vx_norank_"] = [("voxel.hip", "    for (int j = tid; j < n; j += VB_NT) {   // rank within the run by event index",
                          "    for (int j = tid; j < 0; j += VB_NT) {   // rank within the run by event index")]
PATCHES["vx_noplace_"] = [("voxel.hip", "    for (int j = tid; j < n; j += VB_NT) {   // place: off[r] walks",
                           "    for (int j = tid; j < 0; j += VB_NT) {   // place: off[r] walks")]
COMBOS["vx_nofold"] = ["vx_nofold_"]
COMBOS["vx_countonly"] = ["vx_nofold_", "vx_norank_", "vx_noplace_", "vx_noreorder_"]
PATCHES["vx_noreorder_"] = [("voxel.hip", "    if (!ar) {   // the window's events into run order in place", "    if (false) {   // the window's events into run order in place")]
COMBOS["vx_sortonly"] = ["vx_nofold_", "vx_norank_", "vx_noreorder_"]
# the gather's loads only: the window's copies read, nothing counted
PATCHES["vx_loadonly_"] = [("voxel.hip", "        atomicAdd(&L.off[run_of(ev)], 1);", "        if (ev.x == 12345.f) atomicAdd(&L.off[0], 1);")]
COMBOS["vx_loadonly"] = ["vx_nofold_", "vx_norank_", "vx_noreorder_", "vx_noplace_", "vx_loadonly_"]
# operand pass (timing only): no panel stores (the split still computed; a never-true test keeps it)
# / no fmap loads (values from the pixel index; the stores kept)
_PK_ST = """        *reinterpret_cast<halfx8*>(p) = h0;
        *reinterpret_cast<halfx8*>(p + k8) = h1;
        *reinterpret_cast<halfx8*>(p + 1024) = l0;
        *reinterpret_cast<halfx8*>(p + 1024 + k8) = l1;
"""
PATCHES["pk_nostore"] = [("build.hip", _PK_ST, "        if (h0[0] == (_Float16)12345.0f && l1[7] == (_Float16)-3.0f) {\n" + _PK_ST + "        }\n")]
PATCHES["pk_noload"] = [("build.hip", "                v[i][kk] = (pix >= 0 && k < D) ? px[(int64_t)k * N] : 0.f;",
                         "                v[i][kk] = (pix >= 0 && k < D) ? (float)(pix + k) : 0.f;")]
# operand pass (timing + accuracy probe, not bitwise): the split's lo halves rounded down to 8 / 6
# significant bits (fewer toggling multiplier bits in the lo.hi / hi.lo MFMAs of a power-limited GEMM)
PATCHES["lo8"] = [("build.hip", "        lo[j] = (_Float16)(x - (float)h);",
                   "        lo[j] = (_Float16)__uint_as_float(__float_as_uint(x - (float)h) & 0xFFFF0000u);")]
PATCHES["lo6"] = [("build.hip", "        lo[j] = (_Float16)(x - (float)h);",
                   "        lo[j] = (_Float16)__uint_as_float(__float_as_uint(x - (float)h) & 0xFFFC0000u);")]
# voxel count blocks (bitwise): 512 threads x 8 events (245 blocks at 1M events) / 1024 x 4 (245)
PATCHES["vx_cnt512"] = [("voxel.hip", "constexpr int VB_CNT = 1024, VB_EPB = 8 * VB_CNT;", "constexpr int VB_CNT = 512, VB_EPB = 8 * VB_CNT;")]
PATCHES["vx_epb4"] = [("voxel.hip", "constexpr int VB_CNT = 1024, VB_EPB = 8 * VB_CNT;", "constexpr int VB_CNT = 1024, VB_EPB = 4 * VB_CNT;")]

PREDIFF = {"qs": "build_qs.diff", "lkw_": "lookup_win.diff", "mo_ws": "lookup_conv_ws.diff", "cvq": "conv_tiles.diff",
           "cvt": "conv_tiles.diff"}


# Recipes whose patch targets the tree has moved past, with the last commit they apply to (their
# records stay under profiles/): build them from a worktree of that commit.  The presplit convc1
# (8712df9) rewrote conv.hip's column loads and lookup.hip's store path.
RETIRED = {n: "4dc7dd1" for n in (
    "cv_bothoob", "cv_l2ld", "cv_soff", "cv_soff_pf3", "cvq2p1", "cvq4p1", "cvq4p2", "cvt2", "cvt2p3",
    "lkw_bothoob", "lkw_ld1", "lkw_ld16", "lkw_ld17", "lkw_ldoob", "lkw_st1", "lkw_st16", "lkw_st17", "lkw_st19",
    "lkw_st3")}


def build(name):
    if name in RETIRED:
        raise SystemExit(f"{name}: retired, applies to the tree at {RETIRED[name]} "
                         f"(git worktree add /tmp/wt {RETIRED[name]}; run this tool there)")
    dst = os.path.join(ROOT, "tools", f"{name}_lab")
    if os.path.exists(dst):
        shutil.rmtree(dst)
    shutil.copytree(os.path.join(ROOT, "e-raft_amd", "csrc"), os.path.join(dst, "e-raft_amd", "csrc"),
                    ignore=shutil.ignore_patterns("build"))
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(dst, "include"))
    # recipes on top of a rejected variant kept as a diff (tools/lab_patches/): apply it first
    for diff in sorted({d for n in COMBOS.get(name, [name]) for pre, d in PREDIFF.items() if n.startswith(pre)}):
        subprocess.run(["patch", "-s", "-p1", "-d", dst, "-i", os.path.join(ROOT, "tools", "lab_patches", diff)], check=True)
    for fname, old, new in [x for n in COMBOS.get(name, [name]) for x in PATCHES[n]]:
        p = os.path.join(dst, "e-raft_amd", "csrc", fname)
        s = open(p).read()
        if old not in s:
            raise SystemExit(f"{name}: patch target not found in {fname}: {old[:60]!r}")
        s = s.replace(old, new)
        open(p, "w").write(s)
    subprocess.run(["make", "-s", "-j8", "-C", os.path.join(dst, "e-raft_amd", "csrc")], check=True)
    print(f"built tools/{name}_lab/e-raft_amd/libecorr.so")


def check():
    """Every recipe's patch targets exist in the current tree (after its lab_patches diff, if any):
    no build, seconds.  Returns the names of recipes that no longer apply."""
    import tempfile
    csrc = os.path.join(ROOT, "e-raft_amd", "csrc")
    srcs = {f: open(os.path.join(csrc, f)).read() for f in os.listdir(csrc) if f.endswith((".hip", ".h"))}
    bad = []
    for name in sorted(set(PATCHES) | set(COMBOS)):
        if (name.endswith("_") and name not in COMBOS) or name in RETIRED:   # a combo component; retired
            continue
        s = dict(srcs)
        diffs = sorted({d for n in COMBOS.get(name, [name]) for pre, d in PREDIFF.items() if n.startswith(pre)})
        ok = True
        if diffs:
            with tempfile.TemporaryDirectory() as d:
                os.makedirs(os.path.join(d, "e-raft_amd", "csrc"))
                for f, t in srcs.items():
                    open(os.path.join(d, "e-raft_amd", "csrc", f), "w").write(t)
                for diff in diffs:
                    ok = ok and subprocess.run(["patch", "-s", "-p1", "-d", d, "-i",
                                                os.path.join(ROOT, "tools", "lab_patches", diff)],
                                               capture_output=True).returncode == 0
                if ok:
                    s = {f: open(os.path.join(d, "e-raft_amd", "csrc", f)).read() for f in srcs}
        for fname, old, new in ([x for n in COMBOS.get(name, [name]) for x in PATCHES.get(n, [])] if ok else []):
            if old not in s.get(fname, ""):
                ok = False
                break
            s[fname] = s[fname].replace(old, new)
        if not ok:
            bad.append(name)
    return bad


if __name__ == "__main__":
    if sys.argv[1:] == ["--check"]:
        bad = check()
        print(f"{len(set(PATCHES) | set(COMBOS))} recipes ({len(RETIRED)} retired), {len(bad)} stale"
              + (": " + " ".join(bad) if bad else ""))
        sys.exit(1 if bad else 0)
    for n in sys.argv[1:]:
        build(n)
