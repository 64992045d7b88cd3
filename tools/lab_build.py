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
    # K loop without its MFMAs (fragments kept alive)
    "nomfma": [("build.hip", "                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f.th[j], f.ql[i], acc[i][j], 0, 0, 0);",
                "                asm volatile(\"\" :: \"v\"(f.th[j]), \"v\"(f.ql[i]));"),
               ("build.hip", "                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f.tl[j], f.qh[i], acc[i][j], 0, 0, 0);",
                "                asm volatile(\"\" :: \"v\"(f.tl[j]), \"v\"(f.qh[i]));"),
               ("build.hip", "                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f.th[j], f.qh[i], acc[i][j], 0, 0, 0);",
                "                asm volatile(\"\" :: \"v\"(f.th[j]), \"v\"(f.qh[i]));")],
    # store cache policy of the level-0/1 segments: sc1, plain (tree: nt sc1)
    "stsc1": [("build.hip", "constexpr int ST_SC1 = 18;", "constexpr int ST_SC1 = 16;")],
    "stplain": [("build.hip", "constexpr int ST_SC1 = 18;", "constexpr int ST_SC1 = 0;")],
    "stnt": [("build.hip", "constexpr int ST_SC1 = 18;", "constexpr int ST_SC1 = 2;")],
    # the second wave of resident blocks starts ~12 us late (do co-resident blocks run in phase?)
    "stagger": [("build.hip", "    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;\n    const int acol",
                 "    if (blockIdx.x >= 256 && blockIdx.x < 512)\n        for (int z = 0; z < 3; ++z) __builtin_amdgcn_s_sleep(127);\n"
                 "    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;\n    const int acol")],
}
# half-period stagger (~11 us at 1.43 GHz) of the second resident block of every CU
PATCHES["stagger2"] = [(f, o, n.replace("z < 3", "z < 2")) for f, o, n in PATCHES["stagger"]]
# timing only: the K loop without the 4 query-panel LDS-DMA pieces per wave and chunk (the query
# fragments read stale LDS): what does the DMA issue cost the loop?
PATCHES["noqdma"] = [("build.hip", "            if (s < 4) {\n", "            if (s < 4) { continue;\n"),
                     ("build.hip", "        wait_vm<SCOPIES, true>();\n", "        wait_vm<2, true>();\n")]
# stores spread over the K loop (4 store instructions per chunk, level-0-line shaped, junk
# values), epilogue dropped: does spreading the store stream let it overlap the matrix work?
SPREAD_SLOT = """
    auto spread_slot = [&](int kc) {
        const int64_t rows0s = (int64_t)b * P.q_count + q0;
        const int nqs = min(SQ, P.q_count - q0);
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(P.lvl[0] + rows0s * P.lsz[0], 0, (int)(nqs * P.lsz[0] * 4), 0x00020000);
        const int ii = (kc >> 2) & 1, jj = kc & 3, ql = wave * 64 + 32 * ii;
        const int tr = (tc.ty0 >> 2) + (jj & 1), tcl = (tc.tx0 >> 3) + (jj >> 1);
        const int base = (int)((ql + 4 * ((lane & 31) >> 2)) * P.lsz[0] * 4) + ((tr * P.lntx[0] + tcl) * kTile) * 4 + 64 * (lane >> 5) + 16 * (lane & 3);
        const bool ok = kc < 8 && tr < P.lnty[0] && tcl < P.lntx[0];
#pragma unroll
        for (int s = 0; s < 4; ++s)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(uint4v, floatx4{acc[0][0][s], acc[0][1][s], acc[1][0][s], acc[1][1][s]}), rs,
                                                   ok ? base + (int)(s * P.lsz[0] * 4) : SOOB, 0, ST_SC1);
    };
"""
PATCHES["spread"] = PATCHES["noepi"] + [
    ("build.hip", "    Frags fa, fb;\n", SPREAD_SLOT + "    Frags fa, fb;\n"),
    ("build.hip", "        wait_vm<SCOPIES, true>();", "        wait_vm<SCOPIES + 8, true>();"),
    ("build.hip", "        advance(kc + 1);\n        read_lo(kc + 1, fb);", "        advance(kc + 1);\n        spread_slot(kc);\n        read_lo(kc + 1, fb);"),
    ("build.hip", "        advance(kc + 2);\n        read_lo(kc + 2, fa);", "        advance(kc + 2);\n        spread_slot(kc + 1);\n        read_lo(kc + 2, fa);"),
]
PATCHES["burst"] = PATCHES["noepi"] + [
    ("build.hip", "    Frags fa, fb;\n", SPREAD_SLOT + "    Frags fa, fb;\n"),
    ("build.hip", EPI, "#pragma unroll\n    for (int z = 0; z < 8; ++z) spread_slot(z);\n" + EPI),
]
# epilogue pieces: level 0 only (scaling + LDS line transposes + stores); no level-2/3 pixel stores
PATCHES["l0only"] = [("build.hip", "    const int L = P.fused_levels;\n    const int64_t rows0", "    const int L = 1;\n    const int64_t rows0")]
PATCHES["nol23"] = [("build.hip", "        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(val), rs, in ? off : SOOB, 0, 0);",
                     "        asm volatile(\"\" :: \"v\"(val), \"v\"(in ? off : SOOB));")]
# per-block timestamps: [start, K loop done, epilogue done] (s_memrealtime, 100 MHz) + HW_ID + XCC_ID,
# read back with ecorr_lab_stamps(host_ptr, n) (tools/stamps.py)
STAMP_DECL = """
__device__ unsigned long long g_stamps[65536][5];
__device__ __forceinline__ void stamp(int k) {
    if (threadIdx.x == 0 && blockIdx.x < 65536) {
        g_stamps[blockIdx.x][k] = __builtin_amdgcn_s_memrealtime();
        if (k == 0) g_stamps[blockIdx.x][4] = ((unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4) << 32) |
                                             (unsigned long long)__builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20);
    }
}
"""
STAMP_EXPORT = """
extern "C" __attribute__((visibility("default"))) int ecorr_lab_stamps(void* dst, int n) {
    return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(ecorr::g_stamps), (size_t)n * 40, 0, hipMemcpyDeviceToHost);
}
"""
PATCHES["stamps"] = [
    ("build.hip", "constexpr int SQ = 256; ", STAMP_DECL + "constexpr int SQ = 256; "),
    ("build.hip", "    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;\n    const int acol", "    stamp(0);\n    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;\n    const int acol"),
    ("build.hip", "    __builtin_amdgcn_s_barrier();   // ... in every wave: the chunk buffers are the epilogue's scratch\n",
     "    __builtin_amdgcn_s_barrier();   // ... in every wave: the chunk buffers are the epilogue's scratch\n    stamp(1);\n"),
    ("build.hip", "                    r1t < P.lnty[1] && c1t < P.lntx[1]);\n    }\n}\n",
     "                    r1t < P.lnty[1] && c1t < P.lntx[1]);\n    }\n    __builtin_amdgcn_s_barrier();\n    stamp(3);\n    __syncthreads();\n    stamp(2);\n}\n"),
    ("build.hip", "}  // namespace ecorr\n", "}  // namespace ecorr\n" + STAMP_EXPORT),
]
# inside the K loop (wave 0 lane 0 and wave 3): cycles spent in the DMA wait, in the barrier, and
# in total, summed over the chunks (s_memtime) -> g_stamps[block] = {wait, barrier, total, wave-3 wait}
PATCHES["loopstamps"] = [
    ("build.hip", "constexpr int SQ = 256; ", STAMP_DECL + "__device__ unsigned long long g_lw, g_lb;\nconstexpr int SQ = 256; "),
    ("build.hip", """    auto advance = [&](int j) {
        PHASE;
        wait_vm<SCOPIES + QLOADS, true>();
        __builtin_amdgcn_s_barrier();""", """    auto advance = [&](int j) {
        PHASE;
        const unsigned long long ta = __builtin_amdgcn_s_memtime();
        wait_vm<SCOPIES + QLOADS, true>();
        const unsigned long long tb = __builtin_amdgcn_s_memtime();
        __builtin_amdgcn_s_barrier();
        const unsigned long long tcb = __builtin_amdgcn_s_memtime();
        sw += tb - ta; sb += tcb - tb;"""),
    ("build.hip", "    TFrags fa, fb;\n", "    const unsigned long long tl0 = __builtin_amdgcn_s_memtime(), tr0 = __builtin_amdgcn_s_memrealtime();\n    TFrags fa, fb;\n"),
    ("build.hip", "    // VMEM issue order per wave:", "    unsigned long long sw = 0, sb = 0;\n    // VMEM issue order per wave:"),
    ("build.hip", "    wait_vm<0, true>();             // the trailing zero chunks have landed and this wave's reads are done ...\n",
     "    wait_vm<0, true>();             // the trailing zero chunks have landed and this wave's reads are done ...\n"
     "    if (lane == 0 && blockIdx.x < 65536) { if (wave == 0) { g_stamps[blockIdx.x][0] = sw; g_stamps[blockIdx.x][1] = sb; "
     "g_stamps[blockIdx.x][2] = __builtin_amdgcn_s_memtime() - tl0; } g_stamps[blockIdx.x][3] = __builtin_amdgcn_s_memrealtime() - tr0; }\n"),
    ("build.hip", "}  // namespace ecorr\n", "}  // namespace ecorr\n" + STAMP_EXPORT),
]
# epilogue stores issued with out-of-range offsets (TA work, no memory traffic) / not issued at all
PATCHES["epioob"] = [("build.hip", "                                                   ok ? base + (int)(s * lsz * 4) : SOOB, 0, ST_SC1);",
                      "                                                   SOOB, 0, ST_SC1);"),
                     ("build.hip", "        const int off = (int)((qloc * P.lsz[lv] + level_off(r, c, P.lntx[lv], P.lw[lv])) * 4);",
                      "        const int off = SOOB; (void)qloc;")]
PATCHES["epinost"] = [("build.hip", """            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(uint4v, pc[s]), rs,
                                                   ok ? base + (int)(s * lsz * 4) : SOOB, 0, ST_SC1);""",
                       """            asm volatile("" :: "v"(pc[s]), "v"(ok ? base + (int)(s * lsz * 4) : SOOB));"""),
                      ("build.hip", "    auto store_px = [&](__amdgpu_buffer_rsrc_t rs, int lv, int qloc, int r, int c, auto val) {",
                       "    auto store_px = [&](__amdgpu_buffer_rsrc_t rs, int lv, int qloc, int r, int c, auto val) {\n        asm volatile(\"\" :: \"v\"(val), \"v\"(qloc + r + c)); return;")]
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
# lookup ablations (timing only): no window loads / no output stores / no blends (one LDS read)
PATCHES["lk_nostage"] = [("lookup_stage.h", "            vals[c][ry] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsrc, need ? off : OOB, 0, 0));",
                          "            vals[c][ry] = (float)(need ? off : 0);")]
PATCHES["lk_nostore"] = [("lookup.hip", """                const float v = blend(c[0], c[1], c[SW], c[SW + 1], wx[ai], wy[bb]);
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), orsrc, voff,
                                                      sbase + (a * K + bb) * P.q_count * 4, 2);""",
                          """                const float v = blend(c[0], c[1], c[SW], c[SW + 1], wx[ai], wy[bb]);
                asm volatile("" :: "v"(v), "v"(sbase + (a * K + bb) * P.q_count * 4));""")]
PATCHES["lk_noblend"] = [("lookup.hip", "                const float v = blend(c[0], c[1], c[SW], c[SW + 1], wx[ai], wy[bb]);",
                          "                const float v = c[0];")]
# lookup: every staging load issued twice (same bytes, 2x the lane requests): is staging bound by
# the per-lane request rate?
PATCHES["lk_dbl"] = [("lookup_stage.h", "            vals[c][ry] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsrc, need ? off : OOB, 0, 0));",
                      "            vals[c][ry] = __builtin_fmaf(0.0f, __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsrc, need ? off : OOB, 0, 1)), __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsrc, need ? off : OOB, 0, 0)));")]
# lookup: output stores as 2 x dwordx4 + 1 dword per column (same bytes, 3 store instructions
# instead of 9; wrong layout -- timing only): does the store request count bound the lookup?
PATCHES["lk_st4"] = [("lookup.hip", """#pragma unroll
            for (int bb = 0; bb < K; ++bb) {
                const float* c = wc + yo[bb];
                const float v = blend(c[0], c[1], c[S], c[S + 1], wx[ai], wy[bb]);
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), orsrc, voff,
                                                      sbase + (a * K + bb) * P.q_count * 4, 2);
            }""", """            float vv[K];
#pragma unroll
            for (int bb = 0; bb < K; ++bb) {
                const float* c = wc + yo[bb];
                vv[bb] = blend(c[0], c[1], c[S], c[S + 1], wx[ai], wy[bb]);
            }
            if constexpr (K == 9) {
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, floatx4_t{vv[0], vv[1], vv[2], vv[3]}), orsrc, voff * 4, sbase + (a * K) * P.q_count * 4, 2);
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, floatx4_t{vv[4], vv[5], vv[6], vv[7]}), orsrc, voff * 4, sbase + (a * K + 4) * P.q_count * 4, 2);
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(vv[8]), orsrc, voff, sbase + (a * K + 8) * P.q_count * 4, 2);
            }"""),
                     ("lookup.hip", "constexpr int NT = 256;   // threads of the generic kernels",
                      "constexpr int NT = 256;   // threads of the generic kernels\ntypedef float floatx4_t __attribute__((ext_vector_type(4)));")]
# tile order: m-tiles per group of the grouped order (tree: 8)
for _gm in (2, 3, 4, 6):
    PATCHES[f"gm{_gm}"] = [("build.hip", "    constexpr int GM = 8;", f"    constexpr int GM = {_gm};")]
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
# lookup: unneeded window elements skipped by exec mask instead of an out-of-range offset
PATCHES["lk_exec"] = [("lookup_stage.h", "            vals[c][ry] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsrc, need ? off : OOB, 0, 0));",
                       "            vals[c][ry] = need ? __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsrc, off, 0, 0)) : 0.0f;")]
# epilogue ablations (timing only): no scaling (raw accumulators), no LDS transposes (the
# read-back replaced by the lane's own registers)
PATCHES["epi_noscale"] = [("build.hip", "const float x = __fmul_rn(acc[i][j][4 * g4 + t], __fmul_rn(sq, s4[t]));",
                           "const float x = acc[i][j][4 * g4 + t]; (void)s4; (void)sq;")]
PATCHES["epi_nolds"] = [("build.hip", "        for (int s = 0; s < 4; ++s) pc[s] = *reinterpret_cast<const floatx4*>(xp + ro + s * XS);",
                         "        for (int s = 0; s < 4; ++s) pc[s] = floatx4{(float)(ro + s), (float)ql, (float)lo, 1.0f};"),
                        ("build.hip", """                    *reinterpret_cast<floatx4*>(xp + wo + 32 * g4 + 16 * arow) =
                        floatx4{v[jl][g4][0], v[jl][g4][1], v[jl][g4][2], v[jl][g4][3]};""",
                         """                    asm volatile("" :: "v"(floatx4{v[jl][g4][0], v[jl][g4][1], v[jl][g4][2], v[jl][g4][3]}));""")]
# on top of loopstamps: the wait for the chunk's query fragments made explicit and timed before
# each lo*hi MFMA group (g_stamps[block][4] = wave 0's cycles in those waits)
PATCHES["qwait"] = [("build.hip", "        mfma_lohi(fa, qa);", "        { const unsigned long long t0 = __builtin_amdgcn_s_memtime(); wait_vm<6, false>(); sq += __builtin_amdgcn_s_memtime() - t0; }\n        mfma_lohi(fa, qa);"),
                    ("build.hip", "        mfma_lohi(fb, qb);", "        { const unsigned long long t0 = __builtin_amdgcn_s_memtime(); wait_vm<6, false>(); sq += __builtin_amdgcn_s_memtime() - t0; }\n        mfma_lohi(fb, qb);"),
                    ("build.hip", "    unsigned long long sw = 0, sb = 0;", "    unsigned long long sw = 0, sb = 0, sq = 0;"),
                    ("build.hip", "g_stamps[blockIdx.x][3] = __builtin_amdgcn_s_memrealtime() - tr0; }", "g_stamps[blockIdx.x][3] = __builtin_amdgcn_s_memrealtime() - tr0; if (wave == 0) g_stamps[blockIdx.x][4] = sq; }")]
# stamps for the S16 loop (stamp 1 after split_loop16; build.hip with tools/lab_patches/s16_loop.diff applied)
PATCHES["stamps16"] = [x for x in PATCHES["stamps"] if "chunk buffers are the epilogue" not in x[1]] + [
    ("build.hip", "        split_loop16(P, smem, rq, rt, pstride, wave, lane, acc);\n",
     "        split_loop16(P, smem, rq, rt, pstride, wave, lane, acc);\n        stamp(1);\n")]
# in-loop clock and wait/barrier cycles of the S16 loop -> g_stamps[block] = {wait, barrier, total, realtime}
PATCHES["loopstamps16"] = [
    ("build.hip", "constexpr int SQ = 256; ", STAMP_DECL + "constexpr int SQ = 256; "),
    ("build.hip", """    QH qa, qb;
    issue(0);""", """    QH qa, qb;
    unsigned long long sw = 0, sb = 0;
    const unsigned long long tl0 = __builtin_amdgcn_s_memtime(), tr0 = __builtin_amdgcn_s_memrealtime();
    issue(0);"""),
    ("build.hip", """        if (step == 0) wait_vm<6, true>();
        else wait_vm<12, true>();
        __builtin_amdgcn_s_barrier();""", """        const unsigned long long ta = __builtin_amdgcn_s_memtime();
        if (step == 0) wait_vm<6, true>();
        else wait_vm<12, true>();
        const unsigned long long tb = __builtin_amdgcn_s_memtime();
        __builtin_amdgcn_s_barrier();
        sw += tb - ta; sb += __builtin_amdgcn_s_memtime() - tb;"""),
    ("build.hip", """#undef PHASE
    wait_vm<0, true>();
    __builtin_amdgcn_s_barrier();   // every wave is done with the ring""", """#undef PHASE
    wait_vm<0, true>();
    if (lane == 0 && wave == 0 && blockIdx.x < 65536) { g_stamps[blockIdx.x][0] = sw; g_stamps[blockIdx.x][1] = sb;
        g_stamps[blockIdx.x][2] = __builtin_amdgcn_s_memtime() - tl0; g_stamps[blockIdx.x][3] = __builtin_amdgcn_s_memrealtime() - tr0; }
    __builtin_amdgcn_s_barrier();   // every wave is done with the ring"""),
    ("build.hip", "}  // namespace ecorr\n", "}  // namespace ecorr\n" + STAMP_EXPORT),
]
# round-3 per-block stamps of the split build: [start, K loop done, epilogue done, prologue done
# (first barrier: exponents in LDS, t(0) landed), HW_ID | XCC_ID] -> tools/stamps.py --prologue
PATCHES["stamps4"] = [
    ("build.hip", "constexpr int SQ = 256; ", STAMP_DECL + "constexpr int SQ = 256; "),
    ("build.hip", "    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;\n    int b, qt, nt;\n    decode_tile(P, xcd_remap(blockIdx.x, gridDim.x), P.n_qt, b, qt, nt);\n    const NTile tc = ntile_of(P, nt);\n    const int q0 = qt * SQ;\n    const int H = P.H, W = P.W;\n    const int64_t Q = (int64_t)H * W;\n\n    {   // per-pixel",
     "    stamp(0);\n    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;\n    int b, qt, nt;\n    decode_tile(P, xcd_remap(blockIdx.x, gridDim.x), P.n_qt, b, qt, nt);\n    const NTile tc = ntile_of(P, nt);\n    const int q0 = qt * SQ;\n    const int H = P.H, W = P.W;\n    const int64_t Q = (int64_t)H * W;\n\n    {   // per-pixel"),
    ("build.hip", "        wait_vm_n<true>(split_vm_after(0, NK));   // t(0) landed\n        __builtin_amdgcn_s_barrier();\n",
     "        wait_vm_n<true>(split_vm_after(0, NK));   // t(0) landed\n        __builtin_amdgcn_s_barrier();\n        stamp(3);\n"),
    ("build.hip", "    __builtin_amdgcn_s_barrier();   // ... in every wave: the chunk buffers are the epilogue's scratch\n",
     "    __builtin_amdgcn_s_barrier();   // ... in every wave: the chunk buffers are the epilogue's scratch\n    stamp(1);\n"),
    ("build.hip", "    split_epilogue<MUL>(P, acc, smem + wave * (4 * 32 * XS), wave * 64, exq, ext, fst, tc, b, q0, lane);\n}\n\n// ====",
     "    split_epilogue<MUL>(P, acc, smem + wave * (4 * 32 * XS), wave * 64, exq, ext, fst, tc, b, q0, lane);\n    __syncthreads();\n    stamp(2);\n}\n\n// ===="),
    ("build.hip", "}  // namespace ecorr\n", "}  // namespace ecorr\n" + STAMP_EXPORT),
]
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
    decode_tile(P, xcd_remap(blockIdx.x, gridDim.x), P.n_qt, b, qt, nt);
    const NTile tc = ntile_of(P, nt);
    const int q0 = qt * SQ;
    const int H = P.H, W = P.W;
    const int64_t Q = (int64_t)H * W;

    // per-pixel exponents: loaded behind the K loop's last static wait (only the epilogue reads them)""",
     """    const unsigned long long r_start = __builtin_amdgcn_s_memrealtime();
    unsigned long long c_mid = 0;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    int b, qt, nt;
    decode_tile(P, xcd_remap(blockIdx.x, gridDim.x), P.n_qt, b, qt, nt);
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
# split16 epilogue stores issued out of range (timing only: same instructions, no store traffic)
PATCHES["e16oob"] = [("build.hip", "lok && qloc < nq ? (int)(qloc * P.lsz[0] * 4) + loff : SOOB, 0,", "SOOB, 0,"),
                     ("build.hip", "        const bool in = on && qloc < nq && by < P.lnty[lv] && bx < -P.lntx[lv];",
                      "        const bool in = false && on && qloc < nq && by < P.lnty[lv] && bx < -P.lntx[lv];")]
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
# split16 epilogue without its level-0 LDS transpose (timing only: each lane stores its own
# values as the pieces): does the transpose's LDS traffic slow the partner block's K loop?
PATCHES["e16nolds"] = [("build.hip", """#pragma unroll
        for (int tg = 0; tg < 8; ++tg)
            *reinterpret_cast<floatx4*>(xr + lane * S16LS + 16 * tg) = floatx4{v[tg][0], v[tg][1], v[tg][2], v[tg][3]};
#pragma unroll
        for (int s = 0; s < 8; ++s)
            st4(r0, l0off + (16 * qg + s) * l0stride, l0ok && l0q + 16 * qg + s < nq,
                *reinterpret_cast<const floatx4*>(xr + (s + 8 * jl) * S16LS + 16 * pc));""", """        (void)xr;
#pragma unroll
        for (int s = 0; s < 8; ++s)
            st4(r0, l0off + (16 * qg + s) * l0stride, l0ok && l0q + 16 * qg + s < nq,
                floatx4{v[s][0], v[s][1], v[s][2], v[s][3]});""")]
# split16 K loop alone (timing only): the epilogue replaced by one store of the accumulator sum;
# and the same with one block per CU (LDS padded past half the CU), i.e. one wave per SIMD
PATCHES["noepi16"] = [("build.hip", """    split16_epilogue<MUL>(P, acc, smem + wave * (2 * 64 * S16LS), wave * 64, exq, ext, fst, tc, b, q0, lane);
}""", """    {
        float sacc = 0.f;
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
            for (int t = 0; t < 8; ++t)
#pragma unroll
                for (int r = 0; r < 4; ++r) sacc += acc[g][t][r];
        P.lvl[0][(int64_t)blockIdx.x * 256 + tid] = sacc;
    }
}""")]
PATCHES["onecu16"] = [("build.hip", """__global__ __launch_bounds__(256, 2) void build_split16_kernel(BuildParams P) {
    // ALL LDS in this one array (cdna_hip_programming.md trap 4(a), see build_split_kernel)
    __shared__ __attribute__((aligned(16))) char smem[SLDS + (SQ + 256) * 4];""", """__global__ __launch_bounds__(256, 1) void build_split16_kernel(BuildParams P) {
    // ALL LDS in this one array (cdna_hip_programming.md trap 4(a), see build_split_kernel)
    __shared__ __attribute__((aligned(16))) char smem[SLDS + (SQ + 256) * 4 + 16384];""")]
# (round 3: split16 level-0 lines stored straight from their lanes, no LDS transpose -- the source
# option is gone: 4.8 ms and 5.4 GB written, profiles/r03_lab/r3h_*)
# the query-stationary persistent build (build_qs_kernel) in place of build_split16_kernel
PATCHES["qs"] = [("build.hip", "constexpr bool kBuildQS = false;", "constexpr bool kBuildQS = true;")]
# QS with the two half-panel LDS buffers swapped (does LDS-DMA reach beyond 64 KB?)
# QS debug: the previous half's epilogue after this half's MFMAs instead of interleaved
PATCHES["qsseq"] = PATCHES["qs"] + [
    ("build.hip", """            if constexpr (EPI) epi_step(AE, kc);
            __builtin_amdgcn_sched_barrier(0);
        });
""", """            __builtin_amdgcn_sched_barrier(0);
        });
        if constexpr (EPI) {
            asm volatile("s_nop 15");
            asm volatile("s_nop 15");
            qs_static_for<NCP * 16>([&](auto kc) QS_INLINE {
                epi_step(AE, kc);
                __builtin_amdgcn_sched_barrier(0);
            });
        }
""")]
# QS timing probes (wrong results): MFMAs and panel transfers only / epilogue and transfers only
PATCHES["qsnoepi"] = PATCHES["qs"] + [
    ("build.hip", "            if constexpr (EPI) epi_step(AE, kc);\n", ""),
    ("build.hip", "        if constexpr (EPI) flush();\n", ""),
]
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
PATCHES["qspre"] = PATCHES["qs"] + [
    ("build.hip", "        if constexpr (EPI) epi_begin();\n        AF af[2];",
     "        if constexpr (EPI) {\n            epi_begin();\n            qs_static_for<NCP * 16>([&](auto kc) QS_INLINE {\n"
     "                epi_step(AE, kc);\n                __builtin_amdgcn_sched_barrier(0);\n            });\n            flush();\n        }\n        AF af[2];"),
    ("build.hip", "            if constexpr (EPI) epi_step(AE, kc);\n", ""),
    ("build.hip", "        if constexpr (EPI) flush();\n", ""),
]
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
for _pol in (0, 16, 18):
    PATCHES[f"lkst{_pol}"] = [("lookup.hip", "sbase + (a * K + bb) * P.q_count * 4, 2);",
                               f"sbase + (a * K + bb) * P.q_count * 4, {_pol});")]
# the tree as it is (the baseline of an A/B against an edited tree)
PATCHES["base"] = []
# lookup windows staged one column per work item (b32 loads) instead of 8-byte column pairs
PATCHES["nopair"] = [("lookup.hip", "        bool pair = true;", "        bool pair = false;")]
# timing only: no window loads for one level (what does each level's staging cost?)
for _lv in range(4):
    PATCHES[f"lk_skip{_lv}"] = [("lookup_stage.h", "            const bool need = (unsigned)(ry - rlo) < (unsigned)(rhi - rlo);",
                                 f"            const bool need = lv != {_lv} && (unsigned)(ry - rlo) < (unsigned)(rhi - rlo);")]
# lookup wave priority: raised while the window loads issue (phase 1) / while the outputs store
PATCHES["lk_prio1"] = [("lookup_stage.h", "    float vals[NCOL][S][V];\n    int dst[NCOL];\n",
                        "    float vals[NCOL][S][V];\n    int dst[NCOL];\n    __builtin_amdgcn_s_setprio(2);\n"),
                       ("lookup_stage.h", "                for (int v = 0; v < V; ++v) st.win[dst[c] + ry * SW + v] = vals[c][ry][v];\n    __syncthreads();\n}",
                        "                for (int v = 0; v < V; ++v) st.win[dst[c] + ry * SW + v] = vals[c][ry][v];\n    __builtin_amdgcn_s_setprio(0);\n    __syncthreads();\n}")]
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
# round-2 store ablations on the current epilogue (timing only): level-2/3 pixel stores issued out
# of range / as non-temporal stores; level-0/1 line stores out of range
_L23 = ["__builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(uint4v, val), rs, in ? off : SOOB, 0, 0);",
        "__builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(uint2v, val), rs, in ? off : SOOB, 0, 0);"]
PATCHES["l23oob"] = [("build.hip", s, s.replace("in ? off : SOOB", "in ? SOOB : SOOB")) for s in _L23]
PATCHES["l23nt"] = [("build.hip", s, s.replace(", 0, 0);", ", 0, 2);")) for s in _L23]
PATCHES["l01oob"] = [("build.hip", "ok ? base + (int)(s * lsz * 4) : SOOB, 0, ST_L01);", "ok ? SOOB : SOOB, 0, ST_L01);")]
# round-2 K-loop ablations (timing only): no per-chunk barrier; the target-panel DMA / the query
# fragment loads issued out of range (same instructions and wait counts, no memory traffic)
PATCHES["nobar"] = [("build.hip", "            else wait_vm<SCOPIES, true>();\n            __builtin_amdgcn_s_barrier();",
                     "            else wait_vm<SCOPIES, true>();")]
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
COMBOS = {"loopstamps_epioob": ["loopstamps", "epioob"], "stamps_loopprio": ["stamps", "loopprio"], "stamps_stagger2": ["stamps", "stagger2"], "loopstamps_noepi": ["loopstamps", "noepi"], "loopstamps_noqdma": ["loopstamps", "noqdma"], "stamps_noqdma": ["noqdma", "stamps"], "stamps_prio": ["stamps", "prio"], "stamps_epioob": ["stamps", "epioob"], "stamps_epinost": ["stamps", "epinost"]}
COMBOS.update({"loopstamps_qwait": ["loopstamps", "qwait"]})
COMBOS.update({"stamps_epi_noscale": ["stamps", "epi_noscale"], "stamps_epi_nolds": ["stamps", "epi_nolds"]})
COMBOS.update({"sameqt": ["sameq", "samet"]})
COMBOS.update({"dmaqoob": ["dmaoob", "qoob"], "noepi_r2": ["noepi"]})
COMBOS.update({"noepi16_1cu": ["noepi16", "onecu16"]})
COMBOS.update({"st16_e16oob": ["st16", "e16oob"], "st16_e16nolds": ["st16", "e16nolds"], "st16_prio_loop": ["st16", "prio_loop"]})
COMBOS.update({"noepi_mfma16": ["noepi", "mfma16"], "loopstamps_noepi_mfma16": ["loopstamps", "noepi", "mfma16"]})
COMBOS.update({"st16_sscale": ["st16", "sscale"], "st16_noscale": ["st16", "noscale"]})

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

# ---- round 4: per-workgroup timeline of the lookup (lookup_cols_reg): s_memrealtime stamps at the
# start, after the origin barrier, after the staging barrier, and each wave's end after its own
# stores retired (vmcnt(0)); + HW_ID / XCC_ID.  Timing diagnosis only (tools/lkstamps.py).
LK_DECL = """
__device__ unsigned long long g_lk[262144][8];
"""
LK_EXPORT = """
extern "C" __attribute__((visibility("default"))) int ecorr_lab_lkstamps(void* dst, int n) {
    return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(ecorr::g_lk), (size_t)n * 64, 0, hipMemcpyDeviceToHost);
}
"""
PATCHES["lkstamps"] = [
    ("lookup.hip", "constexpr int NT = 256;   // threads of the generic kernels", "constexpr int NT = 256;   // threads of the generic kernels" + LK_DECL),
    ("lookup.hip", """    __shared__ WB st;
    const int tid = threadIdx.x, g = tid % QB;""", """    __shared__ WB st;
    const unsigned long long lk_t0 = __builtin_amdgcn_s_memrealtime();
    const int lk_id = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    const int tid = threadIdx.x, g = tid % QB;"""),
    ("lookup.hip", """    __syncthreads();
    stage_windows<R, QB, NTQ, PAIR>(st, P, lv, b, q0, tid);
""", """    __syncthreads();
    const unsigned long long lk_t1 = __builtin_amdgcn_s_memrealtime();
    stage_windows<R, QB, NTQ, PAIR>(st, P, lv, b, q0, tid);
    const unsigned long long lk_t2 = __builtin_amdgcn_s_memrealtime();
    if (tid == 0 && lk_id < 262144) {
        g_lk[lk_id][0] = lk_t0;
        g_lk[lk_id][1] = lk_t1;
        g_lk[lk_id][2] = lk_t2;
        g_lk[lk_id][6] = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);
        g_lk[lk_id][7] = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20);
    }
"""),
    ("lookup.hip", """                                                      sbase + ((part * AP + ai) * K + bb) * P.q_count * 4, 2);
            }
    }
}""", """                                                      sbase + ((part * AP + ai) * K + bb) * P.q_count * 4, 2);
            }
    }
    __builtin_amdgcn_s_waitcnt(0);
    if (g == 0 && lk_id < 262144) g_lk[lk_id][3 + part] = __builtin_amdgcn_s_memrealtime();
}"""),
    ("lookup.hip", "}  // namespace ecorr\n", "}  // namespace ecorr\n" + LK_EXPORT),
]

# ---- round 4: lookup with only the window end-point chains before the staging loads; the other
# chains (7 y, 3 x per thread) computed while those loads are in flight (bitwise the same)
PATCHES["lk_late"] = [("lookup.hip", """    float fy[K], wy[K], fx[AP], wx[AP], x0 = 0.0f, xl = 0.0f;
    if (valid) {
        const int64_t Q = P.q_count;
        const float inv = 1.0f / (float)(1 << lv);  // coords / 2**i is an exact scaling
        const float cx = __fmul_rn(P.coords[((int64_t)b * 2 + 0) * Q + p], inv);
        const float cy = __fmul_rn(P.coords[((int64_t)b * 2 + 1) * Q + p], inv);
        const float wm1 = (float)(P.lw[lv] - 1), hm1 = (float)(P.lh[lv] - 1);
#pragma unroll
        for (int bb = 0; bb < K; ++bb) coord_chain<R>(cy, bb, hm1, fy[bb], wy[bb]);
#pragma unroll
        for (int ai = 0; ai < AP; ++ai) coord_chain<R>(cx, part * AP + ai, wm1, fx[ai], wx[ai]);
        float dummy;
        coord_chain<R>(cx, 0, wm1, x0, dummy);
        coord_chain<R>(cx, K - 1, wm1, xl, dummy);
    }""", """    float fy[K], wy[K], fx[AP], wx[AP], x0 = 0.0f, xl = 0.0f;
    float cx = 0.0f, cy = 0.0f;
    const float wm1 = (float)(P.lw[lv] - 1), hm1 = (float)(P.lh[lv] - 1);
    if (valid) {
        const int64_t Q = P.q_count;
        const float inv = 1.0f / (float)(1 << lv);  // coords / 2**i is an exact scaling
        cx = __fmul_rn(P.coords[((int64_t)b * 2 + 0) * Q + p], inv);
        cy = __fmul_rn(P.coords[((int64_t)b * 2 + 1) * Q + p], inv);
        coord_chain<R>(cy, 0, hm1, fy[0], wy[0]);
        coord_chain<R>(cy, K - 1, hm1, fy[K - 1], wy[K - 1]);
        float dummy;
        coord_chain<R>(cx, 0, wm1, x0, dummy);
        coord_chain<R>(cx, K - 1, wm1, xl, dummy);
    }"""),
    ("lookup.hip", """    __syncthreads();
    stage_windows<R, QB, NTQ, PAIR>(st, P, lv, b, q0, tid);
""", """    __syncthreads();
    {
        StageRegs<R, QB, NTQ, PAIR> sr;
        stage_issue<R, QB, NTQ, PAIR>(st, P, lv, b, q0, tid, sr);
        if (valid) {   // the remaining chains under the staging loads' latency
#pragma unroll
            for (int bb = 1; bb < K - 1; ++bb) coord_chain<R>(cy, bb, hm1, fy[bb], wy[bb]);
#pragma unroll
            for (int ai = 0; ai < AP; ++ai) coord_chain<R>(cx, part * AP + ai, wm1, fx[ai], wx[ai]);
        }
        stage_commit<R, QB, NTQ, PAIR>(st, sr);
        __syncthreads();
    }
""")]

# ---- round 4: lookup staging with lanes = (query, column pair, row group): a task is one column
# pair of one query's window at rows rg, rg + 4, rg + 8 (rg = lane & 3), so the 64 lanes of a load
# instruction cover 16 (query, pair) items x 4 consecutive rows -- about 9-10 distinct 128-B lines
# per instruction instead of ~21 (one row of ~11 queries' windows) -- and every row step is one
# constant offset (+4 rows: one tile row / two or four block rows).  Bitwise the same.
LK_RG_FN = """
// lab: task-per-(query, pair, row group) staging, PAIR only (see tools/lab_build.py lk_rg)
template <int R, int QB, int NTQ>
struct StageRegsRG {
    static constexpr int S = 2 * R + 3, NPX = (S + 1) / 2, TASKS = QB * NPX * 4;
    static constexpr int NT = (TASKS + NTQ - 1) / NTQ, NR = (S + 3) / 4;
    float vals[NT][NR][2];
    int dst[NT];    // LDS slot of row rg of the task's pair (-1: no task)
    int skip[NT];   // the pair half (0 / 1) outside the S-slot row, else -1
};

template <int R, int QB, int NTQ>
__device__ __forceinline__ void stage_issue_rg(const WindowBuf<R, QB, true>& st, const LookupParams& P, int lv, int b,
                                               int q0, int tid, StageRegsRG<R, QB, NTQ>& sr) {
    using WS = WindowBuf<R, QB, true>;
    using SR = StageRegsRG<R, QB, NTQ>;
    constexpr int S = WS::S, SP = WS::SP, SW = WS::SW, NPX = SR::NPX;
    static_assert(NTQ % 4 == 0 && (NTQ / 4) % NPX == 0, "rg and pair fixed per thread");
    const int h = P.lh[lv], w = P.lw[lv], ntx = P.lntx[lv];
    const int64_t hw = P.lsz[lv];
    const int64_t R0 = (int64_t)b * P.q_count + q0;
    const int64_t g0 = R0 >> 6;
    const float* __restrict__ lvbase = P.lvl[lv] + (ntx < 0 ? g0 * kGroup * hw : R0 * hw);
    const int nq = min(QB, P.q_count - q0);
    const int64_t span = ntx < 0 ? (((R0 + nq - 1) >> 6) - g0 + 1) * kGroup * hw : nq * hw;
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(lvbase), 0, (int)(span * 4), 0x00020000);
    const bool tiled = ntx > 0, ilv = ntx < 0;
    const int sy = ilv ? ilv_sy(lv) : 2, sx = ilv ? ilv_sx(lv) : 3;
    const int ymask = tiled || ilv ? (1 << sy) - 1 : 0;
    const int step4 = tiled ? 128 * ntx : ilv ? (4 >> sy) * -ntx * kGroup * (1 << (sy + sx)) * 4 : 16 * w;
    constexpr int OOB = 0x7ffffff0;
    const int rg = tid & 3, px = (tid >> 2) % NPX, gq0 = (tid >> 2) / NPX;
    constexpr int DQ = NTQ / 4 / NPX;   // queries between a thread's tasks
#pragma unroll
    for (int c = 0; c < SR::NT; ++c) {
        const int gq = gq0 + DQ * c;
        const bool live = gq < QB;
        const int gqs = live ? gq : 0;
        const int xo = st.org[gqs][0], y0 = st.org[gqs][1], info = st.org[gqs][2];
        const int odd = xo & 1;
        const int x = xo - odd + 2 * px;
        const int ny = (info >> 16) & 0xff;
        const bool colin = live && (info & 0xff) == 0 && 2 * px < ((info >> 8) & 0xff) + odd && (unsigned)x < (unsigned)w;
        sr.dst[c] = live ? WS::W0 + gq * SP + rg * SW + 2 * px - odd : -1;
        sr.skip[c] = odd && px == 0 ? 0 : !odd && 2 * px == S - 1 ? 1 : -1;
        const int rlo = max(0, -y0), rhi = colin ? max(rlo, min(ny, h - y0)) : rlo;
        const int y = y0 + rg;
        int off;
        if (tiled) {
            off = (int)(gqs * hw) * 4 + ((((y >> 2) * ntx + (x >> 3)) << 5) + ((y & 3) << 3) + (x & 7)) * 4;
        } else if (ilv) {
            const int64_t Rq = R0 + gqs;
            off = (int)((((Rq >> 6) - g0) * kGroup * hw +
                         ((int64_t)((y >> sy) * -ntx + (x >> sx)) * kGroup + (Rq & (kGroup - 1))) * (1 << (sy + sx)) +
                         ((y & ymask) << sx) + (x & ((1 << sx) - 1))) * 4);
        } else {
            off = (int)(gqs * hw) * 4 + (y * w + x) * 4;
        }
#pragma unroll
        for (int j = 0; j < SR::NR; ++j) {
            const int ry = rg + 4 * j;
            const bool need = ry < S && (unsigned)(ry - rlo) < (unsigned)(rhi - rlo);
            const uint2v u = __builtin_amdgcn_raw_buffer_load_b64(rsrc, need ? off : OOB, 0, 0);
            sr.vals[c][j][0] = __uint_as_float(u.x);
            sr.vals[c][j][1] = __uint_as_float(u.y);
            off += step4;
        }
    }
}

template <int R, int QB, int NTQ>
__device__ __forceinline__ void stage_commit_rg(WindowBuf<R, QB, true>& st, const StageRegsRG<R, QB, NTQ>& sr, int tid) {
    using SR = StageRegsRG<R, QB, NTQ>;
    constexpr int SW = WindowBuf<R, QB, true>::SW, DUMMY = WindowBuf<R, QB, true>::DUMMY, S = SR::S;
    const int rg = tid & 3;
#pragma unroll
    for (int c = 0; c < SR::NT; ++c)
        if (sr.dst[c] >= 0)
#pragma unroll
            for (int j = 0; j < SR::NR; ++j)
                if (rg + 4 * j < S)
#pragma unroll
                    for (int v = 0; v < 2; ++v)
                        st.win[sr.skip[c] == v ? DUMMY : sr.dst[c] + 4 * j * SW + v] = sr.vals[c][j][v];
}
"""
PATCHES["lk_rg"] = [
    ("lookup_stage.h", "// Exact direct gather of one sample of query p", LK_RG_FN + "\n// Exact direct gather of one sample of query p"),
    ("lookup.hip", """    __syncthreads();
    stage_windows<R, QB, NTQ, PAIR>(st, P, lv, b, q0, tid);
""", """    __syncthreads();
    if constexpr (PAIR) {
        StageRegsRG<R, QB, NTQ> sr;
        stage_issue_rg<R, QB, NTQ>(st, P, lv, b, q0, tid, sr);
        stage_commit_rg<R, QB, NTQ>(st, sr, tid);
        __syncthreads();
    } else {
        stage_windows<R, QB, NTQ, PAIR>(st, P, lv, b, q0, tid);
    }
""")]

# ---- round 4: persistent lookup -- a grid of 5 workgroups per CU (the LDS limit) walks the units
# (64-query group, level, batch item) round robin, and each unit's coordinates are loaded one unit
# ahead (phase 0 was 1.9 us of a ~8 us workgroup life, most of it the coordinate load's latency)
PATCHES["lk_pers"] = [
    ("lookup.hip", """template <int R, int QB, bool PAIR>
__global__ __launch_bounds__(3 * QB) void lookup_cols_reg(LookupParams P) {
    constexpr int NTQ = 3 * QB, K = 2 * R + 1, AP = K / 3;
    static_assert(K % 3 == 0 && QB == kWave, "one wave per part, whole columns per part");
    using WB = WindowBuf<R, QB, PAIR>;
    constexpr int S = WB::S, SW = WB::SW, SP = WB::SP, KK = WB::KK;
    __shared__ WB st;
    const int tid = threadIdx.x, g = tid % QB;
    const int part = __builtin_amdgcn_readfirstlane(tid / QB);   // wave-uniform
    const int lv = blockIdx.y, b = blockIdx.z;
    const int q0 = blockIdx.x * QB;""", """template <int R, int QB, bool PAIR>
__device__ __forceinline__ void lookup_cols_unit(const LookupParams& P, WindowBuf<R, QB, PAIR>& st, int lv, int b,
                                                 int q0, float cxraw, float cyraw) {
    constexpr int NTQ = 3 * QB, K = 2 * R + 1, AP = K / 3;
    static_assert(K % 3 == 0 && QB == kWave, "one wave per part, whole columns per part");
    using WB = WindowBuf<R, QB, PAIR>;
    constexpr int S = WB::S, SW = WB::SW, SP = WB::SP, KK = WB::KK;
    const int tid = threadIdx.x, g = tid % QB;
    const int part = __builtin_amdgcn_readfirstlane(tid / QB);   // wave-uniform"""),
    ("lookup.hip", """        const float cx = __fmul_rn(P.coords[((int64_t)b * 2 + 0) * Q + p], inv);
        const float cy = __fmul_rn(P.coords[((int64_t)b * 2 + 1) * Q + p], inv);
        const float wm1 = (float)(P.lw[lv] - 1), hm1 = (float)(P.lh[lv] - 1);
#pragma unroll
        for (int bb = 0; bb < K; ++bb) coord_chain<R>(cy, bb, hm1, fy[bb], wy[bb]);""", """        (void)Q;
        const float cx = __fmul_rn(cxraw, inv);
        const float cy = __fmul_rn(cyraw, inv);
        const float wm1 = (float)(P.lw[lv] - 1), hm1 = (float)(P.lh[lv] - 1);
#pragma unroll
        for (int bb = 0; bb < K; ++bb) coord_chain<R>(cy, bb, hm1, fy[bb], wy[bb]);"""),
    ("lookup.hip", """// Any radius: one thread per output element, direct gather""", """template <int R, int QB, bool PAIR>
__global__ __launch_bounds__(3 * QB) void lookup_cols_reg(LookupParams P, int nqg, int units) {
    __shared__ WindowBuf<R, QB, PAIR> st;
    const int g = threadIdx.x % QB;
    auto coords_of = [&](int uu, float& cx, float& cy) {
        cx = cy = 0.0f;
        if (uu < units) {
            const int bb = uu / nqg / P.levels, p = (uu % nqg) * QB + g;
            if (p < P.q_count) {
                cx = P.coords[((int64_t)bb * 2 + 0) * P.q_count + p];
                cy = P.coords[((int64_t)bb * 2 + 1) * P.q_count + p];
            }
        }
    };
    int u = blockIdx.x;
    float cx, cy;
    coords_of(u, cx, cy);
    while (u < units) {
        const int un = u + (int)gridDim.x;
        float ncx, ncy;
        coords_of(un, ncx, ncy);   // in flight during this unit
        const int r = u / nqg;
        lookup_cols_unit<R, QB, PAIR>(P, st, r % P.levels, r / P.levels, (u % nqg) * QB, cx, cy);
        u = un;
        cx = ncx;
        cy = ncy;
    }
}

// Any radius: one thread per output element, direct gather"""),
    ("lookup.hip", """    if (cols) {
        bool pair = true;""", """    if (cols) {
        const int nqg = (P.q_count + 63) / 64, units = nqg * P.levels * B;
        const dim3 grid(units < 1280 ? units : 1280);
        bool pair = true;"""),
    ("lookup.hip", """            if (pair) hipLaunchKernelGGL((lookup_cols_reg<4, 64, true>), grid, dim3(192), 0, stream, P);
            else hipLaunchKernelGGL((lookup_cols_reg<4, 64, false>), grid, dim3(192), 0, stream, P);
        } else {
            if (pair) hipLaunchKernelGGL((lookup_cols_reg<1, 64, true>), grid, dim3(192), 0, stream, P);
            else hipLaunchKernelGGL((lookup_cols_reg<1, 64, false>), grid, dim3(192), 0, stream, P);""",
     """            if (pair) hipLaunchKernelGGL((lookup_cols_reg<4, 64, true>), grid, dim3(192), 0, stream, P, nqg, units);
            else hipLaunchKernelGGL((lookup_cols_reg<4, 64, false>), grid, dim3(192), 0, stream, P, nqg, units);
        } else {
            if (pair) hipLaunchKernelGGL((lookup_cols_reg<1, 64, true>), grid, dim3(192), 0, stream, P, nqg, units);
            else hipLaunchKernelGGL((lookup_cols_reg<1, 64, false>), grid, dim3(192), 0, stream, P, nqg, units);"""),
]


# ---- lk_persd: lk_pers with a dynamic work queue (one device counter slot per launch, reset by
# the workgroup that takes the last id) instead of round robin
PATCHES["lk_persd"] = [(f, o, n) for f, o, n in PATCHES["lk_pers"] if "lookup_cols_unit<R, QB, PAIR>(P, st" not in n
                       and "const dim3 grid(units < 1280" not in n and "stream, P, nqg, units);" not in n] + [
    ("lookup.hip", """// Any radius: one thread per output element, direct gather""", """__device__ unsigned int g_lkq[4096];

template <int R, int QB, bool PAIR>
__global__ __launch_bounds__(3 * QB) void lookup_cols_reg(LookupParams P, int nqg, int units, unsigned int* ctr) {
    __shared__ WindowBuf<R, QB, PAIR> st;
    __shared__ int next_u;
    const int g = threadIdx.x % QB;
    auto coords_of = [&](int uu, float& cx, float& cy) {
        cx = cy = 0.0f;
        if (uu < units) {
            const int bb = uu / nqg / P.levels, p = (uu % nqg) * QB + g;
            if (p < P.q_count) {
                cx = P.coords[((int64_t)bb * 2 + 0) * P.q_count + p];
                cy = P.coords[((int64_t)bb * 2 + 1) * P.q_count + p];
            }
        }
    };
    int u = blockIdx.x;
    if (u >= units) return;
    float cx, cy;
    coords_of(u, cx, cy);
    while (true) {
        unsigned int old = 0;
        if (threadIdx.x == 0) {   // the next unit, taken now, published after this unit's staging
            old = atomicAdd(ctr, 1u);
            if (old == (unsigned)units - 1u) atomicExch(ctr, 0u);   // the last id of the launch: reset the slot
        }
        const int r = u / nqg;
        lookup_cols_unit<R, QB, PAIR>(P, st, r % P.levels, r / P.levels, (u % nqg) * QB, cx, cy, &next_u,
                                      (int)gridDim.x + (int)old);
        const int un = next_u;   // written before the unit's staging barrier, read after it
        if (un >= units) break;
        u = un;
        coords_of(u, cx, cy);
    }
}

// Any radius: one thread per output element, direct gather"""),
    ("lookup.hip", """                                                 int q0, float cxraw, float cyraw) {""",
     """                                                 int q0, float cxraw, float cyraw, int* next_u, int nxt) {"""),
    ("lookup.hip", """    __syncthreads();
    stage_windows<R, QB, NTQ, PAIR>(st, P, lv, b, q0, tid);
""", """    __syncthreads();
    {
        StageRegs<R, QB, NTQ, PAIR> sr;
        stage_issue<R, QB, NTQ, PAIR>(st, P, lv, b, q0, tid, sr);
        stage_commit<R, QB, NTQ, PAIR>(st, sr);
        if (tid == 0) *next_u = nxt;
        __syncthreads();
    }
"""),
    ("lookup.hip", """    if (cols) {
        bool pair = true;""", """    if (cols) {
        static unsigned slot_seq = 0;
        unsigned int* q = nullptr;
        if (hipGetSymbolAddress((void**)&q, HIP_SYMBOL(g_lkq)) != hipSuccess) return ECORR_EINVAL;
        q += (slot_seq++) % 4096;
        const int nqg = (P.q_count + 63) / 64, units = nqg * P.levels * B;
        const dim3 grid(units < 1280 ? units : 1280);
        bool pair = true;"""),
    ("lookup.hip", """            if (pair) hipLaunchKernelGGL((lookup_cols_reg<4, 64, true>), grid, dim3(192), 0, stream, P);
            else hipLaunchKernelGGL((lookup_cols_reg<4, 64, false>), grid, dim3(192), 0, stream, P);
        } else {
            if (pair) hipLaunchKernelGGL((lookup_cols_reg<1, 64, true>), grid, dim3(192), 0, stream, P);
            else hipLaunchKernelGGL((lookup_cols_reg<1, 64, false>), grid, dim3(192), 0, stream, P);""",
     """            if (pair) hipLaunchKernelGGL((lookup_cols_reg<4, 64, true>), grid, dim3(192), 0, stream, P, nqg, units, q);
            else hipLaunchKernelGGL((lookup_cols_reg<4, 64, false>), grid, dim3(192), 0, stream, P, nqg, units, q);
        } else {
            if (pair) hipLaunchKernelGGL((lookup_cols_reg<1, 64, true>), grid, dim3(192), 0, stream, P, nqg, units, q);
            else hipLaunchKernelGGL((lookup_cols_reg<1, 64, false>), grid, dim3(192), 0, stream, P, nqg, units, q);"""),
]

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
    ("build.hip", """    decode_tile(P, xcd_remap(blockIdx.x, gridDim.x), P.n_qt, b, qt, nt);
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

# ---- round 4: convex upsampling with the softmax's 9 IEEE divisions replaced by one reciprocal
# and 9 multiplies (up_rcp), and + the fast exp (up_fast: __expf); normwise within the test bar
PATCHES["up_rcp"] = [("upsample.hip", """#pragma unroll
        for (int k = 0; k < 9; ++k) m[k] = __fdiv_rn(m[k], s);   // softmax output""",
                      """        const float rs = __builtin_amdgcn_rcpf(s);
#pragma unroll
        for (int k = 0; k < 9; ++k) m[k] = __fmul_rn(m[k], rs);   // softmax output""")]
PATCHES["up_fast"] = PATCHES["up_rcp"] + [("upsample.hip", "            m[k] = expf(__fsub_rn(m[k], mx));",
                                           "            m[k] = __expf(__fsub_rn(m[k], mx));")]

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


# split convc1 (conv.hip): query columns 3 / 4 chunks ahead instead of 2
# the QMAX lookup (split convc1 path) with default-policy output stores instead of nt (corr stays in
# the caches for the conv that reads it next)
PATCHES["lk_qplain"] = [("lookup.hip", """                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), orsrc, voff,
                                                      sbase + (a * K + bb) * P.q_count * 4, 2);""",
                         """                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), orsrc, voff,
                                                      sbase + (a * K + bb) * P.q_count * 4, QMAX ? 0 : 2);""")]
# split convc1: non-temporal query-column loads (read once)
PATCHES["cv_bnt"] = [("conv.hip", "v[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(csrc, off + j * qs, 0, 0));",
                      "v[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(csrc, off + j * qs, 0, 2));")]
COMBOS["qplain_bnt"] = ["lk_qplain", "cv_bnt"]
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
for _gm in (2, 4, 16):
    PATCHES[f"gm{_gm}"] = [("build.hip", "    constexpr int GM = 8;\n", f"    constexpr int GM = {_gm};\n")]

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
    ("splat.hip", "    const int tid = threadIdx.x, band = blockIdx.x, b = blockIdx.y;\n",
     "    sps(0);\n    const int tid = threadIdx.x, band = blockIdx.x, b = blockIdx.y;\n"),
    ("splat.hip", "    __syncthreads();\n    const float* src = staged ? spts : gpts;\n",
     "    __syncthreads();\n    sps(1);\n    const float* src = staged ? spts : gpts;\n"),
    ("splat.hip", "    __syncthreads();\n\n    // 2. exclusive scan of cnt[0 .. nb)", "    __syncthreads();\n    sps(2);\n\n    // 2. exclusive scan of cnt[0 .. nb)"),
    ("splat.hip", "    __syncthreads();\n    // cnt[t] = start of target t's bucket", "    __syncthreads();\n    sps(3);\n    // cnt[t] = start of target t's bucket"),
    ("splat.hip", "            lkey[lo + r] = k;\n        }\n        __syncthreads();\n",
     "            lkey[lo + r] = k;\n        }\n        __syncthreads();\n        sps(4);\n"),
    ("splat.hip", "        for (int t = tid; t < nb; t += NTB) fold_sorted(t, t > 0 ? cnt[t - 1] : 0, cnt[t]);\n        return;\n",
     "        for (int t = tid; t < nb; t += NTB) fold_sorted(t, t > 0 ? cnt[t - 1] : 0, cnt[t]);\n        __syncthreads();\n        sps(5);\n        return;\n"),
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
PATCHES["cvq4n"] = PATCHES["cvq4p2"] + [("conv.hip", "amdgpu_waves_per_eu(QB > 2 ? 4 : 1)", "amdgpu_waves_per_eu(1)")]
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
PATCHES["up_ldplain"] = [("upsample.hip", "m[k] = __builtin_nontemporal_load(mrow + ((int64_t)k * 64 + j) * HW);",
                          "m[k] = mrow[((int64_t)k * 64 + j) * HW];")]
COMBOS["up_i2_ldplain"] = ["up_i2", "up_ldplain"]
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
# timing only: no weight DMA inside the K loop (every chunk multiplies the prologue's stale weights)
PATCHES["cv_nowdma"] = [("conv.hip", "        issue_w(min(c + 2, nkc - 1), (c + 2) % NB);   // past the last chunk a harmless repeat\n", "")]


# recipe-name prefix -> the lab_patches diff it applies on top of
PREDIFF = {"qs": "build_qs.diff", "lkw_": "lookup_win.diff", "mo_ws": "lookup_conv_ws.diff", "cvq": "conv_tiles.diff",
           "cvt": "conv_tiles.diff"}


def build(name):
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


if __name__ == "__main__":
    for n in sys.argv[1:]:
        build(n)
