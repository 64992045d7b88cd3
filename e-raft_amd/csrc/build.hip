// build.hip -- CorrBlock build on gfx950: the all-pairs correlation GEMM with the 1/sqrt(D) scale
// and the 3 pooled pyramid levels fused into its epilogue.
//
// Replaces corr.py:13-27 (CorrBlock.__init__) and corr.py:52-60 (CorrBlock.corr):
//   level0[b*q_count + p][y][x] = (sum_d f1[b][d][p] * f2[b][d][y*W+x]) / sqrt(D)
//   level{i+1} = (((x00 + x01) + x10) + x11) / 4 over 2x2 floor-mode windows of level i,
// stored in the tiled pyramid layout of include/ecorr.h (4 x 8-float tiles per query image).
//
// Two GEMMs, one result contract (include/ecorr.h):
//   split (ecorr_build_split, default): pack_both_kernel splits every fp32 operand into
//     per-pixel-scaled f16 hi + lo halves, written as 8-KB panels in MFMA-fragment order;
//     build_split_kernel sums lo*hi + hi*lo + hi*hi per product on v_mfma_f32_32x32x16_f16.
//   fp32 (ecorr_build): build_kernel on v_mfma_f32_32x32x2_f32, an exact k-ordered fmaf chain.
// Pooling is bit-exact given the same level 0 in both; per-element accumulation order does not
// depend on the tiling, so query-slab (row-sharded) builds are bitwise the whole build's rows.
//
// There are no runtime knobs: every variant that lost an A/B is gone from the source (DESIGN.md
// §3.1 keeps the record); lab builds for new A/Bs are separate .so files (tools/).
#include "ecorr_device.h"
#include "ecorr_internal.h"

#include <type_traits>

namespace ecorr {

namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx2 __attribute__((ext_vector_type(2)));
typedef _Float16 halfx8 __attribute__((ext_vector_type(8)));
typedef unsigned uint4v __attribute__((ext_vector_type(4)));
typedef unsigned uint2v __attribute__((ext_vector_type(2)));

constexpr int TBH = 8, TBW = 16;  // regular target block (rows x cols) of one n-tile
constexpr int PANEL = 8192;       // bytes of one (128-pixel tile, 16-deep K chunk) operand panel

__device__ __forceinline__ float pool4(float a, float b, float c, float d) {
    return __fmul_rn(__fadd_rn(__fadd_rn(__fadd_rn(a, b), c), d), 0.25f);
}

// pool4 as four VALU ops in the same order: left to itself hipcc pairs the split epilogue's pools
// into v_pk_add_f32 whose operands sit in different register pairs (two v_mov per packed add)
__device__ __forceinline__ float pool4_v(float a, float b, float c, float d) {
    float s;
    asm("v_add_f32 %0, %1, %2" : "=v"(s) : "v"(a), "v"(b));
    asm("v_add_f32 %0, %1, %2" : "=v"(s) : "v"(s), "v"(c));
    asm("v_add_f32 %0, %1, %2" : "=v"(s) : "v"(s), "v"(d));
    asm("v_mul_f32 %0, 0.25, %1" : "=v"(s) : "v"(s));
    return s;
}

// 2^e as a float, e in [-126, 127]
__device__ __forceinline__ float exp2i(int e) { return __int_as_float((e + 127) << 23); }

// s_waitcnt vmcnt(N) with lgkmcnt(0) (LGKM0) or left alone; expcnt never waited (gfx9 encoding:
// vmcnt bits 3:0 and 15:14)
template <int N, bool LGKM0>
__device__ __forceinline__ void wait_vm() {
    static_assert(N >= 0 && N < 64, "vmcnt field");
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (LGKM0 ? 0 : (15 << 8)));
}

// Bijective XCD-aware remap (cdna_hip_programming.md §5 T1): consecutive logical tiles land on
// one XCD so tiles sharing operand panels share that XCD's L2.  Speed only, never correctness.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
    const int q = nwg / 8, r = nwg % 8, xcd = bid % 8, k = bid / 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + k;
}

// n-tiles: 8 x 16 target blocks (regular), or, in the last 4 rows when H % 8 is 1..4, 4 x 32
// blocks ("band"): those rows feed pyramid levels 0-2 only (level 3 of an H = 8k + r map, r <= 4,
// has k rows), so the band pools 4 x 8 sub-blocks and no 8-row tile row is padded half empty
// (DSEC H = 60: 6.7% of the matrix work saved).
struct NTile { int ty0, tx0, band; };
__device__ __forceinline__ NTile ntile_of(const BuildParams& P, int nt) {
    NTile n;
    if (nt < P.n_reg) {
        const int nty = nt / P.n_ntx;
        n.ty0 = nty * TBH;
        n.tx0 = (nt - nty * P.n_ntx) * TBW;
        n.band = 0;
    } else {
        n.ty0 = P.band_y0;
        n.tx0 = (nt - P.n_reg) * 32;
        n.band = 1;
    }
    return n;
}

// Grouped tile order: GM m-tiles x all n-tiles per group, so consecutive tiles share panels.  BAL:
// the item's m-tiles split into ceil(n_m / GM) groups of (nearly) equal size instead of full groups
// and a remainder -- at DSEC (19 split16 query tiles) GM 10 makes two groups (10, 9), so every
// target panel leaves the L2 twice per item instead of three times (8, 8, 3): FETCH -20%, the build
// 1.3% shorter (profiles/r05_lab/gm_clock_l2_b.txt); 10 query panels (2.5 MB) + the resident
// blocks' target panels still fit an XCD's 4-MB L2 (GM 16 does not: 4.5 MB, slower).
template <int GM, bool BAL>
__device__ __forceinline__ void decode_tile(const BuildParams& P, int t, int n_m, int& b, int& mt, int& nt) {
    const int per_b = n_m * P.n_nt;
    b = t / per_b;
    const int i = t - b * per_b;
    const int ng = (n_m + GM - 1) / GM;
    const int gm = BAL ? (n_m + ng - 1) / ng : GM;
    const int gsz = gm * P.n_nt;
    const int grp = i / gsz, gi = i - grp * gsz;
    const int first_m = grp * gm;
    const int gsm = min(n_m - first_m, gm);
    mt = first_m + gi % gsm;
    nt = gi / gsm;
}
constexpr int kGM16 = 10;   // build_split16_kernel's group bound (balanced); the other builds: 8

// One pooled-level pixel (row, col) of a query image: tiled (ntx > 0; the tile must exist, cells
// in a tile's padding are written and never read), interleaved (ntx < 0; likewise the block) or
// compact row-major (range-checked).
__device__ __forceinline__ float* level_px(const BuildParams& P, int L, int64_t row_img, int r, int c) {
    if (P.lntx[L] < 0) {   // interleaved (levels 2, 3): the block must exist
        if ((r >> ilv_sy(L)) >= P.lnty[L] || (c >> ilv_sx(L)) >= -P.lntx[L]) return nullptr;
        return P.lvl[L] + pix_off(row_img, r, c, L, P.lntx[L], P.lw[L], P.lsz[L]);
    }
    float* img = P.lvl[L] + row_img * P.lsz[L];
    if (P.lntx[L] > 0) {
        if ((r >> 2) >= P.lnty[L] || (c >> 3) >= P.lntx[L]) return nullptr;
        return img + tiled_off(r, c, P.lntx[L]);
    }
    if (r >= P.lh[L] || c >= P.lw[L]) return nullptr;
    return img + (int64_t)r * P.lw[L] + c;
}

// ============================================================================================
// Split GEMM (default).  Block tile: 256 queries (two 128-query fmap1 panels) x one 128-target
// n-tile (one fmap2 panel); 4 waves, wave w = queries 64 w .. 64 w + 63 x all 128 targets = 2 x 4
// v_mfma_f32_32x32x16_f16 tiles (128 accumulators, pinned to AGPRs).  Two blocks per CU.
//
// The MFMAs take the fmap2 fragment as their A operand: the accumulators hold C^T, lane (acol,
// arow) of tile (i, j) owns query 32 i + acol and targets 32 j + 8 g4 + 4 arow + t (reg 4 g4 + t).
// The fmap2 panel stores the n-tile's targets (split_target) so that target group j of a regular
// 8 x 16 tile is one pyramid tile line: rows 4 (j & 1) + g4, cols 8 (j >> 1) + 4 arow + t -- each
// lane holds 4 x 4 pixels of every line of its query, the 2 x 2 and 4 x 4 pools are in-lane and
// the 8 x 8 pool needs one value from lane acol + 32.  Band tiles (4 x 32): rows g4, cols 8 j +
// 4 arow + t.
//
// K loop: the target panel (shared by the 4 waves) goes global -> LDS verbatim by LDS-DMA
// (buffer_load_dwordx4 ... lds, 2 per wave and chunk) through 3 buffers, two chunks ahead; the
// query fragments (wave-private) go global -> VGPR, two chunks ahead.  One barrier per chunk;
// target fragments are lane-linear ds_read_b128 (conflict-free).  Chunk kc + 1's barrier and
// first fragments are read between chunk kc's lo*hi MFMAs and its hi*lo / hi*hi MFMAs.  Chunks
// past the end are issued as out-of-range loads (they land as zeros), which keeps every wait
// count static.
//
// Epilogue, per wave from its accumulators: scale by 2^-(e_q + e_t) / sqrt(D), pool 8x8 -> 4x4 ->
// 2x2 -> 1 in registers in the reference's order, then store.  Store shape matters more than
// anything else here (tools/store_lab.hip, DSEC level-0 shape): whole 128-byte lines run at
// 5.2-5.5 TB/s with any cache policy; 32-byte pieces only as plain stores, which keep every line
// in L2 and evict the operand panels (PMC: 1 GB of panel re-reads per build).  So level-0 and
// level-1 lines pass through a wave-private LDS transpose and leave whole as non-temporal stores
// (out of L2); levels 2-3 (6% of the bytes) leave as 16- / 8-byte row pieces.
// ============================================================================================
constexpr int SQ = 256;                     // queries per split tile
constexpr int SCHUNK = PANEL;               // LDS bytes per K chunk (the target panel)
constexpr int SDT = 4;                      // target panel: chunks ahead = LDS buffers (NK > 0 loop)
constexpr int SDQ = 3;                      // query fragments: chunks ahead = register sets (NK > 0 loop)
constexpr int SNBUF = SDT;
constexpr int SCOPIES = SCHUNK / 1024 / 4;  // LDS-DMA copies per wave per chunk (2)
constexpr int QLOADS = 4;                   // query fragment loads per wave per chunk (hi, lo x 2 rows)
constexpr int SLDS = 4 * 4 * 32 * 144;      // LDS bytes: the epilogue's transpose regions (> the K loop's)
constexpr int SOOB = 0x7ffffff0;            // buffer offset beyond any panel: loads 0, touches nothing
constexpr int ST_L01 = 2;                   // level-0/1 store cache policy: nt (A/B: 725 vs 731 us for nt sc1;
                                            // plain and sc1 alone ~1000 us: the lines stay in L2 and evict the panels;
                                            // split16, round 3: nt 605 vs nt sc1 627 us)
constexpr int XS = 144;                     // LDS bytes per query of the epilogue's line transpose
static_assert(4 * 4 * 32 * XS <= SLDS && SNBUF * SCHUNK <= SLDS, "LDS regions");

// target (y, x) of position p of a split fmap2 panel, relative to the n-tile origin
__host__ __device__ __forceinline__ void split_target(int p, bool band, int& y, int& x) {
    if (!band) {
        y = 4 * ((p >> 5) & 1) + ((p >> 3) & 3);
        x = 8 * (p >> 6) + (p & 7);
    } else {
        y = (p >> 3) & 3;
        x = 8 * (p >> 5) + (p & 7);
    }
}

// VMEM instructions a wave has issued after t(j) when the NK > 0 loop's advance(j) waits for it
// (chunk j - 1, before its own t issue): the issue order of build_split_kernel replayed at compile
// time (t = SCOPIES LDS-DMA pieces, q = QLOADS fragment loads; q(k) exists for k < nk).
constexpr int split_vm_after(int j, int nk) {
    int n = 0;
    bool seen = false;
    for (int k = 0; k < SDT; ++k) {   // prologue: t(k) q(k)
        if (seen) n += SCOPIES;
        if (k == j) seen = true;
        if (k < SDQ && k < nk && seen) n += QLOADS;
    }
    for (int c = 0; c <= j - 2; ++c) {   // chunk c: t(c + SDT), q(c + SDQ)
        if (seen) n += SCOPIES;
        if (c + SDT == j) seen = true;
        if (c + SDQ < nk && seen) n += QLOADS;
    }
    return n;
}
static_assert(SDT != 4 || SDQ != 3 ||
                  (split_vm_after(0, 16) == 18 && split_vm_after(5, 16) == 16 && split_vm_after(16, 16) == 8),
              "split loop wait counts (hand-checked for SDT 4, SDQ 3)");
static_assert(split_vm_after(0, 16) < 41, "wait_vm_n range");

// wait_vm<n> for an n that is a constant once the loop around the call is unrolled
template <bool LGKM0, int N = 40>
__device__ __forceinline__ void wait_vm_n(int n) {
    if constexpr (N >= 0) {
        if (n == N) wait_vm<N, LGKM0>();
        else wait_vm_n<LGKM0, N - 1>(n);
    }
}

// lanes 32-63 of a <-> lanes 0-31 of b (v_permlane32_swap)
__device__ __forceinline__ void swap32(float& a, float& b) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    a = __uint_as_float(r[0]);
    b = __uint_as_float(r[1]);
}

// Epilogue of the split build for one wave: its 64 queries (block-local qw .. qw + 63) x the
// n-tile tc, from its accumulators (C^T fragments, build_split_kernel); xw = the wave's four
// LDS transpose regions (4 x 32 x XS bytes); exq = the block's query exponents, ext / fst = the
// n-tile's negated target exponents and their powers of two.
template <bool MUL>
__device__ __forceinline__ void split_epilogue(const BuildParams& P, floatx16 (&acc)[2][4], char* const xw, int qw,
                                               const int* exq, const int* ext, const float* fst, const NTile& tc,
                                               int b, int q0, int lane) {
    const int acol = lane & 31, arow = lane >> 5;
    // Line segments through a wave-private LDS transpose (no barrier: a wave's LDS accesses are
    // processed in order): the lane writes its 16-byte pieces into the line image of its query
    // (32 queries x 144 B: conflict-free ds_write_b128 and ds_read_b128), then reads back piece m
    // of segment arow of query 4k + s, so the 4 lanes of a quad store 64 contiguous bytes and
    // lanes acol, acol + 32 the two halves of one line.
    // four regions per wave (one per level-0 line of a tile row; the level-1 line reuses region
    // 0): no line waits for the previous line's read-back before writing
    const int m4 = lane & 3, k4 = acol >> 2;
    const int wo = acol * XS, ro = (4 * k4) * XS + 64 * arow + 16 * m4;
    const int L = P.fused_levels;
    const int64_t rows0 = (int64_t)b * P.q_count + q0;   // the block's first query image
    const int nq = min(SQ, P.q_count - q0);
    // per-level descriptors over the block's query images (range check = query bound); levels 2-3
    // (interleaved): over the 64-row groups the block's rows touch, from group g0 = rows0 / 64
    const int64_t g0 = rows0 >> 6;
    auto rsrc_of = [&](int lv) {
        if (lv >= 1)
            return __builtin_amdgcn_make_buffer_rsrc(P.lvl[lv] + g0 * kGroup * P.lsz[lv], 0,
                                                     (int)((((rows0 + nq - 1) >> 6) - g0 + 1) * kGroup * P.lsz[lv] * 4),
                                                     0x00020000);
        return __builtin_amdgcn_make_buffer_rsrc(P.lvl[lv] + rows0 * P.lsz[lv], 0, (int)(nq * P.lsz[lv] * 4), 0x00020000);
    };
    // read the transposed segments back and store them: line byte offset lo (+ the query image)
    auto store_lines = [&](const char* xp, __amdgpu_buffer_rsrc_t rs, int64_t lsz, int ql, int lo, bool ok) {
        floatx4 pc[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) pc[s] = *reinterpret_cast<const floatx4*>(xp + ro + s * XS);
        const int base = (int)((ql + 4 * k4) * lsz * 4) + lo + 16 * m4;
#pragma unroll
        for (int s = 0; s < 4; ++s)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(uint4v, pc[s]), rs,
                                                   ok ? base + (int)(s * lsz * 4) : SOOB, 0, ST_L01);
    };
    // One block row (r, c .. c + N - 1), N = the block width, of level 2 or 3 (interleaved) for
    // block-local query qloc: lanes on consecutive queries write consecutive 4N-byte pieces, so a
    // store instruction covers whole lines, which leave non-temporally like levels 0-1 (A/B: 656
    // vs 685 us with plain stores, which park the lines in L2).  Queries past the block and
    // blocks outside the level are dropped (padding cells of a block are written, never read).
    auto store_px = [&](__amdgpu_buffer_rsrc_t rs, int lv, int qloc, int r, int c, auto val) {
        constexpr int N = sizeof(val) / 4;
        const int sy = ilv_sy(lv), sx = ilv_sx(lv);
        const int by = r >> sy, bx = c >> sx;
        const bool in = qloc < nq && by < P.lnty[lv] && bx < -P.lntx[lv];
        const int64_t R = rows0 + qloc;
        const int off = (int)((((R >> 6) - g0) * kGroup * P.lsz[lv] +
                               ((int64_t)(by * -P.lntx[lv] + bx) * kGroup + (R & (kGroup - 1))) * (1 << (sy + sx)) +
                               ((r & ((1 << sy) - 1)) << sx)) * 4);
        if constexpr (N == 4)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(uint4v, val), rs, in ? off : SOOB, 0, ST_L01);
        else
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(uint2v, val), rs, in ? off : SOOB, 0, ST_L01);
    };
    // Scaling: x = acc 2^(nqe + ext) (/ sqrt(D) when that is no power of two).  Where every
    // exponent of the wave's queries and of the panel's targets lies in [-63, 63], the 2^nqe 2^ext
    // product is a normal power of two and one multiply by it rounds exactly as ldexpf does: two
    // packed multiplies per element pair instead of an add, a negate and an ldexp per element.
    bool fast_scale;
    {
        bool ok = ext[lane] >= -63 && ext[lane] <= 63 && ext[lane + 64] >= -63 && ext[lane + 64] <= 63;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int n = -(exq[qw + 32 * i + acol] + (MUL ? P.scale_shift : 0));
            ok = ok && n >= -63 && n <= 63;
        }
        fast_scale = __all(ok);
    }
    const __amdgpu_buffer_rsrc_t r0 = rsrc_of(0);
    const __amdgpu_buffer_rsrc_t r1 = rsrc_of(L > 1 ? 1 : 0);
    const __amdgpu_buffer_rsrc_t r2 = rsrc_of(L > 2 ? 2 : 0);
    const __amdgpu_buffer_rsrc_t r3 = rsrc_of(L > 3 ? 3 : 0);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int ql = qw + 32 * i;          // first block-local query of this tile row
        const int nqe = -(exq[ql + acol] + (MUL ? P.scale_shift : 0));
        // level-1 values of the lane's query: [block bb][row][col pair] (band: [half][2 y1 + jl]);
        // level 2: [bb][row r] (band: [bb][jl]); level 3: [bb]
        float l1[2][4][2], l2[2][2], l3[2];
#pragma unroll
        for (int bb = 0; bb < 2; ++bb) {
            // scaled values of lines j = 2 bb + jl, [jl][g4][t]; target exponents
            // ext[32 j + 8 g4 + 4 arow + t]
            float v[2][4][4];
            if (fast_scale) {
                const float sq = exp2i(nqe);
#pragma unroll
                for (int jl = 0; jl < 2; ++jl) {
                    const int j = 2 * bb + jl;
#pragma unroll
                    for (int g4 = 0; g4 < 4; ++g4) {
                        const floatx4 s4 = *reinterpret_cast<const floatx4*>(fst + 32 * j + 8 * g4 + 4 * arow);
#pragma unroll
                        for (int h = 0; h < 2; ++h) {   // exact power-of-two products, v_pk_mul_f32 pairs
                            const floatx2 x = floatx2{acc[i][j][4 * g4 + 2 * h], acc[i][j][4 * g4 + 2 * h + 1]} *
                                              (floatx2{sq, sq} * floatx2{s4[2 * h], s4[2 * h + 1]});
                            v[jl][g4][2 * h] = MUL ? x[0] : __fdiv_rn(x[0], P.scale);
                            v[jl][g4][2 * h + 1] = MUL ? x[1] : __fdiv_rn(x[1], P.scale);
                        }
                    }
                }
            } else {
#pragma unroll
                for (int jl = 0; jl < 2; ++jl) {
                    const int j = 2 * bb + jl;
#pragma unroll
                    for (int g4 = 0; g4 < 4; ++g4) {
                        const int4 e4 = *reinterpret_cast<const int4*>(ext + 32 * j + 8 * g4 + 4 * arow);
                        const int e[4] = {e4.x, e4.y, e4.z, e4.w};
#pragma unroll
                        for (int t = 0; t < 4; ++t) {
                            const float x = ldexpf(acc[i][j][4 * g4 + t], nqe + e[t]);
                            v[jl][g4][t] = MUL ? x : __fdiv_rn(x, P.scale);
                        }
                    }
                }
            }
            // level 0: line j = rows g4 x this lane's 4 columns
#pragma unroll
            for (int jl = 0; jl < 2; ++jl) {
                const int j = 2 * bb + jl;
                char* const xp = xw + j * (32 * XS);
#pragma unroll
                for (int g4 = 0; g4 < 4; ++g4)
                    *reinterpret_cast<floatx4*>(xp + wo + 32 * g4 + 16 * arow) =
                        floatx4{v[jl][g4][0], v[jl][g4][1], v[jl][g4][2], v[jl][g4][3]};
                const int tr = (tc.ty0 >> 2) + (tc.band ? 0 : (j & 1));
                const int tcl = (tc.tx0 >> 3) + (tc.band ? j : (j >> 1));
                store_lines(xp, r0, P.lsz[0], ql, ((tr * P.lntx[0] + tcl) * kTile) * 4 + 64 * arow,
                            tr < P.lnty[0] && tcl < P.lntx[0]);
            }
            if (L < 2) continue;
            if (!tc.band) {
                // regular: line j = rows 4 jl + g4 of 8 x 8 block bb; level 1 rows y1 = 0..3, cols
                // 4 bb + 2 arow + c; level 2 rows r, col 2 bb + arow; level 3 needs lane acol + 32
#pragma unroll
                for (int y1 = 0; y1 < 4; ++y1)
#pragma unroll
                    for (int c = 0; c < 2; ++c) {
                        const int jl = y1 >> 1, g = 2 * (y1 & 1);
                        l1[bb][y1][c] = pool4_v(v[jl][g][2 * c], v[jl][g][2 * c + 1], v[jl][g + 1][2 * c],
                                              v[jl][g + 1][2 * c + 1]);
                    }
                if (L >= 3) {   // level 2: rows r, col 2 bb + arow (stored per i below)
#pragma unroll
                    for (int r = 0; r < 2; ++r)
                        l2[bb][r] = pool4_v(l1[bb][2 * r][0], l1[bb][2 * r][1], l1[bb][2 * r + 1][0], l1[bb][2 * r + 1][1]);
                    // level 3, the 8 x 8 pool: lane acol + 32 holds the right column
                    const float o0 = __shfl_xor(l2[bb][0], 32), o1 = __shfl_xor(l2[bb][1], 32);
                    l3[bb] = pool4_v(l2[bb][0], o0, l2[bb][1], o1);
                }
            } else {
                // band: line j = row g4 x cols 8 j + 4 arow + t; level 1 rows y1 = 0..1, cols
                // 4 j + 2 arow + c (l1[bb][2 y1 + jl][c]); level 2 col 2 j + arow
#pragma unroll
                for (int jl = 0; jl < 2; ++jl)
#pragma unroll
                    for (int y1 = 0; y1 < 2; ++y1)
#pragma unroll
                        for (int c = 0; c < 2; ++c)
                            l1[bb][2 * y1 + jl][c] = pool4_v(v[jl][2 * y1][2 * c], v[jl][2 * y1][2 * c + 1],
                                                           v[jl][2 * y1 + 1][2 * c], v[jl][2 * y1 + 1][2 * c + 1]);
                if (L >= 3) {   // level 2: col 2 (2 bb + jl) + arow (stored per i below)
#pragma unroll
                    for (int jl = 0; jl < 2; ++jl)
                        l2[bb][jl] = pool4_v(l1[bb][jl][0], l1[bb][jl][1], l1[bb][2 + jl][0], l1[bb][2 + jl][1]);
                }
            }
        }
        if (L < 2) continue;
        if (L >= 3) {
            // level 2: one 16-byte row piece per lane.  Regular: the n-tile's 2 x 4 pixels, lane
            // acol row 0, lane acol + 32 row 1, cols {2 bb, 2 bb + 1} = (l2[bb][0] | l2[bb][1]) after
            // swapping row 1 of the arow-0 lanes with row 0 of the arow-1 lanes.  Band: the 1 x 8
            // pixels, lane acol cols 0-3, lane acol + 32 cols 4-7 (swap bb = 1 of the arow-0 lanes
            // with bb = 0 of the arow-1 lanes)
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                if (!tc.band) swap32(l2[k][0], l2[k][1]);
                else swap32(l2[0][k], l2[1][k]);
            }
            const floatx4 row2 = tc.band ? floatx4{l2[0][0], l2[1][0], l2[0][1], l2[1][1]}
                                         : floatx4{l2[0][0], l2[0][1], l2[1][0], l2[1][1]};
            store_px(r2, 2, ql + acol, (tc.ty0 >> 2) + (tc.band ? 0 : arow), (tc.tx0 >> 2) + (tc.band ? 4 * arow : 0), row2);
            if (L >= 4 && !tc.band)   // level 3: the n-tile's 1 x 2 pixels, from the arow-0 lanes
                store_px(r3, 3, arow ? nq : ql + acol, tc.ty0 >> 3, tc.tx0 >> 3, floatx2{l3[0], l3[1]});
        }
        // level 1 (interleaved 2 x 4 blocks): the lane holds cols 2 arow, 2 arow + 1 of each block
        // row; one swap of rows between the arow halves leaves lane acol with row 0 and lane
        // acol + 32 with row 1 of the block, each a 16-byte piece (as level 2).  Regular: blocks
        // (r, bb) = level-1 rows ty0/2 + 2r .. +1, cols tx0/2 + 4 bb .. +3 (l1[bb][y1][c], y1 = 2r,
        // 2r + 1); band: blocks j = 2 bb + jl = rows ty0/2 .. +1, cols tx0/2 + 4j .. +3
        // (l1[bb][2 y1 + jl][c])
#pragma unroll
        for (int bb = 0; bb < 2; ++bb)
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                float x0, x1, y0, y1;
                if (!tc.band) {
                    x0 = l1[bb][2 * r][0], x1 = l1[bb][2 * r][1], y0 = l1[bb][2 * r + 1][0], y1 = l1[bb][2 * r + 1][1];
                } else {
                    x0 = l1[bb][r][0], x1 = l1[bb][r][1], y0 = l1[bb][2 + r][0], y1 = l1[bb][2 + r][1];
                }
                swap32(x0, y0);
                swap32(x1, y1);
                const int yb = (tc.ty0 >> 1) + (tc.band ? 0 : 2 * r) + arow;
                const int xb = (tc.tx0 >> 1) + (tc.band ? 4 * (2 * bb + r) : 4 * bb);
                store_px(r1, 1, ql + acol, yb, xb, floatx4{x0, x1, y0, y1});
            }
    }
}

// NK: K chunks known at compile time (16: D = 256, the E-RAFT feature width) -- the K loop is then
// fully unrolled, which lets hipcc count the in-flight query loads exactly (in the rolled loop it
// drains them at the loop header); 0 = any D.
template <bool MUL, int NK>
__global__ __launch_bounds__(256, 2) void build_split_kernel(BuildParams P) {
    // ALL LDS in this one array: a second __shared__ object can make hipcc wait vmcnt(0) before
    // every ds_read while a buffer_load ... lds is in flight (cdna_hip_programming.md trap 4(a))
    __shared__ __attribute__((aligned(16))) char smem[SLDS + (SQ + 256) * 4];
    int* exq = reinterpret_cast<int*>(smem + SLDS);             // exponents of the 256 queries
    int* ext = exq + SQ;                                        // ... negated, of the 128 panel targets
    float* fst = reinterpret_cast<float*>(ext + 128);           // 2^ext when |ext| <= 63

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    int b, qt, nt;
    decode_tile<8, false>(P, xcd_remap(blockIdx.x, gridDim.x), P.n_qt, b, qt, nt);
    const NTile tc = ntile_of(P, nt);
    const int q0 = qt * SQ;
    const int H = P.H, W = P.W;
    const int64_t Q = (int64_t)H * W;

    // per-pixel exponents: only the epilogue reads them, so they load behind the K loop's last
    // static wait and reach LDS after it (in the prologue, their two dependent global loads with
    // vmcnt(0) waits delayed every block's first DMA)
    int eq = 0, et = 0;
    auto load_exponents = [&]() {
        eq = q0 + tid < P.q_count ? P.ex1[(int64_t)b * P.q_count + q0 + tid] : 0;
        if (tid < 128) {
            int y, x;
            split_target(tid, tc.band, y, x);
            y += tc.ty0;
            x += tc.tx0;
            et = (y < H && x < W) ? P.ex2[(int64_t)b * Q + (int64_t)y * W + x] : 0;   // negated after the loop
        }
    };

    // ---- operand panels of this tile: two query panels (adjacent tiles of pk1), one target panel
    const int dc = (P.D + 15) / 16, nk = NK ? NK : dc;
    const int64_t pstride = (int64_t)dc * PANEL;   // bytes of one 128-pixel tile's panels
    const int qp = 2 * qt;
    const int nqp = min(2, P.n_mt - qp);
    const __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<char*>(P.pk1 + ((int64_t)b * P.n_mt + qp) * pstride), 0, (int)(nqp * pstride), 0x00020000);
    const __amdgpu_buffer_rsrc_t rt = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<char*>(P.pk2 + ((int64_t)b * P.n_nt + nt) * pstride), 0, (int)pstride, 0x00020000);
    // target panel: copy s of this wave = 1-KB piece wave + 4 s of the chunk (lane-linear, as
    // LDS-DMA requires)
    auto issue = [&](int kc) {
        char* dst = smem + (kc % SNBUF) * SCHUNK;
        const bool in = kc < nk;
#pragma unroll
        for (int s = 0; s < SCOPIES; ++s) {
            const int c = wave + 4 * s;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rt, (__attribute__((address_space(3))) void*)(dst + c * 1024), 16,
                                                     in ? kc * PANEL + c * 1024 + lane * 16 : SOOB, 0, 0, 0);
        }
    };

    floatx16 acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;
    // pin the accumulators to AGPRs: left to its heuristics hipcc keeps them in VGPRs with MFMA
    // destinations apart from their sources and spills ~100 registers at 2 waves per SIMD
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) asm volatile("" : "+a"(acc[i][j]));

    // query fragments: wave-private (rows 64 wave .. + 63), so they go global -> VGPR directly,
    // one chunk ahead: query panel wave/2, 32-row group 2 (wave&1) + i, [hi | lo] 1 KB each
    struct QFrags { halfx8 qh[2], ql[2]; };
    const int qgo = (wave >> 1) * (int)pstride + (wave & 1) * 4096 + lane * 16;
    auto load_q = [&](int kc, QFrags& q) {
        const bool in = kc < nk;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            q.qh[i] = __builtin_bit_cast(halfx8, __builtin_amdgcn_raw_buffer_load_b128(
                                                     rq, in ? qgo + kc * PANEL + i * 2048 : SOOB, 0, 0));
            q.ql[i] = __builtin_bit_cast(halfx8, __builtin_amdgcn_raw_buffer_load_b128(
                                                     rq, in ? qgo + kc * PANEL + i * 2048 + 1024 : SOOB, 0, 0));
        }
    };
    // target fragments of one chunk from LDS: group j, [hi k0-15 | lo k0-15] x 32 rows, 16 B per lane
    const int tfo = lane * 16;
    struct TFrags { halfx8 th[4], tl[4]; };
    auto read_lo = [&](int kc, TFrags& f) {   // what the lo*hi MFMAs need besides ql: th
        const char* cb = smem + (kc % SNBUF) * SCHUNK;
#pragma unroll
        for (int j = 0; j < 4; ++j) f.th[j] = *reinterpret_cast<const halfx8*>(cb + tfo + j * 2048);
    };
    auto read_hi = [&](int kc, TFrags& f) {   // tl
        const char* cb = smem + (kc % SNBUF) * SCHUNK;
#pragma unroll
        for (int j = 0; j < 4; ++j) f.tl[j] = *reinterpret_cast<const halfx8*>(cb + tfo + j * 2048 + 1024);
    };
    // per element: lo*hi, then hi*lo, then hi*hi (the accumulation order of the round-1 build)
    auto mfma_lohi = [&](const TFrags& f, const QFrags& q) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f.th[j], q.ql[i], acc[i][j], 0, 0, 0);
    };
    auto mfma_rest = [&](const TFrags& f, const QFrags& q) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f.tl[j], q.qh[i], acc[i][j], 0, 0, 0);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f.th[j], q.qh[i], acc[i][j], 0, 0, 0);
    };
    // VMEM issue order per wave: t(j + 1) [in advance(j - 1)], q(j) [end of chunk j - 2], t(j + 2)
    // [advance(j)], q(j + 1) [end of chunk j - 1], ...  advance(j) (after chunk j - 1's lo*hi
    // MFMAs) waits until t(j) has landed, with the 6 younger t(j + 1), q(j) in flight; the
    // compiler's own vmcnt waits cover the q registers before their MFMAs.  The barrier publishes
    // chunk j and retires every wave's reads of chunk j - 1, whose buffer chunk j + 2 then takes
    // Every wait count above assumes the VMEM issue order of the source, so the loads are fenced
    // from each other and from the waits by sched_barrier (hipcc otherwise hoists the query loads
    // over the LDS-DMA, e.g. q(0) in front of t(0) -- a race on t(0)), and the phases below stay
    // in program order (left free, hipcc gathers each chunk's LDS reads in front of their first
    // MFMA and exposes their latency every chunk).
#define PHASE __builtin_amdgcn_sched_barrier(0)
    auto advance = [&](int j) {
        PHASE;
        wait_vm<SCOPIES + QLOADS, true>();
        __builtin_amdgcn_s_barrier();
        PHASE;
        issue(j + 2);
        PHASE;
    };

    if constexpr (NK > 0) {
        // D known at compile time: the target panel SDT chunks ahead (SDT LDS buffers), the query
        // fragments SDQ chunks ahead in SDQ register sets.  VMEM issue order per wave: prologue
        // t(0) q(0) t(1) q(1) ... t(SDT - 1), then chunk c issues t(c + SDT) in advance(c + 1) and
        // q(c + SDQ) at its end; advance(j)'s wait count is split_vm_after(j) (loads past the last
        // chunk are not issued: hipcc deletes loads whose registers are never read).
        TFrags f[2];
        QFrags qs[SDQ];
        auto advance_n = [&](int j) {
            PHASE;
            wait_vm_n<true>(split_vm_after(j, NK));
            __builtin_amdgcn_s_barrier();
            PHASE;
            issue(j + SDT - 1);
            PHASE;
        };
#pragma unroll
        for (int k = 0; k < SDT; ++k) {
            issue(k);
            PHASE;
            if (k < SDQ) load_q(k, qs[k]);
            PHASE;
        }
        wait_vm_n<true>(split_vm_after(0, NK));   // t(0) landed
        __builtin_amdgcn_s_barrier();
        PHASE;
        read_lo(0, f[0]);
        read_hi(0, f[0]);
        PHASE;
#pragma unroll
        for (int kc = 0; kc < NK; ++kc) {
            mfma_lohi(f[kc & 1], qs[kc % SDQ]);
            PHASE;
            advance_n(kc + 1);
            if (kc == NK - 1) load_exponents();   // after the last static wait
            read_lo(kc + 1, f[(kc + 1) & 1]);
            PHASE;
            mfma_rest(f[kc & 1], qs[kc % SDQ]);
            PHASE;
            read_hi(kc + 1, f[(kc + 1) & 1]);
            if (kc + SDQ < NK) load_q(kc + SDQ, qs[kc % SDQ]);
            PHASE;
        }
    } else {
    TFrags fa, fb;
    QFrags qa, qb;
    issue(0);
    PHASE;
    issue(1);
    PHASE;
    load_q(0, qa);
    PHASE;
    wait_vm<SCOPIES + QLOADS, true>();   // t(0) landed (t(1), q(0) may fly)
    __builtin_amdgcn_s_barrier();
    PHASE;
    issue(2);
    PHASE;
    read_lo(0, fa);
    read_hi(0, fa);
    PHASE;
    load_q(1, qb);
    PHASE;
#pragma unroll NK ? NK : 1
    for (int kc = 0; kc < nk; kc += 2) {
        mfma_lohi(fa, qa);
        PHASE;
        advance(kc + 1);
        read_lo(kc + 1, fb);
        PHASE;
        mfma_rest(fa, qa);
        PHASE;
        read_hi(kc + 1, fb);
        load_q(kc + 2, qa);
        PHASE;
        if (kc + 1 >= nk) break;   // odd chunk count: fb is a zero chunk
        mfma_lohi(fb, qb);
        PHASE;
        advance(kc + 2);
        read_lo(kc + 2, fa);
        PHASE;
        mfma_rest(fb, qb);
        PHASE;
        read_hi(kc + 2, fa);
        load_q(kc + 3, qb);
        PHASE;
    }
    }
#undef PHASE
    if constexpr (NK == 0) load_exponents();
    wait_vm<0, true>();             // the exponents and the trailing zero chunks have landed, this wave's reads are done ...
    exq[tid] = eq;
    if (tid < 128) {
        ext[tid] = -et;
        fst[tid] = exp2i(max(-63, min(-et, 63)));
    }
    __syncthreads();                // ... in every wave: the chunk buffers are the epilogue's scratch
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) asm volatile("" : "+a"(acc[i][j]));

    // ---------------- epilogue (per wave, from registers) ----------------
    split_epilogue<MUL>(P, acc, smem + wave * (4 * 32 * XS), wave * 64, exq, ext, fst, tc, b, q0, lane);
}

// ============================================================================================
// Split GEMM on v_mfma_f32_16x16x32_f16 (D = 256, the E-RAFT feature width: the default build).
// The same block tile, waves and operand split as build_split_kernel (256 queries x one 128-target
// n-tile, wave w = queries 64 w .. + 63 x all 128 targets, two blocks per CU, lo*hi + hi*lo + hi*hi
// per product), on the 16x16x32 MFMA shape: at the same cycles per FLOP the chip holds a higher
// clock under this load on 16x16x32 than on 32x32x16 (MI355X_MICROARCH.md, DVFS give-back item 7;
// round-2 lab: 1.81 vs 1.49 GHz in the K loop alone, profiles/r02_lab/NOTES.md).
//
// K is consumed in 32-deep chunk pairs (the panel layout of pack_body<., true>): per pair and 16x16
// tile three MFMAs, hi*hi, lo*hi, hi*lo, each over the pair's 32 k -- every fragment is loaded once
// and used twice.  The MFMAs take the fmap2 fragment as A (16 targets x 32 k) and the query
// fragment as B (32 k x 16 queries), so lane l of tile (query group qg, target group tg) holds
// query 16 qg + (l & 15) and targets 16 tg + 4 kb + i, kb = l >> 4, i = 0..3.  The fmap2 panel
// stores the n-tile's targets in split16_target order, which makes a lane's 32 targets of a
// query one 4 x 8 quadrant of the 8 x 16 tile (band: one 4 x 8 block of the 4 x 32 tile) -- one
// level-0 tile line, in line order (value 4 tg + i) -- so levels 1 and 2 pool in-lane and the 8 x 8
// pool of level 3 needs one value from lane l ^ 16.
//
// K loop (8 chunk pairs): the target panel of a pair (16 KB, shared by the 4 waves) goes global ->
// LDS by LDS-DMA (4 pieces per wave) through 4 buffers, two pairs ahead; the wave-private query
// fragments (8 x 16 B per lane and pair) global -> VGPR one pair ahead.  One barrier per pair, in
// the middle of the pair's 8 target groups (after group 5): it publishes the next pair (whose first
// A fragments are then read under the last two groups' MFMAs) and retires every wave's reads of the
// pair before, whose buffer the DMA two pairs ahead then takes.  Every wait is a static vmcnt that
// assumes the source's VMEM issue order (s16_vm_after), fenced by sched_barrier; the CPU test
// tests/test_isa_waits.py replays the emitted order.
// ============================================================================================
constexpr int PANEL16 = 2 * PANEL;              // bytes of one (128-pixel tile, 32-deep chunk pair) panel
constexpr int NCP = 8;                          // chunk pairs at D = 256
constexpr int S16NB = 4;                        // LDS buffers (chunk pairs) of the target panel
constexpr int S16COPIES = PANEL16 / 1024 / 4;   // LDS-DMA pieces per wave and pair (4)
constexpr int S16QL = 8;                        // query fragment loads per wave and pair
constexpr int S16LS = 144;                      // LDS bytes per level-0 line in the epilogue transpose
static_assert(S16NB * PANEL16 <= SLDS && 4 * 2 * 64 * S16LS <= SLDS, "split16 LDS regions");

// target (y, x) of position p of a split16 fmap2 panel, relative to the n-tile origin: p = 16 tg +
// 4 kb + i lies in quadrant kb (regular: rows 4 (kb & 1) .., cols 8 (kb >> 1) ..; band: cols 8 kb ..)
// at quadrant row tg >> 1, column 4 (tg & 1) + i
__host__ __device__ __forceinline__ void split16_target(int p, bool band, int& y, int& x) {
    const int tg = p >> 4, kb = (p >> 2) & 3, i = p & 3;
    if (!band) {
        y = 4 * (kb & 1) + (tg >> 1);
        x = 8 * (kb >> 1) + 4 * (tg & 1) + i;
    } else {
        y = tg >> 1;
        x = 8 * kb + 4 * (tg & 1) + i;
    }
}

// VMEM instructions a wave issues after the last piece of t(j) until the wait for t(j) (j >= 1: in
// mid(j - 1)).  Issue order: prologue t(0) .. t(S16NB - 2), q(0); pair c: q(c + 1) (c + 1 < NCP),
// then at its mid barrier (c + 1 < NCP) the wait for t(c + 1) and t(c + S16NB - 1) (< NCP).
constexpr int s16_vm_after(int j) {
    int n = 0;
    bool seen = false;
    for (int k = 0; k < S16NB - 1; ++k) {
        if (seen) n += S16COPIES;
        if (k == j) seen = true;
    }
    if (j == 0) return n + S16QL;   // the prologue's wait: t(1) .. t(NB - 2), q(0)
    n += seen ? S16QL : 0;          // q(0)
    for (int c = 0; c + 1 < NCP; ++c) {
        if (seen) n += S16QL;       // q(c + 1)
        if (c + 1 == j) return n;   // mid(c)
        const int k = c + S16NB - 1;
        if (k < NCP) {
            if (seen) n += S16COPIES;
            if (k == j) seen = true;
        }
    }
    return n;
}
static_assert(S16NB != 4 || S16COPIES != 4 || S16QL != 8 ||
                  (s16_vm_after(0) == 16 && s16_vm_after(1) == 20 && s16_vm_after(2) == 28 &&
                   s16_vm_after(3) == 20 && s16_vm_after(6) == 20 && s16_vm_after(7) == 16),
              "split16 wait counts (hand-checked for 4 buffers, 4 pieces, 8 query loads)");

// Epilogue of build_split16_kernel for one wave: its 64 queries (block-local qw .. qw + 63) x the
// n-tile tc from its accumulators acc[qg][tg]; xw = the wave's two LDS transpose regions (2 x 64
// lines x S16LS bytes).  It runs beside the partner block's K loop, whose MFMAs hold the SIMD's
// vector issue half the time, so its VALU count is the cost: every address is 32-bit and hoisted
// out of the query-group loop (the quadrant geometry is the lane's; only the query row changes),
// and the cross-lane steps are v_permlane16/32_swap.
// FULL (a whole 256-query tile whose first query row starts a 64-row group, as every tile of the
// BASELINE configs does): every store's query-row term is wave-uniform, so it rides in the scalar
// soffset and a lane's voffset is one constant per store kind (SOOB where its piece lies outside
// the level) -- no per-store address VALU, compare or select.
template <bool MUL, bool FULL>
__device__ __forceinline__ void split16_epilogue(const BuildParams& P, floatx4 (&acc)[4][8], char* const xw, int qw,
                                                 const int* exq, const int* ext, const float* fst, const NTile& tc,
                                                 int b, int q0, int lane) {
    const int qn = lane & 15, kb = lane >> 4;
    const int L = P.fused_levels;
    const int64_t rows0 = (int64_t)b * P.q_count + q0;   // the block's first query image
    const int nq = min(SQ, P.q_count - q0);
    const int64_t g0 = rows0 >> 6;
    auto rsrc_of = [&](int lv) {
        if (lv >= 1)
            return __builtin_amdgcn_make_buffer_rsrc(P.lvl[lv] + g0 * kGroup * P.lsz[lv], 0,
                                                     (int)((((rows0 + nq - 1) >> 6) - g0 + 1) * kGroup * P.lsz[lv] * 4),
                                                     0x00020000);
        return __builtin_amdgcn_make_buffer_rsrc(P.lvl[lv] + rows0 * P.lsz[lv], 0, (int)(nq * P.lsz[lv] * 4), 0x00020000);
    };
    const __amdgpu_buffer_rsrc_t r0 = rsrc_of(0);
    const __amdgpu_buffer_rsrc_t r1 = rsrc_of(L > 1 ? 1 : 0);
    const __amdgpu_buffer_rsrc_t r2 = rsrc_of(L > 2 ? 2 : 0);
    const __amdgpu_buffer_rsrc_t r3 = rsrc_of(L > 3 ? 3 : 0);
    // level-0 line (tile row, tile col) of quadrant k of the n-tile
    auto line_tr = [&](int k) { return (tc.ty0 >> 2) + (tc.band ? 0 : (k & 1)); };
    auto line_tc = [&](int k) { return (tc.tx0 >> 3) + (tc.band ? k : (k >> 1)); };
    // Level-0 transpose: lane l writes its line (query qn, quadrant kb) as line l of the region;
    // store instruction s then takes lines s + 8 j, j = 0..7 (queries s, s + 8 of every quadrant),
    // lane l piece pc of line s + 8 jl, with (jl, pc) chosen so that each 16-lane group of the
    // ds_read_b128 ({0-3, 12-15, 20-27}, {4-11, 16-19, 28-31}, +32) reads two lines 8 apart: all 64
    // banks (line stride 144 B = 36 dwords, 8 lines = 32 banks).
    int jl, pc;
    {
        const int l = lane & 31;
        const bool g1 = (l >= 4 && l < 12) || (l >= 16 && l < 20) || l >= 28;
        const bool second = g1 ? l >= 12 : l >= 16;
        pc = g1 ? (second ? (l < 20 ? l - 16 : l - 24) : l - 4) : (second ? l - 20 : (l < 4 ? l : l - 8));
        jl = 4 * (lane >> 5) + 2 * (g1 ? 1 : 0) + (second ? 1 : 0);
    }
    const int l0stride = (int)P.lsz[0] * 4;            // bytes per query image
    int l0off;                                          // this lane's piece of line s + 8 jl, query row qw + s (+ lq)
    bool l0ok;
    {
        const int lk = jl >> 1, ltr = line_tr(lk), ltc = line_tc(lk);
        l0ok = ltr < P.lnty[0] && ltc < P.lntx[0];
        l0off = (qw + (jl & 1 ? 8 : 0)) * l0stride + ((ltr * P.lntx[0] + ltc) * kTile) * 4 + 16 * pc;
    }
    const int l0q = qw + (jl & 1 ? 8 : 0);              // query row of store s = 0 (block-local)
    // Interleaved levels 1-3 ([group][block][row][bh][bw], ecorr_device.h): a piece of query row R
    // (block-local qloc) at byte (grp G + rin bsz + blkoff) 4, grp = (R >> 6) - g0, rin = R & 63,
    // G = kGroup lsz floats per group, bsz = block floats; blkoff = block index kGroup bsz + the
    // piece's in-block offset (the lane's; -1 = outside the level)
    const int rl0 = (int)(rows0 & (kGroup - 1));          // row-in-group of the block's first query
    auto ilv_blkoff = [&](int lv, int r, int c) {          // level pixel (r, c) -> blkoff, or -1
        const int sy = ilv_sy(lv), sx = ilv_sx(lv);
        const int by = r >> sy, bx = c >> sx;
        if (by >= P.lnty[lv] || bx >= -P.lntx[lv]) return -1;
        return (by * -P.lntx[lv] + bx) * kGroup * (1 << (sy + sx)) + ((r & ((1 << sy) - 1)) << sx) + (c & ((1 << sx) - 1));
    };
    // level 1: after the row swap, lane kb holds block row kb & 1 of quadrants kb & ~1 (x) and kb | 1 (y)
    const int b1x = L > 1 ? ilv_blkoff(1, 2 * line_tr(kb & ~1) + (kb & 1), 4 * line_tc(kb & ~1)) : -1;
    const int b1y = L > 1 ? ilv_blkoff(1, 2 * line_tr(kb | 1) + (kb & 1), 4 * line_tc(kb | 1)) : -1;
    // level 2: the quadrant's 1 x 2 pixels at (line_tr, 2 line_tc)
    const int b2 = L > 2 ? ilv_blkoff(2, line_tr(kb), 2 * line_tc(kb)) : -1;
    // level 3 (regular tiles, stored by the kb = 0 lanes): the tile's 1 x 2 at (ty0 / 8, tx0 / 8)
    const int b3 = (L > 3 && !tc.band && kb == 0) ? ilv_blkoff(3, tc.ty0 >> 3, tc.tx0 >> 3) : -1;
    const int G1 = kGroup * (int)P.lsz[L > 1 ? 1 : 0], G2 = kGroup * (int)P.lsz[L > 2 ? 2 : 0],
              G3 = kGroup * (int)P.lsz[L > 3 ? 3 : 0];
    auto st4 = [&](__amdgpu_buffer_rsrc_t rs, int off, bool ok, floatx4 v) {
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(uint4v, v), rs, ok ? off : SOOB, 0, ST_L01);
    };
    auto st2 = [&](__amdgpu_buffer_rsrc_t rs, int off, bool ok, floatx2 v) {
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(uint2v, v), rs, ok ? off : SOOB, 0, ST_L01);
    };
    // FULL: lane-constant offsets (query-row term qn of the 16-query group, the lane's piece; FOOB
    // where the piece lies outside the level) plus a wave-uniform term (qg, the store, the wave's
    // 64-row group = its index: rl0 == 0) -- one v_add per store.  The uniform term stays in the
    // voffset, soffset 0: with it in an SGPR soffset hipcc omits the wait state a 16-byte store needs
    // before a VALU overwrites its data VGPRs (LLVM assumes that hazard only without an soffset
    // register), and such a store wrote the next VALU's value (round 3's "lost" rows; round 5,
    // tools/soff_repro.py; guarded by tests/test_isa_store_hazard.py).
    constexpr int FOOB = 0x70000000;   // + any uniform term stays beyond every slab, below 2^31
    const int qwu = __builtin_amdgcn_readfirstlane(qw);   // wave-uniform (qw = 64 wave)
    const int v0 = l0ok ? l0off - qw * l0stride : FOOB;   // + (qw + 16 qg + s) l0stride
    const int v1x = b1x >= 0 ? (qn * 8 + b1x) * 4 : FOOB, v1y = b1y >= 0 ? (qn * 8 + b1y) * 4 : FOOB;
    const int v2 = b2 >= 0 ? (qn * 8 + b2) * 4 : FOOB, v3 = b3 >= 0 ? (qn * 2 + b3) * 4 : FOOB;
    const int grpw = qwu >> 6;   // FULL: the wave's interleaved group (block-relative)
    auto fst4 = [&](__amdgpu_buffer_rsrc_t rs, int voff, int uoff, floatx4 v) {
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(uint4v, v), rs, voff + uoff, 0, ST_L01);
    };
    auto fst2 = [&](__amdgpu_buffer_rsrc_t rs, int voff, int uoff, floatx2 v) {
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(uint2v, v), rs, voff + uoff, 0, ST_L01);
    };
    // fast scale: every exponent of the wave's queries and of the panel's targets in [-63, 63]
    bool fast_scale;
    {
        const int n = -(exq[qw + lane] + (MUL ? P.scale_shift : 0));
        fast_scale = __all(ext[lane] >= -63 && ext[lane] <= 63 && ext[lane + 64] >= -63 && ext[lane + 64] <= 63 &&
                           n >= -63 && n <= 63);
    }
#pragma unroll
    for (int qg = 0; qg < 4; ++qg) {
        const int ql = qw + 16 * qg;   // block-local first query of the group
        const int nqe = -(exq[ql + qn] + (MUL ? P.scale_shift : 0));
        // v[tg][i] = quadrant pixel (tg >> 1, 4 (tg & 1) + i) of query ql + qn, quadrant kb
        float v[8][4];
        if (fast_scale) {
            // x = acc 2^nqe 2^ext: exact power-of-two products, as v_pk_mul_f32 pairs (the
            // library is built without SLP vectorization, which packed the pooling adds at two
            // v_mov each; packing is spelled out where it pays)
            const float sq = exp2i(nqe);
            const floatx2 sq2 = {sq, sq};
#pragma unroll
            for (int tg = 0; tg < 8; ++tg) {
                const floatx4 s4 = *reinterpret_cast<const floatx4*>(fst + 16 * tg + 4 * kb);
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const floatx2 x = floatx2{acc[qg][tg][2 * h], acc[qg][tg][2 * h + 1]} *
                                      (sq2 * floatx2{s4[2 * h], s4[2 * h + 1]});
                    v[tg][2 * h] = MUL ? x[0] : __fdiv_rn(x[0], P.scale);
                    v[tg][2 * h + 1] = MUL ? x[1] : __fdiv_rn(x[1], P.scale);
                }
            }
        } else {
#pragma unroll
            for (int tg = 0; tg < 8; ++tg) {
                const int4 e4 = *reinterpret_cast<const int4*>(ext + 16 * tg + 4 * kb);
                const int e[4] = {e4.x, e4.y, e4.z, e4.w};
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const float x = ldexpf(acc[qg][tg][i], nqe + e[i]);
                    v[tg][i] = MUL ? x : __fdiv_rn(x, P.scale);
                }
            }
        }
        // level 0: the line through the region (a wave's LDS accesses are processed in order, so
        // group qg + 2's writes cannot overtake group qg's reads of the same region)
        // (stored straight from the lanes instead -- 16-byte pieces of 64 lines per instruction --
        // the same pyramid took 4.8 ms and wrote 5.4 GB: profiles/r03_lab/r3h_*)
        char* const xr = xw + (qg & 1) * (64 * S16LS);
#pragma unroll
        for (int tg = 0; tg < 8; ++tg)
            *reinterpret_cast<floatx4*>(xr + lane * S16LS + 16 * tg) = floatx4{v[tg][0], v[tg][1], v[tg][2], v[tg][3]};
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            const floatx4 x = *reinterpret_cast<const floatx4*>(xr + (s + 8 * jl) * S16LS + 16 * pc);
            if (FULL) fst4(r0, v0, (qwu + 16 * qg + s) * l0stride, x);
            else st4(r0, l0off + (16 * qg + s) * l0stride, l0ok && l0q + 16 * qg + s < nq, x);
        }
        if (L < 2) continue;
        // this lane's query row in its interleaved group
        const int rr = rl0 + ql + qn;
        const int grp = rr >> 6, rin = rr & (kGroup - 1);
        const bool qok = ql + qn < nq;
        // level 1: the quadrant's 2 x 4 block, l1[r][c] from quadrant rows 2r, 2r + 1, cols 2c, 2c + 1
        auto q0v = [&](int yy, int xx) { return v[2 * yy + (xx >> 2)][xx & 3]; };
        float l1[2][4];
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
            for (int c = 0; c < 4; ++c)
                l1[r][c] = pool4(q0v(2 * r, 2 * c), q0v(2 * r, 2 * c + 1), q0v(2 * r + 1, 2 * c), q0v(2 * r + 1, 2 * c + 1));
        float l2[2];
        if (L >= 3) {
#pragma unroll
            for (int c = 0; c < 2; ++c) l2[c] = pool4(l1[0][2 * c], l1[0][2 * c + 1], l1[1][2 * c], l1[1][2 * c + 1]);
        }
        // level-1 stores: one swap of 16-lane rows (kb odd rows <-> kb even rows) leaves lane kb with
        // block row kb & 1 of the blocks of quadrants kb & ~1 (x) and kb | 1 (y): per instruction,
        // 16 queries x 32 B contiguous per block, two blocks
        {
            float x[4], y[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(l1[0][c]), __float_as_uint(l1[1][c]), false, false);
                x[c] = __uint_as_float(sw[0]);
                y[c] = __uint_as_float(sw[1]);
            }
            if (FULL) {
                fst4(r1, v1x, (grpw * G1 + 16 * qg * 8) * 4, floatx4{x[0], x[1], x[2], x[3]});
                fst4(r1, v1y, (grpw * G1 + 16 * qg * 8) * 4, floatx4{y[0], y[1], y[2], y[3]});
            } else {
                const int base1 = grp * G1 + rin * 8;
                st4(r1, (base1 + b1x) * 4, qok && b1x >= 0, floatx4{x[0], x[1], x[2], x[3]});
                st4(r1, (base1 + b1y) * 4, qok && b1y >= 0, floatx4{y[0], y[1], y[2], y[3]});
            }
        }
        if (L < 3) continue;
        // level 2: 4 lanes x 8 B = one query's 2 x 4 block (band: half of two)
        if (FULL) fst2(r2, v2, (grpw * G2 + 16 * qg * 8) * 4, floatx2{l2[0], l2[1]});
        else st2(r2, (grp * G2 + rin * 8 + b2) * 4, qok && b2 >= 0, floatx2{l2[0], l2[1]});
        if (L < 4 || tc.band) continue;
        // level 3 (regular tiles): pixel kb >> 1 of the tile's 1 x 2 from the 2 x 2 level-2 pixels of
        // lanes kb (row 0, kb even) and kb + 1 (row 1), brought over by a row swap; lane kb = 0 takes
        // pixel 1 from kb = 2 by a half swap and stores both
        const auto o0 = __builtin_amdgcn_permlane16_swap(__float_as_uint(l2[0]), __float_as_uint(l2[0]), false, false);
        const auto o1 = __builtin_amdgcn_permlane16_swap(__float_as_uint(l2[1]), __float_as_uint(l2[1]), false, false);
        const float p3 = pool4(l2[0], l2[1], __uint_as_float(o0[1]), __uint_as_float(o1[1]));
        const auto p3s = __builtin_amdgcn_permlane32_swap(__float_as_uint(p3), __float_as_uint(p3), false, false);
        if (FULL) fst2(r3, v3, (grpw * G3 + 16 * qg * 2) * 4, floatx2{p3, __uint_as_float(p3s[1])});
        else st2(r3, (grp * G3 + rin * 2 + b3) * 4, qok && b3 >= 0, floatx2{p3, __uint_as_float(p3s[1])});
    }
}

template <bool MUL>
__global__ __launch_bounds__(256, 2) void build_split16_kernel(BuildParams P) {
    // ALL LDS in this one array (cdna_hip_programming.md trap 4(a), see build_split_kernel)
    __shared__ __attribute__((aligned(16))) char smem[SLDS + (SQ + 256) * 4];
    int* exq = reinterpret_cast<int*>(smem + SLDS);   // exponents of the 256 queries
    int* ext = exq + SQ;                              // ... negated, of the 128 panel targets
    float* fst = reinterpret_cast<float*>(ext + 128);  // 2^ext when |ext| <= 63

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    int b, qt, nt;
    decode_tile<kGM16, true>(P, xcd_remap(blockIdx.x, gridDim.x), P.n_qt, b, qt, nt);
    const NTile tc = ntile_of(P, nt);
    const int q0 = qt * SQ;
    const int H = P.H, W = P.W;
    const int64_t Q = (int64_t)H * W;

    // per-pixel exponents: loaded behind the K loop's last static wait (only the epilogue reads them)
    int eq = 0, et = 0;
    auto load_exponents = [&]() {
        eq = q0 + tid < P.q_count ? P.ex1[(int64_t)b * P.q_count + q0 + tid] : 0;
        if (tid < 128) {
            int y, x;
            split16_target(tid, tc.band, y, x);
            y += tc.ty0;
            x += tc.tx0;
            et = (y < H && x < W) ? P.ex2[(int64_t)b * Q + (int64_t)y * W + x] : 0;   // negated after the loop
        }
    };

    const int64_t pstride = (int64_t)NCP * PANEL16;   // bytes of one 128-pixel tile's panels
    const int qp = 2 * qt;
    const int nqp = min(2, P.n_mt - qp);
    const __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<char*>(P.pk1 + ((int64_t)b * P.n_mt + qp) * pstride), 0, (int)(nqp * pstride), 0x00020000);
    const __amdgpu_buffer_rsrc_t rt = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<char*>(P.pk2 + ((int64_t)b * P.n_nt + nt) * pstride), 0, (int)pstride, 0x00020000);
    // target panel of pair cp: DMA piece c = wave + 4 s of its 16 KB (lane-linear); the pair and
    // piece offsets ride in the scalar soffset, so one VGPR addresses every piece of the loop
    const int tvo = wave * 1024 + lane * 16;
    auto issue = [&](int cp) {
        char* dst = smem + (cp % S16NB) * PANEL16;
#pragma unroll
        for (int s = 0; s < S16COPIES; ++s)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rt, (__attribute__((address_space(3))) void*)(dst + (wave + 4 * s) * 1024),
                                                     16, tvo, cp * PANEL16 + s * 4096, 0, 0);
    };

    floatx4 acc[4][8];
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int t = 0; t < 8; ++t) acc[g][t] = floatx4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int t = 0; t < 8; ++t) asm volatile("" : "+v"(acc[g][t]));

    // query fragments of the wave's 4 groups (panel wave / 2, 16-query groups 4 (wave & 1) + g), one pair
    struct QF { halfx8 h[4], l[4]; };
    const int qgo = (wave >> 1) * (int)pstride + (wave & 1) * (4 * 2048) + lane * 16;
    auto load_q = [&](int cp, QF& q) {   // (pair, group) offset in the scalar soffset
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            q.h[g] = __builtin_bit_cast(halfx8, __builtin_amdgcn_raw_buffer_load_b128(rq, qgo, cp * PANEL16 + g * 2048, 0));
            q.l[g] = __builtin_bit_cast(halfx8, __builtin_amdgcn_raw_buffer_load_b128(rq, qgo + 1024, cp * PANEL16 + g * 2048, 0));
        }
    };
    // target fragments of group tg from LDS (lane-linear ds_read_b128, conflict-free)
    struct AF { halfx8 h, l; };
    auto read_a = [&](int cp, int tg, AF& a) {
        const char* p = smem + (cp % S16NB) * PANEL16 + tg * 2048 + lane * 16;
        a.h = *reinterpret_cast<const halfx8*>(p);
        a.l = *reinterpret_cast<const halfx8*>(p + 1024);
    };
    // per element and pair: hi*hi, lo*hi, hi*lo.  Inline asm with the accumulator constrained to
    // VGPRs at every MFMA (gfx950's register file is unified: 128 accumulator VGPRs + the loop's
    // ~100 fit the 256 of two waves per SIMD, and the epilogue's VALU then reads them without 128
    // v_accvgpr_read per wave); with
    // the builtin, hipcc renames accumulator tiles between AGPRs and VGPRs inside the loop
    // (v_accvgpr copies, 48 spilled VGPRs).  Its waitcnt pass still covers the fragment operands.
    auto mfma = [&](floatx4& c, const halfx8& a, const halfx8& bq) {
        asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(bq));
    };
    // order: hh, lh per query group, then hl x4 -- every accumulator sums its three terms in the
    // same order (hh, lh, hl) wherever its queries sit, so a query-row slab build stays bitwise the
    // whole build (test_split_query_slab_matches_whole).  Round-3 A/B (same instructions and sums):
    // hh x4, lh x4, hl x4 605.9 us -> this order 597.7 us.  A Gray walk over the operand pairs
    // (every MFMA changing one operand of the one before) timed 1% faster again but summed the terms
    // in an order that depends on the query group's parity: not kept.
    auto mfma_tg = [&](const AF& a, const QF& q, int tg) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            mfma(acc[g][tg], a.h, q.h[g]);
            mfma(acc[g][tg], a.l, q.h[g]);
        }
#pragma unroll
        for (int g = 0; g < 4; ++g) mfma(acc[g][tg], a.h, q.l[g]);
    };
#define PHASE __builtin_amdgcn_sched_barrier(0)
    QF qs[2];
    AF af[2];
#pragma unroll
    for (int k = 0; k < S16NB - 1; ++k) {
        issue(k);
        PHASE;
    }
    load_q(0, qs[0]);
    PHASE;
    wait_vm_n<true>(s16_vm_after(0));   // t(0) landed
    __builtin_amdgcn_s_barrier();
    PHASE;
    read_a(0, 0, af[0]);
    PHASE;
#pragma unroll
    for (int cp = 0; cp < NCP; ++cp) {
        if (cp + 1 < NCP) load_q(cp + 1, qs[(cp + 1) & 1]);
        PHASE;
#pragma unroll
        for (int tg = 0; tg < 8; ++tg) {
            if (tg == 6 && cp + 1 < NCP) {   // mid(cp): publish t(cp + 1), retire the reads of t(cp - 1)
                wait_vm_n<true>(s16_vm_after(cp + 1));
                __builtin_amdgcn_s_barrier();
                PHASE;
                if (cp + S16NB - 1 < NCP) issue(cp + S16NB - 1);
                if (cp + 2 == NCP) load_exponents();   // after the last static wait
                PHASE;
            }
            if (tg + 1 < 8) read_a(cp, tg + 1, af[(tg + 1) & 1]);
            else if (cp + 1 < NCP) read_a(cp + 1, 0, af[0]);
            PHASE;
            mfma_tg(af[tg & 1], qs[cp & 1], tg);
            PHASE;
        }
    }
#undef PHASE
    // the last MFMAs' results are read by the epilogue's VALU: the hazard recognizer does not see
    // into the asm, so pad the XDL write -> VALU read distance explicitly
    asm volatile("s_nop 15");
    asm volatile("s_nop 15");
    wait_vm<0, true>();   // the exponents have landed and this wave's reads are done ...
    exq[tid] = eq;
    if (tid < 128) {
        ext[tid] = -et;
        fst[tid] = exp2i(max(-63, min(-et, 63)));
    }
    __syncthreads();      // ... in every wave: the panel buffers are the epilogue's scratch
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int t = 0; t < 8; ++t) asm volatile("" : "+v"(acc[g][t]));
    // FULL: a whole query tile starting a 64-row group (block-uniform)
    if (q0 + SQ <= P.q_count && (((int64_t)b * P.q_count + q0) & (kGroup - 1)) == 0)
        split16_epilogue<MUL, true>(P, acc, smem + wave * (2 * 64 * S16LS), wave * 64, exq, ext, fst, tc, b, q0, lane);
    else
        split16_epilogue<MUL, false>(P, acc, smem + wave * (2 * 64 * S16LS), wave * 64, exq, ext, fst, tc, b, q0, lane);
}

// ============================================================================================
// fp32 GEMM for D = 256 (ecorr_build): build_split_kernel's structure -- 256 x 128 block tile, 4
// waves of 64 queries x 128 targets, two blocks per CU, the register epilogue split_epilogue() --
// on v_mfma_f32_32x32x2_f32 with the fp32 operands read straight from the fmaps (no operand pass):
//   targets: chunk kc (16 k rows) goes global -> LDS by LDS-DMA as [k][128 targets in split_target
//     order] (8 KB; a lane copies 4 adjacent pixels of one row, 16 bytes, so W % 4 == 0); the A
//     fragment of group j, k-step s is one ds_read_b32 (lane (t, kh): target 32 j + t, k 2 s + kh);
//   queries: the B fragment (lane (q, kh): query 32 i + q of the wave, k 2 s + kh) is one dword
//     load per (i, s) from fmap1 [D][q_count] (a lane pair's 32 queries: two whole 128-byte rows).
// Per element the k order is that of the fp32 build_kernel (chunks, k-steps, the MFMA's own k pair:
// an exact k-ordered fmaf chain), so the pyramid is bitwise the same; the MFMA work per chunk (64
// instructions per wave) is 5.3x the split kernel's, so operand traffic no longer binds.
// ============================================================================================
constexpr int FDT = 3;    // target chunks ahead (LDS buffers)
constexpr int FDQ = 2;    // query chunks ahead (register sets)
constexpr int FQL = 16;   // query dword loads per wave and chunk (2 groups x 8 k-steps)

// VMEM instructions issued after t(j) when advance(j) waits for it (see split_vm_after)
constexpr int f32_vm_after(int j, int nk) {
    int n = 0;
    bool seen = false;
    for (int k = 0; k < FDT; ++k) {   // prologue: t(k) q(k)
        if (seen) n += SCOPIES;
        if (k == j) seen = true;
        if (k < FDQ && k < nk && seen) n += FQL;
    }
    for (int c = 0; c <= j - 2; ++c) {   // chunk c: t(c + FDT), q(c + FDQ)
        if (seen) n += SCOPIES;
        if (c + FDT == j) seen = true;
        if (c + FDQ < nk && seen) n += FQL;
    }
    return n;
}
// the waits as literals (hipcc does not fold the replay inside the unrolled loop):
// advance(j) waits with 18 younger ops for j = 1, 2, 16 and 34 for j = 3 .. 15; the prologue with 36
static_assert(f32_vm_after(0, 16) == 36 && f32_vm_after(1, 16) == 18 && f32_vm_after(2, 16) == 18 &&
                  f32_vm_after(3, 16) == 34 && f32_vm_after(15, 16) == 34 && f32_vm_after(16, 16) == 18,
              "fp32 loop wait counts");

template <bool MUL>
__global__ __launch_bounds__(256, 2) void build_f32_kernel(BuildParams P) {
    constexpr int NK = 16;
    __shared__ __attribute__((aligned(16))) char smem[SLDS + (SQ + 256) * 4];
    int* exq = reinterpret_cast<int*>(smem + SLDS);
    int* ext = exq + SQ;
    float* fst = reinterpret_cast<float*>(ext + 128);

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    int b, qt, nt;
    decode_tile<8, false>(P, xcd_remap(blockIdx.x, gridDim.x), P.n_qt, b, qt, nt);
    b = __builtin_amdgcn_readfirstlane(b);
    qt = __builtin_amdgcn_readfirstlane(qt);
    nt = __builtin_amdgcn_readfirstlane(nt);
    const NTile tc = ntile_of(P, nt);
    const int q0 = qt * SQ;
    const int H = P.H, W = P.W;
    const int64_t Q = (int64_t)H * W;
    // no operand scaling: zero exponents make split_epilogue's scale 1 / sqrt(D) alone
    exq[tid] = 0;
    if (tid < 128) {
        ext[tid] = 0;
        fst[tid] = 1.0f;
    }

    const __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(P.f1 + (int64_t)b * P.D * P.q_count), 0, (int)((int64_t)P.D * P.q_count * 4), 0x00020000);
    const __amdgpu_buffer_rsrc_t rt = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(P.f2 + (int64_t)b * P.D * Q), 0, (int)((int64_t)P.D * Q * 4), 0x00020000);
    // DMA piece c = wave + 4 s of a chunk: k rows 2c, 2c + 1; lane l copies targets 4 (l & 31) .. +3
    // of row 2c + (l >> 5) (4 adjacent pixels of one image row in split_target order)
    // per-lane byte offsets fixed for the whole loop (the row-dependent part rides in the scalar
    // soffset; a per-load select on the lane offset makes hipcc branch around every load)
    int tvo;   // the lane's 4 pixels in k row (lane >> 5), or out of range outside the image
    {
        int y, x;
        split_target(4 * (lane & 31), tc.band, y, x);
        y += tc.ty0;
        x += tc.tx0;
        tvo = (y < H && x < W) ? (int)(((lane >> 5) * Q + (int64_t)y * W + x) * 4) : SOOB;
    }
    auto issue = [&](int kc) {
        char* dst = smem + (kc % FDT) * SCHUNK;
#pragma unroll
        for (int s = 0; s < SCOPIES; ++s) {
            const int c = wave + 4 * s;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rt, (__attribute__((address_space(3))) void*)(dst + c * 1024), 16,
                                                     tvo, kc < NK ? (int)((16 * kc + 2 * c) * Q * 4) : SOOB, 0, 0);
        }
    };

    floatx16 acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) asm volatile("" : "+a"(acc[i][j]));

    // query fragments: lane (q, kh) of group i, k-step s = fmap1[16 kc + 2 s + kh][q0 + 64 wave + 32 i + q]
    struct QF { float v[2][8]; };
    const int kh = lane >> 5;
    int qvo[2];   // the lane's query in k row kh, or out of range past the slab
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int qq = q0 + 64 * wave + 32 * i + (lane & 31);
        qvo[i] = qq < P.q_count ? (int)(((int64_t)kh * P.q_count + qq) * 4) : SOOB;
    }
    auto load_q = [&](int kc, QF& q) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int s = 0; s < 8; ++s)
                q.v[i][s] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                    rq, qvo[i], (int)((int64_t)(16 * kc + 2 * s) * P.q_count * 4), 0));
    };
    // target fragments from LDS: group j, k-step s at (2 s + kh) * 512 + (32 j + t) * 4
    struct TF { float v[4][8]; };
    const int tfo = kh * 512 + (lane & 31) * 4;
    auto read_t = [&](int kc, TF& f, int s0) {
        const char* cb = smem + (kc % FDT) * SCHUNK + tfo;
#pragma unroll
        for (int s = s0; s < s0 + 4; ++s)
#pragma unroll
            for (int j = 0; j < 4; ++j) f.v[j][s] = *reinterpret_cast<const float*>(cb + s * 1024 + j * 128);
    };
    auto mfma_half = [&](const TF& f, const QF& q, int s0) {
#pragma unroll
        for (int s = s0; s < s0 + 4; ++s)
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(f.v[j][s], q.v[i][s], acc[i][j], 0, 0, 0);
    };
#define PHASE __builtin_amdgcn_sched_barrier(0)
    auto advance = [&](int j) {
        PHASE;
        if (j == 1 || j == 2 || j == NK) wait_vm<18, true>();
        else wait_vm<34, true>();
        __builtin_amdgcn_s_barrier();
        PHASE;
        issue(j + FDT - 1);
        PHASE;
    };
    TF f[2];
    QF qs[FDQ];
#pragma unroll
    for (int k = 0; k < FDT; ++k) {
        issue(k);
        PHASE;
        if (k < FDQ) load_q(k, qs[k]);
        PHASE;
    }
    wait_vm<36, true>();   // t(0) landed
    __builtin_amdgcn_s_barrier();
    PHASE;
    read_t(0, f[0], 0);
    read_t(0, f[0], 4);
    PHASE;
#pragma unroll
    for (int kc = 0; kc < NK; ++kc) {
        mfma_half(f[kc & 1], qs[kc % FDQ], 0);
        PHASE;
        advance(kc + 1);
        read_t(kc + 1, f[(kc + 1) & 1], 0);
        PHASE;
        mfma_half(f[kc & 1], qs[kc % FDQ], 4);
        PHASE;
        read_t(kc + 1, f[(kc + 1) & 1], 4);
        if (kc + FDQ < NK) load_q(kc + FDQ, qs[kc % FDQ]);
        PHASE;
    }
#undef PHASE
    wait_vm<0, true>();
    __builtin_amdgcn_s_barrier();   // every wave is done with the chunk buffers (epilogue scratch)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) asm volatile("" : "+a"(acc[i][j]));
    split_epilogue<MUL>(P, acc, smem + wave * (4 * 32 * XS), wave * 64, exq, ext, fst, tc, b, q0, lane);
}

// Split-mode operand pass: per pixel, ex = 15 - E with max_d |x| = f 2^E, f in [0.5, 1) (so the
// pixel's largest scaled value lies in [2^14, 2^15); 0 for all-zero or non-finite maxima, so NaN
// inputs propagate through the GEMM as in the reference), and the f16 split of all D values:
// x 2^ex = hi + lo + O(2^-22 |x|), hi = f16(x 2^ex), lo = f16(x 2^ex - hi) (the subtraction is
// exact; lo is exact for values down to 2^-10 of the pixel maximum and keeps 11 bits down to
// 2^-17 of it -- f16 subnormals below; tests/test_build_modes_gpu.py pins the error over those
// ranges).  Written as the build's 8-KB panels: panel (tile, chunk) = [32-row group g][hi k0-7 |
// hi k8-15 | lo k0-7 | lo k8-15][row r][8 halves], i.e. the v_mfma_f32_32x32x16_f16 operand of lane
// (r, h) is the 16 bytes at g*2048 + part*1024 + lane*16.  Positions without a pixel (ragged
// edges) and k >= D are zeros.  ISB = 0: fmap1 slab, tile = 128 consecutive queries; ISB = 1:
// fmap2, tile = the n-tile's targets in split_target order.  Block = 64 positions x 4 chunk
// quarters; the D <= 256 values of a thread stay in registers between the max and the split.
__device__ __forceinline__ void split_f16(const float (&v)[8], float s, halfx8& hi, halfx8& lo) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const float x = v[j] * s;
        const _Float16 h = (_Float16)x;
        hi[j] = h;
        lo[j] = (_Float16)(x - (float)h);
    }
}

// L16: the panel layout of build_split16_kernel (16 KB per 128-pixel tile and 32-deep chunk pair:
// [16-pixel group g][hi | lo][k block kb][pixel r][8 halves], k = 8 kb + j within the pair; fmap2
// positions in split16_target order) instead of build_split_kernel's 8-KB chunk panels.
template <bool ISB, bool L16>
__device__ __forceinline__ void pack_body(const float* __restrict__ x, const BuildParams& P, int* __restrict__ ex,
                                          char* __restrict__ pack) {
    __shared__ float red[4][64];
    const int b = blockIdx.y;
    int tile = blockIdx.x >> 1;
    int pos = (blockIdx.x & 1) * 64 + (threadIdx.x & 63);   // panel position of this lane's pixel
    const int qtr = threadIdx.x >> 6, D = P.D, dc = (D + 15) / 16;
    const int64_t N = ISB ? (int64_t)P.H * P.W : (int64_t)P.q_count;
    int64_t pix = -1;
    bool live = true;   // the lane owns a panel position (it writes its zeros too)
    if (!ISB) {
        const int64_t p = (int64_t)tile * 128 + pos;
        if (p < P.q_count) pix = p;
    } else {
        // lanes on 2 rows x 32 consecutive pixels (whole 128-byte lines of fmap2: an L2 miss
        // fetches the whole line, so 16-pixel row pieces read every line twice): regular blocks
        // cover rows 2 r4, 2 r4 + 1 of a pair of horizontally adjacent 8 x 16 n-tiles, band blocks
        // rows 2 h, 2 h + 1 of one 4 x 32 band tile; each lane goes to its n-tile's panel
        // position (split_target inverted)
        const int l = threadIdx.x & 63, npair = (P.n_ntx + 1) / 2, nreg_blk = 4 * (P.n_reg / P.n_ntx) * npair;
        int y, x;
        bool ok;
        if ((int)blockIdx.x < nreg_blk) {
            const int r4 = blockIdx.x & 3, pr = blockIdx.x >> 2, trow = pr / npair, col = 2 * (pr - trow * npair) + (l >> 4 & 1);
            ok = col < P.n_ntx;
            tile = trow * P.n_ntx + (ok ? col : 0);
            // L16: rows r4, r4 + 4, whose 16 pixels per n-tile row half complete two 16-position
            // groups of the panel (256-byte runs per store); otherwise rows 2 r4, 2 r4 + 1
            y = L16 ? r4 + 4 * (l >> 5) : 2 * r4 + (l >> 5);
            x = l & 15;
            pos = L16 ? 16 * (2 * (y & 3) + ((x >> 2) & 1)) + 4 * ((y >> 2) | ((x >> 3) << 1)) + (x & 3)
                      : 64 * (x >> 3) + 32 * (y >> 2) + 8 * (y & 3) + (x & 7);
        } else {
            const int bb = blockIdx.x - nreg_blk;
            tile = P.n_reg + (bb >> 1);
            ok = tile < P.n_nt;
            y = 2 * (bb & 1) + (l >> 5);
            x = l & 31;
            pos = L16 ? 16 * (2 * y + ((x >> 2) & 1)) + 4 * (x >> 3) + (x & 3) : 32 * (x >> 3) + 8 * y + (x & 7);
        }
        const NTile n = ntile_of(P, ok ? tile : 0);
        live = ok;
        if (ok && n.ty0 + y < P.H && n.tx0 + x < P.W) pix = (int64_t)(n.ty0 + y) * P.W + n.tx0 + x;
    }
    const float* px = x + (int64_t)b * D * N + (pix < 0 ? 0 : pix);
    constexpr int CPT = 4;
    const bool regs = dc <= 4 * CPT;
    float v[CPT][16];
    float m = 0.f;
    if (regs) {
#pragma unroll
        for (int i = 0; i < CPT; ++i)
#pragma unroll
            for (int kk = 0; kk < 16; ++kk) {
                const int k = (qtr + 4 * i) * 16 + kk;
                v[i][kk] = (pix >= 0 && k < D) ? px[(int64_t)k * N] : 0.f;
                m = fmaxf(m, fabsf(v[i][kk]));
            }
    } else if (pix >= 0) {
        for (int k = qtr * 16; k < D; k += 64)
#pragma unroll 4
            for (int kk = 0; kk < 16 && k + kk < D; ++kk) m = fmaxf(m, fabsf(px[(int64_t)(k + kk) * N]));
    }
    red[qtr][threadIdx.x & 63] = m;
    __syncthreads();
    const int l = threadIdx.x & 63;
    m = fmaxf(fmaxf(red[0][l], red[1][l]), fmaxf(red[2][l], red[3][l]));
    int E = 0;
    frexpf(m, &E);
    int e = (m > 0.f && m <= 3.4028235e38f) ? 15 - E : 0;
    e = e < -126 ? -126 : (e > 126 ? 126 : e);
    if (qtr == 0 && pix >= 0) ex[(int64_t)b * N + pix] = e;
    const float s = exp2i(e);
    const int ntiles = ISB ? P.n_nt : P.n_mt;
    char* pan = pack + ((int64_t)b * ntiles + tile) * dc * PANEL +
                (L16 ? (pos >> 4) * 2048 + (pos & 15) * 16 : (pos >> 5) * 2048 + (pos & 31) * 16);
    auto put = [&](int c, const float (&w)[16]) {
        halfx8 h0, l0, h1, l1;
        split_f16(*reinterpret_cast<const float(*)[8]>(w), s, h0, l0);
        split_f16(*reinterpret_cast<const float(*)[8]>(w + 8), s, h1, l1);
        // L16: chunk c is k blocks 2 (c & 1), 2 (c & 1) + 1 of chunk pair c / 2
        char* p = L16 ? pan + (int64_t)(c >> 1) * 2 * PANEL + (c & 1) * 512 : pan + (int64_t)c * PANEL;
        const int k8 = L16 ? 256 : 512;   // the next 8 k
        *reinterpret_cast<halfx8*>(p) = h0;
        *reinterpret_cast<halfx8*>(p + k8) = h1;
        *reinterpret_cast<halfx8*>(p + 1024) = l0;
        *reinterpret_cast<halfx8*>(p + 1024 + k8) = l1;
    };
    if (!live) return;   // (after the block's only barrier)
    if (regs) {
#pragma unroll
        for (int i = 0; i < CPT; ++i)
            if (qtr + 4 * i < dc) put(qtr + 4 * i, v[i]);
        return;
    }
    for (int c = qtr; c < dc; c += 4) {
        float w[16];
#pragma unroll
        for (int kk = 0; kk < 16; ++kk) {
            const int k = c * 16 + kk;
            w[kk] = (pix >= 0 && k < D) ? px[(int64_t)k * N] : 0.f;
        }
        put(c, w);
    }
}

// Both operand passes in ONE launch: grid (2 * max(n_mt, n_nt), B, 2), z = 0 packs fmap1 (128-query
// tiles), z = 1 fmap2 (n-tiles).  Neither pass alone fills the chip; one grid overlaps the two and
// drops a launch boundary (round-1 A/B, profiles/r01_final8/ab_pack.txt).  Surplus x blocks of the
// shorter pass return at once (block-uniform, before pack_body's barrier).
template <bool L16>
__global__ __launch_bounds__(256) void pack_both_kernel(BuildParams P) {
    if (blockIdx.z == 0) {
        if ((int)blockIdx.x < 2 * P.n_mt) pack_body<false, L16>(P.f1, P, P.ex1, const_cast<char*>(P.pk1));
    } else if ((int)blockIdx.x < 4 * (P.n_reg / P.n_ntx) * ((P.n_ntx + 1) / 2) + 2 * (P.n_nt - P.n_reg)) {
        pack_body<true, L16>(P.f2, P, P.ex2, const_cast<char*>(P.pk2));
    }
}

// ============================================================================================
// fp32 GEMM (ecorr_build).  Block tile 128 queries x one 8 x 16 (or 4 x 32 band) target block,
// K staged 16 deep; 4 waves of 64 x 64 = 2 x 2 v_mfma_f32_32x32x2_f32 tiles, 3 blocks per CU.
// GLDS: the K chunks go global -> LDS directly (buffer_load_dwordx4 ... lds, whose range check
// zero-fills the padding) through 3 buffers with two chunks in flight; otherwise (ragged shapes,
// operands beyond the 31-bit buffer range) float4 / scalar register staging, double-buffered.
// The C tile passes through LDS in two 64-query halves; the epilogue pools each (query, 8 x 8
// block) in registers and leaves as whole tiles (levels 0-1) and row pieces (levels 2-3).
// ============================================================================================
constexpr int BM = 128;             // queries per block tile
constexpr int BN = TBH * TBW;       // 128 targets
constexpr int NT = 256;             // threads
constexpr int KB = 16;              // K chunk
constexpr int MR = BM / 2;          // C-tile rows per half
constexpr int CS = BN + 4;          // C-tile LDS row stride (floats): conflict-free ds_read_b128
constexpr int P1S = 36, P2S = 12;   // LDS per-query strides of the pooled staging (conflict-free)
constexpr int FNBUF = 3;
constexpr int FSM = (FNBUF * KB * (BM + BN) > MR * CS) ? FNBUF * KB * (BM + BN) : MR * CS;

template <typename V>
__device__ __forceinline__ void st_nt(V* p, V v) { __builtin_nontemporal_store(v, p); }

struct TileCoord { int b, m0, ty0, tx0, band; };

// Epilogue of a regular tile (all threads; contains barriers).  Cs = scaled C-tile rows ([m][n],
// stride CS, n = ty*16 + tx) of MR of the block's queries starting at mlo.  Level 0: 4 whole tiles
// per query; pooling: thread (query m, 8 x 8 block blk) reduces in registers 8x8 -> 4x4 -> 2x2 ->
// 1, each level from the rounded previous one, parks levels 1-3 in LDS, then level 1 leaves as
// one whole tile per query, level 2 as two 16-byte rows, level 3 as single pixels.
__device__ __forceinline__ void epilogue(const BuildParams& P, const TileCoord& tc, float* Cs, int tid, int mlo) {
    const int64_t row0 = (int64_t)tc.b * P.q_count + tc.m0 + mlo;
    const int mvalid = min(MR, P.q_count - tc.m0 - mlo);
    {   // level 0
        const int ntx = P.lntx[0], nty = P.lnty[0];
        const int tr0 = tc.ty0 / kTileH, tc0 = tc.tx0 / kTileW;
#pragma unroll 4
        for (int s = 0; s < (MR * 32) / NT; ++s) {
            const int idx = tid + NT * s;
            const int m = idx >> 5, rem = idx & 31;
            const int trl = rem >> 4, tcl = (rem >> 3) & 1, j = rem & 7;
            const int tr = tr0 + trl, tcc = tc0 + tcl;
            if (m < mvalid && tr < nty && tcc < ntx) {
                const floatx4 v = *reinterpret_cast<const floatx4*>(
                    Cs + m * CS + (trl * 4 + (j >> 1)) * TBW + tcl * 8 + (j & 1) * 4);
                st_nt(reinterpret_cast<floatx4*>(P.lvl[0] + (row0 + m) * P.lsz[0] + (tr * ntx + tcc) * kTile + 4 * j), v);
            }
        }
    }
    if (P.fused_levels < 2) return;   // uniform over the block
    const bool pooler = tid < 2 * MR;
    const int m = tid % MR, blk = tid / MR;
    float l1[4][4], l2[2][2], l3 = 0.0f;
    if (pooler) {
        float v[8][8];
#pragma unroll
        for (int ty = 0; ty < 8; ++ty) {
            const floatx4 lo = *reinterpret_cast<const floatx4*>(Cs + m * CS + ty * TBW + blk * 8);
            const floatx4 hi = *reinterpret_cast<const floatx4*>(Cs + m * CS + ty * TBW + blk * 8 + 4);
#pragma unroll
            for (int j = 0; j < 4; ++j) { v[ty][j] = lo[j]; v[ty][4 + j] = hi[j]; }
        }
#pragma unroll
        for (int y = 0; y < 4; ++y)
#pragma unroll
            for (int x = 0; x < 4; ++x)
                l1[y][x] = pool4(v[2 * y][2 * x], v[2 * y][2 * x + 1], v[2 * y + 1][2 * x], v[2 * y + 1][2 * x + 1]);
#pragma unroll
        for (int y = 0; y < 2; ++y)
#pragma unroll
            for (int x = 0; x < 2; ++x)
                l2[y][x] = pool4(l1[2 * y][2 * x], l1[2 * y][2 * x + 1], l1[2 * y + 1][2 * x], l1[2 * y + 1][2 * x + 1]);
        l3 = pool4(l2[0][0], l2[0][1], l2[1][0], l2[1][1]);
    }
    __syncthreads();   // all reads of Cs done: reuse it for the pooled staging
    float* S1 = Cs;                       // [MR][4 rows][8 cols] = the level-1 tile, stride P1S
    float* S2 = Cs + MR * P1S;            // [MR][2 rows][4 cols], stride P2S
    float* S3 = S2 + MR * P2S;            // [MR][2 cols]
    if (pooler) {
#pragma unroll
        for (int y = 0; y < 4; ++y)
            *reinterpret_cast<floatx4*>(S1 + m * P1S + y * 8 + blk * 4) = floatx4{l1[y][0], l1[y][1], l1[y][2], l1[y][3]};
#pragma unroll
        for (int y = 0; y < 2; ++y)
            *reinterpret_cast<floatx2*>(S2 + m * P2S + y * 4 + blk * 2) = floatx2{l2[y][0], l2[y][1]};
        S3[m * 2 + blk] = l3;
    }
    __syncthreads();
    {   // level 1 (interleaved): rows ty0/2 .. +3, cols tx0/2 .. +7, 8 float4 block-row pieces per query
#pragma unroll
        for (int s = 0; s < (MR * 8) / NT; ++s) {
            const int idx = tid + NT * s;
            const int mm = idx >> 3, j = idx & 7;
            float* p = mm < mvalid ? level_px(P, 1, row0 + mm, tc.ty0 / 2 + (j >> 1), tc.tx0 / 2 + 4 * (j & 1)) : nullptr;
            if (p) st_nt(reinterpret_cast<floatx4*>(p), *reinterpret_cast<const floatx4*>(S1 + mm * P1S + 4 * j));
        }
    }
    if (P.fused_levels >= 3 && tid < 2 * MR) {   // level 2: rows ty0/4 + {0,1}, cols tx0/4 .. +3
        const int mm = tid >> 1, y = tid & 1;
        if (mm < mvalid) {
            const float* src = S2 + mm * P2S + y * 4;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                float* p = level_px(P, 2, row0 + mm, tc.ty0 / 4 + y, tc.tx0 / 4 + j);
                if (p) *p = src[j];
            }
        }
    }
    if (P.fused_levels >= 4 && tid < MR && tid < mvalid) {   // level 3: row ty0/8, cols tx0/8 .. +1
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            float* p = level_px(P, 3, row0 + tid, tc.ty0 / 8, tc.tx0 / 8 + j);
            if (p) *p = S3[tid * 2 + j];
        }
    }
}

// Epilogue of a band tile (4 target rows x 32 cols; n = ty*32 + tx).  Level 0: one tile row of
// 4 tiles per query.  Pooling: thread (query m, 4x8 block blk = 0..3) reduces 4x8 -> 2x4 -> 1x2 in
// registers (the reference's order, from the rounded previous level); level 1 leaves as two 8-float
// rows of two tiles, level 2 as single pixels.  No level-3 pixel draws on these rows.
__device__ __forceinline__ void epilogue_band(const BuildParams& P, const TileCoord& tc, float* Cs, int tid, int mlo) {
    const int64_t row0 = (int64_t)tc.b * P.q_count + tc.m0 + mlo;
    const int mvalid = min(MR, P.q_count - tc.m0 - mlo);
    {   // level 0: tile row ty0/4, tile cols tx0/8 .. +3
        const int ntx = P.lntx[0];
        const int tr = tc.ty0 / kTileH, tc0 = tc.tx0 / kTileW;
#pragma unroll 4
        for (int s = 0; s < (MR * 32) / NT; ++s) {
            const int idx = tid + NT * s;
            const int m = idx >> 5, rem = idx & 31;
            const int tcl = rem >> 3, j = rem & 7;
            if (m < mvalid && tc0 + tcl < ntx) {
                const floatx4 v = *reinterpret_cast<const floatx4*>(Cs + m * CS + (j >> 1) * 32 + tcl * 8 + (j & 1) * 4);
                st_nt(reinterpret_cast<floatx4*>(P.lvl[0] + (row0 + m) * P.lsz[0] + (tr * ntx + tc0 + tcl) * kTile + 4 * j), v);
            }
        }
    }
    if (P.fused_levels < 2) return;
    constexpr int NU = (4 * MR + NT - 1) / NT;   // (query, block) items per thread
    float l1[NU][2][4], l2[NU][2];
#pragma unroll
    for (int u = 0; u < NU; ++u) {
        const int it = tid + NT * u, m = it % MR, blk = it / MR;
        if (it < 4 * MR) {
            float v[4][8];
#pragma unroll
            for (int ty = 0; ty < 4; ++ty) {
                const floatx4 lo = *reinterpret_cast<const floatx4*>(Cs + m * CS + ty * 32 + blk * 8);
                const floatx4 hi = *reinterpret_cast<const floatx4*>(Cs + m * CS + ty * 32 + blk * 8 + 4);
#pragma unroll
                for (int j = 0; j < 4; ++j) { v[ty][j] = lo[j]; v[ty][4 + j] = hi[j]; }
            }
#pragma unroll
            for (int y = 0; y < 2; ++y)
#pragma unroll
                for (int x = 0; x < 4; ++x)
                    l1[u][y][x] = pool4(v[2 * y][2 * x], v[2 * y][2 * x + 1], v[2 * y + 1][2 * x], v[2 * y + 1][2 * x + 1]);
#pragma unroll
            for (int x = 0; x < 2; ++x)
                l2[u][x] = pool4(l1[u][0][2 * x], l1[u][0][2 * x + 1], l1[u][1][2 * x], l1[u][1][2 * x + 1]);
        }
    }
    __syncthreads();   // all reads of Cs done: reuse it for the pooled staging
    float* S1 = Cs;                 // [MR][2 rows][16 cols], stride P1S
    float* S2 = Cs + MR * P1S;      // [MR][8 cols], stride P2S
#pragma unroll
    for (int u = 0; u < NU; ++u) {
        const int it = tid + NT * u, m = it % MR, blk = it / MR;
        if (it < 4 * MR) {
#pragma unroll
            for (int y = 0; y < 2; ++y)
                *reinterpret_cast<floatx4*>(S1 + m * P1S + y * 16 + blk * 4) =
                    floatx4{l1[u][y][0], l1[u][y][1], l1[u][y][2], l1[u][y][3]};
            *reinterpret_cast<floatx2*>(S2 + m * P2S + blk * 2) = floatx2{l2[u][0], l2[u][1]};
        }
    }
    __syncthreads();
    {   // level 1 (interleaved): rows ty0/2 .. +1, cols tx0/2 .. +15, 8 float4 block-row pieces per query
#pragma unroll
        for (int s = 0; s < (MR * 8 + NT - 1) / NT; ++s) {
            const int idx = tid + NT * s;
            const int mm = idx >> 3, t = idx & 7;
            const int y = t >> 2, tcl = (t >> 1) & 1, hf = t & 1;
            float* p = mm < mvalid ? level_px(P, 1, row0 + mm, tc.ty0 / 2 + y, tc.tx0 / 2 + tcl * 8 + hf * 4) : nullptr;
            if (p)
                st_nt(reinterpret_cast<floatx4*>(p), *reinterpret_cast<const floatx4*>(S1 + mm * P1S + y * 16 + tcl * 8 + hf * 4));
        }
    }
    if (P.fused_levels >= 3 && tid < 2 * MR) {   // level 2: row ty0/4, cols tx0/4 .. +7
        const int mm = tid >> 1, hf = tid & 1;
        if (mm < mvalid) {
            const float* src = S2 + mm * P2S + hf * 4;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                float* p = level_px(P, 2, row0 + mm, tc.ty0 / 4, tc.tx0 / 4 + hf * 4 + j);
                if (p) *p = src[j];
            }
        }
    }
}

// VEC: float4 operand loads (W and q_count multiples of 4, 16-byte aligned fmaps); GLDS: LDS-DMA
// staging (needs VEC and byte offsets below 2^31).  A/B record: LDS-DMA 2.4-4% faster than
// register staging; 16x16x4 tiles 1% slower than 32x32x2; KB = 32 / 4 blocks per CU / setprio /
// k-permuted layouts / fragment prefetch all slower.
template <bool VEC, bool GLDS>
__global__ __launch_bounds__(NT, 3) void build_kernel(BuildParams P) {
    constexpr int AS = BM, BSS = BN;           // LDS row strides
    constexpr int NLD = (KB * BM / 4) / NT;    // float4 of A (and of B) per thread per chunk (2)
    constexpr int NBUF = GLDS ? FNBUF : 2;
    static_assert(!GLDS || VEC, "GLDS: vector path");
    __shared__ __attribute__((aligned(16))) float smem[FSM];
    float* As = smem;                       // [NBUF][KB][AS]
    float* Bs = smem + NBUF * KB * AS;      // [NBUF][KB][BSS]

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    TileCoord tc;
    {
        int mt, nt;
        decode_tile<8, false>(P, xcd_remap(blockIdx.x, gridDim.x), P.n_mt, tc.b, mt, nt);
        const NTile n = ntile_of(P, nt);
        tc.m0 = mt * BM;
        tc.ty0 = n.ty0;
        tc.tx0 = n.tx0;
        tc.band = n.band;
    }
    const int q_end = P.q_count;
    const int H = P.H, W = P.W, D = P.D;
    const int64_t Q = (int64_t)H * W;
    const int64_t QA = P.q_count;
    const float* __restrict__ A = P.f1 + (int64_t)tc.b * D * QA;
    const float* __restrict__ Bm = P.f2 + (int64_t)tc.b * D * Q;

    floatx4 ra[NLD], rb[NLD];
    auto load_chunk = [&](int k0) {
#pragma unroll
        for (int i = 0; i < NLD; ++i) {
            const int s = tid + NT * i;
            const int k = k0 + (s >> 5);
            {   // A: row k, queries m0 + 4c .. +3
                const int m = tc.m0 + 4 * (s & 31);
                floatx4 v = {0.f, 0.f, 0.f, 0.f};
                if (VEC) {
                    if (k < D && m < q_end) v = *reinterpret_cast<const floatx4*>(A + (int64_t)k * QA + m);
                } else {
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        if (k < D && m + j < q_end) v[j] = A[(int64_t)k * QA + m + j];
                }
                ra[i] = v;
            }
            {   // B: row k, target row ty0 + ty, cols tx0 + 4c .. +3 (LDS column 4r = ty*TBW + tx)
                const int r = s & 31;
                const int y = tc.ty0 + (tc.band ? r >> 3 : r >> 2), x = tc.tx0 + 4 * (tc.band ? r & 7 : r & 3);
                floatx4 v = {0.f, 0.f, 0.f, 0.f};
                if (VEC) {
                    if (k < D && y < H && x < W)
                        v = *reinterpret_cast<const floatx4*>(Bm + (int64_t)k * Q + (int64_t)y * W + x);
                } else {
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        if (k < D && y < H && x + j < W) v[j] = Bm[(int64_t)k * Q + (int64_t)y * W + x + j];
                }
                rb[i] = v;
            }
        }
    };
    auto store_chunk = [&](int buf) {
#pragma unroll
        for (int i = 0; i < NLD; ++i) {
            const int s = tid + NT * i;
            const int kk = s >> 5, c = s & 31;
            *reinterpret_cast<floatx4*>(As + (buf * KB + kk) * AS + 4 * c) = ra[i];
            *reinterpret_cast<floatx4*>(Bs + (buf * KB + kk) * BSS + 4 * c) = rb[i];
        }
    };

    floatx16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

    // MFMA 32x32x2 f32 operand maps: lane l holds A[i = l&31][k = l>>5] and B[k = l>>5][j = l&31]
    const int wm = wave & 1, wn = wave >> 1;
    const int arow = lane >> 5, acol = lane & 31;
    const int nk = (D + KB - 1) / KB;

    auto mfma_chunk = [&](int buf) {
        const float* as = As + buf * KB * AS + wm * 64 + acol;
        const float* bs = Bs + buf * KB * BSS + wn * 64 + acol;
#pragma unroll
        for (int kk = 0; kk < KB; kk += 2) {
            const int ro = kk + arow;
            const float a0 = as[ro * AS], a1 = as[ro * AS + 32];
            const float b0 = bs[ro * BSS], b1 = bs[ro * BSS + 32];
            acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
            acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
            acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
            acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
        }
    };

    if constexpr (GLDS) {
        // copy i of this wave covers chunk rows kk = 2 wave + 8 i + (lane >> 5), 4 floats at
        // column 4 (lane & 31): lane-linear 1 KB per wave-instruction, as LDS-DMA requires
        const __amdgpu_buffer_rsrc_t rsa =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(A), 0, (int)((int64_t)D * QA * 4), 0x00020000);
        const __amdgpu_buffer_rsrc_t rsb =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(Bm), 0, (int)((int64_t)D * Q * 4), 0x00020000);
        constexpr int OOB = 0x7ffffff0;   // beyond any operand: reads (and lands in LDS) as 0
        const int c = lane & 31, kl = lane >> 5;
        const int m = tc.m0 + 4 * c;
        const int y = tc.ty0 + (tc.band ? c >> 3 : c >> 2), x = tc.tx0 + 4 * (tc.band ? c & 7 : c & 3);
        const bool aok = m < q_end, bok = y < H && x < W;
        const int abase = m * 4, bbase = (y * W + x) * 4;
        auto issue = [&](int kc) {
            const int buf = kc % NBUF;
#pragma unroll
            for (int i = 0; i < NLD; ++i) {
                const int kk = 2 * wave + 8 * i;   // wave-uniform first row of this copy
                const int k = kc * KB + kk + kl;
                const bool kin = k < D;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    rsa, (__attribute__((address_space(3))) void*)(As + (buf * KB + kk) * AS), 16,
                    aok && kin ? abase + k * (int)QA * 4 : OOB, 0, 0, 0);
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    rsb, (__attribute__((address_space(3))) void*)(Bs + (buf * KB + kk) * BSS), 16,
                    bok && kin ? bbase + k * (int)Q * 4 : OOB, 0, 0, 0);
            }
        };
        for (int kc = 0; kc < NBUF - 1 && kc < nk; ++kc) issue(kc);
        for (int kc = 0; kc < nk; ++kc) {
            // this wave's copies of chunk kc have landed (those of chunk kc + 1 may still fly) ...
            if (kc + 1 < nk) wait_vm<2 * NLD, false>();
            else wait_vm<0, false>();
            // ... and every wave's have once all passed this barrier, which also retires the
            // reads of chunk kc - 1, whose buffer chunk kc + 2 now overwrites
            __builtin_amdgcn_s_barrier();
            if (kc + NBUF - 1 < nk) issue(kc + NBUF - 1);
            mfma_chunk(kc % NBUF);
        }
        __syncthreads();   // the C tile aliases the chunk buffers
    } else {
        load_chunk(0);
        store_chunk(0);
        __syncthreads();
        for (int kc = 0; kc < nk; ++kc) {
            const int buf = kc & 1;
            if (kc + 1 < nk) load_chunk((kc + 1) * KB);
            mfma_chunk(buf);
            if (kc + 1 < nk) store_chunk(buf ^ 1);
            __syncthreads();
        }
    }

    // ---- scaled accumulators -> LDS C tile [m][n] in two 64-query halves; C/D map:
    //      col = lane&31, row = (reg&3) + 8*(reg>>2) + 4*(lane>>5) ----
    float* Cs = smem;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
        if (wm == half) {
            // one uniform branch on the scale mode around the whole tile (a per-element select
            // had the compiler emit an IEEE division next to every element's multiply)
            auto write_c = [&](auto scaled) {
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j)
#pragma unroll
                        for (int r = 0; r < 16; ++r) {
                            const int m = i * 32 + (r & 3) + 8 * (r >> 2) + 4 * arow;
                            const int n = wn * 64 + j * 32 + acol;
                            Cs[m * CS + n] = scaled(acc[i][j][r]);
                        }
            };
            if (P.scale_is_mul) write_c([&](float v) { return __fmul_rn(v, P.scale); });
            else write_c([&](float v) { return __fdiv_rn(v, P.scale); });
        }
        __syncthreads();
        if (tc.band) epilogue_band(P, tc, Cs, tid, half * MR);
        else epilogue(P, tc, Cs, tid, half * MR);
        if (half == 0) __syncthreads();   // half 0 fully consumed before half 1 overwrites Cs
    }
}

// Levels beyond the 4 fused ones (num_levels > 4): plain 2x2 floor-mode pooling, tiled in and
// out, one thread per output pixel.  Not on the E-RAFT path (num_levels = 4, eraft.py:50).
__global__ __launch_bounds__(256) void pool2_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                    int64_t rows, int h, int w, int lv_in, int ntx_in, int64_t sz_in,
                                                    int ntx_out, int64_t sz_out) {
    const int ho = h / 2, wo = w / 2;
    const int64_t n = rows * ho * wo;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t rw = i / ((int64_t)ho * wo);
        const int yx = (int)(i - rw * ho * wo);
        const int y = yx / wo, x = yx - y * wo;
        auto at = [&](int yy, int xx) { return in[pix_off(rw, yy, xx, lv_in, ntx_in, w, sz_in)]; };
        out[rw * sz_out + level_off(y, x, ntx_out, wo)] =
            pool4(at(2 * y, 2 * x), at(2 * y, 2 * x + 1), at(2 * y + 1, 2 * x), at(2 * y + 1, 2 * x + 1));
    }
}

}  // namespace

namespace {
void tile_counts(BuildParams& P) {
    P.n_ntx = (P.W + TBW - 1) / TBW;
    // 8-row tile rows; a remainder of 1..4 rows (the last 8k + r rows, r <= 4) becomes a band of
    // 4 x 32 tiles (see ntile_of), a remainder of 5..7 a padded regular tile row
    const int rem = P.H % TBH;
    const bool band = rem > 0 && rem <= 4;
    P.n_reg = P.n_ntx * (band ? P.H / TBH : (P.H + TBH - 1) / TBH);
    P.band_y0 = (P.H / TBH) * TBH;
    P.n_nt = P.n_reg + (band ? (P.W + 31) / 32 : 0);
    P.n_mt = (P.q_count + BM - 1) / BM;      // 128-query tiles (fp32 blocks, fmap1 panels)
    P.n_qt = (P.q_count + SQ - 1) / SQ;      // 256-query tiles (split blocks)
}

// split workspace: exponents (fmap1 slab, fmap2), then fmap1 and fmap2 panels (256-B aligned)
struct SplitWs { int64_t ex2, pk1, pk2, total; };
SplitWs split_ws(const BuildParams& P, int B) {
    const int64_t dc = (P.D + 15) / 16;
    SplitWs w;
    w.ex2 = (int64_t)B * P.q_count * 4;
    w.pk1 = (w.ex2 + (int64_t)B * P.H * P.W * 4 + 255) & ~(int64_t)255;
    w.pk2 = w.pk1 + (int64_t)B * P.n_mt * dc * PANEL;
    w.total = w.pk2 + (int64_t)B * P.n_nt * dc * PANEL;
    return w;
}
}  // namespace

int64_t build_split_workspace_bytes(int B, int D, int H, int W, int q_count) {
    BuildParams P{};
    P.D = D;
    P.H = H;
    P.W = W;
    P.q_count = q_count;
    tile_counts(P);
    return split_ws(P, B).total;
}

int launch_build(const BuildParams& P0, int B, const PyrGeom& g, float* pyramid, hipStream_t stream, int stages) {
    BuildParams P = P0;
    const int levels = g.levels;
    P.fused_levels = levels < 4 ? levels : 4;
    tile_counts(P);
    for (int i = 0; i < 4; ++i) {
        const bool on = i < levels;
        P.lvl[i] = on ? pyramid + g.off[i] : nullptr;
        P.lh[i] = on ? g.h[i] : 0;
        P.lw[i] = on ? g.w[i] : 0;
        P.lntx[i] = on ? g.ntx[i] : 0;
        P.lnty[i] = on ? g.nty[i] : 0;
        P.lsz[i] = on ? g.sz[i] : 0;
    }
    if ((uintptr_t)pyramid % 16 != 0) return ECORR_EINVAL;   // tile stores are 16-byte vectors
    if (P.ws) {
        // split build: one 128-query tile's panels (dc * 8 KB, the buffer range of the kernel's
        // per-tile descriptors) always fit 31 bits for D < 2^22
        const int64_t ntiles = (int64_t)B * P.n_qt * P.n_nt;
        if (ntiles <= 0 || ntiles > 0x7fffffff || (int64_t)2 * ((P.D + 15) / 16) * PANEL >= 0x7fff0000LL)
            return ECORR_EINVAL;
        const SplitWs w = split_ws(P, B);
        P.ex1 = reinterpret_cast<int*>(P.ws);
        P.ex2 = reinterpret_cast<int*>(P.ws + w.ex2);
        P.pk1 = P.ws + w.pk1;
        P.pk2 = P.ws + w.pk2;
        const int nx2 = 4 * (P.n_reg / P.n_ntx) * ((P.n_ntx + 1) / 2) + 2 * (P.n_nt - P.n_reg);   // fmap2 blocks
        const int nx = 2 * P.n_mt > nx2 ? 2 * P.n_mt : nx2;
        // D = 256: build_split16_kernel and its panel layout; other D: build_split_kernel
        const bool s16 = (P.D + 15) / 16 == 2 * NCP;
        if (stages & 1) {
            if (s16) hipLaunchKernelGGL((pack_both_kernel<true>), dim3((unsigned)nx, B, 2), dim3(256), 0, stream, P);
            else hipLaunchKernelGGL((pack_both_kernel<false>), dim3((unsigned)nx, B, 2), dim3(256), 0, stream, P);
        }
        if (!(stages & 2)) {
            const hipError_t e = hipGetLastError();
            return e == hipSuccess ? ECORR_OK : ECORR_EHIP - (int)e;
        }
        const dim3 grid((unsigned)ntiles);
        if (s16) {
            if (P.scale_is_mul) hipLaunchKernelGGL((build_split16_kernel<true>), grid, dim3(256), 0, stream, P);
            else hipLaunchKernelGGL((build_split16_kernel<false>), grid, dim3(256), 0, stream, P);
        } else {
            if (P.scale_is_mul) hipLaunchKernelGGL((build_split_kernel<true, 0>), grid, dim3(256), 0, stream, P);
            else hipLaunchKernelGGL((build_split_kernel<false, 0>), grid, dim3(256), 0, stream, P);
        }
    } else {
        // D = 256 with 4-aligned rows and 31-bit operand offsets: the 256 x 128 fp32 kernel
        if (P.D == 256 && P.W % 4 == 0 && (uintptr_t)P.f2 % 16 == 0 && (int64_t)P.D * P.H * P.W * 4 < 0x7fff0000LL &&
            (int64_t)P.D * P.q_count * 4 < 0x7fff0000LL) {
            const int64_t nt2 = (int64_t)B * P.n_qt * P.n_nt;
            if (nt2 <= 0 || nt2 > 0x7fffffff) return ECORR_EINVAL;
            if (P.scale_is_mul) hipLaunchKernelGGL((build_f32_kernel<true>), dim3((unsigned)nt2), dim3(256), 0, stream, P);
            else hipLaunchKernelGGL((build_f32_kernel<false>), dim3((unsigned)nt2), dim3(256), 0, stream, P);
        } else {   // any D: the 128 x 128 fp32 kernel
            const int64_t ntiles = (int64_t)B * P.n_mt * P.n_nt;
            if (ntiles <= 0 || ntiles > 0x7fffffff) return ECORR_EINVAL;
            const bool vec = (P.W % 4 == 0) && (P.q_count % 4 == 0) && ((uintptr_t)P.f1 % 16 == 0) &&
                             ((uintptr_t)P.f2 % 16 == 0);
            // LDS-DMA staging whenever both operands' byte offsets fit the 31-bit buffer range
            const bool glds = vec && (int64_t)P.D * P.H * P.W * 4 < 0x7fff0000LL &&
                              (int64_t)P.D * P.q_count * 4 < 0x7fff0000LL;
            const dim3 grid((unsigned)ntiles), block(NT);
            if (glds) hipLaunchKernelGGL((build_kernel<true, true>), grid, block, 0, stream, P);
            else if (vec) hipLaunchKernelGGL((build_kernel<true, false>), grid, block, 0, stream, P);
            else hipLaunchKernelGGL((build_kernel<false, false>), grid, block, 0, stream, P);
        }
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return ECORR_EHIP - (int)e;
    const int64_t rows = (int64_t)B * P.q_count;
    for (int i = 4; i < levels; ++i) {
        const int64_t n = rows * g.h[i] * g.w[i];
        const int grid = (int)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
        hipLaunchKernelGGL(pool2_kernel, dim3(grid), dim3(256), 0, stream, pyramid + g.off[i - 1], pyramid + g.off[i],
                           rows, g.h[i - 1], g.w[i - 1], i - 1, g.ntx[i - 1], g.sz[i - 1], g.ntx[i], g.sz[i]);
        e = hipGetLastError();
        if (e != hipSuccess) return ECORR_EHIP - (int)e;
    }
    return ECORR_OK;
}

}  // namespace ecorr
