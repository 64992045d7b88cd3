// build.hip -- CorrBlock build on gfx950: all-pairs correlation GEMM on fp32 MFMA with the
// 1/sqrt(D) scale and the 3 pooled pyramid levels fused into the epilogue.
//
// Replaces corr.py:13-27 (CorrBlock.__init__) and corr.py:52-60 (CorrBlock.corr):
//   level0[b*q_count + p][y][x] = (sum_d f1[b][d][p] * f2[b][d][y*W+x]) / sqrt(D)
//   level{i+1} = (((x00 + x01) + x10) + x11) / 4 over 2x2 floor-mode windows of level i,
// stored in the tiled pyramid layout of include/ecorr.h (4 x 8-float tiles per query image).
//
// GEMM view per batch item: A = f1[b] as [K=D][M=q_count] (queries contiguous), B = f2[b] as
// [K][N=H*W].  Block tile: 128 queries x one 8x16 block of target pixels (N = 128), K staged 32
// deep through double-buffered LDS by float4 register staging; 4 waves, each 64x64 = 2x2
// v_mfma_f32_32x32x2_f32 tiles.  The N tile is a 2-D target block (2 x 2 pyramid tiles of level
// 0, exactly one tile of level 1), so the epilogue pools locally and every level-0/1 store is a
// whole 128-byte tile.
//
// Numerics: MFMA f32 is an exact k-ordered fmaf chain; the per-element k order does not depend on
// the tiling, so sharded and unsharded builds agree bit for bit.  Against the reference's sgemm
// level 0 agrees normwise (max|d|/rms <= 1e-5); pooling is bit-exact given the same level 0.
//
// A/B history (tools/ab_build.py): a k-permuted LDS layout with one ds_read_b128
// per 4 MFMA steps, persistent tiles, and two K chunks of loads in flight were all slower on
// MI355X; per-thread scattered epilogue stores cost 14%.
#include <stdlib.h>

#include "ecorr_device.h"
#include "ecorr_internal.h"

namespace ecorr {

namespace {

constexpr int BM = 128;           // queries per block tile
constexpr int TBH = 8, TBW = 16;  // target block (rows x cols) per block tile
constexpr int BN = TBH * TBW;     // 128 targets
constexpr int NT = 256;           // threads
constexpr int CS = BN + 4;        // C-tile LDS row stride (floats): conflict-free ds_read_b128
constexpr int P1S = 36, P2S = 12;  // LDS per-query strides of the pooled staging (conflict-free)

// LDS floats for K chunk KB (double-buffered A and B, row strides AS / BS) and a C tile of MR
// query rows.
constexpr int smem_floats(int KB, int MR, int AS, int BS, int NBUF = 2) {
    return NBUF * (KB * AS + KB * BS) > MR * CS ? NBUF * (KB * AS + KB * BS) : MR * CS;
}

// 16-byte pyramid store; NTS = non-temporal: the 2 GB pyramid is not re-read by this kernel, and
// streaming it past the caches took 5% off the build (tools/ab_build.py)
template <bool NTS, typename V>
__device__ __forceinline__ void st(V* p, V v) {
    if (NTS) __builtin_nontemporal_store(v, p);
    else *p = v;
}

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx2 __attribute__((ext_vector_type(2)));
typedef _Float16 halfx8 __attribute__((ext_vector_type(8)));

// Split mode: x * 2^e = hi + lo + O(2^-22 |x|), hi = f16(x 2^e), lo = f16(x 2^e - hi) (the
// subtraction is exact).  e puts the pixel's largest |value| in [2^14, 2^15), so hi never
// overflows and lo stays normal for all but values 2^17 below that maximum.
__device__ __forceinline__ void split_f16(const float (&v)[8], float s, halfx8& hi, halfx8& lo) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const float x = v[j] * s;
        const _Float16 h = (_Float16)x;
        hi[j] = h;
        lo[j] = (_Float16)(x - (float)h);
    }
}

// 2^e as a float, e in [-126, 127]
__device__ __forceinline__ float exp2i(int e) { return __int_as_float((e + 127) << 23); }

__device__ __forceinline__ float pool4(float a, float b, float c, float d) {
    return __fmul_rn(__fadd_rn(__fadd_rn(__fadd_rn(a, b), c), d), 0.25f);
}

// A tile covers 128 queries x 128 targets: a TBH x TBW = 8 x 16 target block (regular), or, in the
// last 4 rows when H % 8 is 1..4, a 4 x 32 block ("band"): those rows feed pyramid levels 0-2 only
// (level 3 of an H = 8k + r map, r <= 4, has k rows), so the band pools 4 x 8 sub-blocks and no
// 8-row tile row is padded half empty (DSEC H = 60: 6.7% of the MFMA work saved).
struct TileCoord { int b, m0, ty0, tx0, band, mt, nt; };

// Grouped tile order (8 m-tiles x all n-tiles per group): consecutive tiles share fmap panels.
__device__ __forceinline__ TileCoord decode_tile(const BuildParams& P, int t) {
    const int GM = P.gm;
    const int per_b = P.n_mt * P.n_nt;
    TileCoord c;
    c.b = t / per_b;
    const int i = t - c.b * per_b;
    const int gsz = GM * P.n_nt;
    const int grp = i / gsz, gi = i - grp * gsz;
    const int first_m = grp * GM;
    const int gsm = min(P.n_mt - first_m, GM);
    const int mt = first_m + gi % gsm, nt = gi / gsm;
    c.m0 = mt * BM;
    c.mt = mt;
    c.nt = nt;
    if (nt < P.n_reg) {
        const int nty = nt / P.n_ntx, ntx = nt - nty * P.n_ntx;
        c.ty0 = nty * TBH;
        c.tx0 = ntx * TBW;
        c.band = 0;
    } else {
        c.ty0 = P.band_y0;
        c.tx0 = (nt - P.n_reg) * 32;
        c.band = 1;
    }
    return c;
}

// Bijective XCD-aware remap (cdna_hip_programming.md §5 T1): consecutive logical tiles land on
// one XCD so tiles sharing fmap1/fmap2 panels share that XCD's L2.  Speed only, never correctness.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
    const int q = nwg / 8, r = nwg % 8, xcd = bid % 8, k = bid / 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + k;
}

// Epilogue (all threads; contains barriers).  Cs = scaled C-tile rows ([m][n], stride CS,
// n = ty*16 + tx) of MR of the block's queries (all 128, or one half of them).  Level 0: 4 whole tiles per query (two 256-byte pieces), 32 float4 per query.
// Pooling: thread (query m, 8x8 block blk) reduces in registers 8x8 -> 4x4 -> 2x2 -> 1, each level
// from the rounded previous one, parks levels 1-3 in LDS, then level 1 leaves as one whole tile
// per query, level 2 as two 16-byte rows, level 3 as 8 bytes.  Tiles beyond a level's padded
// extent are skipped; padding cells inside a tile are written but never read.
template <int MR, bool NTS>
__device__ __forceinline__ void epilogue(const BuildParams& P, const TileCoord& tc, float* Cs, int tid, int mlo) {
    // Cs holds C-tile rows [mlo, mlo + MR) of the block's 128 queries
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
            if (m < mvalid && tr < nty && tcc < ntx && P.dev_skip_epilogue != 2) {
                const floatx4 v = *reinterpret_cast<const floatx4*>(
                    Cs + m * CS + (trl * 4 + (j >> 1)) * TBW + tcl * 8 + (j & 1) * 4);
                st<NTS>(reinterpret_cast<floatx4*>(P.lvl[0] + (row0 + m) * P.lsz[0] + (tr * ntx + tcc) * kTile + 4 * j), v);
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
    {   // level 1: tile (ty0/8, tx0/16), 8 float4 per query
        const int tr = tc.ty0 / 8, tcc = tc.tx0 / 16;
        if (tr < P.lnty[1] && tcc < P.lntx[1]) {
            float* base = P.lvl[1] + (tr * P.lntx[1] + tcc) * kTile;
#pragma unroll
            for (int s = 0; s < (MR * 8) / NT; ++s) {
                const int idx = tid + NT * s;
                const int mm = idx >> 3, j = idx & 7;
                if (mm < mvalid)
                    st<NTS>(reinterpret_cast<floatx4*>(base + (row0 + mm) * P.lsz[1] + 4 * j),
                            *reinterpret_cast<const floatx4*>(S1 + mm * P1S + 4 * j));
            }
        }
    }
    if (P.fused_levels >= 3 && tid < 2 * MR && P.dev_skip_epilogue != -1 && P.dev_skip_epilogue != -4) {   // level 2: rows ty0/4 + {0,1}, cols tx0/4 .. +3
        const int mm = tid >> 1, y = tid & 1;
        if (mm < mvalid) {
            const float* src = S2 + mm * P2S + y * 4;
            float* img = P.lvl[2] + (row0 + mm) * P.lsz[2];
            if (P.lntx[2] > 0) {
                const int tr = tc.ty0 / 16, tcc = tc.tx0 / 32;
                if (tr < P.lnty[2] && tcc < P.lntx[2]) {
                    const int r = ((tc.ty0 / 4) & 3) + y, c0 = (tc.tx0 / 4) & 7;
                    *reinterpret_cast<floatx4*>(img + (tr * P.lntx[2] + tcc) * kTile + r * 8 + c0) =
                        *reinterpret_cast<const floatx4*>(src);
                }
            } else {   // compact row-major: no padding cells, so every pixel is range-checked
                const int r = tc.ty0 / 4 + y, c0 = tc.tx0 / 4;
                if (r < P.lh[2])
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        if (c0 + j < P.lw[2]) img[r * P.lw[2] + c0 + j] = src[j];
            }
        }
    }
    if (P.fused_levels >= 4 && tid < MR && tid < mvalid && P.dev_skip_epilogue != -1 && P.dev_skip_epilogue != -3) {   // level 3: row ty0/8, cols tx0/8 .. +1
        const float* src = S3 + tid * 2;
        float* img = P.lvl[3] + (row0 + tid) * P.lsz[3];
        if (P.lntx[3] > 0) {
            const int tr = tc.ty0 / 32, tcc = tc.tx0 / 64;
            if (tr < P.lnty[3] && tcc < P.lntx[3]) {
                const int r = (tc.ty0 / 8) & 3, c0 = (tc.tx0 / 8) & 7;
                *reinterpret_cast<floatx2*>(img + (tr * P.lntx[3] + tcc) * kTile + r * 8 + c0) =
                    *reinterpret_cast<const floatx2*>(src);
            }
        } else {
            const int r = tc.ty0 / 8, c0 = tc.tx0 / 8;
            if (r < P.lh[3]) {
                float* d = img + r * P.lw[3] + c0;
                // both pixels in range and 8-byte aligned: one 8-byte store instead of two scalars
                // (ECORR_BUILD_SKIP_EPILOGUE=-5 keeps the scalars, A/B only)
                if (c0 + 1 < P.lw[3] && (reinterpret_cast<uintptr_t>(d) & 7) == 0 && P.dev_skip_epilogue != -5) {
                    *reinterpret_cast<floatx2*>(d) = *reinterpret_cast<const floatx2*>(src);
                } else {
                    if (c0 < P.lw[3]) d[0] = src[0];
                    if (c0 + 1 < P.lw[3]) d[1] = src[1];
                }
            }
        }
    }
}

// Epilogue of a band tile (4 target rows x 32 cols; n = ty*32 + tx).  Level 0: one tile row of
// 4 tiles per query.  Pooling: thread (query m, 4x8 block blk = 0..3) reduces 4x8 -> 2x4 -> 1x2 in
// registers (the reference's order, from the rounded previous level); level 1 leaves as two 8-float
// rows of two tiles, level 2 as one 8-float row.  No level-3 pixel draws on these rows.
template <int MR, bool NTS>
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
            if (m < mvalid && tc0 + tcl < ntx && P.dev_skip_epilogue != 2) {
                const floatx4 v = *reinterpret_cast<const floatx4*>(Cs + m * CS + (j >> 1) * 32 + tcl * 8 + (j & 1) * 4);
                st<NTS>(reinterpret_cast<floatx4*>(P.lvl[0] + (row0 + m) * P.lsz[0] + (tr * ntx + tc0 + tcl) * kTile + 4 * j), v);
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
    {   // level 1: rows ty0/2 .. +1 (in-tile rows 0-1 of tile row ty0/8), tile cols tx0/16 .. +1
        const int tr = tc.ty0 / 8, tc0 = tc.tx0 / 16;
        if (tr < P.lnty[1]) {
#pragma unroll
            for (int s = 0; s < (MR * 8 + NT - 1) / NT; ++s) {
                const int idx = tid + NT * s;
                const int mm = idx >> 3, t = idx & 7;
                const int y = t >> 2, tcl = (t >> 1) & 1, hf = t & 1;
                if (mm < mvalid && tc0 + tcl < P.lntx[1])
                    st<NTS>(reinterpret_cast<floatx4*>(P.lvl[1] + (row0 + mm) * P.lsz[1] +
                                                       (tr * P.lntx[1] + tc0 + tcl) * kTile + y * 8 + hf * 4),
                            *reinterpret_cast<const floatx4*>(S1 + mm * P1S + y * 16 + tcl * 8 + hf * 4));
            }
        }
    }
    if (P.fused_levels >= 3 && tid < 2 * MR && P.dev_skip_epilogue != -1 && P.dev_skip_epilogue != -4) {   // level 2: row ty0/4, cols tx0/4 .. +7
        const int mm = tid >> 1, hf = tid & 1;
        if (mm < mvalid) {
            const float* src = S2 + mm * P2S + hf * 4;
            float* img = P.lvl[2] + (row0 + mm) * P.lsz[2];
            const int r = tc.ty0 / 4, c0 = tc.tx0 / 4 + hf * 4;
            if (P.lntx[2] > 0) {
                const int tr = r / 4, tcc = c0 / 8;
                if (tr < P.lnty[2] && tcc < P.lntx[2])
                    *reinterpret_cast<floatx4*>(img + (tr * P.lntx[2] + tcc) * kTile + (r & 3) * 8 + (c0 & 7)) =
                        *reinterpret_cast<const floatx4*>(src);
            } else if (r < P.lh[2]) {
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (c0 + j < P.lw[2]) img[r * P.lw[2] + c0 + j] = src[j];
            }
        }
    }
}

// KB = K chunk depth; HALF = C tile handled in two 64-query halves.  KB = 16 + HALF needs 34 KB of
// LDS and <= 168 VGPRs, so 3 blocks (3 waves per SIMD) share a CU; KB = 32 uses 67.5 KB (2 blocks).
// (A/B: v_mfma_f32_16x16x4_f32 tiles, bitwise the same result, ran 1% slower than 32x32x2.)
//
// GLDS: the K chunks go global -> LDS directly (buffer_load_dwordx4 ... lds, whose range check
// zero-fills the padding) through 3 LDS buffers with two chunks in flight: each wave waits for its
// own copies of chunk kc with a counted vmcnt, one raw barrier publishes them, and chunk kc + 2
// is issued into the buffer chunk kc - 1 was read from.  No staging registers, no ds_write pass,
// one barrier per chunk.  Needs VEC and byte offsets below 2^31 (launch_build checks).
// s_waitcnt vmcnt(N) alone (expcnt / lgkmcnt fields at their "don't wait" maxima), N < 16
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    static_assert(N >= 0 && N < 16, "vmcnt field");
    __builtin_amdgcn_s_waitcnt(N | (7 << 4) | (15 << 8));
}

// SPLIT: the fp32 operands are split into f16 hi + lo per fragment (split_f16, per-pixel
// power-of-two scales from fmap_exp_kernel) and each 16-deep K chunk runs 3 v_mfma_f32_32x32x16_f16
// per 32x32 tile (lo*hi, hi*lo, hi*hi; lo*lo is below fp32 rounding) instead of 8 fp32 MFMAs:
// 3 x 32 vs 8 x 64 matrix-core cycles.  The fragment reads are the fp32 path's: lane (r, h) takes
// k = 2j + h as element j, the same permutation on both operands.  Normwise error vs fp64 is
// below the fp32 path's; the result is scaled back by 2^-(e1+e2) exactly.
//
// PK (split mode, default): the operands arrive pre-split by pack_kernel as 8-KB panels (one per
// 128-pixel tile and 16-deep K chunk) laid out in MFMA-fragment order, so LDS-DMA copies them
// verbatim and each fragment is ONE lane-linear ds_read_b128: no VALU work in the K loop, no zero
// fill (the panels carry their padding).  The MFMAs take the fmap2 fragment as their A operand,
// so the accumulators hold C^T and reach the LDS C tile as 16-byte stores.
// ABL (A/B ablation of the pipelined PK loop only, output invalid; ECORR_BUILD_ABL): 5 no MFMA,
// 6 no fragment reads, 7 no barrier, 8 no chunk copies -- each also without the epilogue.
template <bool VEC, int KB, bool HALF, bool NTS, int GBUF = 0, bool SPLIT = false, bool PK = false, int ABL = 0>
__global__ __launch_bounds__(NT, HALF ? 3 : 2) void build_kernel(BuildParams P) {
    static_assert(!PK || (SPLIT && KB == 16 && GBUF > 0), "PK: split mode, 16-deep panels, LDS-DMA");
    constexpr int MR = HALF ? BM / 2 : BM;
    constexpr int AS = BM, BSS = BN;   // LDS row strides
    constexpr int NLD = (KB * BM / 4) / NT;   // float4 of A (and of B) per thread per chunk
    constexpr bool GLDS = GBUF > 0;
    constexpr int NBUF = GLDS ? GBUF : 2;   // GLDS: chunks kc .. kc + NBUF - 2 in flight
    static_assert(!GLDS || (VEC && NLD >= 1 && NBUF >= 3 && 2 * NLD * (NBUF - 2) < 16),
                  "GLDS: vector path, whole copies per wave, counted vmcnt in range");
    // ALL LDS in this one array: a second __shared__ object can make hipcc wait vmcnt(0) before
    // every ds_read while a buffer_load ... lds is in flight (cdna_hip_programming.md trap 4(a))
    constexpr int SM = smem_floats(KB, MR, AS, BSS, NBUF);
    __shared__ __attribute__((aligned(16))) float smem[SM + (SPLIT ? BM + BN : 0)];
    float* As = smem;                       // [NBUF][KB][AS]
    float* Bs = smem + NBUF * KB * AS;      // [NBUF][KB][BSS]
    int* exs = reinterpret_cast<int*>(smem + SM);   // SPLIT: exponents of the BM queries, BN targets

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const TileCoord tc = decode_tile(P, xcd_remap(blockIdx.x, gridDim.x));
    const int q_end = P.q_count;
    const int H = P.H, W = P.W, D = P.D;
    const int64_t Q = (int64_t)H * W;
    const int64_t QA = P.q_count;
    const float* __restrict__ A = P.f1 + (int64_t)tc.b * D * QA;
    const float* __restrict__ Bm = P.f2 + (int64_t)tc.b * D * Q;
    if constexpr (SPLIT) {
        // LDS column n of the B tile is target (y, x) as the loads below map it
        const int t = threadIdx.x;
        int e = 0;
        if (t < BM) {
            if (tc.m0 + t < P.q_count) e = P.ex1[(int64_t)tc.b * P.q_count + tc.m0 + t];
        } else {
            const int n = t - BM, c = n >> 2;
            const int y = tc.ty0 + (tc.band ? c >> 3 : c >> 2), x = tc.tx0 + 4 * (tc.band ? c & 7 : c & 3) + (n & 3);
            if (y < P.H && x < P.W) e = P.ex2[(int64_t)tc.b * Q + (int64_t)y * P.W + x];
        }
        exs[t] = e;
        __syncthreads();
    }

    // ---- global -> register staging: NLD float4 of A and of B per thread per K chunk ----
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

    float sa0 = 1.f, sa1 = 1.f, sb0 = 1.f, sb1 = 1.f;
    if constexpr (SPLIT && !PK) {
        sa0 = exp2i(exs[wm * 64 + acol]);
        sa1 = exp2i(exs[wm * 64 + 32 + acol]);
        sb0 = exp2i(exs[BM + wn * 64 + acol]);
        sb1 = exp2i(exs[BM + wn * 64 + 32 + acol]);
    }

    auto mfma_chunk = [&](int buf) {
        const float* as = As + buf * KB * AS + wm * 64 + acol;
        const float* bs = Bs + buf * KB * BSS + wn * 64 + acol;
        if constexpr (PK) {
            // panel: [32-row group][hi h0 | hi h1 | lo h0 | lo h1][32 rows][8 halves]
            const char* ap = reinterpret_cast<const char*>(As + buf * KB * AS) + wm * 4096 + lane * 16;
            const char* bp = reinterpret_cast<const char*>(Bs + buf * KB * BSS) + wn * 4096 + lane * 16;
            const halfx8 a0h = *reinterpret_cast<const halfx8*>(ap);
            const halfx8 a0l = *reinterpret_cast<const halfx8*>(ap + 1024);
            const halfx8 a1h = *reinterpret_cast<const halfx8*>(ap + 2048);
            const halfx8 a1l = *reinterpret_cast<const halfx8*>(ap + 3072);
            const halfx8 b0h = *reinterpret_cast<const halfx8*>(bp);
            const halfx8 b0l = *reinterpret_cast<const halfx8*>(bp + 1024);
            const halfx8 b1h = *reinterpret_cast<const halfx8*>(bp + 2048);
            const halfx8 b1l = *reinterpret_cast<const halfx8*>(bp + 3072);
            acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(b0h, a0l, acc[0][0], 0, 0, 0);
            acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(b1h, a0l, acc[0][1], 0, 0, 0);
            acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(b0h, a1l, acc[1][0], 0, 0, 0);
            acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(b1h, a1l, acc[1][1], 0, 0, 0);
            acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(b0l, a0h, acc[0][0], 0, 0, 0);
            acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(b1l, a0h, acc[0][1], 0, 0, 0);
            acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(b0l, a1h, acc[1][0], 0, 0, 0);
            acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(b1l, a1h, acc[1][1], 0, 0, 0);
            acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(b0h, a0h, acc[0][0], 0, 0, 0);
            acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(b1h, a0h, acc[0][1], 0, 0, 0);
            acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(b0h, a1h, acc[1][0], 0, 0, 0);
            acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(b1h, a1h, acc[1][1], 0, 0, 0);
            return;
        }
        if constexpr (SPLIT) {
#pragma unroll
            for (int k16 = 0; k16 < KB; k16 += 16) {
                float va0[8], va1[8], vb0[8], vb1[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int ro = k16 + 2 * j + arow;
                    va0[j] = as[ro * AS];
                    va1[j] = as[ro * AS + 32];
                    vb0[j] = bs[ro * BSS];
                    vb1[j] = bs[ro * BSS + 32];
                }
                halfx8 a0h, a0l, a1h, a1l, b0h, b0l, b1h, b1l;
                split_f16(va0, sa0, a0h, a0l);
                split_f16(va1, sa1, a1h, a1l);
                split_f16(vb0, sb0, b0h, b0l);
                split_f16(vb1, sb1, b1h, b1l);
                acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0l, b0h, acc[0][0], 0, 0, 0);
                acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0l, b1h, acc[0][1], 0, 0, 0);
                acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1l, b0h, acc[1][0], 0, 0, 0);
                acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1l, b1h, acc[1][1], 0, 0, 0);
                acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0h, b0l, acc[0][0], 0, 0, 0);
                acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0h, b1l, acc[0][1], 0, 0, 0);
                acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1h, b0l, acc[1][0], 0, 0, 0);
                acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1h, b1l, acc[1][1], 0, 0, 0);
                acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0h, b0h, acc[0][0], 0, 0, 0);
                acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0h, b1h, acc[0][1], 0, 0, 0);
                acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1h, b0h, acc[1][0], 0, 0, 0);
                acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1h, b1h, acc[1][1], 0, 0, 0);
            }
            return;
        }
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
        // PK: this tile's panels, chunk-major (pack_kernel layout)
        const int dc = (D + 15) / 16;
        const char* pa = PK ? P.pk1 + ((int64_t)tc.b * P.n_mt + tc.mt) * dc * 8192 : nullptr;
        const char* pb = PK ? P.pk2 + ((int64_t)tc.b * P.n_nt + tc.nt) * dc * 8192 : nullptr;
        const __amdgpu_buffer_rsrc_t rpa =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(pa), 0, dc * 8192, 0x00020000);
        const __amdgpu_buffer_rsrc_t rpb =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(pb), 0, dc * 8192, 0x00020000);
        auto issue = [&](int kc) {
            const int buf = kc % NBUF;
            if constexpr (PK) {
#pragma unroll
                for (int i = 0; i < NLD; ++i) {
                    const int slot = i * NT + wave * 64;   // wave-uniform 16-byte slot of this copy
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(
                        rpa, (__attribute__((address_space(3))) void*)(As + buf * KB * AS + 4 * slot), 16,
                        kc * 8192 + (slot + lane) * 16, 0, 0, 0);
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(
                        rpb, (__attribute__((address_space(3))) void*)(Bs + buf * KB * BSS + 4 * slot), 16,
                        kc * 8192 + (slot + lane) * 16, 0, 0, 0);
                }
                return;
            }
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
        if constexpr (PK) {
            if (P.dev_pk_pipe && nk % 2 == 0) {
                // software-pipelined (even chunk counts): chunk kc + 1's fragments are read (after
                // its barrier) between the lo*hi MFMAs of chunk kc and its hi*lo / hi*hi MFMAs, so
                // the barrier and the LDS latency hide behind the matrix pipe; two register sets,
                // loop unrolled by 2
                auto read_frags = [&](int buf, halfx8 (&f)[8]) {
                    if constexpr (ABL == 6) return;
                    const char* ap = reinterpret_cast<const char*>(As + buf * KB * AS) + wm * 4096 + lane * 16;
                    const char* bp = reinterpret_cast<const char*>(Bs + buf * KB * BSS) + wn * 4096 + lane * 16;
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        f[q] = *reinterpret_cast<const halfx8*>(ap + q * 1024);       // a0h a0l a1h a1l
                        f[4 + q] = *reinterpret_cast<const halfx8*>(bp + q * 1024);   // b0h b0l b1h b1l
                    }
                };
                auto mfma_lohi = [&](const halfx8 (&f)[8]) {
                    if constexpr (ABL == 5) {
#pragma unroll
                        for (int q = 0; q < 8; ++q) asm volatile("" ::"v"(f[q]));
                        return;
                    }
                    acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f[4], f[1], acc[0][0], 0, 0, 0);
                    acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f[6], f[1], acc[0][1], 0, 0, 0);
                    acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f[4], f[3], acc[1][0], 0, 0, 0);
                    acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f[6], f[3], acc[1][1], 0, 0, 0);
                };
                auto mfma_rest = [&](const halfx8 (&f)[8]) {
                    if constexpr (ABL == 5) return;
                    acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f[5], f[0], acc[0][0], 0, 0, 0);
                    acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f[7], f[0], acc[0][1], 0, 0, 0);
                    acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f[5], f[2], acc[1][0], 0, 0, 0);
                    acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f[7], f[2], acc[1][1], 0, 0, 0);
                    acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f[4], f[0], acc[0][0], 0, 0, 0);
                    acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f[6], f[0], acc[0][1], 0, 0, 0);
                    acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f[4], f[2], acc[1][0], 0, 0, 0);
                    acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f[6], f[2], acc[1][1], 0, 0, 0);
                };
                // chunk j's buffer is j % NBUF; a chunk is issued into the buffer whose reads the
                // preceding barrier retired.  Exactly one chunk stays in flight at every wait:
                // chunks past the end are still issued (their offsets fall outside the panel range,
                // so they land as zeros in a retired buffer) and the last advance reads such a
                // chunk, which keeps the loop free of branches (and of conservative waitcnts)
                auto advance = [&](int& issued, int j, halfx8 (&f)[8]) {
                    // vmcnt(2 NLD (NBUF - 2)): chunk j landed, the NBUF - 2 after it may fly;
                    // lgkmcnt(0): this wave's reads of chunk j - 1 (half of them not yet consumed
                    // by an MFMA) are done before the barrier hands their buffer to chunk
                    // j + NBUF - 1
                    static_assert(2 * NLD * (NBUF - 2) < 16, "vmcnt field");
                    __builtin_amdgcn_s_waitcnt((2 * NLD * (NBUF - 2)) | (7 << 4));
                    if constexpr (ABL != 7) __builtin_amdgcn_s_barrier();
                    if constexpr (ABL != 8) issue(issued);
                    ++issued;
                    read_frags(j % NBUF, f);
                };
                halfx8 fa[8], fb[8];
                if constexpr (ABL == 6) {
#pragma unroll
                    for (int q = 0; q < 8; ++q) fa[q] = fb[q] = halfx8{};
                }
                int issued = 0;
                while (issued < NBUF - 1) issue(issued++);
                advance(issued, 0, fa);
                for (int kc = 0; kc < nk; kc += 2) {
                    mfma_lohi(fa);
                    advance(issued, kc + 1, fb);
                    mfma_rest(fa);
                    mfma_lohi(fb);
                    advance(issued, kc + 2, fa);
                    mfma_rest(fb);
                }
                wait_vmcnt<0>();
                goto chunks_done;
            }
        }
        for (int kc = 0; kc < NBUF - 1 && kc < nk; ++kc) issue(kc);
        for (int kc = 0; kc < nk; ++kc) {
            // this wave's copies of chunk kc have landed (those of the later issued chunks may
            // still fly: 2 NLD copies each) ...
            const int after = min(nk, kc + NBUF - 1) - (kc + 1);
            static_assert(NBUF <= 6, "wait ladder");
            switch (after) {
                case 0: wait_vmcnt<0>(); break;
                case 1: wait_vmcnt<2 * NLD * (NBUF > 2 ? 1 : 0)>(); break;
                case 2: wait_vmcnt<2 * NLD * (NBUF > 3 ? 2 : 0)>(); break;
                case 3: wait_vmcnt<2 * NLD * (NBUF > 4 ? 3 : 0)>(); break;
                default: wait_vmcnt<2 * NLD * (NBUF > 5 ? 4 : 0)>(); break;
            }
            // ... and every wave's have once all passed this barrier, which also retires the
            // reads of chunk kc - 1, whose buffer chunk kc + NBUF - 1 now overwrites
            __builtin_amdgcn_s_barrier();
            if (kc + NBUF - 1 < nk && P.dev_skip_epilogue < 3) issue(kc + NBUF - 1);
            mfma_chunk(kc % NBUF);
        }
    chunks_done:
        __syncthreads();   // the C tile aliases the chunk buffers
    } else {
        load_chunk(0);
        store_chunk(0);
        __syncthreads();
        for (int kc = 0; kc < nk; ++kc) {
            const int buf = kc & 1;
            if (kc + 1 < nk && P.dev_skip_epilogue < 3) load_chunk((kc + 1) * KB);
            mfma_chunk(buf);
            if (kc + 1 < nk && P.dev_skip_epilogue < 4) store_chunk(buf ^ 1);
            __syncthreads();
        }
    }

    // ---- scaled accumulators -> LDS C tile [m][n]; C/D map: col = lane&31,
    //      row = (reg&3) + 8*(reg>>2) + 4*(lane>>5) ----
    float* Cs = smem;
#pragma unroll
    for (int half = 0; half < (HALF ? 2 : 1); ++half) {
        if (!HALF || wm == half) {
            const int mb = HALF ? 0 : wm * 64;
            // one uniform branch on the scale mode around the whole tile (a per-element select
            // had the compiler emit an IEEE division next to every element's multiply)
            auto write_c = [&](auto scaled) {
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        if constexpr (PK) {
                            // PK tiles are C^T (targets on the rows, queries on the lanes): each
                            // lane's 4 consecutive rows are 4 consecutive targets of one query, one
                            // 16-byte LDS store (row stride 132: conflict-free)
                            const int m = mb + i * 32 + acol;
                            const int ea = exs[(HALF ? half * 64 : 0) + m];
#pragma unroll
                            for (int g4 = 0; g4 < 4; ++g4) {
                                const int n = wn * 64 + j * 32 + 8 * g4 + 4 * arow;
                                floatx4 v;
#pragma unroll
                                for (int t = 0; t < 4; ++t) v[t] = scaled(acc[i][j][4 * g4 + t], ea + exs[BM + n + t]);
                                *reinterpret_cast<floatx4*>(Cs + m * CS + n) = v;
                            }
                        } else {
#pragma unroll
                            for (int r = 0; r < 16; ++r) {
                                const int m = mb + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * arow;
                                const int n = wn * 64 + j * 32 + acol;
                                const int e = SPLIT ? exs[(HALF ? half * 64 : 0) + m] + exs[BM + n] : 0;
                                Cs[m * CS + n] = scaled(acc[i][j][r], e);
                            }
                        }
                    }
            };
            if (P.scale_is_mul) {
                // v * 2^-(e1+e2) * 2^-s as one exact scaling (unless subnormal) when 1/sqrt(D) = 2^-s
                if constexpr (SPLIT) write_c([&](float v, int e) { return ldexpf(v, -(e + P.scale_shift)); });
                else write_c([&](float v, int) { return __fmul_rn(v, P.scale); });
            } else {
                write_c([&](float v, int e) {
                    // SPLIT: undo the 2^(e1+e2) operand scaling (exact unless subnormal), then divide
                    return __fdiv_rn(SPLIT ? ldexpf(v, -e) : v, P.scale);
                });
            }
        }
        __syncthreads();
        if (ABL || P.dev_skip_epilogue == 1 || P.dev_skip_epilogue >= 3) continue;
        if (tc.band) epilogue_band<MR, NTS>(P, tc, Cs, tid, half * MR);
        else epilogue<MR, NTS>(P, tc, Cs, tid, half * MR);
        if (HALF && half == 0) __syncthreads();   // half 0 fully consumed before half 1 overwrites Cs
    }
}

// Levels beyond the 3 fused ones (num_levels > 4): plain 2x2 floor-mode pooling, tiled in and
// out, one thread per output pixel.  Not on the E-RAFT path (num_levels = 4, eraft.py:50).
__global__ __launch_bounds__(256) void pool2_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                    int64_t rows, int h, int w, int ntx_in, int64_t sz_in,
                                                    int ntx_out, int64_t sz_out) {
    const int ho = h / 2, wo = w / 2;
    const int64_t n = rows * ho * wo;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t rw = i / ((int64_t)ho * wo);
        const int yx = (int)(i - rw * ho * wo);
        const int y = yx / wo, x = yx - y * wo;
        const float* s = in + rw * sz_in;
        out[rw * sz_out + level_off(y, x, ntx_out, wo)] =
            pool4(s[level_off(2 * y, 2 * x, ntx_in, w)], s[level_off(2 * y, 2 * x + 1, ntx_in, w)],
                  s[level_off(2 * y + 1, 2 * x, ntx_in, w)], s[level_off(2 * y + 1, 2 * x + 1, ntx_in, w)]);
    }
}

// Split-mode exponent pass: ex[b][n] = 15 - E with max_d |x[b][d][n]| = f 2^E, f in [0.5, 1)
// (so the pixel's largest scaled value lies in [2^14, 2^15)); 0 for all-zero or non-finite maxima
// (NaN inputs propagate through the GEMM as in the reference).  x: [B][D][N].  Block = 64 pixels
// x 4 channel groups (coalesced 256-byte rows per wave), grid (ceil(N / 64), B).
__global__ __launch_bounds__(256) void fmap_exp_kernel(const float* __restrict__ x, int D, int64_t N,
                                                       int* __restrict__ ex) {
    __shared__ float red[4][64];
    const int b = blockIdx.y, l = threadIdx.x & 63, g = threadIdx.x >> 6;
    const int64_t n = (int64_t)blockIdx.x * 64 + l;
    float m = 0.f;
    if (n < N) {
        const float* p = x + (int64_t)b * D * N + n;
        for (int d = g; d < D; d += 4) m = fmaxf(m, fabsf(p[(int64_t)d * N]));
    }
    red[g][l] = m;
    __syncthreads();
    if (g == 0 && n < N) {
        m = fmaxf(fmaxf(red[0][l], red[1][l]), fmaxf(red[2][l], red[3][l]));
        int E = 0;
        frexpf(m, &E);
        int e = (m > 0.f && m <= 3.4028235e38f) ? 15 - E : 0;
        e = e < -126 ? -126 : (e > 126 ? 126 : e);
        ex[(int64_t)b * N + n] = e;
    }
}

// Split-mode operand pass (PK build): per pixel, the power-of-two exponent of fmap_exp_kernel and
// the f16 hi/lo split of all D values, written as the build's 8-KB panels: panel (tile, chunk) =
// [32-row group g][hi k0-7 | hi k8-15 | lo k0-7 | lo k8-15][row r][8 halves], i.e. the
// v_mfma_f32_32x32x16_f16 operand of lane (r, h) is the 16 bytes at g*2048 + part*1024 + lane*16.
// Tile positions without a pixel (ragged edges) and k >= D are written as zeros.
// ISB = 0: fmap1 slab, tile = 128 consecutive queries; ISB = 1: fmap2, tile = the build's 8 x 16
// (or 4 x 32 band) target block in its LDS column order.  Block = 64 positions x 4 chunk
// quarters; grid (2 * tiles, B).  The second pass re-reads the block's 64 KB (L2 / MALL hits).
template <bool ISB>
__device__ __forceinline__ void pack_body(const float* __restrict__ x, const BuildParams& P, int* __restrict__ ex,
                                          char* __restrict__ pack) {
    __shared__ float red[4][64];
    const int b = blockIdx.y, tile = blockIdx.x >> 1, pos = (blockIdx.x & 1) * 64 + (threadIdx.x & 63);
    const int qtr = threadIdx.x >> 6, D = P.D, dc = (D + 15) / 16;
    const int64_t N = ISB ? (int64_t)P.H * P.W : (int64_t)P.q_count;
    int64_t pix = -1;
    if (!ISB) {
        const int64_t p = (int64_t)tile * BM + pos;
        if (p < P.q_count) pix = p;
    } else {
        int y, xx;
        if (tile < P.n_reg) {
            y = (tile / P.n_ntx) * TBH + (pos >> 4);
            xx = (tile % P.n_ntx) * TBW + (pos & 15);
        } else {
            y = P.band_y0 + (pos >> 5);
            xx = (tile - P.n_reg) * 32 + (pos & 31);
        }
        if (y < P.H && xx < P.W) pix = (int64_t)y * P.W + xx;
    }
    const float* px = x + (int64_t)b * D * N + (pix < 0 ? 0 : pix);
    // D <= 256 (E-RAFT: 256): this thread's <= 4 chunks stay in registers between the max and the
    // split, so the operand is read once; larger D re-reads it in the second pass
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
    char* pan = pack + ((int64_t)b * ntiles + tile) * dc * 8192 + (pos >> 5) * 2048 + (pos & 31) * 16;
    auto put = [&](int c, const float (&w)[16]) {
        halfx8 h0, l0, h1, l1;
        split_f16(*reinterpret_cast<const float(*)[8]>(w), s, h0, l0);
        split_f16(*reinterpret_cast<const float(*)[8]>(w + 8), s, h1, l1);
        char* p = pan + (int64_t)c * 8192;
        *reinterpret_cast<halfx8*>(p) = h0;
        *reinterpret_cast<halfx8*>(p + 512) = h1;
        *reinterpret_cast<halfx8*>(p + 1024) = l0;
        *reinterpret_cast<halfx8*>(p + 1536) = l1;
    };
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

template <bool ISB>
__global__ __launch_bounds__(256) void pack_kernel(const float* __restrict__ x, BuildParams P, int* __restrict__ ex,
                                                   char* __restrict__ pack) {
    pack_body<ISB>(x, P, ex, pack);
}

// Both operand passes in ONE launch: grid (2 * max(n_mt, n_nt), B, 2), z = 0 packs fmap1 (slab
// tiles), z = 1 fmap2 (target blocks).  Neither pass alone fills the chip (1,216 blocks at DSEC
// B = 16, all resident at once, latency-bound on their 64 loads per thread); one grid overlaps
// the two and drops a launch boundary: build 0.836 -> 0.826 ms at DSEC B = 16 (rotated A/B,
// profiles/r01_final8/ab_pack.txt; a 128-VGPR cap for 4 waves per SIMD spills and gains nothing,
// 0.829).  Surplus x blocks of the shorter pass return at once (block-uniform, before
// pack_body's barrier).
__global__ __launch_bounds__(256) void pack_both_kernel(BuildParams P) {
    if (blockIdx.z == 0) {
        if ((int)blockIdx.x < 2 * P.n_mt) pack_body<false>(P.f1, P, P.ex1, const_cast<char*>(P.pk1));
    } else if ((int)blockIdx.x < 2 * P.n_nt) {
        pack_body<true>(P.f2, P, P.ex2, const_cast<char*>(P.pk2));
    }
}

}  // namespace

namespace {
void tile_counts(BuildParams& P) {
    P.n_ntx = (P.W + TBW - 1) / TBW;
    // 8-row tile rows; a remainder of 1..4 rows (the last 8k + r rows, r <= 4) becomes a band of
    // 4 x 32 tiles (see TileCoord), a remainder of 5..7 a padded regular tile row
    const int rem = P.H % TBH;
    // dev knob for A/B (tools/ab_build.py): ECORR_BUILD_NOBAND=1 pads the remainder instead
    const bool band = rem > 0 && rem <= 4 && getenv("ECORR_BUILD_NOBAND") == nullptr;
    P.n_reg = P.n_ntx * (band ? P.H / TBH : (P.H + TBH - 1) / TBH);
    P.band_y0 = (P.H / TBH) * TBH;
    P.n_nt = P.n_reg + (band ? (P.W + 31) / 32 : 0);
    P.n_mt = (P.q_count + BM - 1) / BM;
}

// split workspace: exponents (fmap1 slab, fmap2), then fmap1 and fmap2 panels (256-B aligned)
struct SplitWs { int64_t ex2, pk1, pk2, total; };
SplitWs split_ws(const BuildParams& P, int B) {
    const int64_t dc = (P.D + 15) / 16;
    SplitWs w;
    w.ex2 = (int64_t)B * P.q_count * 4;
    w.pk1 = (w.ex2 + (int64_t)B * P.H * P.W * 4 + 255) & ~(int64_t)255;
    w.pk2 = w.pk1 + (int64_t)B * P.n_mt * dc * 8192;
    w.total = w.pk2 + (int64_t)B * P.n_nt * dc * 8192;
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

int launch_build(const BuildParams& P0, int B, const PyrGeom& g, float* pyramid, hipStream_t stream) {
    BuildParams P = P0;
    const int levels = g.levels;
    P.fused_levels = levels < 4 ? levels : 4;
    tile_counts(P);
    // m-tiles per group of the tile order (dev knob ECORR_BUILD_GM for A/B; default 8)
    const char* kgm = getenv("ECORR_BUILD_GM");
    P.gm = kgm && atoi(kgm) > 0 ? atoi(kgm) : 8;
    for (int i = 0; i < 4; ++i) {
        const bool on = i < levels;
        P.lvl[i] = on ? pyramid + g.off[i] : nullptr;
        P.lh[i] = on ? g.h[i] : 0;
        P.lw[i] = on ? g.w[i] : 0;
        P.lntx[i] = on ? g.ntx[i] : 0;
        P.lnty[i] = on ? g.nty[i] : 0;
        P.lsz[i] = on ? g.sz[i] : 0;
    }
    const int64_t ntiles = (int64_t)B * P.n_mt * P.n_nt;
    if (ntiles <= 0 || ntiles > 0x7fffffff) return ECORR_EINVAL;
    P.n_tiles = (int)ntiles;
    // dev knob for A/B ablation (tools/ab_build.py): ECORR_BUILD_SKIP_EPILOGUE=1 drops the pyramid
    // stores (output invalid); unset in production.
    const char* kskip = getenv("ECORR_BUILD_SKIP_EPILOGUE");
    // 2: level-0 stores only; 3: + no K-chunk global loads (LDS refilled from stale registers);
    // 4: + no LDS refill (MFMA + fragment reads only)
    P.dev_skip_epilogue = kskip ? atoi(kskip) : 0;
    const bool vec = (P.W % 4 == 0) && (P.q_count % 4 == 0) && ((uintptr_t)P.f1 % 16 == 0) &&
                     ((uintptr_t)P.f2 % 16 == 0);
    if ((uintptr_t)pyramid % 16 != 0) return ECORR_EINVAL;   // tile stores are 16-byte vectors
    // dev knob for A/B (tools/ab_build.py): ECORR_BUILD_KB32=1 selects the K=32, full-C-tile,
    // 2-blocks-per-CU variant
    const char* kv = getenv("ECORR_BUILD_KB32");
    const bool kb32 = kv && atoi(kv) == 1;
    // LDS-DMA staging (3% faster than register staging, tools/ab_build.py) whenever both operands'
    // byte offsets fit the 31-bit buffer range; dev knob ECORR_BUILD_GLDS=0 selects the register-
    // staged loop for A/B
    const char* kg = getenv("ECORR_BUILD_GLDS");
    const bool glds = !(kg && atoi(kg) == 0) && (int64_t)P.D * P.H * P.W * 4 < 0x7fff0000LL &&
                      (int64_t)P.D * P.q_count * 4 < 0x7fff0000LL;
    const dim3 grid((unsigned)ntiles), block(NT);
    if (P.ws) {
        const int64_t Q = (int64_t)P.H * P.W;
        const SplitWs w = split_ws(P, B);
        P.ex1 = reinterpret_cast<int*>(P.ws);
        P.ex2 = reinterpret_cast<int*>(P.ws + w.ex2);
        P.pk1 = P.ws + w.pk1;
        P.pk2 = P.ws + w.pk2;
        // PK needs one batch item's panels inside the 31-bit buffer range; dev knob
        // ECORR_BUILD_PK=0 selects the in-loop split (A/B)
        const char* kp = getenv("ECORR_BUILD_PK");
        const char* kpp = getenv("ECORR_BUILD_PKPIPE");   // dev knob: 0 = unpipelined PK loop (A/B)
        P.dev_pk_pipe = !(kpp && atoi(kpp) == 0);
        const bool pk = !(kp && atoi(kp) == 0) &&
                        (int64_t)(P.n_mt > P.n_nt ? P.n_mt : P.n_nt) * ((P.D + 15) / 16) * 8192 < 0x7fff0000LL;
        if (pk) {
            const char* k2 = getenv("ECORR_BUILD_PACK2");   // dev knob (A/B): 1 = one launch per operand
            if (k2 && atoi(k2) == 1) {
                hipLaunchKernelGGL(pack_kernel<false>, dim3((unsigned)(2 * P.n_mt), B), dim3(256), 0, stream, P.f1, P,
                                   P.ex1, P.ws + w.pk1);
                hipLaunchKernelGGL(pack_kernel<true>, dim3((unsigned)(2 * P.n_nt), B), dim3(256), 0, stream, P.f2, P,
                                   P.ex2, P.ws + w.pk2);
            } else {
                const int nx = 2 * (P.n_mt > P.n_nt ? P.n_mt : P.n_nt);
                hipLaunchKernelGGL(pack_both_kernel, dim3((unsigned)nx, B, 2), dim3(256), 0, stream, P);
            }
            const char* ka = getenv("ECORR_BUILD_ABL");   // dev knob: loop ablations (A/B only)
            switch (ka && P.dev_pk_pipe ? atoi(ka) : 0) {
                case 5: hipLaunchKernelGGL((build_kernel<true, 16, true, true, 3, true, true, 5>), grid, block, 0, stream, P); break;
                case 6: hipLaunchKernelGGL((build_kernel<true, 16, true, true, 3, true, true, 6>), grid, block, 0, stream, P); break;
                case 7: hipLaunchKernelGGL((build_kernel<true, 16, true, true, 3, true, true, 7>), grid, block, 0, stream, P); break;
                case 8: hipLaunchKernelGGL((build_kernel<true, 16, true, true, 3, true, true, 8>), grid, block, 0, stream, P); break;
                default: hipLaunchKernelGGL((build_kernel<true, 16, true, true, 3, true, true>), grid, block, 0, stream, P);
            }
        } else {   // in-loop split: exponents only, fp32 operands staged as in the fp32 build
            hipLaunchKernelGGL(fmap_exp_kernel, dim3((unsigned)((P.q_count + 63) / 64), B), dim3(256), 0, stream,
                               P.f1, P.D, (int64_t)P.q_count, P.ex1);
            hipLaunchKernelGGL(fmap_exp_kernel, dim3((unsigned)((Q + 63) / 64), B), dim3(256), 0, stream, P.f2, P.D,
                               Q, P.ex2);
            if (!vec) hipLaunchKernelGGL((build_kernel<false, 16, true, true, 0, true>), grid, block, 0, stream, P);
            else if (glds) hipLaunchKernelGGL((build_kernel<true, 16, true, true, 3, true>), grid, block, 0, stream, P);
            else hipLaunchKernelGGL((build_kernel<true, 16, true, true, 0, true>), grid, block, 0, stream, P);
        }
    } else if (!vec) hipLaunchKernelGGL((build_kernel<false, 16, true, true>), grid, block, 0, stream, P);
    else if (kb32) hipLaunchKernelGGL((build_kernel<true, 32, false, true>), grid, block, 0, stream, P);
    else if (glds) hipLaunchKernelGGL((build_kernel<true, 16, true, true, 3>), grid, block, 0, stream, P);
    else hipLaunchKernelGGL((build_kernel<true, 16, true, true>), grid, block, 0, stream, P);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return ECORR_EHIP - (int)e;
    const int64_t rows = (int64_t)B * P.q_count;
    for (int i = 4; i < levels; ++i) {
        const int64_t n = rows * g.h[i] * g.w[i];
        const int grid = (int)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
        hipLaunchKernelGGL(pool2_kernel, dim3(grid), dim3(256), 0, stream, pyramid + g.off[i - 1], pyramid + g.off[i],
                           rows, g.h[i - 1], g.w[i - 1], g.ntx[i - 1], g.sz[i - 1], g.ntx[i], g.sz[i]);
        e = hipGetLastError();
        if (e != hipSuccess) return ECORR_EHIP - (int)e;
    }
    return ECORR_OK;
}

}  // namespace ecorr
