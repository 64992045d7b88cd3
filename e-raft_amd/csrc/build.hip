// build.hip -- CorrBlock build on gfx950: all-pairs correlation GEMM on fp32 MFMA with the
// 1/sqrt(D) scale and the 3 pooled pyramid levels fused into the epilogue.
//
// Replaces corr.py:13-27 (CorrBlock.__init__) and corr.py:52-60 (CorrBlock.corr):
//   level0[b*q_count + p'][y][x] = (sum_d f1[b][d][p] * f2[b][d][y*W+x]) / sqrt(D)
//   level{i+1} = (((x00 + x01) + x10) + x11) / 4 over 2x2 floor-mode windows of level i.
//
// GEMM view per batch item: A = f1[b] as [K=D][M=Q] (M contiguous), B = f2[b] as [K][N=Q].
// Block tile: 128 queries of the fmap1 slab (M) x one 8x16 block of target pixels (N = 128), K staged 32 deep
// through double-buffered LDS; 4 waves, each 64x64 = 2x2 v_mfma_f32_32x32x2_f32 tiles.  The N
// tile is a 2D target block so the epilogue can pool 3 levels locally: each thread owns one
// (query, 8x8 target block) and reduces it 8x8 -> 4x4 -> 2x2 -> 1 in registers, from the rounded
// previous level, in the reference's summation order.
//
// Numerics: MFMA f32 is an exact k-ordered fmaf chain; against the reference's sgemm the level-0
// agreement is normwise (max|d|/rms <= 1e-5), pooling is bit-exact given the same level 0.
#include <stdlib.h>

#include "ecorr_device.h"
#include "ecorr_internal.h"

namespace ecorr {

namespace {

constexpr int BM = 128;           // queries per block tile
constexpr int TBH = 8, TBW = 16;  // target block (rows x cols) per block tile
constexpr int BN = TBH * TBW;     // 128 targets
constexpr int BK = 32;            // K chunk
constexpr int NT = 256;           // threads
constexpr int CS = BN + 4;        // C-tile LDS row stride (floats): conflict-free ds_read_b128
constexpr int STAGE_FLOATS = 2 * (BK * BM + BK * BN);
constexpr int CTILE_FLOATS = BM * CS;
constexpr int SMEM_FLOATS = STAGE_FLOATS > CTILE_FLOATS ? STAGE_FLOATS : CTILE_FLOATS;

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float pool4(float a, float b, float c, float d) {
    return __fmul_rn(__fadd_rn(__fadd_rn(__fadd_rn(a, b), c), d), 0.25f);
}

// Tile decode: XCD-contiguous ranges of a grouped (GM m-tiles x all n-tiles) order, so the 64
// tiles an XCD works on at once form an ~8x8 square of fmap1/fmap2 panels that fits its L2.
struct TileCoord { int b, m0, ty0, tx0; };

__device__ __forceinline__ TileCoord decode_tile(const BuildParams& P, int t) {
    constexpr int GM = 8;
    const int per_b = P.n_mt * P.n_nt;
    TileCoord c;
    c.b = t / per_b;
    const int i = t - c.b * per_b;
    const int gsz = GM * P.n_nt;
    const int grp = i / gsz, gi = i - grp * gsz;
    const int first_m = grp * GM;
    const int gsm = min(P.n_mt - first_m, GM);
    const int mt = first_m + gi % gsm, nt = gi / gsm;
    const int nty = nt / P.n_ntx, ntx = nt - nty * P.n_ntx;
    c.m0 = mt * BM;
    c.ty0 = nty * TBH;
    c.tx0 = ntx * TBW;
    return c;
}

// Epilogue 2: thread = (query m, 8x8 target block blk) pools in registers, 8x8 -> 4x4 -> 2x2 -> 1,
// each level from the rounded previous one, and stores levels 0..fused_levels-1.
template <bool VEC>
__device__ __forceinline__ void epilogue_pool(const BuildParams& P, const TileCoord& tc,
                                              const float* Cs, int tid) {
    const int H = P.H, W = P.W;
    const int64_t Q = (int64_t)H * W;
    const int m = tid & (BM - 1), blk = tid >> 7;
    const int qm = tc.m0 + m;
    if (qm >= P.q_count) return;
    const int64_t row = (int64_t)tc.b * P.q_count + qm;
    const int ty0 = tc.ty0;
    float v[8][8];
#pragma unroll
    for (int ty = 0; ty < 8; ++ty) {
        const floatx4 lo = *reinterpret_cast<const floatx4*>(Cs + m * CS + ty * TBW + blk * 8);
        const floatx4 hi = *reinterpret_cast<const floatx4*>(Cs + m * CS + ty * TBW + blk * 8 + 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) { v[ty][j] = lo[j]; v[ty][4 + j] = hi[j]; }
    }
    const int bx = tc.tx0 + blk * 8;  // level-0 column of this 8x8 block
    {   // level 0
        float* dst = P.lvl[0] + row * Q;
        const bool full_w = bx + 8 <= W;
#pragma unroll
        for (int ty = 0; ty < 8; ++ty) {
            const int y = ty0 + ty;
            if (y >= H) break;
            float* d = dst + (int64_t)y * W + bx;
            if (VEC && full_w) {
                *reinterpret_cast<floatx4*>(d) = floatx4{v[ty][0], v[ty][1], v[ty][2], v[ty][3]};
                *reinterpret_cast<floatx4*>(d + 4) = floatx4{v[ty][4], v[ty][5], v[ty][6], v[ty][7]};
            } else {
#pragma unroll
                for (int tx = 0; tx < 8; ++tx)
                    if (bx + tx < W) d[tx] = v[ty][tx];
            }
        }
    }
    if (P.fused_levels < 2) return;
    float l1[4][4];
#pragma unroll
    for (int y = 0; y < 4; ++y)
#pragma unroll
        for (int x = 0; x < 4; ++x)
            l1[y][x] = pool4(v[2 * y][2 * x], v[2 * y][2 * x + 1], v[2 * y + 1][2 * x], v[2 * y + 1][2 * x + 1]);
    {
        const int h1 = P.lh[1], w1 = P.lw[1], y0 = ty0 / 2, x0 = bx / 2;
        float* dst = P.lvl[1] + row * (int64_t)h1 * w1;
#pragma unroll
        for (int y = 0; y < 4; ++y)
#pragma unroll
            for (int x = 0; x < 4; ++x)
                if (y0 + y < h1 && x0 + x < w1) dst[(int64_t)(y0 + y) * w1 + x0 + x] = l1[y][x];
    }
    if (P.fused_levels < 3) return;
    float l2[2][2];
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
        for (int x = 0; x < 2; ++x)
            l2[y][x] = pool4(l1[2 * y][2 * x], l1[2 * y][2 * x + 1], l1[2 * y + 1][2 * x], l1[2 * y + 1][2 * x + 1]);
    {
        const int h2 = P.lh[2], w2 = P.lw[2], y0 = ty0 / 4, x0 = bx / 4;
        float* dst = P.lvl[2] + row * (int64_t)h2 * w2;
#pragma unroll
        for (int y = 0; y < 2; ++y)
#pragma unroll
            for (int x = 0; x < 2; ++x)
                if (y0 + y < h2 && x0 + x < w2) dst[(int64_t)(y0 + y) * w2 + x0 + x] = l2[y][x];
    }
    if (P.fused_levels < 4) return;
    const float l3 = pool4(l2[0][0], l2[0][1], l2[1][0], l2[1][1]);
    const int h3 = P.lh[3], w3 = P.lw[3], y0 = ty0 / 8, x0 = bx / 8;
    if (y0 < h3 && x0 < w3) P.lvl[3][row * (int64_t)h3 * w3 + (int64_t)y0 * w3 + x0] = l3;
}

// Epilogue v3 (all threads, contains barriers).  Cs holds the scaled 128 x 128 C tile ([m][n],
// stride CS, n = ty*16 + tx).  Stores are arranged so that each wave instruction writes whole
// contiguous row pieces of the pyramid (level 0: 16 pieces of 64 B) instead of 64 scattered
// 16-byte pieces: (1) level 0 from LDS, 4 lanes x float4 per (query, target row); (2) each thread
// pools one (query, 8x8 block) in registers, 8x8 -> 4x4 -> 2x2 -> 1, each level from the rounded
// previous one ((x00 + x01) + x10) + x11) / 4, and parks levels 1-3 in LDS (padded strides,
// conflict-free); (3) levels 1-3 leave as contiguous row pieces.
constexpr int P1S = 36, P2S = 12;   // LDS row strides (floats) of the pooled staging, per query

template <int N>
__device__ __forceinline__ void store_row(float* dst, const float* src, int valid, bool vec) {
    // N consecutive floats; vec = the full piece is in range and 4N-byte aligned
    if (vec) {
        if constexpr (N == 4) *reinterpret_cast<floatx4*>(dst) = *reinterpret_cast<const floatx4*>(src);
        else if constexpr (N == 2) *reinterpret_cast<float2*>(dst) = *reinterpret_cast<const float2*>(src);
        else dst[0] = src[0];
    } else {
#pragma unroll
        for (int j = 0; j < N; ++j)
            if (j < valid) dst[j] = src[j];
    }
}

template <bool VEC>
__device__ __forceinline__ void epilogue_v3(const BuildParams& P, const TileCoord& tc, float* Cs, int tid) {
    const int H = P.H, W = P.W;
    const int64_t Q = (int64_t)H * W;
    const int64_t row0 = (int64_t)tc.b * P.q_count + tc.m0;
    const int mvalid = min(BM, P.q_count - tc.m0);
    // (1) level 0
    {
        const int c = tid & 3;
        const int x = tc.tx0 + 4 * c;
        const bool vx = VEC && (x + 4 <= W);
        const int nx = W - x;
#pragma unroll 4
        for (int s = 0; s < (BM * TBH) / (NT / 4); ++s) {
            const int R = (tid >> 2) + (NT / 4) * s;
            const int m = R >> 3, ty = R & 7;
            const int y = tc.ty0 + ty;
            if (m < mvalid && y < H && nx > 0)
                store_row<4>(P.lvl[0] + (row0 + m) * Q + (int64_t)y * W + x, Cs + m * CS + ty * TBW + 4 * c,
                             nx, vx);
        }
    }
    if (P.fused_levels < 2) return;   // uniform: no barrier below is skipped by a subset
    // (2) pooling in registers
    const int m = tid & (BM - 1), blk = tid >> 7;
    float l1[4][4], l2[2][2], l3;
    {
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
    }
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
        for (int x = 0; x < 2; ++x)
            l2[y][x] = pool4(l1[2 * y][2 * x], l1[2 * y][2 * x + 1], l1[2 * y + 1][2 * x], l1[2 * y + 1][2 * x + 1]);
    l3 = pool4(l2[0][0], l2[0][1], l2[1][0], l2[1][1]);
    __syncthreads();   // all level-0 reads of Cs done: reuse it for the pooled staging
    float* S1 = Cs;                       // [BM][4 rows][8 cols], stride P1S
    float* S2 = Cs + BM * P1S;            // [BM][2 rows][4 cols], stride P2S
    float* S3 = S2 + BM * P2S;            // [BM][2 cols]
#pragma unroll
    for (int y = 0; y < 4; ++y)
        *reinterpret_cast<floatx4*>(S1 + m * P1S + y * 8 + blk * 4) = floatx4{l1[y][0], l1[y][1], l1[y][2], l1[y][3]};
#pragma unroll
    for (int y = 0; y < 2; ++y)
        *reinterpret_cast<float2*>(S2 + m * P2S + y * 4 + blk * 2) = float2{l2[y][0], l2[y][1]};
    S3[m * 2 + blk] = l3;
    __syncthreads();
    // (3) levels 1..3 as contiguous row pieces
    {   // level 1: BM x 4 rows x 8 floats = 2 float4 per row
        const int h1 = P.lh[1], w1 = P.lw[1];
        const int64_t hw1 = (int64_t)h1 * w1;
        const int c = tid & 1, x = tc.tx0 / 2 + 4 * c;
        const bool vx = VEC && x + 4 <= w1 && (w1 % 4 == 0) && (hw1 % 4 == 0);
#pragma unroll
        for (int s = 0; s < (BM * 4) / (NT / 2); ++s) {
            const int R = (tid >> 1) + (NT / 2) * s;
            const int mm = R >> 2, y = tc.ty0 / 2 + (R & 3);
            if (mm < mvalid && y < h1 && x < w1)
                store_row<4>(P.lvl[1] + (row0 + mm) * hw1 + (int64_t)y * w1 + x, S1 + mm * P1S + (R & 3) * 8 + 4 * c,
                             w1 - x, vx);
        }
    }
    if (P.fused_levels >= 3) {   // level 2: BM x 2 rows x 4 floats
        const int h2 = P.lh[2], w2 = P.lw[2];
        const int64_t hw2 = (int64_t)h2 * w2;
        const int x = tc.tx0 / 4;
        const bool vx = VEC && x + 4 <= w2 && (w2 % 4 == 0) && (hw2 % 4 == 0);
        const int mm = tid >> 1, y = tc.ty0 / 4 + (tid & 1);
        if (mm < mvalid && y < h2 && x < w2)
            store_row<4>(P.lvl[2] + (row0 + mm) * hw2 + (int64_t)y * w2 + x, S2 + mm * P2S + (tid & 1) * 4, w2 - x, vx);
    }
    if (P.fused_levels >= 4 && tid < BM) {   // level 3: BM x 1 row x 2 floats
        const int h3 = P.lh[3], w3 = P.lw[3];
        const int64_t hw3 = (int64_t)h3 * w3;
        const int x = tc.tx0 / 8, y = tc.ty0 / 8;
        const bool vx = VEC && x + 2 <= w3 && (w3 % 2 == 0) && (hw3 % 2 == 0);
        if (tid < mvalid && y < h3 && x < w3)
            store_row<2>(P.lvl[3] + (row0 + tid) * hw3 + (int64_t)y * w3 + x, S3 + tid * 2, w3 - x, vx);
    }
}

// Variant v1 (row-major [k][row] LDS operands, one tile per block): kept for A/B timing.
// Bijective XCD-aware remap (cdna_hip_programming.md §5 T1): consecutive logical tiles land on
// one XCD so tiles sharing fmap1/fmap2 panels share that XCD's L2.  Speed only, never correctness.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
    const int q = nwg / 8, r = nwg % 8, xcd = bid % 8, k = bid / 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + k;
}

template <bool VEC, int PF>
__global__ __launch_bounds__(NT, 2) void build_kernel_v1(BuildParams P) {
    __shared__ __attribute__((aligned(16))) float smem[SMEM_FLOATS];
    float* As = smem;                       // [2][BK][BM]
    float* Bs = smem + 2 * BK * BM;         // [2][BK][BN]

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const TileCoord tc = decode_tile(P, xcd_remap(blockIdx.x, gridDim.x));
    const int b = tc.b, m0 = tc.m0, ty0 = tc.ty0, tx0 = tc.tx0;
    const int q_end = P.q_count;
    const int H = P.H, W = P.W, D = P.D;
    const int64_t Q = (int64_t)H * W;
    const int64_t QA = P.q_count;
    const float* __restrict__ A = P.f1 + (int64_t)b * D * QA;
    const float* __restrict__ Bm = P.f2 + (int64_t)b * D * Q;

    // ---- global -> register staging (4 float4 of A and 4 of B per thread per K chunk); PF = how
    // many chunks ahead the loads run (PF register sets)
    floatx4 ra[PF][4], rb[PF][4];
    auto load_chunk = [&](int set, int k0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int s = tid + NT * i;
            const int kk = s >> 5;
            const int k = k0 + kk;
            {   // A: row k, queries m0 + 4c .. +3
                const int m = m0 + 4 * (s & 31);
                floatx4 v = {0.f, 0.f, 0.f, 0.f};
                if (VEC) {
                    if (k < D && m < q_end) v = *reinterpret_cast<const floatx4*>(A + (int64_t)k * QA + m);
                } else {
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        if (k < D && m + j < q_end) v[j] = A[(int64_t)k * QA + m + j];
                }
                ra[set][i] = v;
            }
            {   // B: row k, target row ty0 + ty, cols tx0 + 4c .. +3
                const int r = s & 31, ty = r >> 2, c = r & 3;
                const int y = ty0 + ty, x = tx0 + 4 * c;
                floatx4 v = {0.f, 0.f, 0.f, 0.f};
                if (VEC) {
                    if (k < D && y < H && x < W)
                        v = *reinterpret_cast<const floatx4*>(Bm + (int64_t)k * Q + (int64_t)y * W + x);
                } else {
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        if (k < D && y < H && x + j < W) v[j] = Bm[(int64_t)k * Q + (int64_t)y * W + x + j];
                }
                rb[set][i] = v;
            }
        }
    };
    auto store_chunk = [&](int set, int buf) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int s = tid + NT * i;
            const int kk = s >> 5, c = s & 31;
            *reinterpret_cast<floatx4*>(As + (buf * BK + kk) * BM + 4 * c) = ra[set][i];
            *reinterpret_cast<floatx4*>(Bs + (buf * BK + kk) * BN + 4 * c) = rb[set][i];
        }
    };

    floatx16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

    const int wm = wave & 1, wn = wave >> 1;
    const int arow = lane >> 5, acol = lane & 31;
    const int nk = (D + BK - 1) / BK;
    auto compute = [&](int buf) {
        const float* as = As + buf * BK * BM + wm * 64 + acol;
        const float* bs = Bs + buf * BK * BN + wn * 64 + acol;
#pragma unroll
        for (int kk = 0; kk < BK; kk += 2) {
            const int ro = (kk + arow);
            const float a0 = as[ro * BM], a1 = as[ro * BM + 32];
            const float b0 = bs[ro * BN], b1 = bs[ro * BN + 32];
            acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
            acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
            acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
            acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
        }
    };

    if (PF == 1) {
        load_chunk(0, 0);
        store_chunk(0, 0);
        __syncthreads();
        for (int kc = 0; kc < nk; ++kc) {
            const int buf = kc & 1;
            if (kc + 1 < nk) load_chunk(0, (kc + 1) * BK);
            compute(buf);
            if (kc + 1 < nk) store_chunk(0, buf ^ 1);
            __syncthreads();
        }
    } else {
        // two chunks in flight: set (kc & 1) holds chunk kc+1 while chunk kc+2 loads into the other
        load_chunk(0, 0);
        if (nk > 1) load_chunk(1, BK);
        store_chunk(0, 0);
        __syncthreads();
        for (int kc = 0; kc < nk; kc += 2) {
            // even step: LDS buf 0 holds chunk kc; register set 1 holds chunk kc+1
            if (kc + 2 < nk) load_chunk(0, (kc + 2) * BK);
            compute(0);
            if (kc + 1 < nk) store_chunk(1, 1);
            __syncthreads();
            if (kc + 1 >= nk) break;
            // odd step: LDS buf 1 holds chunk kc+1; register set 0 holds chunk kc+2
            if (kc + 3 < nk) load_chunk(1, (kc + 3) * BK);
            compute(1);
            if (kc + 2 < nk) store_chunk(0, 0);
            __syncthreads();
        }
    }

    // ---- epilogue: scaled accumulators -> LDS C tile [m][n], then the shared pooling epilogue
    float* Cs = smem;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * arow;
                const int n = wn * 64 + j * 32 + acol;
                const float v = acc[i][j][r];
                Cs[m * CS + n] = P.scale_is_mul ? __fmul_rn(v, P.scale) : __fdiv_rn(v, P.scale);
            }
    __syncthreads();
    if (P.dev_skip_epilogue) return;
    if (P.dev_epilogue_v2) epilogue_pool<VEC>(P, tc, Cs, tid);
    else epilogue_v3<VEC>(P, tc, Cs, tid);
}

// LDS operand layout (both A and B): [k/8][(k/4)%2][row][k%4].  MFMA step j of k-group g uses, in
// lane half h, k = 8g + 4h + j for A and B alike, so ONE ds_read_b128 per operand row yields the
// fragments of 4 consecutive v_mfma_f32_32x32x2_f32 steps (the k order is a permutation of the
// reference's sum order: the level-0 contract is normwise).  Rows of a 16-lane ds_read_b128
// group are consecutive 16-byte slots: conflict-free.
template <bool VEC>
__global__ __launch_bounds__(NT, 2) void build_kernel(BuildParams P) {
    __shared__ __attribute__((aligned(16))) float smem[SMEM_FLOATS];
    float* As = smem;                       // [2 buf][BK/8][2][BM][4]
    float* Bs = smem + 2 * BK * BM;         // [2 buf][BK/8][2][BN][4]

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int H = P.H, W = P.W, D = P.D;
    const int64_t Q = (int64_t)H * W;
    const int q_end = P.q_count;
    const int64_t QA = P.q_count;         // fmap1 slab row stride (queries)
    const int nk = (D + BK - 1) / BK;

    // persistent schedule: block -> its XCD's contiguous tile range, strided by the XCD's blocks
    const int nxcd = gridDim.x >= 8 ? 8 : 1;
    const int xcd = blockIdx.x % nxcd, local = blockIdx.x / nxcd, nloc = gridDim.x / nxcd;
    const int qx = P.n_tiles / nxcd, rx = P.n_tiles % nxcd;
    const int t_begin = xcd * qx + min(xcd, rx);
    const int t_end = t_begin + qx + (xcd < rx ? 1 : 0);

    // staging: one 4k x 4 block of A and of B per thread per chunk
    const int kb = tid >> 5, cb = tid & 31;
    floatx4 ra[4], rb[4];
    auto load_chunk = [&](const TileCoord& tc, int k0) {
        const float* __restrict__ A = P.f1 + (int64_t)tc.b * D * QA;
        const float* __restrict__ Bm = P.f2 + (int64_t)tc.b * D * Q;
        const int m = tc.m0 + 4 * cb;
        const int y = tc.ty0 + (cb >> 2), x = tc.tx0 + 4 * (cb & 3);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int k = k0 + 4 * kb + i;
            floatx4 va = {0.f, 0.f, 0.f, 0.f}, vb = {0.f, 0.f, 0.f, 0.f};
            if (VEC) {
                if (k < D && m < q_end) va = *reinterpret_cast<const floatx4*>(A + (int64_t)k * QA + m);
                if (k < D && y < H && x < W)
                    vb = *reinterpret_cast<const floatx4*>(Bm + (int64_t)k * Q + (int64_t)y * W + x);
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    if (k < D && m + j < q_end) va[j] = A[(int64_t)k * QA + m + j];
                    if (k < D && y < H && x + j < W) vb[j] = Bm[(int64_t)k * Q + (int64_t)y * W + x + j];
                }
            }
            ra[i] = va;
            rb[i] = vb;
        }
    };
    auto store_chunk = [&](int buf) {   // transpose 4k x 4 -> 4 rows of [k%4]
        const int g = kb >> 1, h = kb & 1;
        float* as = As + ((buf * (BK / 8) + g) * 2 + h) * BM * 4 + 16 * cb;
        float* bs = Bs + ((buf * (BK / 8) + g) * 2 + h) * BN * 4 + 16 * cb;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            *reinterpret_cast<floatx4*>(as + 4 * e) = floatx4{ra[0][e], ra[1][e], ra[2][e], ra[3][e]};
            *reinterpret_cast<floatx4*>(bs + 4 * e) = floatx4{rb[0][e], rb[1][e], rb[2][e], rb[3][e]};
        }
    };

    const int wm = wave & 1, wn = wave >> 1;
    const int hh = lane >> 5, cc = lane & 31;
    float* Cs = smem;

    int t = t_begin + local;
    if (t >= t_end) return;
    TileCoord tc = decode_tile(P, t);
    load_chunk(tc, 0);
    while (true) {
        const int t_next = t + nloc;
        const bool has_next = t_next < t_end;
        const TileCoord tn = has_next ? decode_tile(P, t_next) : tc;
        store_chunk(0);
        __syncthreads();

        floatx16 acc[2][2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

        for (int kc = 0; kc < nk; ++kc) {
            const int buf = kc & 1;
            if (kc + 1 < nk) load_chunk(tc, (kc + 1) * BK);
            else if (has_next) load_chunk(tn, 0);
            const float* as = As + buf * BK * BM + (hh * BM + wm * 64 + cc) * 4;
            const float* bs = Bs + buf * BK * BN + (hh * BN + wn * 64 + cc) * 4;
            floatx4 fa0 = *reinterpret_cast<const floatx4*>(as);
            floatx4 fa1 = *reinterpret_cast<const floatx4*>(as + 32 * 4);
            floatx4 fb0 = *reinterpret_cast<const floatx4*>(bs);
            floatx4 fb1 = *reinterpret_cast<const floatx4*>(bs + 32 * 4);
#pragma unroll
            for (int g = 0; g < BK / 8; ++g) {
                floatx4 na0, na1, nb0, nb1;
                if (g + 1 < BK / 8) {   // prefetch the next k-group's fragments
                    const float* an = as + (g + 1) * 2 * BM * 4;
                    const float* bn = bs + (g + 1) * 2 * BN * 4;
                    na0 = *reinterpret_cast<const floatx4*>(an);
                    na1 = *reinterpret_cast<const floatx4*>(an + 32 * 4);
                    nb0 = *reinterpret_cast<const floatx4*>(bn);
                    nb1 = *reinterpret_cast<const floatx4*>(bn + 32 * 4);
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa0[j], fb0[j], acc[0][0], 0, 0, 0);
                    acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa0[j], fb1[j], acc[0][1], 0, 0, 0);
                    acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa1[j], fb0[j], acc[1][0], 0, 0, 0);
                    acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa1[j], fb1[j], acc[1][1], 0, 0, 0);
                }
                if (g + 1 < BK / 8) { fa0 = na0; fa1 = na1; fb0 = nb0; fb1 = nb1; }
            }
            if (kc + 1 < nk) {
                store_chunk(buf ^ 1);
                __syncthreads();
            }
        }
        __syncthreads();   // every wave is done reading the staging buffers (C tile overlaps them)

        // ---- epilogue 1: scaled accumulators -> LDS C tile [m][n] (stride CS) ----
        const float scale = P.scale;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int m = wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
                    const int n = wn * 64 + j * 32 + cc;
                    const float v = acc[i][j][r];
                    Cs[m * CS + n] = P.scale_is_mul ? __fmul_rn(v, scale) : __fdiv_rn(v, scale);
                }
        __syncthreads();
        if (P.dev_epilogue_v2) epilogue_pool<VEC>(P, tc, Cs, tid);
        else if (!P.dev_skip_epilogue) epilogue_v3<VEC>(P, tc, Cs, tid);
        if (!has_next) break;
        __syncthreads();   // C tile fully consumed before the next tile's staging overwrites it
        t = t_next;
        tc = tn;
    }
}

// Levels beyond the 3 fused ones (num_levels > 4): plain 2x2 floor-mode pooling, one thread per
// output pixel.  Not on the E-RAFT path (num_levels = 4, eraft.py:50).
__global__ __launch_bounds__(256) void pool2_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                    int64_t rows, int h, int w) {
    const int ho = h / 2, wo = w / 2;
    const int64_t n = rows * ho * wo;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t rw = i / ((int64_t)ho * wo);
        const int yx = (int)(i - rw * ho * wo);
        const int y = yx / wo, x = yx - y * wo;
        const float* s = in + rw * h * w + (int64_t)(2 * y) * w + 2 * x;
        out[i] = pool4(s[0], s[1], s[w], s[w + 1]);
    }
}

}  // namespace

static bool vec_ok(const BuildParams& P, const float* lvl0) {
    return (P.W % 4 == 0) && (P.q_count % 4 == 0) && ((uintptr_t)P.f1 % 16 == 0) &&
           ((uintptr_t)P.f2 % 16 == 0) && ((uintptr_t)lvl0 % 16 == 0);
}

int launch_build(const BuildParams& P0, int B, int levels, const int* lh, const int* lw, float* const* lvl,
                 hipStream_t stream) {
    BuildParams P = P0;
    P.n_ntx = (P.W + TBW - 1) / TBW;
    P.n_nt = P.n_ntx * ((P.H + TBH - 1) / TBH);
    P.n_mt = (P.q_count + BM - 1) / BM;
    P.fused_levels = levels < 4 ? levels : 4;
    for (int i = 0; i < 4; ++i) {
        P.lvl[i] = i < levels ? lvl[i] : nullptr;
        P.lh[i] = i < levels ? lh[i] : 0;
        P.lw[i] = i < levels ? lw[i] : 0;
    }
    const int64_t ntiles = (int64_t)B * P.n_mt * P.n_nt;
    if (ntiles <= 0 || ntiles > 0x7fffffff) return ECORR_EINVAL;
    P.n_tiles = (int)ntiles;
    // persistent grid: 2 resident blocks per CU (LDS 67.5 KB, 140-160 VGPRs), a multiple of the
    // 8 XCDs so every XCD owns an equal set of blocks
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess)
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 256;
    // development knobs for A/B timing (tools/ab_build.py); unset in production:
    //   ECORR_BUILD_V2=1               persistent k-permuted-LDS kernel (v2)
    //   ECORR_BUILD_BLOCKS_PER_CU      v2 persistent blocks per CU (0 = one block per tile)
    //   ECORR_BUILD_PF=2               v1 with two K chunks of global loads in flight
    //   ECORR_BUILD_OLD_EPILOGUE=1     per-thread scattered pyramid stores
    //   ECORR_BUILD_SKIP_EPILOGUE=1    ablation: no pyramid stores (output invalid)
    auto knob = [](const char* k) { const char* v = getenv(k); return v ? atoi(v) : -1; };
    P.dev_skip_epilogue = knob("ECORR_BUILD_SKIP_EPILOGUE") == 1;
    P.dev_epilogue_v2 = knob("ECORR_BUILD_OLD_EPILOGUE") == 1;
    const bool vec = vec_ok(P, lvl[0]);
    if (knob("ECORR_BUILD_V2") == 1) {
        const int bpc = knob("ECORR_BUILD_BLOCKS_PER_CU");
        int64_t grid = bpc != 0 ? (int64_t)(bpc > 0 ? bpc : 2) * cus : ntiles;
        if (grid > ntiles) grid = ntiles;
        if (grid >= 8) grid -= grid % 8;
        if (vec) hipLaunchKernelGGL(build_kernel<true>, dim3((unsigned)grid), dim3(NT), 0, stream, P);
        else hipLaunchKernelGGL(build_kernel<false>, dim3((unsigned)grid), dim3(NT), 0, stream, P);
    } else if (knob("ECORR_BUILD_PF") == 2 && vec) {
        hipLaunchKernelGGL((build_kernel_v1<true, 2>), dim3((unsigned)ntiles), dim3(NT), 0, stream, P);
    } else if (vec) {
        hipLaunchKernelGGL((build_kernel_v1<true, 1>), dim3((unsigned)ntiles), dim3(NT), 0, stream, P);
    } else {
        hipLaunchKernelGGL((build_kernel_v1<false, 1>), dim3((unsigned)ntiles), dim3(NT), 0, stream, P);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return ECORR_EHIP - (int)e;
    const int64_t rows = (int64_t)B * P.q_count;
    for (int i = 4; i < levels; ++i) {
        const int64_t n = rows * (lh[i - 1] / 2) * (lw[i - 1] / 2);
        const int grid = (int)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
        hipLaunchKernelGGL(pool2_kernel, dim3(grid), dim3(256), 0, stream, lvl[i - 1], lvl[i], rows,
                           lh[i - 1], lw[i - 1]);
        e = hipGetLastError();
        if (e != hipSuccess) return ECORR_EHIP - (int)e;
    }
    return ECORR_OK;
}

}  // namespace ecorr
