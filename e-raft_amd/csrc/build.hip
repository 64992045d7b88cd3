// build.hip -- CorrBlock build on gfx950: all-pairs correlation GEMM on fp32 MFMA with the
// 1/sqrt(D) scale and the 3 pooled pyramid levels fused into the epilogue.
//
// Replaces corr.py:13-27 (CorrBlock.__init__) and corr.py:52-60 (CorrBlock.corr):
//   level0[b*q_count + p'][y][x] = (sum_d f1[b][d][p] * f2[b][d][y*W+x]) / sqrt(D)
//   level{i+1} = (((x00 + x01) + x10) + x11) / 4 over 2x2 floor-mode windows of level i.
//
// GEMM view per batch item: A = f1[b] as [K=D][M=Q] (M contiguous), B = f2[b] as [K][N=Q].
// Block tile: 128 queries (M) x one 8x16 block of target pixels (N = 128), K staged 32 deep
// through double-buffered LDS; 4 waves, each 64x64 = 2x2 v_mfma_f32_32x32x2_f32 tiles.  The N
// tile is a 2D target block so the epilogue can pool 3 levels locally: each thread owns one
// (query, 8x8 target block) and reduces it 8x8 -> 4x4 -> 2x2 -> 1 in registers, from the rounded
// previous level, in the reference's summation order.
//
// Numerics: MFMA f32 is an exact k-ordered fmaf chain; against the reference's sgemm the level-0
// agreement is normwise (max|d|/rms <= 1e-5), pooling is bit-exact given the same level 0.
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

// Bijective XCD-aware remap (cdna_hip_programming.md §5 T1): consecutive logical tiles land on
// one XCD so tiles sharing fmap1/fmap2 panels share that XCD's L2.  Speed only, never correctness.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
    const int q = nwg / 8, r = nwg % 8, xcd = bid % 8, k = bid / 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + k;
}

template <bool VEC>
__global__ __launch_bounds__(NT, 2) void build_kernel(BuildParams P) {
    __shared__ __attribute__((aligned(16))) float smem[SMEM_FLOATS];
    float* As = smem;                       // [2][BK][BM]
    float* Bs = smem + 2 * BK * BM;         // [2][BK][BN]

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int tile = xcd_remap(blockIdx.x, gridDim.x);
    const int per_b = P.n_mt * P.n_nt;
    const int b = tile / per_b;
    const int rem = tile - b * per_b;
    const int mt = rem / P.n_nt, nt = rem - mt * P.n_nt;
    const int nty = nt / P.n_ntx, ntx = nt - nty * P.n_ntx;
    const int m0 = P.q_begin + mt * BM;     // first query (within batch item) of this tile
    const int q_end = P.q_begin + P.q_count;
    const int ty0 = nty * TBH, tx0 = ntx * TBW;
    const int H = P.H, W = P.W, D = P.D;
    const int64_t Q = (int64_t)H * W;
    const float* __restrict__ A = P.f1 + (int64_t)b * D * Q;
    const float* __restrict__ Bm = P.f2 + (int64_t)b * D * Q;

    // ---- global -> register staging (4 float4 of A and 4 of B per thread per K chunk) ----
    floatx4 ra[4], rb[4];
    auto load_chunk = [&](int k0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int s = tid + NT * i;
            const int kk = s >> 5;
            const int k = k0 + kk;
            {   // A: row k, queries m0 + 4c .. +3
                const int m = m0 + 4 * (s & 31);
                floatx4 v = {0.f, 0.f, 0.f, 0.f};
                if (VEC) {
                    if (k < D && m < q_end) v = *reinterpret_cast<const floatx4*>(A + (int64_t)k * Q + m);
                } else {
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        if (k < D && m + j < q_end) v[j] = A[(int64_t)k * Q + m + j];
                }
                ra[i] = v;
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
                rb[i] = v;
            }
        }
    };
    auto store_chunk = [&](int buf) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int s = tid + NT * i;
            const int kk = s >> 5, c = s & 31;
            *reinterpret_cast<floatx4*>(As + (buf * BK + kk) * BM + 4 * c) = ra[i];
            *reinterpret_cast<floatx4*>(Bs + (buf * BK + kk) * BN + 4 * c) = rb[i];
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

    load_chunk(0);
    store_chunk(0);
    __syncthreads();
    for (int kc = 0; kc < nk; ++kc) {
        const int buf = kc & 1;
        if (kc + 1 < nk) load_chunk((kc + 1) * BK);
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
        if (kc + 1 < nk) store_chunk(buf ^ 1);
        __syncthreads();
    }

    // ---- epilogue 1: scaled accumulators -> LDS C tile [m][n] (stride CS) ----
    float* Cs = smem;
    const float scale = P.scale;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * arow;
                const int n = wn * 64 + j * 32 + acol;
                const float v = acc[i][j][r];
                Cs[m * CS + n] = P.scale_is_mul ? __fmul_rn(v, scale) : __fdiv_rn(v, scale);
            }
    __syncthreads();

    // ---- epilogue 2: thread = (query m, 8x8 target block blk); pool in registers ----
    const int m = tid & (BM - 1), blk = tid >> 7;
    const int qm = m0 + m;
    if (qm >= q_end) return;
    const int64_t row = (int64_t)b * P.q_count + (qm - P.q_begin);
    float v[8][8];
#pragma unroll
    for (int ty = 0; ty < 8; ++ty) {
        const floatx4 lo = *reinterpret_cast<const floatx4*>(Cs + m * CS + ty * TBW + blk * 8);
        const floatx4 hi = *reinterpret_cast<const floatx4*>(Cs + m * CS + ty * TBW + blk * 8 + 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) { v[ty][j] = lo[j]; v[ty][4 + j] = hi[j]; }
    }
    const int bx = tx0 + blk * 8;  // level-0 column of this 8x8 block
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
    {
        const float l3 = pool4(l2[0][0], l2[0][1], l2[1][0], l2[1][1]);
        const int h3 = P.lh[3], w3 = P.lw[3], y0 = ty0 / 8, x0 = bx / 8;
        if (y0 < h3 && x0 < w3) P.lvl[3][row * (int64_t)h3 * w3 + (int64_t)y0 * w3 + x0] = l3;
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
    const int64_t nblk = (int64_t)B * P.n_mt * P.n_nt;
    if (nblk <= 0 || nblk > 0x7fffffff) return ECORR_EINVAL;
    const bool vec = (P.W % 4 == 0) && (P.q_begin % 4 == 0) && (P.q_count % 4 == 0) &&
                     ((uintptr_t)P.f1 % 16 == 0) && ((uintptr_t)P.f2 % 16 == 0) &&
                     ((uintptr_t)lvl[0] % 16 == 0);
    if (vec)
        hipLaunchKernelGGL(build_kernel<true>, dim3((unsigned)nblk), dim3(NT), 0, stream, P);
    else
        hipLaunchKernelGGL(build_kernel<false>, dim3((unsigned)nblk), dim3(NT), 0, stream, P);
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
