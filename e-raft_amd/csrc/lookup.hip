// lookup.hip -- CorrBlock.__call__ on gfx950: radius-r bilinear window lookup over the pyramid.
//
// Replaces corr.py:29-50 (+ utils.py:7-21 bilinear_sampler, ATen grid_sampler_2d): for query p,
// level i, offsets a (x) and b (y) in [0, 2r]:
//   out[b][i*(2r+1)^2 + a*(2r+1) + b][p] = bilinear(level_i[p], x/2^i + a - r, y/2^i + b - r)
// bit-exact with the reference on CPU (same fp32 op sequence, ecorr_device.h).
//
// The lookup is an HBM-bound gather: each query reads its own (2r+2)^2 window per level and
// nothing is shared between queries.  One workgroup = 64 consecutive queries x 1 level; the
// window staging (phases 0-1) is lookup_stage.h; phase 2 writes every output from LDS with lanes
// = 64 consecutive queries, so each channel store is one 256-byte coalesced row of the NCHW
// output, stored non-temporally.
#include "ecorr_device.h"
#include "ecorr_internal.h"
#include "lookup_stage.h"

namespace ecorr {

namespace {

constexpr int NT = 256;   // threads of the generic kernels

// QB queries per workgroup, 4 threads per query (NTQ = 4 * QB threads); QB = 64 -> 4 waves,
// QB = 16 -> one wave per workgroup (no cross-wave barrier; waves overlap phases freely).
// LDS ~40 KB, so 4 blocks fit a CU.
template <int R, int QB>
__global__ __launch_bounds__(4 * QB) void lookup_staged(LookupParams P) {
    constexpr int NTQ = 4 * QB;
    using WS = WindowStage<R, QB>;
    __shared__ WS st;
    const int tid = threadIdx.x, g = tid % QB, part = tid / QB;
    const int lv = blockIdx.y, b = blockIdx.z;
    const int q0 = blockIdx.x * QB;   // first query of the block (in the slab)
    stage_level<R, QB, NTQ>(st, P, lv, b, q0, tid);

    // ---- phase 2: outputs; lanes = queries -> coalesced channel-row stores
    const int md = st.org[g][2] & 0xff;
    if (md == 2) return;
    float* __restrict__ outp = P.out + ((int64_t)b * P.C + (int64_t)lv * WS::KK) * P.q_count + q0 + g;
    for (int k = part; k < WS::KK; k += 4) {
        const float res = sample_level<R, QB>(st, P, lv, b, q0, g, k, md);
        // non-temporal: the 324-channel output is consumed by the next kernel, not re-read here;
        // keeping it out of the caches leaves the Infinity Cache to the pyramid windows, which the
        // next lookup re-reads (tools/lookup_lab.hip: -11% lookup time)
        __builtin_nontemporal_store(res, outp + (int64_t)k * P.q_count);
    }
}

// 3 threads per query instead of lookup_staged's 4, so that a thread owns whole x-offset columns
// a in {3p, 3p+1, 3p+2} (K = 2r+1 divisible by 3): the x offset and weight load once per column,
// the per-output work is one address add, two ds_read2 and the 8-op ATen blend, and the output
// row of channel k is a buffer store whose channel offset is a scalar (k is wave-uniform because
// a wave is one `part`).  Every thread computes the 2r+1 y chains and the x chains of its own
// columns (+ the two x end points for the window check) in registers, so the only LDS is the
// windows and their origins (31.7 KB at r = 4: 5 blocks per CU).  Round-1 A/B: the 4-thread
// kernel with per-output k decoding 61 vs 48.5 us; chains shared through LDS 2.8% slower.
// PAIR (every level width even): windows staged as 8-byte column pairs (lookup_stage.h).
// QMAX: also the query's largest |sample| over this wave's columns of the level (fmaxf: NaN
// ignored) -> P.qmax[b][3 lv + part][p], the split convc1's column exponent without a re-read.
// PRESPLIT (radius 4): the samples scaled by 2^scale[b][p] and split into f16 hi + lo, written in the
// presplit layout (ecorr_internal.h): the wave's 27 channels as three whole 16-byte groups (hi, lo)
// plus 3 halves packed after all waves' groups -- the conv reads them as its B fragments.
template <int R, int QB, bool PAIR, bool QMAX = false, bool PRESPLIT = false>
__global__ __launch_bounds__(3 * QB) void lookup_cols_reg(LookupParams P) {
    constexpr int NTQ = 3 * QB, K = 2 * R + 1, AP = K / 3;
    static_assert(K % 3 == 0 && QB == kWave, "one wave per part, whole columns per part");
    using WB = WindowBuf<R, QB, PAIR>;
    constexpr int S = WB::S, SW = WB::SW, SP = WB::SP, KK = WB::KK;
    __shared__ WB st;
    const int tid = threadIdx.x, g = tid % QB;
    const int part = __builtin_amdgcn_readfirstlane(tid / QB);   // wave-uniform
    const int lv = blockIdx.y, b = blockIdx.z;
    const int q0 = blockIdx.x * QB;
    const int p = q0 + g;
    const bool valid = p < P.q_count;

    // ---- phase 0 (registers): the window's end-point chains (the origin needs only those); the
    // other chains are computed under the staging loads' latency (round 4: 41.7-41.9 vs 42.0-42.3 us
    // smooth, 45.7-46.0 vs 45.9-46.2 us i.i.d., profiles/r04_lab/)
    float fy[K], wy[K], fx[AP], wx[AP], x0 = 0.0f, xl = 0.0f;
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
    }
    int org[3];
    window_origin<S, PAIR>(valid, x0, xl, fy[0], fy[K - 1], org);
    if (part == 0) {
        st.org[g][0] = org[0];
        st.org[g][1] = org[1];
        st.org[g][2] = org[2];
    }
    __syncthreads();
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

    const int md = org[2] & 0xff;
    // past the range: no barrier follows, except in the presplit form (its leftover exchange), whose
    // lanes past the range stay to reach the barriers and store nothing (a whole wave of them: the
    // workgroup's three waves share their queries, so all three have ended)
    if (md == 2 && !PRESPLIT) return;
    static_assert(!PRESPLIT || (R == 4 && !QMAX), "presplit: radius 4, 27 channels per wave");
    float vv[PRESPLIT ? K * AP : 1];   // presplit: the wave's 27 samples, k = 9 ai + bb
    // presplit stores: groups g = 9 lv + 3 part + j (k = 8 j .. 8 j + 7), each written as soon as its
    // 8th sample exists (their registers die there: 95 -> 144 VGPRs when all 27 stayed live); the
    // halves k = 24 .. 26 go through LDS to the level's two leftover groups 9 L + 2 lv (+ 1), written
    // whole by waves 0 and 1 after the exchange; default store policy (the conv reads them right
    // back).  Wide stores keep soffset = 0 (tests/test_isa_store_hazard.py).
    typedef _Float16 h8 __attribute__((ext_vector_type(8)));
    typedef unsigned int u4 __attribute__((ext_vector_type(4)));
    const int64_t pbytes = PRESPLIT ? presplit_bytes_per_item(presplit_positions(P.levels), P.q_count) : 0;
    const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<char*>(P.out) + (int64_t)b * pbytes, 0, (int)pbytes, 0x00020000);
    const float psc = PRESPLIT && valid ? __int_as_float((P.scale[(int64_t)b * P.q_count + p] + 127) << 23) : 0.0f;
    uint32_t left[3] = {0, 0, 0};   // presplit: the leftover halves, hi | lo << 16
    auto put = [&](int k, float v) __attribute__((always_inline)) {
        vv[k] = v;
        const int Q = P.q_count;
        if (k % 8 == 7 && k < 24) {
            const int j = k / 8;
            h8 hi, lo;
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                const float x = __fmul_rn(vv[8 * j + t], psc);
                const _Float16 h = (_Float16)x;
                hi[t] = h;
                lo[t] = (_Float16)__fsub_rn(x, (float)h);
            }
            const int off = ((9 * lv + 3 * part + j) * 2 * Q + p) * 16;
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, hi), prs, off, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, lo), prs, off + Q * 16, 0, 0);
        }
        if (k >= 24) {
            const float x = __fmul_rn(v, psc);
            const _Float16 h = (_Float16)x, l = (_Float16)__fsub_rn(x, (float)h);
            left[k - 24] = (uint32_t)__builtin_bit_cast(unsigned short, h) |
                           (uint32_t)__builtin_bit_cast(unsigned short, l) << 16;
        }
    };
    const __amdgpu_buffer_rsrc_t orsrc = __builtin_amdgcn_make_buffer_rsrc(
        P.out + (int64_t)b * P.C * P.q_count, 0, P.C * P.q_count * 4, 0x00020000);
    const int voff = p * 4;
    const int sbase = lv * KK * P.q_count * 4;
    // output stores: non-temporal (round 3: 42.4 vs 46.9 us plain); the QMAX lookup's corr is read
    // right back by the split convc1, so it keeps the default policy and the corr stays in the
    // caches: lookup + conv 97.4 vs 111.0 us (profiles/r04_lab/r4o_ab_qmax.txt)
    constexpr int kOutAux = QMAX ? 0 : 2;
    float vmax = 0.0f;
    if (md == 0) {
        int yo[K];
#pragma unroll
        for (int bb = 0; bb < K; ++bb) yo[bb] = ((int)fy[bb] - org[1]) * SW;
        const float* wq = st.win + WB::W0 + g * SP;
#pragma unroll
        for (int ai = 0; ai < AP; ++ai) {
            const int a = part * AP + ai;
            const float* wc = wq + ((int)fx[ai] - org[0]);
#pragma unroll
            for (int bb = 0; bb < K; ++bb) {
                const float* c = wc + yo[bb];
                const float v = blend(c[0], c[1], c[SW], c[SW + 1], wx[ai], wy[bb]);
                if constexpr (QMAX) vmax = fmaxf(vmax, fabsf(v));
                if constexpr (PRESPLIT)
                    put(ai * K + bb, v);
                else
                    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), orsrc, voff,
                                                          sbase + (a * K + bb) * P.q_count * 4, kOutAux);
            }
        }
    } else if (md == 1) {   // coordinates that do not fit the window: exact direct gather
#pragma unroll
        for (int ai = 0; ai < AP; ++ai)
#pragma unroll
            for (int bb = 0; bb < K; ++bb) {
                const float v = sample_direct(P, lv, b, p, fx[ai], fy[bb], wx[ai], wy[bb]);
                if constexpr (QMAX) vmax = fmaxf(vmax, fabsf(v));
                if constexpr (PRESPLIT)
                    put(ai * K + bb, v);
                else
                    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), orsrc, voff,
                                                          sbase + ((part * AP + ai) * K + bb) * P.q_count * 4, kOutAux);
            }
    }
    if constexpr (QMAX)
        if (valid) P.qmax[((int64_t)b * 3 * P.levels + 3 * lv + part) * P.q_count + p] = vmax;
    if constexpr (PRESPLIT) {   // the level's 9 leftover halves per query -> groups 9 L + 2 lv (+ 1)
        __syncthreads();   // every wave's window reads done: the window buffer becomes the exchange
        uint32_t* xch = reinterpret_cast<uint32_t*>(st.win);   // [9][QB], 2.3 KB
#pragma unroll
        for (int i = 0; i < 3; ++i) xch[(3 * part + i) * QB + g] = left[i];
        __syncthreads();
        if (part < 2 && md != 2) {   // wave 0: leftovers 0-7, wave 1: leftover 8 + 7 zero halves
            h8 hi, lo;
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                const uint32_t u = (part == 0 || t == 0) ? xch[(8 * part + t) * QB + g] : 0u;
                hi[t] = __builtin_bit_cast(_Float16, (unsigned short)(u & 0xffff));
                lo[t] = __builtin_bit_cast(_Float16, (unsigned short)(u >> 16));
            }
            const int Q = P.q_count;
            const int off = ((9 * P.levels + 2 * lv + part) * 2 * Q + p) * 16;
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, hi), prs, off, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, lo), prs, off + Q * 16, 0, 0);
        }
    }
}

// Partial maxima for the lookups without a QMAX instantiation: thread = (b, query), the max of |out|
// over all C channels into group 0, zeros into the other 3 * levels - 1.
__global__ __launch_bounds__(NT) void qmax_kernel(LookupParams P, int B) {
    const int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x;
    if (i >= (int64_t)B * P.q_count) return;
    const int64_t b = i / P.q_count, p = i % P.q_count, Q = P.q_count, G = 3 * P.levels;
    float m = 0.0f;
    for (int c = 0; c < P.C; ++c) m = fmaxf(m, fabsf(P.out[(b * P.C + c) * Q + p]));
    for (int g = 0; g < G; ++g) P.qmax[(b * G + g) * Q + p] = g == 0 ? m : 0.0f;
}

// Any radius: one thread per output element, direct gather (reference-shaped; used for radii
// without a staged instantiation).
__global__ __launch_bounds__(NT) void lookup_direct(LookupParams P, int B) {
    const int K = 2 * P.radius + 1, KK = K * K;
    const int64_t n = (int64_t)B * P.C * P.q_count;
    const int64_t Q = P.q_count;
    for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
        const int64_t bc = i / P.q_count;
        const int qq = (int)(i - bc * P.q_count);
        const int b = (int)(bc / P.C), ch = (int)(bc - (int64_t)b * P.C);
        const int lv = ch / KK, k = ch - lv * KK, a = k / K, bb = k - a * K;
        const int h = P.lh[lv], w = P.lw[lv];
        const int p = qq;
        const float inv = 1.0f / (float)(1 << lv);
        const float cx = __fmul_rn(P.coords[((int64_t)b * 2 + 0) * Q + p], inv);
        const float cy = __fmul_rn(P.coords[((int64_t)b * 2 + 1) * Q + p], inv);
        P.out[i] = sample_level_px(P.lvl[lv], (int64_t)b * P.q_count + qq, lv, P.lntx[lv], h, w, P.lsz[lv],
                                   __fadd_rn(cx, (float)(a - P.radius)), __fadd_rn(cy, (float)(bb - P.radius)));
    }
}

// utils.py:7-21 for arbitrary img [N][C][h][w] and pixel grid [N][Hg][Wg][2].
__global__ __launch_bounds__(NT) void sampler_kernel(const float* __restrict__ img, int N, int C, int h, int w,
                                                     const float* __restrict__ coords, int64_t G,
                                                     float* __restrict__ out, float* __restrict__ mask) {
    const int64_t n = (int64_t)N * G;
    for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
        const int64_t ni = i / G, gi = i - ni * G;
        const float x = coords[2 * i], y = coords[2 * i + 1];
        for (int c = 0; c < C; ++c)
            out[(ni * C + c) * G + gi] = sample_px(img + (ni * C + c) * (int64_t)h * w, h, w, x, y);
        if (mask) {  // utils.py:17-19, on the normalized coordinates
            const float gx = __fsub_rn(__fdiv_rn(__fmul_rn(2.0f, x), (float)(w - 1)), 1.0f);
            const float gy = __fsub_rn(__fdiv_rn(__fmul_rn(2.0f, y), (float)(h - 1)), 1.0f);
            mask[i] = ((gx > -1.0f) & (gy > -1.0f) & (gx < 1.0f) & (gy < 1.0f)) ? 1.0f : 0.0f;
        }
    }
}

// utils.py:24-27
__global__ __launch_bounds__(NT) void coords_grid_kernel(int B, int H, int W, float* __restrict__ out) {
    const int64_t hw = (int64_t)H * W, n = (int64_t)B * 2 * hw;
    for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
        const int64_t pix = i % hw;
        const int ch = (int)((i / hw) & 1);
        out[i] = ch == 0 ? (float)(pix % W) : (float)(pix / W);
    }
}

// Presplit column exponents (ecorr_split_column_scale).  Every sample of query p (any level: pooled
// averages and bilinear blends of level-0 values) is bounded by max_t |corr0[p][t]| <=
// sqrt(D) m1_p M2 (Cauchy-Schwarz on |f| <= max |f|), m1_p = max_d |f1[d][p]|, M2 = max |f2| over
// the batch item; with m < 2^(15 - split_exponent(m)) and sqrt(D) <= 2^hd the scale
// 2^(e1 + E2 - 15 - hd) puts every sample below 2^15 (f16 max 65504: 2x headroom for rounding).
// A loose bound only lowers the samples' magnitude, not their 22-bit hi + lo precision, until lo
// falls under f16's normal range (scaled |x| < 2^-3).  The maxima are over finite values: a sample
// touching a non-finite fmap value is non-finite itself (and NaNs its query in the conv, the split
// contract), every other sample is bounded by the finite values it was made of.
__device__ __forceinline__ int colscale_exponent(float m) {   // conv.hip split_exponent
    int E = 0;
    frexpf(m, &E);
    const int e = (m > 0.f && m <= 3.4028235e38f) ? 15 - E : 0;
    return e < -126 ? -126 : (e > 126 ? 126 : e);
}

// max |f2| (finite) per batch item as float bits (non-negative floats order as unsigned ints)
__global__ __launch_bounds__(NT) void colscale_m2_kernel(const float* __restrict__ f2, int64_t n,
                                                         unsigned* __restrict__ m2) {
    __shared__ unsigned red[NT / 64];
    const int b = blockIdx.y;
    const float* x = f2 + (int64_t)b * n;
    unsigned m = 0;
    auto take = [&](float v) {   // finite values only (below)
        const unsigned u = __float_as_uint(v) & 0x7fffffffu;
        m = u < 0x7f800000u ? max(m, u) : m;
    };
    if (n % 4 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0) {   // 16-byte loads
        const float4* x4 = reinterpret_cast<const float4*>(x);
#pragma unroll 4
        for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < n / 4; i += (int64_t)gridDim.x * NT) {
            const float4 v = x4[i];
            take(v.x), take(v.y), take(v.z), take(v.w);
        }
    } else {
        for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) take(x[i]);
    }
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) m = max(m, (unsigned)__shfl_xor((int)m, d));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < NT / 64; ++w) m = max(m, red[w]);
        atomicMax(&m2[b], m);
    }
}

__global__ __launch_bounds__(NT) void colscale_kernel(const float* __restrict__ f1, int B, int D, int Q, int hd,
                                                      const unsigned* __restrict__ m2, int* __restrict__ scale) {
    const int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x;
    if (i >= (int64_t)B * Q) return;
    const int64_t b = i / Q, p = i - b * Q;
    const float* x = f1 + b * D * Q + p;
    unsigned m = 0;
#pragma unroll 16
    for (int d = 0; d < D; ++d) {   // 16 loads in flight per thread (coalesced over the queries)
        const unsigned u = __float_as_uint(x[(int64_t)d * Q]) & 0x7fffffffu;
        m = u < 0x7f800000u ? max(m, u) : m;
    }
    const int s = colscale_exponent(__uint_as_float(m)) + colscale_exponent(__uint_as_float(m2[b])) - 15 - hd;
    scale[i] = s < -126 ? -126 : (s > 126 ? 126 : s);
}

inline unsigned grid_for(int64_t n) {
    const int64_t g = (n + NT - 1) / NT;
    return (unsigned)(g < 8192 ? (g > 0 ? g : 1) : 8192);
}

inline int hip_status() {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? ECORR_OK : ECORR_EHIP - (int)e;
}

}  // namespace

int launch_lookup(const LookupParams& P, int B, hipStream_t stream) {
    // the paths without a QMAX instantiation: the lookup, then qmax_kernel over its output
    auto done = [&]() {
        const int st = hip_status();
        if (st != ECORR_OK || !P.qmax) return st;
        hipLaunchKernelGGL(qmax_kernel, dim3(grid_for((int64_t)B * P.q_count)), dim3(NT), 0, stream, P, B);
        return hip_status();
    };
    if (P.radius > 4) {
        const int64_t n = (int64_t)B * P.C * P.q_count;
        hipLaunchKernelGGL(lookup_direct, dim3(grid_for(n)), dim3(NT), 0, stream, P, B);
        return done();
    }
    const dim3 grid((unsigned)((P.q_count + 63) / 64), (unsigned)P.levels, (unsigned)B);
    const bool cols = (P.radius == 4 || P.radius == 1) && (int64_t)P.C * P.q_count * 4 < 0x7fffffff;
    if (cols) {
        bool pair = true;   // column-pair staging: every level width even, 8-byte aligned levels
        for (int lv = 0; lv < P.levels; ++lv) pair &= P.lw[lv] % 2 == 0 && (uintptr_t)P.lvl[lv] % 8 == 0;
        if (P.radius == 4 && P.scale) {
            if (pair) hipLaunchKernelGGL((lookup_cols_reg<4, 64, true, false, true>), grid, dim3(192), 0, stream, P);
            else hipLaunchKernelGGL((lookup_cols_reg<4, 64, false, false, true>), grid, dim3(192), 0, stream, P);
            return hip_status();
        }
        if (P.radius == 4 && P.qmax) {
            if (pair) hipLaunchKernelGGL((lookup_cols_reg<4, 64, true, true>), grid, dim3(192), 0, stream, P);
            else hipLaunchKernelGGL((lookup_cols_reg<4, 64, false, true>), grid, dim3(192), 0, stream, P);
            return hip_status();
        }
        if (P.radius == 4) {
            if (pair) hipLaunchKernelGGL((lookup_cols_reg<4, 64, true>), grid, dim3(192), 0, stream, P);
            else hipLaunchKernelGGL((lookup_cols_reg<4, 64, false>), grid, dim3(192), 0, stream, P);
        } else {
            if (pair) hipLaunchKernelGGL((lookup_cols_reg<1, 64, true>), grid, dim3(192), 0, stream, P);
            else hipLaunchKernelGGL((lookup_cols_reg<1, 64, false>), grid, dim3(192), 0, stream, P);
        }
        return done();
    }
    switch (P.radius) {
        case 0: hipLaunchKernelGGL((lookup_staged<0, 64>), grid, dim3(256), 0, stream, P); break;
        case 1: hipLaunchKernelGGL((lookup_staged<1, 64>), grid, dim3(256), 0, stream, P); break;
        case 2: hipLaunchKernelGGL((lookup_staged<2, 64>), grid, dim3(256), 0, stream, P); break;
        case 3: hipLaunchKernelGGL((lookup_staged<3, 64>), grid, dim3(256), 0, stream, P); break;
        default: hipLaunchKernelGGL((lookup_staged<4, 64>), grid, dim3(256), 0, stream, P); break;
    }
    return done();
}

int launch_bilinear_sampler(const float* img, int N, int C, int h, int w, const float* coords,
                            int Hg, int Wg, float* out, float* mask, hipStream_t stream) {
    const int64_t G = (int64_t)Hg * Wg;
    hipLaunchKernelGGL(sampler_kernel, dim3(grid_for((int64_t)N * G)), dim3(NT), 0, stream, img, N, C, h,
                       w, coords, G, out, mask);
    return hip_status();
}

int launch_coords_grid(int B, int H, int W, float* out, hipStream_t stream) {
    hipLaunchKernelGGL(coords_grid_kernel, dim3(grid_for((int64_t)B * 2 * H * W)), dim3(NT), 0, stream, B,
                       H, W, out);
    return hip_status();
}

int launch_split_column_scale(const float* f1, const float* f2, int B, int D, int H, int W, int* scale,
                              hipStream_t stream) {
    const int64_t Q = (int64_t)H * W;
    if (B <= 0 || D <= 0 || Q <= 0 || B > 65535 || Q > 0x7fffffff) return ECORR_EINVAL;
    int hd = 0;
    while (((int64_t)1 << (2 * hd)) < D) ++hd;   // sqrt(D) <= 2^hd
    unsigned* m2 = reinterpret_cast<unsigned*>(scale + B * Q);
    const hipError_t e = hipMemsetAsync(m2, 0, (size_t)B * 4, stream);
    if (e != hipSuccess) return ECORR_EHIP - (int)e;
    const int64_t n = (int64_t)D * Q;
    const unsigned gx = (unsigned)std::min<int64_t>((n + NT * 64 - 1) / (NT * 64), 1024);
    hipLaunchKernelGGL(colscale_m2_kernel, dim3(gx, B), dim3(NT), 0, stream, f2, n, m2);
    hipLaunchKernelGGL(colscale_kernel, dim3((unsigned)((B * Q + NT - 1) / NT)), dim3(NT), 0, stream, f1, B, D, (int)Q,
                       hd, m2, scale);
    return hip_status();
}

}  // namespace ecorr
