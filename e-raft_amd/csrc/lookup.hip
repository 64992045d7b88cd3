// lookup.hip -- CorrBlock.__call__ on gfx950: radius-r bilinear window lookup over the pyramid.
//
// Replaces corr.py:29-50 (+ utils.py:7-21 bilinear_sampler, ATen grid_sampler_2d): for query p,
// level i, offsets a (x) and b (y) in [0, 2r]:
//   out[b][i*(2r+1)^2 + a*(2r+1) + b][p] = bilinear(level_i[p], x/2^i + a - r, y/2^i + b - r)
// bit-exact with the reference on CPU (same fp32 op sequence, ecorr_device.h).
//
// The lookup is an HBM-bound gather: each query reads its own (2r+2)^2 window per level and
// nothing is shared between queries.  Design (one workgroup = 64 consecutive queries x 1 level):
//   phase 0  the 2(2r+1) coordinate chains per query (x chains depend on a only, y chains on b
//            only, so 18 instead of 162 chains at r=4) -> floor + fraction into LDS;
//   phase 1  cooperative staging of each query's (2r+3)^2 window (one slack row/column absorbs
//            the +-1 floor flips of the unnormalize round trip) into LDS, zero-filled outside the
//            image, with clamped (always valid) addresses;
//   phase 2  every output from LDS; lanes = 64 consecutive queries so each channel store is one
//            256-byte coalesced row of the NCHW output, stored non-temporally.
// Queries whose floors do not fit the staged window (NaN/inf/huge coordinates) take an exact
// direct-gather path inside phase 2.
#include <stdlib.h>

#include "ecorr_device.h"
#include "ecorr_internal.h"

namespace ecorr {

namespace {

constexpr int NT = 256;   // threads of the generic kernels

// QB queries per workgroup, 4 threads per query (NTQ = 4 * QB threads); QB = 64 -> 4 waves,
// QB = 16 -> one wave per workgroup (no cross-wave barrier; waves overlap phases freely).
template <int R, int QB>
__global__ __launch_bounds__(4 * QB) void lookup_staged(LookupParams P) {
    constexpr int NTQ = 4 * QB;
    constexpr int K = 2 * R + 1;   // samples per axis
    constexpr int KK = K * K;
    constexpr int S = 2 * R + 3;   // staged window side
    constexpr int SS = S * S;
    constexpr int SP = SS | 1;     // odd per-query stride: conflict-free lanes = queries
    __shared__ float win[QB * SP];
    __shared__ float fx[QB][K], wx[QB][K], fy[QB][K], wy[QB][K];
    // per query: window origin x, y and (mode | needed cols << 8 | needed rows << 16), where mode
    // 0 = staged, 1 = direct gather (coordinates that do not fit the window), 2 = past the range.
    // Kept at 40 KB of LDS in total so 4 blocks fit a CU.
    __shared__ int org[QB][3];

    const int tid = threadIdx.x, g = tid & (QB - 1), part = tid / QB;
    const int lv = blockIdx.y, b = blockIdx.z;
    const int h = P.lh[lv], w = P.lw[lv], ntx = P.lntx[lv];
    const int q0 = blockIdx.x * QB;                 // first query of the block (in the slab)
    const int p = q0 + g;
    const bool valid = p < P.q_count;
    const int64_t Q = P.q_count;                    // coords slab stride
    const int64_t hw = P.lsz[lv];                   // floats per query image (tiled, padded)
    const float* __restrict__ lvbase = P.lvl[lv] + ((int64_t)b * P.q_count + q0) * hw;

    // ---- phase 0: coordinate chains (corr.py:41-43, utils.py:11-12, grid_sampler unnormalize)
    if (valid) {
        const float inv = 1.0f / (float)(1 << lv);  // coords / 2**i is an exact scaling
        const float cx = __fmul_rn(P.coords[((int64_t)b * 2 + 0) * Q + p], inv);
        const float cy = __fmul_rn(P.coords[((int64_t)b * 2 + 1) * Q + p], inv);
        const float wm1 = (float)(w - 1), hm1 = (float)(h - 1);
#pragma unroll
        for (int j = part; j < 2 * K; j += 4) {
            const bool isx = j < K;
            const int o = isx ? j : j - K;
            const float c = __fadd_rn(isx ? cx : cy, (float)(o - R));
            const float m1 = isx ? wm1 : hm1;
            const float v = unnormalize(c, m1, m1 * 0.5f);
            const float f = floorf(v);
            if (isx) { fx[g][o] = f; wx[g][o] = __fsub_rn(v, f); }
            else     { fy[g][o] = f; wy[g][o] = __fsub_rn(v, f); }
        }
    }
    __syncthreads();

    // ---- phase 0b: window origin and fast/slow decision per query
    if (part == 0) {
        int md = 2, X0 = 0, Y0 = 0, NX = 0, NY = 0;
        if (valid) {
            const float x0 = fx[g][0], y0 = fy[g][0];
            bool ok = fabsf(x0) < 1.0e7f && fabsf(y0) < 1.0e7f;  // false for NaN / inf / huge
#pragma unroll
            for (int o = 0; o < K; ++o) {
                const float dx = fx[g][o] - x0, dy = fy[g][o] - y0;  // exact: integers < 2^24
                ok &= (dx >= 0.0f) & (dx <= (float)(S - 2)) & (dy >= 0.0f) & (dy <= (float)(S - 2));
            }
            md = ok ? 0 : 1;
            X0 = ok ? (int)x0 : 0;
            Y0 = ok ? (int)y0 : 0;
            // corners span [x0, floor(ix_last) + 1]: monotone round trip, so the last sample bounds it
            NX = ok ? (int)(fx[g][K - 1] - x0) + 2 : 0;
            NY = ok ? (int)(fy[g][K - 1] - y0) + 2 : 0;
        }
        org[g][0] = X0;
        org[g][1] = Y0;
        org[g][2] = md | (NX << 8) | (NY << 16);
    }
    __syncthreads();

    // ---- phase 1: stage windows, zeros outside the image (grid_sample padding_mode='zeros').
    // Work item = (query, window column); each item walks the S rows.  Loads are raw buffer loads
    // over this block's slab of the level: an element outside the image gets an out-of-range
    // offset and the hardware range check returns 0 -- zero padding with no branch and no select,
    // so all NCOL*S loads of a thread issue back to back.
    constexpr int ITEMS = QB * S;
    constexpr int NCOL = (ITEMS + NTQ - 1) / NTQ;
    const int nq = min(QB, P.q_count - q0);
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(lvbase), 0, (int)(nq * hw * 4), 0x00020000);
    constexpr int OOB = 0x7ffffff0;   // beyond any slab: reads as 0
    float vals[NCOL][S];
    int dst[NCOL];
#pragma unroll
    for (int c = 0; c < NCOL; ++c) {
        const int it = tid + c * NTQ;
        const bool live = it < ITEMS;
        const int gq = live ? it / S : 0;
        const int rx = it - gq * S;
        const int x = org[gq][0] + rx, y0 = org[gq][1], info = org[gq][2];
        const int ny = (info >> 16) & 0xff;
        // only the needed corner rectangle touches memory; the slack row/column reads 0 for free
        const bool colin = live && (info & 0xff) == 0 && rx < ((info >> 8) & 0xff) && (unsigned)x < (unsigned)w;
        const int base = (int)(gq * hw);
        dst[c] = live ? gq * SP + rx : -1;
#pragma unroll
        for (int ry = 0; ry < S; ++ry) {
            const int y = y0 + ry;
            const int off = (colin && ry < ny && (unsigned)y < (unsigned)h) ? (base + level_off(y, x, ntx, w)) * 4 : OOB;
            vals[c][ry] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsrc, off, 0, 0));
        }
    }
#pragma unroll
    for (int c = 0; c < NCOL; ++c)
        if (dst[c] >= 0)
#pragma unroll
            for (int ry = 0; ry < S; ++ry) win[dst[c] + ry * S] = vals[c][ry];
    __syncthreads();

    // ---- phase 2: outputs; lanes = queries -> coalesced channel-row stores
    const int md = org[g][2] & 0xff;
    if (md == 2) return;
    float* __restrict__ outp = P.out + ((int64_t)b * P.C + (int64_t)lv * KK) * P.q_count + q0 + g;
    const int X0 = org[g][0], Y0 = org[g][1];
    const float* wq = win + g * SP;
    const float* img = lvbase + (int64_t)g * hw;
    for (int k = part; k < KK; k += 4) {
        const int a = k / K, bb = k - a * K;
        const float xa = fx[g][a], yb = fy[g][bb];
        const float wa = wx[g][a], nb = wy[g][bb];
        float res;
        if (md == 0) {
            const float* c = wq + ((int)yb - Y0) * S + ((int)xa - X0);
            res = blend(c[0], c[1], c[S], c[S + 1], wa, nb);
        } else {
            const float xa1 = __fadd_rn(xa, 1.0f), yb1 = __fadd_rn(yb, 1.0f);
            res = blend(corner(img, h, w, xa, yb, ntx), corner(img, h, w, xa1, yb, ntx),
                        corner(img, h, w, xa, yb1, ntx), corner(img, h, w, xa1, yb1, ntx), wa, nb);
        }
        // non-temporal: the 324-channel output is consumed by the next kernel, not re-read here;
        // keeping it out of the caches leaves the Infinity Cache to the pyramid windows, which the
        // next lookup re-reads (tools/lookup_lab.hip: -11% lookup time)
        __builtin_nontemporal_store(res, outp + (int64_t)k * P.q_count);
    }
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
        const float* img = P.lvl[lv] + ((int64_t)b * P.q_count + qq) * (int64_t)P.lsz[lv];
        P.out[i] = sample_px(img, h, w, __fadd_rn(cx, (float)(a - P.radius)),
                             __fadd_rn(cy, (float)(bb - P.radius)), P.lntx[lv]);
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

inline unsigned grid_for(int64_t n) {
    const int64_t g = (n + NT - 1) / NT;
    return (unsigned)(g < 8192 ? (g > 0 ? g : 1) : 8192);
}

inline int hip_status() {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? ECORR_OK : ECORR_EHIP - (int)e;
}

}  // namespace

template <int QB>
static void launch_staged(const LookupParams& P, int B, hipStream_t stream) {
    const dim3 grid((unsigned)((P.q_count + QB - 1) / QB), (unsigned)P.levels, (unsigned)B);
    const dim3 block(4 * QB);
    switch (P.radius) {
        case 0: hipLaunchKernelGGL((lookup_staged<0, QB>), grid, block, 0, stream, P); break;
        case 1: hipLaunchKernelGGL((lookup_staged<1, QB>), grid, block, 0, stream, P); break;
        case 2: hipLaunchKernelGGL((lookup_staged<2, QB>), grid, block, 0, stream, P); break;
        case 3: hipLaunchKernelGGL((lookup_staged<3, QB>), grid, block, 0, stream, P); break;
        default: hipLaunchKernelGGL((lookup_staged<4, QB>), grid, block, 0, stream, P); break;
    }
}

int launch_lookup(const LookupParams& P, int B, hipStream_t stream) {
    if (P.radius > 4) {
        const int64_t n = (int64_t)B * P.C * P.q_count;
        hipLaunchKernelGGL(lookup_direct, dim3(grid_for(n)), dim3(NT), 0, stream, P, B);
        return hip_status();
    }
    // dev knob for A/B timing (tools/ab_lookup.py): ECORR_LOOKUP_QB = 16 | 64
    const char* kq = getenv("ECORR_LOOKUP_QB");
    const int qb = kq ? atoi(kq) : 64;
    if (qb == 16) launch_staged<16>(P, B, stream);
    else launch_staged<64>(P, B, stream);
    return hip_status();
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

}  // namespace ecorr
