// voxel.hip -- SURVEY §8f row 3: event stream -> voxel grid on gfx950, the input side of E-RAFT.
//
// DSEC  VoxelGrid.convert (utils/dsec_utils.py:26-64): trilinear in (x, y, t) over 8 corner
//       passes, put_(accumulate=True), then nonzero mean/std normalization.
// MVSEC EventSequenceToVoxelGrid_Pytorch (utils/transformers.py:36-126): float64 events, bilinear
//       in t only, two index_add_ passes, same normalization.
//
// The reference runs single-threaded (main.py:2-5), so each cell's sum is a serial fp32 fold over
// (pass, event) in that order.  A float-atomic scatter cannot reproduce it; instead:
//   prep    per event: the reference's fp32/fp64 arithmetic up to the base cell key (the cell its
//           pass-0 corner lands in; DSEC keys live on a grid extended by one cell on the low side
//           because x0 = -1 still reaches x = 0) and the per-event factors the weights need;
//   sort    stable LSD radix sort of (key, event index) pairs (rocPRIM onesweep) -- each base
//           cell's events end up contiguous and in event order;
//   bounds  start/end of every base cell's run (one pass over the sorted keys, no atomics);
//   gather  per target cell, the runs of the base cells its 8 (DSEC) / 2 (MVSEC) passes read, in
//           pass order, each in event order: the reference's fold, bit for bit;
//   normalize  deterministic block reductions (count, double sum -> mean; double sum of squared
//           deviations -> unbiased std), then (v - mean) / std on the nonzero cells.  ATen reduces
//           in its own order, so normalized values agree within an ulp or two.
// HBM-bound with random event access; every phase is a full-chip launch.
#include <cstring>   // rocprim's texture_cache_iterator uses memset without including it

#include <rocprim/device/device_radix_sort.hpp>

#include "ecorr_device.h"
#include "ecorr_internal.h"

namespace ecorr {

namespace {

constexpr int NTV = 256;
constexpr int kRedBlocks = 1024;

// x86 truncating conversions (torch's .int() / .long() on CPU: cvttss2si / cvttsd2si, which give
// INT_MIN for NaN and out-of-range values).
__device__ __forceinline__ int x86_i32(float v) {
    return (v >= -2147483648.0f && v < 2147483648.0f) ? (int)v : (int)0x80000000u;
}
__device__ __forceinline__ long long x86_i64(double v) {
    return (v >= -9223372036854775808.0 && v < 9223372036854775808.0) ? (long long)v : (long long)(1ULL << 63);
}

struct VoxelArgs {
    // DSEC inputs
    const float *p, *t, *x, *y;
    // MVSEC input: [n][4] = t, x, y, p
    const double* ev;
    int64_t n;
    int C, H, W;
    uint32_t K;           // key range; key K = no contribution
    uint32_t *key_in, *key_out;
    int *idx_in, *idx_out;
    float *fa, *fb;       // DSEC: t_norm, value; MVSEC: left, right (0 when the right pass is masked)
    uint32_t *run_start, *run_end;
    float* voxel;
    int* bad;             // MVSEC: an index outside the grid (the reference raises)
};

__global__ __launch_bounds__(NTV) void prep_dsec(VoxelArgs A) {
    const int64_t e = blockIdx.x * (int64_t)NTV + threadIdx.x;
    if (e >= A.n) return;
    const float t0 = A.t[0], dt = __fsub_rn(A.t[A.n - 1], t0);
    // dsec_utils.py:35 (C - 1) * (t - t[0]) / (t[-1] - t[0])
    const float tn = __fdiv_rn(__fmul_rn((float)(A.C - 1), __fsub_rn(A.t[e], t0)), dt);
    const int x0 = x86_i32(A.x[e]), y0 = x86_i32(A.y[e]), ti = x86_i32(tn);
    // base cell on the grid extended by one on the low side: corners x0 .. x0+1 touch [0, W) iff
    // x0 in [-1, W-1]
    const bool in = x0 >= -1 && x0 < A.W && y0 >= -1 && y0 < A.H && ti >= -1 && ti < A.C;
    A.key_in[e] = in ? (uint32_t)(((int64_t)(ti + 1) * (A.H + 1) + (y0 + 1)) * (A.W + 1) + (x0 + 1)) : A.K;
    A.idx_in[e] = (int)e;
    A.fa[e] = tn;
    A.fb[e] = __fsub_rn(__fmul_rn(2.0f, A.p[e]), 1.0f);   // :41 value = 2*p - 1
}

__global__ __launch_bounds__(NTV) void prep_mvsec(VoxelArgs A) {
    const int64_t e = blockIdx.x * (int64_t)NTV + threadIdx.x;
    if (e >= A.n) return;
    const double first = A.ev[0];
    double dT = __dsub_rn(A.ev[4 * (A.n - 1)], first);
    if (dT == 0.0) dT = 1.0;   // transformers.py:84-85
    const double* r = A.ev + 4 * e;
    // :87 (num_bins - 1) * (t - first) / deltaT in float64
    const double ts = __ddiv_rn(__dmul_rn((double)(A.C - 1), __dsub_rn(r[0], first)), dT);
    const long long xs = x86_i64(r[1]), ys = x86_i64(r[2]);
    float pol = (float)r[3];
    if (pol == 0.0f) pol = -1.0f;   // :92
    const double tis = floor(ts);
    const float dts = (float)__dsub_rn(ts, tis);
    const bool vl = tis < (double)A.C && tis >= 0.0;        // :104-105
    const bool vr = tis + 1.0 < (double)A.C && tis >= 0.0;  // :114-115
    const int64_t HW = (int64_t)A.H * A.W, CHW = HW * A.C;
    const long long idx = xs + ys * A.W + x86_i64(tis) * HW;   // :108-110
    if ((vl && (idx < 0 || idx >= CHW)) || (vr && (idx + HW < 0 || idx + HW >= CHW))) atomicOr(A.bad, 1);
    const bool ok = vl && idx >= 0 && idx < CHW;
    A.key_in[e] = ok ? (uint32_t)idx : A.K;
    A.idx_in[e] = (int)e;
    A.fa[e] = __fmul_rn(pol, __fsub_rn(1.0f, dts));           // :96 vals_left
    A.fb[e] = vr ? __fmul_rn(pol, dts) : 0.0f;                 // :97 vals_right (+0: a no-op add)
}

// start/end of each key's run in the sorted keys (buffers zeroed: empty runs read [0, 0)).
__global__ __launch_bounds__(NTV) void run_bounds(VoxelArgs A) {
    const int64_t i = blockIdx.x * (int64_t)NTV + threadIdx.x;
    if (i >= A.n) return;
    const uint32_t k = A.key_out[i];
    if (k >= A.K) return;
    if (i == 0 || A.key_out[i - 1] != k) A.run_start[k] = (uint32_t)i;
    if (i == A.n - 1 || A.key_out[i + 1] != k) A.run_end[k] = (uint32_t)(i + 1);
}

__global__ __launch_bounds__(NTV) void gather_dsec(VoxelArgs A) {
    const int64_t HW = (int64_t)A.H * A.W;
    const int64_t cell = blockIdx.x * (int64_t)NTV + threadIdx.x;
    if (cell >= HW * A.C) return;
    const int tc = (int)(cell / HW), rem = (int)(cell - tc * HW), yc = rem / A.W, xc = rem - yc * A.W;
    const float fx = (float)xc, fy = (float)yc, ft = (float)tc;
    float acc = 0.0f;
    // dsec_utils.py:43-45 pass order: xlim outer, ylim, tlim inner
#pragma unroll
    for (int pass = 0; pass < 8; ++pass) {
        const int a = pass >> 2, b = (pass >> 1) & 1, c = pass & 1;
        const int64_t k = ((int64_t)(tc - c + 1) * (A.H + 1) + (yc - b + 1)) * (A.W + 1) + (xc - a + 1);
        const uint32_t lo = A.run_start[k], hi = A.run_end[k];
        for (uint32_t j = lo; j < hi; ++j) {
            const int e = A.idx_out[j];
            // :48 value * (1 - |xlim - x|) * (1 - |ylim - y|) * (1 - |tlim - t_norm|), left to right
            float wgt = __fmul_rn(A.fb[e], __fsub_rn(1.0f, fabsf(__fsub_rn(fx, A.x[e]))));
            wgt = __fmul_rn(wgt, __fsub_rn(1.0f, fabsf(__fsub_rn(fy, A.y[e]))));
            wgt = __fmul_rn(wgt, __fsub_rn(1.0f, fabsf(__fsub_rn(ft, A.fa[e]))));
            acc = __fadd_rn(acc, wgt);
        }
    }
    A.voxel[cell] = acc;
}

__global__ __launch_bounds__(NTV) void gather_mvsec(VoxelArgs A) {
    const int64_t HW = (int64_t)A.H * A.W;
    const int64_t cell = blockIdx.x * (int64_t)NTV + threadIdx.x;
    if (cell >= HW * A.C) return;
    float acc = 0.0f;
    for (uint32_t j = A.run_start[cell], hi = A.run_end[cell]; j < hi; ++j) acc = __fadd_rn(acc, A.fa[A.idx_out[j]]);
    if (cell >= HW)
        for (uint32_t j = A.run_start[cell - HW], hi = A.run_end[cell - HW]; j < hi; ++j)
            acc = __fadd_rn(acc, A.fb[A.idx_out[j]]);
    A.voxel[cell] = acc;
}

// ---- normalization (dsec_utils.py:55-62, transformers.py:117-124)
struct NormState {
    double mean64;
    float mean, stdv;
    long long count;
};

template <typename T>
__device__ __forceinline__ T block_sum(T v, T* sh) {
    const int tid = threadIdx.x;
    sh[tid] = v;
    __syncthreads();
    for (int s = NTV / 2; s > 0; s >>= 1) {
        if (tid < s) sh[tid] += sh[tid + s];
        __syncthreads();
    }
    const T r = sh[0];
    __syncthreads();
    return r;
}

// pass 0: count + sum of the nonzero cells; pass 1: sum of squared deviations from the mean.
// Fixed partition and tree order -> deterministic.
__global__ __launch_bounds__(NTV) void norm_partials(const float* __restrict__ g, int64_t n, int pass,
                                                     const NormState* st, double* part, long long* cpart) {
    __shared__ double shd[NTV];
    __shared__ long long shc[NTV];
    const double m = pass ? st->mean64 : 0.0;
    double s = 0.0;
    long long c = 0;
    for (int64_t i = blockIdx.x * (int64_t)NTV + threadIdx.x; i < n; i += (int64_t)gridDim.x * NTV) {
        const float v = g[i];
        if (v != 0.0f) {
            const double d = (double)v - m;
            s += pass ? d * d : (double)v;
            ++c;
        }
    }
    s = block_sum(s, shd);
    c = block_sum(c, shc);
    if (threadIdx.x == 0) {
        part[blockIdx.x] = s;
        cpart[blockIdx.x] = c;
    }
}

__global__ __launch_bounds__(NTV) void norm_finalize(int pass, const double* part, const long long* cpart,
                                                     NormState* st) {
    __shared__ double shd[NTV];
    __shared__ long long shc[NTV];
    double s = 0.0;
    long long c = 0;
    for (int i = threadIdx.x; i < kRedBlocks; i += NTV) {
        s += part[i];
        c += cpart[i];
    }
    s = block_sum(s, shd);
    c = block_sum(c, shc);
    if (threadIdx.x == 0) {
        if (pass == 0) {
            st->count = c;
            st->mean64 = c > 0 ? s / (double)c : 0.0;
            st->mean = (float)st->mean64;
        } else {
            st->stdv = c > 1 ? (float)sqrt(s / (double)(c - 1)) : __int_as_float(0x7fc00000);   // NaN for 1 cell
        }
    }
}

__global__ __launch_bounds__(NTV) void norm_apply(float* __restrict__ g, int64_t n, const NormState* st) {
    const float mean = st->mean, sd = st->stdv;
    for (int64_t i = blockIdx.x * (int64_t)NTV + threadIdx.x; i < n; i += (int64_t)gridDim.x * NTV) {
        const float v = g[i];
        if (v != 0.0f) g[i] = sd > 0.0f ? __fdiv_rn(__fsub_rn(v, mean), sd) : __fsub_rn(v, mean);
    }
}

inline unsigned blocks_for(int64_t n) { return (unsigned)((n + NTV - 1) / NTV); }

inline size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

// Workspace carve-up (every piece 256-byte aligned).
struct VoxelWs {
    size_t key_in, key_out, idx_in, idx_out, fa, fb, run_start, run_end, norm, part, cpart, sort_tmp, total;
    size_t sort_bytes;
};

unsigned key_bits(uint32_t K) {
    unsigned b = 1;
    while (b < 32 && ((uint64_t)1 << b) <= K) ++b;
    return b;
}

int plan(int64_t n, uint32_t K, VoxelWs* w) {
    size_t sort_bytes = 0;
    const hipError_t e = rocprim::radix_sort_pairs(nullptr, sort_bytes, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                                   (int*)nullptr, (int*)nullptr, (size_t)n, 0, key_bits(K));
    if (e != hipSuccess) return ECORR_EHIP - (int)e;
    size_t o = 0;
    auto take = [&](size_t bytes) { const size_t at = o; o += align256(bytes); return at; };
    w->key_in = take(4 * (size_t)n);
    w->key_out = take(4 * (size_t)n);
    w->idx_in = take(4 * (size_t)n);
    w->idx_out = take(4 * (size_t)n);
    w->fa = take(4 * (size_t)n);
    w->fb = take(4 * (size_t)n);
    w->run_start = take(4 * (size_t)K);
    w->run_end = take(4 * (size_t)K);
    w->norm = take(sizeof(NormState));
    w->part = take(8 * (size_t)kRedBlocks);
    w->cpart = take(8 * (size_t)kRedBlocks);
    w->sort_bytes = sort_bytes;
    w->sort_tmp = take(sort_bytes);
    w->total = o;
    return ECORR_OK;
}

inline int hip_status() {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? ECORR_OK : ECORR_EHIP - (int)e;
}

}  // namespace

uint32_t voxel_key_range(bool dsec, int C, int H, int W) {
    return dsec ? (uint32_t)((C + 1) * (H + 1) * (W + 1)) : (uint32_t)(C * H * W);
}

int voxel_workspace_bytes(bool dsec, int64_t n, int C, int H, int W, int64_t* bytes) {
    VoxelWs w;
    const int st = plan(n, voxel_key_range(dsec, C, H, W), &w);
    if (st == ECORR_OK) *bytes = (int64_t)w.total;
    return st;
}

int launch_voxel(bool dsec, const float* p, const float* t, const float* x, const float* y, const double* ev,
                 int64_t n, int C, int H, int W, int normalize, float* voxel, int* bad, void* workspace,
                 hipStream_t stream) {
    VoxelArgs A{};
    A.p = p; A.t = t; A.x = x; A.y = y; A.ev = ev;
    A.n = n; A.C = C; A.H = H; A.W = W;
    A.K = voxel_key_range(dsec, C, H, W);
    VoxelWs w;
    int st = plan(n, A.K, &w);
    if (st != ECORR_OK) return st;
    char* base = (char*)workspace;
    A.key_in = (uint32_t*)(base + w.key_in);
    A.key_out = (uint32_t*)(base + w.key_out);
    A.idx_in = (int*)(base + w.idx_in);
    A.idx_out = (int*)(base + w.idx_out);
    A.fa = (float*)(base + w.fa);
    A.fb = (float*)(base + w.fb);
    A.run_start = (uint32_t*)(base + w.run_start);
    A.run_end = (uint32_t*)(base + w.run_end);
    A.voxel = voxel;
    A.bad = bad;
    NormState* ns = (NormState*)(base + w.norm);

    if (dsec) hipLaunchKernelGGL(prep_dsec, dim3(blocks_for(n)), dim3(NTV), 0, stream, A);
    else hipLaunchKernelGGL(prep_mvsec, dim3(blocks_for(n)), dim3(NTV), 0, stream, A);
    if ((st = hip_status()) != ECORR_OK) return st;
    size_t sort_bytes = w.sort_bytes;
    hipError_t e = rocprim::radix_sort_pairs(base + w.sort_tmp, sort_bytes, A.key_in, A.key_out, A.idx_in, A.idx_out,
                                             (size_t)n, 0, key_bits(A.K), stream);
    if (e != hipSuccess) return ECORR_EHIP - (int)e;
    e = hipMemsetAsync(A.run_start, 0, 4 * (size_t)A.K, stream);
    if (e == hipSuccess) e = hipMemsetAsync(A.run_end, 0, 4 * (size_t)A.K, stream);
    if (e != hipSuccess) return ECORR_EHIP - (int)e;
    hipLaunchKernelGGL(run_bounds, dim3(blocks_for(n)), dim3(NTV), 0, stream, A);
    const int64_t cells = (int64_t)C * H * W;
    if (dsec) hipLaunchKernelGGL(gather_dsec, dim3(blocks_for(cells)), dim3(NTV), 0, stream, A);
    else hipLaunchKernelGGL(gather_mvsec, dim3(blocks_for(cells)), dim3(NTV), 0, stream, A);
    if ((st = hip_status()) != ECORR_OK) return st;
    if (normalize) {
        double* part = (double*)(base + w.part);
        long long* cpart = (long long*)(base + w.cpart);
        for (int pass = 0; pass < 2; ++pass) {
            hipLaunchKernelGGL(norm_partials, dim3(kRedBlocks), dim3(NTV), 0, stream, voxel, cells, pass, ns, part,
                               cpart);
            hipLaunchKernelGGL(norm_finalize, dim3(1), dim3(NTV), 0, stream, pass, part, cpart, ns);
        }
        hipLaunchKernelGGL(norm_apply, dim3(kRedBlocks), dim3(NTV), 0, stream, voxel, cells, ns);
    }
    return hip_status();
}

}  // namespace ecorr
