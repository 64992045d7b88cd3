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
//   bucket  counting sort by key: per event its arrival rank in its key (one returning integer
//           atomic, in prep), exclusive scan of the counts (reduce -> scan of the tile sums ->
//           tile scans, 16-byte loads and stores), each event and its weight factors (one float4)
//           dropped at run start + rank -- no second atomic pass (round 6: the two random-atomic
//           passes were 96 of the 282 us per DSEC window, profiles/r06_lab);
//   order   per key with two or more events, its run insertion-sorted by event index (runs are
//           short and the atomics hand out ranks nearly in event order, so this is ~linear) and
//           the run's weight factors re-gathered into that order;
//   gather  per target cell, the runs of the base cells its 8 (DSEC) / 2 (MVSEC) passes read, in
//           pass order, each in event order: the reference's fold, bit for bit.  Neighbouring
//           cells read neighbouring runs, so the payload reads are near-contiguous.  With
//           normalize, each block also folds its nonzero cells into (count, mean, M2) (Chan's
//           pairwise combination, double, fixed tree order);
//   finalize one block combines the block partials in a fixed order -> mean, unbiased std;
//   apply   (v - mean) / std on the nonzero cells.  ATen reduces in its own order, so normalized
//           values agree within an ulp or two.
// Memory-bound with random event access; every phase is a full-chip launch.
#include <algorithm>

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
    uint32_t* key;        // per event: base-cell key (K = none)
    uint32_t* rank;       // per event: its arrival rank among its key's events (atomic order)
    uint32_t* cnt;        // per key: event count (K + 1 entries, zeroed; cnt[K] stays 0)
    uint32_t* off;        // per key: exclusive offset = run start; off[K] = the runs' total
    int* slot;            // run order: event index
    float *fa, *fb;       // DSEC: t_norm, value; MVSEC: left, right (0 when the right pass is masked)
    float4* payload;      // sorted order: DSEC (x, y, t_norm, value); MVSEC (left, right, -, -)
    double* part;         // per gather block: count, mean, M2 of its nonzero cells
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
    const uint32_t k = in ? (uint32_t)(((int64_t)(ti + 1) * (A.H + 1) + (y0 + 1)) * (A.W + 1) + (x0 + 1)) : A.K;
    A.key[e] = k;
    if (in) A.rank[e] = atomicAdd(&A.cnt[k], 1u);
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
    A.key[e] = ok ? (uint32_t)idx : A.K;
    if (ok) A.rank[e] = atomicAdd(&A.cnt[idx], 1u);
    A.fa[e] = __fmul_rn(pol, __fsub_rn(1.0f, dts));           // :96 vals_left
    A.fb[e] = vr ? __fmul_rn(pol, dts) : 0.0f;                 // :97 vals_right (+0: a no-op add)
}

template <bool DSEC>
__device__ __forceinline__ float4 payload_of(const VoxelArgs& A, int64_t e) {
    return DSEC ? make_float4(A.x[e], A.y[e], A.fa[e], A.fb[e]) : make_float4(A.fa[e], A.fb[e], 0.0f, 0.0f);
}

// Drop every event and its weight factors at its run's start + its rank (event-parallel: the
// event fields are read coalesced, no atomics).
template <bool DSEC>
__global__ __launch_bounds__(NTV) void fill_runs(VoxelArgs A) {
    const int64_t e = blockIdx.x * (int64_t)NTV + threadIdx.x;
    if (e >= A.n) return;
    const uint32_t k = A.key[e];
    if (k >= A.K) return;
    const uint32_t i = A.off[k] + A.rank[e];
    A.slot[i] = (int)e;
    A.payload[i] = payload_of<DSEC>(A, e);
}

__device__ __forceinline__ uint2 run_of(const VoxelArgs& A, int64_t k) {
    return make_uint2(A.off[k], A.off[k + 1]);
}

// Per run of two or more events (found by its rank-1 event: event-parallel, 1M threads at DSEC
// instead of one per key, 4.9M): order it by event index, then re-gather its weight factors into
// that order (a one-event run is already in place).
template <bool DSEC>
__global__ __launch_bounds__(NTV) void order_runs(VoxelArgs A) {
    const int64_t e = blockIdx.x * (int64_t)NTV + threadIdx.x;
    if (e >= A.n) return;
    const uint32_t k = A.key[e];
    if (k >= A.K || A.rank[e] != 1u) return;
    const uint2 r = run_of(A, k);
    bool moved = false;
    for (uint32_t i = r.x + 1; i < r.y; ++i) {
        const int v = A.slot[i];
        uint32_t j = i;
        while (j > r.x && A.slot[j - 1] > v) { A.slot[j] = A.slot[j - 1]; --j; }
        A.slot[j] = v;
        moved |= j != i;
    }
    if (moved)
        for (uint32_t i = r.x; i < r.y; ++i) A.payload[i] = payload_of<DSEC>(A, A.slot[i]);
}

// (count, mean, M2) of a set of values; Chan et al.'s pairwise combination, in double.
struct Moments {
    double n, mean, m2;
};
__device__ __forceinline__ Moments combine(Moments a, Moments b) {
    const double n = a.n + b.n;
    if (n == 0.0) return a;
    const double d = b.mean - a.mean;
    return {n, a.mean + d * (b.n / n), a.m2 + b.m2 + d * d * (a.n * b.n / n)};
}

// Fixed-order tree over the block (deterministic); result valid in thread 0.
__device__ __forceinline__ Moments block_moments(Moments m, double* sh) {
    const int tid = threadIdx.x;
    sh[3 * tid] = m.n; sh[3 * tid + 1] = m.mean; sh[3 * tid + 2] = m.m2;
    __syncthreads();
    for (int s = NTV / 2; s > 0; s >>= 1) {
        if (tid < s) {
            const Moments r = combine({sh[3 * tid], sh[3 * tid + 1], sh[3 * tid + 2]},
                                      {sh[3 * (tid + s)], sh[3 * (tid + s) + 1], sh[3 * (tid + s) + 2]});
            sh[3 * tid] = r.n; sh[3 * tid + 1] = r.mean; sh[3 * tid + 2] = r.m2;
        }
        __syncthreads();
    }
    return {sh[0], sh[1], sh[2]};
}

// Block = a contiguous range of grid rows (tc, yc); its threads walk the range's cells in order,
// 256 apart, with (row, xc) stepped incrementally (no per-cell integer division; every lane busy
// whatever W is); the keys of a cell's 8 passes are the row's base key + xc minus constants
// (32-bit: the key range is < 2^32), and lanes on consecutive xc read consecutive run bounds.
template <bool DSEC>
__global__ __launch_bounds__(NTV) void gather(VoxelArgs A, int normalize) {
    __shared__ double sh[3 * NTV];
    const int rows = A.C * A.H;
    const int per = (rows + gridDim.x - 1) / gridDim.x;
    const int r0 = blockIdx.x * per, r1 = min(rows, r0 + per);
    // this thread's nonzero cells as plain fp64 sums (no division per cell), turned into (count,
    // mean, M2) once before the block's fixed-order Chan tree
    double cn = 0.0, cs = 0.0, css = 0.0;
    const uint32_t dB = (uint32_t)A.W + 1, dC = ((uint32_t)A.H + 1) * dB;
    int r = r0 + (int)threadIdx.x / A.W, xc = (int)threadIdx.x % A.W;
    int tc = r / A.H, yc = r - tc * A.H;
    for (; r < r1;) {
        {
            float acc = 0.0f;
            if (DSEC) {
                const float fx = (float)xc, fy = (float)yc, ft = (float)tc;
                // the pass-0 corner's base key (tc, yc, xc) on the extended grid
                const uint32_t k0 = ((uint32_t)(tc + 1) * ((uint32_t)A.H + 1) + (uint32_t)(yc + 1)) * dB + (uint32_t)xc + 1;
                // dsec_utils.py:43-45 pass order: xlim outer, ylim, tlim inner; base key of pass
                // (a, b, c) = k0 - a - b dB - c dC.  All run bounds first (a = 0 and a = 1 are
                // adjacent keys: three consecutive offsets per (b, c)), then the folds in order.
                uint32_t o3[4][3];
#pragma unroll
                for (int bc = 0; bc < 4; ++bc) {
                    const uint32_t k1 = k0 - 1u - (uint32_t)(bc >> 1) * dB - (uint32_t)(bc & 1) * dC;   // a = 1
#pragma unroll
                    for (int i = 0; i < 3; ++i) o3[bc][i] = A.off[k1 + i];
                }
#pragma unroll
                for (int pass = 0; pass < 8; ++pass) {
                    const int aa = pass >> 2, bc = pass & 3;
                    for (uint32_t j = o3[bc][1 - aa]; j < o3[bc][2 - aa]; ++j) {
                        const float4 ev = A.payload[j];
                        // :48 value * (1 - |xlim - x|) * (1 - |ylim - y|) * (1 - |tlim - t_norm|), left to right
                        float wgt = __fmul_rn(ev.w, __fsub_rn(1.0f, fabsf(__fsub_rn(fx, ev.x))));
                        wgt = __fmul_rn(wgt, __fsub_rn(1.0f, fabsf(__fsub_rn(fy, ev.y))));
                        wgt = __fmul_rn(wgt, __fsub_rn(1.0f, fabsf(__fsub_rn(ft, ev.z))));
                        acc = __fadd_rn(acc, wgt);
                    }
                }
            } else {
                // transformers.py:103-113: all left contributions, then all right ones (+W*H)
                const int64_t cell = (int64_t)r * A.W + xc, HW = (int64_t)A.H * A.W;
                const uint2 rl = run_of(A, cell);
                const uint2 rr = tc > 0 ? run_of(A, cell - HW) : make_uint2(0u, 0u);
                for (uint32_t j = rl.x; j < rl.y; ++j) acc = __fadd_rn(acc, A.payload[j].x);
                for (uint32_t j = rr.x; j < rr.y; ++j) acc = __fadd_rn(acc, A.payload[j].y);
            }
            A.voxel[(int64_t)r * A.W + xc] = acc;
            if (normalize && acc != 0.0f) {
                const double v = (double)acc;
                cn += 1.0;
                cs += v;
                css = fma(v, v, css);
            }
        }
        xc += NTV;   // next cell of this thread: 256 further in row-major order
        while (xc >= A.W) {
            xc -= A.W;
            ++r;
            if (++yc == A.H) { yc = 0; ++tc; }
        }
    }
    if (normalize) {   // uniform over the grid
        Moments mom{0.0, 0.0, 0.0};
        if (cn > 0.0) {
            const double mean = cs / cn;
            mom = {cn, mean, fmax(css - cs * mean, 0.0)};
        }
        const Moments m = block_moments(mom, sh);
        if (threadIdx.x == 0) {
            A.part[3 * blockIdx.x] = m.n;
            A.part[3 * blockIdx.x + 1] = m.mean;
            A.part[3 * blockIdx.x + 2] = m.m2;
        }
    }
}

// ---- normalization (dsec_utils.py:55-62, transformers.py:117-124)
struct NormState {
    float mean, stdv;
    int any;
};

// One block: thread t folds partials t, t + NTV, ... in order, then the fixed tree.
// The moments of nparts partials (fixed order) -> the normalization state; block-wide, NTV threads.
// Thread i combines partials i, i + NTV, ... in order, 8 loads in flight per batch.
__device__ __forceinline__ void finalize_moments(const double* part, int nparts, double* sh, NormState* st) {
    Moments m{0.0, 0.0, 0.0};
    for (int i0 = threadIdx.x; i0 < nparts; i0 += 8 * NTV) {
        double v[8][3];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int i = i0 + j * NTV;
#pragma unroll
            for (int c = 0; c < 3; ++c) v[j][c] = i < nparts ? part[3 * i + c] : 0.0;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if (i0 + j * NTV < nparts) m = combine(m, {v[j][0], v[j][1], v[j][2]});
    }
    m = block_moments(m, sh);
    if (threadIdx.x == 0) {
        st->any = m.n > 0.0;
        st->mean = (float)m.mean;
        // unbiased std; one nonzero cell gives NaN like torch.std, and then v - mean
        st->stdv = m.n > 1.0 ? (float)sqrt(m.m2 / (m.n - 1.0)) : __int_as_float(0x7fc00000);
    }
}

__global__ __launch_bounds__(NTV) void norm_finalize(const double* part, int nparts, NormState* st) {
    __shared__ double sh[3 * NTV];
    finalize_moments(part, nparts, sh, st);
}

__device__ __forceinline__ float norm_one(float v, float mean, float sd) {
    return v != 0.0f ? (sd > 0.0f ? __fdiv_rn(__fsub_rn(v, mean), sd) : __fsub_rn(v, mean)) : v;
}

// (v - mean) / std on the nonzero cells; 16-byte accesses (the grid is 16-byte aligned: checked by
// launch_norm_apply), the n % 4 tail by thread 0 of block 0
__global__ __launch_bounds__(NTV) void norm_apply(float* __restrict__ g, int64_t n, const NormState* st) {
    if (!st->any) return;
    const float mean = st->mean, sd = st->stdv;
    float4* g4 = reinterpret_cast<float4*>(g);
    const int64_t n4 = n / 4;
    for (int64_t i = blockIdx.x * (int64_t)NTV + threadIdx.x; i < n4; i += (int64_t)gridDim.x * NTV) {
        float4 v = g4[i];
        if (v.x != 0.0f || v.y != 0.0f || v.z != 0.0f || v.w != 0.0f) {
            v.x = norm_one(v.x, mean, sd);
            v.y = norm_one(v.y, mean, sd);
            v.z = norm_one(v.z, mean, sd);
            v.w = norm_one(v.w, mean, sd);
            g4[i] = v;
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0)
        for (int64_t i = 4 * n4; i < n; ++i) g[i] = norm_one(g[i], mean, sd);
}

__global__ __launch_bounds__(NTV) void norm_apply_scalar(float* __restrict__ g, int64_t n, const NormState* st) {
    if (!st->any) return;
    const float mean = st->mean, sd = st->stdv;
    for (int64_t i = blockIdx.x * (int64_t)NTV + threadIdx.x; i < n; i += (int64_t)gridDim.x * NTV) {
        const float v = g[i];
        if (v != 0.0f) g[i] = norm_one(v, mean, sd);
    }
}

void launch_norm_apply(float* g, int64_t n, const NormState* st, hipStream_t stream) {
    if (((uintptr_t)g & 15) == 0)
        hipLaunchKernelGGL(norm_apply, dim3(kRedBlocks), dim3(NTV), 0, stream, g, n, st);
    else
        hipLaunchKernelGGL(norm_apply_scalar, dim3(kRedBlocks), dim3(NTV), 0, stream, g, n, st);
}

// Exclusive uint32 scan of the per-key counts (wrapping adds, like any uint32 scan): SCAN_T
// elements per block tile; phase 1 writes each tile's sum, phase 2 (one block) scans the sums,
// phase 3 scans each tile from its offset.  Integer arithmetic: exact in any order.
constexpr int SCAN_PER = 16, SCAN_T = NTV * SCAN_PER;

static_assert(NTV % 64 == 0 && NTV <= 1024, "block_exclusive_scan: whole 64-lane waves, sh[NTV / 64]");
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t* sh, uint32_t& total) {
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d);
        if (lane >= d) x += y;
    }
    if (lane == 63) sh[wv] = x;
    __syncthreads();
    uint32_t pre = 0, sum = 0;
#pragma unroll
    for (int w = 0; w < NTV / 64; ++w) {
        if (w < wv) pre += sh[w];
        sum += sh[w];
    }
    total = sum;
    __syncthreads();
    return pre + x - v;
}

// A thread's SCAN_PER consecutive counts: four 16-byte loads (the arrays are 256-byte aligned), the
// range's tail element by element.
__device__ __forceinline__ void load16(const uint32_t* __restrict__ in, int64_t base, int64_t K, uint32_t (&v)[SCAN_PER]) {
    if (base + SCAN_PER <= K) {
#pragma unroll
        for (int q = 0; q < SCAN_PER / 4; ++q) {
            const uint4 u = reinterpret_cast<const uint4*>(in + base)[q];
            v[4 * q] = u.x; v[4 * q + 1] = u.y; v[4 * q + 2] = u.z; v[4 * q + 3] = u.w;
        }
    } else {
#pragma unroll
        for (int k = 0; k < SCAN_PER; ++k) v[k] = base + k < K ? in[base + k] : 0u;
    }
}

__global__ __launch_bounds__(NTV) void scan_reduce(const uint32_t* __restrict__ in, int64_t K, uint32_t* __restrict__ sums) {
    __shared__ uint32_t sh[NTV / 64];
    const int64_t base = (int64_t)blockIdx.x * SCAN_T + threadIdx.x * SCAN_PER;
    uint32_t w[SCAN_PER], v = 0;
    load16(in, base, K, w);
#pragma unroll
    for (int k = 0; k < SCAN_PER; ++k) v += w[k];
    uint32_t total;
    block_exclusive_scan(v, sh, total);
    if (threadIdx.x == 0) sums[blockIdx.x] = total;
}

__global__ __launch_bounds__(NTV) void scan_sums(uint32_t* __restrict__ sums, int nb) {
    __shared__ uint32_t sh[NTV / 64];
    uint32_t carry = 0;
    for (int c = 0; c < nb; c += NTV) {
        const int i = c + threadIdx.x;
        const uint32_t v = i < nb ? sums[i] : 0;
        uint32_t total;
        const uint32_t ex = block_exclusive_scan(v, sh, total);
        if (i < nb) sums[i] = carry + ex;
        carry += total;
    }
}

__global__ __launch_bounds__(NTV) void scan_apply(const uint32_t* __restrict__ in, int64_t K, const uint32_t* __restrict__ sums,
                                                  uint32_t* __restrict__ out) {
    __shared__ uint32_t sh[NTV / 64];
    const int64_t base = (int64_t)blockIdx.x * SCAN_T + threadIdx.x * SCAN_PER;
    uint32_t v[SCAN_PER], s = 0;
    load16(in, base, K, v);
#pragma unroll
    for (int k = 0; k < SCAN_PER; ++k) s += v[k];
    uint32_t total;
    uint32_t run = sums[blockIdx.x] + block_exclusive_scan(s, sh, total);
    uint32_t o[SCAN_PER];
#pragma unroll
    for (int k = 0; k < SCAN_PER; ++k) {
        o[k] = run;
        run += v[k];
    }
    if (base + SCAN_PER <= K) {
#pragma unroll
        for (int q = 0; q < SCAN_PER / 4; ++q)
            reinterpret_cast<uint4*>(out + base)[q] = make_uint4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
    } else {
#pragma unroll
        for (int k = 0; k < SCAN_PER; ++k)
            if (base + k < K) out[base + k] = o[k];
    }
}

inline unsigned blocks_for(int64_t n) { return (unsigned)((n + NTV - 1) / NTV); }

// ============================================================================================
// DSEC, tiled (round 6).  The key-range pipeline above spends most of its time on the key range
// itself (a 4.9 M-entry count array zeroed, scanned and indexed per cell) and on random global
// atomics.  Here the events are bucketed by cell tile: tile (ty, tx) covers grid cells
// [4 ty, 4 ty + 4) x [16 tx, 16 tx + 16), and its window -- the base cells its cells read, all time
// bins -- is extended base cells [4 ty, 4 ty + 4] x [16 tx, 16 tx + 16] (the +1 halo: the first row
// and column of the next tiles).  An event lands in every window holding its base cell (1 to 4 of
// them, 1.33 on average), so a tile's bucket is exactly its window, contiguous in HBM; one
// 256-thread workgroup per tile sorts it in LDS into runs (time bin, base cell), each run by event
// index, and folds its 64 cells from there, 4 time bins at a time:
//   vb_count    per block of VB_EPB events: the prep arithmetic, the windows, a 16-bit slot within
//               (window, block) per copy from an LDS atomic (8 bytes per event: nothing else is
//               kept), the block's counts -> M[block][window];
//   vb_colscan  per window, its counts over the blocks -> prefixes (in place) and its total;
//   vb_starts   one block: exclusive scan of the totals -> window starts S;
//   vb_scatter  the prep again from the event fields (cheaper than storing and re-reading it), each
//               copy's (x, y, t_norm, value) and event index to S[w] + M[blk][w] + slot;
//   vb_gather   per tile: runs counted (LDS atomics), scanned, placed, ranked by event index; then
//               each cell folded in pass order -- the reference's serial fold, bit for bit.  A window
//               holding more than VB_CAP events (a hot pixel, a dense stream) is read where it lies
//               in HBM, its run order kept in a global arena (the run table stays in LDS).
// ============================================================================================
constexpr int VB_TY = 4, VB_TX = 16;              // cell tile
constexpr int VB_NT = 256;                        // gather threads: 4 waves x 64 cells
constexpr int VB_NW = VB_NT / (VB_TY * VB_TX);    // time-bin groups of the fold
constexpr int VB_WX = VB_TX + 1, VB_WK = (VB_TY + 1) * VB_WX;   // base cells of a window, per bin
constexpr int VB_CAP = 512;                       // window events in LDS
constexpr int VB_MAXRUN = 2048;                   // (C + 1) * VB_WK runs per window (C <= 23)
constexpr int VB_CNT = 1024, VB_EPB = 8 * VB_CNT; // count blocks: threads, events per block
constexpr int VB_MAXNB = 12288;                   // windows (LDS counts of vb_count)
static_assert(VB_NT == NTV && VB_NW * VB_TY * VB_TX == VB_NT, "vb_gather: 4 waves of one tile each");
static_assert(VB_CAP == 2 * VB_NT, "vb_gather: two rounds of the in-place reorder");

// a window's copy of an event: (x, y, t_norm, value) and the event index, one 32-byte sector
struct alignas(32) VCopy {
    float4 ev;
    int idx, pad[3];
};

struct VTileArgs {
    const float *p, *t, *x, *y;
    int64_t n;
    int C, H, W;
    int gy, gx, nb, nblk;   // tile grid, windows (gy * gx), count blocks
    uint2* slot;       // per event: 16-bit slots of its copies (own, left, up, up-left) within
                       // (window, block): < VB_EPB; everything else vb_scatter recomputes
    uint32_t* M;       // [nblk][nb]: counts, then their prefixes over the blocks
    uint32_t* tot;     // [nb + 1]: window totals (tot[nb] = 0)
    uint32_t* S;       // [nb + 1]: window starts
    VCopy* pay;        // windowed copies: at most 4n
    double* part;
    float* voxel;
    uint32_t *aord, *aords;   // run order of windows past VB_CAP, at their copies' positions
    NormState* norm;
};

// The windows of extended base cell (ey, ex): copy q = (dy, dx) bits, dy/dx = take the tile above /
// left too (the cell is that tile's halo row / column).  -1 where the copy does not exist.
__device__ __forceinline__ int vt_window(const VTileArgs& A, int ey, int ex, int q) {
    const int dy = q >> 1, dx = q & 1;
    if ((dy && (ey % VB_TY != 0)) || (dx && (ex % VB_TX != 0))) return -1;
    const int ty = ey / VB_TY - dy, tx = ex / VB_TX - dx;
    return (ty >= 0 && ty < A.gy && tx >= 0 && tx < A.gx) ? ty * A.gx + tx : -1;
}

// dsec_utils.py:35-41 as prep_dsec: t_norm, value and the extended base cell of event e; false when
// the event lies in no window (no pass of it lands on the grid)
__device__ __forceinline__ bool vt_prep(const VTileArgs& A, int64_t e, float t0, float dt, float& tn, float& val,
                                        int& ey, int& ex) {
    tn = __fdiv_rn(__fmul_rn((float)(A.C - 1), __fsub_rn(A.t[e], t0)), dt);
    val = __fsub_rn(__fmul_rn(2.0f, A.p[e]), 1.0f);
    const int x0 = x86_i32(A.x[e]), y0 = x86_i32(A.y[e]), ti = x86_i32(tn);
    ey = y0 + 1;
    ex = x0 + 1;
    return x0 >= -1 && x0 < A.W && y0 >= -1 && y0 < A.H && ti >= -1 && ti < A.C;
}
static_assert(VB_EPB <= 65536, "16-bit slots within (window, block)");

__global__ __launch_bounds__(VB_CNT) void vb_count(VTileArgs A) {
    __shared__ uint32_t hist[VB_MAXNB];
    const int tid = threadIdx.x, blk = blockIdx.x;
    for (int i = tid; i < A.nb; i += VB_CNT) hist[i] = 0;
    __syncthreads();
    const float t0 = A.t[0], dt = __fsub_rn(A.t[A.n - 1], t0);
#pragma unroll 2
    for (int k = 0; k < VB_EPB / VB_CNT; ++k) {
        const int64_t e = (int64_t)blk * VB_EPB + k * VB_CNT + tid;
        if (e >= A.n) break;
        float tn, val;
        int ey, ex;
        if (vt_prep(A, e, t0, dt, tn, val, ey, ex)) {
            uint32_t sl[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int w = vt_window(A, ey, ex, q);
                sl[q] = w >= 0 ? atomicAdd(&hist[w], 1u) : 0u;
            }
            A.slot[e] = make_uint2(sl[0] | sl[1] << 16, sl[2] | sl[3] << 16);
        }
    }
    __syncthreads();
    uint32_t* row = A.M + (int64_t)blk * A.nb;
    for (int i = tid; i < A.nb; i += VB_CNT) row[i] = hist[i];
}

// per window: its counts over the blocks -> exclusive prefixes (16 loads in flight per batch) and
// its total (a last-block scan of the totals fused in here was slower: 20 vs 8 + 3 x 5 us)
__global__ __launch_bounds__(NTV) void vb_colscan(VTileArgs A) {
    const int b = blockIdx.x * NTV + threadIdx.x;
    if (b > A.nb) return;
    if (b == A.nb) { A.tot[b] = 0; return; }
    uint32_t* __restrict__ col = A.M + b;
    uint32_t run = 0;
    for (int k0 = 0; k0 < A.nblk; k0 += 16) {
        uint32_t c[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) c[j] = k0 + j < A.nblk ? col[(int64_t)(k0 + j) * A.nb] : 0u;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            if (k0 + j < A.nblk) col[(int64_t)(k0 + j) * A.nb] = run;
            run += c[j];
        }
    }
    A.tot[b] = run;
}

// window starts: exclusive scan of the nb + 1 totals (tot[nb] = 0); one block, each thread a
// contiguous chunk (8 loads in flight per batch)
__global__ __launch_bounds__(NTV) void vb_starts(VTileArgs A) {
    __shared__ uint32_t sh[NTV / kWave];
    const int K = A.nb + 1, per = (K + NTV - 1) / NTV, k0 = threadIdx.x * per, k1 = min(K, k0 + per);
    uint32_t s = 0;
    for (int k = k0; k < k1; k += 8) {
        uint32_t v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = k + j < k1 ? A.tot[k + j] : 0u;
#pragma unroll
        for (int j = 0; j < 8; ++j) s += v[j];
    }
    uint32_t total;
    uint32_t run = block_exclusive_scan(s, sh, total);
    for (int k = k0; k < k1; ++k) {
        A.S[k] = run;
        run += A.tot[k];
    }
}

__global__ __launch_bounds__(NTV) void vb_scatter(VTileArgs A) {
    const int64_t e = blockIdx.x * (int64_t)NTV + threadIdx.x;
    if (e >= A.n) return;
    const float t0 = A.t[0], dt = __fsub_rn(A.t[A.n - 1], t0);
    float tn, val;
    int ey, ex;
    if (!vt_prep(A, e, t0, dt, tn, val, ey, ex)) return;   // the same arithmetic as vb_count's
    const uint2 s = A.slot[e];
    const uint32_t sl[4] = {s.x & 0xffff, s.x >> 16, s.y & 0xffff, s.y >> 16};
    const float4 v = make_float4(A.x[e], A.y[e], tn, val);
    const uint32_t* Mrow = A.M + (e / VB_EPB) * A.nb;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int w = vt_window(A, ey, ex, q);
        if (w < 0) continue;
        const uint32_t i = A.S[w] + Mrow[w] + sl[q];
        A.pay[i].ev = v;
        A.pay[i].idx = (int)e;
    }
}

struct VWin {
    float4 ev[VB_CAP];             // the window's copies (8 KB; the moments' scratch at the end)
    int idx[VB_CAP];
    unsigned short ord[VB_CAP];    // placement order (per run, arbitrary within it)
    unsigned short ords[VB_CAP];   // per run in event-index order
    int off[VB_MAXRUN + 1];        // run starts, then (after placement) run ends
    int wsum[VB_NT / kWave];
};
static_assert(sizeof(float4) * VB_CAP >= 3 * sizeof(double) * VB_NT, "moments scratch");

// :48 value * (1 - |xlim - x|) * (1 - |ylim - y|) * (1 - |tlim - t_norm|), left to right
__device__ __forceinline__ float vt_term(float4 ev, float fx, float fy, float ft) {
    float wgt = __fmul_rn(ev.w, __fsub_rn(1.0f, fabsf(__fsub_rn(fx, ev.x))));
    wgt = __fmul_rn(wgt, __fsub_rn(1.0f, fabsf(__fsub_rn(fy, ev.y))));
    return __fmul_rn(wgt, __fsub_rn(1.0f, fabsf(__fsub_rn(ft, ev.z))));
}

__global__ __launch_bounds__(VB_NT) void vb_gather(VTileArgs A, int normalize) {
    __shared__ VWin L;
    const int tid = threadIdx.x, lane = tid % kWave, wv = tid / kWave;
    const int tile = blockIdx.x, cy = tile / A.gx, cx = tile % A.gx;
    const int ey0 = cy * VB_TY, ex0 = cx * VB_TX;   // window origin on the extended base-cell grid
    const int nrun = (A.C + 1) * VB_WK;
    const uint32_t s0 = A.S[tile];
    const int n = (int)(A.S[tile + 1] - s0);
    const bool ar = n > VB_CAP;   // uniform: the window is read where it lies
    const VCopy* gc = A.pay + s0;
    uint32_t* aord = A.aord + s0;
    uint32_t* aords = A.aords + s0;
    // run of a copy: (bin ti + 1, window row, window column)
    auto run_of = [&](const float4& ev) {
        return ((x86_i32(ev.z) + 1) * (VB_TY + 1) + x86_i32(ev.y) + 1 - ey0) * VB_WX + x86_i32(ev.x) + 1 - ex0;
    };
    for (int k = tid; k <= nrun; k += VB_NT) L.off[k] = 0;
    __syncthreads();
    for (int j = tid; j < n; j += VB_NT) {   // count
        const float4 ev = gc[j].ev;
        if (!ar) {
            L.ev[j] = ev;
            L.idx[j] = gc[j].idx;
        }
        atomicAdd(&L.off[run_of(ev)], 1);
    }
    __syncthreads();
    {   // exclusive scan of the nrun counts: per thread a contiguous chunk, waves, then the block
        constexpr int PER = (VB_MAXRUN + VB_NT - 1) / VB_NT;
        const int k0 = tid * PER;
        int v[PER], s = 0;
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            v[i] = k0 + i < nrun ? L.off[k0 + i] : 0;
            s += v[i];
        }
        int inc = s;
#pragma unroll
        for (int d = 1; d < kWave; d <<= 1) {
            const int u = __shfl_up(inc, d, kWave);
            if (lane >= d) inc += u;
        }
        if (lane == kWave - 1) L.wsum[wv] = inc;
        __syncthreads();
        int base = inc - s;
        for (int w = 0; w < wv; ++w) base += L.wsum[w];
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            if (k0 + i < nrun) L.off[k0 + i] = base;
            base += v[i];
        }
    }
    __syncthreads();
    for (int j = tid; j < n; j += VB_NT) {   // place: off[r] walks from its run's start to its end
        const int r = run_of(ar ? gc[j].ev : L.ev[j]);
        const int pos = atomicAdd(&L.off[r], 1);
        if (ar) aord[pos] = (uint32_t)j;
        else L.ord[pos] = (unsigned short)j;
    }
    __syncthreads();
    for (int j = tid; j < n; j += VB_NT) {   // rank within the run by event index
        const int r = run_of(ar ? gc[j].ev : L.ev[j]);
        const int lo = r > 0 ? L.off[r - 1] : 0, hi = L.off[r];
        int rk = 0;
        if (ar) {
            const int me = gc[j].idx;
            for (int i = lo; i < hi; ++i) rk += gc[aord[i]].idx < me;
            aords[lo + rk] = (uint32_t)j;
        } else {
            const int me = L.idx[j];
            for (int i = lo; i < hi; ++i) rk += L.idx[L.ord[i]] < me;
            L.ords[lo + rk] = (unsigned short)j;
        }
    }
    __syncthreads();

    if (!ar) {   // the window's events into run order in place: the fold reads L.ev[i] directly
        const int j0 = tid, j1 = tid + VB_NT;   // VB_CAP = 2 VB_NT
        const float4 e0 = L.ev[j0 < n ? L.ords[j0] : 0], e1 = L.ev[j1 < n ? L.ords[j1] : 0];
        __syncthreads();
        if (j0 < n) L.ev[j0] = e0;
        if (j1 < n) L.ev[j1] = e1;
        __syncthreads();
    }

    // wave wv folds time bins [tc0, tc1) of its lane's cell
    const int ly = lane / VB_TX, lx = lane % VB_TX;
    const int yc = ey0 + ly, xc = ex0 + lx;
    const int nper = (A.C + VB_NW - 1) / VB_NW, tc0 = wv * nper, tc1 = min(A.C, tc0 + nper);
    double cn = 0.0, cs = 0.0, css = 0.0;
    if (yc < A.H && xc < A.W && tc0 < tc1) {
        const float fx = (float)xc, fy = (float)yc;
        // run bounds of bin e around this cell: row ly + 1 (u) and row ly (d), columns lx and lx + 1:
        // column lx = [x0, x1), column lx + 1 = [x1, x2)
        struct Bounds { int u0, u1, u2, d0, d1, d2; };
        auto bounds = [&](int e) {
            const int ru = (e * (VB_TY + 1) + ly + 1) * VB_WX + lx, rd = ru - VB_WX;
            return Bounds{L.off[ru - 1], L.off[ru], L.off[ru + 1], rd > 0 ? L.off[rd - 1] : 0, L.off[rd], L.off[rd + 1]};
        };
        Bounds bp = bounds(tc0);
        for (int tc = tc0; tc < tc1; ++tc) {
            const Bounds bn = bounds(tc + 1);
            const float ft = (float)tc;
            // dsec_utils.py:43-45 pass order: xlim outer, ylim, tlim inner; pass (a, b, c) reads base
            // cell (tc - c, yc - b, xc - a) = run (bin tc + 1 - c, row ly + 1 - b, column lx + 1 - a)
            const int lo[8] = {bn.u1, bp.u1, bn.d1, bp.d1, bn.u0, bp.u0, bn.d0, bp.d0};
            const int hi[8] = {bn.u2, bp.u2, bn.d2, bp.d2, bn.u1, bp.u1, bn.d1, bp.d1};
            // the 8 runs as one sequence: k -> i = k + dl[p] for the pass p with end[p - 1] <= k < end[p]
            int end[8], dl[8], tot = 0;
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                dl[q] = lo[q] - tot;
                tot += hi[q] - lo[q];
                end[q] = tot;
            }
            float acc = 0.0f;
            for (int k = 0; k < tot; ++k) {
                int i = k + dl[7];
#pragma unroll
                for (int q = 6; q >= 0; --q) i = k < end[q] ? k + dl[q] : i;
                acc = __fadd_rn(acc, vt_term(ar ? gc[aords[i]].ev : L.ev[i], fx, fy, ft));
            }
            A.voxel[((int64_t)tc * A.H + yc) * A.W + xc] = acc;
            if (normalize && acc != 0.0f) {
                const double v = (double)acc;
                cn += 1.0;
                cs += v;
                css = fma(v, v, css);
            }
            bp = bn;
        }
    }
    if (normalize) {   // (count, mean, M2) of this thread's nonzero cells, then a fixed-order tree
        Moments m{0.0, 0.0, 0.0};
        if (cn > 0.0) {
            const double mean = cs / cn;
            m = {cn, mean, fmax(css - cs * mean, 0.0)};
        }
        __syncthreads();   // the fold's reads of L.ev are done: its bytes become the scratch
        m = block_moments(m, reinterpret_cast<double*>(L.ev));
        if (tid == 0) {
            A.part[3 * tile] = m.n;
            A.part[3 * tile + 1] = m.mean;
            A.part[3 * tile + 2] = m.m2;
        }
    }
}

// The tiled DSEC path's tile grid, or false where it does not apply (its LDS counts or run table
// would overflow, or 32-bit copy positions): then the key-range pipeline runs.
struct VTileGeom { int gy, gx, nb, nblk; };
inline bool vtile_geom(int64_t n, int C, int H, int W, VTileGeom* g) {
    g->gy = (H + VB_TY - 1) / VB_TY;
    g->gx = (W + VB_TX - 1) / VB_TX;
    const int64_t nb = (int64_t)g->gy * g->gx;
    g->nb = (int)std::min<int64_t>(nb, 1 << 30);
    g->nblk = (int)((n + VB_EPB - 1) / VB_EPB);
    return nb <= VB_MAXNB && (int64_t)(C + 1) * VB_WK <= VB_MAXRUN && 4 * n < (int64_t)1 << 31 && W < 65535 &&
           H < 65535;
}

inline size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

// Workspace carve-up (every piece 256-byte aligned).
struct VoxelWs {
    size_t key, rank, cnt, off, slot, fa, fb, payload, norm, part, scan_sums, total;
};

// grid-stride gather: this many blocks (normalization partials); one cell per thread (18,000
// blocks at DSEC) was slower, 88 vs 75 us, and its 18,000 partials cost the one-block finalize 31 us
constexpr int kGatherBlocks = 2048;

int plan(int64_t n, uint32_t K, int64_t cells, VoxelWs* w) {
    (void)cells;
    size_t o = 0;
    auto take = [&](size_t bytes) { const size_t at = o; o += align256(bytes); return at; };
    w->key = take(4 * (size_t)n);
    w->rank = take(4 * (size_t)n);
    w->cnt = take(4 * ((size_t)K + 1));
    w->off = take(4 * ((size_t)K + 1));
    w->slot = take(4 * (size_t)n);
    w->fa = take(4 * (size_t)n);
    w->fb = take(4 * (size_t)n);
    w->payload = take(16 * (size_t)n);
    w->norm = take(sizeof(NormState));
    w->part = take(3 * 8 * (size_t)kGatherBlocks);
    w->scan_sums = take(4 * (((size_t)K + 1 + SCAN_T - 1) / SCAN_T));
    w->total = o;
    return ECORR_OK;
}

inline int hip_status() {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? ECORR_OK : ECORR_EHIP - (int)e;
}

// Workspace of the tiled DSEC path.
struct VTileWs {
    size_t slot, M, tot, S, pay, norm, part, aord, aords, total;
};

void plan_tiled(int64_t n, const VTileGeom& g, VTileWs* w) {
    size_t o = 0;
    auto take = [&](size_t bytes) { const size_t at = o; o += align256(bytes); return at; };
    const size_t copies = 4 * (size_t)n;   // an event lies in at most 4 windows
    w->slot = take(8 * (size_t)n);
    w->M = take(4 * (size_t)g.nblk * g.nb);
    w->tot = take(4 * ((size_t)g.nb + 1));
    w->S = take(4 * ((size_t)g.nb + 1));
    w->pay = take(sizeof(VCopy) * copies);
    w->norm = take(sizeof(NormState));
    w->part = take(3 * 8 * (size_t)g.nb);
    w->aord = take(4 * copies);
    w->aords = take(4 * copies);
    w->total = o;
}

int launch_voxel_tiled(const float* p, const float* t, const float* x, const float* y, int64_t n, int C, int H,
                       int W, int normalize, float* voxel, void* workspace, const VTileGeom& g, hipStream_t stream) {
    VTileWs w;
    plan_tiled(n, g, &w);
    char* base = (char*)workspace;
    VTileArgs A{};
    A.p = p; A.t = t; A.x = x; A.y = y;
    A.n = n; A.C = C; A.H = H; A.W = W;
    A.gy = g.gy; A.gx = g.gx; A.nb = g.nb; A.nblk = g.nblk;
    A.slot = (uint2*)(base + w.slot);
    A.M = (uint32_t*)(base + w.M);
    A.tot = (uint32_t*)(base + w.tot);
    A.S = (uint32_t*)(base + w.S);
    A.pay = (VCopy*)(base + w.pay);
    A.part = (double*)(base + w.part);
    A.voxel = voxel;
    A.aord = (uint32_t*)(base + w.aord);
    A.aords = (uint32_t*)(base + w.aords);
    A.norm = (NormState*)(base + w.norm);
    int st;
    hipLaunchKernelGGL(vb_count, dim3(g.nblk), dim3(VB_CNT), 0, stream, A);
    hipLaunchKernelGGL(vb_colscan, dim3((unsigned)((g.nb + 1 + NTV - 1) / NTV)), dim3(NTV), 0, stream, A);
    hipLaunchKernelGGL(vb_starts, dim3(1), dim3(NTV), 0, stream, A);
    hipLaunchKernelGGL(vb_scatter, dim3(blocks_for(n)), dim3(NTV), 0, stream, A);
    hipLaunchKernelGGL(vb_gather, dim3(g.nb), dim3(VB_NT), 0, stream, A, normalize);
    if ((st = hip_status()) != ECORR_OK) return st;
    if (normalize) {
        hipLaunchKernelGGL(norm_finalize, dim3(1), dim3(NTV), 0, stream, A.part, g.nb, A.norm);
        launch_norm_apply(voxel, (int64_t)C * H * W, A.norm, stream);
    }
    return hip_status();
}

}  // namespace

uint32_t voxel_key_range(bool dsec, int C, int H, int W) {
    return dsec ? (uint32_t)((C + 1) * (H + 1) * (W + 1)) : (uint32_t)(C * H * W);
}

int voxel_workspace_bytes(bool dsec, int64_t n, int C, int H, int W, int64_t* bytes) {
    VTileGeom g;
    if (dsec && vtile_geom(n, C, H, W, &g)) {
        VTileWs tw;
        plan_tiled(n, g, &tw);
        *bytes = (int64_t)tw.total;
        return ECORR_OK;
    }
    VoxelWs w;
    const int st = plan(n, voxel_key_range(dsec, C, H, W), (int64_t)C * H * W, &w);
    if (st == ECORR_OK) *bytes = (int64_t)w.total;
    return st;
}

int launch_voxel(bool dsec, const float* p, const float* t, const float* x, const float* y, const double* ev,
                 int64_t n, int C, int H, int W, int normalize, float* voxel, int* bad, void* workspace,
                 hipStream_t stream) {
    VTileGeom g;
    if (dsec && vtile_geom(n, C, H, W, &g))
        return launch_voxel_tiled(p, t, x, y, n, C, H, W, normalize, voxel, workspace, g, stream);
    VoxelArgs A{};
    A.p = p; A.t = t; A.x = x; A.y = y; A.ev = ev;
    A.n = n; A.C = C; A.H = H; A.W = W;
    A.K = voxel_key_range(dsec, C, H, W);
    VoxelWs w;
    const int64_t cells = (int64_t)C * H * W;
    int st = plan(n, A.K, cells, &w);
    if (st != ECORR_OK) return st;
    char* base = (char*)workspace;
    A.key = (uint32_t*)(base + w.key);
    A.rank = (uint32_t*)(base + w.rank);
    A.cnt = (uint32_t*)(base + w.cnt);
    A.off = (uint32_t*)(base + w.off);
    A.slot = (int*)(base + w.slot);
    A.fa = (float*)(base + w.fa);
    A.fb = (float*)(base + w.fb);
    A.payload = (float4*)(base + w.payload);
    A.part = (double*)(base + w.part);
    A.voxel = voxel;
    A.bad = bad;
    NormState* ns = (NormState*)(base + w.norm);

    // (the whole 256-byte-aligned piece: one aligned fill instead of body + tail)
    hipError_t e = hipMemsetAsync(A.cnt, 0, align256(4 * ((size_t)A.K + 1)), stream);
    if (e != hipSuccess) return ECORR_EHIP - (int)e;
    if (dsec) hipLaunchKernelGGL(prep_dsec, dim3(blocks_for(n)), dim3(NTV), 0, stream, A);
    else hipLaunchKernelGGL(prep_mvsec, dim3(blocks_for(n)), dim3(NTV), 0, stream, A);
    if ((st = hip_status()) != ECORR_OK) return st;
    {   // exclusive scan over K + 1 counts (cnt[K] = 0): off[K] = the runs' total
        const int64_t K1 = (int64_t)A.K + 1;
        const unsigned nb = (unsigned)((K1 + SCAN_T - 1) / SCAN_T);
        uint32_t* sums = (uint32_t*)(base + w.scan_sums);
        hipLaunchKernelGGL(scan_reduce, dim3(nb), dim3(NTV), 0, stream, A.cnt, K1, sums);
        hipLaunchKernelGGL(scan_sums, dim3(1), dim3(NTV), 0, stream, sums, (int)nb);
        hipLaunchKernelGGL(scan_apply, dim3(nb), dim3(NTV), 0, stream, A.cnt, K1, sums, A.off);
        if ((st = hip_status()) != ECORR_OK) return st;
    }
    if (dsec) hipLaunchKernelGGL(fill_runs<true>, dim3(blocks_for(n)), dim3(NTV), 0, stream, A);
    else hipLaunchKernelGGL(fill_runs<false>, dim3(blocks_for(n)), dim3(NTV), 0, stream, A);
    if (dsec) hipLaunchKernelGGL(order_runs<true>, dim3(blocks_for(n)), dim3(NTV), 0, stream, A);
    else hipLaunchKernelGGL(order_runs<false>, dim3(blocks_for(n)), dim3(NTV), 0, stream, A);
    const unsigned gblocks = (unsigned)std::min<int64_t>(kGatherBlocks, (int64_t)C * H);
    if (dsec) hipLaunchKernelGGL(gather<true>, dim3(gblocks), dim3(NTV), 0, stream, A, normalize);
    else hipLaunchKernelGGL(gather<false>, dim3(gblocks), dim3(NTV), 0, stream, A, normalize);
    if ((st = hip_status()) != ECORR_OK) return st;
    if (normalize) {
        hipLaunchKernelGGL(norm_finalize, dim3(1), dim3(NTV), 0, stream, A.part, (int)gblocks, ns);
        launch_norm_apply(voxel, cells, ns, stream);
    }
    return hip_status();
}

}  // namespace ecorr
