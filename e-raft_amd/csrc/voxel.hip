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
__global__ __launch_bounds__(NTV) void norm_finalize(const double* part, int nparts, NormState* st) {
    __shared__ double sh[3 * NTV];
    Moments m{0.0, 0.0, 0.0};
    for (int i = threadIdx.x; i < nparts; i += NTV) m = combine(m, {part[3 * i], part[3 * i + 1], part[3 * i + 2]});
    m = block_moments(m, sh);
    if (threadIdx.x == 0) {
        st->any = m.n > 0.0;
        st->mean = (float)m.mean;
        // unbiased std; one nonzero cell gives NaN like torch.std, and then v - mean
        st->stdv = m.n > 1.0 ? (float)sqrt(m.m2 / (m.n - 1.0)) : __int_as_float(0x7fc00000);
    }
}

__global__ __launch_bounds__(NTV) void norm_apply(float* __restrict__ g, int64_t n, const NormState* st) {
    if (!st->any) return;
    const float mean = st->mean, sd = st->stdv;
    for (int64_t i = blockIdx.x * (int64_t)NTV + threadIdx.x; i < n; i += (int64_t)gridDim.x * NTV) {
        const float v = g[i];
        if (v != 0.0f) g[i] = sd > 0.0f ? __fdiv_rn(__fsub_rn(v, mean), sd) : __fsub_rn(v, mean);
    }
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

}  // namespace

uint32_t voxel_key_range(bool dsec, int C, int H, int W) {
    return dsec ? (uint32_t)((C + 1) * (H + 1) * (W + 1)) : (uint32_t)(C * H * W);
}

int voxel_workspace_bytes(bool dsec, int64_t n, int C, int H, int W, int64_t* bytes) {
    VoxelWs w;
    const int st = plan(n, voxel_key_range(dsec, C, H, W), (int64_t)C * H * W, &w);
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
        hipLaunchKernelGGL(norm_apply, dim3(kRedBlocks), dim3(NTV), 0, stream, voxel, cells, ns);
    }
    return hip_status();
}

}  // namespace ecorr
