// splat.hip -- SURVEY §8f row 2: the warm-start forward splat on gfx950.
//
// Replaces utils/image_utils.py:10-47 (grid_sample_values) and :50-83 (forward_interpolate_pytorch,
// the producer of flow_init, test.py:199).  Each point s (x, y, z[c]) adds z*wgt and wgt into the
// four integer neighbours t of (x, y) in pass order (floor,floor), (floor,ceil), (ceil,floor),
// (ceil,ceil), wgt = (1 - |x - xv|) (1 - |y - yv|); the result is values / (wacc + 1e-15).
//
// Determinism and bit-exactness: the reference's put_(accumulate=True) on CPU folds each target's
// contributions serially in (pass, point) order.  A float atomicAdd scatter would sum them in
// arrival order, so instead the scatter is inverted into a gather with a counting sort:
//   1. count contributions per target        (LDS atomics, integer: order-free)
//   2. exclusive scan of the counts          (block scan)
//   3. drop each contribution's key (pass, s) into its target's bucket; integer atomics pick the
//      slot, in rounds of consecutive keys, so a bucket is sorted up to the keys of one round
//   4. per target: insertion-sort the (nearly sorted) bucket, then fold the contributions
//      recomputed from the keys in ascending key order = the reference's order, bit for bit.
// One 1024-thread workgroup per batch item; E-RAFT's flows are 1/8-resolution maps (<= 14720
// points at 1280x720), so the counts live in LDS (<= 16384 targets) and the work is latency-bound
// (a few microseconds), not bandwidth-bound: in LDS mode (DSEC, MVSEC) all four phases run out of
// LDS; larger maps keep keys (and counts past 16384 targets) in the caller's workspace.

#include "ecorr_device.h"
#include "ecorr_internal.h"

namespace ecorr {

namespace {

constexpr int NTS = 1024;
constexpr int kLdsTargets = 16384;   // global mode: counts in LDS up to this many targets
constexpr int kPool = 36864;         // LDS mode: 144 KB holds counts, keys and the points
constexpr int kPassShift = 24;       // key = pass << 24 | point (n < 2^24, checked at the ABI)

struct SplatArgs {
    const float* pts;   // FLOW: flow [B][2][n] (n = h*w); else points [3][n] (x, y, z)
    float* values;      // [B][nz][h*w]
    uint8_t* valid;     // [B][h*w] or null
    int* ws_count;      // [B][h*w] (global mode with h*w > kLdsTargets)
    int* ws_keys;       // [B][4n] (global mode)
    int64_t n;
    int h, w;
};

// Floats per point: FLOW -> (dx, dy); points -> (x, y, z).
template <bool FLOW> constexpr int kPtFloats = FLOW ? 2 : 3;

// The point s: position and value channels, from `src` = the item's point data ([k][n] planes,
// global or its LDS copy).
template <bool FLOW>
__device__ __forceinline__ void point(const float* src, int n, int w, float rcp_w, int s, float& x, float& y, float* z) {
    if (FLOW) {
        z[0] = src[s];
        z[1] = src[n + s];
        // row = s / w without an integer division: the float quotient is within one of it
        int row = (int)((float)s * rcp_w);
        row -= row * w > s;
        row += (row + 1) * w <= s;
        // image_utils.py:62-66: int64 meshgrid + fp32 flow -> fp32 add
        x = __fadd_rn((float)(s - row * w), z[0]);
        y = __fadd_rn((float)row, z[1]);
    } else {
        x = src[s];
        y = src[n + s];
        z[0] = src[2 * n + s];
    }
}

// Contribution (pass, point s) -> target index (or -1 out of bounds) and weight.  Its sort key is
// pass << kPassShift | s: ascending keys = the reference's (pass, point) order.
__device__ __forceinline__ int target_of(int pass, float x, float y, int h, int w, float& wgt) {
    const float xv = (pass & 2) ? ceilf(x) : floorf(x);   // image_utils.py:28 outer loop: x
    const float yv = (pass & 1) ? ceilf(y) : floorf(y);   //                  inner loop: y
    // :31 in_bounds_mask (false for NaN)
    if (!((xv < (float)w) & (xv >= 0.0f) & (yv < (float)h) & (yv >= 0.0f))) return -1;
    // :34 weights = (1 - |x - xv|) * (1 - |y - yv|)
    wgt = __fmul_rn(__fsub_rn(1.0f, fabsf(__fsub_rn(x, xv))), __fsub_rn(1.0f, fabsf(__fsub_rn(y, yv))));
    // :37 indices = (x_vals + width * y_vals).long(), computed in fp32 like the reference
    return (int)__fadd_rn(xv, __fmul_rn((float)w, yv));
}

// LDS mode (counts + keys + points fit kPool: every E-RAFT size up to DSEC, and MVSEC): the item's
// points are staged into LDS once and all four phases run out of LDS.  Global mode: counts in LDS
// when they fit, keys in the workspace, points re-read from global memory.
template <bool FLOW, bool LDS>
__global__ __launch_bounds__(NTS) void splat_kernel(SplatArgs A) {
    constexpr int NZ = FLOW ? 2 : 1, NP = kPtFloats<FLOW>;
    __shared__ int pool[LDS ? kPool : kLdsTargets];
    __shared__ int wsum[NTS / kWave];
    __shared__ int carry_s;
    const int tid = threadIdx.x, b = blockIdx.x;
    const int n = (int)A.n, hw = A.h * A.w, ne = 4 * n;
    const float* gpts = A.pts + (int64_t)b * NP * n;
    const float rcp_w = 1.0f / (float)A.w;
    int* cnt;
    int* keys;
    const float* src;
    if (LDS) {
        cnt = pool;
        keys = pool + hw;
        float* lp = reinterpret_cast<float*>(pool + hw + ne);
        for (int i = tid; i < NP * n; i += NTS) lp[i] = gpts[i];
        src = lp;
    } else {
        cnt = hw <= kLdsTargets ? pool : A.ws_count + (int64_t)b * hw;
        keys = A.ws_keys + (int64_t)b * ne;
        src = gpts;
    }

    for (int t = tid; t < hw; t += NTS) cnt[t] = 0;
    __syncthreads();

    // 1. count
    for (int s = tid; s < n; s += NTS) {
        float x, y, z[NZ], wgt;
        point<FLOW>(src, n, A.w, rcp_w, s, x, y, z);
#pragma unroll
        for (int pass = 0; pass < 4; ++pass) {
            const int t = target_of(pass, x, y, A.h, A.w, wgt);
            if (t >= 0) atomicAdd(&cnt[t], 1);
        }
    }
    __syncthreads();

    // 2. exclusive scan; each thread owns SPT consecutive counts of a super-chunk
    constexpr int SPT = 8;
    if (tid == 0) carry_s = 0;
    const int lane = tid & (kWave - 1), wv = tid / kWave;
    for (int c0 = 0; c0 < hw; c0 += NTS * SPT) {
        __syncthreads();
        const int t0 = c0 + tid * SPT;
        int v[SPT], sum = 0;
#pragma unroll
        for (int j = 0; j < SPT; ++j) {
            v[j] = t0 + j < hw ? cnt[t0 + j] : 0;
            sum += v[j];
        }
        int inc = sum;
#pragma unroll
        for (int d = 1; d < kWave; d <<= 1) {
            const int u = __shfl_up(inc, d, kWave);
            if (lane >= d) inc += u;
        }
        if (lane == kWave - 1) wsum[wv] = inc;
        __syncthreads();
        int run = carry_s + inc - sum;
        for (int i = 0; i < wv; ++i) run += wsum[i];
#pragma unroll
        for (int j = 0; j < SPT; ++j) {
            if (t0 + j < hw) cnt[t0 + j] = run;
            run += v[j];
        }
        __syncthreads();
        if (tid == NTS - 1) carry_s = run;
    }
    __syncthreads();

    // 3. fill buckets (cnt[t] walks from the bucket start to the next bucket's start) in rounds
    // of NTS consecutive points of one pass, a barrier between rounds: slots are handed out in
    // (pass, round) order, so a bucket is already sorted except among the few keys of one round
    // that hit the same target -- the insertion sort of phase 4 then does O(bucket) work.
    for (int pass = 0; pass < 4; ++pass)
        for (int s0 = 0; s0 < n; s0 += NTS) {
            const int s = s0 + tid;
            if (s < n) {
                float x, y, z[NZ], wgt;
                point<FLOW>(src, n, A.w, rcp_w, s, x, y, z);
                const int t = target_of(pass, x, y, A.h, A.w, wgt);
                if (t >= 0) keys[atomicAdd(&cnt[t], 1)] = pass << kPassShift | s;
            }
            __syncthreads();
        }

    // 4. per target: order the bucket, fold in key order from +0 (put_ into torch.zeros)
    float* vout = A.values + (int64_t)b * NZ * hw;
    for (int t = tid; t < hw; t += NTS) {
        const int lo = t > 0 ? cnt[t - 1] : 0, hi = cnt[t];
        for (int i = lo + 1; i < hi; ++i) {
            const int k = keys[i];
            int j = i - 1;
            while (j >= lo && keys[j] > k) { keys[j + 1] = keys[j]; --j; }
            keys[j + 1] = k;
        }
        float acc[NZ], wacc = 0.0f;
#pragma unroll
        for (int c = 0; c < NZ; ++c) acc[c] = 0.0f;
        for (int i = lo; i < hi; ++i) {
            const int e = keys[i];
            const int pass = e >> kPassShift;
            float x, y, z[NZ], wgt = 0.0f;
            point<FLOW>(src, n, A.w, rcp_w, e & ((1 << kPassShift) - 1), x, y, z);
            target_of(pass, x, y, A.h, A.w, wgt);
#pragma unroll
            for (int c = 0; c < NZ; ++c) acc[c] = __fadd_rn(acc[c], __fmul_rn(z[c], wgt));
            wacc = __fadd_rn(wacc, wgt);
        }
        // :44 values_ipl / (weights_acc + 1e-15)
        const float den = __fadd_rn(wacc, 1e-15f);
#pragma unroll
        for (int c = 0; c < NZ; ++c) vout[c * hw + t] = __fdiv_rn(acc[c], den);
        if (A.valid) A.valid[(int64_t)b * hw + t] = wacc > 0.0f;
    }
}

// ============================================================================================
// Round 5: the banded splat.  splat_kernel runs one workgroup per batch item
// (16 of 256 CUs at DSEC B = 16, 47 us).  Here an item's targets are split into G contiguous bands
// (G * B ~ 256 workgroups over the chip) and each workgroup serves one band on its own:
//   1. every contribution (pass, s) of the item is evaluated (target_of), those landing in the band
//      counted per target (LDS atomics) and listed as (key, target) (LDS, arbitrary order);
//   2. exclusive scan of the band's counts;
//   3. the listed keys dropped into their targets' buckets (LDS atomics pick the slots);
//   4. per target: insertion-sort the bucket, fold in ascending key order = the reference's serial
//      (pass, point) order, bit for bit, divide.
// Points are staged in LDS when they fit.  A band whose contributions exceed the list's capacity is
// served in sub-ranges of targets (re-evaluating the contributions per sub-range, buckets ordered by
// rank as in step 3); a single target holding more than the capacity is folded by one wave walking
// the contributions in key order.
// ============================================================================================
constexpr int NTB = 1024;            // threads per band workgroup
constexpr int kBandCap = 6144;       // listed contributions per band (LDS)
constexpr int kBandPts = 10240;      // point floats staged in LDS (FLOW: n <= 5120)
constexpr int kBandTargets = 2048;   // targets per band (counts in LDS)
constexpr int64_t kBandMaxN = 65536; // banded kernel for n <= this (every E-RAFT flow map)

template <bool FLOW>
__global__ __launch_bounds__(NTB) void splat_band_kernel(SplatArgs A, int G) {
    constexpr int NZ = FLOW ? 2 : 1, NP = kPtFloats<FLOW>;
    __shared__ float spts[kBandPts];
    __shared__ int cnt[kBandTargets + 1];
    __shared__ int lkey[kBandCap], ltgt[kBandCap], keys[kBandCap], stgt[kBandCap];
    __shared__ int wsum[NTB / kWave];
    __shared__ int nlist, carry_s;
    __shared__ int sub[kBandTargets + 1];   // sub-range boundaries (overflow path)
    // one linear block index (band fastest): no gridDim.y limit on the batch (B > 65535 launches)
    const int tid = threadIdx.x, band = (int)(blockIdx.x % (unsigned)G), b = (int)(blockIdx.x / (unsigned)G);
    const int n = (int)A.n, hw = A.h * A.w;
    const int t0 = (int)((int64_t)band * hw / G), t1 = (int)((int64_t)(band + 1) * hw / G), nb = t1 - t0;
    const float* gpts = A.pts + (int64_t)b * NP * n;
    const float rcp_w = 1.0f / (float)A.w;
    const bool staged = NP * n <= kBandPts;
    if (staged) {   // every load in flight before the first LDS write (16-byte pieces where aligned)
        constexpr int PER = (kBandPts + 4 * NTB - 1) / (4 * NTB);
        const int nf = NP * n;
        if ((reinterpret_cast<uintptr_t>(gpts) & 15) == 0) {
            float4 v[PER];
#pragma unroll
            for (int j = 0; j < PER; ++j) {
                const int i = 4 * (tid + j * NTB);
                v[j] = i + 3 < nf ? *reinterpret_cast<const float4*>(gpts + i) : float4{0.f, 0.f, 0.f, 0.f};
            }
#pragma unroll
            for (int j = 0; j < PER; ++j) {
                const int i = 4 * (tid + j * NTB);
                if (i + 3 < nf) *reinterpret_cast<float4*>(spts + i) = v[j];
                else
                    for (int k = i; k < nf && k < i + 4; ++k) spts[k] = gpts[k];
            }
        } else {
            for (int i = tid; i < nf; i += NTB) spts[i] = gpts[i];
        }
    }
    for (int t = tid; t <= nb; t += NTB) cnt[t] = 0;
    if (tid == 0) nlist = 0;
    __syncthreads();
    const float* src = staged ? spts : gpts;

    // 1. count + list the band's contributions.  Points read from global memory (maps too large to
    // stage) are gathered PPT at a time, every load in flight before the first use.
    // a point whose two target rows (floor / ceil of y) both miss the band's rows has nothing here
    // (target index = x + w y exactly while h w <= 2^24; NaN never compares true and goes on)
    const bool rows_exact = (int64_t)hw <= (1 << 24);
    const float rlo = (float)(t0 / A.w), rhi = (float)((t1 - 1) / A.w);
    auto count_point = [&](int s, float x, float y) {
        if (rows_exact && (ceilf(y) < rlo || floorf(y) > rhi)) return;
        float wgt;
#pragma unroll
        for (int pass = 0; pass < 4; ++pass) {
            const int t = target_of(pass, x, y, A.h, A.w, wgt);
            const bool in = t >= t0 && t < t1;
            if (in) atomicAdd(&cnt[t - t0], 1);
            // list slot: one LDS atomic per wave (the in-band lanes' count), lanes by their rank
            const uint64_t m = __builtin_amdgcn_ballot_w64(in);
            if (m) {
                int base = 0;
                if (__lane_id() == (int)__builtin_ctzll(m)) base = atomicAdd(&nlist, __builtin_popcountll(m));
                base = __shfl(base, (int)__builtin_ctzll(m), kWave);
                const int i = base + __builtin_popcountll(m & ((1ull << __lane_id()) - 1ull));
                if (in && i < kBandCap) {
                    lkey[i] = pass << kPassShift | s;
                    ltgt[i] = t - t0;
                }
            }
        }
    };
    constexpr int PPT = 16;   // 16 x 1024 points: every E-RAFT map in one round of loads
    if (staged) {
        for (int s = tid; s < n; s += NTB) {
            float x, y, z[NZ];
            point<FLOW>(src, n, A.w, rcp_w, s, x, y, z);
            count_point(s, x, y);
        }
    } else {
        for (int s0 = tid; s0 < n; s0 += PPT * NTB) {
            float x[PPT], y[PPT], z[PPT][NZ];
#pragma unroll
            for (int j = 0; j < PPT; ++j) {
                const int s = s0 + j * NTB;
                x[j] = y[j] = 0.0f;
                if (s < n) point<FLOW>(src, n, A.w, rcp_w, s, x[j], y[j], z[j]);
            }
#pragma unroll
            for (int j = 0; j < PPT; ++j)
                if (s0 + j * NTB < n) count_point(s0 + j * NTB, x[j], y[j]);
        }
    }
    __syncthreads();

    // 2. exclusive scan of cnt[0 .. nb) (nb <= kBandTargets <= NTB * 2): two per thread
    {
        const int lane = tid & (kWave - 1), wv = tid / kWave;
        const int i0 = 2 * tid;
        const int v0 = i0 < nb ? cnt[i0] : 0, v1 = i0 + 1 < nb ? cnt[i0 + 1] : 0;
        const int sum = v0 + v1;
        int inc = sum;
#pragma unroll
        for (int d = 1; d < kWave; d <<= 1) {
            const int u = __shfl_up(inc, d, kWave);
            if (lane >= d) inc += u;
        }
        if (lane == kWave - 1) wsum[wv] = inc;
        __syncthreads();
        int run = inc - sum;
        for (int i = 0; i < wv; ++i) run += wsum[i];
        __syncthreads();
        if (i0 < nb) cnt[i0] = run;
        if (i0 + 1 < nb) cnt[i0 + 1] = run + v0;
        if (tid == NTB - 1) cnt[nb] = run + sum;   // total
    }
    __syncthreads();
    // cnt[t] = start of target t's bucket, cnt[nb] = the band's total

    float* vout = A.values + (int64_t)b * NZ * hw;
    // 4. per target: fold its bucket, already in key order (sorted[lo, hi)), or (huge) fold target t
    // by walking every contribution in key order
    auto fold_sorted = [&](const int* sorted, int t, int lo, int hi) {
        float acc[NZ], wacc = 0.0f;
#pragma unroll
        for (int c = 0; c < NZ; ++c) acc[c] = 0.0f;
        for (int i = lo; i < hi; ++i) {
            const int e = sorted[i];
            float x, y, z[NZ], wgt = 0.0f;
            point<FLOW>(src, n, A.w, rcp_w, e & ((1 << kPassShift) - 1), x, y, z);
            target_of(e >> kPassShift, x, y, A.h, A.w, wgt);
#pragma unroll
            for (int c = 0; c < NZ; ++c) acc[c] = __fadd_rn(acc[c], __fmul_rn(z[c], wgt));
            wacc = __fadd_rn(wacc, wgt);
        }
        const float den = __fadd_rn(wacc, 1e-15f);   // :44 values_ipl / (weights_acc + 1e-15)
#pragma unroll
        for (int c = 0; c < NZ; ++c) vout[c * hw + t0 + t] = __fdiv_rn(acc[c], den);
        if (A.valid) A.valid[(int64_t)b * hw + t0 + t] = wacc > 0.0f;
    };
    // one wave (one thread walking 4n contributions took 3.4 ms at DSEC): its lanes
    // evaluate 64 consecutive contributions of a pass at once, then the hits are folded one after
    // another in lane (= point) order from the lanes' products -- the serial fold, bit for bit
    auto fold_walk = [&](int t) {
        const int lane = __lane_id();
        float acc[NZ], wacc = 0.0f;
#pragma unroll
        for (int c = 0; c < NZ; ++c) acc[c] = 0.0f;
        for (int pass = 0; pass < 4; ++pass)
            for (int s0 = 0; s0 < n; s0 += kWave) {
                const int s = s0 + lane;
                float term[NZ], wgt = 0.0f;
                bool hit = false;
                if (s < n) {
                    float x, y, z[NZ];
                    point<FLOW>(src, n, A.w, rcp_w, s, x, y, z);
                    hit = target_of(pass, x, y, A.h, A.w, wgt) == t0 + t;
#pragma unroll
                    for (int c = 0; c < NZ; ++c) term[c] = __fmul_rn(z[c], wgt);
                }
                for (uint64_t m = __builtin_amdgcn_ballot_w64(hit); m; m &= m - 1) {
                    const int l = (int)__builtin_ctzll(m);
#pragma unroll
                    for (int c = 0; c < NZ; ++c) acc[c] = __fadd_rn(acc[c], __shfl(term[c], l, kWave));
                    wacc = __fadd_rn(wacc, __shfl(wgt, l, kWave));
                }
            }
        if (lane != 0) return;
        const float den = __fadd_rn(wacc, 1e-15f);
#pragma unroll
        for (int c = 0; c < NZ; ++c) vout[c * hw + t0 + t] = __fdiv_rn(acc[c], den);
        if (A.valid) A.valid[(int64_t)b * hw + t0 + t] = wacc > 0.0f;
    };

    const int total = cnt[nb];
    if (total <= kBandCap) {   // block-uniform: the common case
        // 3. bucket the listed keys (cnt[t] walks to the next bucket's start), then order each
        // bucket by rank: slot i's key goes to lo + #{keys of its bucket smaller than it} (keys are
        // distinct) -- k independent LDS reads per slot, so a heavy bucket costs depth k, not k^2
        for (int i = tid; i < total; i += NTB) {
            const int t = ltgt[i];
            const int slot = atomicAdd(&cnt[t], 1);
            keys[slot] = lkey[i];
            stgt[slot] = t;
        }
        __syncthreads();
        for (int i = tid; i < total; i += NTB) {
            const int t = stgt[i], k = keys[i];
            const int lo = t > 0 ? cnt[t - 1] : 0, hi = cnt[t];
            int r = 0;
            for (int j = lo; j < hi; ++j) r += keys[j] < k;
            lkey[lo + r] = k;
        }
        __syncthreads();
        for (int t = tid; t < nb; t += NTB) fold_sorted(lkey, t, t > 0 ? cnt[t - 1] : 0, cnt[t]);
        return;
    }
    // overflow: sub-ranges [sub[r], sub[r + 1]) of targets holding <= kBandCap contributions each,
    // or one target holding more (folded by walking)
    if (tid == 0) {
        int r = 0, a = 0;
        sub[0] = 0;
        while (a < nb) {
            int e = a + 1;
            while (e < nb && cnt[e + 1] - cnt[a] <= kBandCap) ++e;
            sub[++r] = e;
            a = e;
        }
        carry_s = r;
    }
    __syncthreads();
    const int nsub = carry_s;
    for (int r = 0; r < nsub; ++r) {
        const int a = sub[r], e = sub[r + 1];
        const int base = cnt[a];
        if (cnt[e] - base > kBandCap) {   // one target (e = a + 1) beyond the capacity
            if (tid < kWave) fold_walk(a);
            __syncthreads();
            continue;
        }
        // slots of the sub-range: bucket starts relative to base, in the listed-key array (reused)
        for (int t = a + tid; t < e; t += NTB) lkey[t - a] = cnt[t] - base;
        __syncthreads();
        for (int s = tid; s < n; s += NTB) {
            float x, y, z[NZ], wgt;
            point<FLOW>(src, n, A.w, rcp_w, s, x, y, z);
#pragma unroll
            for (int pass = 0; pass < 4; ++pass) {
                const int t = target_of(pass, x, y, A.h, A.w, wgt) - t0;
                if (t >= a && t < e) {
                    const int slot = atomicAdd(&lkey[t - a], 1);
                    keys[slot] = pass << kPassShift | s;
                    ltgt[slot] = t;
                }
            }
        }
        __syncthreads();
        // order each bucket by rank, as the main path (an insertion sort per bucket on one
        // thread cost O(k^2) serial LDS steps -- 178 ms per call on the collision map)
        for (int i = tid; i < cnt[e] - base; i += NTB) {
            const int t = ltgt[i], k = keys[i];
            const int lo = cnt[t] - base, hi = cnt[t + 1] - base;
            int rk = 0;
            for (int j = lo; j < hi; ++j) rk += keys[j] < k;
            stgt[lo + rk] = k;
        }
        __syncthreads();
        for (int t = a + tid; t < e; t += NTB) fold_sorted(stgt, t, cnt[t] - base, cnt[t + 1] - base);
        __syncthreads();
    }
}

bool lds_mode(bool flow_mode, int64_t n, int64_t hw) {
    return hw + 4 * n + (flow_mode ? 2 : 3) * n <= kPool;
}

inline int hip_status() {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? ECORR_OK : ECORR_EHIP - (int)e;
}

bool band_mode(int64_t n) { return n <= kBandMaxN; }

// bands per item: about 256 workgroups over the chip, at most kBandTargets targets per band
int band_count(int B, int64_t hw) {
    const int64_t need = (hw + kBandTargets - 1) / kBandTargets;
    int64_t g = 256 / B;
    g = g < need ? need : g;
    g = g > hw ? hw : g;
    return (int)(g < 1 ? 1 : g);
}

}  // namespace

int64_t splat_workspace_bytes(bool flow_mode, int B, int64_t n, int h, int w) {
    const int64_t hw = (int64_t)h * w;
    if (band_mode(n) || lds_mode(flow_mode, n, hw)) return 0;
    return (int64_t)B * ((hw > kLdsTargets ? hw : 0) + 4 * n) * (int64_t)sizeof(int);
}

int launch_splat(bool flow_mode, const float* pts, int B, int64_t n, int h, int w, float* values, uint8_t* valid,
                 void* workspace, hipStream_t stream) {
    SplatArgs A{};
    A.pts = pts;
    A.values = values;
    A.valid = valid;
    A.n = n;
    A.h = h;
    A.w = w;
    const int64_t hw = (int64_t)h * w;
    int* ws = (int*)workspace;
    A.ws_count = hw > kLdsTargets ? ws : nullptr;
    A.ws_keys = ws ? ws + (hw > kLdsTargets ? (int64_t)B * hw : 0) : nullptr;
    if (band_mode(n)) {
        const int G = band_count(B, hw);
        if ((int64_t)G * B > 0x7fffffff) return ECORR_EINVAL;
        const dim3 grid((unsigned)(G * B));
        if (flow_mode) hipLaunchKernelGGL((splat_band_kernel<true>), grid, dim3(NTB), 0, stream, A, G);
        else hipLaunchKernelGGL((splat_band_kernel<false>), grid, dim3(NTB), 0, stream, A, G);
        return hip_status();
    }
    const bool lds = lds_mode(flow_mode, n, hw);
    if (flow_mode && lds) hipLaunchKernelGGL((splat_kernel<true, true>), dim3(B), dim3(NTS), 0, stream, A);
    else if (flow_mode) hipLaunchKernelGGL((splat_kernel<true, false>), dim3(B), dim3(NTS), 0, stream, A);
    else if (lds) hipLaunchKernelGGL((splat_kernel<false, true>), dim3(B), dim3(NTS), 0, stream, A);
    else hipLaunchKernelGGL((splat_kernel<false, false>), dim3(B), dim3(NTS), 0, stream, A);
    return hip_status();
}

}  // namespace ecorr
