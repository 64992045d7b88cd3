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

bool lds_mode(bool flow_mode, int64_t n, int64_t hw) {
    return hw + 4 * n + (flow_mode ? 2 : 3) * n <= kPool;
}

inline int hip_status() {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? ECORR_OK : ECORR_EHIP - (int)e;
}

}  // namespace

int64_t splat_workspace_bytes(bool flow_mode, int B, int64_t n, int h, int w) {
    const int64_t hw = (int64_t)h * w;
    if (lds_mode(flow_mode, n, hw)) return 0;
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
    const bool lds = lds_mode(flow_mode, n, hw);
    if (flow_mode && lds) hipLaunchKernelGGL((splat_kernel<true, true>), dim3(B), dim3(NTS), 0, stream, A);
    else if (flow_mode) hipLaunchKernelGGL((splat_kernel<true, false>), dim3(B), dim3(NTS), 0, stream, A);
    else if (lds) hipLaunchKernelGGL((splat_kernel<false, true>), dim3(B), dim3(NTS), 0, stream, A);
    else hipLaunchKernelGGL((splat_kernel<false, false>), dim3(B), dim3(NTS), 0, stream, A);
    return hip_status();
}

}  // namespace ecorr
