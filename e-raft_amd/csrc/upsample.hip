// upsample.hip -- SURVEY §8f row 4: convex 8x flow upsampling and the DSEC 16-bit PNG flow codec.
//
// ERAFT.upsample_flow (model/eraft.py:74-85), run after every GRU iteration (eraft.py:137-139):
//   mask  [N][9*64][H][W] viewed [N][1][9][8][8][H][W], softmax over the 9
//   unfold(8 * flow, 3x3, padding 1) viewed [N][2][9][1][1][H][W]
//   out[n][c][8h+i][8w+j] = sum_k softmax(mask[n][k*64 + i*8 + j][h][w])_k * 8 flow[n][c][h+ky-1][w+kx-1]
// with k = 3 ky + kx and zero padding.  The reference runs it as softmax, unfold, a broadcast
// multiply into a [N][2][9][8][8][H][W] tensor, a sum and a permute copy -- ~6 passes over
// 2x the mask size.  Here it is one pass: thread = (n, i, pixel p) with lanes on consecutive
// pixels, so each of its 72 mask loads is a coalesced 256-byte wave row, the 3x3 flow window
// comes from L1/L2, and the 8 sub-pixels j of a row leave as two float4 stores (a wave writes
// 64 x 32 contiguous bytes).  HBM-bound: 2304 B of mask in + 512 B of flow out per pixel.  The mask
// loads use the default cache policy (non-temporal loads: 42.2 vs 36.7 us at DSEC B = 16,
// profiles/r05_lab/up_ab_policy.txt); the output stores stay non-temporal.
//
// Numerics: softmax as max, exp(x - max), in-order sum, times the sum's reciprocal; then the
// in-order sum of the 9 products -- the reference's expression order.  exp is the hardware's
// exp2-based __expf and the division a v_rcp_f32 multiply (round 4: 42.9 vs 51.8 us per call at
// DSEC B=16, profiles/r04_lab/; normwise error vs an fp64 evaluation unchanged, 1.69e-6), so
// results agree with the reference within a few ulp rather than bit for bit (test bar 2e-6).
//
// DSEC submission codec (utils/visualization.py:75-93, utils/dsec_utils.py:66-83):
//   encode  uint16[h][w][3] = (u16)(int32)rint(flow * 128 + 2^15), channel 2 = 0 -- numpy's
//           float32 -> uint16 cast on x86 (cvttss2si, low 16 bits; NaN / out-of-int32 -> 0)
//   decode  flow[h][w][2] = (v - 2^15) / 128 where channel 2 == 1, else 0; valid = channel 2 == 1;
//           channel 2 outside {0, 1} is the reference's assertion failure (counted).
// Both are exact integer/byte work (bit-exact).
#include "ecorr_device.h"
#include "ecorr_internal.h"

namespace ecorr {

namespace {

constexpr int NTU = 256;

typedef float floatx4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(NTU) void upsample_kernel(const float* __restrict__ flow, const float* __restrict__ mask,
                                                      int H, int W, float* __restrict__ out) {
    const int HW = H * W;
    const int p = blockIdx.x * NTU + threadIdx.x;
    const int i = blockIdx.y, n = blockIdx.z;
    if (p >= HW) return;
    const int h = p / W, w = p - h * W;

    // 8 * flow over the 3x3 window, zero padded (F.unfold(8 * flow, [3,3], padding=1))
    float f8[2][9];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        const float* fc = flow + ((int64_t)n * 2 + c) * HW;
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            const int y = h + k / 3 - 1, x = w + k % 3 - 1;
            const bool in = (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W;
            f8[c][k] = in ? __fmul_rn(8.0f, fc[y * W + x]) : 0.0f;
        }
    }

    const float* mrow = mask + ((int64_t)n * 576 + i * 8) * HW + p;
    float res[2][8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        float m[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) m[k] = mrow[((int64_t)k * 64 + j) * HW];   // default policy: 36.7 vs 42.2 us non-temporal
        float mx = m[0];
#pragma unroll
        for (int k = 1; k < 9; ++k) mx = fmaxf(mx, m[k]);
        float s = 0.0f;
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            m[k] = __expf(__fsub_rn(m[k], mx));
            s = __fadd_rn(s, m[k]);
        }
        const float rs = __builtin_amdgcn_rcpf(s);
#pragma unroll
        for (int k = 0; k < 9; ++k) m[k] = __fmul_rn(m[k], rs);   // softmax output
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            float acc = 0.0f;
#pragma unroll
            for (int k = 0; k < 9; ++k) acc = __fadd_rn(acc, __fmul_rn(m[k], f8[c][k]));
            res[c][j] = acc;
        }
    }
    const int W8 = 8 * W;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        float* o = out + (((int64_t)n * 2 + c) * 8 * H + 8 * h + i) * W8 + 8 * w;
        __builtin_nontemporal_store(floatx4{res[c][0], res[c][1], res[c][2], res[c][3]}, (floatx4*)o);
        __builtin_nontemporal_store(floatx4{res[c][4], res[c][5], res[c][6], res[c][7]}, (floatx4*)(o + 4));
    }
}

// numpy float32 -> uint16 on x86: cvttss2si (NaN / beyond int32 -> INT_MIN), keep the low 16 bits.
__device__ __forceinline__ uint16_t x86_f32_to_u16(float v) {
    const int iv = (v >= -2147483648.0f && v < 2147483648.0f) ? (int)v : (int)0x80000000u;
    return (uint16_t)(iv & 0xffff);
}

__global__ __launch_bounds__(NTU) void png16_encode_kernel(const float* __restrict__ flow, int64_t HW, int64_t n,
                                                           uint16_t* __restrict__ out) {
    for (int64_t q = blockIdx.x * (int64_t)NTU + threadIdx.x; q < n; q += (int64_t)gridDim.x * NTU) {
        const int64_t b = q / HW, p = q - b * HW;
        const float u = flow[(b * 2 + 0) * HW + p], v = flow[(b * 2 + 1) * HW + p];
        // visualization.py:82 numpy.rint(flow*128 + 2**15) in float32
        out[3 * q + 0] = x86_f32_to_u16(rintf(__fadd_rn(__fmul_rn(u, 128.0f), 32768.0f)));
        out[3 * q + 1] = x86_f32_to_u16(rintf(__fadd_rn(__fmul_rn(v, 128.0f), 32768.0f)));
        out[3 * q + 2] = 0;   // :84 the third channel is written as zeros
    }
}

__global__ __launch_bounds__(NTU) void png16_decode_kernel(const uint16_t* __restrict__ in, int64_t n,
                                                           float* __restrict__ flow, uint8_t* __restrict__ valid,
                                                           int* __restrict__ bad) {
    for (int64_t q = blockIdx.x * (int64_t)NTU + threadIdx.x; q < n; q += (int64_t)gridDim.x * NTU) {
        const unsigned u = in[3 * q], v = in[3 * q + 1], m = in[3 * q + 2];
        const bool ok = m == 1;   // dsec_utils.py:73
        if (m > 1) atomicAdd(bad, 1);   // :75 assert np.all(flow_16bit[~valid2D, -1] == 0)
        // :79-80 (v - 2**15) / 128, exact in float32
        flow[2 * q + 0] = ok ? (float)((int)u - 32768) * 0.0078125f : 0.0f;
        flow[2 * q + 1] = ok ? (float)((int)v - 32768) * 0.0078125f : 0.0f;
        valid[q] = ok;
    }
}

inline int hip_status() {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? ECORR_OK : ECORR_EHIP - (int)e;
}

inline unsigned grid_for(int64_t n) {
    const int64_t g = (n + NTU - 1) / NTU;
    return (unsigned)(g < 16384 ? (g > 0 ? g : 1) : 16384);
}

}  // namespace

int launch_upsample_flow(const float* flow, const float* mask, int N, int H, int W, float* out, hipStream_t stream) {
    const dim3 grid((unsigned)((H * W + NTU - 1) / NTU), 8, (unsigned)N);
    hipLaunchKernelGGL(upsample_kernel, grid, dim3(NTU), 0, stream, flow, mask, H, W, out);
    return hip_status();
}

int launch_png16_encode(const float* flow, int B, int h, int w, uint16_t* out, hipStream_t stream) {
    const int64_t HW = (int64_t)h * w, n = (int64_t)B * HW;
    hipLaunchKernelGGL(png16_encode_kernel, dim3(grid_for(n)), dim3(NTU), 0, stream, flow, HW, n, out);
    return hip_status();
}

int launch_png16_decode(const uint16_t* in, int B, int h, int w, float* flow, uint8_t* valid, int* bad,
                        hipStream_t stream) {
    const int64_t n = (int64_t)B * h * w;
    hipLaunchKernelGGL(png16_decode_kernel, dim3(grid_for(n)), dim3(NTU), 0, stream, in, n, flow, valid, bad);
    return hip_status();
}

}  // namespace ecorr
