// motion.hip -- SURVEY §8f row 1: the lookup fused with its only consumer, the 1x1 convolution +
// ReLU that opens BasicMotionEncoder (update.py:67,74: cor = F.relu(self.convc1(corr))):
//
//   out[b][o][p] = relu(bias[o] + sum_c W[o][c] * corr[b][c][p]),   c < C = levels (2r+1)^2
//
// where corr is exactly what ecorr_lookup returns (the same LDS-staged, bit-exact samples).  The
// 324-channel corr tile never leaves the CU: per lookup that saves writing and re-reading the
// B*C*Q*4-byte NCHW tensor (2 x 99.5 MB at DSEC B=16) and one launch.
//
// One workgroup = 32 consecutive queries of one batch item, 4 waves:
//   lookup  for each level: stage_level (lookup_stage.h) then blend the level's (2r+1)^2 samples
//           of every query into the LDS tile T[c][q] (c-major, 41.5 KB at C = 324);
//   GEMM    wave w computes output channels [64w, 64w + 64) x the 32 queries as two
//           v_mfma_f32_32x32x2_f32 tiles over K = C: A = W[o][c] fragments loaded per lane in
//           16-channel chunks (float4 register loads one chunk ahead; the 331 KB weight is shared
//           by every workgroup, so it streams from L2) -- from the packed weight (ecorr_conv1x1_pack:
//           fragment order, one contiguous 1-KB piece per wave load) or from the conv weight as
//           stored (64 rows' 16-byte pieces per load) -- B = T from LDS; bias + ReLU in the
//           epilogue, stores coalesced along the queries.
// The GEMM is MFMA-bound (2 * O * C flops per query), the lookup HBM-bound; 76 KB of LDS (the
// weight chunks alias the dead window stage) lets two workgroups share a CU so one's gather
// overlaps the other's MFMAs.
//
// Numerics: the samples are bit-exact; the channel sum is an exact c-ordered fmaf chain (fp32
// MFMA), then + bias, then ReLU (torch.relu semantics: NaN stays NaN) -- normwise agreement with
// the reference's conv (its reduction order belongs to MKL/MIOpen).

#include "ecorr_device.h"
#include "ecorr_internal.h"
#include "lookup_stage.h"

#include <algorithm>

namespace ecorr {

namespace {

constexpr int QBM = 32;    // queries per workgroup
constexpr int NTM = 256;   // threads
constexpr int OW = 64;     // output channels per wave
constexpr int OB = 4 * OW; // output channels per pass of the workgroup
constexpr int KC = 16;     // channels per weight chunk

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

// The weight in the GEMM's A-fragment order (pack_weight_kernel, ecorr_conv1x1_pack): for output
// block ob64 (64 channels = one wave's two 32x32 tiles), channel chunk kc (16 channels) and piece p
// (tile p >> 1, half p & 1), lane l holds W[64 ob64 + 32 (p >> 1) + (l & 31)][16 kc + 8 (l >> 5) +
// 4 (p & 1) + e], e = 0..3 (zeros past O or C), 16 bytes at ((ob64 nkc + kc) 4 + p) 1 KB + 16 l: each
// wave load is one contiguous 1-KB piece (8 whole lines) instead of 64 rows' 16-byte pieces.
__host__ __device__ constexpr int packed_chunks(int C) { return (C + KC - 1) / KC; }

__global__ __launch_bounds__(NTM) void pack_weight_kernel(const float* __restrict__ wt, int O, int C,
                                                          float* __restrict__ packed) {
    const int nkc = packed_chunks(C);
    const int64_t n = (int64_t)(O / OW) * nkc * 4 * 64;   // 16-byte pieces
    for (int64_t i = blockIdx.x * (int64_t)NTM + threadIdx.x; i < n; i += (int64_t)gridDim.x * NTM) {
        const int l = (int)(i & 63), p = (int)((i >> 6) & 3);
        const int64_t r = i >> 8;
        const int kc = (int)(r % nkc), ob = (int)(r / nkc);
        const int o = ob * OW + 32 * (p >> 1) + (l & 31);
        const int c = kc * KC + 8 * (l >> 5) + 4 * (p & 1);
        floatx4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = (o < O && c + e < C) ? wt[(int64_t)o * C + c + e] : 0.0f;
        reinterpret_cast<floatx4*>(packed)[i] = v;
    }
}

// PAIR (every level width even): windows staged as 8-byte column pairs (lookup_stage.h).
// PACKED: wt is the packed weight above; else the conv weight [O][C] as stored.
template <int R, bool PAIR, bool PACKED>
__global__ __launch_bounds__(NTM, 2) void lookup_conv_kernel(LookupParams P, const float* __restrict__ wt,
                                                             const float* __restrict__ bias, int O,
                                                             float* __restrict__ out) {
    using WS = WindowStage<R, QBM, PAIR>;
    constexpr int KK = WS::KK;
    constexpr int CPAD = ((4 * KK + KC - 1) / KC) * KC;   // levels <= 4; rows padded to whole chunks
    __shared__ struct {
        WS st;
    } u;
    // row stride QBM + 4: the GEMM's B reads (lanes 0-31 row r, lanes 32-63 row r + 8) land in
    // opposite bank halves; the lookup phase writes rows r and r + 8 from one wave for the same
    // reason (a wave's two 32-query halves take rows 8 apart, see below)
    constexpr int TS = QBM + 4;
    __shared__ __attribute__((aligned(16))) float T[CPAD][TS];

    const int tid = threadIdx.x, g = tid % QBM, part = tid / QBM, lane = tid & 63, wave = tid >> 6;
    const int half = part & 1;
    const int b = blockIdx.y;
    const int q0 = blockIdx.x * QBM;
    const int C = P.C;

    // ---- lookup: the block's corr tile, level by level, into T (rows >= C zero)
    for (int lv = 0; lv < P.levels; ++lv) {
        stage_level<R, QBM, NTM, PAIR>(u.st, P, lv, b, q0, tid);
        const int md = u.st.org[g][2] & 0xff;
        if (md == 0) {   // staged window: origin hoisted, no mode test per sample
            constexpr int K = WS::K, S = WS::SW;   // S: the staged row length
            const int o0 = u.st.org[g][0], o1 = u.st.org[g][1];
            const float* wq = u.st.win + WS::W0 + g * WS::SP;
            // rows of each 16-row block: wave w, half h takes w + 8h and w + 4 + 8h
            for (int k0 = 0; k0 < KK; k0 += 2 * NTM / QBM)
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const int k = k0 + wave + 4 * e + 8 * half;
                if (k >= KK) continue;
                const int a = k / K, bb = k - a * K;
                const float* c = wq + ((int)u.st.fy[g][bb] - o1) * S + ((int)u.st.fx[g][a] - o0);
                T[lv * KK + k][g] = blend(c[0], c[1], c[S], c[S + 1], u.st.wx[g][a], u.st.wy[g][bb]);
            }
        } else {
            for (int k0 = 0; k0 < KK; k0 += 2 * NTM / QBM)
                for (int e = 0; e < 2; ++e) {
                    const int k = k0 + wave + 4 * e + 8 * half;
                    if (k < KK) T[lv * KK + k][g] = md == 2 ? 0.0f : sample_level<R, QBM, PAIR>(u.st, P, lv, b, q0, g, k, md);
                }
        }
        __syncthreads();   // the stage is rebuilt by the next level / reused by the weight chunks
    }
    for (int i = C * QBM + tid; i < CPAD * QBM; i += NTM) T[i / QBM][i % QBM] = 0.0f;

    // ---- GEMM over the channels, no barrier inside: each lane streams its own weight row
    // W[o][c] (o = ob + lane&31, + 32 for the second tile) straight from L2 in float4 pieces, one
    // 16-channel chunk ahead.  MFMA k-step j of chunk c0 pairs channel c0 + j (lanes 0-31) with
    // c0 + 8 + j (lanes 32-63): A[o][k] = W[o][c0 + 8k + j], B[k][q] = T[c0 + 8k + j][q].  (This
    // sums the channels in a fixed permuted order -- still an exact fmaf chain per output.)
    const int kr = lane >> 5, col = lane & 31;
    const int nkc = CPAD / KC;
    const int pnkc = packed_chunks(C);   // PACKED: chunks of the packed weight (later ones read 0)
    __syncthreads();   // T complete
    const __amdgpu_buffer_rsrc_t wsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(wt), 0, PACKED ? (int)((int64_t)(O / OW) * pnkc * 4096) : (int)((int64_t)O * C * 4), 0x00020000);
    for (int oc = 0; oc < O; oc += OB) {
        const int ob = oc + wave * OW;   // this wave's first output channel
        // W row o starts at o * C floats; rows beyond O and channels beyond C read 0 (range check)
        const int r0 = (ob + col) * C, r1 = (ob + 32 + col) * C;
        floatx4 wc[4], wn[4];   // [tile][half]: tile i, channels c0 + 8 kr + 4 h .. +3
        auto load_w = [&](floatx4 (&w)[4], int c0) {
            if constexpr (PACKED) {   // one 1-KB piece per load; the block / chunk / piece offset is wave-uniform
                // chunks past the packed ones (rows of the padded tile beyond C) read 0: the
                // out-of-range offset goes in the voffset, which the range check covers
                const int kc = c0 / KC;
                const bool in = kc < pnkc;
                const int base = __builtin_amdgcn_readfirstlane(in ? (((ob / OW) * pnkc + kc) * 4) * 1024 : 0);
#pragma unroll
                for (int p = 0; p < 4; ++p)
                    w[p] = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(
                                                           wsrc, in ? lane * 16 : 0x7ffff000, base + p * 1024, 0));
                return;
            }
            const int c = c0 + 8 * kr;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int cc = c + 4 * h;
                // a piece straddling C is cut by zeroing the tail lanes below
                w[h] = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(wsrc, (r0 + cc) * 4, 0, 0));
                w[2 + h] = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(wsrc, (r1 + cc) * 4, 0, 0));
                if (cc + 4 > C) {
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (cc + e >= C) { w[h][e] = 0.0f; w[2 + h][e] = 0.0f; }
                }
            }
        };
        floatx16 acc0, acc1;
#pragma unroll
        for (int r = 0; r < 16; ++r) { acc0[r] = 0.0f; acc1[r] = 0.0f; }
        load_w(wc, 0);
#pragma unroll 1
        for (int kc = 0; kc < nkc; ++kc) {   // rolled (unrolled, even by two, it spills: 256 VGPRs + scratch)
            if (kc + 1 < nkc) load_w(wn, (kc + 1) * KC);
            float bq[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) bq[j] = T[kc * KC + 8 * kr + j][col];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(wc[j >> 2][j & 3], bq[j], acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(wc[2 + (j >> 2)][j & 3], bq[j], acc1, 0, 0, 0);
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) wc[i] = wn[i];
        }
        // ---- epilogue: D map col = lane&31 (query), row = (reg&3) + 8*(reg>>2) + 4*(lane>>5)
        const int q = q0 + col;
        if (q < P.q_count && ob < O) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int orow = (r & 3) + 8 * (r >> 2) + 4 * kr;
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const int o = ob + 32 * i + orow;
                    if (o < O) {
                        const float v = __fadd_rn(i == 0 ? acc0[r] : acc1[r], bias ? bias[o] : 0.0f);
                        out[((int64_t)b * O + o) * P.q_count + q] = v < 0.0f ? 0.0f : v;   // NaN stays NaN
                    }
                }
            }
        }
    }
}

}  // namespace

int64_t conv1x1_packed_floats(int O, int C) { return (int64_t)(O / OW) * packed_chunks(C) * 4 * 64 * 4; }

int launch_conv1x1_pack(const float* wt, int O, int C, float* packed, hipStream_t stream) {
    if (O <= 0 || O % OW != 0 || C <= 0) return ECORR_EINVAL;
    const int64_t n = conv1x1_packed_floats(O, C) / 4;
    const unsigned grid = (unsigned)std::min<int64_t>((n + NTM - 1) / NTM, 4096);
    hipLaunchKernelGGL(pack_weight_kernel, dim3(grid), dim3(NTM), 0, stream, wt, O, C, packed);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? ECORR_OK : ECORR_EHIP - (int)e;
}

int launch_lookup_conv(const LookupParams& P, int B, const float* wt, const float* bias, int O, float* out,
                       hipStream_t stream, bool packed) {
    if (P.radius != 4) return ECORR_ERADIUS;
    if (P.levels > 4) return ECORR_ELEVELS;
    if (O <= 0 || O % OW != 0) return ECORR_EINVAL;
    if (packed && conv1x1_packed_floats(O, P.C) * 4 >= 0x7fffffffLL) return ECORR_EINVAL;
    const dim3 grid((unsigned)((P.q_count + QBM - 1) / QBM), (unsigned)B), block(NTM);
    bool pair = true;   // column-pair staging: every level width even, 8-byte aligned levels
    for (int lv = 0; lv < P.levels; ++lv) pair &= P.lw[lv] % 2 == 0 && (uintptr_t)P.lvl[lv] % 8 == 0;
    if (packed) {
        if (pair) hipLaunchKernelGGL((lookup_conv_kernel<4, true, true>), grid, block, 0, stream, P, wt, bias, O, out);
        else hipLaunchKernelGGL((lookup_conv_kernel<4, false, true>), grid, block, 0, stream, P, wt, bias, O, out);
    } else {
        if (pair) hipLaunchKernelGGL((lookup_conv_kernel<4, true, false>), grid, block, 0, stream, P, wt, bias, O, out);
        else hipLaunchKernelGGL((lookup_conv_kernel<4, false, false>), grid, block, 0, stream, P, wt, bias, O, out);
    }
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? ECORR_OK : ECORR_EHIP - (int)e;
}

}  // namespace ecorr
