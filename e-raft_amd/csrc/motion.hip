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

// ============================================================================================
// Warp-specialized persistent form (round 4): one workgroup of 8 waves per CU walks the 32-query
// tiles.  Waves 0-3 (producers) run the lookup of tile k + 1 into one of two LDS corr tiles while
// waves 4-7 (consumers) run the convc1 GEMM of tile k from the other -- the gather and the MFMAs
// of a CU overlap by construction instead of by two workgroups drifting out of step (the
// two-workgroup kernel above keeps the phases in step: lookup 30 us + GEMM 145 us per launch at
// DSEC B=16).  One barrier per tile; nothing else is shared between the roles.
//
// A producer wave owns 8 queries of the tile and stages, samples and writes their 4 x 81 corr
// rows with no barrier of its own: lane (query qi = lane / 8, part = lane % 8) computes its
// query's window end-point chains and origin in registers, stages its share of the query's
// window (column pairs part + 8 j of the 11 x 6 (row, pair) items) into a wave-private LDS window
// and samples outputs k = part + 8 m.  The levels are software-pipelined: level l + 1's staging
// loads are issued before level l is committed and sampled (two register sets, two windows).
// The samples are the lookup's (same chains, staging and blend: bit-exact); the GEMM is the
// kernel above's (same channel order per output), so the result is bitwise that kernel's.
// Needs every level width even (column pairs), 4 levels, the packed weight.
// ============================================================================================
constexpr int WS_NT = 512;                  // 4 producer + 4 consumer waves
constexpr int WS_QP = 8;                    // queries per producer wave
constexpr int WS_L = 4;                     // levels
constexpr int WS_KK = 81;                   // (2r + 1)^2, r = 4
constexpr int WS_CPAD = 336;                // 324 corr rows padded to 21 chunks of 16
constexpr int WS_TS = QBM + 4;              // corr tile row stride (floats), as above
constexpr int WS_S = 11;                    // staged window side (2r + 3)
constexpr int WS_SP = WS_S * WS_S;          // per-query stride (odd)
constexpr int WS_WIN = 1 + WS_QP * WS_SP + 1;   // W0 = 1, 8 windows, the dummy slot
constexpr int WS_DUMMY = WS_WIN - 1;
constexpr int WS_NJ = 9;                    // staging items per lane: part + 8 j < 66
static_assert(WS_SP % 2 == 1 && 8 * WS_NJ >= WS_S * 6, "window geometry");

struct WsLds {
    float T[2][WS_CPAD][WS_TS];             // the two corr tiles (rows >= 324 stay zero)
    float win[4][2][WS_WIN];                // per producer wave, two levels in flight
    float ch[4][WS_L][WS_QP][4][9];         // per producer wave and level: fx, wx, fy, wy
};

__global__ __launch_bounds__(WS_NT, 1) void lookup_conv_ws_kernel(LookupParams P, const float* __restrict__ wt,
                                                                  const float* __restrict__ bias, int O,
                                                                  float* __restrict__ out, int nqt, int ntiles) {
    __shared__ WsLds sh;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int C = P.C;
    const int G = (int)gridDim.x;

    // rows C .. WS_CPAD - 1 of both corr tiles stay zero for the whole launch (the padded chunks)
    for (int i = tid; i < 2 * (WS_CPAD - C) * WS_TS; i += WS_NT) {
        const int bb = i / ((WS_CPAD - C) * WS_TS), r = i - bb * ((WS_CPAD - C) * WS_TS);
        sh.T[bb][C + r / WS_TS][r % WS_TS] = 0.0f;
    }

    // ======================= producers: the lookup of one tile, wave-private =======================
    const int pw = wave & 3, qi = lane >> 3, part = lane & 7;
    const int gq = WS_QP * pw + qi;   // this lane's query in the tile
    float cxr = 0.0f, cyr = 0.0f;     // its raw coordinates in the tile being produced next
    auto load_coords = [&](int t) __attribute__((always_inline)) {
        cxr = cyr = 0.0f;
        if (t < ntiles) {
            const int b = t / nqt, p = (t - b * nqt) * QBM + gq;
            if (p < P.q_count) {
                cxr = P.coords[((int64_t)b * 2 + 0) * P.q_count + p];
                cyr = P.coords[((int64_t)b * 2 + 1) * P.q_count + p];
            }
        }
    };
    auto produce = [&](int t, int buf) __attribute__((always_inline)) {
        const int b = t / nqt, q0t = (t - b * nqt) * QBM;
        const int p = q0t + gq;
        const bool valid = p < P.q_count;
        const float cxq = cxr, cyq = cyr;
        load_coords(t + G);   // the next tile's, in flight during this one
        const int64_t R0 = (int64_t)b * P.q_count + q0t;   // the tile's first query row
        const int64_t g0 = R0 >> 6;
        const int nq = min(QBM, P.q_count - q0t);
        const int64_t Rq = R0 + gq;
        float vals[WS_L][WS_NJ][2];
        int org[WS_L][3];
        // level lv into register set s: chains (this lane's part) into LDS, origin, staging loads
        auto issue = [&](int lv, int s) __attribute__((always_inline)) {
            const float inv = 1.0f / (float)(1 << lv);   // coords / 2**i: exact
            const float cx = __fmul_rn(cxq, inv), cy = __fmul_rn(cyq, inv);
            const int h = P.lh[lv], w = P.lw[lv], ntx = P.lntx[lv];
            const float wm1 = (float)(w - 1), hm1 = (float)(h - 1);
            float fx0 = 0.0f, fx8 = 0.0f, fy0 = 0.0f, fy8 = 0.0f;
            float* ch = &sh.ch[pw][lv][qi][0][0];
            if (valid) {
                float f, wg, wx8, wy8, dummy;
                coord_chain<4>(cx, part, wm1, f, wg);
                ch[0 * 9 + part] = f;
                ch[1 * 9 + part] = wg;
                coord_chain<4>(cy, part, hm1, f, wg);
                ch[2 * 9 + part] = f;
                ch[3 * 9 + part] = wg;
                coord_chain<4>(cx, 0, wm1, fx0, dummy);
                coord_chain<4>(cy, 0, hm1, fy0, dummy);
                coord_chain<4>(cx, 8, wm1, fx8, wx8);
                coord_chain<4>(cy, 8, hm1, fy8, wy8);
                if (part == 0) {
                    ch[0 * 9 + 8] = fx8;
                    ch[1 * 9 + 8] = wx8;
                    ch[2 * 9 + 8] = fy8;
                    ch[3 * 9 + 8] = wy8;
                }
            }
            window_origin<WS_S, true>(valid, fx0, fx8, fy0, fy8, org[s]);
            const int xo = org[s][0], y0 = org[s][1], info = org[s][2];
            const int md = info & 0xff, nx = (info >> 8) & 0xff, ny = (info >> 16) & 0xff;
            const int odd = xo & 1;   // xo may be negative: & 1 and - odd round toward -inf
            const int64_t hw = P.lsz[lv];
            const bool tiled = ntx > 0, ilv = ntx < 0;
            const float* lvbase = P.lvl[lv] + (ilv ? g0 * kGroup * hw : R0 * hw);
            const int64_t span = ilv ? (((R0 + nq - 1) >> 6) - g0 + 1) * kGroup * hw : nq * hw;
            const __amdgpu_buffer_rsrc_t rsrc =
                __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(lvbase), 0, (int)(span * 4), 0x00020000);
            const int sy = ilv ? ilv_sy(lv) : 2, sx = ilv ? ilv_sx(lv) : 3;
            const int rlo = max(0, -y0);
            const int rhi = md == 0 ? max(rlo, min(ny, h - y0)) : rlo;
#pragma unroll
            for (int j = 0; j < WS_NJ; ++j) {
                const int idx = part + 8 * j;          // item (row, column pair) of this lane's query
                const int row = idx / 6, pr = idx - 6 * row;
                const bool item = idx < WS_S * 6;
                const int x = xo - odd + 2 * pr, y = y0 + row;
                const bool need = item && md == 0 && 2 * pr < nx + odd && (unsigned)x < (unsigned)w &&
                                  (unsigned)(row - rlo) < (unsigned)(rhi - rlo);
                int off;
                if (tiled) {
                    off = (int)(gq * hw) * 4 + ((((y >> 2) * ntx + (x >> 3)) << 5) + ((y & 3) << 3) + (x & 7)) * 4;
                } else if (ilv) {
                    off = (int)((((Rq >> 6) - g0) * kGroup * hw +
                                 ((int64_t)((y >> sy) * -ntx + (x >> sx)) * kGroup + (Rq & (kGroup - 1))) * (1 << (sy + sx)) +
                                 ((y & ((1 << sy) - 1)) << sx) + (x & ((1 << sx) - 1))) * 4);
                } else {
                    off = (int)(gq * hw) * 4 + (y * w + x) * 4;
                }
                // out-of-image, not-needed and non-items read 0 (the range check): zero padding
                const uint2v u = __builtin_amdgcn_raw_buffer_load_b64(rsrc, need ? off : 0x7ffffff0, 0, 0);
                vals[s][j][0] = __uint_as_float(u.x);
                vals[s][j][1] = __uint_as_float(u.y);
            }
        };
        // level lv from set s: commit into window s (this wave's), then sample into corr rows
        auto finish = [&](int lv, int s) __attribute__((always_inline)) {
            float* win = sh.win[pw][lv & 1];
            const int odd = org[s][0] & 1;
#pragma unroll
            for (int j = 0; j < WS_NJ; ++j) {
                const int idx = part + 8 * j;
                if (idx >= WS_S * 6) continue;
                const int row = idx / 6, pr = idx - 6 * row;
                // pair (2 pr - odd, + 1) of row `row`; the half outside the S-slot row -> dummy slot
                const int d = 1 + qi * WS_SP + row * WS_S + 2 * pr - odd;
                const int skip = odd && pr == 0 ? 0 : !odd && 2 * pr == WS_S - 1 ? 1 : -1;
#pragma unroll
                for (int v = 0; v < 2; ++v) win[skip == v ? WS_DUMMY : d + v] = vals[s][j][v];
            }
            // (a wave's LDS accesses are processed in order: the reads below see the writes above)
            const float* ch = &sh.ch[pw][lv][qi][0][0];
            const int md = org[s][2] & 0xff;
            const float* wq = win + 1 + qi * WS_SP;
            float* trow = &sh.T[buf][lv * WS_KK][gq];
            if (md == 0) {   // staged window
#pragma unroll
                for (int m = 0; m < 11; ++m) {
                    const int k = part + 8 * m;
                    if (k >= WS_KK) break;
                    const int a = k / 9, bb = k - 9 * a;
                    const float xa = ch[0 * 9 + a], wa = ch[1 * 9 + a], yb = ch[2 * 9 + bb], nb = ch[3 * 9 + bb];
                    const float* c = wq + ((int)yb - org[s][1]) * WS_S + ((int)xa - org[s][0]);
                    trow[k * WS_TS] = blend(c[0], c[1], c[WS_S], c[WS_S + 1], wa, nb);
                }
            } else {   // coordinates that do not fit the window: exact direct gather; past the range: 0
#pragma unroll 1
                for (int k = part; k < WS_KK; k += 8) {
                    const int a = k / 9, bb = k - 9 * a;
                    trow[k * WS_TS] = md == 1 ? sample_direct(P, lv, b, p, ch[0 * 9 + a], ch[2 * 9 + bb], ch[1 * 9 + a],
                                                              ch[3 * 9 + bb])
                                              : 0.0f;
                }
            }
        };
        // all four levels' staging loads in flight at once (one memory latency per tile; a lone
        // producer wave per SIMD exposed two to three in a row), then commit and sample level by
        // level through two windows
        issue(0, 0);
        issue(1, 1);
        issue(2, 2);
        issue(3, 3);
        finish(0, 0);
        finish(1, 1);
        finish(2, 2);
        finish(3, 3);
    };

    // ======================= consumers: the convc1 GEMM of one tile =======================
    const int cw = wave & 3, kr = lane >> 5, col = lane & 31;
    const int nkc = WS_CPAD / KC, pnkc = packed_chunks(C);
    const __amdgpu_buffer_rsrc_t wsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(wt), 0, (int)((int64_t)(O / OW) * pnkc * 4096), 0x00020000);
    auto consume = [&](int t, int buf) __attribute__((always_inline)) {
        const int b = t / nqt, q0t = (t - b * nqt) * QBM;
        for (int oc = 0; oc < O; oc += OB) {
            const int ob = oc + cw * OW;
            auto load_w = [&](floatx4 (&w)[4], int kc) __attribute__((always_inline)) {
                const bool in = kc < pnkc;
                const int base = __builtin_amdgcn_readfirstlane(in ? (((ob / OW) * pnkc + kc) * 4) * 1024 : 0);
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    w[q] = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(
                                                           wsrc, in ? lane * 16 : 0x7ffff000, base + q * 1024, 0));
            };
            floatx16 acc0, acc1;
#pragma unroll
            for (int r = 0; r < 16; ++r) { acc0[r] = 0.0f; acc1[r] = 0.0f; }
            // one consumer wave per SIMD: the weight two chunks ahead (three register sets) and the
            // corr-tile operand one chunk ahead hide the L2 and LDS latencies a lone wave exposes
            floatx4 w3[3][4];
            float bq[2][8];
            auto load_b = [&](float (&bb)[8], int kc) __attribute__((always_inline)) {
#pragma unroll
                for (int j = 0; j < 8; ++j) bb[j] = sh.T[buf][kc * KC + 8 * kr + j][col];
            };
            auto chunk = [&](const floatx4 (&w)[4], const float (&bb)[8]) __attribute__((always_inline)) {
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(w[j >> 2][j & 3], bb[j], acc0, 0, 0, 0);
                    acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(w[2 + (j >> 2)][j & 3], bb[j], acc1, 0, 0, 0);
                }
            };
            static_assert(WS_CPAD / KC % 3 == 0, "chunks in threes");
            load_w(w3[0], 0);
            load_w(w3[1], 1);
            load_b(bq[0], 0);
#pragma unroll 1
            for (int kc = 0; kc < nkc; kc += 3) {
                load_w(w3[2], kc + 2);
                load_b(bq[1], kc + 1);
                chunk(w3[0], bq[0]);
                if (kc + 3 < nkc) load_w(w3[0], kc + 3);
                load_b(bq[0], kc + 2);
                chunk(w3[1], bq[1]);
                if (kc + 4 < nkc) load_w(w3[1], kc + 4);
                if (kc + 3 < nkc) load_b(bq[1], kc + 3);
                chunk(w3[2], bq[0]);
                if (kc + 3 < nkc) {
#pragma unroll
                    for (int j = 0; j < 8; ++j) bq[0][j] = bq[1][j];
                }
            }
            const int q = q0t + col;
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
    };

    // ======================= the tile pipeline: one barrier per tile =======================
    // step k: the producers make tile k (buffer k & 1) while the consumers use tile k - 1
    const int t0 = (int)blockIdx.x;
    if (wave < 4) load_coords(t0);
    for (int k = 0; t0 + (k - 1) * G < ntiles; ++k) {
        const int t = t0 + k * G;
        if (wave < 4) {
            if (t < ntiles) produce(t, k & 1);
        } else if (k > 0) {
            consume(t - G, (k - 1) & 1);
        }
        __syncthreads();   // the buffers swap roles
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

// the warp-specialized persistent kernel for the packed weight at 4 levels with even widths (every
// BASELINE config); the two-workgroup kernel otherwise
constexpr bool kConvWS = true;

// compute units of the current device (cached per device ordinal; 256 on MI355X)
int device_cus() {
    static int cache[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    int n = __atomic_load_n(&cache[dev], __ATOMIC_RELAXED);
    if (n == 0) {
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
        __atomic_store_n(&cache[dev], n, __ATOMIC_RELAXED);
    }
    return n;
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
    if (kConvWS && packed && pair && P.levels == WS_L) {
        const int nqt = (P.q_count + QBM - 1) / QBM;
        const int64_t ntiles = (int64_t)nqt * B;
        if (ntiles > 0x7fffffff) return ECORR_EINVAL;
        const int g = (int)std::min<int64_t>(ntiles, device_cus());
        hipLaunchKernelGGL(lookup_conv_ws_kernel, dim3(g), dim3(WS_NT), 0, stream, P, wt, bias, O, out, nqt,
                           (int)ntiles);
        const hipError_t e = hipGetLastError();
        return e == hipSuccess ? ECORR_OK : ECORR_EHIP - (int)e;
    }
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
