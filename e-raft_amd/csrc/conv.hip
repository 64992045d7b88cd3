// conv.hip -- SURVEY §8f row 1, two-launch form: relu(convc1(corr)) (update.py:67,74:
// cor = F.relu(self.convc1(corr))) on the lookup's NCHW output, as a split-f16 MFMA GEMM:
//
//   out[b][o][p] = relu(bias[o] + sum_c W[o][c] * corr[b][c][p])
//
// The fused kernels (motion.hip) keep the 324-channel tile in LDS but pay for it in occupancy: their
// gather runs on 4 waves per CU where the standalone lookup keeps 15 in flight, and the fp32 MFMA GEMM
// is 16x slower per flop than f16.  Here the lookup writes corr (99.5 MB at DSEC B=16) and this kernel
// reads it back, with the f16 matrix cores doing the channel sum:
//
//   split arithmetic (as the build, build.hip pack_body): every query column p of corr is scaled by
//   2^e_p (its largest |value| over the C channels in [2^14, 2^15)), every weight row o by 2^e_o, and
//   each scaled value x is split into hi = f16(x), lo = f16(x - hi) (exact subtraction), so
//   x = hi + lo + O(2^-22 |x|); each product is lo.hi + hi.lo + hi.hi on v_mfma_f32_32x32x16_f16
//   with fp32 accumulation, scaled back by 2^-(e_o + e_p) (v_ldexp, exact), then + bias, ReLU.
//   Normwise within 1e-5 of an fp64 conv (tests/test_conv_split_gpu.py); NaN propagates to the
//   query's outputs as in the reference; a +-inf corr or weight value gives NaN (inf - inf in the
//   split), where the reference's fp32 conv can give +-inf -- the build's split mode has the same
//   deviation, and the split build never produces inf samples.
//
// Workgroup = 64 queries x 256 output channels, 4 waves: wave w owns query block qb = w & 1 (32
// queries: the MFMA's N) and channel half oh = w >> 1 (4 x 32 channels: M), 4 accumulator tiles.
//   maxima    per query the max |corr| over C -> e_p: from the lookup's partial maxima
//             (ecorr_lookup_qmax), else a pre-pass (each wave half of the chunks, combined in LDS);
//   K loop    per 16-channel chunk: the weight chunk (16 KB, the A fragments of all 8 channel
//             blocks, hi and lo, pre-split and laid out in fragment order by ecorr_conv1x1_split_pack)
//             goes global -> LDS by LDS-DMA two chunks ahead, three buffers, one barrier per chunk;
//             the B fragment (lane = query, 8 consecutive channels) is loaded from corr as 8 dwords
//             PD chunks ahead, split in registers; 4 x 3 MFMAs per wave.
// Work: 2*O*C flop per query (12.7 GFLOP at DSEC B=16) as 3 f16 MFMAs per product; bytes: corr in
// (C*4 per query; twice without the partial maxima) + out (O*4 per query, non-temporal stores).

#include "ecorr_device.h"
#include "ecorr_internal.h"

#include <algorithm>

namespace ecorr {

namespace {

typedef _Float16 halfx8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef unsigned int uintx4 __attribute__((ext_vector_type(4)));

constexpr int SQ = 64;                 // queries per workgroup
constexpr int SO = 256;                // output channels per workgroup (8 row blocks of 32)
constexpr int SNT = 256;               // threads (4 waves)
constexpr int SKC = 16;                // channels per chunk (one v_mfma_f32_32x32x16_f16 K)
constexpr int SCHUNK = 8 * 2 * 64 * 16;   // bytes per packed weight chunk: [row block][hi | lo][lane][16 B]

__host__ __device__ constexpr int split_chunks(int C) { return (C + SKC - 1) / SKC; }
__host__ __device__ constexpr int split_oblocks(int O) { return (O + SO - 1) / SO; }

__device__ __forceinline__ float pow2(int e) { return __int_as_float((e + 127) << 23); }

// e such that m 2^e lies in [2^14, 2^15); 0 for a zero or non-finite maximum (build.hip pack_body)
__device__ __forceinline__ int split_exponent(float m) {
    int E = 0;
    frexpf(m, &E);
    const int e = (m > 0.f && m <= 3.4028235e38f) ? 15 - E : 0;
    return e < -126 ? -126 : (e > 126 ? 126 : e);
}

__device__ __forceinline__ void split8(const float (&v)[8], float s, halfx8& hi, halfx8& lo) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const float x = v[j] * s;
        const _Float16 h = (_Float16)x;
        hi[j] = h;
        lo[j] = (_Float16)(x - (float)h);
    }
}

// Packed weight: for output block ob (256 channels) and chunk c, 16 KB at (ob nkc + c) SCHUNK:
// [row block rb][hi | lo][lane l][8 halves] = W[256 ob + 32 rb + (l & 31)][16 c + 8 (l >> 5) + j]
// scaled by 2^e_o and split (zeros past O or C) -- the v_mfma_f32_32x32x16_f16 A fragment of lane l;
// then the int exponents e_o of all nob * 256 rows.  One workgroup per output block.  perm_levels:
// K = presplit_positions(levels) positions, position 16 c + 8 (l >> 5) + j holding channel
// presplit_chan(position) (the presplit corr order; zeros where that is -1).
__global__ __launch_bounds__(SNT) void split_pack_kernel(const float* __restrict__ wt, int O, int C,
                                                         char* __restrict__ packed, int perm_levels) {
    __shared__ float sc[SO];
    const int K = perm_levels ? presplit_positions(perm_levels) : C;   // K positions (C: the row length)
    const int ob = blockIdx.x, nob = gridDim.x, nkc = split_chunks(K), t = threadIdx.x;
    const int o = ob * SO + t;
    float m = 0.f;
    if (o < O)
        for (int k = 0; k < C; ++k) m = fmaxf(m, fabsf(wt[(int64_t)o * C + k]));
    const int e = split_exponent(m);
    sc[t] = pow2(e);
    reinterpret_cast<int*>(packed + (int64_t)nob * nkc * SCHUNK)[o] = e;
    __syncthreads();
    char* base = packed + (int64_t)ob * nkc * SCHUNK;
    for (int i = t; i < nkc * (SCHUNK / 16); i += SNT) {
        const int l = i & 63, part = (i >> 6) & 1, rb = (i >> 7) & 7, c = i >> 10;
        const int r = rb * 32 + (l & 31), oo = ob * SO + r, k0 = c * SKC + 8 * (l >> 5);
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int ch = perm_levels ? presplit_chan(k0 + j, perm_levels) : (k0 + j < C ? k0 + j : -1);
            v[j] = (oo < O && ch >= 0) ? wt[(int64_t)oo * C + ch] : 0.f;
        }
        halfx8 hi, lo;
        split8(v, sc[r], hi, lo);
        *reinterpret_cast<halfx8*>(base + (int64_t)i * 16) = part ? lo : hi;
    }
}

// s_waitcnt vmcnt(N) only (gfx9 encoding: vmcnt bits 3:0 and 15:14; expcnt, lgkmcnt not waited)
template <int N>
__device__ __forceinline__ void wait_vm() {
    static_assert(N >= 0 && N < 64, "vmcnt field");
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// The weight chunks go global -> LDS by LDS-DMA (no staging registers; through registers it was
// 63.9 vs 53.9 us, profiles/r04_lab/r4l_ab_conv.txt), three buffers, two chunks ahead, with static
// vmcnt waits (tests/test_isa_waits.py replays them on the emitted ISA); the query columns are
// loaded PD chunks ahead into PD + 1 fixed register sets.
// PRE: `in` is the presplit corr (ecorr_lookup_presplit): the B fragment of chunk c is two 16-byte
// loads (hi, lo of group 2 c + kh) instead of 8 dword loads and the split, and the query exponent
// comes from `scale` (qmax unused); the weight columns are packed in the presplit order.
template <int PD, bool PRE = false>
__global__ __launch_bounds__(SNT) void conv1x1_split_kernel(const float* __restrict__ in, int C, int Q,
                                                            const float* __restrict__ qmax, int G,
                                                            const char* __restrict__ packed,
                                                            const float* __restrict__ bias, int O,
                                                            float* __restrict__ out,
                                                            const int* __restrict__ scale) {
    constexpr int NB = 3;
    // ALL LDS in one object: with a second __shared__ object hipcc waits vmcnt(0) before every
    // ds_read while an LDS-DMA is in flight (cdna_hip_programming.md, the second-__shared__ trap)
    struct Lds {
        char wbuf[NB][SCHUNK];   // weight chunks
        float red[2][SQ];        // per-query maxima of the two channel halves
        int sex[SO];             // the block's weight-row exponents
        float sbias[SO];         // and biases (0 past O or without bias)
    };
    __shared__ __attribute__((aligned(16))) Lds sh;
    auto& wbuf = sh.wbuf;
    auto& red = sh.red;
    auto& sex = sh.sex;
    auto& sbias = sh.sbias;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, qb = w & 1, oh = w >> 1;
    const int ob = blockIdx.y, b = blockIdx.z, nob = gridDim.y, nkc = split_chunks(C);
    const int qi = 32 * qb + (lane & 31), q = blockIdx.x * SQ + qi, kh = lane >> 5;
    const bool qok = q < Q;
    // corr / out of batch item b as range-checked buffers: a lane past Q starts at the end of the
    // range (every access then reads 0 / is dropped), channels past C or O fall outside by
    // themselves -- no branches around the loads and stores
    const int qs = Q * 4;
    // presplit (C = K positions): groups from ceil(K / 8) on lie past the range (zeros); a lane past Q
    // starts past it
    const int prange = PRE ? (C + 7) / 8 * 2 * Q * 16 : 0;
    const __amdgpu_buffer_rsrc_t csrc = PRE
        ? __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(reinterpret_cast<const char*>(in)) +
                                                (int64_t)b * presplit_bytes_per_item(C, Q), 0, prange, 0x00020000)
        : __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(in + (int64_t)b * C * Q), 0, C * Q * 4, 0x00020000);
    const int cbase = PRE ? (qok ? q * 16 : prange) + kh * 2 * Q * 16 : (qok ? q : C * Q) * 4;
    const char* wsrc = packed + (int64_t)ob * nkc * SCHUNK;

    // B fragment of chunk c: corr[b][16 c + 8 kh + j][q], j = 0..7 (zeros past C or Q); presplit:
    // v[0..3] = the hi halves, v[4..7] = the lo halves of group 2 c + kh (chunk offset in soffset)
    auto load_b = [&](int c, float (&v)[8]) __attribute__((always_inline)) {
        if constexpr (PRE) {
            typedef unsigned int u4 __attribute__((ext_vector_type(4)));
            const u4 h = __builtin_amdgcn_raw_buffer_load_b128(csrc, cbase, c * 4 * Q * 16, 0);
            const u4 l = __builtin_amdgcn_raw_buffer_load_b128(csrc, cbase + Q * 16, c * 4 * Q * 16, 0);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                v[j] = __uint_as_float(h[j]);
                v[4 + j] = __uint_as_float(l[j]);
            }
        } else {
            const int off = cbase + (c * SKC + 8 * kh) * qs;
#pragma unroll
            for (int j = 0; j < 8; ++j)
                v[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(csrc, off + j * qs, 0, 0));
        }
    };

    // wave w copies the chunk's 1-KB pieces w, w + 4, w + 8, w + 12 (lane-linear, as LDS-DMA writes
    // them), the chunk offset in the scalar soffset
    const __amdgpu_buffer_rsrc_t wrs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(wsrc), 0, nkc * SCHUNK, 0x00020000);
    auto issue_w = [&](int c, int buf) __attribute__((always_inline)) {
#pragma unroll
        for (int s = 0; s < 4; ++s)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                wrs, (__attribute__((address_space(3))) void*)(wbuf[buf] + (w + 4 * s) * 1024), 16,
                (w + 4 * s) * 1024 + lane * 16, c * SCHUNK, 0, 0);
    };

    // ---- prologue: every load in flight before the first wait (one memory latency, not five):
    // chunks 0-1's weights, chunks 0 .. PD-1's query columns, this block's row exponents and biases,
    // the query's partial maxima
    float bv[PD + 1][8];   // B values of chunks c .. c + PD (fixed register sets: no copies)
    issue_w(0, 0);
    issue_w(nkc > 1 ? 1 : 0, 1);
#pragma unroll
    for (int k = 0; k < PD; ++k) load_b(k, bv[k]);   // past C: out of range, zeros
    // (bias and maxima through range-checked buffers: a null pointer is a 0-byte range reading 0 --
    // no branches, whose merged wait states cost a full drain here)
    const int eo_t = reinterpret_cast<const int*>(packed + (int64_t)nob * nkc * SCHUNK)[ob * SO + tid];
    const __amdgpu_buffer_rsrc_t brs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(bias), 0, bias ? O * 4 : 0, 0x00020000);
    const float bo_t = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(brs, (ob * SO + tid) * 4, 0, 0));
    constexpr int QG = PRE ? 1 : 6;   // partial maxima per wave and pass (G = 12 for 4 levels: one pass)
    const __amdgpu_buffer_rsrc_t qrs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(qmax ? qmax + (int64_t)b * G * Q : nullptr), 0, qmax ? G * Q * 4 : 0, 0x00020000);
    const int qc = min(q, Q - 1);
    float qv[QG];
    int eq = 0;
    if constexpr (PRE) {   // used only by the epilogue: no wait for it here
        eq = scale[(int64_t)b * Q + qc];
    } else {
#pragma unroll
        for (int i = 0; i < QG; ++i)
            qv[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(qrs, (min(oh + 2 * i, G - 1) * Q + qc) * 4, 0, 0));
    }
    __builtin_amdgcn_sched_barrier(0);
    sex[tid] = eo_t;
    sbias[tid] = bo_t;

    // ---- the query's largest |value| over C -> its exponent: from the lookup's partial maxima
    // (ecorr_lookup_qmax; clamped repeats are harmless) or a pre-pass over the column
    float m = 0.f;
    if constexpr (PRE) {
    } else if (qmax) {
#pragma unroll
        for (int i = 0; i < QG; ++i) m = fmaxf(m, qv[i]);
        for (int g = oh + 2 * QG; g < G; g += 2)
            m = fmaxf(m, __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(qrs, (g * Q + qc) * 4, 0, 0)));
        m = qok ? m : 0.f;
    } else
#pragma unroll 1
    for (int c = oh; c < nkc; c += 8) {   // 4 chunks' loads in flight at once (clamped repeats past C)
        float v[4][8];
#pragma unroll
        for (int k = 0; k < 4; ++k) load_b(min(c + 2 * k, nkc - 1), v[k]);
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf(v[k][j]));
    }
    if constexpr (!PRE) {
        m = fmaxf(m, __shfl_xor(m, 32));
        if (kh == 0) red[oh][qi] = m;
    }
    __builtin_amdgcn_sched_barrier(0);
    // chunk 0's pieces (chunk 1's 4 and the PD chunks' B loads may be in flight; presplit: and the
    // exponent load, issued last)
    if constexpr (PRE) wait_vm<4 + 2 * PD + 1>();
    else wait_vm<4 + 8 * PD>();
    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): red / sex / sbias written
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (!PRE) eq = split_exponent(fmaxf(red[0][qi], red[1][qi]));
    const float sq = pow2(eq);

    floatx16 acc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;

    // ---- K loop, step c: chunk c's weights in wbuf[c % 3] (published by the barrier before),
    // chunk c + 2's DMA into wbuf[(c + 2) % 3] (chunk c - 1's, whose readers passed that barrier);
    // chunk c's B values in set cur, chunk c + PD's loads into set nxt (chunk c - 1's, consumed).
    // tail: a remainder step after the loop, whose query-column loads are dead (nothing reads that
    // register set again) and dropped by the compiler -- its wait must not count on them
    auto step = [&](int c, float (&cur)[8], float (&nxt)[8], bool tail) __attribute__((always_inline)) {
        load_b(c + PD, nxt);   // unconditional (past C reads zeros): no branch for the waits to merge over
        issue_w(min(c + 2, nkc - 1), (c + 2) % NB);   // past the last chunk a harmless repeat
        __builtin_amdgcn_sched_barrier(0);   // issued here, ahead of this chunk's work
        halfx8 bh, bl;
        if constexpr (PRE) {
            typedef unsigned int u4 __attribute__((ext_vector_type(4)));
            bh = __builtin_bit_cast(halfx8, u4{__float_as_uint(cur[0]), __float_as_uint(cur[1]), __float_as_uint(cur[2]),
                                               __float_as_uint(cur[3])});
            bl = __builtin_bit_cast(halfx8, u4{__float_as_uint(cur[4]), __float_as_uint(cur[5]), __float_as_uint(cur[6]),
                                               __float_as_uint(cur[7])});
        } else {
            split8(cur, sq, bh, bl);
        }
        const char* wb = wbuf[c % NB] + lane * 16;
        // A fragments double-buffered: tile i + 2's pair is read right after tile i's MFMAs issue, so
        // the LDS latency hides behind them (read just before use: 55.5 vs 52.0 us at DSEC B = 16,
        // profiles/r05_lab/cv_ab_adb.txt)
        halfx8 ah[2], al[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            ah[i] = *reinterpret_cast<const halfx8*>(wb + ((4 * oh + i) * 2 + 0) * 1024);
            al[i] = *reinterpret_cast<const halfx8*>(wb + ((4 * oh + i) * 2 + 1) * 1024);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int s = i & 1;
            acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[s], bl, acc[i], 0, 0, 0);
            acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[s], bh, acc[i], 0, 0, 0);
            acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[s], bh, acc[i], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
            if (i + 2 < 4) {
                ah[s] = *reinterpret_cast<const halfx8*>(wb + ((4 * oh + i + 2) * 2 + 0) * 1024);
                al[s] = *reinterpret_cast<const halfx8*>(wb + ((4 * oh + i + 2) * 2 + 1) * 1024);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        // chunk c + 1's pieces landed (only this step's 8 B loads + 4 pieces may be newer) and this
        // wave's reads of chunk c are done (the next step's DMA overwrites it); a bare s_barrier:
        // __syncthreads()'s release fence would wait for every load in flight (vmcnt(0))
        __builtin_amdgcn_sched_barrier(0);
        if (tail)
            wait_vm<4>();   // (stricter than needed if the loads were kept: still correct)
        else if constexpr (PRE)
            wait_vm<6>();
        else
            wait_vm<12>();
        __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };
    int c = 0;
#pragma unroll 1
    for (; c + PD + 1 <= nkc; c += PD + 1) {
#pragma unroll
        for (int k = 0; k <= PD; ++k) step(c + k, bv[k], bv[(k + PD) % (PD + 1)], false);
    }
#pragma unroll
    for (int k = 0; k < PD; ++k)
        if (c + k < nkc) step(c + k, bv[k], bv[(k + PD) % (PD + 1)], true);

    // ---- epilogue: lane holds query q, channels 32 rb + 8 (r >> 2) + 4 kh + (r & 3)
    const __amdgpu_buffer_rsrc_t osrc = __builtin_amdgcn_make_buffer_rsrc(out + (int64_t)b * O * Q, 0, O * Q * 4,
                                                                          0x00020000);
    const int obase = (qok ? q : O * Q) * 4;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int ol = 32 * (4 * oh + i) + 8 * g + 4 * kh;   // 4 consecutive channels r & 3
            const int4 eo = *reinterpret_cast<const int4*>(&sex[ol]);
            const float4 bo = *reinterpret_cast<const float4*>(&sbias[ol]);
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                float v = ldexpf(acc[i][4 * g + t], -(eo[t] + eq));
                v = v + bo[t];   // a missing bias is 0 (v + 0 = v for every v but -0, which ReLU maps to 0)
                v = v < 0.f ? 0.f : v;   // torch.relu: NaN stays NaN
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), osrc, obase + (ob * SO + ol + t) * qs, 0,
                                                      2);   // nt: 52.2 vs 53.9 us (r4l_ab_conv.txt)
            }
        }
}

constexpr int kConvPD = 2;   // query-column prefetch distance (chunks)

}  // namespace

int64_t conv1x1_split_bytes(int O, int C) {
    return (int64_t)split_oblocks(O) * split_chunks(C) * SCHUNK + (int64_t)split_oblocks(O) * SO * 4;
}

int64_t conv1x1_presplit_bytes(int O, int levels) { return conv1x1_split_bytes(O, presplit_positions(levels)); }

int launch_conv1x1_split_pack(const float* wt, int O, int C, void* packed, hipStream_t stream, int perm_levels) {
    if (O <= 0 || C <= 0 || split_oblocks(O) > 65535) return ECORR_EINVAL;
    if (perm_levels && (perm_levels < 1 || perm_levels > 4 || C != 81 * perm_levels)) return ECORR_EINVAL;
    hipLaunchKernelGGL(split_pack_kernel, dim3(split_oblocks(O)), dim3(SNT), 0, stream, wt, O, C, (char*)packed,
                       perm_levels);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? ECORR_OK : ECORR_EHIP - (int)e;
}

int launch_conv1x1_relu_split(const float* in, int B, int C, int Q, const float* qmax, int G, const void* packed,
                              const float* bias, int O, float* out, hipStream_t stream) {
    if (qmax && (G <= 0 || (int64_t)G * Q * 4 >= 0x7fffffffLL)) return ECORR_EINVAL;
    if (B <= 0 || C <= 0 || Q <= 0 || O <= 0 || B > 65535 || split_oblocks(O) > 65535) return ECORR_EINVAL;
    // 32-bit buffer offsets: a lane past Q reads from C*Q on, the prefetch reaches 3 chunks past C; the stores
    // likewise from O*Q up to the output block's last row
    if ((int64_t)(2 * C + 4 * SKC) * Q * 4 >= 0x7fffffffLL ||
        (int64_t)(O + split_oblocks(O) * SO) * Q * 4 >= 0x7fffffffLL)
        return ECORR_EINVAL;
    if ((const void*)in == (const void*)out) return ECORR_EINVAL;
    const dim3 grid((unsigned)((Q + SQ - 1) / SQ), (unsigned)split_oblocks(O), (unsigned)B);
    hipLaunchKernelGGL((conv1x1_split_kernel<kConvPD, false>), grid, dim3(SNT), 0, stream, in, C, Q, qmax, G,
                       (const char*)packed, bias, O, out, nullptr);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? ECORR_OK : ECORR_EHIP - (int)e;
}

int launch_conv1x1_relu_presplit(const void* in, int B, int levels, int Q, const int* scale, const void* packed,
                                 const float* bias, int O, float* out, hipStream_t stream) {
    const int C = presplit_positions(levels);   // the kernel's K: positions, zeros included
    if (B <= 0 || C <= 0 || Q <= 0 || O <= 0 || B > 65535 || split_oblocks(O) > 65535 || !scale) return ECORR_EINVAL;
    // 32-bit buffer offsets: a lane past Q reads from the range's end on, up to PD + 1 chunks past C
    if (presplit_bytes_per_item(C, Q) + (int64_t)(kConvPD + 2) * 4 * Q * 16 >= 0x7fffffffLL ||
        (int64_t)(O + split_oblocks(O) * SO) * Q * 4 >= 0x7fffffffLL)
        return ECORR_EINVAL;
    if ((const void*)in == (const void*)out) return ECORR_EINVAL;
    const dim3 grid((unsigned)((Q + SQ - 1) / SQ), (unsigned)split_oblocks(O), (unsigned)B);
    hipLaunchKernelGGL((conv1x1_split_kernel<kConvPD, true>), grid, dim3(SNT), 0, stream, (const float*)in, C, Q,
                       nullptr, 0, (const char*)packed, bias, O, out, scale);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? ECORR_OK : ECORR_EHIP - (int)e;
}

}  // namespace ecorr
