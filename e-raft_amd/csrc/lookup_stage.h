// lookup_stage.h -- the per-level window staging shared by the lookup kernel (lookup.hip) and the
// fused lookup + convc1 kernel (motion.hip).  Device code only, gfx950.
//
// For a group of QB consecutive queries of one batch item and one pyramid level (NTQ threads,
// NTQ / QB threads per query):
//   stage_level()   phase 0: the 2(2r+1) coordinate chains per query -- x chains depend on the
//                   x-offset a only, y chains on the y-offset b only (corr.py:41-43), each the
//                   reference's exact fp32 sequence (utils.py:11-12 + ATen's unnormalize) -> floor
//                   and fraction into LDS;
//                   phase 1: each query's (2r+3)^2 window (one slack row/column absorbs the +-1
//                   floor flips of the normalize/unnormalize round trip) staged into LDS with raw
//                   buffer loads whose range check implements grid_sample's zero padding;
//   sample_level()  phase 2: output channel k = a(2r+1) + b of query g, blended from LDS in
//                   ATen's order; coordinates that do not fit the window (NaN/inf/huge) take an
//                   exact direct-gather path.
#pragma once
#include "ecorr_device.h"
#include "ecorr_internal.h"

typedef unsigned uint2v __attribute__((ext_vector_type(2)));

namespace ecorr {

// The staged windows of QB queries and their origins (all phase 1 needs).  PAIR: the window is
// loaded as 8-byte column pairs from the even column at or left of the origin (every level width
// even) and written into LDS shifted by that one column, so the LDS image starts at the true
// origin column in both modes: phase 2's offset of sample a from the origin is a (+ a floor flip)
// for every query, and lanes = queries at the odd stride SP hit distinct banks.  (Unshifted, the
// even rounding made the offsets a or a + 1 at random across lanes: 49% of the LDS cycles were
// bank conflicts.)  The half of a pair that falls outside the S-slot row (the shifted-out column
// of an odd origin, or column S of an even one; never read) goes to the dummy slot at the end of win[],
// so rows hold S slots: 31.7 KB at r = 4, five workgroups per CU (S + 1 slots: 34.8 KB, four;
// round 3 A/B 41.7 / 45.4 / 41.3 vs 41.9 / 45.8 / 42.8 us on the smooth / sigma-3 / sigma-40 fields).
template <int R, int QB, bool PAIR = false>
struct WindowBuf {
    static constexpr int K = 2 * R + 1;   // samples per axis
    static constexpr int KK = K * K;
    static constexpr int S = 2 * R + 3;   // staged window side (rows)
    static constexpr int SW = S;          // staged row length
    static constexpr int SP = (S * SW) | 1;   // odd per-query stride: conflict-free lanes = queries
    static constexpr int W0 = PAIR ? 1 : 0;   // query g's window starts at win[W0 + g SP] (PAIR: the
                                              // first item's base W0 - 1 stays >= 0, "no item" < 0)
    static constexpr int DUMMY = W0 + QB * SP;   // the never-read slot of out-of-row pair halves
    float win[W0 + QB * SP + 1];
    // per query: window origin x, y and (mode | needed cols << 8 | needed rows << 16), where mode
    // 0 = staged, 1 = direct gather (coordinates that do not fit the window), 2 = past the range.
    int org[QB][3];
};

// ... plus the per-query coordinate chains in LDS (kernels whose threads share them).
template <int R, int QB, bool PAIR = false>
struct WindowStage : WindowBuf<R, QB, PAIR> {
    static constexpr int K = 2 * R + 1;
    float fx[QB][K], wx[QB][K], fy[QB][K], wy[QB][K];
};

// One coordinate chain (corr.py:41-43, utils.py:11-12, grid_sampler unnormalize): sample o of the
// axis whose scaled coordinate is cs = coords / 2^lv, on a level side of m1 + 1 pixels.
template <int R>
__device__ __forceinline__ void coord_chain(float cs, int o, float m1, float& f, float& wgt) {
    const float c = __fadd_rn(cs, (float)(o - R));
    const float v = unnormalize(c, m1, m1 * 0.5f);
    f = floorf(v);
    wgt = __fsub_rn(v, f);
}

// Phase 0b for one query from its first / last x and y floors: origin and mode word (WindowBuf::org).
template <int S, bool PAIR = false>
__device__ __forceinline__ void window_origin(bool valid, float x0, float xl, float y0, float yl, int org[3]) {
    int md = 2, X0 = 0, Y0 = 0, NX = 0, NY = 0;
    if (valid) {
        bool ok = fabsf(x0) < 1.0e7f && fabsf(y0) < 1.0e7f;  // false for NaN / inf / huge
        // every step of the chain (exact-or-rounded add of the offset, the normalize /
        // unnormalize roundings by positive factors, floor) is monotone, so the floors are
        // non-decreasing in the offset and the end points bound the whole window
        const float dx = xl - x0, dy = yl - y0;   // exact: integers < 2^24
        ok &= (dx >= 0.0f) & (dx <= (float)(S - 2)) & (dy >= 0.0f) & (dy <= (float)(S - 2));
        md = ok ? 0 : 1;
        X0 = ok ? (int)x0 : 0;
        Y0 = ok ? (int)y0 : 0;
        // corners span [x0, floor(ix_last) + 1]: monotone round trip, so the last sample bounds it
        NX = ok ? (int)dx + 2 : 0;
        NY = ok ? (int)dy + 2 : 0;
    }
    org[0] = X0;
    org[1] = Y0;
    org[2] = md | (NX << 8) | (NY << 16);
}

template <int R, int QB, int NTQ, bool PAIR = false>
__device__ __forceinline__ void stage_windows(WindowBuf<R, QB, PAIR>& st, const LookupParams& P, int lv, int b,
                                              int q0, int tid);

// Phases 0 and 1 for level lv of queries [q0, q0 + QB) of batch item b; ends with a barrier.
template <int R, int QB, int NTQ, bool PAIR = false>
__device__ __forceinline__ void stage_level(WindowStage<R, QB, PAIR>& st, const LookupParams& P, int lv, int b,
                                            int q0, int tid) {
    using WS = WindowStage<R, QB, PAIR>;
    constexpr int K = WS::K, S = WS::S;
    constexpr int TPQ = NTQ / QB;   // threads per query
    const int g = tid % QB, part = tid / QB;
    const int h = P.lh[lv], w = P.lw[lv];
    const int p = q0 + g;
    const bool valid = p < P.q_count;
    const int64_t Q = P.q_count;   // coords slab stride

    // ---- phase 0: coordinate chains (corr.py:41-43, utils.py:11-12, grid_sampler unnormalize)
    if (valid) {
        const float inv = 1.0f / (float)(1 << lv);  // coords / 2**i is an exact scaling
        const float cx = __fmul_rn(P.coords[((int64_t)b * 2 + 0) * Q + p], inv);
        const float cy = __fmul_rn(P.coords[((int64_t)b * 2 + 1) * Q + p], inv);
        const float wm1 = (float)(w - 1), hm1 = (float)(h - 1);
#pragma unroll
        for (int j = part; j < 2 * K; j += TPQ) {
            const bool isx = j < K;
            const int o = isx ? j : j - K;
            float f, wgt;
            coord_chain<R>(isx ? cx : cy, o, isx ? wm1 : hm1, f, wgt);
            if (isx) { st.fx[g][o] = f; st.wx[g][o] = wgt; }
            else     { st.fy[g][o] = f; st.wy[g][o] = wgt; }
        }
    }
    __syncthreads();

    // ---- phase 0b: window origin and fast/slow decision per query
    if (part == 0) window_origin<S, PAIR>(valid, st.fx[g][0], st.fx[g][K - 1], st.fy[g][0], st.fy[g][K - 1], st.org[g]);
    __syncthreads();
    stage_windows<R, QB, NTQ, PAIR>(st, P, lv, b, q0, tid);
}

// Phase 1's loads in flight: this thread's work items (window columns or column pairs, each S rows)
// and their LDS destinations (-1: no item).
template <int R, int QB, int NTQ, bool PAIR>
struct StageRegs {
    static constexpr int S = 2 * R + 3, V = PAIR ? 2 : 1;
    static constexpr int NPX = (WindowBuf<R, QB, PAIR>::SW + V - 1) / V;   // work items per query
    static constexpr int ITEMS = QB * NPX;
    static constexpr int NCOL = (ITEMS + NTQ - 1) / NTQ;
    float vals[NCOL][S][V];
    int dst[NCOL];
    int skip[NCOL];   // PAIR: the half (0 or 1) of the item that lies outside the row, else -1
};

// Phase 1, first half: issue this thread's window loads for level lv of queries [q0, q0 + QB) of
// batch item b (origins from st.org) into registers; stage_commit() writes them to st.win.
template <int R, int QB, int NTQ, bool PAIR>
__device__ __forceinline__ void stage_issue(const WindowBuf<R, QB, PAIR>& st, const LookupParams& P, int lv, int b,
                                            int q0, int tid, StageRegs<R, QB, NTQ, PAIR>& sr);

// Phase 1, second half: the staged values into the LDS windows (no barrier).
template <int R, int QB, int NTQ, bool PAIR>
__device__ __forceinline__ void stage_commit(WindowBuf<R, QB, PAIR>& st, const StageRegs<R, QB, NTQ, PAIR>& sr) {
    using SR = StageRegs<R, QB, NTQ, PAIR>;
    constexpr int SW = WindowBuf<R, QB, PAIR>::SW, DUMMY = WindowBuf<R, QB, PAIR>::DUMMY;
#pragma unroll
    for (int c = 0; c < SR::NCOL; ++c)
        if (sr.dst[c] >= 0)
#pragma unroll
            for (int ry = 0; ry < SR::S; ++ry)
#pragma unroll
                for (int v = 0; v < SR::V; ++v)
                    st.win[sr.skip[c] == v ? DUMMY : sr.dst[c] + ry * SW + v] = sr.vals[c][ry][v];
}

// Phase 1 for level lv of queries [q0, q0 + QB) of batch item b, from st.org; ends with a barrier.
template <int R, int QB, int NTQ, bool PAIR>
__device__ __forceinline__ void stage_windows(WindowBuf<R, QB, PAIR>& st, const LookupParams& P, int lv, int b,
                                              int q0, int tid) {
    StageRegs<R, QB, NTQ, PAIR> sr;
    stage_issue<R, QB, NTQ, PAIR>(st, P, lv, b, q0, tid, sr);
    stage_commit<R, QB, NTQ, PAIR>(st, sr);
    __syncthreads();
}

template <int R, int QB, int NTQ, bool PAIR>
__device__ __forceinline__ void stage_issue(const WindowBuf<R, QB, PAIR>& st, const LookupParams& P, int lv, int b,
                                            int q0, int tid, StageRegs<R, QB, NTQ, PAIR>& sr) {
    using WS = WindowBuf<R, QB, PAIR>;
    constexpr int S = WS::S, SP = WS::SP;
    constexpr int V = PAIR ? 2 : 1;   // window columns per work item (PAIR: one 8-byte load)
    const int h = P.lh[lv], w = P.lw[lv], ntx = P.lntx[lv];
    const int64_t hw = P.lsz[lv];  // floats per query image
    const int64_t R0 = (int64_t)b * P.q_count + q0;   // first query row of the group
    // interleaved levels (ntx < 0, ecorr_device.h): the slab starts at the 64-row group of R0
    const int64_t g0 = R0 >> 6;
    const float* __restrict__ lvbase = P.lvl[lv] + (ntx < 0 ? g0 * kGroup * hw : R0 * hw);

    // ---- phase 1: stage windows, zeros outside the image (grid_sample padding_mode='zeros').
    // Work item = (query, window column or, PAIR, column pair from the even column xe at or left
    // of the origin); each item walks the S rows.  A pair never straddles the image edge (even
    // start, even width) and its two floats are adjacent in every layout (tile rows of 8, block
    // rows of 4 or 2, image rows); it lands at LDS slots rx - odd, rx - odd + 1 of the row (odd =
    // origin - xe), so the image starts at the origin.  Loads are raw buffer loads
    // over this group's slab of the level: an element outside the image gets an out-of-range
    // offset and the hardware range check returns 0 -- zero padding with no branch and no select,
    // so all NCOL*S loads of a thread issue back to back.
    using SR = StageRegs<R, QB, NTQ, PAIR>;
    constexpr int NPX = SR::NPX, ITEMS = SR::ITEMS, NCOL = SR::NCOL;
    const int nq = min(QB, P.q_count - q0);
    const int64_t span = ntx < 0 ? (((R0 + nq - 1) >> 6) - g0 + 1) * kGroup * hw : nq * hw;
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(lvbase), 0, (int)(span * 4), 0x00020000);
    // row walk down a window column: in-block steps and block-row wraps (tiled: 4 x 8 tiles;
    // interleaved: bh x bw blocks; compact: every step is a wrap of one image row)
    const bool tiled = ntx > 0, ilv = ntx < 0;
    const int sy = ilv ? ilv_sy(lv) : 2, sx = ilv ? ilv_sx(lv) : 3;
    const int ymask = tiled || ilv ? (1 << sy) - 1 : 0;
    const int step_in = 4 << sx;
    const int step_wrap = tiled ? 128 * ntx - 96 : ilv ? 4 * (-ntx * kGroup * (1 << (sy + sx)) - ymask * (1 << sx)) : 4 * w;
    constexpr int OOB = 0x7ffffff0;   // beyond any slab: reads as 0
    auto& vals = sr.vals;
    auto& dst = sr.dst;
#pragma unroll
    for (int c = 0; c < NCOL; ++c) {
        const int it = tid + c * NTQ;
        const bool live = it < ITEMS;
        const int gq = live ? it / NPX : 0;
        const int rx = (it - gq * NPX) * V;
        const int xo = st.org[gq][0], y0 = st.org[gq][1], info = st.org[gq][2];
        const int odd = PAIR ? xo & 1 : 0;   // xo may be negative: & 1 / - odd round toward -inf
        const int x = xo - odd + rx;
        const int ny = (info >> 16) & 0xff;
        // only the needed corner rectangle touches memory; the slack row/column reads 0 for free
        const bool colin = live && (info & 0xff) == 0 && rx < ((info >> 8) & 0xff) + odd && (unsigned)x < (unsigned)w;
        dst[c] = live ? WS::W0 + gq * SP + rx - odd : -1;
        sr.skip[c] = PAIR && odd && rx == 0 ? 0 : PAIR && !odd && rx == S - 1 ? 1 : -1;
        // rows ry in [rlo, rhi) are needed and inside the image; the column's byte offset walks
        // down the rows incrementally (tiled: +8 floats inside a tile, + one tile row minus 24 from
        // in-tile row 3; interleaved likewise per block; compact: +w) instead of re-deriving the
        // offset per row (y0 may be negative: the shift / mask decomposition stays consistent)
        const int rlo = max(0, -y0), rhi = colin ? max(rlo, min(ny, h - y0)) : rlo;   // rhi >= rlo
        int off;
        if (tiled) {
            off = (int)(gq * hw) * 4 + ((((y0 >> 2) * ntx + (x >> 3)) << 5) + ((y0 & 3) << 3) + (x & 7)) * 4;
        } else if (ilv) {
            const int64_t Rq = R0 + gq;
            off = (int)((((Rq >> 6) - g0) * kGroup * hw +
                         ((int64_t)((y0 >> sy) * -ntx + (x >> sx)) * kGroup + (Rq & (kGroup - 1))) * (1 << (sy + sx)) +
                         ((y0 & ymask) << sx) + (x & ((1 << sx) - 1))) * 4);
        } else {
            off = (int)(gq * hw) * 4 + (y0 * w + x) * 4;
        }
        int ym = y0 & ymask;
#pragma unroll
        for (int ry = 0; ry < S; ++ry) {
            const bool need = (unsigned)(ry - rlo) < (unsigned)(rhi - rlo);
            if constexpr (PAIR) {
                const uint2v u = __builtin_amdgcn_raw_buffer_load_b64(rsrc, need ? off : OOB, 0, 0);
                vals[c][ry][0] = __uint_as_float(u.x);
                vals[c][ry][1] = __uint_as_float(u.y);
            } else {
            vals[c][ry][0] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsrc, need ? off : OOB, 0, 0));
            }
            off += ym == ymask ? step_wrap : step_in;
            ym = (ym + 1) & ymask;
        }
    }
}

// Exact direct gather of one sample of query p (slab index) from its floors and weights, for
// coordinates that do not fit the window (NaN / inf / huge: corner() range-checks in float).
__device__ __forceinline__ float sample_direct(const LookupParams& P, int lv, int b, int p, float xa, float yb,
                                               float wa, float nb) {
    const int h = P.lh[lv], w = P.lw[lv], ntx = P.lntx[lv];
    const int64_t Rq = (int64_t)b * P.q_count + p, sz = P.lsz[lv];
    const float* base = P.lvl[lv];
    const float xa1 = __fadd_rn(xa, 1.0f), yb1 = __fadd_rn(yb, 1.0f);
    return blend(level_corner(base, Rq, lv, ntx, h, w, sz, xa, yb), level_corner(base, Rq, lv, ntx, h, w, sz, xa1, yb),
                 level_corner(base, Rq, lv, ntx, h, w, sz, xa, yb1), level_corner(base, Rq, lv, ntx, h, w, sz, xa1, yb1),
                 wa, nb);
}

// Phase 2: sample k = a(2r+1) + b of query g (staged mode md = 0 or direct mode md = 1).
template <int R, int QB, bool PAIR = false>
__device__ __forceinline__ float sample_level(const WindowStage<R, QB, PAIR>& st, const LookupParams& P, int lv,
                                              int b, int q0, int g, int k, int md) {
    using WS = WindowStage<R, QB, PAIR>;
    constexpr int K = WS::K, S = WS::SW, SP = WS::SP;   // S: the staged row length
    const int a = k / K, bb = k - a * K;
    const float xa = st.fx[g][a], yb = st.fy[g][bb];
    const float wa = st.wx[g][a], nb = st.wy[g][bb];
    if (md == 0) {
        const float* c = st.win + WS::W0 + g * SP + ((int)yb - st.org[g][1]) * S + ((int)xa - st.org[g][0]);
        return blend(c[0], c[1], c[S], c[S + 1], wa, nb);
    }
    return sample_direct(P, lv, b, q0 + g, xa, yb, wa, nb);
}

}  // namespace ecorr
