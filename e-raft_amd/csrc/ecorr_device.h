// ecorr_device.h -- device helpers shared by the build and lookup kernels (gfx950 only).
//
// Exactness contract: every helper below performs the reference's fp32 operations in the
// reference's order with explicit round-to-nearest intrinsics, so no -ffp-contract setting or
// compiler reassociation can change a bit.  The library is additionally compiled with
// -ffp-contract=off.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ecorr.h"

namespace ecorr {

constexpr int kWave = 64;

// Pyramid level storage (include/ecorr.h): each query's level image [h][w] is stored as
// row-major 4 x 8-float tiles (128 B = one L2 line); ntx = padded width / 8 tiles per tile row.
constexpr int kTileH = 4, kTileW = 8, kTile = kTileH * kTileW;
__host__ __device__ __forceinline__ int tiled_off(int y, int x, int ntx) {
    return (((y >> 2) * ntx + (x >> 3)) << 5) + ((y & 3) << 3) + (x & 7);
}
__host__ __device__ __forceinline__ int pad_h(int h) { return (h + kTileH - 1) & ~(kTileH - 1); }
__host__ __device__ __forceinline__ int pad_w(int w) { return (w + kTileW - 1) & ~(kTileW - 1); }

// Levels >= 4 (levels 2-3 are interleaved, below) whose tile padding would exceed half the image
// are stored compact row-major instead: the window covers most of such an image, so the padding
// would only add lines to every lookup's read footprint.
__host__ __device__ __forceinline__ bool level_compact(int level, int h, int w) {
    return level >= 2 && 2 * pad_h(h) * pad_w(w) > 3 * h * w;
}

// Offset of pixel (y, x) in one query image: tiled (ntx = tiles per tile row > 0) or row-major
// (ntx <= 0, width w).
__host__ __device__ __forceinline__ int level_off(int y, int x, int ntx, int w) {
    return ntx > 0 ? tiled_off(y, x, ntx) : y * w + x;
}

// Levels 1-3 are stored interleaved (ntx = -nbx < 0): query rows in groups of kGroup = 64, and a
// group holds, for each bh x bw block of the level image (2 x 4 at levels 1 and 2, 1 x 2 at level
// 3: what one 8 x 16 target block of level 0 pools to at levels 2 and 3), that block of its 64 rows
// back to back: [group][block][row][bh][bw], blocks row-major (nbx per block row).  One build tile
// then writes each block of its 256 query rows as whole lines (the per-row pieces are 32 / 8
// bytes), and the lookup reads a window's blocks with lines shared by adjacent queries.
constexpr int kGroup = ECORR_ROW_GROUP;
__host__ __device__ __forceinline__ int ilv_sy(int lv) { return lv == 3 ? 0 : 1; }   // log2 block height
__host__ __device__ __forceinline__ int ilv_sx(int lv) { return lv == 3 ? 1 : 2; }   // log2 block width

// Float offset of pixel (y, x) of query row R (0 .. B*q_count - 1) from the level's base, any
// format; sz = floats per query image (an interleaved group spans kGroup * sz floats).
__host__ __device__ __forceinline__ int64_t pix_off(int64_t R, int y, int x, int lv, int ntx, int w, int64_t sz) {
    if (ntx >= 0) return R * sz + level_off(y, x, ntx, w);
    const int sy = ilv_sy(lv), sx = ilv_sx(lv);
    return (R >> 6) * (kGroup * sz) +
           ((int64_t)((y >> sy) * -ntx + (x >> sx)) * kGroup + (R & (kGroup - 1))) * (1 << (sy + sx)) +
           ((y & ((1 << sy) - 1)) << sx) + (x & ((1 << sx) - 1));
}

// model/utils.py:11-12 then ATen grid_sampler unnormalize (align_corners=True):
//   g  = RN(RN(2x / (size-1)) - 1)
//   ix = RN(RN(g + 1) * ((size-1)/2))
// 2x and (size-1)/2 are exact; the division is IEEE (v_div_scale/fmas/fixup sequence).
__device__ __forceinline__ float unnormalize(float x, float size_m1, float half_size_m1) {
    const float g = __fsub_rn(__fdiv_rn(__fmul_rn(2.0f, x), size_m1), 1.0f);
    return __fmul_rn(__fadd_rn(g, 1.0f), half_size_m1);
}

// Bilinear blend exactly as ATen's AVX512 grid_sampler (nw product, then FMA chain).
// w = x-frac, n = y-frac; out-of-image corners must already be 0.
__device__ __forceinline__ float blend(float vnw, float vne, float vsw, float vse, float w, float n) {
    const float e = __fsub_rn(1.0f, w);
    const float s = __fsub_rn(1.0f, n);
    float acc = __fmul_rn(vnw, __fmul_rn(s, e));
    acc = __builtin_fmaf(vne, __fmul_rn(s, w), acc);
    acc = __builtin_fmaf(vsw, __fmul_rn(n, e), acc);
    acc = __builtin_fmaf(vse, __fmul_rn(n, w), acc);
    return acc;
}

// Zeros-padding corner fetch by float coordinates (float compare: NaN and +-huge read 0, exactly
// as ATen's int32-converted masks do).  Used by the generic / fallback paths only.
// ntx <= 0: row-major image (bilinear_sampler, compact levels); otherwise a tiled pyramid level.
__device__ __forceinline__ float corner(const float* __restrict__ img, int h, int w, float fx, float fy,
                                        int ntx = 0) {
    const bool in = (fx >= 0.0f) & (fx < (float)w) & (fy >= 0.0f) & (fy < (float)h);
    if (!in) return 0.0f;
    const int y = (int)fy, x = (int)fx;
    return img[ntx <= 0 ? (int64_t)y * w + x : (int64_t)tiled_off(y, x, ntx)];
}

// The same corner fetch from pyramid level lv (base lvbase, any format) for query row R.
__device__ __forceinline__ float level_corner(const float* __restrict__ lvbase, int64_t R, int lv, int ntx, int h,
                                              int w, int64_t sz, float fx, float fy) {
    const bool in = (fx >= 0.0f) & (fx < (float)w) & (fy >= 0.0f) & (fy < (float)h);
    if (!in) return 0.0f;
    return lvbase[pix_off(R, (int)fy, (int)fx, lv, ntx, w, sz)];
}

// One bilinear sample of img[h][w] at pixel coordinates (x, y) (model/utils.py:7-21).
__device__ __forceinline__ float sample_px(const float* __restrict__ img, int h, int w, float x, float y,
                                           int ntx = 0) {
    const float ix = unnormalize(x, (float)(w - 1), (float)(w - 1) * 0.5f);
    const float iy = unnormalize(y, (float)(h - 1), (float)(h - 1) * 0.5f);
    const float x0 = floorf(ix), y0 = floorf(iy);
    const float wx = __fsub_rn(ix, x0), wy = __fsub_rn(iy, y0);
    const float x1 = __fadd_rn(x0, 1.0f), y1 = __fadd_rn(y0, 1.0f);
    return blend(corner(img, h, w, x0, y0, ntx), corner(img, h, w, x1, y0, ntx),
                 corner(img, h, w, x0, y1, ntx), corner(img, h, w, x1, y1, ntx), wx, wy);
}

// sample_px on query row R of pyramid level lv (any format).
__device__ __forceinline__ float sample_level_px(const float* __restrict__ lvbase, int64_t R, int lv, int ntx, int h,
                                                 int w, int64_t sz, float x, float y) {
    const float ix = unnormalize(x, (float)(w - 1), (float)(w - 1) * 0.5f);
    const float iy = unnormalize(y, (float)(h - 1), (float)(h - 1) * 0.5f);
    const float x0 = floorf(ix), y0 = floorf(iy);
    const float wx = __fsub_rn(ix, x0), wy = __fsub_rn(iy, y0);
    const float x1 = __fadd_rn(x0, 1.0f), y1 = __fadd_rn(y0, 1.0f);
    return blend(level_corner(lvbase, R, lv, ntx, h, w, sz, x0, y0), level_corner(lvbase, R, lv, ntx, h, w, sz, x1, y0),
                 level_corner(lvbase, R, lv, ntx, h, w, sz, x0, y1), level_corner(lvbase, R, lv, ntx, h, w, sz, x1, y1),
                 wx, wy);
}

}  // namespace ecorr
