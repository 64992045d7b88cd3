// ecorr_internal.h -- host-side launch interfaces between abi.hip and the kernel files.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ecorr.h"

namespace ecorr {

// Pyramid storage geometry (include/ecorr.h), computed once by pyramid_geometry() (abi.hip) and
// shared by the build and the lookup.
struct PyrGeom {
    int levels;
    int h[ECORR_MAX_LEVELS], w[ECORR_MAX_LEVELS];   // true level sizes
    int ntx[ECORR_MAX_LEVELS];                       // tiles per tile row; 0 = compact row-major
    int nty[ECORR_MAX_LEVELS];                       // tile rows (compact: image rows)
    int64_t sz[ECORR_MAX_LEVELS];                    // floats per query image
    int64_t off[ECORR_MAX_LEVELS + 1];               // float offset of each level; off[levels] = total
};

int pyramid_geometry(int64_t rows, int H, int W, int levels, PyrGeom* g);

struct BuildParams {
    const float* f1;
    const float* f2;
    int D, H, W;
    int q_count;        // query pixels in the fmap1 slab
    float scale;        // sqrt(D) (divide) or 1/sqrt(D) when sqrt(D) is a power of two (multiply)
    int scale_is_mul;
    int scale_shift;    // scale_is_mul: 1/sqrt(D) = 2^-scale_shift
    // split mode (ecorr_build_split): per-pixel power-of-two exponents of fmap1 ([B][q_count]) and
    // fmap2 ([B][H*W]) written by the exponent pass; null = the fp32-MFMA fmaf-chain build
    char* ws;           // split workspace (build_split_workspace_bytes), null = fp32 build
    int* ex1;
    int* ex2;
    const char* pk1;    // f16 hi/lo operand panels of fmap1 / fmap2 (pack_both_kernel)
    const char* pk2;
    // filled by launch_build
    int n_mt;           // 128-query tiles (fp32 blocks; fmap1 panels)
    int n_qt;           // 256-query tiles (split blocks)
    int n_nt, n_ntx;    // n-tiles (target blocks); regular n-tiles per tile row
    int n_reg, band_y0;  // regular (8 x 16) n-tiles per m-tile; first row of the 4-row band tiles
    int fused_levels;   // levels written by the GEMM epilogue (<= 4)
    float* lvl[4];
    int lh[4], lw[4];
    int lntx[4], lnty[4];   // tiles per tile row (0 = compact row-major) / tile rows of each fused level
    int64_t lsz[4];         // floats per query image of each fused level
};

// stages (split build only; the fp32 build is one launch): 1 = operand pass, 2 = GEMM + fused
// pyramid (+ levels > 4), 3 = both
int launch_build(const BuildParams& P, int B, const PyrGeom& g, float* pyramid, hipStream_t stream, int stages = 3);
int64_t build_split_workspace_bytes(int B, int D, int H, int W, int q_count);

struct LookupParams {
    const float* coords;  // [B][2][q_count]
    float* out;           // [B][C][q_count]
    int H, W;
    int q_count;
    int levels, radius;
    int C;                // levels * (2r+1)^2
    const float* lvl[ECORR_MAX_LEVELS];
    int lh[ECORR_MAX_LEVELS], lw[ECORR_MAX_LEVELS];
    int lntx[ECORR_MAX_LEVELS];      // tiles per tile row (0 = compact row-major)
    int lsz[ECORR_MAX_LEVELS];       // floats per query image
    float* qmax;          // null, or [B][3 * levels][q_count]: per-query partial maxima of |out|
                          // (ecorr_lookup_qmax: the split convc1's column exponents)
    const int* scale;     // non-null: ecorr_lookup_presplit, out is the presplit layout and
                          // scale[b][q] the query's column exponent (launch_split_column_scale)
};

int launch_lookup(const LookupParams& P, int B, hipStream_t stream);

int launch_lookup_conv(const LookupParams& P, int B, const float* wt, const float* bias, int O, float* out,
                       hipStream_t stream, bool packed);
int64_t conv1x1_packed_floats(int O, int C);
int launch_conv1x1_pack(const float* wt, int O, int C, float* packed, hipStream_t stream);
// conv.hip: split-f16 1x1 conv + ReLU on an NCHW tensor (ecorr_conv1x1_relu_split)
int64_t conv1x1_split_bytes(int O, int C);
// perm_levels > 0: the weight columns in the presplit channel order of that many radius-4 levels
int launch_conv1x1_split_pack(const float* wt, int O, int C, void* packed, hipStream_t stream, int perm_levels = 0);
// the presplit pack's byte count (its K = presplit_positions(levels))
int64_t conv1x1_presplit_bytes(int O, int levels);
int launch_conv1x1_relu_split(const float* in, int B, int C, int Q, const float* qmax, int G, const void* packed,
                              const float* bias, int O, float* out, hipStream_t stream);

// Presplit corr (ecorr_lookup_presplit -> ecorr_conv1x1_relu_presplit), radius 4, L <= 4 levels,
// C = 81 L channels at K = 88 L positions.  Channel ch = 81 lv + 27 part + k (lookup_cols_reg: wave
// `part` owns the 27 channels 9 ai + bb, k < 27) sits at K position
//   72 lv + 24 part + k               for k < 24 (three whole 8-channel groups of one wave)
//   72 L + 16 lv + 3 part + (k - 24)  for k >= 24 (the level's 9 last channels, 2 groups per level:
//                                      positions 9 .. 15 of them are zeros)
// so every group is written whole by one wave (the leftovers through LDS, by waves 0 and 1 of the
// level's workgroup): 2-byte stores shared between waves cost the lookup 7.5 us per call
// (profiles/r06_lab/ab_presplit_stores.json).  The conv's weight columns are permuted the same way
// (the channel sum is order-free up to rounding).  Layout per batch item: [group g][hi | lo][query]
// [8 halves], 16 B per (g, hi|lo, query), presplit_groups(K) groups (even: whole 16-channel K
// chunks); groups from 11 L on are never written (the conv reads them out of range: zeros).
__host__ __device__ inline int presplit_positions(int L) { return 88 * L; }
__host__ __device__ inline int presplit_groups(int K) { return 2 * ((K + 15) / 16); }
__host__ __device__ inline int presplit_pos(int ch, int L) {
    const int lv = ch / 81, r = ch - 81 * lv, part = r / 27, k = r - 27 * part;
    return k < 24 ? 72 * lv + 24 * part + k : 72 * L + 16 * lv + 3 * part + (k - 24);
}
__host__ __device__ inline int presplit_chan(int pos, int L) {   // inverse; -1 for a zero position
    if (pos < 72 * L) {
        const int lv = pos / 72, r = pos - 72 * lv, part = r / 24;
        return 81 * lv + 27 * part + (r - 24 * part);
    }
    const int j = pos - 72 * L, lv = j / 16, r = j - 16 * lv;
    if (lv >= L || r >= 9) return -1;
    const int part = r / 3;
    return 81 * lv + 27 * part + 24 + (r - 3 * part);
}
// bytes of one batch item's presplit corr at K positions
__host__ __device__ inline int64_t presplit_bytes_per_item(int K, int Q) { return (int64_t)presplit_groups(K) * 2 * Q * 16; }
int launch_conv1x1_relu_presplit(const void* in, int B, int levels, int Q, const int* scale, const void* packed,
                                 const float* bias, int O, float* out, hipStream_t stream);
// scale[b][q] (+ B trailing scratch entries): the presplit column exponents from the fmaps (lookup.hip)
int launch_split_column_scale(const float* f1, const float* f2, int B, int D, int H, int W, int* scale,
                              hipStream_t stream);

int launch_bilinear_sampler(const float* img, int N, int C, int h, int w, const float* coords,
                            int Hg, int Wg, float* out, float* mask, hipStream_t stream);

int launch_coords_grid(int B, int H, int W, float* out, hipStream_t stream);

// rows.hip: [world][chunk] all-gathered row chunks -> [B][C][H][W] (include/ecorr.h)
int launch_rows_assemble(const float* chunks, int64_t chunk, int world, int B, int C, int H, int W, float* out,
                         hipStream_t stream);

int launch_upsample_flow(const float* flow, const float* mask, int N, int H, int W, float* out, hipStream_t stream);
int launch_png16_encode(const float* flow, int B, int h, int w, uint16_t* out, hipStream_t stream);
int launch_png16_decode(const uint16_t* in, int B, int h, int w, float* flow, uint8_t* valid, int* bad,
                        hipStream_t stream);

uint32_t voxel_key_range(bool dsec, int C, int H, int W);
int voxel_workspace_bytes(bool dsec, int64_t n, int C, int H, int W, int64_t* bytes);
int launch_voxel(bool dsec, const float* p, const float* t, const float* x, const float* y, const double* ev,
                 int64_t n, int C, int H, int W, int normalize, float* voxel, int* bad, void* workspace,
                 hipStream_t stream);

int64_t splat_workspace_bytes(bool flow_mode, int B, int64_t n, int h, int w);
int launch_splat(bool flow_mode, const float* pts, int B, int64_t n, int h, int w, float* values, uint8_t* valid,
                 void* workspace, hipStream_t stream);

}  // namespace ecorr
