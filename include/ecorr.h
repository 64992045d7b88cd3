/*
 * ecorr.h -- C ABI of the MI355X-native E-RAFT correlation hot path (libecorr.so, gfx950).
 *
 * Drop-in boundary for wzygzlm/E-RAFT's model/corr.py CorrBlock and the model/utils.py helpers.
 * Every entry point is stream-ordered and asynchronous on `stream` (a hipStream_t passed as
 * void*, e.g. torch.cuda.current_stream().cuda_stream); all buffers are device pointers owned by
 * the caller (PyTorch's caching allocator); the library allocates nothing and keeps no global
 * mutable state.  Return value: ECORR_OK (0) or a negative code; ecorr_strerror() names it.  No
 * C++ exception crosses this boundary.
 *
 * Pyramid storage (what ecorr_build writes, ecorr_lookup reads) -- a layout chosen for the gather:
 * `levels` blocks concatenated at float offsets off_i (each a multiple of 32 floats, i.e. 128-byte
 * aligned); level i holds rows = B * q_count query images of h_i x w_i (h_0 = H, w_0 = W,
 * h_{i+1} = h_i / 2, w_{i+1} = w_i / 2, floor -- the shapes of the reference's corr_pyramid[i],
 * corr.py:16-27).  Each level is stored in one of three formats (ecorr_pyramid_formats):
 *   tiled (ntx_i > 0; levels 0 and >= 4): row-major ECORR_TILE_H x ECORR_TILE_W tiles of 32
 *     floats (128 bytes, one L2 line); image r starts at off_i + r * hp_i * wp_i,
 *     hp_i = roundup(h_i, 4), wp_i = roundup(w_i, 8) = 8 * ntx_i, and pixel (y, x) sits at
 *     ((y / 4) * ntx_i + x / 8) * 32 + (y % 4) * 8 + x % 8.  A radius-4 window then touches ~7
 *     lines per level instead of ~13 with row-major images; padding cells are never read.
 *   interleaved (ntx_i = -nbx < 0; levels 1, 2 and 3): blocks of bh x bw = 2 x 4 (levels 1 and 2)
 *     or 1 x 2 (level 3) pixels (at levels 2 and 3 what one 8 x 16 block of level 0 pools to),
 *     nby = ceil(h_i / bh) by nbx =
 *     ceil(w_i / bw) of them per image, sz = nby * nbx * bh * bw floats per image; the rows are
 *     taken in groups of ECORR_ROW_GROUP = 64 (the level holds roundup(rows, 64) * sz floats) and
 *     pixel (y, x) of row r sits at (r / 64) * 64 * sz + (((y / bh) * nbx + x / bw) * 64 + r % 64)
 *     * bh * bw + (y % bh) * bw + x % bw: a block's pixels of 64 consecutive rows are contiguous,
 *     so the build stores them as whole lines and adjacent queries' window reads share lines.
 *   compact (ntx_i = 0): plain row-major h_i x w_i, image r at off_i + r * h_i * w_i.  Used for
 *     levels i >= 4 whose tile padding would exceed half the image (2 hp wp > 3 h w).
 * The Python shim materializes reference-layout corr_pyramid views on demand.
 *
 * Query slabs (multi-GPU query-row sharding): fmap1, coords and the lookup output hold
 * the q_count query pixels being served -- all H*W of them for the plain CorrBlock, a contiguous
 * block of image rows on a query-row shard.  fmap2 is always the whole [B][D][H][W] target map.
 */
#ifndef ECORR_H
#define ECORR_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ECORR_ABI_VERSION 16
#define ECORR_MAX_LEVELS 16
#define ECORR_TILE_H 4
#define ECORR_TILE_W 8
#define ECORR_ROW_GROUP 64

enum ecorr_status {
    ECORR_OK = 0,
    ECORR_EINVAL = -1,   /* null pointer, non-positive size, q_count outside [1, H*W] */
    ECORR_ESHAPE = -2,   /* a pyramid level would be 0 pixels tall or wide (reference: avg_pool2d
                            raises "Output size is too small", corr.py:26) */
    ECORR_ERADIUS = -3,  /* radius < 0 or > 32 */
    ECORR_ELEVELS = -4,  /* levels < 1 or > ECORR_MAX_LEVELS */
    ECORR_EHIP = -1000   /* HIP error e is reported as ECORR_EHIP - e */
};

/* Layout of the pyramid for `rows` query rows (rows = B * q_count).  Writes h[levels],
 * w[levels] (true level sizes), off[levels + 1] (float offsets including tile padding and the
 * 128-byte alignment of each level; off[levels] = total floats).
 * Replaces: the shapes produced by CorrBlock.__init__'s reshape + avg_pool2d loop, corr.py:21-27. */
int ecorr_pyramid_layout(int64_t rows, int H, int W, int levels, int* h, int* w, int64_t* off);

/* Build the correlation pyramid: level 0 = fmap1^T fmap2 / sqrt(D), levels 1.. = 2x2 floor-mode
 * average pools.  fmap1: float[B][D][q_count] (the query slab; = [B][D][H][W] when q_count = H*W),
 * fmap2: float[B][D][H][W], both contiguous.  pyramid: ecorr_pyramid_layout(B*q_count, ...) floats.
 * Replaces: CorrBlock.__init__ (corr.py:13-27) and CorrBlock.corr (corr.py:52-60). */
int ecorr_build(const float* fmap1, const float* fmap2, int B, int D, int H, int W, int q_count,
                int levels, float* pyramid, void* stream);

/* Same result contract as ecorr_build (level 0 within the 1e-5 normwise bar of the reference's
 * fp32 GEMM, levels 1.. pooled bit-exactly from it), computed on the f16 matrix cores: each fp32
 * operand is scaled by a per-pixel power of two and split into f16 hi + lo, and every product is
 * summed as lo*hi + hi*lo + hi*hi in fp32 -- error vs fp64 below the fp32-MFMA path's.  Per-pixel
 * scales depend only on that pixel's D values, so row-sharded and whole builds agree bit for bit.
 * workspace: ecorr_build_split_workspace_size() bytes of device memory, 256-byte aligned (the
 * exponents and the pre-split operands in MFMA-fragment order, about the two fmaps' size; free
 * once the call has completed on `stream`).  B <= 65535.
 * Replaces: CorrBlock.__init__ (corr.py:13-27) and CorrBlock.corr (corr.py:52-60). */
int ecorr_build_split_workspace_size(int B, int D, int H, int W, int q_count, int64_t* bytes);
int ecorr_build_split(const float* fmap1, const float* fmap2, int B, int D, int H, int W, int q_count,
                      int levels, float* pyramid, void* workspace, void* stream);

/* ecorr_build_split as its two stream-ordered stages, for callers that overlap or time them:
 * _pack = the operand pass (per-pixel exponents + f16 hi/lo panels into the workspace; reads
 * fmap1/fmap2), _gemm = the correlation GEMM with the fused pyramid (reads only the workspace).
 * pack then gemm on one stream == ecorr_build_split, bit for bit.  Contract: both stages take the
 * SAME workspace and IDENTICAL geometry (B, D, H, W, q_count), gemm stream-ordered after pack.  The
 * workspace carries no header (a check would need a host read of device memory, i.e. a sync), so a
 * gemm on a workspace packed for other geometry, or never packed, yields garbage exponents and
 * panels rather than an error. */
int ecorr_build_split_pack(const float* fmap1, const float* fmap2, int B, int D, int H, int W, int q_count,
                           void* workspace, void* stream);
int ecorr_build_split_gemm(int B, int D, int H, int W, int q_count, int levels, float* pyramid,
                           void* workspace, void* stream);

/* Radius-r lookup: out float[B][levels*(2r+1)^2][q_count] (= [B][C][H][W] when q_count = H*W),
 * channel 81*i + 9*a + b (r = 4) = bilinear sample of level i at (x/2^i + a - r, y/2^i + b - r),
 * zeros padding.  coords: float[B][2][q_count] contiguous (channel 0 = x, 1 = y, pixel units of
 * the H x W map).  Bit-exact with the reference on CPU.
 * Replaces: CorrBlock.__call__ (corr.py:29-50) incl. bilinear_sampler (utils.py:7-21). */
int ecorr_lookup(const float* pyramid, const float* coords, int B, int H, int W, int q_count,
                 int levels, int radius, float* out, void* stream);

/* ecorr_lookup + per-query partial maxima for ecorr_conv1x1_relu_split (ABI 15): qmax
 * float[B][3*levels][q_count], max over its 3*levels entries of query p = max_c |out[b][c][p]|
 * (fmaxf: NaN ignored); out bitwise what ecorr_lookup writes.  Replaces: corr.py:29-50 as above. */
int ecorr_lookup_qmax(const float* pyramid, const float* coords, int B, int H, int W, int q_count,
                      int levels, int radius, float* out, float* qmax, void* stream);

/* Lookup fused with its consumer, BasicMotionEncoder's convc1 + ReLU:
 * out float[B][O][q_count] = relu(bias[o] + sum_c weight[o][c] * corr[b][c][p]), where corr is
 * exactly what ecorr_lookup would return (C = levels*(2r+1)^2 channels) and never leaves the chip.
 * weight: float[O][C] (the conv weight [O][C][1][1] as stored), bias: float[O] or NULL.
 * radius must be 4 (else ECORR_ERADIUS), levels <= 4 (else ECORR_ELEVELS), O a positive multiple
 * of 64 (else ECORR_EINVAL).
 * Replaces: CorrBlock.__call__ (corr.py:29-50) + F.relu(self.convc1(corr)) (update.py:67,74). */
int ecorr_lookup_conv1x1_relu(const float* pyramid, const float* coords, int B, int H, int W, int q_count,
                              int levels, int radius, const float* weight, const float* bias, int O,
                              float* out, void* stream);

/* The same with the weight re-laid once in the fused kernel's MFMA fragment order (ABI 14): each
 * wave load of the weight stream is then one contiguous 1-KB piece.  ecorr_conv1x1_packed_size
 * gives the packed float count for O output and C = levels*(2r+1)^2 input channels (O a positive
 * multiple of 64); ecorr_conv1x1_pack writes it from weight float[O][C] (stream-ordered);
 * ecorr_lookup_conv1x1_relu_packed takes it in place of the weight -- bitwise the same result as
 * ecorr_lookup_conv1x1_relu with that weight.  The packed weight stays valid until the weight
 * changes (the Python binding re-packs on every in-place update of the weight tensor). */
int ecorr_conv1x1_packed_size(int O, int C, int64_t* floats);
int ecorr_conv1x1_pack(const float* weight, int O, int C, float* packed, void* stream);
int ecorr_lookup_conv1x1_relu_packed(const float* pyramid, const float* coords, int B, int H, int W, int q_count,
                                     int levels, int radius, const float* packed, const float* bias, int O,
                                     float* out, void* stream);

/* convc1 + ReLU on a materialized lookup (ABI 15; SURVEY §8f row 1 as two launches: ecorr_lookup,
 * then this): out float[B][O][Q] = relu(bias[o] + sum_c weight[o][c] * in[b][c][p]) for any
 * in float[B][C][Q] (the lookup's [B][C][H][W] with Q = H*W or a q_count slab), on the f16 matrix
 * cores with split operands (each fp32 value as hi + lo f16 under a per-query / per-output-row
 * power-of-two scale; three MFMAs per product): normwise within 1e-5 of the fp32 conv, not bitwise.
 * ecorr_conv1x1_split_size gives the packed weight's byte count, ecorr_conv1x1_split_pack writes it
 * from weight float[O][C] (stream-ordered); valid until the weight changes.  bias float[O] or NULL;
 * in and out must not overlap (ECORR_EINVAL when they are the same pointer, or when the 32-bit
 * buffer offsets, about (2C + 64) * Q * 4 bytes, would overflow).  qmax: NULL (the kernel finds each
 * query's largest |in| itself, one extra pass over in) or float[B][G][Q] partial maxima whose max
 * over g is max_c |in[b][c][p]| (fmaxf semantics, NaN ignored) -- what ecorr_lookup_qmax writes
 * with G = 3 * levels; the result is bitwise the same either way.
 * Non-finite input (the contract, tests/test_conv_split_gpu.py): a single +-inf or NaN value in a
 * query column in[b][.][p] makes EVERY output out[b][.][p] of that query NaN (the split's lo half
 * of an inf is inf - inf), where the reference's fp32 conv + ReLU gives +-inf / 0 / NaN per output;
 * the other queries are unaffected.  The split CorrBlock build never produces +-inf samples; the
 * fused entry (ecorr_lookup_conv1x1_relu_packed, fp32 sums) keeps the reference's pattern.
 * Replaces: F.relu(self.convc1(corr)) (update.py:67,74). */
int ecorr_conv1x1_split_size(int O, int C, int64_t* bytes);
int ecorr_conv1x1_split_pack(const float* weight, int O, int C, void* packed, void* stream);
int ecorr_conv1x1_relu_split(const float* in, int B, int C, int Q, const float* qmax, int G, const void* packed,
                             const float* bias, int O, float* out, void* stream);

/* Presplit convc1 (ABI 16): the lookup writes corr already split for the split conv, so the conv
 * loads each 8-channel B fragment as two 16-byte pieces and runs no split arithmetic and no maxima.
 * The query's scale must be known before any level's samples are written, so it is a bound, not
 * the samples' maximum: every sample of query p (level-0 values, their 2x2 averages and bilinear
 * blends) is at most sqrt(D) * max_d |fmap1[b][d][p]| * max |fmap2[b]| in magnitude.
 * ecorr_split_column_scale: fmap1, fmap2 float[B][D][H][W] -> scale int[B*H*W + B] (the last B
 *   entries are scratch): scale[b*H*W + p] = s_p, with every sample of p times 2^s_p below 2^15.
 * ecorr_presplit_size: bytes of the presplit corr of B items of Q queries (88 * levels positions
 *   for the 81 * levels channels).
 * ecorr_lookup_presplit: radius 4 (else ECORR_ERADIUS), levels <= 4 (else ECORR_ELEVELS):
 *   ecorr_lookup's samples x 2^s_p, split into f16 hi + lo (exactly: x 2^s = hi + lo + O(2^-22)),
 *   in the presplit layout (groups of 8 positions, 16 B per group / hi|lo / query; the channel
 *   order of e-raft_amd/csrc/ecorr_internal.h presplit_pos, zeros at the 7 * levels padding
 *   positions).  scale as written above.
 * ecorr_conv1x1_presplit_size / ecorr_conv1x1_split_pack_presplit: ecorr_conv1x1_split_pack with the
 *   weight columns at those positions (C = 81 * levels).
 * ecorr_conv1x1_relu_presplit: ecorr_conv1x1_relu_split's result from the presplit corr and the
 *   same scale: normwise within 1e-5 of the fp32 conv, not bitwise the split conv (other column
 *   scales, other channel order); the non-finite contract of ecorr_conv1x1_relu_split.
 * Replaces: CorrBlock.__call__ (corr.py:29-50) + F.relu(self.convc1(corr)) (update.py:67,74). */
int ecorr_split_column_scale(const float* fmap1, const float* fmap2, int B, int D, int H, int W, int* scale,
                             void* stream);
int ecorr_presplit_size(int B, int levels, int q_count, int64_t* bytes);
int ecorr_lookup_presplit(const float* pyramid, const float* coords, int B, int H, int W, int q_count, int levels,
                          int radius, const int* scale, void* out, void* stream);
int ecorr_conv1x1_presplit_size(int O, int levels, int64_t* bytes);
int ecorr_conv1x1_split_pack_presplit(const float* weight, int O, int levels, void* packed, void* stream);
int ecorr_conv1x1_relu_presplit(const void* in, int B, int levels, int Q, const int* scale, const void* packed,
                                const float* bias, int O, float* out, void* stream);

/* Generic bilinear_sampler: img float[N][C][h][w], coords float[N][Hg][Wg][2] in pixels ->
 * out float[N][C][Hg][Wg]; mask (nullable) float[N][Hg][Wg] = 1 where the normalized sample
 * lies strictly inside (-1, 1)^2.  Replaces: model/utils.py:7-21. */
int ecorr_bilinear_sampler(const float* img, int N, int C, int h, int w, const float* coords,
                           int Hg, int Wg, float* out, float* mask, void* stream);

/* coords_grid: out float[B][2][H][W], channel 0 = x (column), 1 = y (row).
 * Replaces: model/utils.py:24-27. */
int ecorr_coords_grid(int B, int H, int W, float* out, void* stream);

/* ---- SURVEY §8e, configs[4]: the query-row sharded CorrBlock's exchange (rowshard.py) ----
 * Reassembly after an all-gather of `world` fixed-size chunks: chunk r (floats [r*chunk,
 * (r+1)*chunk) of `chunks`) starts with rank r's rows as float[B][C][rows_r][W], where rows_r is
 * the contiguous near-equal partition of H (the first H % world ranks own H/world + 1 rows, rank r
 * starts at row r*(H/world) + min(r, H % world)); the rest of the chunk is padding.  Writes
 * out float[B][C][H][W].  chunk >= B*C*ceil(H/world)*W and H >= world (else ECORR_EINVAL).
 * Replaces: the torch.cat reassembly of the per-iteration lookup all-gather (the reference
 * keeps the GRU replicated, eraft.py:128-132, so every rank needs the full map). */
int ecorr_rows_assemble(const float* chunks, int64_t chunk, int world, int B, int C, int H, int W,
                        float* out, void* stream);

/* ---- the warm-start splat (utils/image_utils.py) ----
 * Deterministic and bit-exact with the reference's serial CPU put_(accumulate=True): the scatter
 * runs as a counting sort + ordered gather in a caller-provided workspace. */

/* Workspace bytes for B items of n points splatted onto an h x w grid (B = 1 for
 * ecorr_grid_sample_values, n = h*w for ecorr_forward_interpolate). */
int ecorr_splat_workspace_size(int B, int64_t n, int h, int w, int64_t* bytes);

/* forward_interpolate_pytorch: flow float[B][2][h][w] -> out float[B][2][h][w]; every pixel moves
 * to (col + dx, row + dy) and is splatted bilinearly; pixels nothing lands on read 0.
 * Replaces: utils/image_utils.py:50-83 (and its per-sample Python loop, :78-80). */
int ecorr_forward_interpolate(const float* flow, int B, int h, int w, float* out, void* workspace,
                              void* stream);

/* grid_sample_values: pts float[3][n] rows x, y, z -> values float[h][w] (interpolated z) and
 * valid uint8[h][w] (nullable; 1 where some weight landed).  0 <= n < 2^24.
 * Replaces: utils/image_utils.py:10-47. */
int ecorr_grid_sample_values(const float* pts, int64_t n, int h, int w, float* values, uint8_t* valid,
                             void* workspace, void* stream);

/* ---- convex upsampling and the DSEC 16-bit PNG flow codec ---- */

/* ERAFT.upsample_flow: flow float[N][2][H][W], mask float[N][576][H][W] (the update block's
 * 0.25 * mask head) -> out float[N][2][8H][8W]; softmax over the 9 taps, convex combination of
 * the zero-padded 3x3 window of 8 * flow.  Within a few ulp of the reference (device expf).
 * Replaces: model/eraft.py:74-85. */
int ecorr_upsample_flow(const float* flow, const float* mask, int N, int H, int W, float* out, void* stream);

/* DSEC submission encoding: flow float[B][2][h][w] -> out uint16[B][h][w][3] =
 * (u16)rint(flow * 128 + 2^15) with numpy's x86 float32 -> uint16 cast, channel 2 = 0.
 * Bit-exact.  Replaces: utils/visualization.py:81-84 (before imageio.imwrite). */
int ecorr_flow_to_png16(const float* flow, int B, int h, int w, uint16_t* out, void* stream);

/* DSEC ground-truth decoding: in uint16[B][h][w][3] -> flow float[B][h][w][2] = (v - 2^15) / 128
 * where channel 2 == 1 (else 0), valid uint8[B][h][w] = channel 2 == 1.  *bad (device int, zeroed
 * by the caller) counts pixels whose channel 2 is neither 0 nor 1 (the reference asserts).
 * Bit-exact.  Replaces: utils/dsec_utils.py:66-83 (after imageio.imread). */
int ecorr_png16_to_flow(const uint16_t* in, int B, int h, int w, float* flow, uint8_t* valid, int* bad,
                        void* stream);

/* ---- event stream -> voxel grid ----
 * The accumulated grid is bit-exact with the reference's single-threaded serial fold (stable sort
 * of the events by base cell + ordered per-cell gather); normalization (nonzero mean / unbiased
 * std) agrees within an ulp or two.  n >= 1 events; voxel float[C][H][W]. */

/* Workspace bytes for n events on a C x H x W grid (dsec != 0: ecorr_voxel_grid_dsec, else
 * ecorr_voxel_grid_mvsec). */
int ecorr_voxel_workspace_size(int dsec, int64_t n, int C, int H, int W, int64_t* bytes);

/* VoxelGrid.convert: p, t, x, y float[n] (t ascending), trilinear in (x, y, t).
 * Replaces: utils/dsec_utils.py:26-64 (as called by loader/loader_dsec.py:245-257). */
int ecorr_voxel_grid_dsec(const float* p, const float* t, const float* x, const float* y, int64_t n, int C,
                          int H, int W, int normalize, float* voxel, void* workspace, void* stream);

/* EventSequenceToVoxelGrid_Pytorch: events double[n][4] = (t, x, y, p), bilinear in t.
 * *bad_index (device int, zeroed by the caller) becomes nonzero where the reference's index_add_
 * would raise (an index outside the grid); the grid is then undefined.
 * Replaces: utils/transformers.py:36-126. */
int ecorr_voxel_grid_mvsec(const double* events, int64_t n, int C, int H, int W, int normalize, float* voxel,
                           int* bad_index, void* workspace, void* stream);

/* Tile shape of the pyramid storage (ECORR_TILE_H, ECORR_TILE_W). */
int ecorr_pyramid_tile(int* tile_h, int* tile_w);

/* Storage format of each level of an H x W pyramid: ntx[i] = tiles per tile row (tiled), 0
 * (compact row-major) or -nbx (interleaved, nbx blocks per block row).  Same errors as
 * ecorr_pyramid_layout. */
int ecorr_pyramid_formats(int H, int W, int levels, int* ntx);

/* Human-readable name of a status code (static storage). */
const char* ecorr_strerror(int status);

/* ECORR_ABI_VERSION of the loaded library. */
int ecorr_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* ECORR_H */
