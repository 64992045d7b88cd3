// abi.hip -- extern "C" entry points of libecorr.so (declared in include/ecorr.h).
//
// Validation mirrors the reference's failure behaviour where it has one (a pyramid level of zero
// pixels raises in avg_pool2d, corr.py:26) and rejects what the C ABI cannot express; nothing
// throws across the boundary.
#include <math.h>

#include "ecorr_device.h"
#include "ecorr_internal.h"

#define ECORR_EXPORT extern "C" __attribute__((visibility("default")))

using namespace ecorr;

namespace ecorr {

int pyramid_geometry(int64_t rows, int H, int W, int levels, PyrGeom* g) {
    if (rows <= 0 || H <= 0 || W <= 0) return ECORR_EINVAL;
    if (levels < 1 || levels > ECORR_MAX_LEVELS) return ECORR_ELEVELS;
    int hh = H, ww = W;
    int64_t o = 0;
    g->levels = levels;
    for (int i = 0; i < levels; ++i) {
        if (i > 0) { hh /= 2; ww /= 2; }
        if (hh == 0 || ww == 0) return ECORR_ESHAPE;
        g->h[i] = hh;
        g->w[i] = ww;
        int64_t nrows = rows;
        if (i >= 1 && i <= 3) {   // interleaved (ecorr_device.h pix_off): 2 x 4 / 2 x 4 / 1 x 2 blocks
            const int bh = 1 << ilv_sy(i), bw = 1 << ilv_sx(i);
            const int nby = (hh + bh - 1) / bh, nbx = (ww + bw - 1) / bw;
            g->ntx[i] = -nbx;
            g->nty[i] = nby;
            g->sz[i] = (int64_t)nby * nbx * bh * bw;
            nrows = (rows + kGroup - 1) / kGroup * kGroup;
        } else if (level_compact(i, hh, ww)) {
            g->ntx[i] = 0;
            g->nty[i] = hh;
            g->sz[i] = (int64_t)hh * ww;
        } else {
            g->ntx[i] = pad_w(ww) / kTileW;
            g->nty[i] = pad_h(hh) / kTileH;
            g->sz[i] = (int64_t)pad_h(hh) * pad_w(ww);
        }
        g->off[i] = o;
        o += nrows * g->sz[i];
        o = (o + kTile - 1) & ~(int64_t)(kTile - 1);   // every level starts on a 128-byte line
    }
    g->off[levels] = o;
    return ECORR_OK;
}

}  // namespace ecorr

namespace {

bool q_count_ok(int H, int W, int q_count) {
    const int64_t Q = (int64_t)H * W;
    return H > 0 && W > 0 && Q <= 0x7fffffff && q_count > 0 && q_count <= Q;
}

}  // namespace

ECORR_EXPORT int ecorr_abi_version(void) { return ECORR_ABI_VERSION; }

ECORR_EXPORT int ecorr_pyramid_tile(int* tile_h, int* tile_w) {
    if (!tile_h || !tile_w) return ECORR_EINVAL;
    *tile_h = kTileH;
    *tile_w = kTileW;
    return ECORR_OK;
}

ECORR_EXPORT const char* ecorr_strerror(int status) {
    switch (status) {
        case ECORR_OK: return "ok";
        case ECORR_EINVAL: return "invalid argument (null pointer, non-positive size or q_count outside [1, H*W])";
        case ECORR_ESHAPE: return "Output size is too small (a pyramid level would be 0 pixels tall or wide)";
        case ECORR_ERADIUS: return "radius out of range [0, 32]";
        case ECORR_ELEVELS: return "num_levels out of range [1, 16]";
        default: break;
    }
    if (status <= ECORR_EHIP) return hipGetErrorString((hipError_t)(ECORR_EHIP - status));
    return "unknown ecorr status";
}

ECORR_EXPORT int ecorr_pyramid_layout(int64_t rows, int H, int W, int levels, int* h, int* w, int64_t* off) {
    PyrGeom g;
    const int st = pyramid_geometry(rows, H, W, levels, &g);
    if (st != ECORR_OK) return st;
    for (int i = 0; i < levels; ++i) {
        if (h) h[i] = g.h[i];
        if (w) w[i] = g.w[i];
        if (off) off[i] = g.off[i];
    }
    if (off) off[levels] = g.off[levels];
    return ECORR_OK;
}

ECORR_EXPORT int ecorr_pyramid_formats(int H, int W, int levels, int* ntx) {
    if (!ntx) return ECORR_EINVAL;
    PyrGeom g;
    const int st = pyramid_geometry(1, H, W, levels, &g);
    if (st != ECORR_OK) return st;
    for (int i = 0; i < levels; ++i) ntx[i] = g.ntx[i];
    return ECORR_OK;
}

namespace {

int build_common(const float* fmap1, const float* fmap2, int B, int D, int H, int W, int q_count, int levels,
                 float* pyramid, void* workspace, void* stream, int stages = 3) {
    if ((stages & 1) && (!fmap1 || !fmap2)) return ECORR_EINVAL;
    if ((stages & 2) && !pyramid) return ECORR_EINVAL;
    if (B <= 0 || D <= 0) return ECORR_EINVAL;
    if (!q_count_ok(H, W, q_count)) return ECORR_EINVAL;
    PyrGeom g;
    const int st = pyramid_geometry((int64_t)B * q_count, H, W, levels, &g);
    if (st != ECORR_OK) return st;

    BuildParams P{};
    P.f1 = fmap1;
    P.f2 = fmap2;
    P.D = D;
    P.H = H;
    P.W = W;
    P.q_count = q_count;
    // corr.py:60 divides by torch.sqrt(torch.tensor(dim).float()) (IEEE sqrtf).  When that is a
    // power of two the division is an exact scaling and is done as a multiply.
    const float s = sqrtf((float)D);
    int e = 0;
    const float mant = frexpf(s, &e);
    P.scale_is_mul = (mant == 0.5f) ? 1 : 0;
    P.scale = P.scale_is_mul ? 1.0f / s : s;
    P.scale_shift = P.scale_is_mul ? e - 1 : 0;   // s = 0.5 * 2^e
    if (workspace) {
        if (B > 65535 || ((uintptr_t)workspace & 255)) return ECORR_EINVAL;
        P.ws = static_cast<char*>(workspace);
    }
    return launch_build(P, B, g, pyramid, (hipStream_t)stream, stages);
}

}  // namespace

ECORR_EXPORT int ecorr_build(const float* fmap1, const float* fmap2, int B, int D, int H, int W, int q_count,
                             int levels, float* pyramid, void* stream) {
    return build_common(fmap1, fmap2, B, D, H, W, q_count, levels, pyramid, nullptr, stream);
}

ECORR_EXPORT int ecorr_build_split_workspace_size(int B, int D, int H, int W, int q_count, int64_t* bytes) {
    if (!bytes || B <= 0 || B > 65535 || D <= 0 || !q_count_ok(H, W, q_count)) return ECORR_EINVAL;
    *bytes = build_split_workspace_bytes(B, D, H, W, q_count);
    return ECORR_OK;
}

ECORR_EXPORT int ecorr_build_split(const float* fmap1, const float* fmap2, int B, int D, int H, int W, int q_count,
                                   int levels, float* pyramid, void* workspace, void* stream) {
    if (!workspace) return ECORR_EINVAL;
    return build_common(fmap1, fmap2, B, D, H, W, q_count, levels, pyramid, workspace, stream);
}

ECORR_EXPORT int ecorr_build_split_pack(const float* fmap1, const float* fmap2, int B, int D, int H, int W,
                                        int q_count, void* workspace, void* stream) {
    if (!workspace) return ECORR_EINVAL;
    return build_common(fmap1, fmap2, B, D, H, W, q_count, 1, nullptr, workspace, stream, 1);
}

ECORR_EXPORT int ecorr_build_split_gemm(int B, int D, int H, int W, int q_count, int levels, float* pyramid,
                                        void* workspace, void* stream) {
    if (!workspace) return ECORR_EINVAL;
    return build_common(nullptr, nullptr, B, D, H, W, q_count, levels, pyramid, workspace, stream, 2);
}

namespace {

int lookup_params(const float* pyramid, const float* coords, int B, int H, int W, int q_count, int levels,
                  int radius, float* out, LookupParams* P) {
    if (!pyramid || !coords || !out || B <= 0) return ECORR_EINVAL;
    if (!q_count_ok(H, W, q_count)) return ECORR_EINVAL;
    if (radius < 0 || radius > 32) return ECORR_ERADIUS;
    PyrGeom g;
    const int st = pyramid_geometry((int64_t)B * q_count, H, W, levels, &g);
    if (st != ECORR_OK) return st;
    for (int i = 0; i < levels; ++i) {
        P->lvl[i] = pyramid + g.off[i];
        P->lh[i] = g.h[i];
        P->lw[i] = g.w[i];
        P->lntx[i] = g.ntx[i];
        P->lsz[i] = (int)g.sz[i];
    }
    P->coords = coords;
    P->out = out;
    P->H = H;
    P->W = W;
    P->q_count = q_count;
    P->levels = levels;
    P->radius = radius;
    P->C = levels * (2 * radius + 1) * (2 * radius + 1);
    if ((int64_t)B * P->C > 0xffff * 64) return ECORR_EINVAL;
    return ECORR_OK;
}

}  // namespace

ECORR_EXPORT int ecorr_lookup(const float* pyramid, const float* coords, int B, int H, int W, int q_count,
                              int levels, int radius, float* out, void* stream) {
    LookupParams P{};
    const int st = lookup_params(pyramid, coords, B, H, W, q_count, levels, radius, out, &P);
    if (st != ECORR_OK) return st;
    return launch_lookup(P, B, (hipStream_t)stream);
}

ECORR_EXPORT int ecorr_lookup_qmax(const float* pyramid, const float* coords, int B, int H, int W, int q_count,
                                   int levels, int radius, float* out, float* qmax, void* stream) {
    if (!qmax) return ECORR_EINVAL;
    LookupParams P{};
    const int st = lookup_params(pyramid, coords, B, H, W, q_count, levels, radius, out, &P);
    if (st != ECORR_OK) return st;
    P.qmax = qmax;
    return launch_lookup(P, B, (hipStream_t)stream);
}

ECORR_EXPORT int ecorr_lookup_conv1x1_relu(const float* pyramid, const float* coords, int B, int H, int W,
                                           int q_count, int levels, int radius, const float* weight,
                                           const float* bias, int O, float* out, void* stream) {
    if (!weight) return ECORR_EINVAL;
    LookupParams P{};
    const int st = lookup_params(pyramid, coords, B, H, W, q_count, levels, radius, out, &P);
    if (st != ECORR_OK) return st;
    return launch_lookup_conv(P, B, weight, bias, O, out, (hipStream_t)stream, false);
}

ECORR_EXPORT int ecorr_conv1x1_packed_size(int O, int C, int64_t* floats) {
    if (!floats || O <= 0 || O % 64 != 0 || C <= 0) return ECORR_EINVAL;
    *floats = conv1x1_packed_floats(O, C);
    return ECORR_OK;
}

ECORR_EXPORT int ecorr_conv1x1_pack(const float* weight, int O, int C, float* packed, void* stream) {
    if (!weight || !packed) return ECORR_EINVAL;
    return launch_conv1x1_pack(weight, O, C, packed, (hipStream_t)stream);
}

ECORR_EXPORT int ecorr_lookup_conv1x1_relu_packed(const float* pyramid, const float* coords, int B, int H, int W,
                                                  int q_count, int levels, int radius, const float* packed,
                                                  const float* bias, int O, float* out, void* stream) {
    if (!packed) return ECORR_EINVAL;
    LookupParams P{};
    const int st = lookup_params(pyramid, coords, B, H, W, q_count, levels, radius, out, &P);
    if (st != ECORR_OK) return st;
    return launch_lookup_conv(P, B, packed, bias, O, out, (hipStream_t)stream, true);
}

ECORR_EXPORT int ecorr_conv1x1_split_size(int O, int C, int64_t* bytes) {
    if (!bytes || O <= 0 || C <= 0) return ECORR_EINVAL;
    *bytes = conv1x1_split_bytes(O, C);
    return ECORR_OK;
}

ECORR_EXPORT int ecorr_conv1x1_split_pack(const float* weight, int O, int C, void* packed, void* stream) {
    if (!weight || !packed) return ECORR_EINVAL;
    return launch_conv1x1_split_pack(weight, O, C, packed, (hipStream_t)stream);
}

ECORR_EXPORT int ecorr_conv1x1_relu_split(const float* in, int B, int C, int Q, const float* qmax, int G,
                                          const void* packed, const float* bias, int O, float* out, void* stream) {
    if (!in || !packed || !out) return ECORR_EINVAL;
    return launch_conv1x1_relu_split(in, B, C, Q, qmax, G, packed, bias, O, out, (hipStream_t)stream);
}

ECORR_EXPORT int ecorr_split_column_scale(const float* fmap1, const float* fmap2, int B, int D, int H, int W,
                                          int* scale, void* stream) {
    if (!fmap1 || !fmap2 || !scale) return ECORR_EINVAL;
    return launch_split_column_scale(fmap1, fmap2, B, D, H, W, scale, (hipStream_t)stream);
}

ECORR_EXPORT int ecorr_presplit_size(int B, int levels, int q_count, int64_t* bytes) {
    if (!bytes || B <= 0 || q_count <= 0) return ECORR_EINVAL;
    if (levels < 1 || levels > 4) return ECORR_ELEVELS;
    *bytes = (int64_t)B * presplit_bytes_per_item(presplit_positions(levels), q_count);
    return ECORR_OK;
}

ECORR_EXPORT int ecorr_lookup_presplit(const float* pyramid, const float* coords, int B, int H, int W, int q_count,
                                       int levels, int radius, const int* scale, void* out, void* stream) {
    if (!scale || !out) return ECORR_EINVAL;
    if (radius != 4) return ECORR_ERADIUS;
    if (levels < 1 || levels > 4) return ECORR_ELEVELS;
    LookupParams P{};
    const int st = lookup_params(pyramid, coords, B, H, W, q_count, levels, radius, (float*)out, &P);
    if (st != ECORR_OK) return st;
    if (presplit_bytes_per_item(presplit_positions(levels), q_count) >= 0x7fffffffLL)
        return ECORR_EINVAL;   // 32-bit store offsets
    P.scale = scale;
    return launch_lookup(P, B, (hipStream_t)stream);
}

ECORR_EXPORT int ecorr_conv1x1_presplit_size(int O, int levels, int64_t* bytes) {
    if (!bytes || O <= 0) return ECORR_EINVAL;
    if (levels < 1 || levels > 4) return ECORR_ELEVELS;
    *bytes = conv1x1_presplit_bytes(O, levels);
    return ECORR_OK;
}

ECORR_EXPORT int ecorr_conv1x1_split_pack_presplit(const float* weight, int O, int levels, void* packed,
                                                   void* stream) {
    if (!weight || !packed) return ECORR_EINVAL;
    if (levels < 1 || levels > 4) return ECORR_ELEVELS;
    return launch_conv1x1_split_pack(weight, O, 81 * levels, packed, (hipStream_t)stream, levels);
}

ECORR_EXPORT int ecorr_conv1x1_relu_presplit(const void* in, int B, int levels, int Q, const int* scale,
                                             const void* packed, const float* bias, int O, float* out, void* stream) {
    if (!in || !packed || !out || !scale) return ECORR_EINVAL;
    if (levels < 1 || levels > 4) return ECORR_ELEVELS;
    return launch_conv1x1_relu_presplit(in, B, levels, Q, scale, packed, bias, O, out, (hipStream_t)stream);
}

ECORR_EXPORT int ecorr_bilinear_sampler(const float* img, int N, int C, int h, int w, const float* coords,
                                        int Hg, int Wg, float* out, float* mask, void* stream) {
    if (!img || !coords || !out || N <= 0 || C < 0 || h <= 0 || w <= 0 || Hg <= 0 || Wg <= 0)
        return ECORR_EINVAL;
    return launch_bilinear_sampler(img, N, C, h, w, coords, Hg, Wg, out, mask, (hipStream_t)stream);
}

ECORR_EXPORT int ecorr_coords_grid(int B, int H, int W, float* out, void* stream) {
    if (!out || B <= 0 || H <= 0 || W <= 0) return ECORR_EINVAL;
    return launch_coords_grid(B, H, W, out, (hipStream_t)stream);
}

ECORR_EXPORT int ecorr_rows_assemble(const float* chunks, int64_t chunk, int world, int B, int C, int H, int W,
                                     float* out, void* stream) {
    if (!chunks || !out || world < 1 || B <= 0 || C <= 0 || H < world || W <= 0) return ECORR_EINVAL;
    const int64_t rows_max = H / world + (H % world ? 1 : 0);
    if (chunk < (int64_t)B * C * rows_max * W || (int64_t)B * C > 0x7fffffff) return ECORR_EINVAL;
    return launch_rows_assemble(chunks, chunk, world, B, C, H, W, out, (hipStream_t)stream);
}

namespace {

bool splat_dims_ok(int B, int64_t n, int h, int w) {
    return B > 0 && n >= 0 && n < (1 << 24) && h > 0 && w > 0 && (int64_t)h * w <= 0x7fffffff;
}

}  // namespace

ECORR_EXPORT int ecorr_splat_workspace_size(int B, int64_t n, int h, int w, int64_t* bytes) {
    if (!bytes || !splat_dims_ok(B, n, h, w)) return ECORR_EINVAL;
    *bytes = splat_workspace_bytes(false, B, n, h, w);   // points mode is the stricter LDS fit
    return ECORR_OK;
}

ECORR_EXPORT int ecorr_forward_interpolate(const float* flow, int B, int h, int w, float* out, void* workspace,
                                           void* stream) {
    const int64_t n = (int64_t)h * w;
    if (!flow || !out || !splat_dims_ok(B, n, h, w)) return ECORR_EINVAL;
    if (!workspace && splat_workspace_bytes(true, B, n, h, w) > 0) return ECORR_EINVAL;
    return launch_splat(true, flow, B, n, h, w, out, nullptr, workspace, (hipStream_t)stream);
}

ECORR_EXPORT int ecorr_grid_sample_values(const float* pts, int64_t n, int h, int w, float* values, uint8_t* valid,
                                          void* workspace, void* stream) {
    if (!values || (!pts && n > 0) || !splat_dims_ok(1, n, h, w)) return ECORR_EINVAL;
    if (!workspace && splat_workspace_bytes(false, 1, n, h, w) > 0) return ECORR_EINVAL;
    return launch_splat(false, pts, 1, n, h, w, values, valid, workspace, (hipStream_t)stream);
}

ECORR_EXPORT int ecorr_upsample_flow(const float* flow, const float* mask, int N, int H, int W, float* out,
                                     void* stream) {
    if (!flow || !mask || !out || N <= 0 || N > 65535 || H <= 0 || W <= 0 || (int64_t)H * W > (1 << 26))
        return ECORR_EINVAL;
    return launch_upsample_flow(flow, mask, N, H, W, out, (hipStream_t)stream);
}

ECORR_EXPORT int ecorr_flow_to_png16(const float* flow, int B, int h, int w, uint16_t* out, void* stream) {
    if (!flow || !out || B <= 0 || h <= 0 || w <= 0) return ECORR_EINVAL;
    return launch_png16_encode(flow, B, h, w, out, (hipStream_t)stream);
}

ECORR_EXPORT int ecorr_png16_to_flow(const uint16_t* in, int B, int h, int w, float* flow, uint8_t* valid, int* bad,
                                     void* stream) {
    if (!in || !flow || !valid || !bad || B <= 0 || h <= 0 || w <= 0) return ECORR_EINVAL;
    return launch_png16_decode(in, B, h, w, flow, valid, bad, (hipStream_t)stream);
}

namespace {

bool voxel_dims_ok(int64_t n, int C, int H, int W) {
    // keys (extended grid for DSEC) must stay below 2^32 - 1; event indices are int32
    return n >= 1 && n <= 0x7fffffff && C > 0 && H > 0 && W > 0 &&
           (int64_t)(C + 1) * (H + 1) * (W + 1) < 0xffffffffLL;
}

}  // namespace

ECORR_EXPORT int ecorr_voxel_workspace_size(int dsec, int64_t n, int C, int H, int W, int64_t* bytes) {
    if (!bytes || !voxel_dims_ok(n, C, H, W)) return ECORR_EINVAL;
    return voxel_workspace_bytes(dsec != 0, n, C, H, W, bytes);
}

ECORR_EXPORT int ecorr_voxel_grid_dsec(const float* p, const float* t, const float* x, const float* y, int64_t n,
                                       int C, int H, int W, int normalize, float* voxel, void* workspace,
                                       void* stream) {
    if (!p || !t || !x || !y || !voxel || !workspace || !voxel_dims_ok(n, C, H, W)) return ECORR_EINVAL;
    return launch_voxel(true, p, t, x, y, nullptr, n, C, H, W, normalize, voxel, nullptr, workspace,
                        (hipStream_t)stream);
}

ECORR_EXPORT int ecorr_voxel_grid_mvsec(const double* events, int64_t n, int C, int H, int W, int normalize,
                                        float* voxel, int* bad_index, void* workspace, void* stream) {
    if (!events || !voxel || !bad_index || !workspace || !voxel_dims_ok(n, C, H, W)) return ECORR_EINVAL;
    return launch_voxel(false, nullptr, nullptr, nullptr, nullptr, events, n, C, H, W, normalize, voxel, bad_index,
                        workspace, (hipStream_t)stream);
}
