/*
 * ecorr_oracle.c -- CPU restatement of E-RAFT's CorrBlock hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker: only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it.  The product path (e-raft_amd/) never links it and
 * has no CPU fallback.
 *
 * Parity pinning: every function below is checked against golden vectors captured from the
 * imported reference (tests/golden/make_golden.py -> tests/golden/corr_NAME.npz) by
 * tests/test_oracle_golden.py: pooling and lookup bit-exact, level-0 within the normwise GEMM
 * tolerance (the reference's sgemm accumulation order is MKL's and not reproducible).
 *
 * Reference: /root/reference/model/corr.py, /root/reference/model/utils.py (wzygzlm/E-RAFT), whose
 * arithmetic lives in ATen (torch 2.10 CPU, AVX512 capability): aten::bmm, aten::div,
 * aten::avg_pool2d, aten::grid_sampler_2d.  The exact fp32 op orders restated here are:
 *   corr:    C = sum_d f1*f2 (fp64 here, rounded once), then C / sqrtf(D)      corr.py:52-60
 *   pool:    (((x00 + x01) + x10) + x11) / 4 from the rounded previous level    corr.py:25-27
 *   sample:  gx = RN(RN(2x / (W-1)) - 1)                                         utils.py:11
 *            ix = RN(RN(gx + 1) * ((W-1)/2))     (grid_sample, align_corners)    utils.py:15
 *            x0 = floor(ix); w = ix - x0; e = 1 - w; (same for y: n, s)
 *            nw = s*e, ne = s*w, sw = n*e, se = n*w
 *            acc = v_nw*nw; acc = fma(v_ne,ne,acc); fma(v_sw,sw,acc); fma(v_se,se,acc)
 *            with out-of-image corners read as 0 (zeros padding).
 *   lookup:  channel 81*i + 9*a + b samples level i at (x/2^i + (a-r), y/2^i + (b-r))   corr.py:35-47
 *
 * Build: gcc -O2 -ffp-contract=off -fno-fast-math -fopenmp (oracle/Makefile).  -ffp-contract=off
 * matters: only the explicit fmaf() calls may fuse.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define EXPORT __attribute__((visibility("default")))

/* corr.py:52-60 -- level-0 volume, out[b][p - q_begin][q] for p in [q_begin, q_begin+q_count). */
EXPORT void oracle_corr_level0(const float* f1, const float* f2, int B, int D, int H, int W,
                               int q_begin, int q_count, float* out) {
    const long Q = (long)H * W;
    const float s = sqrtf((float)D);  /* torch.sqrt(torch.tensor(dim).float()) */
    for (int b = 0; b < B; ++b) {
        const float* A = f1 + (long)b * D * Q;
        const float* Bm = f2 + (long)b * D * Q;
#pragma omp parallel for schedule(static)
        for (long pp = 0; pp < q_count; ++pp) {
            const long p = q_begin + pp;
            double* acc = (double*)calloc((size_t)Q, sizeof(double));
            for (int d = 0; d < D; ++d) {
                const double a = (double)A[(long)d * Q + p];
                const float* brow = Bm + (long)d * Q;
                for (long q = 0; q < Q; ++q) acc[q] += a * (double)brow[q];
            }
            float* orow = out + ((long)b * q_count + pp) * Q;
            for (long q = 0; q < Q; ++q) orow[q] = (float)acc[q] / s;
            free(acc);
        }
    }
}

/* corr.py:25-27 -- F.avg_pool2d(x, 2, stride=2), floor mode; in [N][h][w] -> out [N][h/2][w/2]. */
EXPORT void oracle_avg_pool2(const float* in, long N, int h, int w, float* out) {
    const int ho = h / 2, wo = w / 2;
#pragma omp parallel for schedule(static)
    for (long n = 0; n < N; ++n) {
        const float* src = in + n * (long)h * w;
        float* dst = out + n * (long)ho * wo;
        for (int y = 0; y < ho; ++y)
            for (int x = 0; x < wo; ++x) {
                const float* r0 = src + (long)(2 * y) * w + 2 * x;
                const float* r1 = r0 + w;
                float t = r0[0] + r0[1];
                t = t + r1[0];
                t = t + r1[1];
                dst[(long)y * wo + x] = t / 4.0f;
            }
    }
}

/* utils.py:11-12 + ATen grid_sampler (align_corners=True): pixel coord -> sampling coord. */
static inline float unnormalize_roundtrip(float x, int size) {
    const float g = (2.0f * x) / (float)(size - 1) - 1.0f;
    return (g + 1.0f) * ((float)(size - 1) / 2.0f);
}

static inline float corner(const float* img, int h, int w, float fx, float fy) {
    /* zeros padding: a corner outside [0,w) x [0,h) reads 0 */
    if (!(fx >= 0.0f && fx < (float)w && fy >= 0.0f && fy < (float)h)) return 0.0f;
    return img[(long)fy * w + (long)fx];
}

/* One bilinear sample at pixel coordinates (x, y) of image img[h][w] (utils.py:7-21). */
static inline float sample_px(const float* img, int h, int w, float x, float y) {
    const float ix = unnormalize_roundtrip(x, w);
    const float iy = unnormalize_roundtrip(y, h);
    const float x0 = floorf(ix), y0 = floorf(iy);
    const float we = ix - x0, e = 1.0f - we;
    const float n = iy - y0, s = 1.0f - n;
    const float nw = s * e, ne = s * we, sw = n * e, se = n * we;
    const float vnw = corner(img, h, w, x0, y0);
    const float vne = corner(img, h, w, x0 + 1.0f, y0);
    const float vsw = corner(img, h, w, x0, y0 + 1.0f);
    const float vse = corner(img, h, w, x0 + 1.0f, y0 + 1.0f);
    float acc = vnw * nw;
    acc = fmaf(vne, ne, acc);
    acc = fmaf(vsw, sw, acc);
    acc = fmaf(vse, se, acc);
    return acc;
}

/*
 * corr.py:29-50 -- CorrBlock.__call__.
 * pyr: levels concatenated, level i at pyr + level_off[i], layout [B*H*W][hs[i]][ws[i]].
 * coords: [B][2][H][W] (channel 0 = x, channel 1 = y).  out: [B][L*(2r+1)^2][H][W].
 */
EXPORT void oracle_lookup(const float* pyr, const int64_t* level_off, const int* hs, const int* ws,
                          int L, int r, const float* coords, int B, int H, int W, float* out) {
    const long Q = (long)H * W;
    const int K = 2 * r + 1, C = L * K * K;
#pragma omp parallel for schedule(static)
    for (long bq = 0; bq < (long)B * Q; ++bq) {
        const long b = bq / Q, p = bq % Q;
        const float cx = coords[(b * 2 + 0) * Q + p];
        const float cy = coords[(b * 2 + 1) * Q + p];
        for (int i = 0; i < L; ++i) {
            const float inv = 1.0f / (float)(1 << i);   /* coords / 2**i, exact */
            const float ccx = cx * inv, ccy = cy * inv;
            const int h = hs[i], w = ws[i];
            const float* img = pyr + level_off[i] + bq * (long)h * w;
            for (int a = 0; a < K; ++a) {
                const float x = ccx + (float)(a - r);   /* delta[...,0] = dy[a] (meshgrid 'ij') */
                for (int bb = 0; bb < K; ++bb) {
                    const float y = ccy + (float)(bb - r);
                    const int ch = i * K * K + a * K + bb;
                    out[(b * C + ch) * Q + p] = sample_px(img, h, w, x, y);
                }
            }
        }
    }
}

/*
 * utils.py:7-21 -- bilinear_sampler(img, coords, mask): img [N][Cc][h][w], coords [N][Hg][Wg][2]
 * (pixel units) -> out [N][Cc][Hg][Wg]; optional mask [N][Hg][Wg] (utils.py:17-19).
 */
EXPORT void oracle_bilinear_sampler(const float* img, int N, int Cc, int h, int w,
                                    const float* coords, int Hg, int Wg, float* out, float* mask) {
    const long G = (long)Hg * Wg;
    for (long n = 0; n < N; ++n)
        for (long g = 0; g < G; ++g) {
            const float x = coords[(n * G + g) * 2 + 0], y = coords[(n * G + g) * 2 + 1];
            for (int c = 0; c < Cc; ++c)
                out[(n * Cc + c) * G + g] =
                    sample_px(img + (n * Cc + c) * (long)h * w, h, w, x, y);
            if (mask) {
                const float gx = (2.0f * x) / (float)(w - 1) - 1.0f;
                const float gy = (2.0f * y) / (float)(h - 1) - 1.0f;
                mask[n * G + g] = (gx > -1.0f && gy > -1.0f && gx < 1.0f && gy < 1.0f) ? 1.0f : 0.0f;
            }
        }
}

/* utils.py:24-27 -- coords_grid: [B][2][H][W], channel 0 = x (column), channel 1 = y (row). */
EXPORT void oracle_coords_grid(int B, int H, int W, float* out) {
    for (int b = 0; b < B; ++b)
        for (int y = 0; y < H; ++y)
            for (int x = 0; x < W; ++x) {
                out[(((long)b * 2 + 0) * H + y) * W + x] = (float)x;
                out[(((long)b * 2 + 1) * H + y) * W + x] = (float)y;
            }
}
