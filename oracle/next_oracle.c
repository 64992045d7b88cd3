/*
 * next_oracle.c -- CPU restatement of the SURVEY §8f "next" rows around the CorrBlock hot path.
 *
 * TEST INFRASTRUCTURE ONLY, like ecorr_oracle.c: loaded by tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg, never by the product package.  Pinned by golden vectors captured
 * from the imported reference (tests/golden/make_golden_next.py -> tests/golden/next_*.npz,
 * checked by tests/test_oracle_next.py).
 *
 * Row 2 -- warm-start splat, /root/reference/utils/image_utils.py:10-83
 *   grid_sample_values(input[3][n], h, w):  for (x_vals in {floor, ceil}) for (y_vals in {floor,
 *   ceil}): in-bounds points add z*wgt and wgt, wgt = (1 - |x - xv|) * (1 - |y - yv|), into
 *   values / weights_acc with put_(accumulate=True).  ATen's CPU put_ accumulates serially in
 *   index order while the masked index list is shorter than at::internal::GRAIN_SIZE (32768) --
 *   every E-RAFT use (1/8-resolution flows, <= 14720 points) -- so the sum for each target is the
 *   fp32 left fold over (pass, point) in that order, starting from +0.  Then
 *   values / (weights_acc + 1e-15f) and valid = weights_acc > 0.
 *   forward_interpolate_pytorch(flow[B][2][h][w]): points x = col + dx, y = row + dy (fp32 add of
 *   the int64 meshgrid promoted to float), z = dx then dy (image_utils.py:50-83).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define EXPORT __attribute__((visibility("default")))

/* image_utils.py:10-47 for nz value channels sharing the points: x[n], y[n], z[nz][n] ->
 * values[nz][h*w], valid[h*w] (1 = some weight landed). */
EXPORT void oracle_grid_sample_values(const float* x, const float* y, const float* z, int nz, long n,
                                      int h, int w, float* values, uint8_t* valid) {
    const long hw = (long)h * w;
    float* wacc = (float*)calloc((size_t)hw, sizeof(float));
    memset(values, 0, sizeof(float) * (size_t)(nz * hw));
    for (int px = 0; px < 2; ++px)
        for (int py = 0; py < 2; ++py)
            for (long s = 0; s < n; ++s) {
                const float xv = px ? ceilf(x[s]) : floorf(x[s]);
                const float yv = py ? ceilf(y[s]) : floorf(y[s]);
                if (!((xv < (float)w) & (xv >= 0.0f) & (yv < (float)h) & (yv >= 0.0f))) continue;
                const float wx = 1.0f - fabsf(x[s] - xv);
                const float wy = 1.0f - fabsf(y[s] - yv);
                const float wgt = wx * wy;
                const long idx = (long)(xv + (float)w * yv);
                for (int c = 0; c < nz; ++c) values[c * hw + idx] += z[c * n + s] * wgt;
                wacc[idx] += wgt;
            }
    for (long t = 0; t < hw; ++t) {
        const float den = wacc[t] + 1e-15f;
        for (int c = 0; c < nz; ++c) values[c * hw + t] = values[c * hw + t] / den;
        if (valid) valid[t] = wacc[t] > 0.0f;
    }
    free(wacc);
}

/* image_utils.py:50-83: flow [B][2][h][w] -> flow_new [B][2][h][w]. */
EXPORT void oracle_forward_interpolate(const float* flow, int B, int h, int w, float* out) {
    const long n = (long)h * w;
    float* x = (float*)malloc(sizeof(float) * (size_t)n);
    float* y = (float*)malloc(sizeof(float) * (size_t)n);
    for (int b = 0; b < B; ++b) {
        const float* f = flow + (long)b * 2 * n;
        for (long s = 0; s < n; ++s) {
            x[s] = (float)(s % w) + f[s];
            y[s] = (float)(s / w) + f[n + s];
        }
        oracle_grid_sample_values(x, y, f, 2, n, h, w, out + (long)b * 2 * n, NULL);
    }
    free(x);
    free(y);
}

/*
 * Row 4 -- convex upsampling, /root/reference/model/eraft.py:74-85 (ERAFT.upsample_flow):
 *   p_k = softmax_k(mask[n][64k + 8i + j][h][w]) as max, e_k = exp(x_k - max), s = sum_k e_k in
 *   order, p_k = e_k / s (recip != 0: p_k = e_k * (1/s)); out = sum_k p_k * (8 flow)[window k] in
 *   order from +0.  exp is libm expf, so agreement with ATen is within an ulp or two, not exact.
 */
EXPORT void oracle_upsample_flow(const float* flow, const float* mask, int N, int H, int W, int recip,
                                 float* out) {
    const long HW = (long)H * W;
    for (int n = 0; n < N; ++n)
        for (int h = 0; h < H; ++h)
            for (int w = 0; w < W; ++w) {
                float f8[2][9];
                for (int c = 0; c < 2; ++c)
                    for (int k = 0; k < 9; ++k) {
                        const int y = h + k / 3 - 1, x = w + k % 3 - 1;
                        f8[c][k] = (y >= 0 && y < H && x >= 0 && x < W)
                                       ? 8.0f * flow[((long)n * 2 + c) * HW + (long)y * W + x] : 0.0f;
                    }
                for (int i = 0; i < 8; ++i)
                    for (int j = 0; j < 8; ++j) {
                        float m[9], mx, s = 0.0f;
                        for (int k = 0; k < 9; ++k)
                            m[k] = mask[((long)n * 576 + k * 64 + i * 8 + j) * HW + (long)h * W + w];
                        mx = m[0];
                        for (int k = 1; k < 9; ++k) mx = m[k] > mx ? m[k] : mx;
                        for (int k = 0; k < 9; ++k) {
                            m[k] = expf(m[k] - mx);
                            s += m[k];
                        }
                        const float rs = 1.0f / s;
                        for (int k = 0; k < 9; ++k) m[k] = recip ? m[k] * rs : m[k] / s;
                        for (int c = 0; c < 2; ++c) {
                            float acc = 0.0f;
                            for (int k = 0; k < 9; ++k) acc += m[k] * f8[c][k];
                            out[(((long)n * 2 + c) * 8 * H + 8 * h + i) * 8 * W + 8 * w + j] = acc;
                        }
                    }
            }
}

/* DSEC PNG codec, utils/visualization.py:75-93 (encode) and utils/dsec_utils.py:66-83 (decode). */
static uint16_t x86_f32_to_u16(float v) {
    const int iv = (v >= -2147483648.0f && v < 2147483648.0f) ? (int)v : (int)0x80000000u;
    return (uint16_t)(iv & 0xffff);
}

EXPORT void oracle_png16_encode(const float* flow, int B, int h, int w, uint16_t* out) {
    const long HW = (long)h * w;
    for (long q = 0; q < (long)B * HW; ++q) {
        const long b = q / HW, p = q % HW;
        for (int c = 0; c < 2; ++c)
            out[3 * q + c] = x86_f32_to_u16(rintf(flow[(b * 2 + c) * HW + p] * 128.0f + 32768.0f));
        out[3 * q + 2] = 0;
    }
}

EXPORT int oracle_png16_decode(const uint16_t* in, long n, float* flow, uint8_t* valid) {
    int bad = 0;
    for (long q = 0; q < n; ++q) {
        const int ok = in[3 * q + 2] == 1;
        bad += in[3 * q + 2] > 1;
        for (int c = 0; c < 2; ++c) flow[2 * q + c] = ok ? (float)((int)in[3 * q + c] - 32768) / 128.0f : 0.0f;
        valid[q] = (uint8_t)ok;
    }
    return bad;
}
