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
