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

/*
 * Row 3 -- event -> voxel grid.
 *
 * DSEC, utils/dsec_utils.py:26-64 (VoxelGrid.convert; the loader passes fp32 p, t, x, y,
 * loader/loader_dsec.py:245-257): t_norm = ((C-1) * (t - t[0])) / (t[-1] - t[0]); x0 = x.int()
 * (truncation, x86 cvttss2si: NaN / out of int32 -> INT_MIN); value = 2p - 1; for xlim in {x0,
 * x0+1} / ylim in {y0, y0+1} / tlim in {t0, t0+1} (that nesting = the pass order): in-bounds
 * entries add value * (1-|xlim-x|) * (1-|ylim-y|) * (1-|tlim-t_norm|) (left to right, fp32) with
 * put_(accumulate=True) -- serial in event order, since main.py:2-5 pins torch to one thread.
 *
 * MVSEC, utils/transformers.py:36-126 (EventSequenceToVoxelGrid_Pytorch, float64 events
 * [n][4] = t, x, y, p): ts = (bins-1) * (t - t0) / dT (f64, dT = 1 if 0); xs, ys = .long();
 * pol = float(p), 0 -> -1; tis = floor(ts); dts = ts - tis; left = pol * (1 - float(dts)),
 * right = pol * float(dts); index_add_ (serial) of all left values at xs + ys W + tis W H where
 * 0 <= tis < bins, then all right values at +W H where 0 <= tis and tis + 1 < bins.  An index
 * outside the grid raises in the reference (returned here as nonzero).
 *
 * normalize (both, dsec_utils.py:55-62 / transformers.py:117-124): over the nonzero cells,
 * mean (sum in double, rounded), std (unbiased, double two-pass, rounded); v = (v - mean) / std,
 * or v - mean when std == 0.  ATen reduces in its own order, so normalized values agree within a
 * few ulp; the accumulated grid itself is bit-exact.
 */
static int x86_f32_to_i32(float v) {
    return (v >= -2147483648.0f && v < 2147483648.0f) ? (int)v : (int)0x80000000u;
}

static long long x86_f64_to_i64(double v) {
    return (v >= -9223372036854775808.0 && v < 9223372036854775808.0) ? (long long)v : (long long)(1ULL << 63);
}

static void voxel_normalize(float* g, long n) {
    long cnt = 0;
    double sum = 0.0;
    for (long i = 0; i < n; ++i)
        if (g[i] != 0.0f) { ++cnt; sum += g[i]; }
    if (cnt == 0) return;
    const double m64 = sum / (double)cnt;
    double m2 = 0.0;
    for (long i = 0; i < n; ++i)
        if (g[i] != 0.0f) { const double d = g[i] - m64; m2 += d * d; }
    const float mean = (float)m64;
    const float std = cnt > 1 ? (float)sqrt(m2 / (double)(cnt - 1)) : NAN;
    for (long i = 0; i < n; ++i)
        if (g[i] != 0.0f) g[i] = std > 0.0f ? (g[i] - mean) / std : g[i] - mean;
}

EXPORT void oracle_voxel_dsec(const float* p, const float* t, const float* x, const float* y, long n, int C,
                              int H, int W, int normalize, float* out) {
    const long HW = (long)H * W;
    memset(out, 0, sizeof(float) * (size_t)(C * HW));
    const float dt = t[n - 1] - t[0];
    float* tn = (float*)malloc(sizeof(float) * (size_t)n);
    for (long e = 0; e < n; ++e) tn[e] = ((float)(C - 1) * (t[e] - t[0])) / dt;
    for (int a = 0; a < 2; ++a)
        for (int b = 0; b < 2; ++b)
            for (int c = 0; c < 2; ++c)
                for (long e = 0; e < n; ++e) {
                    const int xl = x86_f32_to_i32(x[e]) + a, yl = x86_f32_to_i32(y[e]) + b,
                              tl = x86_f32_to_i32(tn[e]) + c;
                    if (!(xl < W && xl >= 0 && yl < H && yl >= 0 && tl >= 0 && tl < C)) continue;
                    const float v = 2.0f * p[e] - 1.0f;
                    const float wgt = ((v * (1.0f - fabsf((float)xl - x[e]))) * (1.0f - fabsf((float)yl - y[e]))) *
                                      (1.0f - fabsf((float)tl - tn[e]));
                    out[(long)tl * HW + (long)yl * W + xl] += wgt;
                }
    free(tn);
    if (normalize) voxel_normalize(out, C * HW);
}

EXPORT int oracle_voxel_mvsec(const double* ev, long n, int C, int H, int W, int normalize, float* out) {
    const long HW = (long)H * W, CHW = C * HW;
    memset(out, 0, sizeof(float) * (size_t)CHW);
    const double first = ev[0], last = ev[4 * (n - 1)];
    double dT = last - first;
    if (dT == 0.0) dT = 1.0;
    int bad = 0;
    for (int pass = 0; pass < 2; ++pass)
        for (long e = 0; e < n; ++e) {
            const double ts = (double)(C - 1) * (ev[4 * e] - first) / dT;
            const long long xs = x86_f64_to_i64(ev[4 * e + 1]), ys = x86_f64_to_i64(ev[4 * e + 2]);
            float pol = (float)ev[4 * e + 3];
            if (pol == 0.0f) pol = -1.0f;
            const double tis = floor(ts);
            const float dts = (float)(ts - tis);
            const int ok = pass == 0 ? (tis < C && tis >= 0) : (tis + 1 < C && tis >= 0);
            if (!ok) continue;
            const long long idx = xs + ys * W + (x86_f64_to_i64(tis) + pass) * HW;
            if (idx < 0 || idx >= CHW) { bad = 1; continue; }
            out[idx] += pass == 0 ? pol * (1.0f - dts) : pol * dts;
        }
    if (normalize && !bad) voxel_normalize(out, CHW);
    return bad;
}
