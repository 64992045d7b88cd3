// lookup_lab.hip -- standalone timing lab for the CorrBlock lookup (dev tool, not shipped).
//
// Question it answers: how much of the lookup's time is the pyramid LAYOUT (tile shape per level,
// padded vs compact small levels) and the cache POLICY of the loads/stores, at the bench shape
// (DSEC 60x80 fmap, batch 16, radius 4, 4 levels).  The pyramid is synthetic: value(b,q,lvl,y,x)
// is a hash, written at the layout's position, so every variant must produce the same output
// (checked) while only the memory layout differs.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off tools/lookup_lab.hip -o tools/lookup_lab
//   ./tools/lookup_lab [batch]
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));           \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

constexpr int L = 4, R = 4, K = 2 * R + 1, KK = K * K, S = 2 * R + 3, SS = S * S, SP = SS | 1;

struct Lvl {
    int h, w;
    int ths, tws;   // tile = (1<<ths) x (1<<tws); tws < 0: row-major compact image
    int ntx;        // tiles per tile row
    int64_t sz;     // floats per query image
    int64_t off;    // float offset of the level in the pyramid
};
struct P {
    const float* coords;
    float* out;
    const float* pyr;
    int q_count;
    int rev;   // traverse the grid in reverse block order
    Lvl l[L];
};

__device__ __forceinline__ int loff(const Lvl& v, int y, int x) {
    if (v.tws < 0) return y * v.w + x;
    const int tm = (1 << v.ths) - 1, wm = (1 << v.tws) - 1;
    return ((((y >> v.ths) * v.ntx + (x >> v.tws)) << (v.ths + v.tws)) | ((y & tm) << v.tws) | (x & wm));
}

__device__ __forceinline__ float hval(int b, int q, int lv, int y, int x) {
    uint32_t h = (uint32_t)(b * 7919 + q) * 2654435761u ^ (uint32_t)(lv * 131 + y * 1031 + x * 17) * 40503u;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
    return (float)(h & 0xffff) * (1.0f / 65536.0f) - 0.5f;
}

__global__ void fill(P p, int B) {
    for (int lv = 0; lv < L; ++lv) {
        const Lvl& v = p.l[lv];
        const int64_t n = (int64_t)B * p.q_count * v.h * v.w;
        for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
            const int64_t img = i / (v.h * v.w);
            const int yx = (int)(i - img * v.h * v.w), y = yx / v.w, x = yx - y * v.w;
            const int b = (int)(img / p.q_count), q = (int)(img - (int64_t)b * p.q_count);
            float* base = const_cast<float*>(p.pyr) + v.off + img * v.sz;
            base[loff(v, y, x)] = hval(b, q, lv, y, x);
        }
    }
}

__device__ __forceinline__ float unnormalize(float x, float m1, float hm1) {
    const float g = __fsub_rn(__fdiv_rn(__fmul_rn(2.0f, x), m1), 1.0f);
    return __fmul_rn(__fadd_rn(g, 1.0f), hm1);
}
__device__ __forceinline__ float blend(float a, float b, float c, float d, float w, float n) {
    const float e = __fsub_rn(1.0f, w), s = __fsub_rn(1.0f, n);
    float acc = __fmul_rn(a, __fmul_rn(s, e));
    acc = __builtin_fmaf(b, __fmul_rn(s, w), acc);
    acc = __builtin_fmaf(c, __fmul_rn(n, e), acc);
    return __builtin_fmaf(d, __fmul_rn(n, w), acc);
}

// The production kernel's structure (lookup.hip lookup_staged<4,64>), generic layout, cache policy
// AUXL on pyramid loads of levels in NTL (bitmask), AUXS on output stores.
template <int QB, int AUXL, int NTL, int AUXS>
__global__ __launch_bounds__(4 * QB) void lab_staged(P p) {
    constexpr int NTQ = 4 * QB;
    __shared__ float win[QB * SP];
    __shared__ float fx[QB][K], wx[QB][K], fy[QB][K], wy[QB][K];
    __shared__ int org[QB][3];
    const int tid = threadIdx.x, g = tid & (QB - 1), part = tid / QB;
    int bx = blockIdx.x, lv = blockIdx.y, b = blockIdx.z;
    if (p.rev) { bx = gridDim.x - 1 - bx; lv = gridDim.y - 1 - lv; b = gridDim.z - 1 - b; }
    const Lvl v = p.l[lv];
    const int h = v.h, w = v.w;
    const int q0 = bx * QB, q = q0 + g;
    const bool valid = q < p.q_count;
    const int64_t Q = p.q_count, hw = v.sz;
    const float* lvbase = p.pyr + v.off + ((int64_t)b * Q + q0) * hw;
    if (valid) {
        const float inv = 1.0f / (float)(1 << lv);
        const float cx = __fmul_rn(p.coords[((int64_t)b * 2 + 0) * Q + q], inv);
        const float cy = __fmul_rn(p.coords[((int64_t)b * 2 + 1) * Q + q], inv);
        const float wm1 = (float)(w - 1), hm1 = (float)(h - 1);
#pragma unroll
        for (int j = part; j < 2 * K; j += 4) {
            const bool isx = j < K;
            const int o = isx ? j : j - K;
            const float c = __fadd_rn(isx ? cx : cy, (float)(o - R));
            const float m1 = isx ? wm1 : hm1;
            const float t = unnormalize(c, m1, m1 * 0.5f);
            const float f = floorf(t);
            if (isx) { fx[g][o] = f; wx[g][o] = __fsub_rn(t, f); }
            else     { fy[g][o] = f; wy[g][o] = __fsub_rn(t, f); }
        }
    }
    __syncthreads();
    if (part == 0) {
        int md = 2, X0 = 0, Y0 = 0, NX = 0, NY = 0;
        if (valid) {
            const float x0 = fx[g][0], y0 = fy[g][0];
            bool ok = fabsf(x0) < 1.0e7f && fabsf(y0) < 1.0e7f;
#pragma unroll
            for (int o = 0; o < K; ++o) {
                const float dx = fx[g][o] - x0, dy = fy[g][o] - y0;
                ok &= (dx >= 0.0f) & (dx <= (float)(S - 2)) & (dy >= 0.0f) & (dy <= (float)(S - 2));
            }
            md = ok ? 0 : 1;
            X0 = ok ? (int)x0 : 0;
            Y0 = ok ? (int)y0 : 0;
            NX = ok ? (int)(fx[g][K - 1] - x0) + 2 : 0;
            NY = ok ? (int)(fy[g][K - 1] - y0) + 2 : 0;
        }
        org[g][0] = X0; org[g][1] = Y0; org[g][2] = md | (NX << 8) | (NY << 16);
    }
    __syncthreads();
    constexpr int ITEMS = QB * S, NCOL = (ITEMS + NTQ - 1) / NTQ;
    const int nq = min(QB, p.q_count - q0);
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(lvbase), 0, (int)(nq * hw * 4), 0x00020000);
    constexpr int OOB = 0x7ffffff0;
    const bool ntl = (NTL >> lv) & 1;
    float vals[NCOL][S];
    int dst[NCOL];
#pragma unroll
    for (int c = 0; c < NCOL; ++c) {
        const int it = tid + c * NTQ;
        const bool live = it < ITEMS;
        const int gq = live ? it / S : 0;
        const int rx = it - gq * S;
        const int x = org[gq][0] + rx, y0 = org[gq][1], info = org[gq][2];
        const int ny = (info >> 16) & 0xff;
        const bool colin = live && (info & 0xff) == 0 && rx < ((info >> 8) & 0xff) && (unsigned)x < (unsigned)w;
        const int base = (int)(gq * hw);
        dst[c] = live ? gq * SP + rx : -1;
#pragma unroll
        for (int ry = 0; ry < S; ++ry) {
            const int y = y0 + ry;
            const int off = (colin && ry < ny && (unsigned)y < (unsigned)h) ? (base + loff(v, y, x)) * 4 : OOB;
            vals[c][ry] = ntl ? __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsrc, off, 0, AUXL))
                              : __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsrc, off, 0, 0));
        }
    }
#pragma unroll
    for (int c = 0; c < NCOL; ++c)
        if (dst[c] >= 0)
#pragma unroll
            for (int ry = 0; ry < S; ++ry) win[dst[c] + ry * S] = vals[c][ry];
    __syncthreads();
    const int md = org[g][2] & 0xff;
    if (md != 0) return;   // lab: direct path not exercised (coords stay finite)
    float* outp = p.out + ((int64_t)b * L * KK + (int64_t)lv * KK) * Q + q0 + g;
    const int X0 = org[g][0], Y0 = org[g][1];
    const float* wq = win + g * SP;
    for (int k = part; k < KK; k += 4) {
        const int a = k / K, bb = k - a * K;
        const float xa = fx[g][a], yb = fy[g][bb];
        const float* c = wq + ((int)yb - Y0) * S + ((int)xa - X0);
        const float res = blend(c[0], c[1], c[S], c[S + 1], wx[g][a], wy[g][bb]);
        if (AUXS) __builtin_nontemporal_store(res, outp + (int64_t)k * Q);
        else outp[(int64_t)k * Q] = res;
    }
}

// Calibration: stream `nread` floats (float4 loads) and write `nwrite` floats.
__global__ void stream_kernel(const float4* __restrict__ in, int64_t nread4, float4* __restrict__ out, int64_t nwrite4) {
    float4 acc = {0, 0, 0, 0};
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nread4; i += (int64_t)gridDim.x * blockDim.x) {
        const float4 v = in[i];
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nwrite4; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = acc;
}

// Random-line gather calibration: each group of G lanes reads one random chunk of G*16 bytes.
template <int G>
__global__ void gather_kernel(const float4* __restrict__ in, int64_t nchunks, int64_t reads, float* __restrict__ sink) {
    float acc = 0.f;
    const int lane = threadIdx.x % G;
    for (int64_t i = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / G; i < reads; i += (int64_t)gridDim.x * blockDim.x / G) {
        uint64_t hsh = (uint64_t)i * 0x9E3779B97F4A7C15ull;
        hsh ^= hsh >> 29;
        const int64_t c = (int64_t)(hsh % (uint64_t)nchunks);
        const float4 v = in[c * G + lane];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 12345.f) sink[0] = acc;
}

struct Variant {
    const char* name;
    int ths[L], tws[L];   // tws < 0 row-major
    int pad16;            // round each compact image up to 16 floats
};

static void layout(P& p, const Variant& vt, int64_t rows, const int* h, const int* w, int64_t& total) {
    int64_t off = 0;
    for (int i = 0; i < L; ++i) {
        Lvl& v = p.l[i];
        v.h = h[i]; v.w = w[i]; v.ths = vt.ths[i]; v.tws = vt.tws[i];
        if (v.tws < 0) {
            v.ntx = 0;
            v.sz = (int64_t)h[i] * w[i];
            if (vt.pad16) v.sz = (v.sz + 15) & ~15LL;
        } else {
            const int th = 1 << v.ths, tw = 1 << v.tws;
            const int hp = (h[i] + th - 1) / th * th, wp = (w[i] + tw - 1) / tw * tw;
            v.ntx = wp / tw;
            v.sz = (int64_t)hp * wp;
        }
        v.off = off;
        off += rows * v.sz;
        off = (off + 63) & ~63LL;
    }
    total = off;
}

int main(int argc, char** argv) {
    const int B = argc > 1 ? atoi(argv[1]) : 16;
    const int mode = argc > 2 ? atoi(argv[2]) : 1;   // 0: coords jump between iterations, 1: bench-like small steps
    const int H = 60, W = 80, Q = H * W;
    int h[L], w[L];
    h[0] = H; w[0] = W;
    for (int i = 1; i < L; ++i) { h[i] = h[i - 1] / 2; w[i] = w[i - 1] / 2; }
    const int64_t rows = (int64_t)B * Q;
    const int64_t outn = rows * L * KK;
    const double algo = (double)rows * 2904.0;

    // coords: grid + smooth flow, 12 fields
    std::vector<float> hc((size_t)B * 2 * Q * 12);
    srand(1);
    std::vector<float> fx0(B), fy0(B);
    for (int b = 0; b < B; ++b) { fx0[b] = (rand() % 1000) / 100.0f - 5.0f; fy0[b] = (rand() % 1000) / 100.0f - 5.0f; }
    for (int it = 0; it < 12; ++it)
        for (int b = 0; b < B; ++b) {
            const float fx = (rand() % 1000) / 100.0f - 5.0f, fy = (rand() % 1000) / 100.0f - 5.0f;
            for (int y = 0; y < H; ++y)
                for (int x = 0; x < W; ++x) {
                    const float jx = (rand() % 1000) / 500.0f - 1.0f, jy = (rand() % 1000) / 500.0f - 1.0f;
                    const float ph = mode ? 0.0f : (float)it;
                    const float sc = mode ? 0.25f : 1.0f;
                    const float sx = 3.0f * sinf(0.1f * y + ph), sy = 3.0f * cosf(0.07f * x - ph);
                    const float fxi = mode ? fx0[b] : fx, fyi = mode ? fy0[b] : fy;
                    hc[(((size_t)it * B + b) * 2 + 0) * Q + y * W + x] = x + fxi + sx + sc * jx;
                    hc[(((size_t)it * B + b) * 2 + 1) * Q + y * W + x] = y + fyi + sy + sc * jy;
                }
        }
    float *dc, *dout, *dref;
    CK(hipMalloc(&dc, hc.size() * 4));
    CK(hipMemcpy(dc, hc.data(), hc.size() * 4, hipMemcpyHostToDevice));
    CK(hipMalloc(&dout, outn * 4));
    CK(hipMalloc(&dref, outn * 4));

    const Variant vs[] = {
        {"t4x8, L3 compact (prod)", {2, 2, 2, 0}, {3, 3, 3, -1}, 0},
        {"t4x8, L2+L3 compact", {2, 2, 0, 0}, {3, 3, -1, -1}, 0},
    };
    const int nv = sizeof(vs) / sizeof(vs[0]);
    float* dpyr = nullptr;
    int64_t cap = 0;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    typedef void (*KFn)(P);
    struct KV { const char* name; KFn fn; int qb; };
    const KV kvs[] = {
        {"default", lab_staged<64, 0, 0, 0>, 64},
        {"nt L0L1 loads", lab_staged<64, 2, 3, 0>, 64},
        {"nt L0L1 + nt stores", lab_staged<64, 2, 3, 1>, 64},
        {"nt stores", lab_staged<64, 0, 0, 1>, 64},
        {"qb32", lab_staged<32, 0, 0, 0>, 32},
    };
    bool have_ref = false;
    for (int vi = 0; vi < nv; ++vi) {
        P p{};
        int64_t total;
        layout(p, vs[vi], rows, h, w, total);
        if (total > cap) {
            if (dpyr) CK(hipFree(dpyr));
            CK(hipMalloc(&dpyr, total * 4));
            cap = total;
        }
        p.pyr = dpyr;
        p.q_count = Q;
        p.out = dout;
        hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, p, B);
        CK(hipDeviceSynchronize());
        const int four[] = {0, 3, 3, 4};
        for (int kj = 0; kj < 4; ++kj) {
            const KV& kv = kvs[four[kj]];
            const int alt = kj == 2;
            const dim3 grid((Q + kv.qb - 1) / kv.qb, L, B), block(4 * kv.qb);
            // correctness: iteration-0 output equal across variants
            p.coords = dc;
            p.rev = 0;
            CK(hipMemset(dout, 0, outn * 4));
            hipLaunchKernelGGL(kv.fn, grid, block, 0, 0, p);
            CK(hipDeviceSynchronize());
            if (!have_ref) { CK(hipMemcpy(dref, dout, outn * 4, hipMemcpyDeviceToDevice)); have_ref = true; }
            else {
                std::vector<float> a(outn), r(outn);
                CK(hipMemcpy(a.data(), dout, outn * 4, hipMemcpyDeviceToHost));
                CK(hipMemcpy(r.data(), dref, outn * 4, hipMemcpyDeviceToHost));
                if (memcmp(a.data(), r.data(), outn * 4) != 0) printf("  !! %s / %s output differs\n", vs[vi].name, kv.name);
            }
            std::vector<float> ts;
            for (int rep = 0; rep < 8; ++rep) {
                CK(hipEventRecord(e0));
                for (int it = 0; it < 12; ++it) {
                    p.coords = dc + (size_t)it * B * 2 * Q;
                    p.rev = alt && (it & 1);
                    hipLaunchKernelGGL(kv.fn, grid, block, 0, 0, p);
                }
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (rep >= 2) ts.push_back(ms / 12);
            }
            std::sort(ts.begin(), ts.end());
            const double med = ts[ts.size() / 2];
            printf("%-28s %-18s%s pyr %6.0f MB  %7.1f us/call  %6.0f GB/s algorithmic (%.1f%%)\n", vs[vi].name, kv.name, alt ? " alt-rev" : "        ",
                   total * 4e-6, med * 1e3, algo / (med * 1e-3) / 1e9, algo / (med * 1e-3) / 8e12 * 100);
            fflush(stdout);
        }
    }
    // calibration: stream read of the lookup's byte count, and random chunk gathers
    {
        const int64_t rd4 = (int64_t)(rows * (3000.0 / 16)), wr4 = outn / 4;
        const dim3 grid(4096), block(256);
        for (int rep = 0; rep < 3; ++rep) {
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(stream_kernel, grid, block, 0, 0, (const float4*)dpyr, rd4, (float4*)dout, wr4);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (rep == 2)
                printf("stream: read %.0f MB + write %.0f MB in %.1f us -> %.0f GB/s\n", rd4 * 16e-6, wr4 * 16e-6,
                       ms * 1e3, (rd4 + wr4) * 16 / (ms * 1e-3) / 1e9);
        }
        const int64_t nfl = cap;   // floats in the pyramid buffer
        auto gather = [&](auto kern, int G, const char* nm) {
            const int64_t nchunks = nfl / (4 * G);
            const int64_t reads = (int64_t)(200e6 / (16 * G));
            for (int rep = 0; rep < 3; ++rep) {
                CK(hipEventRecord(e0));
                hipLaunchKernelGGL(kern, dim3(8192), dim3(256), 0, 0, (const float4*)dpyr, nchunks, reads, dout);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (rep == 2)
                    printf("random %-5s chunks from %.0f MB: %.0f MB in %.1f us -> %.0f GB/s\n", nm, nfl * 4e-6,
                           reads * 16.0 * G * 1e-6, ms * 1e3, reads * 16.0 * G / (ms * 1e-3) / 1e9);
            }
        };
        gather(gather_kernel<2>, 2, "32B");
        gather(gather_kernel<4>, 4, "64B");
        gather(gather_kernel<8>, 8, "128B");
        gather(gather_kernel<16>, 16, "256B");
    }
    printf("done\n");
    return 0;
}
