// copy_lab.hip -- what rate does a plain device copy reach at the operand pass's size (two fmaps of
// 78.6 MB in, the same bytes out: DSEC B = 16, D = 256, 60 x 80)?  Lab probe for the pack's bound
// (the pass runs at torch's copy rate, 4.9 TB/s, vs the guide's 6.29 TB/s f4
// copy).  Variants: f4 plain / non-temporal loads + stores, grid-stride with 1-4 f4 per
// thread per iteration, blocks of 256.  Median of 20 launches each, hipEvent timing.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/copy_lab tools/copy_lab.hip && /tmp/copy_lab
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void copy4(const f4* __restrict__ in, f4* __restrict__ out, long n4) {
    const long stride = (long)gridDim.x * 256 * U;
    for (long i = (long)blockIdx.x * 256 * U + threadIdx.x; i < n4; i += stride) {
        f4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long j = i + u * 256;
            if (j < n4) v[u] = NT ? __builtin_nontemporal_load(in + j) : in[j];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long j = i + u * 256;
            if (j < n4) {
                if (NT) __builtin_nontemporal_store(v[u], out + j);
                else out[j] = v[u];
            }
        }
    }
}

template <int U, bool NT>
float run(const f4* in, f4* out, long n4, int blocks) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    std::vector<float> ts;
    for (int r = 0; r < 23; ++r) {
        hipEventRecord(e0, 0);
        hipLaunchKernelGGL((copy4<U, NT>), dim3(blocks), dim3(256), 0, 0, in, out, n4);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        if (r >= 3) ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2] * 1e3f;
}

int main() {
    const long bytes = 2L * 16 * 256 * 4800 * 4;   // both fmaps: 157.3 MB
    const long n4 = bytes / 16;
    f4 *in, *out;
    if (hipMalloc(&in, bytes) != hipSuccess || hipMalloc(&out, bytes) != hipSuccess) return 1;
    hipMemset(in, 0, bytes);
    hipDeviceSynchronize();
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    for (int mult : {4, 8, 16, 32, 64}) {
        const int blocks = cus * mult;
        const float a = run<1, false>(in, out, n4, blocks), b = run<1, true>(in, out, n4, blocks);
        const float c = run<4, false>(in, out, n4, blocks), d = run<4, true>(in, out, n4, blocks);
        std::printf("blocks %6d  u1 %.1f us (%.2f TB/s)  u1nt %.1f (%.2f)  u4 %.1f (%.2f)  u4nt %.1f (%.2f)\n", blocks, a,
                    2 * bytes / a / 1e6, b, 2 * bytes / b / 1e6, c, 2 * bytes / c / 1e6, d, 2 * bytes / d / 1e6);
    }
    hipFree(in);
    hipFree(out);
    return 0;
}
