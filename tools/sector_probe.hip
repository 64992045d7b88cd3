// sector_probe.hip -- does an L2 miss on gfx950 fetch the whole 128-byte line or only the 64-byte
// half a wave touches?  Lab probe for the pyramid tile layout: a 10x10 lookup
// window over 4x8-float tiles needs ~6.9 lines of 128 B, over 4x4 sub-tiles ~10.6 pieces of 64 B.
//   half: each 128-B line of a 2 GiB buffer read as its first 64 B (4 lanes x 16 B), stride 128 B
//   full: each line read whole (8 lanes x 16 B), half as many lines (same bytes requested)
//   both: every line read whole (twice the bytes)
// If `half` runs near `full`'s time, the fetch is sectored (64 B); near `both`, whole lines.
// build: hipcc --offload-arch=gfx950 -O3 -o tools/sector_probe tools/sector_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef unsigned uint4v __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void probe(const char* __restrict__ buf, long long nlines, int mode, unsigned* out) {
    // mode 0 = half (64 B of each line), 1 = full (every other line, whole), 2 = both (every line, whole)
    const int per = mode == 0 ? 4 : 8;                       // lanes per line
    const long long step = mode == 1 ? 256 : 128;            // bytes between the lines read
    const long long nread = mode == 1 ? nlines / 2 : nlines;
    const long long tid = blockIdx.x * 256LL + threadIdx.x, nt = (long long)gridDim.x * 256;
    unsigned acc = 0;
    for (long long i = tid; i < nread * per; i += nt) {
        const long long line = i / per, part = i % per;
        const uint4v v = __builtin_nontemporal_load(reinterpret_cast<const uint4v*>(buf + line * step + part * 16));
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;   // keeps the loads alive
}

int main() {
    const long long bytes = 2LL << 30, nlines = bytes / 128;
    char* buf;
    unsigned* out;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) return 1;
    hipMemset(buf, 1, bytes);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char* names[3] = {"half (64 B of every line)", "full (every other line, 128 B)", "both (every line, 128 B)"};
    float best[3] = {1e9f, 1e9f, 1e9f};
    for (int rep = 0; rep < 6; ++rep)
        for (int m = 0; m < 3; ++m) {
            hipEventRecord(e0);
            hipLaunchKernelGGL(probe, dim3(8192), dim3(256), 0, 0, buf, nlines, m, out);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (rep > 0 && ms < best[m]) best[m] = ms;
        }
    for (int m = 0; m < 3; ++m) {
        const double used = m == 0 ? nlines * 64.0 : m == 1 ? nlines * 64.0 : nlines * 128.0;
        printf("%-34s %8.3f ms  %6.2f TB/s of bytes used\n", names[m], best[m], used / best[m] / 1e9);
    }
    return 0;
}
