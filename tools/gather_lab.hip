// gather_lab.hip -- microbenchmark of the lookup's memory pattern on gfx950 (dev tool, not product):
// random line reads from a pyramid-sized buffer (1.96 GB, DSEC B=16), alone and beside a stream of
// 256-byte channel-row stores, to price the lookup's read side against its roofline.
//   line128 : a wave reads 8 random 128-B lines, 8 lanes x 16 B per line
//   half64  : 16 random 64-B half lines, 4 lanes x 16 B
//   seg32   : 32 random 32-B segments, 4 lanes x 8 B (the lookup's 8-byte pair loads)
//   seg48   : the lookup's phase-1 shape: 10.7 queries x 6 lanes x 8 B per row (48-B runs)
// Every variant reads the same number of useful bytes per wave-instruction group; GB/s counts the
// bytes the lanes asked for.  With "+st" each wave also stores 256-B rows into a 100 MB output
// (the lookup's 99.5 MB of NCHW output), the same bytes as it reads.
// usage: gather_lab [reps]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned uint2v __attribute__((ext_vector_type(2)));
typedef unsigned uint4v __attribute__((ext_vector_type(4)));

constexpr size_t BUF = (size_t)1963 << 20;   // the DSEC B=16 pyramid
constexpr size_t OUTB = (size_t)100 << 20;   // the lookup output
constexpr int ITEMS = 1 << 20;               // wave-items per launch

__device__ __forceinline__ uint32_t hash(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

// each wave-item: 4 load instructions (one per "row"), then optionally 4 store instructions
template <int PAT, bool ST>
__global__ __launch_bounds__(256) void gather_kernel(const char* __restrict__ buf, float* __restrict__ out, uint32_t seed,
                                                     float* sink) {
    const int lane = threadIdx.x & 63;
    const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(buf), 0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(out, 0, 0x7fffffff, 0x00020000);
    float acc = 0.0f;
    const uint32_t nlines = (uint32_t)(BUF / 128) - 2;
    for (int item = blockIdx.x * 4 + (threadIdx.x >> 6); item < ITEMS; item += gridDim.x * 4) {
        uint32_t off[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            uint32_t key;
            if (PAT == 0) key = hash(seed ^ (item * 32 + r * 8 + (lane >> 3)));
            else if (PAT == 1) key = hash(seed ^ (item * 64 + r * 16 + (lane >> 2)));
            else if (PAT == 2) key = hash(seed ^ (item * 128 + r * 32 + (lane >> 1)));
            else key = hash(seed ^ (item * 64 + r * 11 + lane / 6));
            const uint32_t line = key % nlines;
            // byte offset (buffer offsets are 31-bit: lines beyond 2 GB would wrap; BUF < 2 GB)
            if (PAT == 0) off[r] = line * 128 + (lane & 7) * 16;
            else if (PAT == 1) off[r] = line * 128 + ((key >> 28) & 1) * 64 + (lane & 3) * 16;
            else if (PAT == 2) off[r] = line * 128 + ((key >> 28) & 3) * 32 + (lane & 1) * 16;
            else off[r] = line * 128 + ((key >> 28) & 1) * 64 + (lane % 6) * 8;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            if (PAT <= 1 || PAT == 2) {
                const uint4v v = __builtin_amdgcn_raw_buffer_load_b128(rb, (int)off[r], 0, 0);
                acc += __uint_as_float(v.x ^ v.w);
            } else {
                const uint2v v = __builtin_amdgcn_raw_buffer_load_b64(rb, (int)off[r], 0, 0);
                acc += __uint_as_float(v.x ^ v.y);
            }
        }
        if (ST) {
            const uint32_t row = (uint32_t)item % (uint32_t)(OUTB / 1024);
#pragma unroll
            for (int r = 0; r < 4; ++r)
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc + r), ro, (int)(row * 1024 + r * 256 + lane * 4), 0, 2);
        }
    }
    if (acc == 1234.5f) *sink = acc;
}

// bytes the lanes ask for per wave-item
constexpr double item_bytes(int pat) { return pat == 3 ? 4 * 64 * 8.0 : 4 * 64 * 16.0; }

template <int PAT, bool ST>
float run(const char* buf, float* out, float* sink, int reps) {
    const dim3 grid(2048);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL((gather_kernel<PAT, ST>), grid, dim3(256), 0, 0, buf, out, 1u, sink);
    (void)hipEventRecord(a, 0);
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((gather_kernel<PAT, ST>), grid, dim3(256), 0, 0, buf, out, (uint32_t)(i * 7919 + 3), sink);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms / reps;
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 20;
    char* buf;
    float *out, *sink;
    if (hipMalloc(&buf, BUF) != hipSuccess || hipMalloc(&out, OUTB) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    (void)hipMemset(buf, 1, BUF);
    const char* names[] = {"line128", "half64", "seg32", "seg48"};
    float t[2][4];
    for (int rnd = 0; rnd < 2; ++rnd) {
        t[0][0] = run<0, false>(buf, out, sink, reps); t[1][0] = run<0, true>(buf, out, sink, reps);
        t[0][1] = run<1, false>(buf, out, sink, reps); t[1][1] = run<1, true>(buf, out, sink, reps);
        t[0][2] = run<2, false>(buf, out, sink, reps); t[1][2] = run<2, true>(buf, out, sink, reps);
        t[0][3] = run<3, false>(buf, out, sink, reps); t[1][3] = run<3, true>(buf, out, sink, reps);
    }
    printf("pattern   read GB/s (alone)   read GB/s (+256-B row stores)   read+write GB/s   us per 80 MB read + 100 MB write\n");
    for (int p = 0; p < 4; ++p) {
        const double rb = item_bytes(p) * ITEMS, wb = 4 * 256.0 * ITEMS;
        const double a = rb / (t[0][p] * 1e-3) / 1e9, s = rb / (t[1][p] * 1e-3) / 1e9, sw = (rb + wb) / (t[1][p] * 1e-3) / 1e9;
        printf("%-8s  %10.0f  %26.0f  %20.0f  %10.1f\n", names[p], a, s, sw, 80e6 / (a * 1e9) * 1e6);
    }
    return 0;
}
