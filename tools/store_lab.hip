// store_lab.hip -- microbenchmark of pyramid-style store patterns on gfx950 (dev tool, not product).
// Writes a 1.47 GB buffer of 76,800 "query images" of 150 x 128-B lines (DSEC B=16 level 0) with
// different lane -> address shapes per wave-instruction, to price the build epilogue's options:
//   coal     : 1 KB contiguous per instruction (one image's 8-line run)
//   oct128   : 8 images x 128 B (8 lanes per line)
//   quad64   : 16 images x 64 B (4 lanes per 64-B half line)
//   pair32   : 32 images x 32 B (lanes q, q+32 = one 32-B tile row)
//   scat16   : 64 images x 16 B (one 16-B piece per lane, 8 instructions finish a line)
//   dword128 : 2 images x 128 B, 4 B per lane (one line per half-wave)
// usage: store_lab [reps]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int LINES = 144;     // lines per image used (150 in the real level; 144 = 18 x 8)
constexpr int IMG_B = 150 * 128;
constexpr int NIMG = 16 * 4800;

// AUX: cache-policy bits of the buffer store (gfx950: 1 sc0, 2 nt, 16 sc1)
// one descriptor over the whole buffer (built from the kernel argument: SGPRs), per-lane offsets
#define g_base gbase
template <int AUX>
__device__ __forceinline__ void st(floatx4* p, floatx4 v, char* gbase) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(g_base, 0, 0x7fffffff, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v), r,
                                           (int)((char*)p - g_base), 0, AUX);
}
template <int AUX>
__device__ __forceinline__ void st(float* p, float v, char* gbase) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(g_base, 0, 0x7fffffff, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, (int)((char*)p - g_base), 0, AUX);
}

// one wave item = 64 images x 8 lines (64 KB); block = 4 waves
template <int PAT, int NT>
__global__ __launch_bounds__(256) void store_kernel(char* buf, float val) {
  const int lane = threadIdx.x & 63;
  for (int item = blockIdx.x * 4 + (threadIdx.x >> 6); item < (NIMG / 64) * (LINES / 8); item += gridDim.x * 4) {
    const int ig = item / (LINES / 8), lr = item % (LINES / 8);
    char* base = buf + (size_t)ig * 64 * IMG_B + (size_t)lr * 8 * 128;
    const floatx4 v = {val, val + 1, val + 2, val + 3};
    if (PAT == 0) {   // coal
        for (int q = 0; q < 64; ++q) st<NT>(reinterpret_cast<floatx4*>(base + (size_t)q * IMG_B + lane * 16), v, buf);
    } else if (PAT == 1) {   // oct128
        const int q = lane >> 3, p = lane & 7;
        for (int g = 0; g < 8; ++g)
            for (int L = 0; L < 8; ++L)
                st<NT>(reinterpret_cast<floatx4*>(base + (size_t)(8 * g + q) * IMG_B + L * 128 + p * 16), v, buf);
    } else if (PAT == 2) {   // quad64
        const int q = lane >> 2, p = lane & 3;
        for (int g = 0; g < 4; ++g)
            for (int L = 0; L < 8; ++L)
                for (int s = 0; s < 2; ++s)
                    st<NT>(reinterpret_cast<floatx4*>(base + (size_t)(16 * g + q) * IMG_B + L * 128 + s * 64 + p * 16), v, buf);
    } else if (PAT == 3) {   // pair32
        const int q = lane & 31, h = lane >> 5;
        for (int g = 0; g < 2; ++g)
            for (int L = 0; L < 8; ++L)
                for (int r = 0; r < 4; ++r)
                    st<NT>(reinterpret_cast<floatx4*>(base + (size_t)(32 * g + q) * IMG_B + L * 128 + r * 32 + h * 16), v, buf);
    } else if (PAT == 4) {   // scat16
        for (int L = 0; L < 8; ++L)
            for (int k = 0; k < 8; ++k)
                st<NT>(reinterpret_cast<floatx4*>(base + (size_t)lane * IMG_B + L * 128 + k * 16), v, buf);
    } else {   // dword128
        const int h = lane >> 5, w = lane & 31;
        for (int i = 0; i < 32; ++i)
            for (int L = 0; L < 8; ++L)
                st<NT>(reinterpret_cast<float*>(base + (size_t)(2 * i + h) * IMG_B + L * 128 + w * 4), val, buf);
    }
  }
}

int g_blocks = 0;
template <int PAT, int NT>
float run(char* buf, int reps) {
    const int items = (NIMG / 64) * (LINES / 8);
    const dim3 grid(g_blocks > 0 ? g_blocks : (items + 3) / 4);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL((store_kernel<PAT, NT>), grid, dim3(256), 0, 0, buf, 1.0f);
    hipEventRecord(a, 0);
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((store_kernel<PAT, NT>), grid, dim3(256), 0, 0, buf, (float)i);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms / reps;
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 10;
    if (argc > 2) {   // per-CU rate: oct128 nt|sc1 and plain with a limited number of blocks
        char* b2;
        if (hipMalloc(&b2, (size_t)NIMG * IMG_B) != hipSuccess) return 1;
        const double mv = (double)NIMG * LINES * 128;
        for (int nb : {32, 64, 128, 256, 512, 1024, 2048}) {
            g_blocks = nb;
            const float a = run<1, 18>(b2, reps), c = run<1, 0>(b2, reps), d = run<0, 18>(b2, reps);
            const float e = run<2, 18>(b2, reps), f = run<2, 0>(b2, reps);
            printf("blocks %5d: oct128 nt|sc1 %7.0f GB/s  plain %7.0f  coal nt|sc1 %7.0f  quad64 nt|sc1 %7.0f  plain %7.0f\n", nb,
                   mv / (a * 1e-3) / 1e9, mv / (c * 1e-3) / 1e9, mv / (d * 1e-3) / 1e9, mv / (e * 1e-3) / 1e9,
                   mv / (f * 1e-3) / 1e9);
        }
        return 0;
    }
    char* buf;
    const size_t bytes = (size_t)NIMG * IMG_B;
    if (hipMalloc(&buf, bytes) != hipSuccess) { printf("alloc failed\n"); return 1; }
    const double moved = (double)NIMG * LINES * 128;
    const char* names[] = {"coal", "oct128", "quad64", "pair32", "scat16", "dword128"};
    float t[4][6];
#define RUNP(P) t[0][P] = run<P, 0>(buf, reps); t[1][P] = run<P, 2>(buf, reps); t[2][P] = run<P, 16>(buf, reps); t[3][P] = run<P, 18>(buf, reps);
    for (int rnd = 0; rnd < 2; ++rnd) { RUNP(0) RUNP(1) RUNP(2) RUNP(3) RUNP(4) RUNP(5) }
    printf("GB/s       plain     nt    sc1  nt|sc1\n");
    for (int p = 0; p < 6; ++p) {
        printf("%-9s", names[p]);
        for (int a = 0; a < 4; ++a) printf(" %7.0f", moved / (t[a][p] * 1e-3) / 1e9);
        printf("\n");
    }
    hipFree(buf);
    return 0;
}
