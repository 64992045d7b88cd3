// soff_lab.hip -- does a raw buffer access's scalar soffset take part in the range check on gfx950?
// (dev tool)  A descriptor of NREC bytes over a larger sentinel-filled allocation;
// each case stores (or loads) 64 dwords with per-lane voffset = 4 lane + V and scalar soffset S, then
// reports which lanes' stores landed (and where) / which loads returned data instead of 0.
//   hipcc --offload-arch=gfx950 -O2 -o tools/soff_lab tools/soff_lab.hip && tools/soff_lab
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr int NREC = 1024;          // bytes the descriptor covers
constexpr int ALLOC = 64 * 1024;    // bytes behind it (sentinel-filled)

__global__ void store_case(float* buf, int v, int s) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(buf, 0, NREC, 0x00020000);
    const int lane = threadIdx.x;
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(1.0f + lane), r, 4 * lane + v, s, 0);
}

__global__ void load_case(const float* buf, float* out, int v, int s) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(buf), 0, NREC, 0x00020000);
    const int lane = threadIdx.x;
    out[lane] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, 4 * lane + v, s, 0));
}

int main() {
    float *buf, *out;
    hipMalloc(&buf, ALLOC);
    hipMalloc(&out, 256);
    static float h[ALLOC / 4], o[64];
    struct { int v, s; } cases[] = {{0, 0}, {0, 768}, {0, 1024}, {0, 4096}, {768, 0}, {1024, 0}, {512, 256},
                                   {960, 64}, {-64, 128}, {1024, -1024}};
    for (auto c : cases) {
        for (int i = 0; i < ALLOC / 4; ++i) h[i] = -1.0f;
        hipMemcpy(buf, h, ALLOC, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(store_case, dim3(1), dim3(64), 0, 0, buf, c.v, c.s);
        hipMemcpy(h, buf, ALLOC, hipMemcpyDeviceToHost);
        int landed = 0, first = -1, last = -1;
        for (int i = 0; i < ALLOC / 4; ++i)
            if (h[i] != -1.0f) { ++landed; if (first < 0) first = i * 4; last = i * 4; }
        // loads: the allocation holds i at dword i
        for (int i = 0; i < ALLOC / 4; ++i) h[i] = (float)(i + 1);
        hipMemcpy(buf, h, ALLOC, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(load_case, dim3(1), dim3(64), 0, 0, buf, out, c.v, c.s);
        hipMemcpy(o, out, 256, hipMemcpyDeviceToHost);
        int nz = 0, lo = -1, hi = -1;
        for (int l = 0; l < 64; ++l)
            if (o[l] != 0.0f) { ++nz; if (lo < 0) lo = l; hi = l; }
        printf("voffset 4*lane%+6d soffset %6d (lane bytes %6d..%6d, +soffset %6d..%6d; NREC %d): "
               "stores landed %2d [bytes %d..%d]  loads nonzero %2d (lanes %d..%d, first value from byte %d)\n",
               c.v, c.s, c.v, c.v + 252, c.v + c.s, c.v + c.s + 252, NREC, landed, first, last, nz, lo, hi,
               lo >= 0 ? (int)(o[lo] - 1) * 4 : -1);
    }
    return 0;
}
