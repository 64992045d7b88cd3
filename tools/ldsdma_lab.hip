// ldsdma_lab.hip -- does a buffer_load ... lds land at LDS byte addresses >= 64 KB on gfx950?
// (dev tool, not product).  One wave DMAs 1 KB pieces of a pattern to LDS offsets 0, 60 KB,
// 64 KB, 96 KB and 136 KB of a 140 KB array, then reads each piece back with ds_read and
// compares; also reports whether the piece aimed above 64 KB appeared at (offset mod 64 KB).
// usage: ldsdma_lab
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr int LDSB = 140 * 1024;
constexpr int NOFF = 5;
__constant__ int kOff[NOFF] = {0, 60 * 1024, 64 * 1024, 96 * 1024, 136 * 1024};

__global__ __launch_bounds__(64) void dma_kernel(const unsigned* src, unsigned* out) {
    __shared__ __attribute__((aligned(16))) char smem[LDSB];
    const int lane = threadIdx.x;
    for (int i = lane; i < LDSB / 4; i += 64) reinterpret_cast<unsigned*>(smem)[i] = 0xdeadbeefu;
    __syncthreads();
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned*>(src), 0, NOFF * 1024, 0x00020000);
#pragma unroll
    for (int p = 0; p < NOFF; ++p)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(smem + kOff[p]), 16, lane * 16,
                                                 p * 1024, 0, 0);
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    // out[p][0..255]: the words at kOff[p]; out[NOFF + p][..]: the words at kOff[p] mod 64 KB
    for (int p = 0; p < NOFF; ++p)
        for (int i = lane; i < 256; i += 64) {
            out[p * 256 + i] = reinterpret_cast<const unsigned*>(smem + kOff[p])[i];
            out[(NOFF + p) * 256 + i] = reinterpret_cast<const unsigned*>(smem + (kOff[p] & 0xffff))[i];
        }
}

int main() {
    unsigned h[NOFF * 256], o[2 * NOFF * 256];
    for (int i = 0; i < NOFF * 256; ++i) h[i] = 0x1000000u * (i / 256 + 1) + i;
    unsigned *ds, *dout;
    (void)hipMalloc(&ds, sizeof h);
    (void)hipMalloc(&dout, sizeof o);
    (void)hipMemcpy(ds, h, sizeof h, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(dma_kernel, dim3(1), dim3(64), 0, 0, ds, dout);
    (void)hipMemcpy(o, dout, sizeof o, hipMemcpyDeviceToHost);
    const int offs[NOFF] = {0, 60 * 1024, 64 * 1024, 96 * 1024, 136 * 1024};
    for (int p = 0; p < NOFF; ++p) {
        int at = 0, wrapped = 0;
        for (int i = 0; i < 256; ++i) {
            at += o[p * 256 + i] == h[p * 256 + i];
            wrapped += o[(NOFF + p) * 256 + i] == h[p * 256 + i];
        }
        printf("piece %d aimed at %6d: %3d/256 words there, %3d/256 at offset mod 64 KB (%d)\n", p, offs[p], at, wrapped,
               offs[p] & 0xffff);
    }
    return 0;
}
