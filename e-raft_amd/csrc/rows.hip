// rows.hip -- reassembly step of the query-row sharded CorrBlock's all-gathers (rowshard.py).
//
// After an all-gather of fixed-size chunks, chunk r holds rank r's rows as [B][C][rows_r][W]
// (rows_r of the contiguous near-equal partition: the first H % world ranks own H / world + 1
// rows), followed by unused padding up to the chunk size.  The full map [B][C][H][W] takes, per
// (b, c) plane, the rows of every rank in rank order -- so each plane is `world` contiguous copies
// of rows_r * W floats.  One block per plane; 16-byte loads and stores when the geometry allows.
// HBM-bound: 2 * B * C * H * W * 4 bytes.  Replaces the torch.cat reassembly of the round-1
// rowshard.gather_rows (the reference has no counterpart: it never shards, eraft.py:128-132).
#include "ecorr_internal.h"

namespace ecorr {

namespace {

constexpr int RT = 256;

template <bool VEC>
__global__ __launch_bounds__(RT) void rows_assemble_kernel(const float* __restrict__ chunks, int64_t chunk,
                                                           int world, int H, int W, float* __restrict__ out) {
    const int64_t bc = blockIdx.x;
    const int base = H / world, extra = H % world;
    float* dst_plane = out + bc * H * W;
    for (int r = 0; r < world; ++r) {
        const int cnt = base + (r < extra ? 1 : 0);
        const int start = r * base + min(r, extra);
        const float* src = chunks + (int64_t)r * chunk + bc * cnt * W;
        float* dst = dst_plane + (int64_t)start * W;
        const int n = cnt * W;
        if (VEC) {
            const float4* s4 = reinterpret_cast<const float4*>(src);
            float4* d4 = reinterpret_cast<float4*>(dst);
            for (int i = threadIdx.x; i < n / 4; i += RT) d4[i] = s4[i];
        } else {
            for (int i = threadIdx.x; i < n; i += RT) dst[i] = src[i];
        }
    }
}

}  // namespace

int launch_rows_assemble(const float* chunks, int64_t chunk, int world, int B, int C, int H, int W, float* out,
                         hipStream_t stream) {
    const bool vec = W % 4 == 0 && chunk % 4 == 0 && ((uintptr_t)chunks & 15) == 0 && ((uintptr_t)out & 15) == 0;
    const dim3 grid((unsigned)((int64_t)B * C));
    if (vec)
        hipLaunchKernelGGL(rows_assemble_kernel<true>, grid, dim3(RT), 0, stream, chunks, chunk, world, H, W, out);
    else
        hipLaunchKernelGGL(rows_assemble_kernel<false>, grid, dim3(RT), 0, stream, chunks, chunk, world, H, W, out);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? ECORR_OK : ECORR_EHIP - (int)e;
}

}  // namespace ecorr
