// Lab record (round 2): the 8-wave, two-n-tile split GEMM -- bitwise the same pyramid as
// build_split_kernel, 714 vs 659 us at DSEC B=16 (profiles/r02_lab2/ab_split2.txt): a third fewer
// operand bytes into the CU, but one block per CU leaves every epilogue exposed.  Not built; it
// slots into build.hip before the operand pass (launch: B * n_qt * ceil(n_nt / 2) blocks of 512).
// ============================================================================================
// Split GEMM, 8-wave form (D = 256): one block = 256 queries x TWO adjacent n-tiles, one block per
// CU.  Wave w computes query group w & 3 (64 queries) x n-tile w >> 2 exactly as a wave of
// build_split_kernel does (same fragments, same MFMA order: bitwise the same pyramid), but both
// operands pass through LDS by LDS-DMA, each query chunk shared by the two n-tiles' waves and each
// target chunk by the four query groups: 32 KB moved into the CU per chunk for 2 x 32768 outputs
// instead of 2 x 24 KB (the K loop pays for operand bytes moved to the CU).
// Chunk layout in LDS: [target panel of n-tile 0 | of n-tile 1 | query panel 0 | query panel 1],
// 8 KB each; 4 DMA pieces per wave and chunk, S2DT chunks ahead in S2DT buffers.
// ============================================================================================
constexpr bool kSplit2 = true;               // D = 256 builds use this kernel (A/B: tools/lab_build.py)
constexpr int S2CHUNK = 4 * PANEL;
constexpr int S2DT = 3;
constexpr int S2COPIES = S2CHUNK / 1024 / 8;   // 4
constexpr int S2LDS = 8 * 4 * 32 * XS;        // the 8 waves' epilogue transpose regions
static_assert(S2DT * S2CHUNK <= S2LDS, "split2 LDS regions");

template <bool MUL>
__global__ __launch_bounds__(512, 1) void build_split2_kernel(BuildParams P) {
    constexpr int NK = 16;
    __shared__ __attribute__((aligned(16))) char smem[S2LDS + (SQ + 512) * 4];
    int* exq = reinterpret_cast<int*>(smem + S2LDS);             // exponents of the 256 queries
    int* ext = exq + SQ;                                         // [2][128] negated target exponents
    float* fst = reinterpret_cast<float*>(ext + 256);            // [2][128] 2^ext when |ext| <= 63

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // uniform: DMA destinations need it
    const int qg = wave & 3, th = wave >> 2;   // query group, n-tile of this wave
    const int n_np = (P.n_nt + 1) / 2;
    int b, qt, np;
    decode_tile(P, xcd_remap(blockIdx.x, gridDim.x), P.n_qt, b, qt, np, n_np);
    // provably uniform descriptor inputs (else hipcc wraps every DMA in a waterfall loop, guide T20)
    b = __builtin_amdgcn_readfirstlane(b);
    qt = __builtin_amdgcn_readfirstlane(qt);
    np = __builtin_amdgcn_readfirstlane(np);
    const int nt0 = 2 * np;
    const bool has1 = nt0 + 1 < P.n_nt;
    const NTile tc = ntile_of(P, has1 ? nt0 + th : nt0);
    const int q0 = qt * SQ;
    const int H = P.H, W = P.W;
    const int64_t Q = (int64_t)H * W;

    {   // per-pixel exponents (before the first barrier; the first wait drains them with lgkmcnt(0))
        if (tid < SQ) {
            exq[tid] = q0 + tid < P.q_count ? P.ex1[(int64_t)b * P.q_count + q0 + tid] : 0;
        } else {
            const int u = tid - SQ, g = u >> 7, pos = u & 127;
            int e = 0;
            if (g == 0 || has1) {
                const NTile tg = ntile_of(P, nt0 + g);
                int y, x;
                split_target(pos, tg.band, y, x);
                y += tg.ty0;
                x += tg.tx0;
                e = (y < H && x < W) ? -P.ex2[(int64_t)b * Q + (int64_t)y * W + x] : 0;
            }
            ext[u] = e;
            fst[u] = exp2i(max(-63, min(e, 63)));
        }
    }

    // operand panels: two query panels (adjacent tiles of pk1), the two n-tiles' target panels
    const int64_t pstride = (int64_t)NK * PANEL;
    const int qp = 2 * qt;
    const int nqp = min(2, P.n_mt - qp);
    const __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<char*>(P.pk1 + ((int64_t)b * P.n_mt + qp) * pstride), 0, (int)(nqp * pstride), 0x00020000);
    const __amdgpu_buffer_rsrc_t rt0 = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<char*>(P.pk2 + ((int64_t)b * P.n_nt + nt0) * pstride), 0, (int)pstride, 0x00020000);
    const int nt1 = __builtin_amdgcn_readfirstlane(has1 ? nt0 + 1 : nt0);
    const int rng1 = __builtin_amdgcn_readfirstlane(has1 ? (int)pstride : 0);
    const __amdgpu_buffer_rsrc_t rt1 = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<char*>(P.pk2 + ((int64_t)b * P.n_nt + nt1) * pstride), 0, rng1, 0x00020000);
    // chunk kc: piece c = wave + 8 s of the 32 1-KB pieces: s = 0 -> target panel 0, 1 -> target
    // panel 1, 2 -> query panel 0, 3 -> query panel 1 (piece wave of each 8-KB panel)
    auto issue = [&](int kc) {
        char* dst = smem + (kc % S2DT) * S2CHUNK + wave * 1024;
        const bool in = kc < NK;
        const int po = in ? kc * PANEL + wave * 1024 + lane * 16 : SOOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rt0, (__attribute__((address_space(3))) void*)(dst), 16, po, 0, 0, 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rt1, (__attribute__((address_space(3))) void*)(dst + PANEL), 16, po, 0, 0, 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rq, (__attribute__((address_space(3))) void*)(dst + 2 * PANEL), 16, po, 0, 0, 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rq, (__attribute__((address_space(3))) void*)(dst + 3 * PANEL), 16,
                                                 in ? (int)pstride + po : SOOB, 0, 0, 0);
    };

    floatx16 acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) asm volatile("" : "+a"(acc[i][j]));

    // fragments of one chunk from LDS: target group j of n-tile th, query 32-row group i of query
    // group qg ([hi k0-15 | lo k0-15] x 32 rows, 16 B per lane)
    const int tfo = th * PANEL + lane * 16;
    const int qfo = 2 * PANEL + (qg >> 1) * PANEL + (qg & 1) * 4096 + lane * 16;
    struct Frags { halfx8 th[4], tl[4], qh[2], ql[2]; };
    auto read_lo = [&](int kc, Frags& f) {   // what the lo*hi MFMAs need: th, ql
        const char* cb = smem + (kc % S2DT) * S2CHUNK;
#pragma unroll
        for (int j = 0; j < 4; ++j) f.th[j] = *reinterpret_cast<const halfx8*>(cb + tfo + j * 2048);
#pragma unroll
        for (int i = 0; i < 2; ++i) f.ql[i] = *reinterpret_cast<const halfx8*>(cb + qfo + i * 2048 + 1024);
    };
    auto read_hi = [&](int kc, Frags& f) {   // tl, qh
        const char* cb = smem + (kc % S2DT) * S2CHUNK;
#pragma unroll
        for (int j = 0; j < 4; ++j) f.tl[j] = *reinterpret_cast<const halfx8*>(cb + tfo + j * 2048 + 1024);
#pragma unroll
        for (int i = 0; i < 2; ++i) f.qh[i] = *reinterpret_cast<const halfx8*>(cb + qfo + i * 2048);
    };
    auto mfma_lohi = [&](const Frags& f) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f.th[j], f.ql[i], acc[i][j], 0, 0, 0);
    };
    auto mfma_rest = [&](const Frags& f) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f.tl[j], f.qh[i], acc[i][j], 0, 0, 0);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f.th[j], f.qh[i], acc[i][j], 0, 0, 0);
    };
    // VMEM per wave: the S2COPIES DMA pieces of t(0) .. t(S2DT - 1), then chunk c issues those of
    // t(c + S2DT) in advance(c + 1); advance(j) waits for t(j) with t(j + 1) .. t(j + S2DT - 2) in
    // flight.  Loads, waits and phases are fenced with sched_barrier as in build_split_kernel.
#define PHASE __builtin_amdgcn_sched_barrier(0)
    auto advance = [&](int j) {
        PHASE;
        wait_vm<S2COPIES * (S2DT - 2), true>();
        __builtin_amdgcn_s_barrier();
        PHASE;
        issue(j + S2DT - 1);
        PHASE;
    };
    Frags f[2];
#pragma unroll
    for (int k = 0; k < S2DT; ++k) {
        issue(k);
        PHASE;
    }
    wait_vm<S2COPIES * (S2DT - 1), true>();   // t(0) landed
    __builtin_amdgcn_s_barrier();
    PHASE;
    read_lo(0, f[0]);
    read_hi(0, f[0]);
    PHASE;
#pragma unroll
    for (int kc = 0; kc < NK; ++kc) {
        mfma_lohi(f[kc & 1]);
        PHASE;
        advance(kc + 1);
        read_lo(kc + 1, f[(kc + 1) & 1]);
        PHASE;
        mfma_rest(f[kc & 1]);
        PHASE;
        read_hi(kc + 1, f[(kc + 1) & 1]);
        PHASE;
    }
#undef PHASE
    wait_vm<0, true>();
    __builtin_amdgcn_s_barrier();   // every wave is done with the chunk buffers (epilogue scratch)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) asm volatile("" : "+a"(acc[i][j]));
    if (th == 1 && !has1) return;   // odd n-tile count: the pair's second tile does not exist
    split_epilogue<MUL>(P, acc, smem + wave * (4 * 32 * XS), qg * 64, exq, ext + th * 128, fst + th * 128, tc, b,
                        q0, lane);
}

