// Lab record (round 3, not kept): lookup_pipe, a resident software-pipelined form of
// lookup_cols_reg (lookup.hip). Bitwise the same outputs, but 55.9 / 60.7 / 59.9 us vs 41.9 / 45.8 /
// 42.8 us on the smooth / sigma-3 / sigma-40 fields (168 VGPRs with spills whose reloads wait for
// every queued store; at 2 waves per SIMD without spills 52.0 / 55.2 / 53.9 us).
// It used resident_blocks() (hipOccupancyMaxActiveBlocksPerMultiprocessor) to size the grid.

// lookup_cols_reg as a software pipeline: a resident grid (4 workgroups per CU) walks the (query
// group, level, batch item) units with stride gridDim.x, and issues the window loads of its next
// unit into registers before it writes the outputs of the current one from LDS, so the loads'
// latency hides under the output stores instead of every workgroup paying load latency, then
// store time, in turn.  Per unit the arithmetic and the LDS image are lookup_cols_reg's (bitwise
// the same outputs).  Barriers per unit: origins of the next unit published (B1), the current
// windows retired (B2), the next windows published (B3); one LDS window buffer and one origin
// array suffice because each is rewritten only after the barrier that retires its readers.
template <int R, bool PAIR>
__global__ __launch_bounds__(192, 3) void lookup_pipe(LookupParams P, int units, int nqb) {
    constexpr int QB = kWave, NTQ = 3 * QB, K = 2 * R + 1, AP = K / 3;
    static_assert(K % 3 == 0, "one wave per part, whole columns per part");
    using WB = WindowBuf<R, QB, PAIR>;
    using SR = StageRegs<R, QB, NTQ, PAIR>;
    constexpr int SW = WB::SW, SP = WB::SP, KK = WB::KK;
    __shared__ WB st;
    const int tid = threadIdx.x, g = tid % QB;
    const int part = __builtin_amdgcn_readfirstlane(tid / QB);   // wave-uniform
    const int64_t Q = P.q_count;

    struct Unit { int lv, b, q0; };
    auto decode = [&](int u) {
        const int r = u / nqb;
        return Unit{r % P.levels, r / P.levels, (u - r * nqb) * QB};
    };
    // this thread's chains of one unit (lookup_cols_reg's phase 0) and its query's window origin;
    // origin() alone (4 chains) is what the staging of the unit needs, so the next unit's full
    // chains are formed only after the current unit's outputs (register pressure)
    struct Chains { float fy[K], wy[K], fx[AP], wx[AP]; int org[3]; };
    auto load_coords = [&](int u, float& cx, float& cy) {
        const Unit t = decode(u);
        const int p = t.q0 + g;
        if (p < P.q_count) {
            cx = P.coords[((int64_t)t.b * 2 + 0) * Q + p];
            cy = P.coords[((int64_t)t.b * 2 + 1) * Q + p];
        }
    };
    auto origin = [&](int u, float cxr, float cyr, int org[3]) {
        const Unit t = decode(u);
        const bool valid = t.q0 + g < P.q_count;
        float x0 = 0.0f, xl = 0.0f, y0 = 0.0f, yl = 0.0f, dummy;
        if (valid) {
            const float inv = 1.0f / (float)(1 << t.lv);  // coords / 2**i is an exact scaling
            const float cx = __fmul_rn(cxr, inv), cy = __fmul_rn(cyr, inv);
            const float wm1 = (float)(P.lw[t.lv] - 1), hm1 = (float)(P.lh[t.lv] - 1);
            coord_chain<R>(cx, 0, wm1, x0, dummy);
            coord_chain<R>(cx, K - 1, wm1, xl, dummy);
            coord_chain<R>(cy, 0, hm1, y0, dummy);
            coord_chain<R>(cy, K - 1, hm1, yl, dummy);
        }
        window_origin<WB::S, PAIR>(valid, x0, xl, y0, yl, org);
    };
    auto chains = [&](int u, float cxr, float cyr, Chains& c) {
        const Unit t = decode(u);
        if (t.q0 + g < P.q_count) {
            const float inv = 1.0f / (float)(1 << t.lv);
            const float cx = __fmul_rn(cxr, inv), cy = __fmul_rn(cyr, inv);
            const float wm1 = (float)(P.lw[t.lv] - 1), hm1 = (float)(P.lh[t.lv] - 1);
#pragma unroll
            for (int bb = 0; bb < K; ++bb) coord_chain<R>(cy, bb, hm1, c.fy[bb], c.wy[bb]);
#pragma unroll
            for (int ai = 0; ai < AP; ++ai) coord_chain<R>(cx, part * AP + ai, wm1, c.fx[ai], c.wx[ai]);
        }
    };
    auto publish_org = [&](const int org[3]) {
        if (part == 0) {
            st.org[g][0] = org[0];
            st.org[g][1] = org[1];
            st.org[g][2] = org[2];
        }
    };
    auto issue = [&](int u, SR& sr) {
        const Unit t = decode(u);
        stage_issue<R, QB, NTQ, PAIR>(st, P, t.lv, t.b, t.q0, tid, sr);
    };
    // lookup_cols_reg's phase 2 for unit u from the staged windows
    auto outputs = [&](int u, const Chains& c) {
        const Unit t = decode(u);
        const int md = c.org[2] & 0xff;
        if (md == 2) return;   // past the range
        const int p = t.q0 + g;
        const __amdgpu_buffer_rsrc_t orsrc = __builtin_amdgcn_make_buffer_rsrc(
            P.out + (int64_t)t.b * P.C * P.q_count, 0, P.C * P.q_count * 4, 0x00020000);
        const int voff = p * 4;
        const int sbase = t.lv * KK * P.q_count * 4;
        if (md == 0) {
            int yo[K];
#pragma unroll
            for (int bb = 0; bb < K; ++bb) yo[bb] = ((int)c.fy[bb] - c.org[1]) * SW;
            const float* wq = st.win + WB::W0 + g * SP;
#pragma unroll
            for (int ai = 0; ai < AP; ++ai) {
                const int a = part * AP + ai;
                const float* wc = wq + ((int)c.fx[ai] - c.org[0]);
#pragma unroll
                for (int bb = 0; bb < K; ++bb) {
                    const float* s = wc + yo[bb];
                    const float v = blend(s[0], s[1], s[SW], s[SW + 1], c.wx[ai], c.wy[bb]);
                    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), orsrc, voff,
                                                          sbase + (a * K + bb) * P.q_count * 4, 2);
                }
            }
        } else {   // coordinates that do not fit the window: exact direct gather
#pragma unroll
            for (int ai = 0; ai < AP; ++ai)
#pragma unroll
                for (int bb = 0; bb < K; ++bb) {
                    const float v = sample_direct(P, t.lv, t.b, p, c.fx[ai], c.fy[bb], c.wx[ai], c.wy[bb]);
                    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), orsrc, voff,
                                                          sbase + ((part * AP + ai) * K + bb) * P.q_count * 4, 2);
                }
        }
    };

    int u = blockIdx.x;   // the grid never exceeds the unit count
    const int G = gridDim.x;
    float cx = 0.0f, cy = 0.0f, cx2 = 0.0f, cy2 = 0.0f;   // coordinates of units u + G, u + 2G
    Chains cur;
    SR sr;
    load_coords(u, cx, cy);
    origin(u, cx, cy, cur.org);
    publish_org(cur.org);
    __syncthreads();
    issue(u, sr);
    chains(u, cx, cy, cur);
    if (u + G < units) load_coords(u + G, cx, cy);
    stage_commit<R, QB, NTQ, PAIR>(st, sr);
    __syncthreads();
    for (;;) {
        const int un = u + G;   // workgroup-uniform
        const bool more = un < units;
        int orgn[3];
        if (more) {
            origin(un, cx, cy, orgn);
            publish_org(orgn);
        }
        __syncthreads();   // B1: the next unit's origins
        if (more) {
            issue(un, sr);
            if (un + G < units) load_coords(un + G, cx2, cy2);
        }
        __builtin_amdgcn_sched_barrier(0);   // keep the outputs' LDS reads behind the loads
        outputs(u, cur);
        if (!more) break;
        __builtin_amdgcn_sched_barrier(0);
        chains(un, cx, cy, cur);
        cur.org[0] = orgn[0];
        cur.org[1] = orgn[1];
        cur.org[2] = orgn[2];
        cx = cx2;
        cy = cy2;
        __syncthreads();   // B2: every read of the current windows done
        stage_commit<R, QB, NTQ, PAIR>(st, sr);
        __syncthreads();   // B3: the next windows
        u = un;
    }
}

