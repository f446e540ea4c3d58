// ---- pipelined roles (rx_back): stage s of the wave pipeline works on call it - s in
//      iteration it; hand-offs through double-buffered LDS, one barrier per iteration ----
#define BACK_ROLE_LOOP(ST)                                                                     \
    for (int it = 0; it < l.calls + back_roles(DM) - 1; ++it)                                  \
    {                                                                                          \
        const int call = it - (ST);                                                            \
        if (call >= 0 && call < l.calls)                                                       \
        {
#define BACK_ROLE_END                                                                          \
        }                                                                                      \
        __syncthreads();                                                                       \
    }

template <int L, int DM>
__device__ __forceinline__ void rx_back_demod(const BackArgs& a, BackLds lds)
{
    const BackLane l(a);
    constexpr int NDC = BLK / L;
    DemodStage<L, DM> s;
    s.load(a, l);
    s.fetch(a, l, 0);
    BACK_ROLE_LOOP(0)
        s.begin(a, l, call);
        float* dout = lds.dem + (call & 1) * NDC * BACK_CH + l.lane;
#pragma unroll
        for (int m = 0; m < NDC; ++m) dout[m * BACK_CH] = s.step(m);
    BACK_ROLE_END
    s.store(a, l);
}

// IIR lattice pre-filter; input: rx_front's decimated I +- Q (SSB) or the demod role's output
template <int PRE, int L, int DM>
__device__ __forceinline__ void rx_back_pre(const BackArgs& a, BackLds lds)
{
    const BackLane l(a);
    constexpr int NDC = BLK / L;
    const uhsdr_rx_plan* __restrict__ P = a.plan;
    InStage<L> in;
    LatticeStage<PRE> s;
    s.load(l, P->pre_k, P->pre_v, a.s.pre);
    if (!DM) in.fetch(a, l, 0);
    BACK_ROLE_LOOP(DM ? 1 : 0)
        float xin[NDC];
        if (DM)
        {
            const float* di = lds.dem + (call & 1) * NDC * BACK_CH + l.lane;
#pragma unroll
            for (int m = 0; m < NDC; ++m) xin[m] = di[m * BACK_CH];
        }
        else
            in.begin(a, l, call, xin);
        float* po = lds.pre + (call & 1) * NDC * BACK_CH + l.lane;
#pragma unroll
        for (int m = 0; m < NDC; ++m) po[m * BACK_CH] = s.step(xin[m]);
    BACK_ROLE_END
    s.store(l, a.s.pre);
}

template <int L, int W, int DM>
__device__ __forceinline__ void rx_back_agc(const BackArgs& a, BackLds lds)
{
    const BackLane l(a);
    constexpr int NDC = BLK / L;
    const uhsdr_rx_plan* __restrict__ P = a.plan;
    const uhsdr_agc_plan A = P->agc;
    AgcStage<L, W> s;
    s.load(a, l, A);
    s.fetch(a, l, 0);
    BACK_ROLE_LOOP(DM ? 2 : 1)
        const float* pi = lds.pre + (call & 1) * NDC * BACK_CH + l.lane;
        float* ao = lds.agc + (call & 1) * NDC * BACK_CH + l.lane;
        s.begin(a, l, call);
#pragma unroll
        for (int m = 0; m < NDC; ++m) ao[m * BACK_CH] = s.step(m, pi[m * BACK_CH], l, A);
        s.end();
    BACK_ROLE_END
    s.store(a, l);
}

template <int L, int PH, int DM>
__device__ __forceinline__ void rx_back_audio(const BackArgs& a, BackLds lds)
{
    const BackLane l(a);
    constexpr int NDC = BLK / L;
    AudioStage<L, PH, DM> s;
    s.load(a, l);
    BACK_ROLE_LOOP(DM ? 3 : 2)
        const float* ai = lds.agc + (call & 1) * NDC * BACK_CH + l.lane;
        float* mo = lds.mid + (call & 1) * BLK * BACK_CH + l.lane;
#pragma unroll
        for (int m = 0; m < NDC; ++m)
        {
            float u[L];
            s.step(ai[m * BACK_CH], u);
#pragma unroll
            for (int j = 0; j < L; ++j) mo[(m * L + j) * BACK_CH] = u[j];
        }
        s.end(a, l, call);
    BACK_ROLE_END
    s.store(a, l);
}

// anti-alias lattice at 48 ksps
template <int AA, int DM>
__device__ __forceinline__ void rx_back_aa(const BackArgs& a, BackLds lds)
{
    const BackLane l(a);
    const uhsdr_rx_plan* __restrict__ P = a.plan;
    LatticeStage<AA> s;
    s.load(l, P->aa_k, P->aa_v, a.s.aa);
    BACK_ROLE_LOOP(DM ? 4 : 3)
        const float* mi = lds.mid + (call & 1) * BLK * BACK_CH + l.lane;
        float* mo = lds.aa + (call & 1) * BLK * BACK_CH + l.lane;
#pragma unroll 4
        for (int n = 0; n < BLK; ++n) mo[n * BACK_CH] = s.step(mi[n * BACK_CH]);
    BACK_ROLE_END
    s.store(l, a.s.aa);
}

template <int DM>
__device__ __forceinline__ void rx_back_output(const BackArgs& a, BackLds lds)
{
    const BackLane l(a);
    OutputStage s;
    s.load(a, l);
    BACK_ROLE_LOOP(DM ? 5 : 4)
        const float* mi = lds.aa + (call & 1) * BLK * BACK_CH + l.lane;
#pragma unroll 2
        for (int n0 = 0; n0 < BLK; n0 += 4)
        {
            float y[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) y[j] = s.step(mi[(n0 + j) * BACK_CH]);
            back_store4(a, l, call, n0, y);
        }
    BACK_ROLE_END
    s.store(a, l);
}
#undef BACK_ROLE_LOOP
#undef BACK_ROLE_END

// PRE / AA lattice stages, L interpolation factor, PH polyphase length, W AGC window,
// DM demodulator (DM_NONE: SSB/CW/DIGI)
template <int PRE, int AA, int L, int PH, int W, int DM>
__global__ void __launch_bounds__(6 * BACK_CH) rx_back(BackArgs a)
{
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const BackLds lds = back_lds_carve<BLK / L>(smem);
    // readfirstlane makes the role provably wave-uniform (scalar branches)
    const int role = __builtin_amdgcn_readfirstlane(threadIdx.x / BACK_CH) - (DM ? 1 : 0);
    if (role < 0)
        rx_back_demod<L, DM>(a, lds);
    else if (role == 0)
        rx_back_pre<PRE, L, DM>(a, lds);
    else if (role == 1)
        rx_back_agc<L, W, DM>(a, lds);
    else if (role == 2)
        rx_back_audio<L, PH, DM>(a, lds);
    else if (role == 3)
        rx_back_aa<AA, DM>(a, lds);
    else
        rx_back_output<DM>(a, lds);
}

// Fused back end for large batches: one wave per 64 channels runs every stage per sample with
// all state in registers -- no LDS, no barriers, no pipeline fill / drain.  With enough
// channels to keep every SIMD busy this beats the wave pipeline, whose only purpose is to
// shorten the per-call critical path when channels are few.
template <int PRE, int AA, int L, int PH, int W, int DM>
__global__ void __launch_bounds__(BACK_CH) rx_back_fused(BackArgs a)
{
    const BackLane l(a);
    constexpr int NDC = BLK / L;
    static_assert(L == 2 || L == 4, "4 output frames per 1 or 2 decimated samples");
    const uhsdr_rx_plan* __restrict__ P = a.plan;
    const uhsdr_agc_plan A = P->agc;
    DemodStage<L, DM> dm;
    InStage<L> in;
    LatticeStage<PRE> pre;
    AgcStage<L, W> ag;
    AudioStage<L, PH, DM> au;
    LatticeStage<AA> aa;
    OutputStage ou;
    if (DM) { dm.load(a, l); dm.fetch(a, l, 0); }
    else in.fetch(a, l, 0);
    pre.load(l, P->pre_k, P->pre_v, a.s.pre);
    ag.load(a, l, A);
    ag.fetch(a, l, 0);
    au.load(a, l);
    aa.load(l, P->aa_k, P->aa_v, a.s.aa);
    ou.load(a, l);
    for (int call = 0; call < l.calls; ++call)
    {
        float xin[NDC];
        if (DM)
        {
            dm.begin(a, l, call);
#pragma unroll
            for (int m = 0; m < NDC; ++m) xin[m] = dm.step(m);
        }
        else
            in.begin(a, l, call, xin);
        ag.begin(a, l, call);
        // the call's 32 output frames are stored in one burst at its end: interleaved with the
        // chain's arithmetic, the partial-line stores of 64 rows get evicted from L2 before
        // their lines fill, doubling the HBM write bytes
        float y[BLK];
#pragma unroll
        for (int m = 0; m < NDC; ++m)
        {
            float u[L];
            au.step(ag.step(m, pre.step(xin[m]), l, A), u);
#pragma unroll
            for (int j = 0; j < L; ++j) y[m * L + j] = ou.step(aa.step(u[j]));
        }
#pragma unroll
        for (int n0 = 0; n0 < BLK; n0 += 4)
        {
            const float y4[4] = { y[n0], y[n0 + 1], y[n0 + 2], y[n0 + 3] };
            back_store4(a, l, call, n0, y4);
        }
        ag.end();
        au.end(a, l, call);
    }
    if (DM) dm.store(a, l);
    pre.store(l, a.s.pre);
    ag.store(a, l);
    au.store(a, l);
    aa.store(l, a.s.aa);
    ou.store(a, l);
}
