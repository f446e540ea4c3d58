"""One-off source transformation: split the back-end stages for the 5-role wave pipeline."""
p = '/root/repo/uhsdr_amd/csrc/uhsdr_rx.hip'
s = open(p).read()

# ---- AgcStage: drop the lattice and the input fetch ----
old_hdr = s[s.index('// ---- agc stage: IIR lattice pre-filter'):s.index('    __device__ __forceinline__ void load(const BackArgs& a, const BackLane& l, const uhsdr_agc_plan& A)')]
new_hdr = '''// ---- input stage (SSB / CW / DIGI): rx_front's decimated I +- Q, fetched one call ahead ----
template <int L>
struct InStage
{
    static constexpr int NDC = BLK / L;
    float xnext[NDC];

    __device__ __forceinline__ void fetch(const BackArgs& a, const BackLane& l, int call)
    {
        const float* src = a.adec + (size_t)l.cl * a.Nd + call * NDC;
#pragma unroll
        for (int m = 0; m < NDC; m += 4)
        {
            const float4 v = *(const float4*)(src + m);
            xnext[m] = v.x; xnext[m + 1] = v.y; xnext[m + 2] = v.z; xnext[m + 3] = v.w;
        }
    }

    __device__ __forceinline__ void begin(const BackArgs& a, const BackLane& l, int call, float (&xin)[NDC])
    {
#pragma unroll
        for (int m = 0; m < NDC; ++m) xin[m] = xnext[m];
        if (call + 1 < l.calls) fetch(a, l, call + 1);
    }
};

// ---- IIR lattice (arm_iir_lattice_f32): the pre-filter on a_buffer[0] at the decimated rate
//      (IIR_PreFilter, audio_driver.c:2473-2482) or the anti-alias filter at 48 ksps
//      (IIR_AntiAlias, :2581-2590); state [S][C] in `st` ----
template <int S>
struct LatticeStage
{
    float k[S > 0 ? S : 1], v[S + 1], g[S > 0 ? S : 1];

    __device__ __forceinline__ void load(const BackLane& l, const float* kc, const float* vc, const float* st)
    {
#pragma unroll
        for (int i = 0; i < S; ++i) k[i] = kc[i];
#pragma unroll
        for (int i = 0; i <= S; ++i) v[i] = vc[i];
#pragma unroll
        for (int i = 0; i < S; ++i) g[i] = st[i * l.C + l.cl];
    }

    __device__ __forceinline__ float step(float x)
    {
        if constexpr (S > 0) return lattice_step<S>(x, g, k, v);
        return x;
    }

    __device__ __forceinline__ void store(const BackLane& l, float* st)
    {
        if (!l.live) return;
#pragma unroll
        for (int i = 0; i < S; ++i) st[i * l.C + l.c] = g[i];
    }
};

// ---- agc stage: AudioAgc_RunAgcWdsp (audio_agc.c:349-595) on the pre-filtered samples ----
template <int L, int W>
struct AgcStage
{
    static constexpr int NDC = BLK / L;
    static_assert(W == AGC_Q * NDC + 1, "AGC window must be AGC_Q calls + 1 sample");
    // The AGC plan values live in the caller's local copy of P->agc, passed to step() (uniform
    // -> SGPRs; reading them through P inside the loop would reload them every sample since the
    // state stores may alias, and a struct member copy of it defeats SROA and lands in scratch).
    bool agc_on;
    float volts, save_volts, fast_bavg, hang_bavg, wold;
    float cmax[AGC_Q - 1];                               // maxima of calls k-Q+1 .. k-1 (oldest first)
    float leave_last;                                    // last sample of call k-Q-1
    int hang_counter, decay_type, state;
    float rnext[NDC];                                    // ring slot of the next call
    float old[NDC], sfx[NDC], wmax, pmax;                // this call's ring slot, suffix maxima
    float* ring_out;

'''
s = s.replace(old_hdr, new_hdr)


def sub(old, new):
    global s
    assert old in s, old[:80]
    s = s.replace(old, new)


sub('''    __device__ __forceinline__ void load(const BackArgs& a, const BackLane& l, const uhsdr_agc_plan& A)
    {
        const uhsdr_rx_plan* __restrict__ P = a.plan;
        const int C = l.C, cl = l.cl;
#pragma unroll
        for (int i = 0; i < PRE; ++i) pk[i] = P->pre_k[i];
#pragma unroll
        for (int i = 0; i <= PRE; ++i) pv[i] = P->pre_v[i];
#pragma unroll
        for (int i = 0; i < PRE; ++i) pre[i] = a.s.pre[i * C + cl];
        agc_on = A.mode != 5;''', '''    __device__ __forceinline__ void load(const BackArgs& a, const BackLane& l, const uhsdr_agc_plan& A)
    {
        const int C = l.C, cl = l.cl;
        agc_on = A.mode != 5;''')

sub('''    // the decimated input and the ring slot of a call are fetched one call ahead
    __device__ __forceinline__ void fetch(const BackArgs& a, const BackLane& l, int call)
    {
        if (!DM)
        {
            const float* src = a.adec + (size_t)l.cl * a.Nd + call * NDC;
#pragma unroll
            for (int m = 0; m < NDC; m += 4)
            {
                const float4 v = *(const float4*)(src + m);
                xnext[m] = v.x; xnext[m + 1] = v.y; xnext[m + 2] = v.z; xnext[m + 3] = v.w;
            }
        }
        if (agc_on)''', '''    // the ring slot of a call is fetched one call ahead
    __device__ __forceinline__ void fetch(const BackArgs& a, const BackLane& l, int call)
    {
        if (agc_on)''')

sub('''    // start of call `call`: take the fetched data (xin: SSB input; AM/SAM get theirs from the
    // demod stage), issue the next call's fetch, suffix maxima of call k-Q, maximum of the
    // whole calls k-Q+1 .. k-1
    __device__ __forceinline__ void begin(const BackArgs& a, const BackLane& l, int call, float (&xin)[NDC])
    {
#pragma unroll
        for (int m = 0; m < NDC; ++m) { if (!DM) xin[m] = xnext[m]; old[m] = rnext[m]; }''',
    '''    // start of call `call`: take the fetched ring slot, issue the next call's fetch, suffix
    // maxima of call k-Q, maximum of the whole calls k-Q+1 .. k-1
    __device__ __forceinline__ void begin(const BackArgs& a, const BackLane& l, int call)
    {
#pragma unroll
        for (int m = 0; m < NDC; ++m) old[m] = rnext[m];''')

sub('''    {
        if (PRE > 0) x = lattice_step<PRE>(x, pre, pk, pv);
        // ---- AudioAgc_RunAgcWdsp, audio_agc.c:349-595 ----''', '''    {
        // ---- AudioAgc_RunAgcWdsp, audio_agc.c:349-595 ----''')

sub('''        const int C = l.C, c = l.c;
#pragma unroll
        for (int i = 0; i < PRE; ++i) a.s.pre[i * C + c] = pre[i];
        a.s.agc[1 * C + c] = volts;''', '''        const int C = l.C, c = l.c;
        a.s.agc[1 * C + c] = volts;''')

# ---- OutputStage -> biquad_2 + line-out only ----
i0 = s.index('// ---- output stage: anti-alias lattice')
i1 = s.index('// four consecutive output frames n0..n0+3 of a call')
s = s[:i0] + '''// ---- output stage: biquad_2 (audio_driver.c:2832), line-out scale (:2860); f32 audio and
//      int32 codec frames (:2911-2923) by the caller ----
struct OutputStage
{
    float bq2[4], b2[5], lo;

    __device__ __forceinline__ void load(const BackArgs& a, const BackLane& l)
    {
        const uhsdr_rx_plan* __restrict__ P = a.plan;
#pragma unroll
        for (int i = 0; i < 5; ++i) b2[i] = P->biquad2[i];
#pragma unroll
        for (int i = 0; i < 4; ++i) bq2[i] = a.s.bq2[i * l.C + l.cl];
        lo = P->line_out_scale;
    }

    __device__ __forceinline__ float step(float v)
    {
        v = biquad_step(v, bq2[0], bq2[1], bq2[2], bq2[3], b2);
        return v * lo;
    }

    __device__ __forceinline__ void store(const BackArgs& a, const BackLane& l)
    {
        if (!l.live) return;
#pragma unroll
        for (int i = 0; i < 4; ++i) a.s.bq2[i * l.C + l.c] = bq2[i];
    }
};

''' + s[i1:]

# ---- pipelined roles + kernels: rewrite from the roles comment to rx_fm ----
i0 = s.index('// ---- pipelined roles (rx_back)')
i1 = s.index('// ------------------------------------------------------------------------------------\n// rx_fm: FM receive')
s = s[:i0] + open('/root/repo/tools/dev/back_roles5.hip').read() + '\n' + s[i1:]

# ---- LDS hand-off buffers ----
sub('''struct BackLds
{
    float* dem;   // [2][NDC][64]  demod -> agc
    float* agc;   // [2][NDC][64]  agc -> audio
    float* mid;   // [2][BLK][64]  audio -> output
};

template <int NDC>
__device__ __forceinline__ BackLds back_lds_carve(float* smem)
{
    BackLds l;
    l.mid = smem;
    l.agc = smem + 2 * BLK * BACK_CH;
    l.dem = l.agc + 2 * NDC * BACK_CH;
    return l;
}''', '''struct BackLds
{
    float* dem;   // [2][NDC][64]  demod -> pre
    float* pre;   // [2][NDC][64]  pre -> agc
    float* agc;   // [2][NDC][64]  agc -> audio
    float* mid;   // [2][BLK][64]  audio -> aa
    float* aa;    // [2][BLK][64]  aa -> output
};

// floats of the hand-off buffers (host: back_lds)
__host__ __device__ constexpr int back_lds_floats(int ndc) { return BACK_CH * 2 * (3 * ndc + 2 * BLK); }

template <int NDC>
__device__ __forceinline__ BackLds back_lds_carve(float* smem)
{
    BackLds l;
    l.mid = smem;
    l.aa = l.mid + 2 * BLK * BACK_CH;
    l.agc = l.aa + 2 * BLK * BACK_CH;
    l.pre = l.agc + 2 * NDC * BACK_CH;
    l.dem = l.pre + 2 * NDC * BACK_CH;
    return l;
}''')

sub('''__host__ __device__ constexpr int back_roles(int dm) { return dm == DM_FM ? 2 : dm ? 4 : 3; }''',
    '''__host__ __device__ constexpr int back_roles(int dm) { return dm == DM_FM ? 2 : dm ? 6 : 5; }''')

sub('''    return sizeof(float) * (size_t)BACK_CH * 2 * (BLK + 2 * (BLK / h->plan.interp_L));''',
    '''    return sizeof(float) * (size_t)back_lds_floats(BLK / h->plan.interp_L);''')

open(p, 'w').write(s)
print("patched")
