// Batched arm_fir_f32 over channels (include/uhsdr.h, uhsdr_fir_*): every channel of the batch
// is one CMSIS FIR instance (FilteringFunctions/arm_fir_f32.c:482-560) with its own carried
// samples and the shared taps.  This is C5's long narrow filter (a
// synthetic 513-tap low-pass at 12 ksps; the firmware's own FIRs stop at 201 taps) and the
// north_star's "batched FIR as a GEMM on MFMA".  Two arithmetic modes:
//
//   UHSDR_FIR_EXACT  VALU, the reference's binary32 sequence (tap order from +0.0f, separate
//                    multiply and add): bit-identical to arm_fir_f32.
//   UHSDR_FIR_MFMA   the FIR as a GEMM on the matrix cores.  256 outputs of a channel form one
//                    16 x 16 tile Y[m][i] = y[16m + i] = sum_j X[m][j] Cm[j][i] with
//                    X[m][j] = w[16m + j] (overlapping rows of the channel's window) and the
//                    Toeplitz tap matrix Cm[j][i] = c[j - i] (zero outside 0..T-1), depth
//                    K = T + 15 rounded up to 16 (+3 % MACs at 513 taps), on
//                    v_mfma_f32_16x16x4_f32: each output the tap sum with every multiply-add
//                    fused, summed in a permuted tap order (fir_group), within ~1e-7 * sum|c x|
//                    of the reference's, not bit-identical (tests/test_gpu_fir.py: 1e-5
//                    relative, north_star's bar).
//
// Layout: one wave owns FIR_CPW = 4 channels (4 independent MFMA accumulators hide the
// 40-cycle dependent latency); each channel's window [T-1 carried | B new | 32 zero] sits in
// LDS (EXACT: one pad word per 16, fpad, so its lanes 16 samples apart hit distinct banks;
// MFMA: plain, for 16-byte aligned ds_read_b128 operand loads); the taps sit in LDS once per
// workgroup with 16 zeros on each side (MFMA: four copies, copy p shifted by p, so every lane's
// four consecutive B values start 16-byte aligned).  B % 256 == 0; a channel's block is
// B / 256 tiles.  HBM per channel and call: 4 B in + 4 B out per sample, the carried samples
// read and written once.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "uhsdr_internal.h"
#include "uhsdr_dsp.h"

namespace {

constexpr int FIR_TILE = 256;   // outputs of one 16 x 16 MFMA tile
constexpr int FIR_CPW = 4;      // EXACT: channels per wave
// MFMA: channels per wave and group.  One (one accumulator chain per wave, 16 waves per CU
// cover its 40-cycle dependent latency); two measured the same (0.355 vs 0.353 ms at C5, 12
// waves per CU, the B reads shared)
constexpr int FIR_MCPW = 1;

// MFMA window layout: float4 chunk u of a window sits at chunk u ^ 2 in odd 64-float rows
// (bit 4 of u set).  A lane's A fragment reads chunk 4(r + q) + kq; unswizzled, the 16 lanes of a
// ds_read_b128 group hit 8 bank quads twice (39 % of the LDS cycles were conflicts, PMC r04); with
// the swizzle they hit 16 distinct ones for every chunk q.  An involution within 16-float
// blocks: the glds fill writes physical chunk P from logical chunk swz(P).
__host__ __device__ constexpr int fir_swz(int i) { return i ^ ((i >> 3) & 8); }   // float index
constexpr int FIR_TAIL = 32;    // zero samples after a window (K round-up, EXACT chunk over-read)
constexpr int FIR_MTAIL = 64;   // MFMA: K round-up plus the operand prefetch two chunks past the last

typedef float f32x4 __attribute__((ext_vector_type(4)));

__host__ __device__ constexpr int fpad(int i) { return i + (i >> 4); }

struct FirArgs
{
    const float* taps;   // [T]
    float* hist;         // [C][T-1] carried samples (oldest first)
    const float* src;    // [C][B]
    float* dst;          // [C][B]
    int C, B, T, K;      // K: MFMA depth, T + 15 rounded up to 16
    int lw;              // LDS floats per channel window
    int cp;              // LDS floats of the tap copies (MFMA 4, EXACT 1)
    int cpl;             // floats per tap copy: copy p holds cp0[y - p], cp0[16 + k] = c[k], zeros around
    int v4;              // MFMA: 16-byte window fills (carried length % 4 == 0, block 16-byte aligned)
};

// EXACT: the tiles of one channel group from its LDS windows Wb (4 channels from c0)
__device__ __forceinline__ void fir_group(const FirArgs& a, const float* Wb, const float* cp, int c0, int lane)
{
    const int r = lane & 15, kq = lane >> 4;
    for (int t = 0; t < a.B / FIR_TILE; ++t)
    {
        const int base = FIR_TILE * t;
        {
            // lane (channel j = kq, block r): 16 consecutive outputs, a 32-sample register
            // window sliding 16 samples per 16-tap chunk, taps from LDS (VGPR operands)
            const int j = kq;
            const float* W = Wb + j * a.lw;
            const int o0 = base + 16 * r;
            float acc[16], win[32];
#pragma unroll
            for (int q = 0; q < 16; ++q) acc[q] = 0.0f;
#pragma unroll
            for (int q = 0; q < 16; ++q) win[q] = W[fpad(o0 + q)];
            const int nch = a.T / 16, tr = a.T % 16;
            for (int ch = 0; ch < nch; ++ch)
            {
                const int k0 = 16 * ch;
#pragma unroll
                for (int q = 0; q < 16; ++q) win[16 + q] = W[fpad(o0 + k0 + 16 + q)];
#pragma unroll
                for (int kk = 0; kk < 16; ++kk)
                {
                    const float ck = cp[16 + k0 + kk];
#pragma unroll
                    for (int q = 0; q < 16; ++q) acc[q] += win[q + kk] * ck;
                }
#pragma unroll
                for (int q = 0; q < 16; ++q) win[q] = win[16 + q];
            }
            {
                const int k0 = 16 * nch;
#pragma unroll
                for (int q = 0; q < 16; ++q) win[16 + q] = W[fpad(o0 + k0 + 16 + q)];
                for (int kk = 0; kk < tr; ++kk)
                {
                    const float ck = cp[16 + k0 + kk];
#pragma unroll
                    for (int q = 0; q < 16; ++q)
                    {
                        // runtime tap index: select the window sample without dynamic indexing
                        float x = win[q];
#pragma unroll
                        for (int s = 1; s < 16; ++s) x = kk == s ? win[q + s] : x;
                        acc[q] += x * ck;
                    }
                }
            }
            const int c = c0 + j;
            if (c < a.C)
            {
                float* d = a.dst + (size_t)c * a.B + o0;
#pragma unroll
                for (int q = 0; q < 16; q += 4) *(float4*)(d + q) = make_float4(acc[q], acc[q + 1], acc[q + 2], acc[q + 3]);
            }
        }
    }
}

// EXACT: one group per wave, windows filled straight from HBM (VALU-bound: the fill hides behind
// the other waves; a persistent form's prefetch registers cost it 20 %)
__global__ void __launch_bounds__(256) fir_batch_direct(FirArgs a)
{
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const int H = a.T - 1, n = H + a.B;
    float* cp = sm;                                   // cp[16 + k] = c[k], zeros around
    for (int i = threadIdx.x; i < a.cp; i += blockDim.x)
        cp[i] = (i >= 16 && i < 16 + a.T) ? a.taps[i - 16] : 0.0f;
    float* Wb = sm + a.cp + (size_t)w * FIR_CPW * a.lw;
    const int c0 = (blockIdx.x * nw + w) * FIR_CPW;
#pragma unroll
    for (int j = 0; j < FIR_CPW; ++j)
    {
        const int c = c0 + j;
        const int cl = c < a.C ? c : a.C - 1;
        const float* h = a.hist + (size_t)cl * H;
        const float* s = a.src + (size_t)cl * a.B;
        float* W = Wb + j * a.lw;
        for (int i = lane; i < n + FIR_TAIL; i += 64)
            W[fpad(i)] = i < H ? h[i] : (i < n ? s[i - H] : 0.0f);
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < FIR_CPW; ++j)
    {
        const int c = c0 + j;
        if (c < a.C)
        {
            const float* W = Wb + j * a.lw;
            for (int i = lane; i < H; i += 64) a.hist[(size_t)c * H + i] = W[fpad(i + a.B)];
        }
    }
    fir_group(a, Wb, cp, c0, lane);
}

// ---- MFMA ----
// One wave owns FIR_MCPW channels per group, persistent over groups; up to 16 waves per
// workgroup, one workgroup per CU (the waves' windows fill its LDS).  Windows [carried | block |
// zeros] (fir_swz layout) are double-buffered in LDS: the next group's windows stream in by
// global_load_lds (no VGPRs, no VALU) while this group's MFMAs run, and the only waits on HBM
// are for loads issued a whole group earlier.

// the glds fill of one window: SZ bytes per lane (16 when the carried length keeps float4s
// aligned, else 4); lanes past the data are masked off, so the slots after it keep their zeros
template <int SZ>
__device__ __forceinline__ void fir_fill_glds(float* W, const float* hrow, const float* srow, int H, int n, int lane)
{
    constexpr int F = SZ / 4, STEP = 64 * F;
    for (int k0 = 0; k0 < n; k0 += STEP)
    {
        const int e = fir_swz(k0 + lane * F);        // the logical sample this lane's slot holds
        const float* g = e < H ? hrow + e : srow + (e - H);
        const __attribute__((address_space(1))) void* gs = (const __attribute__((address_space(1))) void*)g;
        __attribute__((address_space(3))) void* ls = (__attribute__((address_space(3))) void*)(W + k0);
        if (e < n)
        {
            if constexpr (SZ == 16) __builtin_amdgcn_global_load_lds(gs, ls, 16, 0, 0);
            else __builtin_amdgcn_global_load_lds(gs, ls, 4, 0, 0);
        }
    }
}

// One 256-output tile per channel of the group.  A[m = r][k] = w[base + 16r + k], B[k][i = r] =
// c[k - i].  The MFMA's k-sum is a permutation away from any other, so in 16-deep chunk q lane
// (r, kq) takes k = 16q + 4kq + s in k-step s: its four A values are four consecutive window
// samples (one ds_read_b128 per channel for four k-steps) and its four B values four consecutive
// taps, read from tap copy p = r & 3 (shifted by p) where they start 16-byte aligned.  The
// operands of chunk q + 1 load into the other register set while chunk q's MFMAs run.
__device__ __forceinline__ void fir_tile(const FirArgs& a, const float* Wg, const float* cp, int base, int lane,
                                         f32x4 (&acc)[FIR_MCPW])
{
    static_assert(FIR_MCPW == 1, "one window per wave");
    const int r = lane & 15, kq = lane >> 4;
    const int ai = base + 16 * r + 4 * kq;           // logical window index of chunk 0's A values
    // fir_swz flips bit 3 of a window index by its bit 6, so the layout repeats every 128 floats:
    // chunk 8t + k of this lane sits at aoff[k] + 128 t from pa
    const float* pa = Wg + ai;
    int aoff[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) aoff[k] = fir_swz(ai + 16 * k) - ai;
    const float* bp = cp + (r & 3) * a.cpl + 16 + 4 * kq - 4 * (r >> 2);
    const int nq = a.K / 16;
    // one accumulator chain per wave: 16 waves per CU cover its 40-cycle dependent latency (two
    // alternating accumulators measured the same, 0.351 vs 0.345 ms)
    acc[0] = f32x4{ 0.0f, 0.0f, 0.0f, 0.0f };
    // Four operand sets in rotation: chunk q + 2's loads are issued as chunk q's MFMAs start, two
    // chunks before their use, so the wait before a chunk leaves the next set in flight (explicit
    // waits, which the compiler's waitcnt pass counts, and scheduling barriers keep it from
    // waiting on loads it has just issued).  Unrolled by the layout's 8-chunk period, every
    // address is a per-lane offset plus an immediate: one VALU add per chunk.  Reads past the
    // last chunk land in the window's zero tail and the tap copy's slack, unused.
    constexpr unsigned LGKM2 = 0xC07F | (2 << 8);    // s_waitcnt lgkmcnt(2) (vmcnt, expcnt: no wait)
    f32x4 av[4], bv[4];
    // chunk 8t + k (k may pass 7: the next period) from the period's pointers pt = pa + 128 t, bt
#define FIR_LOAD(SET, K, PT, BT)                                                                \
    av[SET] = *(const f32x4*)((PT) + aoff[(K) & 7] + 128 * ((K) >> 3));                         \
    bv[SET] = *(const f32x4*)((BT) + 16 * (K));
#define FIR_STEP(K, PT, BT)                                                                     \
    __builtin_amdgcn_s_waitcnt(LGKM2);                                                          \
    FIR_LOAD(((K) + 2) & 3, (K) + 2, PT, BT)                                                    \
    __builtin_amdgcn_sched_barrier(0);                                                          \
    acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[(K) & 3][0], bv[(K) & 3][0], acc[0], 0, 0, 0); \
    acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[(K) & 3][1], bv[(K) & 3][1], acc[0], 0, 0, 0); \
    acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[(K) & 3][2], bv[(K) & 3][2], acc[0], 0, 0, 0); \
    acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[(K) & 3][3], bv[(K) & 3][3], acc[0], 0, 0, 0); \
    __builtin_amdgcn_sched_barrier(0);
    const float* pt = pa;
    const float* bt = bp;
    FIR_LOAD(0, 0, pt, bt)
    __builtin_amdgcn_sched_barrier(0);
    FIR_LOAD(1, 1, pt, bt)
    __builtin_amdgcn_sched_barrier(0);
    int q = 0;
    for (; q + 8 <= nq; q += 8, pt += 128, bt += 128)
    {
        FIR_STEP(0, pt, bt) FIR_STEP(1, pt, bt) FIR_STEP(2, pt, bt) FIR_STEP(3, pt, bt)
        FIR_STEP(4, pt, bt) FIR_STEP(5, pt, bt) FIR_STEP(6, pt, bt) FIR_STEP(7, pt, bt)
    }
    const int rem = nq - q;                          // 0 .. 7 chunks left, the pipeline continues
    if (rem > 0) { FIR_STEP(0, pt, bt) }
    if (rem > 1) { FIR_STEP(1, pt, bt) }
    if (rem > 2) { FIR_STEP(2, pt, bt) }
    if (rem > 3) { FIR_STEP(3, pt, bt) }
    if (rem > 4) { FIR_STEP(4, pt, bt) }
    if (rem > 5) { FIR_STEP(5, pt, bt) }
    if (rem > 6) { FIR_STEP(6, pt, bt) }
#undef FIR_STEP
#undef FIR_LOAD
}

// D[row = 4 kq + i][col = r] of channel c0 + j's tile at `base` is output base + 16 row + col
__device__ __forceinline__ void fir_store_tile(const FirArgs& a, int c0, int base, int lane, const f32x4 (&acc)[FIR_MCPW])
{
    const int r = lane & 15, kq = lane >> 4;
#pragma unroll
    for (int j = 0; j < FIR_MCPW; ++j)
    {
        const int c = c0 + j;
        if (c >= a.C) continue;
        float* d = a.dst + (size_t)c * a.B + base + 64 * kq + r;
#pragma unroll
        for (int i = 0; i < 4; ++i) d[16 * i] = acc[j][i];
    }
}

__global__ void __launch_bounds__(1024) fir_mfma(FirArgs a)
{
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int lane = threadIdx.x & 63, nw = blockDim.x >> 6;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int H = a.T - 1, n = H + a.B;
    float* cp = sm;
    for (int i = threadIdx.x; i < a.cp; i += blockDim.x)
    {
        const int x = i % a.cpl - i / a.cpl - 16;    // copy i / cpl, shifted by its index
        cp[i] = (x >= 0 && x < a.T) ? a.taps[x] : 0.0f;
    }
    float* const Wb = sm + a.cp + (size_t)w * 2 * FIR_MCPW * a.lw;   // [buffer][channel][lw]
    for (int i = lane; i < 2 * FIR_MCPW * a.lw; i += 64) Wb[i] = 0.0f;
    __syncthreads();                                  // taps ready, windows zeroed
    const bool v4 = a.v4 != 0;
    const int ng = (a.C + FIR_MCPW - 1) / FIR_MCPW;
    const int nwt = gridDim.x * nw;
    auto fill = [&](int g, int buf) {
#pragma unroll
        for (int j = 0; j < FIR_MCPW; ++j)
        {
            const int c = g * FIR_MCPW + j;
            const int cl = c < a.C ? c : a.C - 1;
            float* W = Wb + (buf * FIR_MCPW + j) * a.lw;
            if (v4) fir_fill_glds<16>(W, a.hist + (size_t)cl * H, a.src + (size_t)cl * a.B, H, n, lane);
            else fir_fill_glds<4>(W, a.hist + (size_t)cl * H, a.src + (size_t)cl * a.B, H, n, lane);
        }
    };
    int g = blockIdx.x * nw + w, buf = 0;
    if (g < ng) fill(g, 0);
    // the last tile's outputs are stored one group later, after that group's wait: the wait then
    // never covers stores issued just before it
    f32x4 last[FIR_MCPW];
    int last_c0 = -1;
    for (; g < ng; g += nwt, buf ^= 1)
    {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this group's windows have landed
        if (g + nwt < ng) fill(g + nwt, buf ^ 1);
        if (last_c0 >= 0) fir_store_tile(a, last_c0, a.B - FIR_TILE, lane, last);
        const float* Wg = Wb + buf * FIR_MCPW * a.lw;
        const int c0 = g * FIR_MCPW;
        // the next call's carried samples: window [B, B + H)
#pragma unroll
        for (int j = 0; j < FIR_MCPW; ++j)
        {
            const int c = c0 + j;
            if (c >= a.C) continue;
            const float* W = Wg + j * a.lw + a.B;
            float* hr = a.hist + (size_t)c * H;
            if (v4)   // B % 256 == 0: window chunks of the carried samples stay whole
                for (int i = 4 * lane; i < H; i += 256) *(f32x4*)(hr + i) = *(const f32x4*)(W + fir_swz(a.B + i) - a.B);
            else
                for (int i = lane; i < H; i += 64) hr[i] = W[fir_swz(a.B + i) - a.B];
        }
        for (int t = 0; t < a.B / FIR_TILE; ++t)
        {
            f32x4 acc[FIR_MCPW];
            fir_tile(a, Wg, cp, FIR_TILE * t, lane, acc);
            if (t + 1 < a.B / FIR_TILE) fir_store_tile(a, c0, FIR_TILE * t, lane, acc);
            else
            {
#pragma unroll
                for (int j = 0; j < FIR_MCPW; ++j) last[j] = acc[j];
            }
        }
        last_c0 = c0;
        // every lane's LDS reads of this buffer are done before the fill two groups on reuses it
        wave_sync();
    }
    if (last_c0 >= 0) fir_store_tile(a, last_c0, a.B - FIR_TILE, lane, last);
}

// ---- MFMA, the taps' B fragments in registers (round 5) ----
// The B operand of chunk q (four consecutive taps per lane, the Toeplitz tile's columns) is the same
// for every tile of every channel: a wave loads its NQ fragments once and keeps them in registers
// (4 NQ floats per lane, AGPRs or VGPRs), so a chunk reads only its A fragment from LDS -- one
// ds_read_b128 per four MFMAs instead of two.  The register budget allows two waves per SIMD (8 per
// workgroup, one workgroup per CU).  For fir_mfma's 2,332 LDS reads per wave at 80 % of its cycles
// waiting (PMC r04).  NQ = K / 16 is a template parameter: C5's 513 taps, K = 528.
constexpr int FIR_RB_NQ = 33;
#ifndef UHSDR_FIR_RB_WAVES
#define UHSDR_FIR_RB_WAVES 8
#endif
constexpr int FIR_RB_WAVES = UHSDR_FIR_RB_WAVES;

// CH channels per wave (their windows lw floats apart), one accumulator chain each, interleaved
// per k-step: the 40-cycle dependent latency of v_mfma_f32_16x16x4_f32 (32-cycle issue,
// MI355X_MICROARCH.md) is covered by the other chain instead of the other wave.
#ifndef UHSDR_FIR_RB_CH
#define UHSDR_FIR_RB_CH 1
#endif
constexpr int FIR_RB_CH = UHSDR_FIR_RB_CH;

template <int NQ, int CH>
__device__ __forceinline__ void fir_tile_rb(const float* Wg, int lw, int base, int lane, const f32x4 (&bq)[NQ], f32x4 (&acc)[CH])
{
    const int r = lane & 15, kq = lane >> 4;
    const int ai = base + 16 * r + 4 * kq;
    const float* pa[CH];
#pragma unroll
    for (int j = 0; j < CH; ++j) pa[j] = Wg + j * lw + ai;
    int aoff[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) aoff[k] = fir_swz(ai + 16 * k) - ai;
#pragma unroll
    for (int j = 0; j < CH; ++j) acc[j] = f32x4{ 0.0f, 0.0f, 0.0f, 0.0f };
#ifndef UHSDR_FIR_RB_AHEAD
#define UHSDR_FIR_RB_AHEAD 2
#endif
    // A fragments load AH chunks ahead (CH (AH - 1) loads in flight while a chunk's MFMAs run)
    constexpr int AH = UHSDR_FIR_RB_AHEAD;
    constexpr unsigned LGKMW = 0xC07F | ((CH * (AH - 1)) << 8);   // s_waitcnt lgkmcnt(CH (AH - 1))
    f32x4 av[4][CH];
#pragma unroll
    for (int q = 0; q < AH; ++q)
    {
#pragma unroll
        for (int j = 0; j < CH; ++j) av[q][j] = *(const f32x4*)(pa[j] + aoff[q]);
        __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q)
    {
        // chunk q's A fragments have landed (the next AH - 1 chunks' may still be in flight)
        if (q + AH <= NQ) __builtin_amdgcn_s_waitcnt(LGKMW);
        else __builtin_amdgcn_s_waitcnt(0xC07F);
        if (q + AH < NQ)
        {
#pragma unroll
            for (int j = 0; j < CH; ++j)
                av[(q + AH) & 3][j] = *(const f32x4*)(pa[j] + aoff[(q + AH) & 7] + 128 * ((q + AH) >> 3));
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int s = 0; s < 4; ++s)
        {
#pragma unroll
            for (int j = 0; j < CH; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[q & 3][j][s], bq[q][s], acc[j], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
}

template <int CH>
__device__ __forceinline__ void fir_store_tile_rb(const FirArgs& a, int c0, int base, int lane, const f32x4 (&acc)[CH])
{
    const int r = lane & 15, kq = lane >> 4;
#pragma unroll
    for (int j = 0; j < CH; ++j)
    {
        const int c = c0 + j;
        if (c >= a.C) continue;
        float* d = a.dst + (size_t)c * a.B + base + 64 * kq + r;
#pragma unroll
        for (int i = 0; i < 4; ++i) d[16 * i] = acc[j][i];
    }
}

template <int NQ, int CH>
__global__ void __launch_bounds__(64 * FIR_RB_WAVES) fir_mfma_rb(FirArgs a)
{
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int lane = threadIdx.x & 63, nw = blockDim.x >> 6;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int H = a.T - 1, n = H + a.B;
    float* cp = sm;
    for (int i = threadIdx.x; i < a.cp; i += blockDim.x)
    {
        const int x = i % a.cpl - i / a.cpl - 16;
        cp[i] = (x >= 0 && x < a.T) ? a.taps[x] : 0.0f;
    }
    float* const Wb = sm + a.cp + (size_t)w * 2 * CH * a.lw;     // [buffer][channel][lw]
    for (int i = lane; i < 2 * CH * a.lw; i += 64) Wb[i] = 0.0f;
    __syncthreads();
    // the wave's B fragments, chunk q at bp + 16 q (fir_tile's layout)
    f32x4 bq[NQ];
    {
        const int r = lane & 15, kq = lane >> 4;
        const float* bp = cp + (r & 3) * a.cpl + 16 + 4 * kq - 4 * (r >> 2);
#pragma unroll
        for (int q = 0; q < NQ; ++q) bq[q] = *(const f32x4*)(bp + 16 * q);
    }
    const bool v4 = a.v4 != 0;
    const int ng = (a.C + CH - 1) / CH;
    const int nwt = gridDim.x * nw;
    auto fill = [&](int g, int buf) {
#pragma unroll
        for (int j = 0; j < CH; ++j)
        {
            const int c = g * CH + j;
            const int cl = c < a.C ? c : a.C - 1;
            float* W = Wb + (buf * CH + j) * a.lw;
            if (v4) fir_fill_glds<16>(W, a.hist + (size_t)cl * H, a.src + (size_t)cl * a.B, H, n, lane);
            else fir_fill_glds<4>(W, a.hist + (size_t)cl * H, a.src + (size_t)cl * a.B, H, n, lane);
        }
    };
    int g = blockIdx.x * nw + w, buf = 0;
    if (g < ng) fill(g, 0);
    f32x4 last[CH];
    int last_c0 = -1;
    for (; g < ng; g += nwt, buf ^= 1)
    {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (g + nwt < ng) fill(g + nwt, buf ^ 1);
        if (last_c0 >= 0) fir_store_tile_rb<CH>(a, last_c0, a.B - FIR_TILE, lane, last);
        const float* Wg = Wb + buf * CH * a.lw;
        const int c0 = g * CH;
#pragma unroll
        for (int j = 0; j < CH; ++j)
        {
            if (c0 + j >= a.C) continue;
            const float* W = Wg + j * a.lw + a.B;
            float* hr = a.hist + (size_t)(c0 + j) * H;
            if (v4)
                for (int i = 4 * lane; i < H; i += 256) *(f32x4*)(hr + i) = *(const f32x4*)(W + fir_swz(a.B + i) - a.B);
            else
                for (int i = lane; i < H; i += 64) hr[i] = W[fir_swz(a.B + i) - a.B];
        }
        for (int t = 0; t < a.B / FIR_TILE; ++t)
        {
            f32x4 acc[CH];
            fir_tile_rb<NQ, CH>(Wg, a.lw, FIR_TILE * t, lane, bq, acc);
            if (t + 1 < a.B / FIR_TILE) fir_store_tile_rb<CH>(a, c0, FIR_TILE * t, lane, acc);
            else
            {
#pragma unroll
                for (int j = 0; j < CH; ++j) last[j] = acc[j];
            }
        }
        last_c0 = c0;
        wave_sync();
    }
    if (last_c0 >= 0) fir_store_tile_rb<CH>(a, last_c0, a.B - FIR_TILE, lane, last);
}

} // namespace

constexpr size_t LDS_PER_CU = 160 * 1024;        // MI355X_MICROARCH.md §LDS

struct uhsdr_fir_s
{
    int C, B, T, K, mode, lw, cp, cpl, waves, grid;
    int rb;                  // MFMA with the B fragments in registers (fir_mfma_rb; K == 16 FIR_RB_NQ)
    hipStream_t stream;
    float* taps;
    float* hist;
};

#define HIPCHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { uhsdr_set_error("%s: %s", #x, hipGetErrorString(e_)); return UHSDR_DEVICE_ERROR; } } while (0)

// the workgroup's LDS: tap copies + per wave its windows (MFMA: two buffers of FIR_MCPW)
static size_t fir_lds(const uhsdr_fir_s* h, int waves)
{
    const size_t per_wave = h->mode == UHSDR_FIR_MFMA ? 2 * (h->rb ? FIR_RB_CH : FIR_MCPW) : FIR_CPW;
    return sizeof(float) * ((size_t)h->cp + (size_t)waves * per_wave * h->lw);
}

extern "C" uhsdr_status uhsdr_fir_destroy(uhsdr_fir_handle h)
{
    if (!h) return UHSDR_ARGUMENT_ERROR;
    if (h->taps) (void)hipFree(h->taps);
    if (h->hist) (void)hipFree(h->hist);
    free(h);
    return UHSDR_OK;
}

extern "C" uhsdr_status uhsdr_fir_reset(uhsdr_fir_handle h)
{
    if (!h) return UHSDR_ARGUMENT_ERROR;
    if (h->T > 1) HIPCHK(hipMemsetAsync(h->hist, 0, sizeof(float) * (size_t)h->C * (h->T - 1), h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    return UHSDR_OK;
}

// waves per workgroup and the launch grid for them.  strict: the exact count or an error;
// otherwise halved until the workgroup's LDS fits.
static uhsdr_status fir_configure(uhsdr_fir_s* h, int waves, bool strict)
{
    const bool mf = h->mode == UHSDR_FIR_MFMA;
    const int wmax = h->rb ? FIR_RB_WAVES : 16;
    if (mf ? (waves < 1 || waves > wmax) : (waves != 1 && waves != 2 && waves != 4))
    {
        uhsdr_set_error("waves per workgroup %d not %s", waves, mf ? (h->rb ? "1 .. 8" : "1 .. 16") : "1, 2 or 4");
        return UHSDR_ARGUMENT_ERROR;
    }
    // MFMA: one workgroup may hold the whole CU's LDS (MI355X_MICROARCH.md §LDS)
    const size_t cap = mf ? LDS_PER_CU : 64 * 1024;
    if (!strict)
        while (waves > 1 && fir_lds(h, waves) > cap) waves = mf ? waves - 1 : waves / 2;
    if (fir_lds(h, waves) > cap)
    {
        uhsdr_set_error("num_taps - 1 + block_size %d too long for %d waves per workgroup", h->T - 1 + h->B, waves);
        return UHSDR_LENGTH_ERROR;
    }
    // the attribute belongs to the kernel, not to this handle: raise it once to the whole CU's LDS,
    // so a later handle of another shape never lowers the cap an earlier handle launches with
    const void* kfn = h->rb ? (const void*)fir_mfma_rb<FIR_RB_NQ, FIR_RB_CH> : (const void*)fir_mfma;
    if (mf && fir_lds(h, waves) > 64 * 1024 &&
        hipFuncSetAttribute(kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS_PER_CU) != hipSuccess)
    {
        uhsdr_set_error("cannot raise the MFMA FIR kernel's LDS to %zu bytes", (size_t)LDS_PER_CU);
        return UHSDR_DEVICE_ERROR;
    }
    // persistent grid: as many workgroups as the CUs hold at once (LDS-limited), each wave
    // walking channel groups
    int dev = 0, cus = 256;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
        cus = prop.multiProcessorCount;
    const size_t lds = fir_lds(h, waves);
    int per_cu = (int)(LDS_PER_CU / lds);
    const int thread_cap = 2048 / (64 * waves);
    if (per_cu > thread_cap) per_cu = thread_cap;
    if (mf)
    {
        // the register file may admit fewer workgroups than the LDS: a persistent grid larger than
        // what is resident would leave its last workgroups to run after the others
        int occ = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kfn, 64 * waves, lds) == hipSuccess && occ > 0 && occ < per_cu)
            per_cu = occ;
    }
    if (per_cu < 1) per_cu = 1;
    const int cpg = h->mode == UHSDR_FIR_MFMA ? FIR_MCPW : FIR_CPW;
    const int groups = (h->C + cpg - 1) / cpg;
    const int need = (groups + waves - 1) / waves;
    // MFMA: persistent (fir_mfma); EXACT: fir_batch_direct, one group per wave (0.99 ms; 1.20 in
    // a persistent form)
    h->waves = waves;
    h->grid = (h->mode == UHSDR_FIR_MFMA && need > cus * per_cu) ? cus * per_cu : need;
    return UHSDR_OK;
}

extern "C" uhsdr_status uhsdr_fir_create(const float* coeffs, int32_t num_taps, int32_t num_channels, int32_t block_size,
                                         int32_t mode, void* stream, uhsdr_fir_handle* out)
{
    if (!coeffs || !out || num_taps <= 0 || num_channels <= 0 || block_size <= 0 ||
        (mode != UHSDR_FIR_EXACT && mode != UHSDR_FIR_MFMA))
    {
        uhsdr_set_error("bad argument");
        return UHSDR_ARGUMENT_ERROR;
    }
    if (block_size % FIR_TILE)
    {
        uhsdr_set_error("block_size %d not a multiple of %d", block_size, FIR_TILE);
        return UHSDR_LENGTH_ERROR;
    }
    *out = nullptr;
    uhsdr_fir_s* h = (uhsdr_fir_s*)calloc(1, sizeof(uhsdr_fir_s));
    if (!h) return UHSDR_DEVICE_ERROR;
    h->C = num_channels; h->B = block_size; h->T = num_taps; h->mode = mode;
    h->K = (num_taps + 15 + 15) & ~15;                 // MFMA depth: 16-deep chunks
    h->stream = (hipStream_t)stream;
    const bool mf = mode == UHSDR_FIR_MFMA;
    // MFMA: a multiple of 16 floats (fir_swz permutes within 16-float blocks)
    h->lw = mf ? (num_taps - 1 + block_size + FIR_MTAIL + 15) & ~15 : (fpad(num_taps - 1 + block_size + FIR_TAIL) + 4) & ~3;
    h->cpl = h->K + FIR_MTAIL;
    h->cp = (mf ? 4 : 1) * h->cpl;
#ifndef UHSDR_FIR_NO_RB
    h->rb = mf && h->K == 16 * FIR_RB_NQ;
#endif
    // waves per workgroup: EXACT 2 (one group per wave, more resident waves per CU: C5 513-tap
    // 1.048 -> 0.927 ms per call); MFMA as many as one workgroup's LDS holds, up to 16 (one
    // persistent workgroup per CU); uhsdr_fir_set_waves picks the count explicitly
    const uhsdr_status st = fir_configure(h, mode == UHSDR_FIR_MFMA ? (h->rb ? FIR_RB_WAVES : 16) : 2, false);
    if (st != UHSDR_OK)
    {
        free(h);
        return st;
    }
    hipError_t e = hipMalloc((void**)&h->taps, sizeof(float) * num_taps);
    if (e == hipSuccess)
        e = hipMalloc((void**)&h->hist, sizeof(float) * (size_t)num_channels * (num_taps > 1 ? num_taps - 1 : 1));
    if (e == hipSuccess) e = hipMemcpy(h->taps, coeffs, sizeof(float) * num_taps, hipMemcpyHostToDevice);
    if (e != hipSuccess)
    {
        uhsdr_set_error("device allocation failed: %s", hipGetErrorString(e));
        uhsdr_fir_destroy(h);
        return UHSDR_DEVICE_ERROR;
    }
    *out = h;
    return uhsdr_fir_reset(h);
}

extern "C" uhsdr_status uhsdr_fir_process(uhsdr_fir_handle h, const float* src, float* dst)
{
    if (!h || !src || !dst) { uhsdr_set_error("null argument"); return UHSDR_ARGUMENT_ERROR; }
    FirArgs a;
    a.taps = h->taps; a.hist = h->hist; a.src = src; a.dst = dst;
    a.C = h->C; a.B = h->B; a.T = h->T; a.K = h->K; a.lw = h->lw; a.cp = h->cp; a.cpl = h->cpl;
    // 16-byte window fills: carried rows and the caller's block 16-byte aligned
    a.v4 = (h->T - 1) % 4 == 0 && ((uintptr_t)src & 15) == 0;
    const dim3 grid(h->grid), block(64 * h->waves);
    if (h->mode == UHSDR_FIR_MFMA && h->rb)
        hipLaunchKernelGGL((fir_mfma_rb<FIR_RB_NQ, FIR_RB_CH>), grid, block, fir_lds(h, h->waves), h->stream, a);
    else if (h->mode == UHSDR_FIR_MFMA)
        hipLaunchKernelGGL(fir_mfma, grid, block, fir_lds(h, h->waves), h->stream, a);
    else
        hipLaunchKernelGGL(fir_batch_direct, grid, block, fir_lds(h, h->waves), h->stream, a);
    HIPCHK(hipGetLastError());
    return UHSDR_OK;
}

extern "C" uhsdr_status uhsdr_fir_set_waves(uhsdr_fir_handle h, int32_t waves)
{
    if (!h) { uhsdr_set_error("null handle"); return UHSDR_ARGUMENT_ERROR; }
    const int old = h->waves;
    const uhsdr_status st = fir_configure(h, waves, true);
    if (st != UHSDR_OK) fir_configure(h, old, true);
    return st;
}

extern "C" int32_t uhsdr_fir_get_waves(uhsdr_fir_handle h) { return h ? h->waves : 0; }

extern "C" uhsdr_status uhsdr_fir_synchronize(uhsdr_fir_handle h)
{
    if (!h) return UHSDR_ARGUMENT_ERROR;
    HIPCHK(hipStreamSynchronize(h->stream));
    return UHSDR_OK;
}
