/*
 * Device DSP building blocks shared by the receive (uhsdr_rx.hip) and transmit (uhsdr_tx.hip)
 * kernels: the CMSIS-DSP f32 primitives restated in the reference's operation order
 * (arm_fir_f32 / arm_fir_decimate_f32 as register-window FIR blocks over LDS windows,
 * arm_iir_lattice_f32, arm_biquad_cascade_df1_f32) and the time-parallel FIR window plumbing
 * (history rows, lane map, LDS pitch model).
 */
#ifndef UHSDR_DSP_H
#define UHSDR_DSP_H

#include <hip/hip_runtime.h>
#include <stdint.h>
#include "uhsdr_internal.h"

#define BLK UHSDR_IQ_BLOCK_SIZE
#define IQ_BIT_SCALE_DOWN 0.0000152587890625f

// native 4-float vector: arrays of HIP's float4 (a struct with a union) loaded from global
// memory defeat SROA and end up in scratch
typedef float vf4 __attribute__((ext_vector_type(4)));

// acc[r] = sum_{k<T} c[k] * win[r*M + k], r < R; tap order k = 0..T-1 from +0.0f exactly as
// arm_fir_f32 / arm_fir_decimate_f32 (CMSIS .../arm_fir_f32.c:482-560).  `win` is the lane's
// first window sample in LDS (16-byte aligned); `c` the tap table in the plan (global, read
// with scalar loads: the index is wave-uniform).  Taps run in chunks of 8 and a final chunk
// of T % 8: the register window (WA samples, a multiple of 8) slides by 8 samples per chunk and
// the next 8 samples (two ds_read_b128) and taps are fetched before the current MACs, so the
// live set stays at R accumulators + one window; the chunk loop is unrolled by the window's
// rotation period, which turns the slide into register renaming.  Reads run up to FRONT_TAIL
// samples past the last one used.
// LDS load of V (4 or 2) consecutive floats into w[j..j+V)
template <int V, int N>
__device__ __forceinline__ void lds_vec(const float* p, float (&w)[N], int j)
{
    if (V == 4)
    {
        const float4 v = *(const float4*)p;
        w[j] = v.x; w[j + 1] = v.y; w[j + 2] = v.z; w[j + 3] = v.w;
    }
    else
    {
        const float2 v = *(const float2*)p;
        w[j] = v.x; w[j + 1] = v.y;
    }
}

// tap tables are read through the constant address space: wave-uniform indices then become
// scalar loads (SGPR operands for the MACs) instead of vector loads
typedef const __attribute__((address_space(4))) float ctaps_t;
__device__ __forceinline__ ctaps_t* as_taps(const float* p) { return (ctaps_t*)p; }

// One MAC of the FIR dot products.  F = false: the reference's binary32 sequence, a rounded
// multiply then a rounded add (CMSIS arm_fir_f32 built without contraction, SURVEY.md §8(c)
// c3-i).  F = true: one fused multiply-add (v_fma_f32 / v_pk_fma_f32) -- half the VALU issue of
// a FIR, one rounding per tap instead of two; within north_star's 1e-5 normwise tolerance of the
// reference (tests/test_gpu_fma.py), not bit-identical (UHSDR_PRECISION_FMA).
template <bool F, typename V>
__device__ __forceinline__ V fir_mac(V acc, V x, V c)
{
    if constexpr (F) return __builtin_elementwise_fma(x, c, acc);
    else return acc + x * c;
}

// V: LDS read width in floats (the lane base is 4V bytes aligned)
template <int T, int R, int M, int V = 4, bool F = false, bool TP = false>
__device__ __forceinline__ void fir_block(const float* win, ctaps_t* c, float (&acc)[R])
{
    constexpr int WA = (M * (R - 1) + 8 + 7) & ~7;
    constexpr int NCH = T / 8, TR = T % 8;           // full 8-tap chunks, then TR taps
    // unrolled by the window's rotation period (register renaming), or fully for short filters
    // (the decimators: a rolled loop of few MACs per chunk waited on each chunk's LDS and tap loads)
    constexpr int ROT = NCH <= 8 ? (NCH > 0 ? NCH : 1) : WA / 8 + 1;
    float w[WA];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = 0.0f;
#pragma unroll
    for (int j = 0; j < WA; j += V) lds_vec<V>(win + j, w, j);
    // TP: taps one chunk ahead (fir_block2); here the table is read up to 7 taps past T only in
    // the tail chunk, which it holds (the plan's decimator taps are UHSDR_MAX_DEC_TAPS = 96 long)
    float cn[8];
    if constexpr (TP)
    {
#pragma unroll
        for (int q = 0; q < 8; ++q) cn[q] = c[q];
    }
#pragma unroll ROT
    for (int ch = 0; ch < NCH; ++ch)
    {
        float cc[8];
        if constexpr (TP)
        {
#pragma unroll
            for (int q = 0; q < 8; ++q) cc[q] = cn[q];
#pragma unroll
            for (int q = 0; q < 8; ++q) cn[q] = c[8 * (ch + 1) + q];
        }
        else
        {
#pragma unroll
            for (int q = 0; q < 8; ++q) cc[q] = c[8 * ch + q];
        }
        float nw[8];
#pragma unroll
        for (int q = 0; q < 8; q += V) lds_vec<V>(win + 8 * ch + WA + q, nw, q);
#pragma unroll
        for (int kk = 0; kk < 8; ++kk)
        {
#pragma unroll
            for (int r = 0; r < R; ++r) acc[r] = fir_mac<F>(acc[r], w[r * M + kk], cc[kk]);
        }
#pragma unroll
        for (int j = 0; j < WA - 8; ++j) w[j] = w[j + 8];
#pragma unroll
        for (int q = 0; q < 8; ++q) w[WA - 8 + q] = nw[q];
    }
#pragma unroll
    for (int kk = 0; kk < TR; ++kk)
    {
        const float ck = TP ? cn[kk] : c[8 * NCH + kk];
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r] = fir_mac<F>(acc[r], w[r * M + kk], ck);
    }
}

// Two filters in one pass over an interleaved window {x0[n], x1[n]} -- the I and Q branches
// of a pair (Hilbert I / Q, or the I and Q decimators): acc[r] = { sum_k c0[k] * x0[rM+k],
// sum_k c1[k] * x1[rM+k] } with taps c[k] = {c0[k], c1[k]}.  Per element this is exactly the
// binary32 sequence of fir_block (tap order k = 0..T-1 from +0.0f, separate multiply and add),
// but each v_pk_mul_f32 / v_pk_add_f32 does two of them in one issue slot: packed f32 issues
// at the scalar VALU rate on gfx950 (tools/micro/pk_rate.hip: 4.3 vs 4.1 cycles per wave
// instruction), so a FIR pair costs half the VALU time of two fir_block calls.
typedef float v2f __attribute__((ext_vector_type(2)));
typedef const __attribute__((address_space(4))) v2f ctaps2_t;
__device__ __forceinline__ ctaps2_t* as_taps2(const float* p) { return (ctaps2_t*)p; }

// Padded pair window (pass 1 of the one- and two-channel-per-wave front shapes, R = 8 outputs per
// lane): PB floats after every 8 pairs.  Lane bases then lie 16 + PB floats apart, so the 16 lanes
// of a ds_read_b128 group hit 16 distinct bank quads at PB = 4 (20-float stride) instead of 4 of
// them at 16 floats (one channel: 74 % of the front's LDS cycles were conflicts, PMC r03).  A
// register-window read (2 pairs, even pair index) never straddles a pad, so its offset is the lane
// base plus a compile-time constant.
template <int PB>
__host__ __device__ constexpr int pwin_off(int i) { return 2 * i + PB * (i >> 3); }
// the front's pass-1 padding (floats per 8 pairs) for a family: R outputs per lane, decimate-first,
// decimation M (1: FM)
__host__ __device__ constexpr int front_pad1(int R, bool decim_first, int M) { return R == 8 && (decim_first || M == 1) ? 4 : 0; }

// PB: the window's pad floats per 8 pairs (pwin_off); win is the lane's first window pair, which
// starts an 8-pair block when PB > 0
// TP: the next chunk's taps are loaded one chunk ahead (SGPRs carried across the loop), so a wave
// that runs alone on its SIMD does not wait on the scalar loads at every chunk (SMEM and LDS share
// lgkmcnt: the wait for a chunk's taps also drained its window prefetch); rx_stream's front
template <int T, int R, int M, bool F = false, int PB = 0, bool TP = false>
__device__ __forceinline__ void fir_block2(const float* win, ctaps2_t* c, v2f (&acc)[R])
{
    constexpr int WA = (M * (R - 1) + 8 + 7) & ~7;   // window pairs in registers
    constexpr int NCH = T / 8, TR = T % 8;           // full 8-tap chunks, then TR taps
    constexpr int ROT = WA / 8 + 1;                  // chunks until the window registers repeat
    v2f w[WA];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = v2f{ 0.0f, 0.0f };
#pragma unroll
    for (int j = 0; j < WA; j += 2)
    {
        const vf4 v = *(const vf4*)(win + pwin_off<PB>(j));
        w[j] = v.xy; w[j + 1] = v.zw;
    }
    v2f cn[8];
    if constexpr (TP)
    {
#pragma unroll
        for (int q = 0; q < 8; ++q) cn[q] = c[q];
    }
    // unrolled by the rotation period, the window slide is pure register renaming
#pragma unroll ROT
    for (int ch = 0; ch < NCH; ++ch)
    {
        v2f cc[8];
        if constexpr (TP)
        {
#pragma unroll
            for (int q = 0; q < 8; ++q) cc[q] = cn[q];
            // chunk ch + 1's taps (the table is zero-padded to a multiple of 8 taps: the last
            // chunk's look-ahead reads the tail chunk, or padding)
#pragma unroll
            for (int q = 0; q < 8; ++q) cn[q] = c[8 * (ch + 1) + q];
        }
        else
        {
#pragma unroll
            for (int q = 0; q < 8; ++q) cc[q] = c[8 * ch + q];
        }
        v2f nw[8];
#pragma unroll
        for (int q = 0; q < 8; q += 2)
        {
            // pair 8 ch + WA + q: block ch + (WA + q) / 8 (WA is a multiple of 8, q < 8)
            const vf4 v = *(const vf4*)(win + (16 + PB) * ch + pwin_off<PB>(WA + q));
            nw[q] = v.xy; nw[q + 1] = v.zw;
        }
#pragma unroll
        for (int kk = 0; kk < 8; ++kk)
        {
#pragma unroll
            for (int r = 0; r < R; ++r) acc[r] = fir_mac<F>(acc[r], w[r * M + kk], cc[kk]);
        }
#pragma unroll
        for (int j = 0; j < WA - 8; ++j) w[j] = w[j + 8];
#pragma unroll
        for (int q = 0; q < 8; ++q) w[WA - 8 + q] = nw[q];
    }
#pragma unroll
    for (int kk = 0; kk < TR; ++kk)
    {
        const v2f ck = TP ? cn[kk] : c[8 * NCH + kk];
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r] = fir_mac<F>(acc[r], w[r * M + kk], ck);
    }
}

// samples after the end of a window that the register-window FIRs read (never use): the last
// chunk's next-8 prefetch runs -R + 8*floor(T/8) + WA - T + 1 samples past the data, at most 8
// for every (T, R, M) instantiated here; zeroed all the same
constexpr int FRONT_TAIL = 8;

// LDS accesses of one wave are processed in order; the fences only stop the compiler from
// moving a lane's LDS access across a hand-off between lanes of the same wave.
// A wave-uniform value held in a VGPR: a VOP2 with an SGPR operand issues at half the rate of
// one with VGPR operands, and gfx9's one-SGPR-per-VALU-instruction limit plus a
// full SGPR file otherwise cost v_readlane refills of spilled SGPRs.  The asm keeps the compiler
// from folding the value back into an SGPR.
__device__ __forceinline__ float to_vgpr(float x)
{
    float r;
    asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "s"(x));
    return r;
}
template <int N>
__device__ __forceinline__ void to_vgpr(float (&x)[N])
{
#pragma unroll
    for (int i = 0; i < N; ++i) x[i] = to_vgpr(x[i]);
}

__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Workgroup barrier for LDS hand-offs between the waves of a pipeline: the writers' LDS
// operations complete (lgkmcnt(0)), then s_barrier.  __syncthreads() would also wait for every
// outstanding global load and store of the wave (its workgroup-scope fence emits vmcnt(0)): the
// next call's prefetched inputs and this call's output stores would then cost a full HBM round
// trip per pipeline step.  Only LDS data crosses waves here; global data stays wave-private.
__device__ __forceinline__ void lds_barrier()
{
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

constexpr int FRONT_WAVE = 64;
#define FRONT_WAVE_L 64

// history rows: HS = T-1 rounded up to 4 floats; lane b of a channel loads float4s b, b+nb, ...
__host__ __device__ constexpr int hist_stride(int T) { return (T - 1 + 3) & ~3; }
// float4s of a T-tap history row prefetched per lane (all of it when nb >= 8 lanes per channel;
// with fewer lanes the rest is loaded when the window is filled)
__host__ __device__ constexpr int hist_q(int T) { return (hist_stride(T) / 4 + 7) / 8; }


// history row of a T-tap filter for channel cl: lane b of nb loads float4s b, b+nb, ... (HQ per lane)
template <int T, int HQM>
__device__ __forceinline__ void front_load_row(const float* row, int cl, int b, int nb, vf4 (&buf)[HQM])
{
    constexpr int hs4 = hist_stride(T) / 4, HQ = hist_q(T);
    const vf4* h = (const vf4*)(row + (size_t)cl * (hs4 * 4));
#pragma unroll
    for (int i = 0; i < HQ; ++i)
    {
        const int q = b + nb * i;
        buf[i] = h[q < hs4 ? q : hs4 - 1];
    }
}

// One FIR pass's window: history row (registers) + NV new samples per lane, tail zeroed, and
// the history row of the next call (window samples nnew .. nnew+T-2) written back to HBM.
template <int T, int HQM>
__device__ __forceinline__ void front_fill(float* W, float* row, int c, bool act, bool live, int b, int nb,
                                           const vf4 (&buf)[HQM], const float* vals, int NV)
{
    constexpr int hs4 = hist_stride(T) / 4, HQ = hist_q(T);
    const int nnew = nb * NV;
    if (act)
    {
        // the row's pad floats (T-1 .. HS-1) land where the new samples go: written first,
        // overwritten below (one wave's LDS accesses are processed in order)
#pragma unroll
        for (int i = 0; i < HQ; ++i)
        {
            const int q = b + nb * i;
            if (q < hs4) *(vf4*)(W + 4 * q) = buf[i];
        }
        const vf4* h = (const vf4*)(row + (size_t)(live ? c : 0) * (hs4 * 4));
        for (int q = b + nb * HQ; q < hs4; q += nb) *(vf4*)(W + 4 * q) = h[q];
    }
    wave_sync();
    if (act)
    {
        for (int j = 0; j < NV; ++j) W[T - 1 + b * NV + j] = vals[j];
        for (int t = b; t < FRONT_TAIL; t += nb) W[T - 1 + nnew + t] = 0.0f;
    }
    wave_sync();
    float* ho = row + (size_t)c * (hs4 * 4);
    for (int q = b; q < hs4; q += nb)
    {
        const float4 v = *(const float4*)(W + nnew + 4 * q);
        if (live) *(float4*)(ho + 4 * q) = v;
    }
}

// front_fill for a FIR pair: the window holds interleaved pairs {x0[n], x1[n]} (8 bytes per
// sample) built from the two history rows (row0 / row1, prefetched as buf0 / buf1) and NV new
// pairs per lane; the next call's history rows are de-interleaved back to HBM.  DUP: both
// filters of the pair run on the same signal (the TX Hilbert pair): one row, written once.
template <int T, int HQM, bool DUP = false>
__device__ __forceinline__ void front_fill2(float* W, float* row0, float* row1, int c, bool act, bool live, int b,
                                            int nb, const vf4 (&buf0)[HQM], const vf4 (&buf1)[HQM],
                                            const v2f* vals, int NV)
{
    constexpr int hs4 = hist_stride(T) / 4, HQ = hist_q(T);
    const int nnew = nb * NV;
    if (act)
    {
        // pad samples (T-1 .. HS-1) land where the new samples go and are overwritten below
#pragma unroll
        for (int i = 0; i < HQ; ++i)
        {
            const int q = b + nb * i;
            if (q < hs4)
            {
                const vf4 x = buf0[i], y = buf1[i];
                *(vf4*)(W + 8 * q) = vf4{ x.x, y.x, x.y, y.y };
                *(vf4*)(W + 8 * q + 4) = vf4{ x.z, y.z, x.w, y.w };
            }
        }
        const size_t ro = (size_t)(live ? c : 0) * (hs4 * 4);
        const vf4* h0 = (const vf4*)(row0 + ro);
        const vf4* h1 = (const vf4*)(row1 + ro);
        for (int q = b + nb * HQ; q < hs4; q += nb)
        {
            const vf4 x = h0[q], y = h1[q];
            *(vf4*)(W + 8 * q) = vf4{ x.x, y.x, x.y, y.y };
            *(vf4*)(W + 8 * q + 4) = vf4{ x.z, y.z, x.w, y.w };
        }
    }
    wave_sync();
    if (act)
    {
        float* d = W + 2 * (T - 1 + b * NV);
        if constexpr (((T - 1) & 1) == 0)           // 16-byte aligned: two pairs per store
            for (int j = 0; j < NV; j += 2)
                *(vf4*)(d + 2 * j) = vf4{ vals[j].x, vals[j].y, vals[j + 1].x, vals[j + 1].y };
        else
            for (int j = 0; j < NV; ++j) *(v2f*)(d + 2 * j) = vals[j];
        for (int t = b; t < FRONT_TAIL; t += nb) *(v2f*)(W + 2 * (T - 1 + nnew + t)) = v2f{ 0.0f, 0.0f };
    }
    wave_sync();
    const size_t ro = (size_t)c * (hs4 * 4);
    for (int q = b; q < hs4; q += nb)
    {
        const vf4 p0 = *(const vf4*)(W + 2 * (nnew + 4 * q));
        const vf4 p1 = *(const vf4*)(W + 2 * (nnew + 4 * q) + 4);
        if (live)
        {
            *(vf4*)(row0 + ro + 4 * q) = vf4{ p0.x, p0.z, p1.x, p1.z };
            if (!DUP) *(vf4*)(row1 + ro + 4 * q) = vf4{ p0.y, p0.w, p1.y, p1.w };
        }
    }
}

// ---- group-coalesced history rows ----
// The CPW channels of a front wave own consecutive rows [c0, c0 + CPW) of a [C][HS] history array:
// one contiguous region of CPW * HS floats.  Lane l moves its float4s l, l + 64, ... of that region,
// so every wave instruction reads or writes whole 1 KB runs (the per-channel lane map would touch
// CPW partial 128-byte lines per instruction).  Float4 q of the region is channel q / (HS/4) at
// offset 4 * (q % (HS/4)) of its row.  HQ = hist_q(T) float4s per lane are prefetched; a wave with
// more than 64 * HQ float4s (fewer than 8 lanes per channel) loads the rest when it fills.
template <int T, int HQM>
__device__ __forceinline__ void group_load_rows(const float* row, int c0, int nlive, int lane, vf4 (&buf)[HQM])
{
    constexpr int hs4 = hist_stride(T) / 4, HQ = hist_q(T);
    const vf4* h = (const vf4*)(row + (size_t)c0 * (hs4 * 4));
    const int qmax = nlive * hs4 - 1;                    // loads clamped to the live channels' rows
#pragma unroll
    for (int i = 0; i < HQ; ++i)
    {
        const int q = lane + FRONT_WAVE_L * i;
        buf[i] = h[q < qmax ? q : qmax];
    }
}

// pass window of a FIR pair (interleaved {x0[n], x1[n]}): the history part from the two rows
template <int T, int HQM>
__device__ __forceinline__ void group_fill_rows2(float* smem, int LW, const float* row0, const float* row1, int c0,
                                                 int cpw, int nlive, int lane, const vf4 (&buf0)[HQM], const vf4 (&buf1)[HQM])
{
    constexpr int hs4 = hist_stride(T) / 4, HQ = hist_q(T);
    const int nq = cpw * hs4;
#pragma unroll
    for (int i = 0; i < HQ; ++i)
    {
        const int q = lane + FRONT_WAVE_L * i;
        if (q < nq)
        {
            float* d = smem + (q / hs4) * LW + 8 * (q % hs4);
            const vf4 x = buf0[i], y = buf1[i];
            *(vf4*)d = vf4{ x.x, y.x, x.y, y.y };
            *(vf4*)(d + 4) = vf4{ x.z, y.z, x.w, y.w };
        }
    }
    const vf4* h0 = (const vf4*)(row0 + (size_t)c0 * (hs4 * 4));
    const vf4* h1 = (const vf4*)(row1 + (size_t)c0 * (hs4 * 4));
    const int qmax = nlive * hs4 - 1;
    for (int q = lane + FRONT_WAVE_L * HQ; q < nq; q += FRONT_WAVE_L)
    {
        const int qs = q < qmax ? q : qmax;
        const vf4 x = h0[qs], y = h1[qs];
        float* d = smem + (q / hs4) * LW + 8 * (q % hs4);
        *(vf4*)d = vf4{ x.x, y.x, x.y, y.y };
        *(vf4*)(d + 4) = vf4{ x.z, y.z, x.w, y.w };
    }
}

// the next call's history rows (window samples nnew .. nnew + T - 2 of each channel) back to HBM,
// de-interleaved; DUP: one row only
template <int T, bool DUP = false>
__device__ __forceinline__ void group_store_rows2(const float* smem, int LW, float* row0, float* row1, int c0, int nlive,
                                                  int lane, int nnew)
{
    constexpr int hs4 = hist_stride(T) / 4;
    vf4* h0 = (vf4*)(row0 + (size_t)c0 * (hs4 * 4));
    vf4* h1 = (vf4*)(row1 + (size_t)c0 * (hs4 * 4));
    for (int q = lane; q < nlive * hs4; q += FRONT_WAVE_L)
    {
        const float* sp = smem + (q / hs4) * LW + 2 * (nnew + 4 * (q % hs4));
        const vf4 p0 = *(const vf4*)sp, p1 = *(const vf4*)(sp + 4);
        h0[q] = vf4{ p0.x, p0.z, p1.x, p1.z };
        if (!DUP) h1[q] = vf4{ p0.y, p0.w, p1.y, p1.w };
    }
}

// scalar window (the audio decimator): history part, and the write-back
template <int T, int HQM>
__device__ __forceinline__ void group_fill_rows(float* smem, int LW, const float* row, int c0, int cpw, int nlive,
                                                int lane, const vf4 (&buf)[HQM])
{
    constexpr int hs4 = hist_stride(T) / 4, HQ = hist_q(T);
    const int nq = cpw * hs4;
#pragma unroll
    for (int i = 0; i < HQ; ++i)
    {
        const int q = lane + FRONT_WAVE_L * i;
        if (q < nq) *(vf4*)(smem + (q / hs4) * LW + 4 * (q % hs4)) = buf[i];
    }
    const vf4* h = (const vf4*)(row + (size_t)c0 * (hs4 * 4));
    const int qmax = nlive * hs4 - 1;
    for (int q = lane + FRONT_WAVE_L * HQ; q < nq; q += FRONT_WAVE_L)
        *(vf4*)(smem + (q / hs4) * LW + 4 * (q % hs4)) = h[q < qmax ? q : qmax];
}

template <int T>
__device__ __forceinline__ void group_store_rows(const float* smem, int LW, float* row, int c0, int nlive, int lane, int nnew)
{
    constexpr int hs4 = hist_stride(T) / 4;
    vf4* h = (vf4*)(row + (size_t)c0 * (hs4 * 4));
    for (int q = lane; q < nlive * hs4; q += FRONT_WAVE_L)
        h[q] = *(const vf4*)(smem + (q / hs4) * LW + nnew + 4 * (q % hs4));
}

// ---- pair history rows: a FIR pair's two T-1 sample histories stored interleaved {x0[n], x1[n]}
//      (hist_stride(T) pairs, 2 * hist_stride(T) floats per channel), the window's own layout, so a
//      float4 (two pairs) moves between HBM and LDS as is ----
__host__ __device__ constexpr int hist_p4(int T) { return hist_stride(T) / 2; }       // float4s per pair row
__host__ __device__ constexpr int hist_qp(int T) { return (hist_p4(T) + 7) / 8; }      // prefetched per lane

template <int T, int HQM>
__device__ __forceinline__ void group_load_prow(const float* row, int c0, int nlive, int lane, vf4 (&buf)[HQM])
{
    constexpr int hp4 = hist_p4(T), HQ = hist_qp(T);
    const vf4* h = (const vf4*)(row + (size_t)c0 * (hp4 * 4));
    const int qmax = nlive * hp4 - 1;                    // loads clamped to the live channels' rows
#pragma unroll
    for (int i = 0; i < HQ; ++i)
    {
        const int q = lane + FRONT_WAVE_L * i;
        buf[i] = h[q < qmax ? q : qmax];
    }
}

// float4 q of the group's rows is channel q / hp4, pairs 2 (q % hp4) .. + 1 of its window
// PB: padded window (pwin_off)
template <int T, int PB = 0, int HQM>
__device__ __forceinline__ void group_fill_prow(float* smem, int LW, const float* row, int c0, int cpw, int nlive,
                                                int lane, const vf4 (&buf)[HQM])
{
    constexpr int hp4 = hist_p4(T), HQ = hist_qp(T);
    const int nq = cpw * hp4;
#pragma unroll
    for (int i = 0; i < HQ; ++i)
    {
        const int q = lane + FRONT_WAVE_L * i;
        if (q < nq) *(vf4*)(smem + (q / hp4) * LW + pwin_off<PB>(2 * (q % hp4))) = buf[i];
    }
    const vf4* h = (const vf4*)(row + (size_t)c0 * (hp4 * 4));
    const int qmax = nlive * hp4 - 1;
    for (int q = lane + FRONT_WAVE_L * HQ; q < nq; q += FRONT_WAVE_L)
        *(vf4*)(smem + (q / hp4) * LW + pwin_off<PB>(2 * (q % hp4))) = h[q < qmax ? q : qmax];
}

// the next call's pair rows: window pairs nnew .. nnew + hist_stride(T) - 1 of each channel
template <int T, int PB = 0>
__device__ __forceinline__ void group_store_prow(const float* smem, int LW, float* row, int c0, int nlive, int lane, int nnew)
{
    constexpr int hp4 = hist_p4(T);
    vf4* h = (vf4*)(row + (size_t)c0 * (hp4 * 4));
    for (int q = lane; q < nlive * hp4; q += FRONT_WAVE_L)
        h[q] = *(const vf4*)(smem + (q / hp4) * LW + pwin_off<PB>(nnew + 2 * (q % hp4)));
}

// new samples of one channel's window (the lane's own NV values).  No zero tail: the windows of
// a wave sit lw floats apart and the register-window FIRs' over-read (at most FRONT_TAIL samples
// past the data, never used in a product) lands in the next channel's window, or, for the last
// one, in the slack the LDS allocation adds after the windows.
// PB: padded window (pwin_off); two pairs at an even index never straddle a pad
template <int PB = 0>
__device__ __forceinline__ void window_new2(float* W, int T, bool act, int b, const v2f* vals, int NV)
{
    if (act)
    {
        const int i0 = T - 1 + b * NV;
        if (((T - 1) & 1) == 0)                           // 16-byte aligned: two pairs per store
            for (int j = 0; j < NV; j += 2)
                *(vf4*)(W + pwin_off<PB>(i0 + j)) = vf4{ vals[j].x, vals[j].y, vals[j + 1].x, vals[j + 1].y };
        else
            for (int j = 0; j < NV; ++j) *(v2f*)(W + pwin_off<PB>(i0 + j)) = vals[j];
    }
}

__device__ __forceinline__ void window_new(float* W, int T, bool act, int b, const float* vals, int NV)
{
    if (act)
    {
        float* d = W + T - 1 + b * NV;
        if (((T - 1 + b * NV) & 3) == 0 && (NV & 3) == 0)
            for (int j = 0; j < NV; j += 4) *(vf4*)(d + j) = vf4{ vals[j], vals[j + 1], vals[j + 2], vals[j + 3] };
        else if (((T - 1 + b * NV) & 1) == 0 && (NV & 1) == 0)
            for (int j = 0; j < NV; j += 2) *(v2f*)(d + j) = v2f{ vals[j], vals[j + 1] };
        else
            for (int j = 0; j < NV; ++j) d[j] = vals[j];
    }
}

// Lane -> (channel g, block b) of a front wave.  Window reads are ds_read_b128 at g*lw + b*S
// (S = R floats), serviced in four 16-lane groups (MI355X_MICROARCH.md §LDS).  A run of
// K = 64/S consecutive blocks of one channel covers one bank in four of every S; S/4
// consecutive channels with lw = 4 (mod S) interleave into all 64 banks.  So each 16-lane group
// gets S/4 (channel, run) pairs of consecutive channels: conflict-free.  Batches whose shape
// does not allow that (nb not a power of two, too few channels or blocks) use g = l / nb.
__host__ __device__ inline void front_lane(int l, int nb, int S, int& g, int& b)
{
    const int cpw = 64 / nb, K = 64 / S, cpg = S / 4;
    if ((nb & (nb - 1)) || nb < K || cpw < cpg)
    {
        g = l / nb;
        b = l % nb;
        return;
    }
    // b128 groups: {0-3,12-15,20-27}, {4-11,16-19,28-31}, then the same + 32
    const int h = l & 31;
    int k, j;
    if (h < 4) { k = 0; j = h; }
    else if (h < 12) { k = 1; j = h - 4; }
    else if (h < 16) { k = 0; j = h - 8; }
    else if (h < 20) { k = 1; j = h - 8; }
    else if (h < 28) { k = 0; j = h - 12; }
    else { k = 1; j = h - 16; }
    k += (l >> 5) * 2;
    const int pr = k * cpg + j / K;          // (channel, run) pair
    g = pr % cpw;
    b = (pr / cpw) * K + j % K;
}

// arm_iir_lattice_f32 (CMSIS .../arm_iir_lattice_f32.c:348-447), one sample, S stages:
// stage i of the next sample reads the g stage i+1 produced; the last reads the final f.
template <int S>
__device__ __forceinline__ float lattice_step(float x, float (&g)[S > 0 ? S : 1], const float* k, const float* v)
{
    float fcurr = x, fnext = 0.0f, acc = 0.0f;
    float gn[S > 0 ? S : 1];
#pragma unroll
    for (int i = 0; i < S; ++i)
    {
        const float gcurr = g[i];
        fnext = fcurr - (k[i] * gcurr);
        const float gnext = (fnext * k[i]) + gcurr;
        acc += (gnext * v[i]);
        gn[i] = gnext;
        fcurr = fnext;
    }
    acc += (fnext * v[S]);
#pragma unroll
    for (int i = 0; i + 1 < S; ++i) g[i] = gn[i + 1];
    if (S > 0) g[S - 1] = fnext;
    return acc;
}

// The same sample on packed f32 (v_pk_mul_f32 / v_pk_add_f32): every product and sum is the
// reference's binary32 operation on the same operands, two independent ones per instruction.
// Stages are taken in pairs (i, i+1): both k*g products of a pair up front (old states), the
// f chain as scalar subtracts, then {f_i k_i, f_i+1 k_i+1} + {g_i, g_i+1} -> {gn_i, gn_i+1} and
// {gn_i v_i, gn_i+1 v_i+1} for the output sum, which is added in the reference's order.  The state
// shifts by one stage per sample (g_i <- gn_i+1), so the pairing alternates with the sample's
// parity PAR: pairs (0,1),(2,3)... on even samples, stage 0 alone then (1,2),(3,4)... on odd
// ones -- each sample's pairs are then exactly the register pairs the previous sample produced,
// and no moves are needed to form them.  Results are bit-identical for either parity.
template <int S, int PAR>
__device__ __forceinline__ float lattice_step_pk(float x, float (&g)[S > 0 ? S : 1], const float* k, const float* v)
{
    if constexpr (S < 3) return lattice_step<S>(x, g, k, v);
    else
    {
        float gn[S], q[S];
        float f = x;
        int i = 0;
        if (PAR)
        {
            f = f - (k[0] * g[0]);
            gn[0] = (f * k[0]) + g[0];
            q[0] = gn[0] * v[0];
            i = 1;
        }
#pragma unroll
        for (; i + 1 < S; i += 2)
        {
            const v2f gp = v2f{ g[i], g[i + 1] }, kp = v2f{ k[i], k[i + 1] };
            const v2f kg = kp * gp;
            const float f0 = f - kg.x;
            const float f1 = f0 - kg.y;
            const v2f gnp = (v2f{ f0, f1 } * kp) + gp;
            const v2f qp = gnp * v2f{ v[i], v[i + 1] };
            gn[i] = gnp.x; gn[i + 1] = gnp.y;
            q[i] = qp.x; q[i + 1] = qp.y;
            f = f1;
        }
        if (i < S)
        {
            f = f - (k[i] * g[i]);
            gn[i] = (f * k[i]) + g[i];
            q[i] = gn[i] * v[i];
        }
        float acc = 0.0f;
#pragma unroll
        for (int j = 0; j < S; ++j) acc += q[j];
        acc += (f * v[S]);
#pragma unroll
        for (int j = 0; j + 1 < S; ++j) g[j] = gn[j + 1];
        g[S - 1] = f;
        return acc;
    }
}

// Two consecutive samples x0 (even position) and x1 of lattice_step_pk, with the output (ladder)
// sums of both on packed f32: each sample's recursion runs as in lattice_step_pk, its ladder
// products q_0 .. q_S = {gn_i v_i}, f v_S are kept, and acc = ((0 + q_0) + q_1) + ... runs for both
// samples at once (v_pk_add_f32), element-wise the reference's order.  The ladder does not feed
// the recursion, so pairing two samples' sums only removes S + 1 adds per pair from the issue of a
// latency-bound single wave (the anti-alias role of the C2 back end, round 6).
template <int S>
__device__ __forceinline__ void lattice_step2_pk(float x0, float x1, float (&g)[S > 0 ? S : 1], const float* k,
                                                 const float* v, float& y0, float& y1)
{
    static_assert(S >= 3, "packed form");
    float q[2][S + 1];
#pragma unroll
    for (int h = 0; h < 2; ++h)
    {
        float gn[S];
        float f = h ? x1 : x0;
        int i = 0;
        if (h)
        {
            f = f - (k[0] * g[0]);
            gn[0] = (f * k[0]) + g[0];
            q[h][0] = gn[0] * v[0];
            i = 1;
        }
#pragma unroll
        for (; i + 1 < S; i += 2)
        {
            const v2f gp = v2f{ g[i], g[i + 1] }, kp = v2f{ k[i], k[i + 1] };
            const v2f kg = kp * gp;
            const float f0 = f - kg.x;
            const float f1 = f0 - kg.y;
            const v2f gnp = (v2f{ f0, f1 } * kp) + gp;
            const v2f qp = gnp * v2f{ v[i], v[i + 1] };
            gn[i] = gnp.x; gn[i + 1] = gnp.y;
            q[h][i] = qp.x; q[h][i + 1] = qp.y;
            f = f1;
        }
        if (i < S)
        {
            f = f - (k[i] * g[i]);
            gn[i] = (f * k[i]) + g[i];
            q[h][i] = gn[i] * v[i];
        }
        q[h][S] = f * v[S];
#pragma unroll
        for (int j = 0; j + 1 < S; ++j) g[j] = gn[j + 1];
        g[S - 1] = f;
    }
    v2f acc = v2f{ 0.0f, 0.0f };
#pragma unroll
    for (int j = 0; j <= S; ++j) acc = acc + v2f{ q[0][j], q[1][j] };
    y0 = acc.x;
    y1 = acc.y;
}

// arm_biquad_cascade_df1_f32 (.../arm_biquad_cascade_df1_f32.c:349-418), one stage
__device__ __forceinline__ float biquad_step(float x, float& x1, float& x2, float& y1, float& y2, const float* c)
{
    const float acc = (c[0] * x) + (c[1] * x1) + (c[2] * x2) + (c[3] * y1) + (c[4] * y2);
    x2 = x1; x1 = x; y2 = y1; y1 = acc;
    return acc;
}

// ---- host: LDS bank-conflict model of the front's window accesses (MI355X_MICROARCH.md §LDS) ----
// ds_read_b128: four 16-lane groups, bank (a/4) mod 64; ds_write_b128: eight groups of 8
// contiguous lanes, bank (a/4) mod 32; ds_write_b64: four groups of 16; ds_read/write_b32: two
// groups of 32, bank (a/4) mod 32.  One LDS cycle per group, plus one per extra distinct dword
// on a busy bank (identical addresses broadcast).
enum LdsOp { LDS_R128, LDS_W128, LDS_W64, LDS_W32 };
static const int kB128Groups[4][16] = {
    { 0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27 },
    { 4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31 },
    { 32, 33, 34, 35, 44, 45, 46, 47, 52, 53, 54, 55, 56, 57, 58, 59 },
    { 36, 37, 38, 39, 40, 41, 42, 43, 48, 49, 50, 51, 60, 61, 62, 63 } };

// LDS-array cycles of one wave instruction; addr[l] < 0: lane l inactive
static inline int lds_op_cycles(LdsOp op, const int (&addr)[64])
{
    const int ngroups = op == LDS_R128 ? 4 : op == LDS_W128 ? 8 : op == LDS_W64 ? 4 : 2;
    const int glen = 64 / ngroups, banks = op == LDS_R128 ? 64 : 32;
    const int nd = op == LDS_W64 ? 2 : op == LDS_W32 ? 1 : 4;
    int cycles = 0;
    for (int gi = 0; gi < ngroups; ++gi)
    {
        int load[64] = { 0 }, seen[64], nseen = 0;
        for (int k = 0; k < glen; ++k)
        {
            const int l = op == LDS_R128 ? kB128Groups[gi][k] : gi * glen + k;
            if (addr[l] < 0) continue;
            for (int d = 0; d < nd; ++d)
            {
                const int ad = addr[l] + d;
                bool dup = false;
                for (int i = 0; i < nseen; ++i) dup = dup || seen[i] == ad;
                if (dup) continue;
                if (nseen < 64) seen[nseen++] = ad;
                load[ad & (banks - 1)] += 1;
            }
        }
        int mx = 0;
        for (int k = 0; k < 64; ++k) mx = load[k] > mx ? load[k] : mx;
        cycles += mx;
    }
    return cycles;
}

// lane -> (channel g, block b) maps of a front wave, packed g << 8 | b
// (a) front_lane (below): runs of consecutive blocks per channel, laid out for the b128 read groups
// (b) interleaved: lane l -> channel l % 4 + 4 * (l / (4 nb)), block (l % (4 nb)) / 4 -- each group
//     of 8 contiguous lanes (a ds_write_b128 group) holds 4 channels x 2 consecutive blocks and
//     each b128 read group 4 channels x 4 blocks of distinct b mod 4 (nb <= 16, >= 4 channels)
__host__ __device__ inline void front_lane(int l, int nb, int S, int& g, int& b);
static inline bool front_lane_interleaved(int l, int nb, int& g, int& b)
{
    if (nb > 16 || (nb & (nb - 1)) || 64 % (4 * nb)) return false;
    g = l % 4 + 4 * (l / (4 * nb));
    b = (l % (4 * nb)) / 4;
    return true;
}

// modeled LDS-array cycles of one front wave's window traffic at pitch lw.  Pass 1: a FIR pair
// over {x0, x1} (T1 taps, R outputs per lane, new pairs at 2 (T1-1)), lane map lm.
static inline int front_lds_pass1(int lw, const uint16_t* lm, int cpw, int T1, int R, int pb = 0)
{
    auto off = [&](int i) { return 2 * i + pb * (i >> 3); };     // pwin_off
    int addr[64], cycles = 0;
    // new samples (R pairs per lane: ds_write_b128 two pairs at a time when aligned)
    for (int l = 0; l < 64; ++l)
    {
        const int g = lm[l] >> 8, b = lm[l] & 0xff;
        addr[l] = g < cpw ? g * lw + off(T1 - 1 + b * R) : -1;
    }
    cycles += lds_op_cycles(((T1 - 1) & 1) ? LDS_W64 : LDS_W128, addr) * (((T1 - 1) & 1) ? R : R / 2);
    // reads (ds_read_b128, every one at the same bank phase): the register window's first WA
    // pairs, then 8 pairs per 8-tap chunk
    const int WA = (R - 1 + 8 + 7) & ~7;
    for (int l = 0; l < 64; ++l)
    {
        const int g = lm[l] >> 8, b = lm[l] & 0xff;
        addr[l] = g < cpw ? g * lw + off(b * R) : -1;
    }
    return cycles + lds_op_cycles(LDS_R128, addr) * (WA / 2 + (T1 / 8) * 4);
}

// Pass 2: its new samples (NV per pass-1 lane; pairs when pair2) are written by the lanes of the
// pass-1 map lm1, its FIR (RD outputs per lane, decimation M2: a pair over a window of stride
// 2 NV, or the mono decimator, stride NV) reads by the lanes of map lm2.
static inline int front_lds_pass2(int lw, const uint16_t* lm1, const uint16_t* lm2, int cpw, int T2, bool pair2, int NV,
                                  int RD, int M2)
{
    int addr[64], cycles = 0;
    const int off = pair2 ? 2 * (T2 - 1) : T2 - 1, per = pair2 ? 2 * NV : NV;
    for (int l = 0; l < 64; ++l)
    {
        const int g = lm1[l] >> 8, b = lm1[l] & 0xff;
        addr[l] = g < cpw ? g * lw + off + b * per : -1;
    }
    LdsOp wop = LDS_W32;
    int nw = per;
    if ((off & 3) == 0 && (per & 3) == 0) { wop = LDS_W128; nw = per / 4; }
    else if ((off & 1) == 0 && (per & 1) == 0) { wop = LDS_W64; nw = per / 2; }
    cycles += lds_op_cycles(wop, addr) * nw;
    const int WA = (M2 * (RD - 1) + 8 + 7) & ~7;
    const int nread = pair2 ? WA / 2 + (T2 / 8) * 4 : WA / 4 + (T2 / 8) * 2;
    for (int l = 0; l < 64; ++l)
    {
        const int g = lm2[l] >> 8, b = lm2[l] & 0xff;
        addr[l] = g < cpw ? g * lw + b * per : -1;
    }
    return cycles + lds_op_cycles(LDS_R128, addr) * nread;
}

// the history rows' LDS traffic of one pass (group_fill_prow / _rows, group_store_prow / _rows):
// float4 q of the group's rows (hq float4s per channel) lands at (q / hq) lw + 4 (q % hq) + base
// (the store reads the window at base = the new samples' offset); lane l moves float4s l, l + 64, ...
static inline int front_lds_hist(int lw, int cpw, int hq, int nnew_floats)
{
    int addr[64], cycles = 0;
    const int nq = cpw * hq;
    for (int i = 0; i * 64 < nq; ++i)
        for (int pass = 0; pass < 2; ++pass)
        {
            for (int l = 0; l < 64; ++l)
            {
                const int q = l + 64 * i;
                addr[l] = q < nq ? (q / hq) * lw + 4 * (q % hq) + (pass ? nnew_floats : 0) : -1;
            }
            cycles += lds_op_cycles(pass ? LDS_R128 : LDS_W128, addr);
        }
    return cycles;
}

// extra LDS cycles of one FIR window read (ds_read_b128) for lane bases g*lw + b*stride (floats)
// under lane map lm (TX pitch choice)
static inline int window_conflicts(int lw, const uint16_t* lm, int cpw, int stride)
{
    int addr[64];
    for (int l = 0; l < 64; ++l)
    {
        const int g = lm[l] >> 8, b = lm[l] & 0xff;
        addr[l] = g < cpw ? g * lw + b * stride : -1;
    }
    return lds_op_cycles(LDS_R128, addr) - 4;
}

#endif /* UHSDR_DSP_H */
