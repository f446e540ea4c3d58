// MI355X (gfx950) RX chain of the UHSDR firmware, batched over channels.
//
// One uhsdr_rx_process() call == N/32 consecutive AudioDriver_RxProcessor invocations
// (drivers/audio/audio_driver.c:2603-2942) on each of C independent channels.  Two kernels:
//
//  rx_front  (time-parallel, all lanes busy whatever C is)
//      int32 I/Q -> f32, x 2^-16          audio_driver.c:2660-2685
//      I/Q correction (manual / auto)     audio_driver.c:2254-2316
//      FreqShift (Fs/4 or oscillator)     freq_shift.c:219-334
//      Hilbert FIR pair + I +- Q + decimator, or decimator pair + Hilbert pair + I +- Q
//                                         audio_driver.c:2718-2810, CMSIS arm_fir_f32 /
//                                         arm_fir_decimate_f32
//    -> decimated audio adec[C][N/M] (12 or 24 ksps), FIR delay lines updated.
//    Workgroup = G channels; their windows (history + block) sit in LDS; each lane computes
//    R consecutive FIR outputs from a register-resident sliding window.
//
//  rx_back   (sequential per channel: one lane == one channel, 64 channels per wave)
//      IIR lattice pre-filter -> WDSP AGC -> scale -> biquad_1 -> polyphase interpolator
//      -> anti-alias lattice -> biquad_2 -> line-out scale -> f32 + int32 codec frames
//                                         audio_driver.c:2436-2592, 2832-2923
//    All recursions run per sample in the reference order; state lives in registers for the
//    whole launch; the AGC look-ahead ring lives in LDS.
//
// Arithmetic: exactly the reference's binary32 operation sequence (this file is compiled
// with -ffp-contract=off), so the device output is bit-identical to the firmware built for
// x86 (tests/test_gpu_parity.py).

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
#include <math.h>
#include "uhsdr_internal.h"

#define BLK UHSDR_IQ_BLOCK_SIZE
#define IQ_BIT_SCALE_DOWN 0.0000152587890625f

// ------------------------------------------------------------------------------------
// LDS window addressing: one pad word every 8 so that lanes reading windows 8 or 16
// samples apart hit different banks.
__device__ __forceinline__ int sk(int p) { return p + (p >> 3); }
__host__ __device__ constexpr int sk_len(int n) { return n + (n >> 3) + 1; }

// y[j] = sum_{k<Tpad} c[k] * win[j*M + k] for j = j0 .. j0+R-1 (coefficients zero padded
// to a multiple of 8: a +-0 product never changes a finite accumulator that started at +0).
template <int R, int M>
__device__ __forceinline__ void fir_run(const float* win, const float* __restrict__ c, int Tpad, int j0,
                                        float (&acc)[R])
{
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = 0.0f;
    constexpr int W = 8 + M * (R - 1);
    const int base = j0 * M;
    for (int k0 = 0; k0 < Tpad; k0 += 8)
    {
        float w[W];
#pragma unroll
        for (int q = 0; q < W; ++q) w[q] = win[sk(base + k0 + q)];
#pragma unroll
        for (int kk = 0; kk < 8; ++kk)
        {
            const float cc = c[k0 + kk];
#pragma unroll
            for (int r = 0; r < R; ++r) acc[r] += w[r * M + kk] * cc;
        }
    }
}

struct FrontArgs
{
    const uhsdr_rx_plan* plan;
    const int2* iq;          // [C][N] IqSample_t
    float* hist1_i;          // [C][T1-1]: stage-1 FIR history (Hilbert, or I decimator)
    float* hist1_q;          // [C][T1-1]
    float* hist2_i;          // [C][T2-1]: stage-2 FIR history (audio decimator, or Hilbert I)
    float* hist2_q;          // [C][T2-1]  (decimated-IQ paths only)
    float* teta;             // [3][C] auto I/Q correction low-pass state
    float* osc;              // [2][C] oscillator {I, Q}
    float* adec;             // [C][Nd] output
    int C, N, G;
    int T1, T1pad, T2, T2pad;
};

// Stage-1 window: x[g][0 .. T1-2] history, x[g][T1-1 .. T1-1+N-1] new samples.
template <int R1, int M2>
__global__ void __launch_bounds__(256) rx_front(FrontArgs a)
{
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const uhsdr_rx_plan* __restrict__ P = a.plan;
    const int N = a.N, G = a.G, C = a.C;
    const int T1 = a.T1, T2 = a.T2;
    const int M = P->decimation_rate;
    const bool decim_iq = P->use_decimated_iq;
    const int N2 = decim_iq ? N / M : N;                // stage-2 input length
    const int L1 = sk_len(T1 - 1 + N + 8);             // + 8 zero words read by the padded taps
    const int L2 = sk_len(T2 - 1 + N2 + 8);
    float* xi = smem;                                   // [G][L1]
    float* xq = xi + G * L1;                            // [G][L1]
    float* yi = xq + G * L1;                            // [G][L2]  stage-2 window(s)
    float* yq = yi + G * L2;                            // [G][L2]  (decim_iq only)
    float* mc = yq + (decim_iq ? G * L2 : 0);           // [G][2][N/32] auto-IQ factors
    const int c0 = blockIdx.x * G;
    const int tid = threadIdx.x;
    const int nblk32 = N / BLK;

    // ---- zero the window tails, load stage-1 history + convert new I/Q ----
    for (int e = tid; e < G * 8; e += blockDim.x)
    {
        const int g = e / 8, k = e % 8;
        xi[g * L1 + sk(T1 - 1 + N + k)] = 0.0f;
        xq[g * L1 + sk(T1 - 1 + N + k)] = 0.0f;
    }
    for (int e = tid; e < G * (T1 - 1); e += blockDim.x)
    {
        const int g = e / (T1 - 1), k = e % (T1 - 1);
        const int c = c0 + g;
        if (c < C)
        {
            xi[g * L1 + sk(k)] = a.hist1_i[(size_t)c * (T1 - 1) + k];
            xq[g * L1 + sk(k)] = a.hist1_q[(size_t)c * (T1 - 1) + k];
        }
    }
    const float gi = P->iq_gain_i, gq = P->iq_gain_q, ph = P->iq_phase_balance;
    const bool iq_auto = P->iq_auto_correction;
    for (int e = tid; e < G * N; e += blockDim.x)
    {
        const int g = e / N, n = e % N;
        const int c = c0 + g;
        if (c >= C) continue;
        const int2 v = a.iq[(size_t)c * N + n];
        float I = (float)v.x, Q = (float)v.y;
        I = I * IQ_BIT_SCALE_DOWN;
        Q = Q * IQ_BIT_SCALE_DOWN;
        if (!iq_auto)
        {
            I = I * gi;
            Q = Q * gq;
            if (ph < 0) { const float e3 = I * ph; Q = Q + e3; }
            else if (ph > 0) { const float e3 = Q * ph; I = I + e3; }
        }
        xi[g * L1 + sk(T1 - 1 + n)] = I;
        xq[g * L1 + sk(T1 - 1 + n)] = Q;
    }
    __syncthreads();

    // ---- automatic I/Q correction: per-32-frame statistics, sequential low-pass ----
    if (iq_auto)
    {
        float* m1 = mc;                 // [G][nblk32]
        float* m2 = mc + G * nblk32;    // [G][nblk32]
        // statistics need the whole block: one lane per (channel, block), sequential sum
        // (audio_driver.c:2280-2285), then one lane per channel runs the low-pass.
        float* t1s = yi;                // reuse stage-2 window as scratch (3 x G x nblk32)
        for (int e = tid; e < G * nblk32; e += blockDim.x)
        {
            const int g = e / nblk32, b = e % nblk32;
            float t1 = 0.0f, t2 = 0.0f, t3 = 0.0f;
            for (int i = 0; i < BLK; ++i)
            {
                const float I = xi[g * L1 + sk(T1 - 1 + b * BLK + i)];
                const float Q = xq[g * L1 + sk(T1 - 1 + b * BLK + i)];
                const float sI = (I < 0) ? -1.0f : ((I > 0) ? 1.0f : 0.0f);
                const float sQ = (Q < 0) ? -1.0f : ((Q > 0) ? 1.0f : 0.0f);
                t1 += sI * Q;
                t2 += sI * I;
                t3 += sQ * Q;
            }
            t1s[(0 * G + g) * nblk32 + b] = t1;
            t1s[(1 * G + g) * nblk32 + b] = t2;
            t1s[(2 * G + g) * nblk32 + b] = t3;
        }
        __syncthreads();
        for (int g = tid; g < G; g += blockDim.x)
        {
            const int c = c0 + g;
            if (c >= C) continue;
            float o1 = a.teta[c], o2 = a.teta[C + c], o3 = a.teta[2 * C + c];
            for (int b = 0; b < nblk32; ++b)
            {
                float t1 = t1s[(0 * G + g) * nblk32 + b];
                float t2 = t1s[(1 * G + g) * nblk32 + b];
                float t3 = t1s[(2 * G + g) * nblk32 + b];
                t1 = (float)(-0.003 * (double)(t1 / (float)BLK) + 0.997 * (double)o1);
                t2 = (float)(0.003 * (double)(t2 / (float)BLK) + 0.997 * (double)o2);
                t3 = (float)(0.003 * (double)(t3 / (float)BLK) + 0.997 * (double)o3);
                const float M_c1 = (t2 != 0.0f) ? t1 / t2 : 0.0f;
                float help = (t2 * t2);
                if (help > 0.0f) help = (t3 * t3 - t1 * t1) / help;
                const float M_c2 = (help > 0.0f) ? sqrtf(help) : 1.0f;
                m1[g * nblk32 + b] = M_c1;
                m2[g * nblk32 + b] = M_c2;
                o1 = t1; o2 = t2; o3 = t3;
            }
            a.teta[c] = o1; a.teta[C + c] = o2; a.teta[2 * C + c] = o3;
        }
        __syncthreads();
        for (int e = tid; e < G * N; e += blockDim.x)
        {
            const int g = e / N, n = e % N;
            const int b = n / BLK;
            const int p = g * L1 + sk(T1 - 1 + n);
            const float I = xi[p];
            const float Q = xq[p] + m1[g * nblk32 + b] * I;
            xq[p] = Q;
            xi[p] = I * m2[g * nblk32 + b];
        }
        __syncthreads();
    }

    // ---- frequency translation ----
    if (P->freq_shift_hz != 0)
    {
        float* ib = P->shift_up ? xi : xq;
        float* qb = P->shift_up ? xq : xi;
        if (P->shift_kind == 1)
        {
            for (int e = tid; e < G * N; e += blockDim.x)
            {
                const int g = e / N, n = e % N;
                const int p = g * L1 + sk(T1 - 1 + n);
                const float iv = ib[p], qv = qb[p];
                switch (n & 3)
                {
                case 0: break;
                case 1: ib[p] = qv; qb[p] = -iv; break;
                case 2: ib[p] = -iv; qb[p] = -qv; break;
                case 3: ib[p] = -qv; qb[p] = iv; break;
                }
            }
        }
        else
        {
            // recursive quadrature oscillator: sequential in time, one lane per channel
            const float oc = P->osc_cos, os = P->osc_sin;
            for (int g = tid; g < G; g += blockDim.x)
            {
                const int c = c0 + g;
                if (c >= C) continue;
                float vi = a.osc[c], vq = a.osc[C + c];
                for (int n = 0; n < N; ++n)
                {
                    const int p = g * L1 + sk(T1 - 1 + n);
                    const float oq = (vq * oc) - (vi * os);
                    const float oi = (vi * oc) + (vq * os);
                    const float qt = qb[p], it = ib[p];
                    qb[p] = (qt * oq) - (it * oi);
                    ib[p] = (it * oq) + (qt * oi);
                    vq = oq; vi = oi;
                    if ((n & (BLK - 1)) == BLK - 1)
                    {
                        const float gn = (3 - ((vq * vq) + (vi * vi))) / 2;
                        vq = gn * vq; vi = gn * vi;
                    }
                }
                a.osc[c] = vi; a.osc[C + c] = vq;
            }
        }
        __syncthreads();
    }

    // ---- save stage-1 history, load stage-2 history ----
    for (int e = tid; e < G * (T1 - 1); e += blockDim.x)
    {
        const int g = e / (T1 - 1), k = e % (T1 - 1);
        const int c = c0 + g;
        if (c >= C) continue;
        a.hist1_i[(size_t)c * (T1 - 1) + k] = xi[g * L1 + sk(N + k)];
        a.hist1_q[(size_t)c * (T1 - 1) + k] = xq[g * L1 + sk(N + k)];
    }
    for (int e = tid; e < G * 8; e += blockDim.x)
    {
        const int g = e / 8, k = e % 8;
        yi[g * L2 + sk(T2 - 1 + N2 + k)] = 0.0f;
        if (decim_iq) yq[g * L2 + sk(T2 - 1 + N2 + k)] = 0.0f;
    }
    for (int e = tid; e < G * (T2 - 1); e += blockDim.x)
    {
        const int g = e / (T2 - 1), k = e % (T2 - 1);
        const int c = c0 + g;
        if (c >= C) continue;
        yi[g * L2 + sk(k)] = a.hist2_i[(size_t)c * (T2 - 1) + k];
        if (decim_iq) yq[g * L2 + sk(k)] = a.hist2_q[(size_t)c * (T2 - 1) + k];
    }
    __syncthreads();

    const bool lsb = P->lsb;
    if (!decim_iq)
    {
        // stage 1: Hilbert pair at 48 ksps, a = I +- Q into the decimator window
        const int nb = N / R1;
        for (int e = tid; e < G * nb; e += blockDim.x)
        {
            const int g = e / nb, b = e % nb;
            float hi[R1], hq[R1];
            fir_run<R1, 1>(xi + g * L1, P->hilbert_i, a.T1pad, b * R1, hi);
            fir_run<R1, 1>(xq + g * L1, P->hilbert_q, a.T1pad, b * R1, hq);
#pragma unroll
            for (int r = 0; r < R1; ++r)
                yi[g * L2 + sk(T2 - 1 + b * R1 + r)] = lsb ? (hi[r] - hq[r]) : (hi[r] + hq[r]);
        }
        __syncthreads();
        // stage 2: decimator -> adec
        const int Nd = N / M;
        constexpr int R2 = 4;
        const int nb2 = Nd / R2;
        for (int e = tid; e < G * nb2; e += blockDim.x)
        {
            const int g = e / nb2, b = e % nb2;
            const int c = c0 + g;
            float d[R2];
            fir_run<R2, M2>(yi + g * L2, P->dec, a.T2pad, b * R2, d);
            if (c < C)
            {
#pragma unroll
                for (int r = 0; r < R2; ++r) a.adec[(size_t)c * Nd + b * R2 + r] = d[r];
            }
        }
    }
    else
    {
        // stage 1: decimator pair at 48 ksps into the Hilbert windows
        const int Nd = N / M;
        constexpr int R2 = 4;
        const int nb = Nd / R2;
        for (int e = tid; e < G * nb; e += blockDim.x)
        {
            const int g = e / nb, b = e % nb;
            float di[R2], dq[R2];
            fir_run<R2, M2>(xi + g * L1, P->dec, a.T1pad, b * R2, di);
            fir_run<R2, M2>(xq + g * L1, P->dec, a.T1pad, b * R2, dq);
#pragma unroll
            for (int r = 0; r < R2; ++r)
            {
                yi[g * L2 + sk(T2 - 1 + b * R2 + r)] = di[r];
                yq[g * L2 + sk(T2 - 1 + b * R2 + r)] = dq[r];
            }
        }
        __syncthreads();
        // stage 2: Hilbert pair at the decimated rate, a = I +- Q -> adec
        const int nb2 = Nd / R2;
        for (int e = tid; e < G * nb2; e += blockDim.x)
        {
            const int g = e / nb2, b = e % nb2;
            const int c = c0 + g;
            float hi[R2], hq[R2];
            fir_run<R2, 1>(yi + g * L2, P->hilbert_i, a.T2pad, b * R2, hi);
            fir_run<R2, 1>(yq + g * L2, P->hilbert_q, a.T2pad, b * R2, hq);
            if (c < C)
            {
#pragma unroll
                for (int r = 0; r < R2; ++r)
                    a.adec[(size_t)c * Nd + b * R2 + r] = lsb ? (hi[r] - hq[r]) : (hi[r] + hq[r]);
            }
        }
    }
    __syncthreads();
    // ---- save stage-2 history ----
    for (int e = tid; e < G * (T2 - 1); e += blockDim.x)
    {
        const int g = e / (T2 - 1), k = e % (T2 - 1);
        const int c = c0 + g;
        if (c >= C) continue;
        a.hist2_i[(size_t)c * (T2 - 1) + k] = yi[g * L2 + sk(N2 + k)];
        if (decim_iq) a.hist2_q[(size_t)c * (T2 - 1) + k] = yq[g * L2 + sk(N2 + k)];
    }
}

// ------------------------------------------------------------------------------------
// rx_back: per-channel recursions.  State arrays are [field][C] (lane-coalesced).

struct BackState
{
    float* pre;      // [10][C]
    float* aa;       // [10][C]
    float* bq1;      // [16][C]
    float* bq2;      // [4][C]
    float* interp;   // [15][C]
    float* ring;     // [W][C]   AGC look-ahead ring, slot = sample index mod W
    float* agc;      // [6][C]   ring_max volts save_volts fast_bavg hang_bavg wold
    int* agci;       // [3][C]   hang_counter decay_type state
};

struct BackArgs
{
    const uhsdr_rx_plan* plan;
    const float* adec;   // [C][Nd]
    float* audio;        // [C][N]  or null
    int2* dst;           // [C][N]  or null
    BackState s;
    int C, N, Nd;
    int ring_phase;      // (decimated samples processed so far) mod W
};

// arm_iir_lattice_f32 (generic order), one sample
template <int SMAX>
__device__ __forceinline__ float lattice_step(float x, float (&g)[SMAX], const float* __restrict__ k,
                                              const float* __restrict__ v, int S)
{
    float fcurr = x, fnext = 0.0f, acc = 0.0f;
    float gn[SMAX];
#pragma unroll
    for (int i = 0; i < SMAX; ++i)
    {
        if (i < S)
        {
            const float gcurr = g[i];
            fnext = fcurr - (k[i] * gcurr);
            const float gnext = (fnext * k[i]) + gcurr;
            acc += (gnext * v[i]);
            gn[i] = gnext;
            fcurr = fnext;
        }
    }
    acc += (fnext * v[S]);
#pragma unroll
    for (int i = 0; i < SMAX - 1; ++i)
        if (i < S - 1) g[i] = gn[i + 1];
#pragma unroll
    for (int i = 0; i < SMAX; ++i)
        if (i == S - 1) g[i] = fnext;
    return acc;
}

__device__ __forceinline__ float biquad_step(float x, float& x1, float& x2, float& y1, float& y2,
                                             const float* __restrict__ c)
{
    const float acc = (c[0] * x) + (c[1] * x1) + (c[2] * x2) + (c[3] * y1) + (c[4] * y2);
    x2 = x1; x1 = x; y2 = y1; y1 = acc;
    return acc;
}

__device__ __forceinline__ float log10f_fast(float X)
{
    int E;
    const float F = frexpf(fabsf(X), &E);
    float Y = 1.23149591368684f;
    Y *= F;
    Y += -4.11852516267426f;
    Y *= F;
    Y += 6.02197014179219f;
    Y *= F;
    Y += -3.13396450166353f;
    Y += (float)E;
    return (Y * 0.3010299956639812f);
}

__device__ __forceinline__ int to_dma(float f)
{
    const int v = (f > -2147483904.0f && f < 2147483648.0f) ? (int)f : INT32_MIN;
    return (int)((unsigned)v << 16);
}

#define BACK_WAVE 64
#define GROUP 8

__global__ void __launch_bounds__(BACK_WAVE) rx_back(BackArgs a)
{
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const uhsdr_rx_plan* __restrict__ P = a.plan;
    const uhsdr_agc_plan* __restrict__ A = &P->agc;
    const int lane = threadIdx.x;
    const int cbase = blockIdx.x * BACK_WAVE;
    const int c = cbase + lane;
    const bool live = c < a.C;
    const int C = a.C;
    const int W = A->attack_buffsize;
    const int NG = (W + GROUP - 1) / GROUP;
    const int L = P->interp_L, PH = P->interp_phase;
    const int Nd = a.Nd;
    const int ndc = BLK / P->decimation_rate;     // decimated samples per 32-frame call

    float* ring = smem;                            // [W][64]
    float* gmax = ring + W * BACK_WAVE;            // [NG][64]
    float* ostage = gmax + NG * BACK_WAVE;         // [64][BLK+1]
    float* istage = ostage + BACK_WAVE * (BLK + 1);// [64][ndc+1]

    // ---- state in ----
    float pre[UHSDR_MAX_LATTICE], aa[UHSDR_MAX_LATTICE], bq1[16], bq2[4], ip[UHSDR_MAX_INTERP];
#pragma unroll
    for (int i = 0; i < UHSDR_MAX_LATTICE; ++i)
    {
        pre[i] = live ? a.s.pre[i * C + c] : 0.0f;
        aa[i] = live ? a.s.aa[i * C + c] : 0.0f;
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) bq1[i] = live ? a.s.bq1[i * C + c] : 0.0f;
#pragma unroll
    for (int i = 0; i < 4; ++i) bq2[i] = live ? a.s.bq2[i * C + c] : 0.0f;
#pragma unroll
    for (int i = 0; i < UHSDR_MAX_INTERP; ++i) ip[i] = (live && i < 15) ? a.s.interp[i * C + c] : 0.0f;
    for (int k = 0; k < W; ++k) ring[k * BACK_WAVE + lane] = live ? a.s.ring[(size_t)k * C + c] : 0.0f;
    for (int gq = 0; gq < NG; ++gq)
    {
        float m = 0.0f;
        for (int k = gq * GROUP; k < min(W, (gq + 1) * GROUP); ++k) m = fmaxf(m, fabsf(ring[k * BACK_WAVE + lane]));
        gmax[gq * BACK_WAVE + lane] = m;
    }
    float ring_max = live ? a.s.agc[0 * C + c] : 0.0f;
    float volts = live ? a.s.agc[1 * C + c] : 0.0f;
    float save_volts = live ? a.s.agc[2 * C + c] : 0.0f;
    float fast_bavg = live ? a.s.agc[3 * C + c] : 0.0f;
    float hang_bavg = live ? a.s.agc[4 * C + c] : 0.0f;
    float wold = live ? a.s.agc[5 * C + c] : 0.0f;
    int hang_counter = live ? a.s.agci[0 * C + c] : 0;
    int decay_type = live ? a.s.agci[1 * C + c] : 0;
    int state = live ? a.s.agci[2 * C + c] : 0;

    const int S_pre = P->pre_stages, S_aa = P->aa_stages;
    const float scale = P->post_agc_scale, lo = P->line_out_scale;
    int slot = a.ring_phase;

    for (int call = 0; call < a.N / BLK; ++call)
    {
        // stage this call's decimated input (coalesced rows of ndc floats)
        for (int e = lane; e < BACK_WAVE * ndc; e += BACK_WAVE)
        {
            const int row = e / ndc, col = e % ndc;
            const int cc = cbase + row;
            istage[row * (ndc + 1) + col] = (cc < C) ? a.adec[(size_t)cc * Nd + call * ndc + col] : 0.0f;
        }
        __syncthreads();
        int oidx = 0;
        for (int m = 0; m < ndc; ++m)
        {
            float x = istage[lane * (ndc + 1) + m];
            if (S_pre > 0) x = lattice_step<UHSDR_MAX_LATTICE>(x, pre, P->pre_k, P->pre_v, S_pre);

            // ---- AudioAgc_RunAgcWdsp, audio_agc.c:349-595 ----
            if (A->mode == 5)
            {
                x = x * A->fixed_gain;
            }
            else
            {
                const float out_sample = ring[slot * BACK_WAVE + lane];
                const float abs_out = fabsf(out_sample);
                ring[slot * BACK_WAVE + lane] = x;
                fast_bavg = A->fast_backmult * abs_out + A->onemfast_backmult * fast_bavg;
                hang_bavg = A->hang_backmult * abs_out + A->onemhang_backmult * hang_bavg;
                // ring_max == max |x| over the W newest samples (the reference's incremental
                // rescan maintains exactly this window maximum; max is order independent)
                const int gsel = slot / GROUP;
                float gm = 0.0f;
                for (int k = gsel * GROUP; k < min(W, (gsel + 1) * GROUP); ++k)
                    gm = fmaxf(gm, fabsf(ring[k * BACK_WAVE + lane]));
                gmax[gsel * BACK_WAVE + lane] = gm;
                float rm = 0.0f;
                for (int gq = 0; gq < NG; ++gq) rm = fmaxf(rm, gmax[gq * BACK_WAVE + lane]);
                ring_max = rm;
                if (++slot == W) slot = 0;

                if (hang_counter > 0) --hang_counter;
                const float rv = ring_max - volts;
                switch (state)
                {
                case 0:
                    if (ring_max >= volts) volts += rv * A->attack_mult;
                    else if (volts > A->pop_ratio * fast_bavg) { state = 1; volts += rv * A->fast_decay_mult; }
                    else if (A->hang_enable && (hang_bavg > A->hang_level))
                    { state = 2; hang_counter = A->hang_counter_init; decay_type = 1; }
                    else { state = 3; volts += rv * A->decay_mult; decay_type = 0; }
                    break;
                case 1:
                    if (ring_max >= volts) { state = 0; volts += rv * A->attack_mult; }
                    else if (volts > save_volts) volts += rv * A->fast_decay_mult;
                    else if (hang_counter > 0) state = 2;
                    else if (decay_type == 0) { state = 3; volts += rv * A->decay_mult; }
                    else { state = 4; volts += rv * A->hang_decay_mult; }
                    break;
                case 2:
                    if (ring_max >= volts) { state = 0; save_volts = volts; volts += rv * A->attack_mult; }
                    else if (hang_counter == 0) { state = 4; volts += rv * A->hang_decay_mult; }
                    break;
                case 3:
                    if (ring_max >= volts) { state = 0; save_volts = volts; volts += rv * A->attack_mult; }
                    else volts += rv * A->decay_mult;
                    break;
                default:
                    if (ring_max >= volts) { state = 0; save_volts = volts; volts += rv * A->attack_mult; }
                    else volts += rv * A->hang_decay_mult;
                    break;
                }
                if (volts < A->min_volts) volts = A->min_volts;
                float vo = log10f_fast(A->inv_max_input * volts);
                if (vo > 0.0f) vo = 0.0f;
                const float mult = (A->out_target - A->slope_constant * vo) / volts;
                x = out_sample * mult;
            }
            if (A->remove_dc)
            {
                const float w = (float)((double)x + (double)wold * 0.9999);
                x = w - wold;
                wold = w;
            }
            x = x * scale;
#pragma unroll
            for (int st = 0; st < 4; ++st)
                x = biquad_step(x, bq1[4 * st], bq1[4 * st + 1], bq1[4 * st + 2], bq1[4 * st + 3], P->biquad1 + 5 * st);

            // ---- polyphase interpolator (phase L-1-j for output j) ----
            float win[UHSDR_MAX_INTERP];
#pragma unroll
            for (int t = 0; t < UHSDR_MAX_INTERP; ++t) win[t] = (t < PH - 1) ? ip[t] : 0.0f;
#pragma unroll
            for (int t = 0; t < UHSDR_MAX_INTERP; ++t)
                if (t == PH - 1) win[t] = x;
            for (int i = L; i > 0; --i)
            {
                float sum = 0.0f;
#pragma unroll
                for (int t = 0; t < UHSDR_MAX_INTERP; ++t)
                    if (t < PH) sum += win[t] * P->interp[(i - 1) + t * L];
                float y = sum;
                if (S_aa > 0) y = lattice_step<UHSDR_MAX_LATTICE>(y, aa, P->aa_k, P->aa_v, S_aa);
                y = biquad_step(y, bq2[0], bq2[1], bq2[2], bq2[3], P->biquad2);
                y = y * lo;
                ostage[lane * (BLK + 1) + oidx++] = y;
            }
#pragma unroll
            for (int t = 0; t < UHSDR_MAX_INTERP - 1; ++t)
                if (t < PH - 1) ip[t] = win[t + 1];
        }
        __syncthreads();
        // coalesced store of this call's 32 frames per channel
        for (int e = lane; e < BACK_WAVE * BLK; e += BACK_WAVE)
        {
            const int row = e / BLK, col = e % BLK;
            const int cc = cbase + row;
            if (cc >= C) continue;
            const float y = ostage[row * (BLK + 1) + col];
            const size_t o = (size_t)cc * a.N + call * BLK + col;
            if (a.audio) a.audio[o] = y;
            if (a.dst) { const int d = to_dma(y); a.dst[o] = make_int2(d, d); }
        }
        __syncthreads();
    }

    // ---- state out ----
    if (!live) return;
#pragma unroll
    for (int i = 0; i < UHSDR_MAX_LATTICE; ++i) { a.s.pre[i * C + c] = pre[i]; a.s.aa[i * C + c] = aa[i]; }
#pragma unroll
    for (int i = 0; i < 16; ++i) a.s.bq1[i * C + c] = bq1[i];
#pragma unroll
    for (int i = 0; i < 4; ++i) a.s.bq2[i * C + c] = bq2[i];
#pragma unroll
    for (int i = 0; i < 15; ++i) a.s.interp[i * C + c] = ip[i];
    for (int k = 0; k < W; ++k) a.s.ring[(size_t)k * C + c] = ring[k * BACK_WAVE + lane];
    a.s.agc[0 * C + c] = ring_max;
    a.s.agc[1 * C + c] = volts;
    a.s.agc[2 * C + c] = save_volts;
    a.s.agc[3 * C + c] = fast_bavg;
    a.s.agc[4 * C + c] = hang_bavg;
    a.s.agc[5 * C + c] = wold;
    a.s.agci[0 * C + c] = hang_counter;
    a.s.agci[1 * C + c] = decay_type;
    a.s.agci[2 * C + c] = state;
}

// ------------------------------------------------------------------------------------
// host runtime

struct uhsdr_rx_s
{
    uhsdr_rx_plan plan;
    uhsdr_rx_plan* d_plan;
    int C, N, Nd, G;
    int T1, T1pad, T2, T2pad;
    hipStream_t stream;
    // front state
    float *hist1_i, *hist1_q, *hist2_i, *hist2_q, *teta, *osc, *adec;
    // back state
    BackState bs;
    void* arena;
    size_t arena_bytes;
    long long dec_samples;   // decimated samples processed (AGC ring phase)
    int kernels_last;
    // per-kernel timing (uhsdr_rx_enable_timing)
    int timing;
    int nev;                 // events used
    int nev_cap;
    hipEvent_t* ev;          // [cap][2 kernels][start, stop]
    float total_ms[2];
    int launches[2];
};

static const char* kKernelNames[2] = { "rx_front", "rx_back" };

// record event slot (kernel k, 0=start / 1=stop) of the current timed call
static void time_mark(uhsdr_rx_s* h, int k, int which)
{
    if (!h->timing) return;
    if (h->nev >= h->nev_cap) return;
    (void)hipEventRecord(h->ev[(size_t)h->nev * 4 + 2 * k + which], h->stream);
}

static void time_harvest(uhsdr_rx_s* h)
{
    if (!h->nev) return;
    (void)hipStreamSynchronize(h->stream);
    for (int i = 0; i < h->nev; ++i)
        for (int k = 0; k < 2; ++k)
        {
            float ms = 0.0f;
            if (hipEventElapsedTime(&ms, h->ev[(size_t)i * 4 + 2 * k], h->ev[(size_t)i * 4 + 2 * k + 1]) == hipSuccess)
            {
                h->total_ms[k] += ms;
                h->launches[k] += 1;
            }
        }
    h->nev = 0;
}

#define HIPCHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { uhsdr_set_error("%s: %s", #x, hipGetErrorString(e_)); return UHSDR_DEVICE_ERROR; } } while (0)

static int pad8(int t) { return (t + 7) & ~7; }

static size_t front_lds(const uhsdr_rx_s* h, int G)
{
    const int N = h->N;
    const bool dq = h->plan.use_decimated_iq;
    const int N2 = dq ? N / h->plan.decimation_rate : N;
    size_t L1 = sk_len(h->T1 - 1 + N + 8), L2 = sk_len(h->T2 - 1 + N2 + 8);
    size_t f = 2 * G * L1 + (dq ? 2 : 1) * G * L2 + 2 * G * (N / BLK);
    return f * sizeof(float);
}

static size_t back_lds(const uhsdr_rx_s* h)
{
    const int W = h->plan.agc.attack_buffsize > 0 ? h->plan.agc.attack_buffsize : 1;
    const int NG = (W + GROUP - 1) / GROUP;
    const int ndc = BLK / h->plan.decimation_rate;
    return sizeof(float) * (size_t)BACK_WAVE * (W + NG + (BLK + 1) + (ndc + 1));
}

extern "C" uhsdr_status uhsdr_rx_reset(uhsdr_rx_handle h)
{
    if (!h) return UHSDR_ARGUMENT_ERROR;
    HIPCHK(hipMemsetAsync(h->arena, 0, h->arena_bytes, h->stream));
    // oscillator starts at {I=0, Q=1} (freq_shift.c:48-49)
    float* one = (float*)malloc(sizeof(float) * h->C);
    for (int i = 0; i < h->C; ++i) one[i] = 1.0f;
    hipError_t e = hipMemcpyAsync(h->osc + h->C, one, sizeof(float) * h->C, hipMemcpyHostToDevice, h->stream);
    hipError_t e2 = hipStreamSynchronize(h->stream);
    free(one);
    HIPCHK(e);
    HIPCHK(e2);
    h->dec_samples = 0;
    return UHSDR_OK;
}

extern "C" uhsdr_status uhsdr_rx_create(const uhsdr_rx_config* cfg, int32_t C, int32_t N, void* stream,
                                        uhsdr_rx_handle* out)
{
    if (!cfg || !out || C <= 0 || N <= 0) { uhsdr_set_error("bad argument"); return UHSDR_ARGUMENT_ERROR; }
    if (N % BLK) { uhsdr_set_error("frames_per_call %d not a multiple of %d", N, BLK); return UHSDR_LENGTH_ERROR; }
    *out = nullptr;
    uhsdr_rx_s* h = (uhsdr_rx_s*)calloc(1, sizeof(uhsdr_rx_s));
    uhsdr_status st = uhsdr_rx_plan_build(cfg, &h->plan);
    if (st != UHSDR_OK) { free(h); return st; }
    if (!uhsdr_rx_plan_supported(&h->plan)) { free(h); uhsdr_set_error("demodulation mode %d not supported on device", cfg->dmod_mode); return UHSDR_UNSUPPORTED; }
    const uhsdr_rx_plan& p = h->plan;
    h->C = C; h->N = N; h->Nd = N / p.decimation_rate;
    h->stream = (hipStream_t)stream;
    if (p.use_decimated_iq) { h->T1 = p.dec_taps; h->T2 = p.hilbert_taps; }
    else { h->T1 = p.hilbert_taps; h->T2 = p.dec_taps; }
    h->T1pad = pad8(h->T1); h->T2pad = pad8(h->T2);
    // channels per front workgroup: enough FIR blocks for 256 lanes, LDS <= 64 KiB
    int G = (256 * 8) / N;
    if (G < 1) G = 1;
    if (G > 64) G = 64;
    while (G > 1 && front_lds(h, G) > 64 * 1024) --G;
    if (front_lds(h, G) > 160 * 1024) { free(h); uhsdr_set_error("block too long for LDS"); return UHSDR_LENGTH_ERROR; }
    h->G = G;
    const int W = p.agc.attack_buffsize > 0 ? p.agc.attack_buffsize : 1;

    // one arena: [front histories][teta][osc][back state]; adec separate (not state)
    size_t fl = 0;
    auto take = [&](size_t n) { size_t o = fl; fl += (n + 63) & ~(size_t)63; return o; };
    const size_t o_h1i = take((size_t)C * (h->T1 - 1)), o_h1q = take((size_t)C * (h->T1 - 1));
    const size_t o_h2i = take((size_t)C * (h->T2 - 1)), o_h2q = take((size_t)C * (h->T2 - 1));
    const size_t o_teta = take((size_t)3 * C), o_osc = take((size_t)2 * C);
    const size_t o_pre = take((size_t)10 * C), o_aa = take((size_t)10 * C), o_bq1 = take((size_t)16 * C);
    const size_t o_bq2 = take((size_t)4 * C), o_ip = take((size_t)15 * C), o_ring = take((size_t)W * C);
    const size_t o_agc = take((size_t)6 * C), o_agci = take((size_t)3 * C);
    h->arena_bytes = fl * sizeof(float);
    if (hipMalloc(&h->arena, h->arena_bytes) != hipSuccess ||
        hipMalloc((void**)&h->adec, sizeof(float) * (size_t)C * h->Nd) != hipSuccess ||
        hipMalloc((void**)&h->d_plan, sizeof(uhsdr_rx_plan)) != hipSuccess)
    {
        uhsdr_set_error("hipMalloc failed (%zu bytes state)", h->arena_bytes);
        if (h->arena) (void)hipFree(h->arena);
        if (h->adec) (void)hipFree(h->adec);
        free(h);
        return UHSDR_DEVICE_ERROR;
    }
    float* A = (float*)h->arena;
    h->hist1_i = A + o_h1i; h->hist1_q = A + o_h1q; h->hist2_i = A + o_h2i; h->hist2_q = A + o_h2q;
    h->teta = A + o_teta; h->osc = A + o_osc;
    h->bs.pre = A + o_pre; h->bs.aa = A + o_aa; h->bs.bq1 = A + o_bq1; h->bs.bq2 = A + o_bq2;
    h->bs.interp = A + o_ip; h->bs.ring = A + o_ring; h->bs.agc = A + o_agc; h->bs.agci = (int*)(A + o_agci);
    if (hipMemcpy(h->d_plan, &h->plan, sizeof(uhsdr_rx_plan), hipMemcpyHostToDevice) != hipSuccess)
    {
        uhsdr_set_error("plan upload failed");
        return UHSDR_DEVICE_ERROR;
    }
    *out = h;
    return uhsdr_rx_reset(h);
}

extern "C" uhsdr_status uhsdr_rx_set_stream(uhsdr_rx_handle h, void* stream)
{
    if (!h) return UHSDR_ARGUMENT_ERROR;
    h->stream = (hipStream_t)stream;
    return UHSDR_OK;
}

extern "C" uhsdr_status uhsdr_rx_process(uhsdr_rx_handle h, const int32_t* iq, float* audio, int32_t* dst)
{
    if (!h || !iq) { uhsdr_set_error("null argument"); return UHSDR_ARGUMENT_ERROR; }
    const uhsdr_rx_plan& p = h->plan;
    FrontArgs fa;
    fa.plan = h->d_plan;
    fa.iq = (const int2*)iq;
    fa.hist1_i = h->hist1_i; fa.hist1_q = h->hist1_q; fa.hist2_i = h->hist2_i; fa.hist2_q = h->hist2_q;
    fa.teta = h->teta; fa.osc = h->osc; fa.adec = h->adec;
    fa.C = h->C; fa.N = h->N; fa.G = h->G;
    fa.T1 = h->T1; fa.T1pad = h->T1pad; fa.T2 = h->T2; fa.T2pad = h->T2pad;
    const dim3 fgrid((h->C + h->G - 1) / h->G);
    const size_t flds = front_lds(h, h->G);
    if (h->timing && h->nev >= h->nev_cap) time_harvest(h);
    time_mark(h, 0, 0);
    if (p.decimation_rate == 4)
        hipLaunchKernelGGL((rx_front<8, 4>), fgrid, dim3(256), flds, h->stream, fa);
    else
        hipLaunchKernelGGL((rx_front<8, 2>), fgrid, dim3(256), flds, h->stream, fa);
    HIPCHK(hipGetLastError());
    time_mark(h, 0, 1);

    BackArgs ba;
    ba.plan = h->d_plan;
    ba.adec = h->adec;
    ba.audio = audio;
    ba.dst = (int2*)dst;
    ba.s = h->bs;
    ba.C = h->C; ba.N = h->N; ba.Nd = h->Nd;
    const int W = p.agc.attack_buffsize > 0 ? p.agc.attack_buffsize : 1;
    ba.ring_phase = (int)(h->dec_samples % W);
    time_mark(h, 1, 0);
    hipLaunchKernelGGL(rx_back, dim3((h->C + BACK_WAVE - 1) / BACK_WAVE), dim3(BACK_WAVE), back_lds(h), h->stream, ba);
    HIPCHK(hipGetLastError());
    time_mark(h, 1, 1);
    if (h->timing) h->nev++;
    h->dec_samples += h->Nd;
    h->kernels_last = 2;
    return UHSDR_OK;
}

extern "C" uhsdr_status uhsdr_rx_process_host(uhsdr_rx_handle h, const int32_t* iq, float* audio, int32_t* dst)
{
    if (!h || !iq) return UHSDR_ARGUMENT_ERROR;
    const size_t nf = (size_t)h->C * h->N;
    int32_t* d_iq = nullptr; float* d_a = nullptr; int32_t* d_d = nullptr;
    HIPCHK(hipMalloc((void**)&d_iq, nf * 8));
    if (audio) HIPCHK(hipMalloc((void**)&d_a, nf * 4));
    if (dst) HIPCHK(hipMalloc((void**)&d_d, nf * 8));
    HIPCHK(hipMemcpyAsync(d_iq, iq, nf * 8, hipMemcpyHostToDevice, h->stream));
    uhsdr_status st = uhsdr_rx_process(h, d_iq, d_a, d_d);
    if (st == UHSDR_OK)
    {
        if (audio) HIPCHK(hipMemcpyAsync(audio, d_a, nf * 4, hipMemcpyDeviceToHost, h->stream));
        if (dst) HIPCHK(hipMemcpyAsync(dst, d_d, nf * 8, hipMemcpyDeviceToHost, h->stream));
        HIPCHK(hipStreamSynchronize(h->stream));
    }
    (void)hipFree(d_iq);
    if (d_a) (void)hipFree(d_a);
    if (d_d) (void)hipFree(d_d);
    return st;
}

extern "C" uhsdr_status uhsdr_rx_get_plan(uhsdr_rx_handle h, uhsdr_rx_plan* plan)
{
    if (!h || !plan) return UHSDR_ARGUMENT_ERROR;
    memcpy(plan, &h->plan, sizeof *plan);
    return UHSDR_OK;
}

extern "C" int32_t uhsdr_rx_kernel_count(uhsdr_rx_handle h) { return h ? 2 : 0; }

extern "C" uhsdr_status uhsdr_rx_enable_timing(uhsdr_rx_handle h, int32_t enable)
{
    if (!h) return UHSDR_ARGUMENT_ERROR;
    if (enable && !h->ev)
    {
        h->nev_cap = 1024;
        h->ev = (hipEvent_t*)calloc((size_t)h->nev_cap * 4, sizeof(hipEvent_t));
        for (int i = 0; i < h->nev_cap * 4; ++i) HIPCHK(hipEventCreate(&h->ev[i]));
    }
    if (h->timing) time_harvest(h);
    h->timing = enable != 0;
    h->nev = 0;
    h->total_ms[0] = h->total_ms[1] = 0.0f;
    h->launches[0] = h->launches[1] = 0;
    return UHSDR_OK;
}

extern "C" int32_t uhsdr_rx_kernel_times(uhsdr_rx_handle h, float* total_ms, int32_t* launches, int32_t max_kernels)
{
    if (!h) return 0;
    time_harvest(h);
    const int n = max_kernels < 2 ? max_kernels : 2;
    for (int k = 0; k < n; ++k)
    {
        if (total_ms) total_ms[k] = h->total_ms[k];
        if (launches) launches[k] = h->launches[k];
    }
    return 2;
}

extern "C" const char* uhsdr_rx_kernel_name(int32_t index) { return (index >= 0 && index < 2) ? kKernelNames[index] : ""; }

extern "C" uhsdr_status uhsdr_rx_destroy(uhsdr_rx_handle h)
{
    if (!h) return UHSDR_ARGUMENT_ERROR;
    (void)hipStreamSynchronize(h->stream);
    if (h->ev)
    {
        for (int i = 0; i < h->nev_cap * 4; ++i) (void)hipEventDestroy(h->ev[i]);
        free(h->ev);
    }
    (void)hipFree(h->arena);
    (void)hipFree(h->adec);
    (void)hipFree(h->d_plan);
    free(h);
    return UHSDR_OK;
}
