// MI355X (gfx950) RX chain of the UHSDR firmware, batched over channels.
//
// One uhsdr_rx_process() call == N/32 consecutive AudioDriver_RxProcessor invocations
// (drivers/audio/audio_driver.c:2603-2942) on each of C independent channels.  Two kernels:
//
//  rx_front  (time-parallel: every lane busy whatever C is)
//      int32 I/Q -> f32, x 2^-16          audio_driver.c:2660-2685
//      I/Q correction (manual / auto)     audio_driver.c:2254-2316
//      FreqShift (Fs/4 or oscillator)     freq_shift.c:219-334
//      Hilbert FIR pair -> I +- Q -> decimator        (wide paths, audio_driver.c:2748-2810)
//      or decimator pair -> Hilbert pair -> I +- Q    (narrow paths, use_decimatedIQ :2718-2753)
//    -> decimated audio adec[C][N/M] (12 or 24 ksps); FIR delay lines carried in HBM.
//    Workgroup = G channels.  One LDS window per channel is filled with history + block for
//    I, then reused for Q; each lane computes R consecutive FIR outputs with the taps fully
//    unrolled (tap counts are template parameters): the sliding window lives in registers,
//    every window sample is read from LDS once per pass, coefficients come in via SGPRs.
//
//  rx_back   (sequential per channel: lane == channel, 64 channels per workgroup)
//      wave 0: IIR lattice pre-filter -> WDSP AGC -> scale -> biquad_1 -> polyphase interp
//      wave 1: anti-alias lattice -> biquad_2 -> line-out scale -> f32 / int32 codec frames
//                                         audio_driver.c:2436-2592, 2832-2923
//    The two waves form a 2-stage pipeline over 32-frame calls (wave 1 works on call k while
//    wave 0 works on call k+1), halving the serial dependency chain per channel.  All state
//    sits in registers for the whole launch; the AGC look-ahead ring sits in LDS.
//
// Arithmetic: exactly the reference's binary32 operation sequence (compiled with
// -ffp-contract=off), so outputs are bit-identical to the firmware built for x86
// (tests/test_gpu_parity.py).

#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
#include <math.h>
#include <chrono>
#include "uhsdr_internal.h"
#include "uhsdr_libm.h"
#include "uhsdr_dsp.h"

// channels per back-end workgroup (lane == channel): the unit of the device hand-off's arrival counters
#define BACK_CH 64
// arrival counters one 128-byte line apart: the front's 32 adds per group then queue on their own
// line (the atomics of a line serialise at ~12 ns each, MI355X_MICROARCH.md fanin; 64 counters
// packed in two lines made every C2 front wait for ~2048 of them)
constexpr int CNT_PITCH = 32;

struct FrontArgs
{
    const uhsdr_rx_plan* plan;
    const int2* iq;          // frame 0 of this launch; row stride ld frames (IqSample_t)
    float* hist1;            // [C][HS1][2] stage-1 FIR pair history {I, Q} (Hilbert, or I/Q decimators),
                             // HS = T-1 rounded to 4
    float* hist2;            // stage 2: [C][HS2] audio decimator history, or [C][HS2][2] pair history
                             // (decimate-first: the Hilbert pair; stereo: the decimator pair)
    const uint16_t* lanemap; // [64] pass-1 lane map of every lane: channel g << 8 | block b
    const uint16_t* lanemap2; // [64] the pass-2 FIR's lane map (front_window_pitch)
    int nb, cpw;             // lanes per channel, channels per wave
    float* teta;             // [3][C] auto I/Q correction low-pass state
    int* tp;                 // [5][C] twin-peaks detector: state, counter, restarts, runs, phase (f32 bits)
    unsigned* clip;          // optional [C]: ADC clip flags OR-ed in (uhsdr_rx_set_clip_output)
    const float* osc_in;     // [2] oscillator {I, Q} at the start of this launch (shared by all channels)
    float* osc_out;          // [2] written by workgroup 0
    float* adec;             // decimated output of this launch; row stride ldd
    float* adec_q;           // AM / SAM: decimated Q (adec holds I)
    const float* taps2a;     // first FIR pair, interleaved {c_i[k], c_q[k]} (zero-padded to 8k taps)
    const float* taps2b;     // decimate-first paths: the Hilbert pair on the decimated I/Q
    int C, N, ld, ldd;
    int lw;                  // LDS window pitch per channel (floats, multiple of 4; host picks it
                             // for conflict-free ds_read_b128, front_window_pitch)
    int comb;                // demodulator of the Hilbert pair (audio_driver.c:2755-2790, FRONT_COMB_*)
    float* fm_prev;          // FM: [2][C] the last {I, Q} of the previous launch (rx_fm's i_prev, q_prev)
    // pipelined device hand-off: the arrival counters of this launch's hand-off buffer, one per
    // 64-channel back-end group ([groups]).  Non-null: adec is stored write-through (sc1), and each
    // wave, once its stores have completed (vmcnt(0)), adds 1 to the counter of every group its
    // channels belong to -- rx_back polls them with sc1 loads (MI355X_MICROARCH.md, inter-workgroup
    // visibility: sc1 payload, drained, one agent-scope add per storing workgroup, sc1 poll and loads)
    unsigned* gcnt;
};

// what rx_front makes of the Hilbert pair (I', Q'): a_buffer[0] (and a_buffer[1] in stereo)
enum { FRONT_COMB_USB = 0,       // I + Q                      (USB, CW/DIGI upper, SSB stereo mono)
       FRONT_COMB_LSB = 1,       // I - Q
       FRONT_COMB_I = 2,         // I                          (DEMOD_IQ without stereo)
       FRONT_COMB_SSB_ST = 3,    // {I + Q, I - Q}             (DEMOD_SSBSTEREO, use_stereo)
       FRONT_COMB_IQ_ST = 4 };   // {I, Q}                     (DEMOD_IQ, use_stereo)

// the Hilbert pair's combination into a_buffer[0] for the mono families (audio_driver.c:2755-2790):
// I + Q (USB), I - Q (LSB, as I + (-Q): the same binary32 result), I (IQ mono); one wave-uniform
// branch per block instead of one per sample
template <int R>
__device__ __forceinline__ void front_comb_block(int comb, const v2f (&h)[R], float (&o)[R])
{
    if (comb == FRONT_COMB_I)
    {
#pragma unroll
        for (int r = 0; r < R; ++r) o[r] = h[r].x;
    }
    else if (comb == FRONT_COMB_LSB)
    {
#pragma unroll
        for (int r = 0; r < R; ++r) o[r] = h[r].x - h[r].y;   // I + (-Q): the same binary32 result
    }
    else
    {
#pragma unroll
        for (int r = 0; r < R; ++r) o[r] = h[r].x + h[r].y;
    }
}
__device__ __forceinline__ v2f front_comb2(int comb, v2f h)
{
    return comb == FRONT_COMB_SSB_ST ? v2f{ h.x + h.y, h.x - h.y } : h;
}

// converted, corrected, frequency-shifted sample n of a channel (audio_driver.c:2660-2705)
struct InputStage
{
    float gi, gq, ph;
    int iq_auto, shift, shift_up;
};

// FreqShift on one lane's R frames, in place on (ib, qb) = (I, Q) for FREQ_SHIFT_UP and (Q, I)
// otherwise (freq_shift.c:324).  Fs/4 exchange (freq_shift.c:219-262): frame n of a group of 4
// gets {x0, -j x1, -x2, j x3}; the lane's first frame is a multiple of 4, so n & 3 == j & 3 and
// the exchange is register renaming.  Recursive oscillator (FreqShift_Approx,
// freq_shift.c:57-101): the shared trajectory osc[2n] / osc[2n+1] from LDS.
template <int R>
__device__ __forceinline__ void freq_shift_block(float (&ib)[R], float (&qb)[R], int kind, const float* osc, int n0)
{
    if (kind == 1)
    {
#pragma unroll
        for (int j = 0; j < R; ++j)
        {
            const float iv = ib[j], qv = qb[j];
            switch (j & 3)
            {
            case 0: break;
            case 1: ib[j] = qv; qb[j] = -iv; break;
            case 2: ib[j] = -iv; qb[j] = -qv; break;
            default: ib[j] = -qv; qb[j] = iv; break;
            }
        }
    }
    else
    {
#pragma unroll
        for (int j = 0; j < R; ++j)
        {
            const float oq = osc[2 * (n0 + j)], oi = osc[2 * (n0 + j) + 1];
            const float qt = qb[j], it = ib[j];
            qb[j] = (qt * oq) - (it * oi);
            ib[j] = (it * oq) + (qt * oi);
        }
    }
}

// AudioDriver_RxHandleTwinpeaks (audio_driver.c:2173-2248) for one channel and one call, on the
// call's low-passed teta1 / teta3.  st: ts.twinpeaks_tested; cnt, rst, runs, ph: the function's
// statics twinpeaks_counter, codec_restarts, phase_IQ_runs, phase_IQ.  The smoothing and the
// threshold are double arithmetic as in the reference (0.05, 0.95 and M_PI/8.0 are doubles).
__device__ __forceinline__ void twinpeaks_step(float t1, float t3, int& st, int& cnt, int& rst, int& runs, float& ph)
{
    if (st == UHSDR_TWINPEAKS_WAIT) ++cnt;
    if (cnt > 1000)
    {
        st = UHSDR_TWINPEAKS_SAMPLING;
        cnt = 0; ph = 0.0f; runs = 0;
    }
    if (t3 != 0.0f && st == UHSDR_TWINPEAKS_SAMPLING)
    {
        const float cur = ul_asinf(t1 / t3);
        ph = runs == 0 ? cur : (float)(0.05 * (double)cur + 0.95 * (double)ph);
        if (++runs == 50)
        {
            if ((double)fabsf(ph) > (M_PI / 8.0))
            {
                st = UHSDR_TWINPEAKS_CODEC_RESTART;
                if (++rst >= 4) { st = UHSDR_TWINPEAKS_UNCORRECTABLE; rst = 0; }
            }
            else
            {
                st = UHSDR_TWINPEAKS_DONE;
                rst = 0;
            }
        }
    }
}

// ADC clip indicators of R frames (audio_driver.c:2660-2676): |I| >> IQ_BIT_SHIFT against
// ADC_CLIP_WARN_THRESHOLD (4096) and its half / quarter, magnitude taken unsigned
template <int R>
__device__ __forceinline__ unsigned clip_flags(const int4 (&raw)[R / 2])
{
    unsigned lv = 0;
#pragma unroll
    for (int j = 0; j < R; ++j)
    {
        const int v = (j & 1) ? raw[j / 2].z : raw[j / 2].x;
        const unsigned m = (unsigned)(v < 0 ? -(long long)v : (long long)v) >> 16;
        lv = lv > m ? lv : m;
    }
    return (lv > 4096u / 4 ? (unsigned)UHSDR_ADC_QUARTER_CLIP : 0u) | (lv > 4096u / 2 ? (unsigned)UHSDR_ADC_HALF_CLIP : 0u) |
           (lv > 4096u ? (unsigned)UHSDR_ADC_CLIP : 0u);
}

// R consecutive frames n0.. of one channel: int32 -> f32 x 2^-16 (audio_driver.c:2660-2685),
// I/Q correction (manual :2294-2313 via AudioDriver_IQPhaseAdjust :1776-1801, or auto with
// this call's factors m1 / m2, :2274-2293), FreqShift (:2700-2705).  Every branch is
// wave-uniform and hoisted out of the per-frame loops, so each case is straight-line code.
template <int R>
__device__ __forceinline__ void convert_block(const int4 (&raw)[R / 2], const InputStage& s, int n0, const float* m1,
                                              const float* m2, const float* osc, float (&xi)[R], float (&xq)[R])
{
#pragma unroll
    for (int j = 0; j < R; ++j)
    {
        const int vi = (j & 1) ? raw[j / 2].z : raw[j / 2].x;
        const int vq = (j & 1) ? raw[j / 2].w : raw[j / 2].y;
        xi[j] = ((float)vi) * IQ_BIT_SCALE_DOWN;
        xq[j] = ((float)vq) * IQ_BIT_SCALE_DOWN;
    }
    if (!s.iq_auto)
    {
        // x * 1.0f == x exactly: the default gains (ts.rx_adj_gain_var 1.0) skip the multiplies
        if (s.gi != 1.0f || s.gq != 1.0f)
        {
#pragma unroll
            for (int j = 0; j < R; ++j) { xi[j] = xi[j] * s.gi; xq[j] = xq[j] * s.gq; }
        }
        if (s.ph < 0)
        {
#pragma unroll
            for (int j = 0; j < R; ++j) { const float e3 = xi[j] * s.ph; xq[j] = xq[j] + e3; }
        }
        else if (s.ph > 0)
        {
#pragma unroll
            for (int j = 0; j < R; ++j) { const float e3 = xq[j] * s.ph; xi[j] = xi[j] + e3; }
        }
    }
    else
    {
        // R <= 16 frames never straddle a 32-frame call: one factor pair per lane
        const int bb = n0 / BLK;
        const float f1 = m1[bb], f2 = m2[bb];
#pragma unroll
        for (int j = 0; j < R; ++j) { xq[j] += f1 * xi[j]; xi[j] = xi[j] * f2; }
    }
    if (s.shift)
    {
        if (s.shift_up) freq_shift_block<R>(xi, xq, s.shift, osc, n0);
        else freq_shift_block<R>(xq, xi, s.shift, osc, n0);
    }
}

// One wave owns CPW = 64 / (N/R) whole channels: all data exchange stays inside the wave, so
// there is no workgroup barrier and waves from many workgroups interleave freely on a CU.
// The wave has one LDS window per channel, reused by every FIR pass:
//   Hilbert-first (wide paths):  I -> Hilbert-I (regs), Q -> Hilbert-Q, a = I +- Q (regs),
//                                a -> decimator /M -> adec
//   decimate-first (narrow):     I -> decimator (regs), Q -> decimator, dI -> Hilbert-I,
//                                dQ -> Hilbert-Q, a = hI +- hQ -> adec
// Each pass: history row + this call's samples (registers) into the window, history row for
// the next call back to HBM, then every lane runs its R-output FIR block.  All global loads
// are issued early: the I/Q frames and the first two history rows at entry, and the row of
// pass p+2 as soon as pass p has put its row into LDS (double-buffered registers), so each
// pass's HBM latency hides behind the previous pass's FIR.
// ST: use_stereo (DEMOD_SSBSTEREO / DEMOD_IQ): both channels of the pair continue -- through a
// decimator pair (DECIMATE_RX_I / _Q, audio_driver.c:2792-2801) on the Hilbert-first paths --
// into adec (a_buffer[0]) and adec_q (a_buffer[1])
// The pass of one channel group `grp` (CPW channels) by one wave over its LDS region `smem`.
// Its decimated output o[RD] (lane: channel g of the group, block b) goes to `sink(live, c, g, b,
// o)`: rx_front's sink stores it to adec in HBM, rx_chain's keeps it in LDS for the back end.
template <int T1, int T2, int M, bool DECIM_FIRST, int R, bool F, bool ST, typename Sink>
__device__ __forceinline__ void front_body(const FrontArgs& a, const int grp, float* smem, Sink&& sink)
{
    const uhsdr_rx_plan* __restrict__ P = a.plan;
    const int N = a.N, C = a.C;
    const int lane = threadIdx.x & (FRONT_WAVE - 1);
    const int nb = a.nb;                             // lanes per channel (>= 4) = N / R
    const int CPW = a.cpw;                           // channels per wave (one channel group)
    // (Measured and dropped: four independent waves per workgroup, 0.617 vs 0.600 ms at 1M x 64.)
    // lane map for the pair window (front_lane, 2R floats per lane), precomputed by the host
    const unsigned lm = a.lanemap[lane];
    const int g = (int)(lm >> 8), b = (int)(lm & 0xffu);
    const bool act = g < CPW;
    const int gs = act ? g : 0;
    const int nblk32 = N / BLK;
    constexpr int RD = R / M;                        // decimated samples per lane
    constexpr int HQ1 = hist_qp(T1), HQ2 = hist_q(T2 > 0 ? T2 : 1), HQP2 = hist_qp(T2 > 0 ? T2 : 1);
    const int LW = a.lw;
    // pass 1's pair window padded (pwin_off) where a wave holds few channels: the decimate-first
    // families (AM / SAM, narrow SSB / CW) and FM, at 8 outputs per lane (host: front_pad1)
    constexpr int PB1 = front_pad1(R, DECIM_FIRST, M);
    float* W = smem + gs * LW;                       // this channel's window
    float* aux = smem + CPW * LW;                    // auto-IQ factors [2][CPW][nblk32], osc [2N]
    float* m1 = aux;
    float* m2 = aux + CPW * nblk32;
    float* osc = aux + (P->iq_auto_correction ? 2 * CPW * nblk32 : 0);
    float* fmx = osc + ((P->freq_shift_hz != 0 && P->shift_kind == 2) ? 2 * N : 0);   // [64][2]

    InputStage in;
    in.gi = P->iq_gain_i; in.gq = P->iq_gain_q; in.ph = P->iq_phase_balance;
    in.iq_auto = P->iq_auto_correction;
    in.shift = P->freq_shift_hz != 0 ? P->shift_kind : 0;
    in.shift_up = P->shift_up;
    ctaps2_t* tA = as_taps2(a.taps2a);
    const int comb = a.comb;

    // One wave per channel group.  The I/Q frames and the stage-1 history rows are issued at
    // entry; the stage-2 rows are issued before the stage-1 FIR, so their latency hides behind it.
    // (A persistent variant that prefetched the next group's frames and rows into registers
    // doubled the VGPRs and halved the waves per SIMD: 0.67 vs 0.59 ms at 1M x 64; so did a
    // re-measurement of it in round 2, 0.656 ms, compute-bound at 2 waves per SIMD.)
    // History rows move group-coalesced (group_load_rows: whole 1 KB runs per wave instruction);
    // the I/Q frames in the lane's own (channel, block) layout.
    int4 raw[R / 2];
    vf4 hA[HQ1];
    const int c = grp * CPW + g;
    const bool live = act && c < C;
    const int cl = c < C ? c : C - 1;                // loads clamped: no exec-masked load branches
    const int c0 = grp * CPW;
    const int nlive = C - c0 < CPW ? C - c0 : CPW;   // live channels of the group
    {
        const int4* src = (const int4*)(a.iq + (size_t)cl * a.ld + b * R);
#pragma unroll
        for (int j = 0; j < R / 2; ++j) raw[j] = src[j];
        group_load_prow<T1>(a.hist1, c0, nlive, lane, hA);
    }
    if (a.clip)
    {
        const unsigned f = clip_flags<R>(raw);
        if (f && live) atomicOr(a.clip + c, f);
    }
    if (in.shift == 2 && lane == 0)
    {
        // FreqShift_Approx (freq_shift.c:57-101): the oscillator does not depend on the data,
        // so all channels share one trajectory.
        const float oc = P->osc_cos, os = P->osc_sin;
        float vi = a.osc_in[0], vq = a.osc_in[1];
        for (int n = 0; n < N; ++n)
        {
            const float oq = (vq * oc) - (vi * os);
            const float oi = (vi * oc) + (vq * os);
            osc[2 * n] = oq;
            osc[2 * n + 1] = oi;
            vq = oq; vi = oi;
            if ((n & (BLK - 1)) == BLK - 1)
            {
                const float gn = (3 - ((vq * vq) + (vi * vi))) / 2;
                vq = gn * vq; vi = gn * vi;
            }
        }
        if (grp == 0) { a.osc_out[0] = vi; a.osc_out[1] = vq; }
    }

    {
        // ---- auto I/Q statistics per 32-frame call of this group (audio_driver.c:2274-2293) ----
        if (in.iq_auto)
        {
            for (int e = lane; e < CPW * nblk32; e += FRONT_WAVE)
            {
                const int gg = e / nblk32, bb = e % nblk32;
                const int cc = grp * CPW + gg;
                float t1 = 0.0f, t2 = 0.0f, t3 = 0.0f;
                if (cc < C)
                    for (int i = 0; i < BLK; ++i)
                    {
                        const int2 v = a.iq[(size_t)cc * a.ld + bb * BLK + i];
                        const float I = ((float)v.x) * IQ_BIT_SCALE_DOWN;
                        const float Q = ((float)v.y) * IQ_BIT_SCALE_DOWN;
                        const float sI = (I < 0) ? -1.0f : ((I > 0) ? 1.0f : 0.0f);
                        const float sQ = (Q < 0) ? -1.0f : ((Q > 0) ? 1.0f : 0.0f);
                        t1 += sI * Q;
                        t2 += sI * I;
                        t3 += sQ * Q;
                    }
                m1[e] = t1;
                m2[e] = t2;
                smem[e] = t3;                        // scratch; the windows are filled later
            }
            wave_sync();
            for (int gg = lane; gg < CPW; gg += FRONT_WAVE)
            {
                const int cc = grp * CPW + gg;
                if (cc >= C) continue;
                float o1 = a.teta[cc], o2 = a.teta[C + cc], o3 = a.teta[2 * C + cc];
                int tst = a.tp[cc], tcnt = a.tp[C + cc], trst = a.tp[2 * C + cc], truns = a.tp[3 * C + cc];
                float tph = __int_as_float(a.tp[4 * C + cc]);
                for (int bb = 0; bb < nblk32; ++bb)
                {
                    const int e = gg * nblk32 + bb;
                    float t1 = m1[e], t2 = m2[e], t3 = smem[e];
                    t1 = (float)(-0.003 * (double)(t1 / (float)BLK) + 0.997 * (double)o1);
                    t2 = (float)(0.003 * (double)(t2 / (float)BLK) + 0.997 * (double)o2);
                    t3 = (float)(0.003 * (double)(t3 / (float)BLK) + 0.997 * (double)o3);
                    const float M_c1 = (t2 != 0.0f) ? t1 / t2 : 0.0f;
                    float help = (t2 * t2);
                    if (help > 0.0f) help = (t3 * t3 - t1 * t1) / help;
                    const float M_c2 = (help > 0.0f) ? sqrtf(help) : 1.0f;
                    twinpeaks_step(t1, t3, tst, tcnt, trst, truns, tph);
                    m1[e] = M_c1;
                    m2[e] = M_c2;
                    o1 = t1; o2 = t2; o3 = t3;
                }
                a.teta[cc] = o1; a.teta[C + cc] = o2; a.teta[2 * C + cc] = o3;
                a.tp[cc] = tst; a.tp[C + cc] = tcnt; a.tp[2 * C + cc] = trst; a.tp[3 * C + cc] = truns;
                a.tp[4 * C + cc] = __float_as_int(tph);
            }
        }
        wave_sync();

        // ---- this lane's R frames, converted; the I/Q branches run as FIR pairs (fir_block2)
        //      over the window {I[n], Q[n]} ----
        v2f x2[R];
        {
            float xi[R], xq[R];
            convert_block<R>(raw, in, b * R, m1 + gs * nblk32, m2 + gs * nblk32, osc, xi, xq);
#pragma unroll
            for (int j = 0; j < R; ++j) x2[j] = v2f{ xi[j], xq[j] };
        }
        group_fill_prow<T1, PB1>(smem, LW, a.hist1, c0, CPW, nlive, lane, hA);
        wave_sync();
        window_new2<PB1>(W, T1, act, b, x2, R);
        wave_sync();
        group_store_prow<T1, PB1>(smem, LW, a.hist1, c0, nlive, lane, nb * R);

        // the pass-2 FIR's own lane -> (channel, block) map: its window is filled through LDS by
        // the pass-1 lanes, so any map reads it; the host picks the one with the fewest bank
        // conflicts for the pass-2 window stride (the sink takes this identity)
        const unsigned lm2 = T2 ? a.lanemap2[lane] : lm;
        const int g2 = (int)(lm2 >> 8), b2 = (int)(lm2 & 0xffu);
        const bool act2 = g2 < CPW;
        const int c2 = grp * CPW + g2;
        const bool live2 = act2 && c2 < C;
        float* const W2 = smem + (act2 ? g2 : 0) * LW;
        float o[RD];
        if constexpr (T2 == 0)
        {
            // AM / SAM: decimate I and Q with the path's own tables (DECIMATE_RX_I / _Q,
            // audio_filter.c:1167-1176, audio_driver.c:2742-2746), no Hilbert (:2748);
            // FM: the Hilbert / low-pass pair at 48 ksps (:2748-2753), no decimation.
            // The demodulator in rx_back / rx_fm takes both I and Q.
                v2f d2[RD];
            fir_block2<T1, RD, M, F, PB1>(W + pwin_off<PB1>(b * R), tA, d2);
            if constexpr (M == 1)
            {
                // FM (the only undecimated pair): the discriminator's angle per sample
                // (AudioDriver_DemodFM, audio_driver.c:1588-1592) is not recursive, so it runs
                // here on the time-parallel lanes and rx_fm receives the angle in adec.  Each
                // sample needs the one before: in the lane, from the lane holding block b-1 of
                // the channel (LDS exchange), or for block 0 the previous launch's last sample.
                // No translation: the reference skips the demodulator and keeps its state (:1548).
                const bool translate = P->freq_shift_hz != 0;
                if (act)
                {
                    fmx[2 * (g * nb + b)] = d2[RD - 1].x;
                    fmx[2 * (g * nb + b) + 1] = d2[RD - 1].y;
                }
                wave_sync();
                const int pb = 2 * (g * nb + (b > 0 ? b - 1 : 0));
                const float li = fmx[pb], lq = fmx[pb + 1];
                const float si = a.fm_prev[cl], sq = a.fm_prev[C + cl];
                float ip = b > 0 ? li : si, qp = b > 0 ? lq : sq;
#pragma unroll
                for (int r = 0; r < RD; ++r)
                {
                    const float xi = d2[r].x, xq = d2[r].y;
                    const float y = (ip * xq) - (xi * qp);
                    const float x = (ip * xi) + (xq * qp);
                    o[r] = translate ? ul_atan2f(y, x) : 0.0f;
                    ip = xi; qp = xq;
                }
                if (translate && live && b == nb - 1)
                {
                    a.fm_prev[c] = d2[RD - 1].x;
                    a.fm_prev[C + c] = d2[RD - 1].y;
                }
            }
            else
            {
#pragma unroll
                for (int r = 0; r < RD; ++r) o[r] = d2[r].x;
                if (live)
                {
                    float* dst = a.adec_q + (size_t)c * a.ldd + b * RD;
#pragma unroll
                    for (int r = 0; r < RD; ++r) dst[r] = d2[r].y;
                }
            }
        }
        else if constexpr (!DECIM_FIRST && ST)
        {
            // stereo: {a_buffer[0], a_buffer[1]} through the decimator pair (taps2b = {dec, dec})
            vf4 hC[HQP2];
            group_load_prow<T2>(a.hist2, c0, nlive, lane, hC);
            v2f h2[R], d2[RD];
            fir_block2<T1, R, 1, F, PB1>(W + pwin_off<PB1>(b * R), tA, h2);
#pragma unroll
            for (int r = 0; r < R; ++r) h2[r] = front_comb2(comb, h2[r]);
            wave_sync();
            group_fill_prow<T2>(smem, LW, a.hist2, c0, CPW, nlive, lane, hC);
            wave_sync();
            window_new2(W, T2, act, b, h2, R);
            wave_sync();
            group_store_prow<T2>(smem, LW, a.hist2, c0, nlive, lane, nb * R);
            fir_block2<T2, RD, M, F>(W2 + 2 * b2 * R, as_taps2(a.taps2b), d2);
#pragma unroll
            for (int r = 0; r < RD; ++r) o[r] = d2[r].x;
            if (live2)
            {
                float* dst = a.adec_q + (size_t)c2 * a.ldd + b2 * RD;
#pragma unroll
                for (int r = 0; r < RD; ++r) dst[r] = d2[r].y;
            }
        }
        else if constexpr (!DECIM_FIRST)
        {
            vf4 hC[HQ2];
            group_load_rows<T2>(a.hist2, c0, nlive, lane, hC);
            v2f h2[R];
            float hs[R];
            fir_block2<T1, R, 1, F, PB1>(W + pwin_off<PB1>(b * R), tA, h2);
            front_comb_block<R>(comb, h2, hs);
            wave_sync();
            group_fill_rows<T2>(smem, LW, a.hist2, c0, CPW, nlive, lane, hC);
            wave_sync();
            window_new(W, T2, act, b, hs, R);
            wave_sync();
            group_store_rows<T2>(smem, LW, a.hist2, c0, nlive, lane, nb * R);
            fir_block<T2, RD, M, 4, F>(W2 + b2 * R, as_taps(P->dec), o);
        }
        else
        {
            vf4 hC[HQP2];
            group_load_prow<T2>(a.hist2, c0, nlive, lane, hC);
            v2f d2[RD], h2[RD];
            fir_block2<T1, RD, M, F, PB1>(W + pwin_off<PB1>(b * R), tA, d2);
            wave_sync();
            group_fill_prow<T2>(smem, LW, a.hist2, c0, CPW, nlive, lane, hC);
            wave_sync();
            window_new2(W, T2, act, b, d2, RD);
            wave_sync();
            group_store_prow<T2>(smem, LW, a.hist2, c0, nlive, lane, nb * RD);
            fir_block2<T2, RD, 1, F>(W2 + 2 * b2 * RD, as_taps2(a.taps2b), h2);
            if constexpr (ST)
            {
#pragma unroll
                for (int r = 0; r < RD; ++r)
                {
                    const v2f st2 = front_comb2(comb, h2[r]);
                    o[r] = st2.x;
                    h2[r].y = st2.y;
                }
                if (live2)
                {
                    float* dst = a.adec_q + (size_t)c2 * a.ldd + b2 * RD;
#pragma unroll
                    for (int r = 0; r < RD; ++r) dst[r] = h2[r].y;
                }
            }
            else
            {
                front_comb_block<RD>(comb, h2, o);
            }
        }
        sink(live2, c2, g2, b2, o);
    }
}

template <int T1, int T2, int M, bool DECIM_FIRST, int R, bool F, bool ST = false>
__global__ void __launch_bounds__(FRONT_WAVE) rx_front(FrontArgs a)
{
    extern __shared__ __attribute__((aligned(16))) float smem[];
    constexpr int RD = R / M;
    front_body<T1, T2, M, DECIM_FIRST, R, F, ST>(a, blockIdx.x, smem,
        [&](bool live, int c, int, int b, const float (&o)[RD])
        {
            if (!live) return;
            float* dst = a.adec + (size_t)c * a.ldd + b * RD;
            if (a.gcnt)
            {
                // device hand-off: write-through stores (the back end may be reading from another XCD)
#pragma unroll
                for (int r = 0; r < RD; ++r) __hip_atomic_store(dst + r, o[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            else if (RD % 4 == 0)
            {
#pragma unroll
                for (int r = 0; r < RD; r += 4) *(float4*)(dst + r) = make_float4(o[r], o[r + 1], o[r + 2], o[r + 3]);
            }
            else
            {
#pragma unroll
                for (int r = 0; r < RD; ++r) dst[r] = o[r];
            }
        });
    if (a.gcnt)
    {
        // arrival: every store of this wave (the workgroup) has completed, then one add per back-end
        // group its channels belong to (at most two: cpw need not divide 64)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if ((threadIdx.x & (FRONT_WAVE - 1)) == 0)
        {
            const int c0 = blockIdx.x * a.cpw;
            const int c1 = (c0 + a.cpw < a.C ? c0 + a.cpw : a.C) - 1;
            __hip_atomic_fetch_add(a.gcnt + (c0 / BACK_CH) * CNT_PITCH, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (c1 / BACK_CH != c0 / BACK_CH)
                __hip_atomic_fetch_add(a.gcnt + (c1 / BACK_CH) * CNT_PITCH, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// ------------------------------------------------------------------------------------
// rx_back: per-channel recursions.  State arrays are [field][C] (lane-coalesced).

// AGC look-ahead window (AudioAgc_RunAgcWdsp, audio_agc.c:365-429): the sample leaving the
// ring is the one W = attack_buffsize samples old, and ring_max is the maximum |x| of the W
// newest samples.  With B decimated samples per 32-frame call, W = Q*B + 1 for both rates
// (12 ksps: 49 = 6*8 + 1; 24 ksps: 97 = 6*16 + 1), so for sample j of call k the window is
//   prefix of call k [0..j]  +  calls k-1 .. k-Q+1 whole  +  suffix of call k-Q [j..B-1]
// and the leaving sample is call k-Q's sample j-1 (j > 0) or call k-Q-1's last sample.
// Per channel the kernel keeps in HBM the last Q calls' AGC inputs ([Q][B][C]: call k
// overwrites the slot of call k-Q after reading it), the Q-1 whole-call maxima and call
// k-Q-1's last sample.  max() is exact, so this equals the reference's incremental rescan.
constexpr int AGC_Q = 6;

struct BackState
{
    float* pre;      // [10][C]
    float* aa;       // [10][C]
    float* bq1;      // [16][C]
    float* bq2;      // [4][C]
    float* interp;   // [15][C]
    float* ring;     // [AGC_Q][B][C]  AGC inputs of the last AGC_Q calls
    float* ring1;    // [AGC_Q][B][C]  stereo: the second channel's AGC inputs
    float* agc;      // [8 + AGC_Q][C]  spare volts save_volts fast_bavg hang_bavg wold | call maxima[Q-1], leaving
                     // sample | stereo: wold, leaving sample of the second channel
    int* agci;       // [3][C]   hang_counter decay_type state
    float* sam;      // AM / SAM: [7 + 96][C] phs omega2 fil_out dsI dsQ dc27 dc_insert | allpass a,b,c,d[24]
    float* cw;       // CW decoder front end: [5][C] goertzel buf[1] buf[2], old_siglevel, cw_state, change
    float *pre1, *aa1, *bq1_1, *bq2_1, *interp1;   // stereo: instances [1] (audio_driver.c:78-161)
    float* notch;    // LMS auto notch: [64][C] coefficients, [64][C] state (63 used), [2][C] energy x0,
                     // [128][C] de-correlation delay line (lmsData, audio_driver.c:58-66)
};

struct BackArgs
{
    const uhsdr_rx_plan* plan;
    const float* adec;   // [C][Nd]  (AM / SAM: decimated I)
    const float* adec_q; // [C][Nd]  AM / SAM: decimated Q
    float* audio;        // [C][N]  or null: adb.a_buffer[1]
    float* audio0;       // [C][N]  or null: adb.a_buffer[0]: stereo (the second channel) or mcHF (line out)
    int2* dst;           // [C][N]  or null
    BackState s;
    int C, N, Nd;
    int ring_phase;      // (32-frame calls processed so far) mod AGC_Q
    uint8_t* cw_signal;  // optional [C][N/32]: ads.CW_signal after each call
    float* cw_energy;    // optional [C][cw_bmax]: Goertzel energy per completed CW block
    int cw_count0;       // CwDecode_RxProcessor's sample_counter at launch start (same for all channels)
    int cw_bmax;
    // LMS notch delay line (AudioDriver_NotchFilter's lms2_inbuf / lms2_outbuf, audio_driver.c:
    // 1749-1761): slot of the launch's first call in units of one call's samples, and whether that
    // call is the first since reset (both statics start at 0, so call 0 reads its own input back)
    int notch_slot0, notch_first;
    // key beep (audio_driver.c:2891-2898): frames [beep_n0, beep_n1) of this launch get the softdds
    // tone; beep_acc = the DDS accumulator at frame beep_n0 (common to all channels)
    int beep_n0, beep_n1;
    uint32_t beep_acc;
    int tone_phase;      // FM subaudible tone detector: fm_data.gcount at launch start (mod 400)
    int mchf;            // the mcHF board's output stage in line_out4 (plan.single_channel)
    // pipelined device hand-off (uhsdr_rx_set_pipelined 2): the launch reads adec once the arrival
    // counter of its group, dwait[group * CNT_PITCH] (FrontArgs::gcnt of the call's buffer), has reached
    // dtarget x the front waves of the group (dtarget = front launches into that buffer since reset;
    // wrap-safe compare), by sc1 loads; null: adec is complete at launch (a stream event ordered it).
    // The poll is bounded by spin_max polls; a give-up stores 1 to *fail (the handle's host-mapped
    // failure word: the host reports UHSDR_TIMEOUT from it) and poisons the launch (NaN inputs and
    // NaN audio for every frame).  fcpw: the front's channels per wave.
    const unsigned* dwait;
    unsigned dtarget;
    int fcpw;
    unsigned spin_max;
    unsigned* fail;
    // skewed pipeline (BackSched, rx_back with the device hand-off): adec_next = the next call's
    // hand-off buffer, read once its counters dwait_next[group] have reached dnext x the group's
    // front waves (a peek, never a wait; null: no running ahead); skew[group] = the group's pipeline
    // ends skewed; bnd = each role's pending input sub-call ([6 NDC + 2 BLK][C]: AGC role pre / rmax
    // / fb / hb, audio role agc / volts, aa mid, output aa)
    const float* adec_next;
    const unsigned* dwait_next;
    unsigned dnext;
    int* skew;
    float* bnd;
    int bnd_mid;         // bnd's field of the aa role's pending input (6 NDC); the output role's follows it
    // persistent back end (uhsdr_rx_set_pipelined 3, PersistCtl): pctl = the handle's host-mapped
    // control words, pdesc = its host-mapped ring of call descriptors, seq0 = this launch's first call;
    // null pctl: one call per launch
    unsigned* pctl;
    const struct BackDesc* pdesc;
    unsigned* pdec;
    unsigned seq0;
    unsigned pepoch;     // this launch's epoch: PC_GRANT's top byte while the host grants it calls
};

// Persistent back end (uhsdr_rx_set_pipelined 3).  One rx_back launch runs call after call with its
// roles' state in registers and their LDS hand-offs in place, instead of one launch per call: each
// launch's dispatch, state loads and stores (~5 us of a ~21 us C2 call: 3.2 us outside the waves,
// ~1.6 us entry, ~0.4 us exit; UHSDR_TRACE r06) are paid once per run of calls.  The host writes call
// k's descriptor into a ring in host-mapped memory, then grants k (PC_GRANT); the pre role, four
// sub-calls before the end of call k - 1, reads the grant and the descriptor and runs on into call k
// (BackSched's running ahead, every call), the other roles following at the step barriers.  With no
// grant it closes: it stores k - 1 to PC_EXIT, re-reads the grant after a sequentially consistent
// fence and stores its decision to PC_DECIDED; the host, after granting k, reads PC_EXIT and, when it
// finds k - 1 there, waits for that decision and relaunches if the kernel closed (Dekker: one of the
// two sees the other's store).  The grant word carries the launch's epoch (BackArgs::pepoch): uhsdr_rx_join
// and every synchronisation point end a launch after the calls granted so far by moving the host on to
// the next epoch, so the launch finds no more grants of its own (grant and close in one word: lanes of
// one load may see two words at different times).  PC_CONSUMED orders the hand-off buffers' reuse (the
// host waits before overwriting the buffer of call k - PIPE_BUFS until every channel group has read it).  The decision is
// the launch's, not each workgroup's: group 0's pre role makes it (the host protocol above) and
// publishes it per call in device memory (BackArgs::pdec); the other groups read it there, so all of
// them run the same calls.
constexpr int DESC_RING = 16;
struct BackDesc
{
    const float* adec;       // the call's hand-off buffer
    const unsigned* cnt;     // its arrival counters (FrontArgs::gcnt row)
    float* audio;
    float* audio0;
    int2* dst;
    unsigned target;         // BackArgs::dtarget of the call
    unsigned seq;            // written last: the descriptor is complete
    int beep_n0, beep_n1;
    uint32_t beep_acc;
    unsigned pad;
};
static_assert(sizeof(BackDesc) == 64, "one descriptor per 64 B");
// control words (unsigned, 64 B apart)
enum { PC_GRANT = 0, PC_EXIT = 32, PC_DECIDED = 48, PC_WORDS = 64 };
// then the descriptors, then one PC_CONSUMED word per channel group (PC_MAX_GROUPS)
constexpr int PC_CONSUMED = PC_WORDS + DESC_RING * 16, PC_MAX_GROUPS = 256;
constexpr int PC_BYTES = 4 * (PC_CONSUMED + PC_MAX_GROUPS);
// the launch's decision per call, made by group 0 and read by the others (device memory, BackArgs::pdec,
// DESC_RING words 32 apart): (call << 1) | closed
constexpr int PDEC_PITCH = 32;

// softdds_addSingleToneToTwobuffers (softdds.c:142-152): the tone of launch frame n
__device__ __forceinline__ float beep_tone(const BackArgs& a, int n)
{
    const uhsdr_rx_plan* __restrict__ P = a.plan;
    const uint32_t acc = a.beep_acc + (uint32_t)(n - a.beep_n0) * P->beep_step;
    return (float)P->dds_table[(acc >> 22) % 1024] * P->beep_scale;
}

// Math_log10f_fast, misc/uhsdr_math.c:26-39
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

// float -> int32 as the x86 reference converts (cvttss2si: out of range / NaN -> INT32_MIN),
// then << AUDIO_BIT_SHIFT (audio_driver.c:2911-2923)
__device__ __forceinline__ int to_dma(float f)
{
    const int v = (f > -2147483904.0f && f < 2147483648.0f) ? (int)f : INT32_MIN;
    return (int)((unsigned)v << 16);
}

// rx_back_fused: waves per SIMD the register allocation targets (2: 256 VGPRs, no scratch; 3
// spills to scratch and measured 0.265 vs 0.217 ms at 1M x 64)
#ifndef UHSDR_FUSED_WAVES
#define UHSDR_FUSED_WAVES 2
#endif

// demodulator kinds of rx_back (DM): the SSB/CW/DIGI sum I +- Q happens in rx_front
enum { DM_NONE = 0, DM_AM = 1, DM_SAM = 2, DM_SAM_SB = 3 /* SAM with the allpass sideband selector */,
       DM_FM = 4 /* separate kernel, rx_fm */, DM_SAM_ST = 5 /* SAM stereo: LSB and USB channels */ };
__host__ __device__ constexpr int back_roles(int dm) { return dm == DM_FM ? 2 : dm ? 6 : 5; }

// The back end of one channel group runs as a pipeline over 32-frame calls, one wave per
// stage (lane == channel); stage s works on call it - s in iteration it and hands its results
// to stage s+1 through double-buffered LDS, one workgroup barrier per iteration:
//   [demod]  AM envelope / SAM PLL (AM, SAM only)              (decimated rate)
//   pre      IIR lattice pre-filter                            (decimated rate)
//   agc      WDSP AGC                                          (decimated rate)
//   audio    post-AGC scale -> biquad_1 -> polyphase interp    (decimated rate -> 48 ksps)
//   aa       anti-alias lattice                                (48 ksps)
//   output   biquad_2 -> line-out scale -> f32 / int32 stores  (48 ksps)
// Splitting the serial chain shortens the critical path per call, which is what bounds small
// batches (one wave per SIMD).  Large batches use rx_back_fused (all stages in one wave).
// the wave pipeline splits the AGC after its recursion when there is no demod role (whose
// hand-off buffer then carries the volts) and no DC removal (AM / SAM, also behind rx_notch)
__host__ __device__ constexpr bool back_agc_split(int dm) { return dm == 0; }

struct BackLds
{
    float* dem;   // [2][NDC][64]  demod -> pre
    float* pre;   // [2][NDC][64]  pre -> agc
    float* agc;   // [2][NDC][64]  agc -> audio
    float* mid;   // [2][BLK][64]  audio -> aa
    float* aa;    // [2][BLK][64]  aa -> output
    float* prep;  // [3][2][NDC][64]  pre -> agc: window maximum, fast / hang averages
    unsigned* poison;  // [1]  pre -> output: the launch's device hand-off gave up (DM_NONE only)
    unsigned* ext;     // [1]  pre -> every role: the launch runs ahead into the next call (BackSched)
    unsigned* desc;    // [2][16]  pre -> tail: the persistent back end's call outputs (BackDesc words)
    unsigned* ctl;     // [2][32]  control tail wave -> pre role: a call's descriptor (words 0-15) and the
                       //          grant word (16), read from host memory a call ahead (PersistCtl)
    float* ys;         // [2][64][BLK + 1]  output -> tail: the output role's call, one row per channel
};

// floats of the hand-off buffers (host: back_lds)
__host__ __device__ constexpr int back_lds_floats(int ndc) { return BACK_CH * 2 * (6 * ndc + 2 * BLK) + 4 + 32 + 64 + 2 * BACK_CH * (BLK + 1); }

template <int NDC>
__device__ __forceinline__ BackLds back_lds_carve(float* smem)
{
    BackLds l;
    l.mid = smem;
    l.aa = l.mid + 2 * BLK * BACK_CH;
    l.agc = l.aa + 2 * BLK * BACK_CH;
    l.pre = l.agc + 2 * NDC * BACK_CH;
    l.dem = l.pre + 2 * NDC * BACK_CH;
    l.prep = l.dem + 2 * NDC * BACK_CH;
    l.poison = (unsigned*)(l.prep + 3 * 2 * NDC * BACK_CH);
    l.ext = l.poison + 1;
    l.desc = l.poison + 4;
    l.ctl = l.desc + 32;
    l.ys = (float*)(l.poison + 4 + 32 + 64);
    return l;
}

// Lane == channel.  c: this lane's channel; cl: clamped for loads (no exec-masked load branches).
struct BackLane
{
    int lane, c, cl, C, calls;
    bool live;
    __device__ __forceinline__ explicit BackLane(const BackArgs& a) : BackLane(a, (int)blockIdx.x) {}
    // channel group grp (channels 64 grp ..): rx_chain's waves name their group themselves
    __device__ __forceinline__ BackLane(const BackArgs& a, int grp)
    {
        lane = threadIdx.x & (BACK_CH - 1);
        c = grp * BACK_CH + lane;
        live = c < a.C;
        cl = live ? c : a.C - 1;
        C = a.C;
        calls = a.N / BLK;
    }
};

// The back-end stages below hold one channel's state in registers for a launch: load() reads
// it ([field][C], lane-coalesced), the per-call / per-sample steps run the reference's
// arithmetic, store() writes it back.  The pipelined kernel (rx_back) runs each stage in its own
// wave; the fused kernel (rx_back_fused) runs all of them per sample in one wave.

// ---- input stage (SSB / CW / DIGI): rx_front's decimated I +- Q, fetched one call ahead ----
// LDS_IN (rx_chain): the decimated samples come from the wave's own LDS hand-off `lds`,
// [sample][lane] with row pitch CHAIN_ADP, instead of adec in HBM
constexpr int CHAIN_ADP = BACK_CH + 4;

// default bound of the device hand-off's poll (uhsdr_rx_set_handoff_bound): 2^24 polls
constexpr unsigned DFLAG_SPIN_MAX = 1u << 24;
// pipelined device hand-off: the published sequence number reaches dtarget.  Bounded: after
// a.spin_max polls (>= 128 cycles each; the default 2^24 is seconds, past any rx_front the caller's
// stream can hold back behind its own work between calls) the wave gives up, stores 1 to the
// handle's host-mapped failure word (system scope: the host reads it without a synchronisation)
// and its launch is poisoned (NaN inputs in InStage::fetch, NaN audio from the output role for every
// frame), so the give-up can never pass for output
// front waves of group g (FrontArgs::gcnt's arrivals per front launch): cpw need not divide 64
__device__ __forceinline__ unsigned front_waves_of(const BackArgs& a, int g)
{
    const int c0 = g * BACK_CH, c1 = (c0 + BACK_CH < a.C ? c0 + BACK_CH : a.C) - 1;
    return (unsigned)(c1 / a.fcpw - c0 / a.fcpw + 1);
}
__device__ __forceinline__ void dflag_wait(const BackArgs& a, const unsigned* cnt, unsigned target, bool& gave_up)
{
    const int g = blockIdx.x;
    const unsigned want = target * front_waves_of(a, g);
    unsigned v = __hip_atomic_load(cnt + g * CNT_PITCH, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (unsigned spins = 0; (int)(v - want) < 0 && !gave_up; ++spins)
    {
        if (spins >= a.spin_max)
        {
            if ((threadIdx.x & (BACK_CH - 1)) == 0) __hip_atomic_store(a.fail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            gave_up = true;
        }
        __builtin_amdgcn_s_sleep(2);
        v = __hip_atomic_load(cnt + g * CNT_PITCH, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // no load moves above the poll
}

// DW: the launch may take the pipelined device hand-off (BackArgs::dwait; rx_back's pre role
// only -- the fused back ends keep the code out of their register budget)
template <int L, bool LDS_IN = false, bool DW = false, bool PERS = false>
struct InStage
{
    static constexpr int NDC = BLK / L;
    float xnext[NDC];
    const float* lds;
    bool gave_up = false;                                // DW: this launch's poll gave up
#ifdef UHSDR_PDEBUG
    unsigned arrived = 0;
#endif
    int lim = -1;                                        // prefetch bound (sub-calls); -1: the launch's calls

    __device__ __forceinline__ void fetch(const BackArgs& a, const BackLane& l, int call)
    {
        if constexpr (LDS_IN)
        {
            // a lane past the last channel reads channel C-1's column (the clamped-load rule: it
            // then stores exactly what that channel stores to the same ring address)
            const int col = l.cl - (l.c - l.lane);
#pragma unroll
            for (int m = 0; m < NDC; ++m) xnext[m] = lds[(call * NDC + m) * CHAIN_ADP + col];
            return;
        }
        if (DW && a.dwait)
        {
            // device hand-off: once per launch, wait until every front wave of the group has arrived
            // (FrontArgs::gcnt); then sc1 loads (the front's write-through stores may come from
            // another XCD while this launch runs).  After a give-up
            // every input of the launch is NaN (the failure contract of uhsdr_rx_set_pipelined)
            // (sub-calls past the launch's own: the next call's buffer, BackSched's running ahead,
            // read only after the pre role's peek found it published)
            if (call == 0) dflag_wait(a, a.dwait, a.dtarget, gave_up);
            // the persistent back end runs on into a granted call before its front has arrived
            if (PERS && a.pctl && call == l.calls)
            {
                dflag_wait(a, a.dwait_next, a.dnext, gave_up);
#ifdef UHSDR_PDEBUG
                arrived = __hip_atomic_load(a.dwait_next + blockIdx.x * CNT_PITCH, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
            }
            const float* src = call < l.calls ? a.adec + (size_t)l.cl * a.Nd + call * NDC
                                              : a.adec_next + (size_t)l.cl * a.Nd + (call - l.calls) * NDC;
#pragma unroll
            for (int m = 0; m < NDC; ++m)
            {
                const float v = __hip_atomic_load(src + m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                xnext[m] = gave_up ? __builtin_nanf("") : v;
            }
            return;
        }
        // uniform row base (SGPRs) + the lane's 32-bit offset: no 64-bit per-lane address to keep
        const float* src = a.adec + call * NDC;
        const unsigned off = (unsigned)l.cl * (unsigned)a.Nd;
#pragma unroll
        for (int m = 0; m < NDC; m += 4)
        {
            const float4 v = *(const float4*)(src + m + off);
            xnext[m] = v.x; xnext[m + 1] = v.y; xnext[m + 2] = v.z; xnext[m + 3] = v.w;
        }
    }

    __device__ __forceinline__ void begin(const BackArgs& a, const BackLane& l, int call, float (&xin)[NDC])
    {
#pragma unroll
        for (int m = 0; m < NDC; ++m) xin[m] = xnext[m];
        if (call + 1 < (lim < 0 ? l.calls : lim)) fetch(a, l, call + 1);
    }
};

// ---- IIR lattice (arm_iir_lattice_f32): the pre-filter on a_buffer[0] at the decimated rate
//      (IIR_PreFilter, audio_driver.c:2473-2482) or the anti-alias filter at 48 ksps
//      (IIR_AntiAlias, :2581-2590); state [S][C] in `st` ----
// PK: the packed form (lattice_step_pk); the fused back end keeps the scalar one, where the
// packed form's extra live pairs cost SGPR spills and scratch at no gain (it is not issue-bound)
#ifndef UHSDR_FUSED_PK
#define UHSDR_FUSED_PK false
#endif
template <int S, bool PK = true>
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

    // par: the sample's position parity in an unrolled loop (a compile-time constant there), which
    // only selects the register pairing of the packed form
    __device__ __forceinline__ float step(float x, int par = 0)
    {
        if constexpr (S > 0 && PK) return (par & 1) ? lattice_step_pk<S, 1>(x, g, k, v) : lattice_step_pk<S, 0>(x, g, k, v);
        if constexpr (S > 0 && !PK) return lattice_step<S>(x, g, k, v);
        return x;
    }

    // two consecutive samples from an even position: the ladder sums paired (lattice_step2_pk)
    __device__ __forceinline__ void step2(float x0, float x1, float& y0, float& y1)
    {
        if constexpr (S >= 3 && PK) lattice_step2_pk<S>(x0, x1, g, k, v, y0, y1);
        else
        {
            y0 = step(x0, 0);
            y1 = step(x1, 1);
        }
    }

    __device__ __forceinline__ void store(const BackLane& l, float* st)
    {
        if (!l.live) return;
#pragma unroll
        for (int i = 0; i < S; ++i) st[i * l.C + l.c] = g[i];
    }
};

// ---- agc stage: AudioAgc_RunAgcWdsp (audio_agc.c:349-595) on the pre-filtered samples ----
// NCH = 2: use_stereo (audio_agc.c:366-393, 575-593): both channels in the look-ahead ring, the
// window maximum over the larger magnitude of the pair, one gain for both, DC removal per channel
template <int L, int W, int NCH = 1>
struct AgcStage
{
    static constexpr int NDC = BLK / L;
    static_assert(W == AGC_Q * NDC + 1, "AGC window must be AGC_Q calls + 1 sample");
    // The AGC plan values live in the caller's local copy of P->agc, passed to step() (uniform
    // -> SGPRs; reading them through P inside the loop would reload them every sample since the
    // state stores may alias, and a struct member copy of it defeats SROA and lands in scratch).
    bool agc_on, dc;                                     // mode != 5; DC removal (AM / SAM)
    bool dc_sel;                                         // DC removal applied by select, not a branch
    float volts, save_volts, fast_bavg, hang_bavg, wold[NCH];
    float cmax[AGC_Q - 1];                               // maxima of calls k-Q+1 .. k-1 (oldest first)
    float leave_last[NCH];                               // last sample of call k-Q-1
    int hang_counter, decay_type, state;
    float rnext[NCH][NDC];                               // ring slot of the next call
    float old[NCH][NDC], sfx[NDC], wmax, pmax;           // this call's ring slot, suffix maxima
    float* ring_out[NCH];
    int lim = -1;                                        // ring prefetch bound (sub-calls); -1: the launch's calls

    __device__ __forceinline__ static float* ring_of(const BackArgs& a, int ch) { return ch ? a.s.ring1 : a.s.ring; }

    __device__ __forceinline__ void load(const BackArgs& a, const BackLane& l, const uhsdr_agc_plan& A)
    {
        const int C = l.C, cl = l.cl;
        agc_on = A.mode != 5;
        dc = A.remove_dc != 0;
        dc_sel = false;
        volts = a.s.agc[1 * C + cl];
        save_volts = a.s.agc[2 * C + cl];
        fast_bavg = a.s.agc[3 * C + cl];
        hang_bavg = a.s.agc[4 * C + cl];
        wold[0] = a.s.agc[5 * C + cl];
#pragma unroll
        for (int i = 0; i < AGC_Q - 1; ++i) cmax[i] = a.s.agc[(6 + i) * C + cl];
        leave_last[0] = a.s.agc[(5 + AGC_Q) * C + cl];
        if (NCH == 2)
        {
            wold[NCH - 1] = a.s.agc[(6 + AGC_Q) * C + cl];
            leave_last[NCH - 1] = a.s.agc[(7 + AGC_Q) * C + cl];
        }
        hang_counter = a.s.agci[0 * C + cl];
        decay_type = a.s.agci[1 * C + cl];
        state = a.s.agci[2 * C + cl];
    }

    // the ring slot of a call is fetched one call ahead
    __device__ __forceinline__ void fetch(const BackArgs& a, const BackLane& l, int call)
    {
        if (agc_on)
        {
            const int slot = (a.ring_phase + call) % AGC_Q;
#pragma unroll
            for (int ch = 0; ch < NCH; ++ch)
            {
                const float* rs = ring_of(a, ch) + (size_t)slot * NDC * l.C;
#pragma unroll
                for (int m = 0; m < NDC; ++m) rnext[ch][m] = rs[(size_t)m * l.C + (unsigned)l.cl];
            }
        }
    }

    // |sample| as the reference's abs_ring holds it: the larger magnitude of the pair in stereo
    template <typename F>
    __device__ __forceinline__ static float absn(F&& v)
    {
        float r = fabsf(v(0));
#pragma unroll
        for (int ch = 1; ch < NCH; ++ch) r = fmaxf(r, fabsf(v(ch)));
        return r;
    }

    // start of call `call`: take the fetched ring slot, issue the next call's fetch, suffix
    // maxima of call k-Q, maximum of the whole calls k-Q+1 .. k-1
    __device__ __forceinline__ void begin(const BackArgs& a, const BackLane& l, int call)
    {
#pragma unroll
        for (int ch = 0; ch < NCH; ++ch)
#pragma unroll
            for (int m = 0; m < NDC; ++m) old[ch][m] = rnext[ch][m];
        if (call + 1 < (lim < 0 ? l.calls : lim)) fetch(a, l, call + 1);
        sfx[NDC - 1] = absn([&](int ch) { return old[ch][NDC - 1]; });
#pragma unroll
        for (int m = NDC - 2; m >= 0; --m) sfx[m] = fmaxf(sfx[m + 1], absn([&](int ch) { return old[ch][m]; }));
        wmax = cmax[0];
#pragma unroll
        for (int i = 1; i < AGC_Q - 1; ++i) wmax = fmaxf(wmax, cmax[i]);
        pmax = 0.0f;
#pragma unroll
        for (int ch = 0; ch < NCH; ++ch)
            ring_out[ch] = ring_of(a, ch) + (size_t)((a.ring_phase + call) % AGC_Q) * NDC * l.C;
    }

    // sample m of the call, x[ch] in place.  Branch-free: the per-lane state machine is a set of
    // selects, and the ring store is unconditional (a lane past the last channel computes exactly
    // what channel C-1 computes from the clamped loads, so it stores the same value to the same
    // address), so a whole call of the fused back end is one basic block.
    // the gain the reference applies after the state update (audio_agc.c:553-560): not part of
    // the recursion, so the wave pipeline runs it in the next role
    __device__ __forceinline__ static float gain(float volts, const uhsdr_agc_plan& A)
    {
        float vo = log10f_fast(A.inv_max_input * volts);
        vo = (vo > 0.0f) ? 0.0f : vo;
        return (A.out_target - A.slope_constant * vo) / volts;
    }

    // the gain state's update from the window maximum and the two averages of the delayed
    // magnitude (audio_agc.c:431-551)
    __device__ __forceinline__ void recur(float ring_max, float fast_bavg, float hang_bavg, const uhsdr_agc_plan& A)
    {
        hang_counter = hang_counter > 0 ? hang_counter - 1 : hang_counter;
        // the 5-state attack / decay / hang machine (audio_agc.c:436-551): every case is
        // evaluated and the lane's state selects; mu = the multiplier the taken branch applies
        const float rv = ring_max - volts;
        const bool atk = ring_max >= volts;
        // bools combine with & and | (no short-circuit), so the compiler emits selects, not
        // exec-masked branches
        const bool s0 = state == 0, s1 = state == 1, s2 = state == 2, s34 = !(s0 | s1 | s2);
        const bool fast = volts > A.pop_ratio * fast_bavg;                    // case 0
        const bool hang = (A.hang_enable != 0) & (hang_bavg > A.hang_level);
        const bool fd = volts > save_volts;                                   // case 1
        const bool hc = hang_counter > 0;
        const bool dt0 = decay_type == 0;
        const bool hz = hang_counter == 0;                                    // case 2
        // without attack
        const int ns0 = fast ? 1 : hang ? 2 : 3;
        const int ns1 = fd ? 1 : hc ? 2 : dt0 ? 3 : 4;
        const int ns2 = hz ? 4 : 2;
        const int nsn = s0 ? ns0 : s1 ? ns1 : s2 ? ns2 : state;
        const bool updn = (s0 & (fast | !hang)) | (s1 & (fd | !hc)) | (s2 & hz) | s34;
        const float dm = A.decay_mult, fdm = A.fast_decay_mult, hdm = A.hang_decay_mult;
        const float mu0 = fast ? fdm : dm;
        const float mu1 = fd ? fdm : dt0 ? dm : hdm;
        const float mu3 = state == 3 ? dm : hdm;
        const float mun = s0 ? mu0 : s1 ? mu1 : s2 ? hdm : mu3;
        const bool s0_decay = s0 & !atk & !fast;                              // case 0, no attack, slow
        hang_counter = (s0_decay & hang) ? A.hang_counter_init : hang_counter;
        decay_type = s0_decay ? (hang ? 1 : 0) : decay_type;
        state = atk ? 0 : nsn;
        const bool save = atk & !s0 & !s1;
        save_volts = save ? volts : save_volts;
        const float mu = atk ? A.attack_mult : mun;
        const bool upd = atk | updn;
        const float nv = volts + rv * mu;
        volts = upd ? nv : volts;
        volts = (volts < A.min_volts) ? A.min_volts : volts;
    }

    // NCH == 1: the part of a sample that does not depend on the gain state -- the ring store,
    // the window maximum and both averages of the delayed magnitude (audio_agc.c:397-430).  The
    // wave pipeline runs it in the pre role and recur() in the AGC role; out is the delayed sample.
    struct Prep { float out, rmax, fb, hb; };
    __device__ __forceinline__ Prep prep(int m, float x, const BackLane& l, const uhsdr_agc_plan& A)
    {
        const float out = m ? old[0][m - 1] : leave_last[0];
        const float abs_out = fabsf(out);
        ring_out[0][(size_t)m * l.C + (unsigned)l.cl] = x;
        fast_bavg = A.fast_backmult * abs_out + A.onemfast_backmult * fast_bavg;
        hang_bavg = A.hang_backmult * abs_out + A.onemhang_backmult * hang_bavg;
        pmax = fmaxf(pmax, fabsf(x));
        return Prep{ out, fmaxf(fmaxf(pmax, wmax), sfx[m]), fast_bavg, hang_bavg };
    }

    __device__ __forceinline__ void stepn(int m, float (&x)[NCH], const BackLane& l, const uhsdr_agc_plan& A)
    {
        float v;
        stepn_t<true>(m, x, l, A, v);
    }

    // TAIL false (no DC removal): x <- the delayed sample, vout <- volts; the caller applies
    // gain(vout) when agc_on
    template <bool TAIL>
    __device__ __forceinline__ void stepn_t(int m, float (&x)[NCH], const BackLane& l, const uhsdr_agc_plan& A, float& vout)
    {
        // ---- AudioAgc_RunAgcWdsp, audio_agc.c:349-595 ----
        if (!agc_on)
        {
#pragma unroll
            for (int ch = 0; ch < NCH; ++ch) x[ch] = x[ch] * A.fixed_gain;
        }
        else
        {
            float out_sample[NCH];
#pragma unroll
            for (int ch = 0; ch < NCH; ++ch) out_sample[ch] = m ? old[ch][m - 1] : leave_last[ch];
            const float abs_out = absn([&](int ch) { return out_sample[ch]; });
#pragma unroll
            for (int ch = 0; ch < NCH; ++ch) ring_out[ch][(size_t)m * l.C + (unsigned)l.cl] = x[ch];
            fast_bavg = A.fast_backmult * abs_out + A.onemfast_backmult * fast_bavg;
            hang_bavg = A.hang_backmult * abs_out + A.onemhang_backmult * hang_bavg;
            pmax = fmaxf(pmax, absn([&](int ch) { return x[ch]; }));
            const float ring_max = fmaxf(fmaxf(pmax, wmax), sfx[m]);
            recur(ring_max, fast_bavg, hang_bavg, A);
            if (TAIL)
            {
                const float mult = gain(volts, A);
#pragma unroll
                for (int ch = 0; ch < NCH; ++ch) x[ch] = out_sample[ch] * mult;
            }
            else
            {
#pragma unroll
                for (int ch = 0; ch < NCH; ++ch) x[ch] = out_sample[ch];
                vout = volts;
            }
        }
        if (!TAIL) return;
        if (agc_on && dc_sel)
        {
            // the same as a select (no branch): bodies that must not split their basic block
#pragma unroll
            for (int ch = 0; ch < NCH; ++ch)
            {
                const float w = (float)((double)x[ch] + (double)wold[ch] * 0.9999);
                x[ch] = dc ? w - wold[ch] : x[ch];
                wold[ch] = dc ? w : wold[ch];
            }
        }
        else if (agc_on && dc)                          // mode 5 returns first (audio_agc.c:354-365)
        {
#pragma unroll
            for (int ch = 0; ch < NCH; ++ch)
            {
                const float w = (float)((double)x[ch] + (double)wold[ch] * 0.9999);
                x[ch] = w - wold[ch];
                wold[ch] = w;
            }
        }
    }

    __device__ __forceinline__ float step(int m, float x, const BackLane& l, const uhsdr_agc_plan& A)
    {
        float v[NCH] = { x };
        stepn(m, v, l, A);
        return v[0];
    }

    __device__ __forceinline__ void end(const BackLane& l)
    {
#pragma unroll
        for (int ch = 0; ch < NCH; ++ch) leave_last[ch] = old[ch][NDC - 1];
#pragma unroll
        for (int i = 0; i + 1 < AGC_Q - 1; ++i) cmax[i] = cmax[i + 1];
        cmax[AGC_Q - 2] = pmax;
    }

    // which[0]: the prep() side (ring, averages, DC state), which[1]: the recur() side;
    // wold_out false: the DC state belongs to another role (rx_back's audio role with DM)
    __device__ __forceinline__ void store(const BackArgs& a, const BackLane& l, const bool (&which)[2] = { true, true },
                                          bool wold_out = true)
    {
        if (!l.live) return;
        const int C = l.C, c = l.c;
        if (which[1])
        {
            a.s.agc[1 * C + c] = volts;
            a.s.agc[2 * C + c] = save_volts;
            a.s.agci[0 * C + c] = hang_counter;
            a.s.agci[1 * C + c] = decay_type;
            a.s.agci[2 * C + c] = state;
        }
        if (!which[0]) return;
        a.s.agc[3 * C + c] = fast_bavg;
        a.s.agc[4 * C + c] = hang_bavg;
        if (wold_out) a.s.agc[5 * C + c] = wold[0];
#pragma unroll
        for (int i = 0; i < AGC_Q - 1; ++i) a.s.agc[(6 + i) * C + c] = cmax[i];
        a.s.agc[(5 + AGC_Q) * C + c] = leave_last[0];
        if (NCH == 2)
        {
            a.s.agc[(6 + AGC_Q) * C + c] = wold[NCH - 1];
            a.s.agc[(7 + AGC_Q) * C + c] = leave_last[NCH - 1];
        }
    }
};

// ---- audio stage: post-AGC scale (audio_driver.c:2513-2524), biquad_1 (:2527), CW decoder
//      front end (:2550-2557), interpolator (:2560-2577) ----
template <int L, int PH, int DM>
struct AudioStage
{
    float b1[20], ic[L * PH], scale;
    float bq1[16], ip[PH > 1 ? PH - 1 : 1];
    // CW decoder front end (CwDecode_RxProcessor + CW_Decode_exe steps 1-5, cw_decoder.c:182-316,
    // 383-397) on a_buffer[0] after biquad_1; 12 ksps paths only (L == 4)
    bool cw;
    float g1, g2, cw_old, cw_r;
    bool cw_state, cw_change;
    int cw_count, cw_block, cw_bs;

    __device__ __forceinline__ void load(const BackArgs& a, const BackLane& l)
    {
        const uhsdr_rx_plan* __restrict__ P = a.plan;
        const int C = l.C, cl = l.cl;
#pragma unroll
        for (int i = 0; i < 20; ++i) b1[i] = P->biquad1[i];
#pragma unroll
        for (int i = 0; i < L * PH; ++i) ic[i] = P->interp[i];
        scale = P->post_agc_scale;
#pragma unroll
        for (int i = 0; i < 16; ++i) bq1[i] = a.s.bq1[i * C + cl];
#pragma unroll
        for (int i = 0; i < PH - 1; ++i) ip[i] = a.s.interp[i * C + cl];
        cw = L == 4 && P->cw_enabled;
        g1 = 0.0f; g2 = 0.0f; cw_old = 0.0f;
        cw_state = false; cw_change = false;
        cw_count = a.cw_count0; cw_block = 0;
        cw_bs = P->cw_blocksize;
        cw_r = P->cw_r;
        if (cw)
        {
            g1 = a.s.cw[cl]; g2 = a.s.cw[C + cl]; cw_old = a.s.cw[2 * C + cl];
            cw_state = a.s.cw[3 * C + cl] != 0.0f; cw_change = a.s.cw[4 * C + cl] != 0.0f;
        }
    }

    // one decimated sample in, L samples at 48 ksps out (out[j], j = 0..L-1)
    __device__ __forceinline__ void step(float x, float (&out)[L])
    {
        interp(step_dec(x), out);
    }

    // the decimated-rate part: scale, biquad_1, CW decoder front end
    __device__ __forceinline__ float step_dec(float x)
    {
        x = x * scale;
#pragma unroll
        for (int st = 0; st < 4; ++st)
            x = biquad_step(x, bq1[4 * st], bq1[4 * st + 1], bq1[4 * st + 2], bq1[4 * st + 3], b1 + 5 * st);
        if (cw)
        {
            // raw_signal_buffer[sample_counter++] = x; samples past blocksize are dropped
            if (cw_count < cw_bs)
            {
                const float g0 = cw_r * g1 - g2 + x;    // AudioFilter_GoertzelInput (audio_filter.c:1290-1295)
                g2 = g1;
                g1 = g0;
            }
            ++cw_count;
        }
        return x;
    }

    // polyphase interpolator: output j uses phase L-1-j (arm_fir_interpolate_f32.c:482-575)
    __device__ __forceinline__ void interp(float x, float (&out)[L])
    {
        float win[PH];
#pragma unroll
        for (int t = 0; t < PH - 1; ++t) win[t] = ip[t];
        win[PH - 1] = x;
#pragma unroll
        for (int i = L; i > 0; --i)
        {
            float sum = 0.0f;
#pragma unroll
            for (int t = 0; t < PH; ++t) sum += win[t] * ic[(i - 1) + t * L];
            out[L - i] = sum;
        }
#pragma unroll
        for (int t = 0; t + 1 < PH; ++t) ip[t] = win[t + 1];
    }

    // end of a call: a completed CW block (AudioFilter_GoertzelEnergy, audio_filter.c:1296-1305,
    // then the signal state: exponential smoothing, threshold, noise cancel, cw_decoder.c:288-316)
    __device__ __forceinline__ void end(const BackArgs& a, const BackLane& l, int call)
    {
        if (!cw) return;
        const uhsdr_rx_plan* __restrict__ P = a.plan;
        if (cw_count >= cw_bs)
        {
            const float ga = (g1 - (g2 * P->cw_cos));
            const float gb = (g2 * P->cw_sin);
            const float e = sqrtf(ga * ga + gb * gb);
            g1 = 0.0f; g2 = 0.0f;
            const float siglevel = (float)((double)e * 0.1 + (1.0 - 0.1) * (double)cw_old);
            cw_old = e;
            const bool newstate = siglevel >= P->cw_thresh;
            if (P->cw_noisecancel)
            {
                if (cw_change) { cw_state = newstate; cw_change = false; }
                else if (newstate != cw_state) cw_change = true;
            }
            else cw_state = newstate;
            if (a.cw_energy && l.live) a.cw_energy[(size_t)l.c * a.cw_bmax + cw_block] = e;
            ++cw_block;
            cw_count = 0;
        }
        if (a.cw_signal && l.live) a.cw_signal[(size_t)l.c * l.calls + call] = cw_state;
    }

    __device__ __forceinline__ void store(const BackArgs& a, const BackLane& l)
    {
        store_dec(a, l);
        store_interp(a, l);
    }

    __device__ __forceinline__ void store_interp(const BackArgs& a, const BackLane& l)
    {
        if (!l.live) return;
#pragma unroll
        for (int i = 0; i < PH - 1; ++i) a.s.interp[i * l.C + l.c] = ip[i];
    }

    __device__ __forceinline__ void store_dec(const BackArgs& a, const BackLane& l)
    {
        if (!l.live) return;
        const int C = l.C, c = l.c;
#pragma unroll
        for (int i = 0; i < 16; ++i) a.s.bq1[i * C + c] = bq1[i];
        if (cw)
        {
            a.s.cw[c] = g1; a.s.cw[C + c] = g2; a.s.cw[2 * C + c] = cw_old;
            a.s.cw[3 * C + c] = cw_state ? 1.0f : 0.0f; a.s.cw[4 * C + c] = cw_change ? 1.0f : 0.0f;
        }
    }
};

// ---- output stage: biquad_2 (audio_driver.c:2832), line-out scale (:2860; 1 on mcHF); the rest
//      of the board's output stage and the f32 audio / int32 codec frames (:2845-2923) by the
//      caller (line_out4) ----
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

// The board's output stage on four consecutive frames fr0..fr0+3 of a channel, from u = biquad_2's
// output x plan.line_out_scale (OutputStage::step); rb + off = the offset of frame fr0 in the [C][N]
// outputs (the fused back end passes a wave-uniform rb, so its addresses are an SGPR base plus a
// 32-bit lane offset); call = its 32-frame call (the key beep's test per call is wave-uniform).
//   OVI40 (USE_TWO_CHANNEL_AUDIO, audio_driver.c:2845-2923): a_buffer[1] x LINE_OUT_SCALING_FACTOR
//     in place (line_out_scale), the key beep added, dst {a1, a1}.
//   mcHF (audio_driver.c:2870-2897, 2911-2923; a.mchf): line_out_scale is 1, so u is biquad_2's
//     output; a_buffer[0] = u x LINE_OUT_SCALING_FACTOR (line_out0_scale, audio0), a_buffer[1] =
//     u x the speaker's software gain (spkr_scale, audio), the beep on a_buffer[1] only, dst {a1, a0}.
// on == false: do_mute_output (FM squelch) zeroes the buffers before the scaling and the codec frames;
// the key beep is still added to the audio.  (Round 4 ran the mcHF stage as a separate pass over a
// [C][N] scratch row the back ends wrote: +8 B per frame of HBM and one more launch per call.)
__device__ __forceinline__ void line_out4(const BackArgs& a, size_t rb, unsigned off, int call, int fr0,
                                          const float (&u)[4], bool on = true)
{
    const bool beep = a.beep_n1 > call * BLK && a.beep_n0 < (call + 1) * BLK;     // key beep in this call
    if (a.mchf)
    {
        const uhsdr_rx_plan* __restrict__ P = a.plan;
        const float sp = P->spkr_scale, lo0 = P->line_out0_scale;
        float y1[4], y0[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
        {
            const float v = on ? u[j] : 0.0f;        // +0 when squelched, before the gains as in the reference
            y1[j] = v * sp;
            y0[j] = v * lo0;
        }
        if (beep)
        {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (fr0 + j >= a.beep_n0 && fr0 + j < a.beep_n1) y1[j] += beep_tone(a, fr0 + j);
        }
        if (a.audio) *(float4*)((a.audio + rb) + off) = make_float4(y1[0], y1[1], y1[2], y1[3]);
        if (a.audio0) *(float4*)((a.audio0 + rb) + off) = make_float4(y0[0], y0[1], y0[2], y0[3]);
        if (a.dst)
        {
            int2* dd = (a.dst + rb) + off;
            int d1[4], d0[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) { d1[j] = on ? to_dma(y1[j]) : 0; d0[j] = on ? to_dma(y0[j]) : 0; }
            *(int4*)(dd) = make_int4(d1[0], d0[0], d1[1], d0[1]);
            *(int4*)(dd + 2) = make_int4(d1[2], d0[2], d1[3], d0[3]);
        }
        return;
    }
    float y[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) y[j] = on ? u[j] : 0.0f;
    if (beep)
    {
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (fr0 + j >= a.beep_n0 && fr0 + j < a.beep_n1) y[j] += beep_tone(a, fr0 + j);
    }
    if (a.audio) *(float4*)((a.audio + rb) + off) = make_float4(y[0], y[1], y[2], y[3]);
    if (a.dst)
    {
        int2* dd = (a.dst + rb) + off;
        const int d0 = on ? to_dma(y[0]) : 0, d1 = on ? to_dma(y[1]) : 0;
        const int d2 = on ? to_dma(y[2]) : 0, d3 = on ? to_dma(y[3]) : 0;
        *(int4*)(dd) = make_int4(d0, d0, d1, d1);
        *(int4*)(dd + 2) = make_int4(d2, d2, d3, d3);
    }
}


// pitch of a channel's row in the LDS output staging of the fused back end and the wave pipeline's output role (odd: conflict-free)
constexpr int FUSED_YPITCH = BLK + 1;

// a call's 32 output frames of the wave's 64 channels from LDS to HBM: lane (g, j) = (lane / 8,
// lane % 8) takes frames 4j..4j+3 of channels 8k + g, so one store instruction covers 8 rows
__device__ __forceinline__ void fused_store_call(const BackArgs& a, const BackLane& l, int call, const float* ys)
{
    wave_sync();                                         // the wave's rows are complete
    const int g = l.lane >> 3, j = l.lane & 7;
    const int c0 = l.c - l.lane;
#pragma unroll
    for (int k = 0; k < 8; ++k)
    {
        const int cc = 8 * k + g;
        const float* r = ys + cc * FUSED_YPITCH + 4 * j;
        const float v[4] = { r[0], r[1], r[2], r[3] };
        const int c = c0 + cc;
        if (c >= a.C) continue;
        // uniform base of rows c0 + 8k.. (SGPRs) + the lane's 32-bit offset
        const size_t rb = (size_t)(c0 + 8 * k) * a.N + call * BLK;
        const unsigned off = (unsigned)g * (unsigned)a.N + 4 * j;
        line_out4(a, rb, off, call, call * BLK + 4 * j, v);
    }
    wave_sync();                                         // rows read before the next call writes
}


// ---- demod stage: AudioDriver_DemodSAM (audio_driver.c:1990-2166): AM envelope
//      (:2008-2020) or the SAM PLL (:2021-2147), fade leveler (:1911-1923) ----
// LEV false (rx_back, DM_SAM): the fade leveler runs in the pre role (FadeStage) on the
// demodulated audio and corr0 (step's `corr`), which owns its state; the PLL role is the wave
// pipeline's longest, and the leveler is not part of its recursion
template <int L, int DM, bool LEV = true>
struct DemodStage
{
    static_assert(LEV || DM == DM_SAM, "the leveler leaves the demod role only for DM_SAM");
    static constexpr int NDC = BLK / L;
    static constexpr bool SB = DM == DM_SAM_SB || DM == DM_SAM_ST;   // allpass sideband selector
    static constexpr int NA = SB ? 24 : 1;                // allpass delay lines (sam_data.a..d)
    bool fade, lsb_sb;
    float dc27_1, dc_insert_1, y1;                        // stereo: channel 1 fade leveler, its output
    float mtauR, onem_mtauR, mtauI, onem_mtauI;
    float g1, g2, omega_min, omega_max;
    float phs, omega2, fil_out, dsI, dsQ, dc27, dc_insert;
    float corr;                                           // !LEV: the last step's corr0
    float ap[4][NA];
    float inext[NDC], qnext[NDC];
    float xi[NDC], xq[NDC];

    __device__ __forceinline__ void load(const BackArgs& a, const BackLane& l)
    {
        const uhsdr_rx_plan* __restrict__ P = a.plan;
        const int C = l.C, cl = l.cl;
        fade = P->fade_leveler;
        mtauR = P->fade_mtauR; onem_mtauR = P->fade_onem_mtauR;
        mtauI = P->fade_mtauI; onem_mtauI = P->fade_onem_mtauI;
        g1 = P->sam_g1; g2 = P->sam_g2; omega_min = P->sam_omega_min; omega_max = P->sam_omega_max;
        // SAM_SIDEBAND_STEREO puts the LSB demodulation in channel 0 (audio_driver.c:2091-2094)
        lsb_sb = P->sam_sideband == UHSDR_SAM_SIDEBAND_LSB || P->sam_sideband == UHSDR_SAM_SIDEBAND_STEREO;
        phs = a.s.sam[0 * C + cl]; omega2 = a.s.sam[1 * C + cl]; fil_out = a.s.sam[2 * C + cl];
        dsI = a.s.sam[3 * C + cl]; dsQ = a.s.sam[4 * C + cl];
        dc27 = a.s.sam[5 * C + cl]; dc_insert = a.s.sam[6 * C + cl];
        dc27_1 = 0.0f; dc_insert_1 = 0.0f; y1 = 0.0f;
        if (DM == DM_SAM_ST) { dc27_1 = a.s.sam[103 * C + cl]; dc_insert_1 = a.s.sam[104 * C + cl]; }
        if (SB)
        {
#pragma unroll
            for (int f = 0; f < 4; ++f)
#pragma unroll
                for (int j = 0; j < NA; ++j) ap[f][j] = a.s.sam[(7 + f * 24 + j) * C + cl];
        }
    }

    __device__ __forceinline__ void fetch(const BackArgs& a, const BackLane& l, int call)
    {
        const float* si = a.adec + call * NDC;
        const float* sq = a.adec_q + call * NDC;
        const unsigned off = (unsigned)l.cl * (unsigned)a.Nd;
#pragma unroll
        for (int m = 0; m < NDC; m += 4)
        {
            const float4 v = *(const float4*)(si + m + off);
            const float4 w = *(const float4*)(sq + m + off);
            inext[m] = v.x; inext[m + 1] = v.y; inext[m + 2] = v.z; inext[m + 3] = v.w;
            qnext[m] = w.x; qnext[m + 1] = w.y; qnext[m + 2] = w.z; qnext[m + 3] = w.w;
        }
    }

    __device__ __forceinline__ void begin(const BackArgs& a, const BackLane& l, int call)
    {
#pragma unroll
        for (int m = 0; m < NDC; ++m) { xi[m] = inext[m]; xq[m] = qnext[m]; }
        if (call + 1 < l.calls) fetch(a, l, call + 1);
    }

    __device__ __forceinline__ float fade_leveler(float audio, float corr)
    {
        dc27 = mtauR * dc27 + onem_mtauR * audio;
        dc_insert = mtauI * dc_insert + onem_mtauI * corr;
        return audio + dc_insert - dc27;
    }

    __device__ __forceinline__ float step(int m)
    {
        // demod_sam_const (audio_driver.c:1931-1953), binary32 as the firmware stores them
        const float sc0[7] = { -0.328201924180698f, -0.744171491539427f, -0.923022915444215f, -0.978490468768238f,
                               -0.994128272402075f, -0.998458978159551f, -0.999790306259206f };
        const float sc1[7] = { -0.0991227952747244f, -0.565619728761389f, -0.857467122550052f, -0.959123933111275f,
                               -0.988739372718090f, -0.996959189310611f, -0.999282492800792f };
        const double two_pi = 2.0 * (double)3.14159265358979f;   // 2.0 * PI (CMSIS/Include/arm_math.h:334)
        float audio;
        if (DM == DM_AM)
        {
            const float in = xi[m] * xi[m] + xq[m] * xq[m];
            audio = (in >= 0.0f) ? sqrtf(in) : 0.0f;      // arm_sqrt_f32, arm_math.h:5745-5771
            if (fade) audio = fade_leveler(audio, 0.0f);
        }
        else
        {
            float Sin, Cos;
            ul_sincosf(phs, &Sin, &Cos);                   // glibc-exact (uhsdr_libm.h)
            const float ai = Cos * xi[m];
            const float bi = Sin * xi[m];
            const float aq = Cos * xq[m];
            const float bq = Sin * xq[m];
            const float corr0 = ai + bq, corr1 = -bi + aq;
            if (SB)
            {
                // 7-stage allpass pair per path (audio_driver.c:2059-2097)
                ap[0][0] = dsI; ap[1][0] = bi; ap[2][0] = dsQ; ap[3][0] = aq;
                dsI = ai; dsQ = bq;
#pragma unroll
                for (int j = 0; j < 7; ++j)
                {
                    const int k = 3 * j;
#pragma unroll
                    for (int f = 0; f < 4; ++f)
                    {
                        const float cc = (f & 1) ? sc1[j] : sc0[j];
                        ap[f][k + 3] = cc * (ap[f][k] - ap[f][k + 5]) + ap[f][k + 2];
                    }
                }
                const float ai_ps = ap[0][21], bi_ps = ap[1][21], bq_ps = ap[2][21], aq_ps = ap[3][21];
#pragma unroll
                for (int j = NA - 1; j > 0; --j)
#pragma unroll
                    for (int f = 0; f < 4; ++f) ap[f][j] = ap[f][j - 1];
                audio = lsb_sb ? (ai_ps + bi_ps) - (aq_ps - bq_ps) : (ai_ps - bi_ps) + (aq_ps + bq_ps);
                if (DM == DM_SAM_ST) y1 = (ai_ps - bi_ps) + (aq_ps + bq_ps);
            }
            else
            {
                audio = corr0;
            }
            corr = corr0;
            // The whole SAM step is one basic block (fade leveler and phase wrap as bit-mask
            // selects, ul_sel; ul_sincosf / ul_atan2f branch-free): sample n + 1's phase needs only fil_out(n - 1), so the
            // scheduler overlaps two samples' sincosf -> atan2f chains.
            if (LEV)
            {
                // AudioDriver_FadeLeveler(0, ...), audio_driver.c:1911-1923
                const float d27 = mtauR * dc27 + onem_mtauR * audio;
                const float dci = mtauI * dc_insert + onem_mtauI * corr0;
                const float lev = audio + dci - d27;
                dc27 = ul_sel(fade, d27, dc27); dc_insert = ul_sel(fade, dci, dc_insert);
                audio = ul_sel(fade, lev, audio);
                if (DM == DM_SAM_ST)
                {
                    // AudioDriver_FadeLeveler(1, ...)
                    const float d27_1 = mtauR * dc27_1 + onem_mtauR * y1;
                    const float dci_1 = mtauI * dc_insert_1 + onem_mtauI * corr0;
                    const float lev1 = y1 + dci_1 - d27_1;
                    dc27_1 = ul_sel(fade, d27_1, dc27_1); dc_insert_1 = ul_sel(fade, dci_1, dc_insert_1);
                    y1 = ul_sel(fade, lev1, y1);
                }
            }
            // PLL (audio_driver.c:2128-2147)
            const float phzerror = ul_atan2f(corr1, corr0);
            const float del_out = fil_out;
            omega2 = omega2 + g2 * phzerror;
            omega2 = ul_sel(omega2 < omega_min, omega_min, ul_sel(omega2 > omega_max, omega_max, omega2));
            fil_out = g1 * phzerror + omega2;
            phs = phs + del_out;
            // The reference's while loops (in double: 2.0 * PI is a double) run at most once each:
            // |del_out| <= g1 * pi + omega_max < 2 pi for the plan's parameter ranges
            // (uhsdr_setup.c), so phs + del_out stays inside (-2 pi, 4 pi).  2 pi is a binary32
            // value T, so the comparisons are exact in binary32; phs - T is exact (Sterbenz, phs in
            // [T, 2T)); phs + T for phs in (-T, 0) is exact in double unless |phs| < 2^-27, where
            // both roundings give T -- so binary32 arithmetic returns the reference's value.
            const float two_pi_f = (float)two_pi;
            phs = ul_sel(phs >= two_pi_f, phs - two_pi_f, phs);
            phs = ul_sel(phs < 0.0f, phs + two_pi_f, phs);
        }
        return audio;
    }

    __device__ __forceinline__ void store(const BackArgs& a, const BackLane& l)
    {
        if (!l.live) return;
        const int C = l.C, c = l.c;
        a.s.sam[0 * C + c] = phs; a.s.sam[1 * C + c] = omega2; a.s.sam[2 * C + c] = fil_out;
        a.s.sam[3 * C + c] = dsI; a.s.sam[4 * C + c] = dsQ;
        if (LEV) { a.s.sam[5 * C + c] = dc27; a.s.sam[6 * C + c] = dc_insert; }
        if (DM == DM_SAM_ST) { a.s.sam[103 * C + c] = dc27_1; a.s.sam[104 * C + c] = dc_insert_1; }
        if (SB)
        {
#pragma unroll
            for (int f = 0; f < 4; ++f)
#pragma unroll
                for (int j = 0; j < NA; ++j) a.s.sam[(7 + f * 24 + j) * C + c] = ap[f][j];
        }
    }
};

// ---- fade leveler of the SAM demodulator (AudioDriver_FadeLeveler(0, ...), audio_driver.c:
//      1911-1923) as its own stage: rx_back's pre role runs it for DM_SAM (DemodStage LEV false),
//      with the state DemodStage keeps otherwise (BackState.sam rows 5, 6) ----
struct FadeStage
{
    bool fade;
    float mtauR, onem_mtauR, mtauI, onem_mtauI, dc27, dc_insert;

    __device__ __forceinline__ void load(const BackArgs& a, const BackLane& l)
    {
        const uhsdr_rx_plan* __restrict__ P = a.plan;
        fade = P->fade_leveler;
        mtauR = P->fade_mtauR; onem_mtauR = P->fade_onem_mtauR;
        mtauI = P->fade_mtauI; onem_mtauI = P->fade_onem_mtauI;
        dc27 = a.s.sam[5 * l.C + l.cl]; dc_insert = a.s.sam[6 * l.C + l.cl];
    }

    __device__ __forceinline__ float step(float audio, float corr)
    {
        const float d27 = mtauR * dc27 + onem_mtauR * audio;
        const float dci = mtauI * dc_insert + onem_mtauI * corr;
        const float lev = audio + dci - d27;
        dc27 = ul_sel(fade, d27, dc27); dc_insert = ul_sel(fade, dci, dc_insert);
        return ul_sel(fade, lev, audio);
    }

    __device__ __forceinline__ void store(const BackArgs& a, const BackLane& l)
    {
        if (!l.live) return;
        a.s.sam[5 * l.C + l.c] = dc27; a.s.sam[6 * l.C + l.c] = dc_insert;
    }
};

// ---- pipelined roles (rx_back): stage s of the wave pipeline works on call it - s in
//      iteration it; hand-offs through double-buffered LDS, one barrier per iteration ----
#ifdef UHSDR_TRACE
// timing build (tools/trace_back.py): per workgroup, role and iteration the shader clock when the
// role starts its call, ends it, and leaves the barrier
__device__ unsigned long long g_trace[64][10][40][3];
#define TRACE_MARK(k) do { if (l.lane == 0 && blockIdx.x < 64 && it < 40) \
    g_trace[blockIdx.x][threadIdx.x / BACK_CH][it][k] = __builtin_readcyclecounter(); } while (0)
extern "C" int uhsdr_trace_read(void* out)
{
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_trace), sizeof(g_trace)) == hipSuccess ? 0 : -1;
}
#else
#define TRACE_MARK(k) do { } while (0)
#endif
// Skewed pipeline (the device hand-off's back end, DM_NONE).  A launch of n
// 32-frame calls used to take n + 4 lockstep steps: 4 of them pipeline fill (the later roles idle)
// and drain (the earlier roles idle).  Sub-calls are numbered g relative to the launch's first; role
// r at step `it` works on g = it - r + gofs.  When the next call's rx_front has already published
// (the pre role peeks the sequence word; it never waits for it), roles 0 .. 3 run ahead into the
// next call's first 4 - r sub-calls instead of idling (`ext`: role r's range ends at n + 4 - r
// instead of n), every role stores its state as usual, and each role r >= 1 writes the one sub-call
// of input it has not consumed (its LDS hand-off slot) to `bnd` in HBM.  The group's skew word
// records it, and the next launch starts skewed (`pin`: gofs = 4, n steps, no fill): role r loads
// its pending input from `bnd` and continues at g = 4 - r.  Each role still runs its recursion over
// the same samples in the same order, so outputs stay bit-identical; the output role (r = 4) always
// covers exactly the launch's own n sub-calls.  A launch that finds the next call unpublished drains
// as before and the next one fills.
constexpr int BACK_SKEW = 4;            // back_roles(DM_NONE) - 1
// BackSched's second chance at running ahead (rx_back_pre): 0 decides on the early peek alone
#ifndef UHSDR_LATE_EXT
#define UHSDR_LATE_EXT 1
#endif
// and its pre role's speculative first input of a skewed launch: 0 loads it after the skew word
#ifndef UHSDR_SPEC_IN
#define UHSDR_SPEC_IN 1
#endif
struct BackSched
{
    int steps, gofs;
    bool pin;       // this launch starts skewed (the previous one ran ahead into its call)
    bool may_ext;   // it may run ahead into the next call (device hand-off, a.adec_next)
    // the group's skew word is loaded first (word) and consumed after the role's state loads and
    // its speculative `bnd` loads (make), so one memory latency covers all of them at launch start
    // (consumed at once it cost a second round trip: ~1.5 k cycles of entry, UHSDR_TRACE r06)
    template <int DM>
    __device__ __forceinline__ static int word(const BackArgs& a)
    {
        if constexpr (DM == DM_NONE) return a.skew ? a.skew[blockIdx.x] : 0;
        else return 0;
    }
    template <int DM, bool PERS = false>
    __device__ __forceinline__ static BackSched make(const BackArgs& a, const BackLane& l, int w)
    {
        BackSched s;
        s.pin = false;
        s.may_ext = false;
        if constexpr (DM == DM_NONE)
        {
            s.pin = __builtin_amdgcn_readfirstlane(w) != 0;
            s.may_ext = a.adec_next != nullptr || (PERS && a.pctl != nullptr);
        }
        s.gofs = s.pin ? BACK_SKEW : 0;
        s.steps = l.calls + (s.pin ? 0 : back_roles(DM) - 1);
#ifdef UHSDR_TRACE
        // (tools/trace_back.py) the skew word consumed: the role's launch-start loads have arrived
        if ((threadIdx.x & (BACK_CH - 1)) == 0 && blockIdx.x < 64)
            g_trace[blockIdx.x][threadIdx.x / BACK_CH][39][2] = __builtin_readcyclecounter();
#endif
        return s;
    }
    // the persistent back end's next call (PersistCtl): it started skewed, its predecessor ran ahead
    __device__ __forceinline__ static BackSched next(const BackLane& l)
    {
        BackSched s;
        s.pin = true;
        s.may_ext = true;
        s.gofs = BACK_SKEW;
        s.steps = l.calls;
        return s;
    }
};
#ifdef UHSDR_PDEBUG
// (tools/debug_persist2.py) per call (seq % 64), group 0's pre role: seq, adec_next, cnt, target,
// arrival count after the wait, dst from the descriptor, fast path, gave up
__device__ unsigned long long g_pdbg[64][8];
__device__ unsigned long long g_pdbg2[64][4][2];   // per call and group 0..3: decision word seen, polls
__device__ unsigned long long g_ptime[1024][8];    // per call (seq % 1024): group 0 at g = 4 / n-4 / n-1 / after the decision / n-3 after the grant / n-2; group 1 before / after its decision
extern "C" int uhsdr_pdbg_read(void* out)
{
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pdbg), sizeof(g_pdbg)) != hipSuccess) return -1;
    if (hipMemcpyFromSymbol((char*)out + sizeof(g_pdbg), HIP_SYMBOL(g_pdbg2), sizeof(g_pdbg2)) != hipSuccess) return -1;
    return hipMemcpyFromSymbol((char*)out + sizeof(g_pdbg) + sizeof(g_pdbg2), HIP_SYMBOL(g_ptime), sizeof(g_ptime)) == hipSuccess ? 0 : -1;
}
#endif
// the persistent back end (PersistCtl): its control words and descriptors live in host memory
__device__ __forceinline__ unsigned sys_load(const unsigned* p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// PC_GRANT = epoch << 24 | the last call granted (24 bits): one word, so a launch never sees a later
// launch's grant (a close is the host moving on to the next epoch); call s may run in the launch of
// epoch `epoch` if the word carries that epoch and a call at or past s
__device__ __forceinline__ bool pers_granted(unsigned epoch, unsigned s, unsigned grant)
{
    return (grant >> 24) == (epoch & 0xFFu) && (int)(((grant & 0xFFFFFFu) - (s & 0xFFFFFFu)) << 8) >= 0;
}
// a descriptor, one 32-bit word per lane 0..15 (one VGPR while its loads are in flight; PersistCtl)
__device__ __forceinline__ unsigned desc_word_load(const BackDesc* d, int lane)
{
    return sys_load((const unsigned*)d + (lane & 15));
}
// (the builtins return int: through unsigned, so a low word is never sign-extended into the high one)
__device__ __forceinline__ unsigned desc_u32(unsigned w, int i) { return (unsigned)__builtin_amdgcn_readlane(w, i); }
__device__ __forceinline__ unsigned long long desc_u64(unsigned w, int i)
{
    return (unsigned long long)desc_u32(w, i + 1) << 32 | desc_u32(w, i);
}
// BackDesc's word offsets
enum { DW_ADEC = 0, DW_CNT = 2, DW_AUDIO = 4, DW_AUDIO0 = 6, DW_DST = 8, DW_TARGET = 10, DW_SEQ = 11,
       DW_BEEP0 = 12, DW_BEEP1 = 13, DW_BACC = 14 };
// the tail waves' copy of a call's descriptor (lds.desc [2][16])
__device__ __forceinline__ void desc_get(BackArgs& a, const unsigned* slot)
{
    auto w = [&](int i) { return (unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane(slot[i]); };
    a.audio = (float*)(w(DW_AUDIO + 1) << 32 | w(DW_AUDIO));
    a.audio0 = (float*)(w(DW_AUDIO0 + 1) << 32 | w(DW_AUDIO0));
    a.dst = (int2*)(w(DW_DST + 1) << 32 | w(DW_DST));
    a.beep_n0 = (int)w(DW_BEEP0);
    a.beep_n1 = (int)w(DW_BEEP1);
    a.beep_acc = (uint32_t)w(DW_BACC);
}
// BackSched's pending input sub-call of a role, loaded from `bnd` before the role knows whether the
// launch starts skewed (unused otherwise); put() moves rows [R0, R0 + n) into an LDS hand-off slot
template <int ROWS>
struct BndRegs
{
    float v[ROWS];
    template <int DM>
    __device__ __forceinline__ void load(const BackArgs& a, const BackLane& l, int f0)
    {
        if constexpr (DM == DM_NONE)
        {
            if (a.bnd)
            {
#pragma unroll
                for (int m = 0; m < ROWS; ++m) v[m] = a.bnd[(size_t)(f0 + m) * l.C + l.cl];
            }
        }
    }
    template <int R0, int NR>
    __device__ __forceinline__ void put(const BackLane& l, float* slot) const
    {
#pragma unroll
        for (int m = 0; m < NR; ++m) slot[m * BACK_CH + l.lane] = v[R0 + m];
    }
};
// role ST's range of sub-calls is [.., glim): l.calls, or with `ext` l.calls + BACK_SKEW - ST -- roles
// ST >= 1 learn `ext` from the pre role's LDS word (written in the step that made the decision, at
// g = n - 1 of role 0, a step barrier before any other role reaches g = n)
#define BACK_ROLE_LOOP(ST)                                                                     \
    for (int it = 0; it < sch.steps; ++it)                                                     \
    {                                                                                          \
        const int call = it - (ST) + sch.gofs;                                                 \
        if ((ST) > 0 && sch.may_ext && call == l.calls)                                        \
            glim = __builtin_amdgcn_readfirstlane(*lds.ext) ? l.calls + BACK_SKEW - (ST) : l.calls; \
        TRACE_MARK(0);                                                                         \
        if (call >= 0 && call < glim)                                                          \
        {
#define BACK_ROLE_END                                                                          \
        }                                                                                      \
        TRACE_MARK(1);                                                                         \
        lds_barrier();                                                                         \
        TRACE_MARK(2);                                                                         \
    }

template <int L, int DM>
__device__ __forceinline__ void rx_back_demod(const BackArgs& a, BackLds lds)
{
    const BackLane l(a);
    constexpr int NDC = BLK / L;
    constexpr bool LEV = DM != DM_SAM;                   // DM_SAM: the leveler runs in the pre role
    const BackSched sch = BackSched::make<DM>(a, l, 0);
    int glim = l.calls;
    DemodStage<L, DM, LEV> s;
    s.load(a, l);
    s.fetch(a, l, 0);
    BACK_ROLE_LOOP(0)
        s.begin(a, l, call);
        float* dout = lds.dem + (call & 1) * NDC * BACK_CH + l.lane;
        float* cout = lds.prep + (call & 1) * NDC * BACK_CH + l.lane;   // corr0 (prep is free with DM)
#pragma unroll
        for (int m = 0; m < NDC; ++m)
        {
            dout[m * BACK_CH] = s.step(m);
            if (!LEV) cout[m * BACK_CH] = s.corr;
        }
    BACK_ROLE_END
    s.store(a, l);
}

// BackSched's pending input sub-call of a role: ROWS rows of its LDS hand-off slot ([m][64]) to bnd's
// fields f0 .. f0 + ROWS - 1 ([field][C], lane-coalesced; BndRegs loads them back)
template <int ROWS>
__device__ __forceinline__ void bnd_store(const BackArgs& a, const BackLane& l, int f0, const float* slot)
{
    if (!l.live) return;
#pragma unroll
    for (int m = 0; m < ROWS; ++m) a.bnd[(size_t)(f0 + m) * l.C + l.c] = slot[m * BACK_CH + l.lane];
}
// the launch ran ahead (the pre role's word; BackSched): read after the loop's last barrier
__device__ __forceinline__ bool back_ext(const BackSched& sch, const BackLds& lds)
{
    return sch.may_ext && __builtin_amdgcn_readfirstlane(*lds.ext) != 0;
}

// the AGC's ring side (AgcStage::prep) runs in the pre role, its recursion in the AGC role and
// its gain in the audio role: SSB / CW / DIGI with the AGC on and no DC removal
__device__ __forceinline__ bool back_agc_prep_in_pre(int dm, const uhsdr_agc_plan& A)
{
    return back_agc_split(dm) && !A.remove_dc && A.mode != 5;
}

// IIR lattice pre-filter; input: rx_front's decimated I +- Q (SSB) or the demod role's output
template <int PRE, int L, int W, int DM, bool PERS>
__device__ __forceinline__ void rx_back_pre(const BackArgs& a0, BackLds lds)
{
    BackArgs a = a0;                                   // the call's (the persistent back end moves it on)
    const BackLane l(a);
    constexpr int NDC = BLK / L;
    const uhsdr_rx_plan* __restrict__ P = a.plan;
    const int skw = BackSched::word<DM>(a);
    InStage<L, false, true, PERS> in;
    LatticeStage<PRE> s;
    s.load(l, P->pre_k, P->pre_v, a.s.pre);
    const uhsdr_agc_plan A = P->agc;
    const bool prep = back_agc_prep_in_pre(DM, A);
    AgcStage<L, W> ag;
    if (prep) ag.load(a, l, A);
    // a launch that starts skewed takes sub-call BACK_SKEW first: its input (found arrived by the
    // previous launch's peek, a kernel boundary ago) and ring slot are loaded before the skew word is
    // consumed, so the role's entry waits one memory latency, not two (UHSDR_SPEC_IN)
    const bool spec = UHSDR_SPEC_IN && DM == DM_NONE && a.skew && l.calls > BACK_SKEW;
    if (spec)
    {
        in.fetch(a, l, BACK_SKEW);
        if (prep) ag.fetch(a, l, BACK_SKEW);
    }
    BackSched sch = BackSched::make<DM, PERS>(a, l, skw);
    const bool have = spec && sch.pin;                 // g0's input and ring slot are in flight
    int glim = l.calls;
    // BackSched: the first sub-call of this role, and whether it runs ahead into the next call -- a
    // peek of the next buffer's arrival counter (never a wait) issued at g = n - 3 and consumed two
    // steps later, at g = n - 1, so its latency stays off the step (a load consumed at once cost
    // ~1-2 us in the pipeline's lockstep); at once when the launch's range starts past those points
    const int g0 = sch.gofs;
    unsigned seen = 0;                                 // per lane until decide() (no wait at the peek)
    bool ext = false;
    auto peek = [&]() {
        seen = __hip_atomic_load(a.dwait_next + blockIdx.x * CNT_PITCH, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    auto decide = [&]() {
        ext = (int)(__builtin_amdgcn_readfirstlane(seen) - a.dnext * front_waves_of(a, blockIdx.x)) >= 0;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // the next call's loads stay below
        glim = ext ? l.calls + BACK_SKEW : l.calls;
        in.lim = glim;
        if (l.lane == 0) *lds.ext = ext ? 1u : 0u;
    };
    // the persistent back end (PersistCtl): four sub-calls before the end of a call the grant, the
    // close word and the next descriptor's seq are read; the descriptor itself once its seq has
    // arrived (written before it); the decision at the call's last sub-call (pers_decide)
    const bool pers = PERS && DM == DM_NONE && a.pctl != nullptr;
    unsigned seq = a.seq0;
    // lane 0 PC_GRANT, lane 2 the next descriptor's seq (one load: the two may be seen at different
    // times, hence the grant's epoch in the same word as the call); then the descriptor, word per lane
    // (one VGPR each while in flight)
    unsigned pv = 0, dw = 0, dv = 0;
    bool fast = false;                                 // the next descriptor was found complete
    bool ldone = false;                                // group 0: the decision is published
    const bool leader = blockIdx.x == 0;
    auto pdesc = [&](unsigned k) { return a.pdesc + (k % DESC_RING); };
    auto pctl_load = [&]() {
        const unsigned* p = l.lane == 0 ? a.pctl + PC_GRANT : (const unsigned*)pdesc(seq + 1) + DW_SEQ;
        pv = sys_load(p);
    };
    auto pdec = [&](unsigned k) { return a.pdec + (k % DESC_RING) * PDEC_PITCH; };
    auto publish = [&](unsigned k, bool go) {
        if (l.lane == 0) (void)__hip_atomic_exchange(pdec(k), (k << 1) | (go ? 0u : 1u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    auto pers_decide = [&]() {
        const unsigned s1 = seq + 1;
        bool go = ldone;
        if (leader && !ldone)
        {
            // closing: announce it, then look again (the host, having granted s1, looks at PC_EXIT)
            if (l.lane == 0) __hip_atomic_store(a.pctl + PC_EXIT, seq, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_SYSTEM);
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "");
            pctl_load();
            go = pers_granted(a.pepoch, s1, desc_u32(pv, 0));
            if (go)
            {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // the descriptor was written before the grant
                dw = desc_word_load(pdesc(s1), l.lane);
            }
            publish(s1, go);
            if (l.lane == 0)
                __hip_atomic_store(a.pctl + PC_DECIDED, (seq << 1) | (go ? 0u : 1u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        if (!leader)
        {
            // group 0's decision (loaded a step ago; polled if not there yet, bounded)
            const unsigned want = s1 & 0x7FFFFFFFu;
            unsigned v = __builtin_amdgcn_readfirstlane(dv);
            for (unsigned spins = 0; (v >> 1) != want && !in.gave_up; ++spins)
            {
                if (spins >= a.spin_max)
                {
                    if (l.lane == 0) __hip_atomic_store(a.fail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    in.gave_up = true;                 // this group stops here, its output poisoned
                }
                __builtin_amdgcn_s_sleep(2);
                v = __builtin_amdgcn_readfirstlane(__hip_atomic_load(pdec(s1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            }
            go = (v >> 1) == want && !(v & 1u);
#ifdef UHSDR_PDEBUG
            if (blockIdx.x < 4 && l.lane == 0) { g_pdbg2[s1 % 64][blockIdx.x][0] = v; g_pdbg2[s1 % 64][blockIdx.x][1] = in.gave_up; }
#endif
            if (go && !fast)
            {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // written before the grant group 0 saw
                dw = desc_word_load(pdesc(s1), l.lane);
            }
        }
        ext = go;
        if (go)
        {
            a.adec_next = (const float*)desc_u64(dw, DW_ADEC);
            a.dwait_next = (const unsigned*)desc_u64(dw, DW_CNT);
            a.dnext = desc_u32(dw, DW_TARGET);
            if (l.lane < 16) lds.desc[(s1 & 1) * 16 + l.lane] = dw;   // the tail waves' copy
#ifdef UHSDR_PDEBUG
            if (blockIdx.x == 0 && l.lane == 0)
            {
                unsigned long long* r = g_pdbg[s1 % 64];
                r[0] = s1; r[1] = (unsigned long long)a.adec_next; r[2] = (unsigned long long)a.dwait_next;
                r[3] = a.dnext; r[5] = desc_u64(dw, DW_DST); r[6] = fast;
            }
#endif
        }
        glim = go ? l.calls + BACK_SKEW : l.calls;
        in.lim = go ? l.calls + BACK_SKEW + 1 : l.calls;  // + the next call's first sub-call of this role
        if (l.lane == 0) *lds.ext = go ? 1u : 0u;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    if (sch.may_ext)
    {
        ag.lim = l.calls + BACK_SKEW + (pers ? 1 : 0);   // the ring slots do not depend on the front
        if (!pers && g0 > l.calls - 3) peek();
        if (!pers && g0 >= l.calls) decide();
    }
    if (!DM)
    {
        if (g0 < glim && !have) in.fetch(a, l, g0);
        // the failure contract: a give-up (InStage's poll, call 0) poisons the whole launch's output,
        // including the frames the AGC's look-ahead delay still takes from the previous launch's
        // samples -- the output role reads this after the step-0 barrier
        if (l.lane == 0) *lds.poison = in.gave_up ? 1u : 0u;
    }
    if (prep && !have) ag.fetch(a, l, g0);
    FadeStage fl;
    if (DM == DM_SAM) fl.load(a, l);
    for (;;)
    {
    BACK_ROLE_LOOP(DM ? 1 : 0)
        if (pers)
        {
#ifdef UHSDR_PDEBUG
            if (blockIdx.x == 0 && l.lane == 0)
            {
                if (call == 4) g_ptime[seq % 1024][0] = __builtin_amdgcn_s_memrealtime();
                if (call == l.calls - 4) g_ptime[seq % 1024][1] = __builtin_amdgcn_s_memrealtime();
                if (call == l.calls - 1) g_ptime[seq % 1024][2] = __builtin_amdgcn_s_memrealtime();
            }
#endif
            // after the launch's first call the control tail wave has read this call's grant and
            // descriptor from host memory during the previous call (rx_back_tail): LDS reads here. A
            // host-memory load of this wave's own would hold up its next HBM load's wait (one in-order
            // vmcnt): 5-9 us per call measured (UHSDR_PDEBUG, tools/debug_persist3.py)
            const bool have_ctl = seq != a.seq0;
            if (call == l.calls - 4 && !have_ctl) pctl_load();
            if (call == l.calls - 3)
            {
                unsigned gw;
                if (have_ctl)
                {
                    const unsigned* c = lds.ctl + ((seq + 1) & 1) * 32;
                    dw = c[l.lane & 15];
                    gw = __builtin_amdgcn_readfirstlane(c[16]);
                    // complete only if the control wave saw the grant before reading it (the host
                    // writes the descriptor first; lanes of one load may see it half written)
                    fast = desc_u32(dw, DW_SEQ) == seq + 1 && pers_granted(a.pepoch, seq + 1, gw);
                }
                else
                {
                    fast = desc_u32(pv, 2) == seq + 1;
                    gw = desc_u32(pv, 0);
                    if (fast)
                    {
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                        dw = desc_word_load(pdesc(seq + 1), l.lane);
                    }
                }
#ifdef UHSDR_PDEBUG
                if (blockIdx.x == 0 && l.lane == 0) g_ptime[seq % 1024][4] = __builtin_amdgcn_s_memrealtime();
#endif
                // group 0: granted already -- published now, two steps before the others need it
                if (leader && fast && pers_granted(a.pepoch, seq + 1, gw))
                {
                    publish(seq + 1, true);
                    ldone = true;
                }
            }
            if (call == l.calls - 2 && !leader) dv = __hip_atomic_load(pdec(seq + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#ifdef UHSDR_PDEBUG
            if (call == l.calls - 2 && blockIdx.x == 0 && l.lane == 0) g_ptime[seq % 1024][5] = __builtin_amdgcn_s_memrealtime();
            if (call == l.calls - 1 && blockIdx.x == 1 && l.lane == 0) g_ptime[seq % 1024][6] = __builtin_amdgcn_s_memrealtime();
#endif
            if (call == l.calls - 1) pers_decide();
#ifdef UHSDR_PDEBUG
            if (call == l.calls - 1 && blockIdx.x == 1 && l.lane == 0) g_ptime[seq % 1024][7] = __builtin_amdgcn_s_memrealtime();
            if (call == l.calls - 1 && blockIdx.x == 0 && l.lane == 0) g_ptime[seq % 1024][3] = __builtin_amdgcn_s_memrealtime();
#endif
        }
        else if (sch.may_ext)
        {
            if (call == l.calls - 3) peek();
            if (call == l.calls - 1)
            {
                decide();
                // second chance (UHSDR_LATE_EXT): the next call had not arrived two steps ago -- peek
                // again now and consume it at this step's end, where the step's work has hidden it
                if (UHSDR_LATE_EXT && !ext) peek();
            }
        }
        float xin[NDC];
        if (DM)
        {
            const float* di = lds.dem + (call & 1) * NDC * BACK_CH + l.lane;
#pragma unroll
            for (int m = 0; m < NDC; ++m) xin[m] = di[m * BACK_CH];
            if (DM == DM_SAM)
            {
                const float* ci = lds.prep + (call & 1) * NDC * BACK_CH + l.lane;
                float cr[NDC];
#pragma unroll
                for (int m = 0; m < NDC; ++m) cr[m] = ci[m * BACK_CH];
#pragma unroll
                for (int m = 0; m < NDC; ++m) xin[m] = fl.step(xin[m], cr[m]);
            }
        }
        else
            in.begin(a, l, call, xin);
        float* po = lds.pre + (call & 1) * NDC * BACK_CH + l.lane;
        if (prep)
        {
            // to the AGC role: the delayed sample, window maximum and both averages
            float* pr = lds.prep + (call & 1) * NDC * BACK_CH + l.lane;
            float* pf = pr + 2 * NDC * BACK_CH;
            float* ph = pf + 2 * NDC * BACK_CH;
            float y[NDC];
#pragma unroll
            for (int m = 0; m < NDC; ++m) y[m] = s.step(xin[m], m);
            ag.begin(a, l, call);
#pragma unroll
            for (int m = 0; m < NDC; ++m)
            {
                const auto q = ag.prep(m, y[m], l, A);
                po[m * BACK_CH] = q.out;
                pr[m * BACK_CH] = q.rmax;
                pf[m * BACK_CH] = q.fb;
                ph[m * BACK_CH] = q.hb;
            }
            ag.end(l);
        }
        else
        {
#pragma unroll
            for (int m = 0; m < NDC; ++m) po[m * BACK_CH] = s.step(xin[m], m);
        }
        if (UHSDR_LATE_EXT && !pers && sch.may_ext && call == l.calls - 1 && !ext)
        {
            decide();                                  // the LDS word is read after this step's barrier
            if (ext) in.fetch(a, l, l.calls);          // g = n, consumed by in.begin at the next step
        }
#ifdef UHSDR_PDEBUG
        if (pers && call == l.calls - 1 && ext && blockIdx.x == 0 && l.lane == 0)
        {
            g_pdbg[(seq + 1) % 64][4] = __builtin_amdgcn_readfirstlane(in.arrived);
            g_pdbg[(seq + 1) % 64][7] = in.gave_up;
        }
#endif
        if (pers)
        {
            // a give-up poisons the output from here on (the output role reads the word every sub-call)
            if (l.lane == 0 && in.gave_up) *lds.poison = 1u;
            // (PC_CONSUMED: stored by the control tail wave a step later, off this wave's vmcnt)
        }
    BACK_ROLE_END
        if (!pers || !ext) break;
        // on into the next call: its buffer and counters become the launch's own
        a.adec = a.adec_next;
        a.dwait = a.dwait_next;
        a.dtarget = a.dnext;
        a.ring_phase = (a.ring_phase + l.calls) % AGC_Q;
        seq += 1;
        sch = BackSched::next(l);
        glim = l.calls;
        in.lim = l.calls;
        ext = false;
        fast = false;
        ldone = false;
    }
    s.store(l, a.s.pre);
    if (DM == DM_SAM) fl.store(a, l);
    if (prep) ag.store(a, l, { true, false });
    if (DM == DM_NONE && a.skew && l.lane == 0) a.skew[blockIdx.x] = ext ? 1 : 0;   // the next launch's `pin`
}

template <int L, int W, int DM, bool PERS>
__device__ __forceinline__ void rx_back_agc(const BackArgs& a0, BackLds lds)
{
    BackArgs a = a0;                                   // the call's ring phase moves on (PersistCtl)
    const BackLane l(a);
    constexpr int NDC = BLK / L;
    const uhsdr_rx_plan* __restrict__ P = a.plan;
    const uhsdr_agc_plan A = P->agc;
    const int skw = BackSched::word<DM>(a);
    AgcStage<L, W> s;
    s.load(a, l, A);
    BndRegs<4 * NDC> br;
    br.template load<DM>(a, l, 0);
    BackSched sch = BackSched::make<DM, PERS>(a, l, skw);
    int glim = l.calls;
    const bool prep = back_agc_prep_in_pre(DM, A);
    const bool pers = PERS && DM == DM_NONE && a.pctl != nullptr;
    const int g0 = sch.gofs - 1;                      // BackSched: this role's first sub-call (if >= 0)
    if (sch.may_ext) s.lim = l.calls + BACK_SKEW - 1 + (pers ? 1 : 0);
    if (!prep) s.fetch(a, l, g0 > 0 ? g0 : 0);
    if (sch.pin)
    {
        // the pre role's output for g0, left by the previous launch
        const int o = (g0 & 1) * NDC * BACK_CH;
        br.template put<0, NDC>(l, lds.pre + o);
        br.template put<NDC, NDC>(l, lds.prep + o);
        br.template put<2 * NDC, NDC>(l, lds.prep + 2 * NDC * BACK_CH + o);
        br.template put<3 * NDC, NDC>(l, lds.prep + 4 * NDC * BACK_CH + o);
    }
    for (;;)
    {
    BACK_ROLE_LOOP(DM ? 2 : 1)
        const float* pi = lds.pre + (call & 1) * NDC * BACK_CH + l.lane;
        float* ao = lds.agc + (call & 1) * NDC * BACK_CH + l.lane;
        float x[NDC];
#pragma unroll
        for (int m = 0; m < NDC; ++m) x[m] = pi[m * BACK_CH];
        if (prep)
        {
            // the recursion on the pre role's values; volts on to the audio role
            const float* pr = lds.prep + (call & 1) * NDC * BACK_CH + l.lane;
            const float* pf = pr + 2 * NDC * BACK_CH;
            const float* ph = pf + 2 * NDC * BACK_CH;
            float r[NDC], fb[NDC], hb[NDC];
#pragma unroll
            for (int m = 0; m < NDC; ++m) { r[m] = pr[m * BACK_CH]; fb[m] = pf[m * BACK_CH]; hb[m] = ph[m * BACK_CH]; }
            float* vo = lds.dem + (call & 1) * NDC * BACK_CH + l.lane;
#pragma unroll
            for (int m = 0; m < NDC; ++m)
            {
                s.recur(r[m], fb[m], hb[m], A);
                ao[m * BACK_CH] = x[m];
                vo[m * BACK_CH] = s.volts;
            }
        }
        else
        {
        s.begin(a, l, call);
        if ((back_agc_split(DM) && !A.remove_dc) || DM)
        {
            // volts to the audio role, which applies the gain (and with DM the DC removal after
            // it): through the demod role's hand-off buffer (unused without DM), or with DM the
            // second slab of `prep` (the first carries the demod role's corr0)
            float* vo = (DM ? lds.prep + 2 * NDC * BACK_CH : lds.dem) + (call & 1) * NDC * BACK_CH + l.lane;
#pragma unroll
            for (int m = 0; m < NDC; ++m)
            {
                float xv[1] = { x[m] }, v = 0.0f;
                s.template stepn_t<false>(m, xv, l, A, v);
                ao[m * BACK_CH] = xv[0];
                vo[m * BACK_CH] = v;
            }
        }
        else
        {
#pragma unroll
            for (int m = 0; m < NDC; ++m) ao[m * BACK_CH] = s.step(m, x[m], l, A);
        }
        s.end(l);
        }
    BACK_ROLE_END
        if (!pers || !back_ext(sch, lds)) break;
        a.ring_phase = (a.ring_phase + l.calls) % AGC_Q;   // the persistent back end's next call
        sch = BackSched::next(l);
        glim = l.calls;
    }
    s.store(a, l, { !prep, true }, !DM);
    if (back_ext(sch, lds))
    {
        const int o = ((l.calls + BACK_SKEW - 1) & 1) * NDC * BACK_CH;
        bnd_store<NDC>(a, l, 0, lds.pre + o);
        bnd_store<NDC>(a, l, NDC, lds.prep + o);
        bnd_store<NDC>(a, l, 2 * NDC, lds.prep + 2 * NDC * BACK_CH + o);
        bnd_store<NDC>(a, l, 3 * NDC, lds.prep + 4 * NDC * BACK_CH + o);
    }
}

template <int L, int PH, int W, int DM, bool PERS>
__device__ __forceinline__ void rx_back_audio(const BackArgs& a, BackLds lds)
{
    const BackLane l(a);
    constexpr int NDC = BLK / L;
    const int skw = BackSched::word<DM>(a);
    AudioStage<L, PH, DM> s;
    s.load(a, l);
    const uhsdr_agc_plan A = a.plan->agc;
    const bool agc_on = A.mode != 5;
    // DM: the AGC's DC removal (audio_agc.c:575-593) runs here after the gain, with its state
    float wold = DM ? a.s.agc[5 * l.C + l.cl] : 0.0f;
    const bool dc = DM && agc_on && A.remove_dc;
    BndRegs<2 * NDC> br;
    br.template load<DM>(a, l, 4 * NDC);
    BackSched sch = BackSched::make<DM, PERS>(a, l, skw);
    int glim = l.calls;
    const bool pers = PERS && DM == DM_NONE && a.pctl != nullptr;
    if (sch.pin)
    {
        // the AGC role's output (delayed samples, volts) for this role's first sub-call
        const int o = ((sch.gofs - 2) & 1) * NDC * BACK_CH;
        br.template put<0, NDC>(l, lds.agc + o);
        br.template put<NDC, NDC>(l, lds.dem + o);
    }
    for (;;)
    {
    BACK_ROLE_LOOP(DM ? 3 : 2)
        const float* ai = lds.agc + (call & 1) * NDC * BACK_CH + l.lane;
        float* mo = lds.mid + (call & 1) * BLK * BACK_CH + l.lane;
        float x[NDC];
#pragma unroll
        for (int m = 0; m < NDC; ++m) x[m] = ai[m * BACK_CH];
        if (agc_on && (DM || (back_agc_split(DM) && !A.remove_dc)))
        {
            // the AGC role's gain step (AgcStage::gain) on its delayed samples
            const float* vi = (DM ? lds.prep + 2 * NDC * BACK_CH : lds.dem) + (call & 1) * NDC * BACK_CH + l.lane;
            float v[NDC];
#pragma unroll
            for (int m = 0; m < NDC; ++m) v[m] = vi[m * BACK_CH];
#pragma unroll
            for (int m = 0; m < NDC; ++m) x[m] = x[m] * AgcStage<L, W, 1>::gain(v[m], A);
            if (dc)
            {
#pragma unroll
                for (int m = 0; m < NDC; ++m)
                {
                    const float w = (float)((double)x[m] + (double)wold * 0.9999);
                    x[m] = w - wold;
                    wold = w;
                }
            }
        }
#pragma unroll
        for (int m = 0; m < NDC; ++m)
        {
            float u[L];
            s.step(x[m], u);
#pragma unroll
            for (int j = 0; j < L; ++j) mo[(m * L + j) * BACK_CH] = u[j];
        }
        s.end(a, l, call);
    BACK_ROLE_END
        if (!pers || !back_ext(sch, lds)) break;
        sch = BackSched::next(l);                      // the persistent back end's next call
        glim = l.calls;
    }
    s.store(a, l);
    if (DM && l.live) a.s.agc[5 * l.C + l.c] = wold;
    if (back_ext(sch, lds))
    {
        const int o = ((l.calls + BACK_SKEW - 2) & 1) * NDC * BACK_CH;
        bnd_store<NDC>(a, l, 4 * NDC, lds.agc + o);
        bnd_store<NDC>(a, l, 5 * NDC, lds.dem + o);
    }
}

// anti-alias lattice at 48 ksps
template <int AA, int DM, bool PERS>
__device__ __forceinline__ void rx_back_aa(const BackArgs& a, BackLds lds)
{
    const BackLane l(a);
    const uhsdr_rx_plan* __restrict__ P = a.plan;
    // (Measured and dropped: the scalar lattice with VGPR coefficients, full-rate VOP2 instead of
    // packed f32 with SGPR pairs, here and in the pre role: C2 0.0327 -> 0.0366 ms per step.)
    const int skw = BackSched::word<DM>(a);
    LatticeStage<AA> s;
    s.load(l, P->aa_k, P->aa_v, a.s.aa);
    BndRegs<BLK> br;
    br.template load<DM>(a, l, a.bnd_mid);
    BackSched sch = BackSched::make<DM, PERS>(a, l, skw);
    int glim = l.calls;
    const bool pers = PERS && DM == DM_NONE && a.pctl != nullptr;
    if (sch.pin) br.template put<0, BLK>(l, lds.mid + ((sch.gofs - 3) & 1) * BLK * BACK_CH);
    for (;;)
    {
    BACK_ROLE_LOOP(DM ? 4 : 3)
        const float* mi = lds.mid + (call & 1) * BLK * BACK_CH + l.lane;
        float* mo = lds.aa + (call & 1) * BLK * BACK_CH + l.lane;
        // the call's inputs in one batch of LDS reads, then the recursion: a single wave issues
        // one VALU instruction per ~4 cycles, so a read waited on per sample would add its whole
        // latency to every sample of the step
        float x[BLK];
#pragma unroll
        for (int n = 0; n < BLK; ++n) x[n] = mi[n * BACK_CH];
        // samples in pairs: the two ladder sums on packed f32 (4440 -> ~3900 cycles per step, the
        // pipeline's critical role; UHSDR_TRACE r06)
#pragma unroll
        for (int n = 0; n < BLK; n += 2)
        {
            float y0, y1;
            s.step2(x[n], x[n + 1], y0, y1);
            mo[n * BACK_CH] = y0;
            mo[(n + 1) * BACK_CH] = y1;
        }
    BACK_ROLE_END
        if (!pers || !back_ext(sch, lds)) break;
        sch = BackSched::next(l);                      // the persistent back end's next call
        glim = l.calls;
    }
    s.store(l, a.s.aa);
    if (back_ext(sch, lds)) bnd_store<BLK>(a, l, a.bnd_mid, lds.mid + ((l.calls + BACK_SKEW - 3) & 1) * BLK * BACK_CH);
}

// (2 tail waves took 4500-5500 cycles per step with mcHF codec frames, above the anti-alias role)
#ifndef UHSDR_BACK_TAILS
#define UHSDR_BACK_TAILS 4
#endif
constexpr int BACK_TAILS = UHSDR_BACK_TAILS;
// tail waves of a back end: BACK_TAILS for the demodulator-free pipeline; UHSDR_DM_TAILS for the AM /
// SAM ones, 0 (the output role stores its call itself): their grids are large (C3: 512 workgroups)
// and 4 more waves per workgroup took C3's SAM back end from 0.118 to 0.193 ms
// (profiles/r06_configs_tails.jsonl)
#ifndef UHSDR_DM_TAILS
#define UHSDR_DM_TAILS 0
#endif
__host__ __device__ constexpr int back_tails(int dm) { return dm == DM_NONE ? BACK_TAILS : UHSDR_DM_TAILS; }
template <int DM, bool PERS>
__device__ __forceinline__ void rx_back_output(const BackArgs& a, BackLds lds)
{
    const BackLane l(a);
    const int skw = BackSched::word<DM>(a);
    OutputStage s;
    s.load(a, l);
    BndRegs<BLK> br;
    br.template load<DM>(a, l, a.bnd_mid + BLK);
    BackSched sch = BackSched::make<DM, PERS>(a, l, skw);
    int glim = l.calls;
    const bool pers = PERS && DM == DM_NONE && a.pctl != nullptr;
    if (sch.pin) br.template put<0, BLK>(l, lds.aa + ((sch.gofs - 4) & 1) * BLK * BACK_CH);
    bool pread = !sch.pin;                             // the poison word is written (see below)
    for (;;)
    {
    BACK_ROLE_LOOP(DM ? 5 : 4)
        const float* mi = lds.aa + (call & 1) * BLK * BACK_CH + l.lane;
        float y[BLK];
#pragma unroll
        for (int n = 0; n < BLK; ++n) y[n] = mi[n * BACK_CH];      // one batch of LDS reads
#pragma unroll
        for (int n = 0; n < BLK; ++n) y[n] = s.step(y[n]);
        if constexpr (DM == DM_NONE)
        {
            // the pre role's device hand-off gave up (its step-0 word): NaN audio for every frame.
            // Only a launch that starts unskewed waits (BackSched); a skewed one has this role at
            // work in step 0, before the word is written, so it must not read it.  The persistent
            // back end waits at every call: its pre role sets the word at a give-up, read every
            // sub-call after the launch's first call
            if (pread && a.dwait && __builtin_amdgcn_readfirstlane(*lds.poison))
            {
#pragma unroll
                for (int n = 0; n < BLK; ++n) y[n] = __builtin_nanf("");
            }
        }
        // to the tail waves (rx_back_tail), one row per channel: the board's output stage and the
        // stores are elementwise, and as this role's own per-sample tail they made it the
        // pipeline's critical role (int32 codec frames 4400-5700, mcHF 8800-9800 cycles per step
        // against the anti-alias role's 4300; UHSDR_TRACE r06)
        float* yl = lds.ys + (call & 1) * BACK_CH * FUSED_YPITCH + l.lane * FUSED_YPITCH;
#pragma unroll
        for (int n = 0; n < BLK; ++n) yl[n] = y[n];
        if constexpr (back_tails(DM) == 0) fused_store_call(a, l, call, lds.ys + (call & 1) * BACK_CH * FUSED_YPITCH);
    BACK_ROLE_END
        if (!pers || !back_ext(sch, lds)) break;
        sch = BackSched::next(l);                      // the persistent back end's next call
        glim = l.calls;
        pread = true;
    }
    s.store(a, l);
    if (back_ext(sch, lds)) bnd_store<BLK>(a, l, a.bnd_mid + BLK, lds.aa + ((l.calls + BACK_SKEW - 4) & 1) * BLK * BACK_CH);
}
#undef BACK_ROLE_LOOP

// Tail waves of the wave pipeline: the output role's call of the previous step (its transposed
// rows in ys) through the board's output stage (line_out4: key beep, mcHF gains, codec frames) to
// coalesced row stores, each tail wave 64 / BACK_TAILS of the 64 channels' rows; the launch's last call after the
// final barrier.  Elementwise, so it needs no state and no place in BackSched's skew.
template <int DM, bool PERS>
__device__ __forceinline__ void rx_back_tail(const BackArgs& a0, BackLds lds, int half)
{
    BackArgs a = a0;                                   // the call's outputs (PersistCtl: from lds.desc)
    const BackLane l(a);
    BackSched sch = BackSched::make<DM, PERS>(a, l, BackSched::word<DM>(a));
    const bool pers = PERS && DM == DM_NONE && a.pctl != nullptr;
    constexpr int ST = back_roles(DM);                  // one step behind the output role
    const int g8 = l.lane >> 3, j = l.lane & 7;
    const int c0 = l.c - l.lane;
    auto store_call = [&](int call) {
        const float* ys = lds.ys + (call & 1) * BACK_CH * FUSED_YPITCH;
        constexpr int KT = 8 / (back_tails(DM) ? back_tails(DM) : 1);   // row groups of 8 channels per tail wave
#pragma unroll
        for (int kk = 0; kk < KT; ++kk)
        {
            const int k = half * KT + kk;
            const int cc = 8 * k + g8;
            const float* r = ys + cc * FUSED_YPITCH + 4 * j;
            const float v[4] = { r[0], r[1], r[2], r[3] };
            if (c0 + cc >= a.C) continue;
            const size_t rb = (size_t)(c0 + 8 * k) * a.N + call * BLK;
            const unsigned off = (unsigned)g8 * (unsigned)a.N + 4 * j;
            line_out4(a, rb, off, call, call * BLK + 4 * j, v);
        }
    };
    // the persistent back end's control wave (the last tail): the host-memory reads of the call after
    // next (grant word, then its descriptor once the grant has been seen: the host writes it first)
    // and the PC_CONSUMED store, so no role wave waits on a PCIe round trip; the results go to
    // lds.ctl at the call's last step (read by the pre role during the next call)
    const bool ctlw = pers && half == BACK_TAILS - 1;
    unsigned cg = 0, cd = 0;
    for (unsigned seq = a.seq0;; ++seq)
    {
        for (int it = 0; it < sch.steps; ++it)
        {
            const int call = it - ST + sch.gofs;
            TRACE_MARK(0);
            if (call >= 0 && call < l.calls) store_call(call);
            if (ctlw)
            {
                const BackDesc* d2 = a.pdesc + (seq + 2) % DESC_RING;
                if (it == 0) cg = sys_load(a.pctl + PC_GRANT);
                if (it == 3)
                {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");          // the grant first
                    cd = sys_load((const unsigned*)d2 + (l.lane & 15));
                }
                // the pre role's last read of this call's buffer was in the step before
                if (it == l.calls - sch.gofs && l.lane == 0)
                    __hip_atomic_store(a.pctl + PC_CONSUMED + blockIdx.x, seq + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                if (it == sch.steps - 1)
                {
                    unsigned* c = lds.ctl + ((seq + 2) & 1) * 32;
                    if (l.lane < 16) c[l.lane] = cd;
                    if (l.lane == 0) c[16] = __builtin_amdgcn_readfirstlane(cg);
                }
            }
            TRACE_MARK(1);
            lds_barrier();
            TRACE_MARK(2);
        }
        store_call(l.calls - 1);
        if (!pers || !back_ext(sch, lds)) break;
        desc_get(a, lds.desc + ((seq + 1) & 1) * 16);  // the persistent back end's next call
        sch = BackSched::next(l);
    }
}
#undef BACK_ROLE_END

// PRE / AA lattice stages, L interpolation factor, PH polyphase length, W AGC window,
// DM demodulator (DM_NONE: SSB/CW/DIGI)
template <int PRE, int AA, int L, int PH, int W, int DM, bool PERS = false>
__global__ void __launch_bounds__((back_roles(DM) + back_tails(DM)) * BACK_CH) rx_back(BackArgs a)
{
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const BackLds lds = back_lds_carve<BLK / L>(smem);
    // raised issue priority: with the pipelined mode's rx_front of the next call sharing these
    // CUs, the pipeline's per-call critical path keeps the SIMDs' issue slots first (C2 pipelined
    // 25.5 -> 26.5-27.1 Gsamples/s; no effect when the kernels run back to back)
    __builtin_amdgcn_s_setprio(3);
    // readfirstlane makes the role provably wave-uniform (scalar branches)
    const int role = __builtin_amdgcn_readfirstlane(threadIdx.x / BACK_CH) - (DM ? 1 : 0);
#ifndef UHSDR_ROLE_PRIO
#define UHSDR_ROLE_PRIO 1
#endif
    // AM / SAM: the demod role (the per-sample PLL recursion) is the pipeline's longest; the other
    // roles, sharing its SIMD, issue after it (still above a concurrent rx_front)
    if (UHSDR_ROLE_PRIO && DM && role >= 0) __builtin_amdgcn_s_setprio(2);
#ifdef UHSDR_TRACE
    // (tools/trace_back.py) the wave's entry and exit in slot 39
    if ((threadIdx.x & (BACK_CH - 1)) == 0 && blockIdx.x < 64)
    {
        g_trace[blockIdx.x][threadIdx.x / BACK_CH][39][0] = __builtin_readcyclecounter();
        g_trace[blockIdx.x][threadIdx.x / BACK_CH][38][0] = __builtin_amdgcn_s_memrealtime();   // 100 MHz
    }
#endif
    if (role < 0)
        rx_back_demod<L, DM>(a, lds);
    else if (role == 0)
        rx_back_pre<PRE, L, W, DM, PERS>(a, lds);
    else if (role == 1)
        rx_back_agc<L, W, DM, PERS>(a, lds);
    else if (role == 2)
        rx_back_audio<L, PH, W, DM, PERS>(a, lds);
    else if (role == 3)
        rx_back_aa<AA, DM, PERS>(a, lds);
    else if (role == 4)
        rx_back_output<DM, PERS>(a, lds);
    else if constexpr (back_tails(DM) > 0)
    {
        // below every role: a tail wave shares a SIMD with a role wave (9-10 waves on 4 SIMDs), and
        // the roles are the per-step critical path
        __builtin_amdgcn_s_setprio(1);
        rx_back_tail<DM, PERS>(a, lds, role - back_roles(DM) + (DM ? 1 : 0));
    }
#ifdef UHSDR_TRACE
    if ((threadIdx.x & (BACK_CH - 1)) == 0 && blockIdx.x < 64)
    {
        g_trace[blockIdx.x][threadIdx.x / BACK_CH][39][1] = __builtin_readcyclecounter();
        g_trace[blockIdx.x][threadIdx.x / BACK_CH][38][1] = __builtin_amdgcn_s_memrealtime();
    }
#endif
}

// Fused back end for large batches: one wave per 64 channels runs every stage per sample with
// all state in registers -- no LDS, no barriers, no pipeline fill / drain.  With enough
// channels to keep every SIMD busy this beats the wave pipeline, whose only purpose is to
// shorten the per-call critical path when channels are few.
// AGC_ON (mode != 5) and CW (decoder front end) are launch constants, made compile-time so the
// per-sample code carries no uniform branches; the AGC's DC removal is on for AM / SAM (compile-
// time for the demodulating bodies, a select behind rx_notch)
// LDS_IN (rx_chain): channel group grp, input from the wave's LDS hand-off adl
// B1S: biquad_1's taps stay in SGPRs (it runs once per decimated sample; 20 VGPRs freed)
template <int PRE, int AA, int L, int PH, int W, int DM, bool AGC_ON, bool CW, bool LDS_IN = false, bool DC = true,
          bool B1S = false>
__device__ __forceinline__ void back_fused_body(const BackArgs& a, float* ys, int grp, const float* adl = nullptr)
{
    const BackLane l(a, grp);
    constexpr int NDC = BLK / L;
    static_assert(L == 2 || L == 4, "4 output frames per 1 or 2 decimated samples");
    static_assert(!LDS_IN || DM == DM_NONE, "rx_chain: SSB / CW / DIGI back ends only");
    const uhsdr_rx_plan* __restrict__ P = a.plan;
    const uhsdr_agc_plan A = P->agc;
    DemodStage<L, DM> dm;
    InStage<L, LDS_IN> in;
    in.lds = adl;
    LatticeStage<PRE, UHSDR_FUSED_PK> pre;
    AgcStage<L, W> ag;
    AudioStage<L, PH, DM> au;
    LatticeStage<AA, UHSDR_FUSED_PK> aa;
    OutputStage ou;
    if (DM) { dm.load(a, l); dm.fetch(a, l, 0); }
    else in.fetch(a, l, 0);
    pre.load(l, P->pre_k, P->pre_v, a.s.pre);
    ag.load(a, l, A);
    ag.fetch(a, l, 0);
    au.load(a, l);
    aa.load(l, P->aa_k, P->aa_v, a.s.aa);
    ou.load(a, l);
    // coefficients of the per-sample recursions into VGPRs (full-rate VOP2, no SGPR spills:
    // v_readlane refills 699 -> 104 per kernel, 0.220 -> 0.211 ms at 1M x 64)
#ifndef UHSDR_FUSED_SGPR_COEF
    if (PRE > 0) { to_vgpr(pre.k); to_vgpr(pre.v); }
    if (AA > 0) { to_vgpr(aa.k); to_vgpr(aa.v); }
    to_vgpr(ou.b2);
    ou.lo = to_vgpr(ou.lo);
    if (!B1S) to_vgpr(au.b1);
#endif
    ag.agc_on = AGC_ON;
    if (DM != DM_NONE) ag.dc = true;
    else if (DC) ag.dc_sel = true;
    else { ag.dc = false; ag.dc_sel = false; }        // SSB / CW / DIGI: no DC removal to select
    au.cw = CW;
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
        // The call's 32 output frames go to LDS (row per channel, 33-float pitch: conflict-free)
        // and leave in one burst at its end, each store instruction writing 8 whole 128-byte
        // rows: holding them in registers costs 32 VGPRs of occupancy, and storing them as they
        // come leaves partial lines that L2 evicts before they fill (twice the HBM write bytes).
        float* yl = ys + l.lane * FUSED_YPITCH;
#pragma unroll
        for (int m = 0; m < NDC; ++m)
        {
            float u[L];
            au.step(ag.step(m, pre.step(xin[m], m), l, A), u);
#pragma unroll
            for (int j = 0; j < L; ++j) yl[m * L + j] = ou.step(aa.step(u[j], j));
        }
        fused_store_call(a, l, call, ys);
        ag.end(l);
        au.end(a, l, call);
    }
    if (DM) dm.store(a, l);
    pre.store(l, a.s.pre);
    ag.store(a, l);
    au.store(a, l);
    aa.store(l, a.s.aa);
    ou.store(a, l);
}

// runs the body with the launch's AGC / CW flags as template arguments
// DC: the AGC removes DC (AM / SAM; for the demodulator-free bodies only after an AM / SAM
// demodulator that ran in rx_notch) -- a separate kernel instance for the SSB / CW / DIGI back end
// without it (the select form cost its f64 arithmetic on every sample)
template <int PRE, int AA, int L, int PH, int W, int DM, bool CW, bool LDS_IN = false, bool DC = true>
__device__ __forceinline__ void back_fused_agc(const BackArgs& a, float* ys, int grp, const float* adl = nullptr)
{
    if (a.plan->agc.mode == 5) back_fused_body<PRE, AA, L, PH, W, DM, false, CW, LDS_IN, DC>(a, ys, grp, adl);
    else back_fused_body<PRE, AA, L, PH, W, DM, true, CW, LDS_IN, DC>(a, ys, grp, adl);
}

// FORM 0: the launch's AGC / CW flags dispatched inside the kernel (its registers are the
// largest body's: 199 VGPRs at P48, 2 waves per SIMD).  FORM 1: AGC on, CW off only (the SSB /
// DIGI default, the north-star chain), one body with biquad_1's taps in SGPRs: 160 VGPRs at P48,
// no scratch, 3 waves per SIMD.
// (the compiler's resource report: the 24 ksps bodies with a pre-filter lattice need 207-220
// VGPRs at FORM 0 and spill to scratch at 3 waves, so they keep 2)
#ifndef UHSDR_FUSED1_WAVES
#define UHSDR_FUSED1_WAVES 3
#endif
__host__ __device__ constexpr int fused1_waves(int pre, int L) { return (L == 2 && pre > 0) ? 2 : UHSDR_FUSED1_WAVES; }
template <int PRE, int AA, int L, int PH, int W, int DM, bool DC = true, int FORM = 0>
__global__ void __launch_bounds__(BACK_CH)
__attribute__((amdgpu_waves_per_eu(FORM == 1 ? fused1_waves(PRE, L) : DM == DM_SAM_SB ? 1 : UHSDR_FUSED_WAVES))) rx_back_fused(BackArgs a)
{
    __shared__ float ys[BACK_CH * FUSED_YPITCH];
    if constexpr (FORM == 1)
    {
        back_fused_body<PRE, AA, L, PH, W, DM, true, false, false, DC, true>(a, ys, blockIdx.x);
        return;
    }
    if constexpr (L == 4)
    {
        if (a.plan->cw_enabled) { back_fused_agc<PRE, AA, L, PH, W, DM, true, false, DC>(a, ys, blockIdx.x); return; }
    }
    back_fused_agc<PRE, AA, L, PH, W, DM, false, false, DC>(a, ys, blockIdx.x);
}

// ------------------------------------------------------------------------------------
// rx_chain: the whole call in one kernel for large batches (SSB / CW / DIGI, mono).  One wave
// owns 64 channels: it runs rx_front's pass over them CPW channels at a time (64 / CPW passes,
// the decimated output of each kept in LDS, [sample][channel] with pitch CHAIN_ADP), then
// rx_back_fused's per-sample recursions with lane == channel, reading that LDS instead of adec.
// The decimated hand-off never reaches HBM and there is no kernel boundary; since every wave
// alternates a FIR phase (VALU + HBM stream) and a recursion phase (dependent VALU chains),
// waves in different phases share a SIMD and its HBM stream.  The register budget is the back
// end's (2 waves per SIMD); the front window and the back's output staging share one LDS region.
template <int T1, int T2, int M, bool DF, int R, bool F, int PRE, int AA, int L, int PH, int W>
__global__ void __launch_bounds__(FRONT_WAVE) __attribute__((amdgpu_waves_per_eu(UHSDR_FUSED_WAVES)))
rx_chain(FrontArgs fa, BackArgs ba, int front_floats)
{
    static_assert(M == L, "decimation and interpolation rates agree");
    extern __shared__ __attribute__((aligned(16))) float smem[];
    constexpr int RD = R / M;
    float* adl = smem + front_floats;                  // [N / M][CHAIN_ADP]
    const int nb = fa.N / R, cpw = FRONT_WAVE / nb, passes = BACK_CH / cpw;
    const int grp = blockIdx.x;
    for (int p = 0; p < passes; ++p)
    {
        if ((grp * passes + p) * cpw >= fa.C) break;   // past the last channel (wave-uniform)
        front_body<T1, T2, M, DF, R, F, false>(fa, grp * passes + p, smem,
            [&](bool, int, int g, int b, const float (&o)[RD])
            {
                float* d = adl + p * cpw + g;
#pragma unroll
                for (int r = 0; r < RD; ++r) d[(b * RD + r) * CHAIN_ADP] = o[r];
            });
        wave_sync();                                   // the window region is reused by the next pass
    }
    if constexpr (L == 4)
    {
        if (ba.plan->cw_enabled) { back_fused_agc<PRE, AA, L, PH, W, DM_NONE, true, true, false>(ba, smem, grp, adl); return; }
    }
    back_fused_agc<PRE, AA, L, PH, W, DM_NONE, false, true, false>(ba, smem, grp, adl);
}

// ------------------------------------------------------------------------------------
// rx_back_stereo: the OVI40 two-channel back end (use_stereo, audio_driver.c:2618): channel 0
// (a_buffer[0] at the decimated rate) and channel 1 (a_buffer[1]) each through their own
// instances of the pre-filter, scale + biquad_1, interpolator, anti-alias lattice, biquad_2 and
// line-out scale (audio_driver.c:2475-2479, 2527-2534, 2560-2590, 2832-2837, 2860-2866), with one
// stereo AGC between them (audio_agc.c:366-393, 575-593).  After the interpolation the channels
// swap buffers (:2563-2576): channel 0 ends in a_buffer[1] (audio, codec left), channel 1 in
// a_buffer[0] (audio0, codec right).  The CW decoder front end reads channel 0.  Lane == channel,
// all state in registers (the fused schedule; no small-batch pipeline variant).
// DM: DM_NONE (SSB stereo / IQ: both channels from rx_front in adec / adec_q, or from rx_notch)
// or DM_SAM_ST (the SAM PLL demodulator splitting LSB / USB here).
template <int PRE, int AA, int L, int PH, int W, int DM>
__global__ void __launch_bounds__(BACK_CH) rx_back_stereo(BackArgs a)
{
    const BackLane l(a);
    constexpr int NDC = BLK / L;
    static_assert(L == 2 || L == 4, "4 output frames per 1 or 2 decimated samples");
    const uhsdr_rx_plan* __restrict__ P = a.plan;
    const uhsdr_agc_plan A = P->agc;
    BackArgs b = a;                                      // channel 1: instances [1], input a_buffer[1]
    b.adec = a.adec_q;
    b.s.bq1 = a.s.bq1_1; b.s.bq2 = a.s.bq2_1; b.s.interp = a.s.interp1;
    DemodStage<L, DM> dm;
    InStage<L> in0, in1;
    LatticeStage<PRE> pre0, pre1;
    AgcStage<L, W, 2> ag;
    AudioStage<L, PH, DM> au0, au1;
    LatticeStage<AA> aa0, aa1;
    OutputStage ou0, ou1;
    if (DM) { dm.load(a, l); dm.fetch(a, l, 0); }
    else { in0.fetch(a, l, 0); in1.fetch(b, l, 0); }
    pre0.load(l, P->pre_k, P->pre_v, a.s.pre);
    pre1.load(l, P->pre_k, P->pre_v, a.s.pre1);
    ag.load(a, l, A);
    ag.fetch(a, l, 0);
    au0.load(a, l);
    au1.load(b, l);
    au1.cw = false;                                      // CwDecode_RxProcessor reads a_buffer[0] only
    aa0.load(l, P->aa_k, P->aa_v, a.s.aa);
    aa1.load(l, P->aa_k, P->aa_v, a.s.aa1);
    ou0.load(a, l);
    ou1.load(b, l);
    for (int call = 0; call < l.calls; ++call)
    {
        float x0[NDC], x1[NDC];
        if (DM)
        {
            dm.begin(a, l, call);
#pragma unroll
            for (int m = 0; m < NDC; ++m) { x0[m] = dm.step(m); x1[m] = dm.y1; }
        }
        else
        {
            in0.begin(a, l, call, x0);
            in1.begin(b, l, call, x1);
        }
        ag.begin(a, l, call);
        float y0[BLK], y1[BLK];
#pragma unroll
        for (int m = 0; m < NDC; ++m)
        {
            float v[2] = { pre0.step(x0[m]), pre1.step(x1[m]) };
            ag.stepn(m, v, l, A);
            float u0[L], u1[L];
            au0.step(v[0], u0);
            au1.step(v[1], u1);
#pragma unroll
            for (int j = 0; j < L; ++j)
            {
                y0[m * L + j] = ou0.step(aa0.step(u0[j]));
                y1[m * L + j] = ou1.step(aa1.step(u1[j]));
            }
        }
        if (a.beep_n1 > call * BLK && a.beep_n0 < (call + 1) * BLK)
        {
#pragma unroll
            for (int n = 0; n < BLK; ++n)
            {
                const int fr = call * BLK + n;
                if (fr >= a.beep_n0 && fr < a.beep_n1)
                {
                    const float t = beep_tone(a, fr);
                    y1[n] += t;                          // softdds_addSingleToneToTwobuffers(a_buffer[0], [1])
                    y0[n] += t;
                }
            }
        }
        if (l.live)
        {
            const size_t row = (size_t)l.c * a.N + call * BLK;
#pragma unroll
            for (int n0 = 0; n0 < BLK; n0 += 4)
            {
                if (a.audio) *(float4*)(a.audio + row + n0) = make_float4(y0[n0], y0[n0 + 1], y0[n0 + 2], y0[n0 + 3]);
                if (a.audio0) *(float4*)(a.audio0 + row + n0) = make_float4(y1[n0], y1[n0 + 1], y1[n0 + 2], y1[n0 + 3]);
                if (a.dst)
                {
                    // dst.l = a_buffer[1] (channel 0), dst.r = a_buffer[0] (channel 1), :2911-2923
                    *(int4*)(a.dst + row + n0) = make_int4(to_dma(y0[n0]), to_dma(y1[n0]), to_dma(y0[n0 + 1]), to_dma(y1[n0 + 1]));
                    *(int4*)(a.dst + row + n0 + 2) = make_int4(to_dma(y0[n0 + 2]), to_dma(y1[n0 + 2]), to_dma(y0[n0 + 3]), to_dma(y1[n0 + 3]));
                }
            }
        }
        ag.end(l);
        au0.end(a, l, call);
    }
    if (DM) dm.store(a, l);
    pre0.store(l, a.s.pre);
    pre1.store(l, a.s.pre1);
    ag.store(a, l);
    au0.store(a, l);
    au1.store(b, l);
    aa0.store(l, a.s.aa);
    aa1.store(l, a.s.aa1);
    ou0.store(a, l);
    ou1.store(b, l);
}

// ------------------------------------------------------------------------------------
// rx_notch: the LMS auto notch (AudioDriver_NotchFilter, audio_driver.c:1746-1763, called from
// RxProcessor_DemodAudioPostprocessing :2443-2456 when DSP_NOTCH_ENABLE is set), in place on the
// decimated audio a_buffer[0] between the demodulator and the IIR pre-filter.  Lane == channel:
// arm_lms_norm_f32 (CMSIS .../FilteringFunctions/arm_lms_norm_f32.c) is a per-sample recursion
// over its 64 coefficients, so each lane holds its channel's coefficients and the 63-sample
// state window in registers for the launch.  Per call:
//   arm_copy_f32(a_buffer[0] -> delay[inbuf])            (the de-correlation delay line)
//   arm_lms_norm_f32(src = a_buffer[0], ref = delay[outbuf], out = errsig2, err = a_buffer[0])
//   inbuf += B; outbuf = inbuf + B (mod 128)
// and per sample, in CMSIS order: state[63] = in; energy -= x0*x0; energy += in*in;
// y = sum_k state[k] * w[k] (k = 0..63 from +0.0f); e = ref - y; out = e;
// mu_w = (e * mu) / (energy + 1.19209289e-7); w[k] += mu_w * state[k]; x0 = state[0]; slide.
// AM / SAM (DM != DM_NONE): the demodulator runs here first (DemodStage, its state in
// BackState.sam), the notched audio goes to adec and rx_back runs its DM_NONE variant.
constexpr int NOTCH_TAPS = 64, NOTCH_DELAY = 128;

template <int L, int DM>
__global__ void __launch_bounds__(BACK_CH) rx_notch(BackArgs a)
{
    const BackLane l(a);
    constexpr int NDC = BLK / L;
    constexpr int SLOTS = NOTCH_DELAY / NDC;             // delay line in units of one call
    const uhsdr_rx_plan* __restrict__ P = a.plan;
    const int C = l.C, cl = l.cl;
    DemodStage<L, DM> dm;
    InStage<L> in;
    if (DM) { dm.load(a, l); dm.fetch(a, l, 0); }
    else in.fetch(a, l, 0);
    float* const W = a.s.notch;                          // [64][C] coefficients
    float* const H = W + (size_t)NOTCH_TAPS * C;         // [64][C] state (63 carried samples)
    float* const E = H + (size_t)NOTCH_TAPS * C;         // [2][C]  energy, x0
    float* const R = E + (size_t)2 * C;                  // [128][C] delay line
    float w[NOTCH_TAPS], st[NOTCH_TAPS - 1 + NDC];
#pragma unroll
    for (int k = 0; k < NOTCH_TAPS; ++k) w[k] = W[(size_t)k * C + cl];
#pragma unroll
    for (int k = 0; k < NOTCH_TAPS - 1; ++k) st[k] = H[(size_t)k * C + cl];
    float energy = E[cl], x0 = E[C + cl];
    const float mu = P->notch_mu;
    for (int call = 0; call < l.calls; ++call)
    {
        float x[NDC], x1[NDC];
        if (DM)
        {
            dm.begin(a, l, call);
#pragma unroll
            for (int m = 0; m < NDC; ++m) { x[m] = dm.step(m); x1[m] = dm.y1; }
            if (DM == DM_SAM_ST && l.live)
            {
                // SAM stereo: channel 1 (a_buffer[1]) continues un-notched to rx_back_stereo
                float* d1 = const_cast<float*>(a.adec_q) + (size_t)l.c * a.Nd + call * NDC;
#pragma unroll
                for (int m = 0; m < NDC; m += 4) *(float4*)(d1 + m) = make_float4(x1[m], x1[m + 1], x1[m + 2], x1[m + 3]);
            }
        }
        else
            in.begin(a, l, call, x);
        const int si = (a.notch_slot0 + call) % SLOTS, so = (a.notch_slot0 + call + 1) % SLOTS;
        const bool first = a.notch_first && call == 0;   // lms2_outbuf == lms2_inbuf == 0
        float d[NDC];
#pragma unroll
        for (int m = 0; m < NDC; ++m) d[m] = first ? x[m] : R[(size_t)(so * NDC + m) * C + cl];
        if (l.live)
        {
#pragma unroll
            for (int m = 0; m < NDC; ++m) R[(size_t)(si * NDC + m) * C + l.c] = x[m];
        }
        float o[NDC];
#pragma unroll
        for (int m = 0; m < NDC; ++m)
        {
            const float xin = x[m];
            st[NOTCH_TAPS - 1 + m] = xin;
            energy -= x0 * x0;
            energy += xin * xin;
            float sum = 0.0f;
#pragma unroll
            for (int k = 0; k < NOTCH_TAPS; ++k) sum += st[m + k] * w[k];
            const float e = d[m] - sum;
            o[m] = e;
            const float wf = (e * mu) / (energy + 0.000000119209289f);
#pragma unroll
            for (int k = 0; k < NOTCH_TAPS; ++k) w[k] += wf * st[m + k];
            x0 = st[m];
        }
#pragma unroll
        for (int k = 0; k < NOTCH_TAPS - 1; ++k) st[k] = st[k + NDC];
        if (l.live)
        {
            float* dst = const_cast<float*>(a.adec) + (size_t)l.c * a.Nd + call * NDC;
#pragma unroll
            for (int m = 0; m < NDC; m += 4) *(float4*)(dst + m) = make_float4(o[m], o[m + 1], o[m + 2], o[m + 3]);
        }
    }
    if (!l.live) return;
    if (DM) dm.store(a, l);
#pragma unroll
    for (int k = 0; k < NOTCH_TAPS; ++k) W[(size_t)k * C + l.c] = w[k];
#pragma unroll
    for (int k = 0; k < NOTCH_TAPS - 1; ++k) H[(size_t)k * C + l.c] = st[k];
    E[l.c] = energy;
    E[C + l.c] = x0;
}

// ------------------------------------------------------------------------------------
// rx_fm: FM receive after the Hilbert pair (AudioDriver_DemodFM, audio_driver.c:1544-1737,
// and the FM branch of AudioDriver_RxProcessor, :2818-2850).  Two waves over 64 channels:
//   wave 0  discriminator atan2f -> de-emphasis LPF -> HPF (or 0 when squelched) per sample;
//           squelch noise lattice (IIR_15k_hpf) over the call, averaged energy of its first
//           output, squelch decision every FM_SQUELCH_PROC_DECIMATION = 200 calls
//   wave 1  x FM_RX_SCALING, biquad_2 (:2832), mute when squelched / line-out x10 (:2843-2860),
//           f32 audio and int32 codec frames
// The AGC the reference runs on a_buffer[0] in FM (:2827) is not run: the output stage
// overwrites that buffer with the line-out copy (:2868), so it never reaches the audio.
// Subaudible tone detection (:1665-1734, ts.fm_subaudible_tone_det_select): three Goertzels on the
// de-emphasised audio, a decision every FM_SUBAUDIBLE_GOERTZEL_WINDOW = 400 calls; with it on, the
// audio passes only while a tone is detected.  FM state: [field][C] in BackState.sam:
//   0 i_prev 1 q_prev 2 lpf_prev 3 hpf_prev_a 4 hpf_prev_b 5 sql_avg 6 open (!squelched) 7..12 lattice
//   13..18 Goertzel buf[1], buf[2] of FM_HIGH, FM_LOW, FM_CTR  19 subdet  20 tdet  21 tone detected
template <int SQ>
__global__ void __launch_bounds__(2 * BACK_CH) rx_fm(BackArgs a)
{
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const uhsdr_rx_plan* __restrict__ P = a.plan;
    const int lane = threadIdx.x & (BACK_CH - 1);
    const int role = __builtin_amdgcn_readfirstlane(threadIdx.x / BACK_CH);
    const int c = blockIdx.x * BACK_CH + lane;
    const bool live = c < a.C;
    const int cl = live ? c : a.C - 1;
    const int C = a.C;
    const int calls = a.N / BLK;
    float* dem = smem;                                   // [2][BLK][64] demodulated audio
    float* act = smem + 2 * BLK * BACK_CH;               // [2][64] signal_active of the call
    float* S = a.s.sam;
    if (role == 0)
    {
        float sk[SQ], sv[SQ + 1], g[SQ];
#pragma unroll
        for (int i = 0; i < SQ; ++i) sk[i] = P->sq_k[i];
#pragma unroll
        for (int i = 0; i <= SQ; ++i) sv[i] = P->sq_v[i];
#pragma unroll
        for (int i = 0; i < SQ; ++i) g[i] = S[(7 + i) * C + cl];
        float lpf_prev = S[2 * C + cl];                   // fields 0, 1 (i_prev, q_prev): rx_front's
        float hpf_a = S[3 * C + cl], hpf_b = S[4 * C + cl], sql_avg = S[5 * C + cl];
        bool squelched = S[6 * C + cl] == 0.0f;          // field 6 = "open": zeroed state starts squelched (:475)
        const int thr = P->fm_sql_threshold;
        const bool tone_en = P->tone_det_enabled;
        float tg[6];                                     // {buf[1], buf[2]} of FM_HIGH, FM_LOW, FM_CTR
#pragma unroll
        for (int i = 0; i < 6; ++i) tg[i] = tone_en ? S[(13 + i) * C + cl] : 0.0f;
        float subdet = tone_en ? S[19 * C + cl] : 0.0f;
        int tdet = tone_en ? (int)S[20 * C + cl] : 0;
        bool detected = tone_en && S[21 * C + cl] != 0.0f;
        const bool translate = P->freq_shift_hz != 0;   // no translation: the demod bails out (:1548)
        // the discriminator's angle per sample, computed by rx_front (audio_driver.c:1588-1592)
        float inext[BLK];
        auto fetch = [&](int call) {
            const float* si = a.adec + (size_t)cl * a.Nd + call * BLK;
#pragma unroll
            for (int m = 0; m < BLK; m += 4)
            {
                const float4 v = *(const float4*)(si + m);
                inext[m] = v.x; inext[m + 1] = v.y; inext[m + 2] = v.z; inext[m + 3] = v.w;
            }
        };
        fetch(0);
        for (int it = 0; it <= calls; ++it)
        {
            if (it < calls)
            {
                float xa[BLK];
#pragma unroll
                for (int m = 0; m < BLK; ++m) xa[m] = inext[m];
                if (it + 1 < calls) fetch(it + 1);
                float* out = dem + (it & 1) * BLK * BACK_CH + lane;
                if (translate)
                {
                    // audio gate (:1571-1586)
                    const bool pass = (!squelched && !tone_en) || (detected && tone_en) || !thr;
                    float sq0 = 0.0f;
#pragma unroll 4
                    for (int m = 0; m < BLK; ++m)
                    {
                        const float angle = xa[m];
                        const float aa = (float)((double)lpf_prev + (0.05 * (double)(angle - lpf_prev)));
                        lpf_prev = aa;
                        if (tone_en)
                        {
                            // AudioFilter_GoertzelInput (audio_filter.c:1290-1295) x 3 (:1683-1691)
#pragma unroll
                            for (int gi = 0; gi < 3; ++gi)
                            {
                                const float g0 = P->tone_r[gi] * tg[2 * gi] - tg[2 * gi + 1] + aa;
                                tg[2 * gi + 1] = tg[2 * gi];
                                tg[2 * gi] = g0;
                            }
                        }
                        float o = 0.0f;
                        if (pass)
                        {
                            const float bb = (float)(0.96 * (double)(hpf_b + aa - hpf_a));
                            hpf_a = aa;
                            hpf_b = bb;
                            o = bb;
                        }
                        out[m * BACK_CH] = o;
                        // squelch HPF (:1594); the packed lattice, pairing by the sample's parity
                        const float sqo = (m & 1) ? lattice_step_pk<SQ, 1>(angle, g, sk, sv)
                                                  : lattice_step_pk<SQ, 0>(angle, g, sk, sv);
                        if (m == 0) sq0 = sqo;
                    }
                    sql_avg = (float)(((1 - 0.005) * (double)sql_avg) + (0.005 * (double)sqrtf(fabsf(sq0))));
                    if ((a.ring_phase + it + 1) % 200 == 0)     // fm_data.count (:1604-1605)
                    {
                        if ((double)sql_avg > 0.175) sql_avg = 0.175f;
                        float scaled = sql_avg * 172;
                        if (scaled > 24) scaled = 24;
                        scaled = 22 - scaled;
                        if (thr == 0) squelched = false;
                        else if (squelched) { if (scaled >= (float)(thr + 3)) squelched = false; }
                        else if (thr > 3) { if (scaled < (float)(thr - 3)) squelched = true; }
                        else if (scaled < (float)thr) squelched = true;
                    }
                    if (tone_en && (a.tone_phase + it + 1) % 400 == 0)   // fm_data.gcount (:1679, 1693)
                    {
                        // AudioFilter_GoertzelEnergy (audio_filter.c:1296-1305), :1693-1725
                        float en[3];
#pragma unroll
                        for (int gi = 0; gi < 3; ++gi)
                        {
                            const float ga = (tg[2 * gi] - (tg[2 * gi + 1] * P->tone_cos[gi]));
                            const float gb = (tg[2 * gi + 1] * P->tone_sin[gi]);
                            en[gi] = sqrtf(ga * ga + gb * gb);
                            tg[2 * gi] = 0.0f;
                            tg[2 * gi + 1] = 0.0f;
                        }
                        const float s_off = en[0] + en[1];
                        const float r_on = en[2];
                        subdet = (float)(((1 - 0.9) * (double)subdet) + ((double)(r_on / (s_off / 2)) * 0.9));
                        if ((double)subdet > 1.75)
                        {
                            ++tdet;
                            if (tdet > 5) tdet = 5;
                        }
                        else if (tdet)
                            --tdet;
                        detected = tdet >= 2;
                    }
                }
                else
                {
                    // a_buffer[0] keeps its previous contents in the reference; not offered
#pragma unroll
                    for (int m = 0; m < BLK; ++m) out[m * BACK_CH] = 0.0f;
                }
                act[(it & 1) * BACK_CH + lane] = squelched ? 0.0f : 1.0f;
            }
            lds_barrier();
        }
        if (live)
        {
            S[2 * C + c] = lpf_prev;
            S[3 * C + c] = hpf_a; S[4 * C + c] = hpf_b; S[5 * C + c] = sql_avg;
            S[6 * C + c] = squelched ? 0.0f : 1.0f;
#pragma unroll
            for (int i = 0; i < SQ; ++i) S[(7 + i) * C + c] = g[i];
            if (tone_en)
            {
#pragma unroll
                for (int i = 0; i < 6; ++i) S[(13 + i) * C + c] = tg[i];
                S[19 * C + c] = subdet;
                S[20 * C + c] = (float)tdet;
                S[21 * C + c] = detected ? 1.0f : 0.0f;
            }
        }
    }
    else
    {
        float bq2[4], b2[5];
#pragma unroll
        for (int i = 0; i < 5; ++i) b2[i] = P->biquad2[i];
#pragma unroll
        for (int i = 0; i < 4; ++i) bq2[i] = a.s.bq2[i * C + cl];
        const float lo = P->line_out_scale, fs = P->fm_scale;
        for (int it = 0; it <= calls; ++it)
        {
            if (it > 0)
            {
                const int call = it - 1;
                const float* mi = dem + (call & 1) * BLK * BACK_CH + lane;
                const bool on = act[(call & 1) * BACK_CH + lane] != 0.0f;
#pragma unroll 2
                for (int n0 = 0; n0 < BLK; n0 += 4)
                {
                    float v[4];
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        v[j] = biquad_step(mi[(n0 + j) * BACK_CH] * fs, bq2[0], bq2[1], bq2[2], bq2[3], b2) * lo;
                    // muted: both buffers zero, the beep still added (audio_driver.c:2845-2898)
                    if (live) line_out4(a, (size_t)c * a.N + call * BLK + n0, 0u, call, call * BLK + n0, v, on);
                }
            }
            lds_barrier();
        }
        if (live)
        {
#pragma unroll
            for (int i = 0; i < 4; ++i) a.s.bq2[i * C + c] = bq2[i];
        }
    }
}

// ------------------------------------------------------------------------------------
// kernel selection: the filter-path families of FilterPathInfo (audio_filter.c:147-922)

typedef void (*front_fn)(FrontArgs);
typedef void (*back_fn)(BackArgs);

typedef void (*chain_fn)(FrontArgs, BackArgs, int);
struct FrontVariant { int t1, t2, m, decim_first; front_fn fn; int R; front_fn fn_fma; int st; };
// fused_nodc: rx_back_fused without the AGC's DC removal (the demodulator-free back end when the
// AGC does not remove DC: SSB / CW / DIGI); the same kernel as `fused` for the demodulators
// fused_ssb: fused_nodc for a launch with the AGC on and the CW decoder off (FORM 1), or null
// fn_pers: the persistent back end's instance of fn (uhsdr_rx_set_pipelined 3; DM_NONE only)
struct BackVariant { int pre, aa, L, ph, w, dm; back_fn fn; back_fn fused; back_fn fused_nodc; back_fn fused_ssb; back_fn fn_pers; };
template <int PRE, int AA, int L, int PH, int W, int DM>
constexpr back_fn pers_of()
{
    if constexpr (DM == DM_NONE) return rx_back<PRE, AA, L, PH, W, DM, true>;
    else return nullptr;
}
template <int PRE, int AA, int L, int PH, int W, int DM>
constexpr back_fn fused_nodc_of()
{
    if constexpr (DM == DM_NONE) return rx_back_fused<PRE, AA, L, PH, W, DM, false>;
    else return rx_back_fused<PRE, AA, L, PH, W, DM>;
}
template <int PRE, int AA, int L, int PH, int W, int DM>
constexpr back_fn fused_ssb_of()
{
    if constexpr (DM == DM_NONE) return rx_back_fused<PRE, AA, L, PH, W, DM, false, 1>;
    else return nullptr;
}
// rx_chain instances: a front family (t1, t2, m, decim_first, R = 8) with a DM_NONE back end
struct ChainVariant { int t1, t2, m, decim_first, R, pre, aa, L, ph, w; chain_fn fn, fn_fma; };
#define CHAIN_V(t1, t2, m, df, pre, aa, ph, w) { t1, t2, m, df, 8, pre, aa, m, ph, w, \
    rx_chain<t1, t2, m, df, 8, false, pre, aa, m, ph, w>, rx_chain<t1, t2, m, df, 8, true, pre, aa, m, ph, w> }

// R = FIR outputs per lane: 16 for large batches (more MACs per window load), 8 for small
// batches (twice the waves in flight).  fn: reference MAC order (bit-exact); fn_fma: fused MACs
// (UHSDR_PRECISION_FMA)
#define FRONT_V(t1, t2, m, df, R) { t1, t2, m, df, rx_front<t1, t2, m, df, R, false>, R, rx_front<t1, t2, m, df, R, true>, 0 }
#define FRONT_ST(t1, t2, m, df, R) { t1, t2, m, df, rx_front<t1, t2, m, df, R, false, true>, R, rx_front<t1, t2, m, df, R, true, true>, 1 }
struct NotchVariant { int L, dm; back_fn fn; };
#include <uhsdr_rx_variants.inc>
#undef CHAIN_V

static int plan_dm(const uhsdr_rx_plan& p)
{
    if (p.dmod_mode == UHSDR_DEMOD_FM) return DM_FM;
    if (p.dmod_mode == UHSDR_DEMOD_AM) return DM_AM;
    if (p.dmod_mode == UHSDR_DEMOD_SAM)
        return p.sam_sideband == UHSDR_SAM_SIDEBAND_BOTH ? DM_SAM : p.stereo == 3 ? DM_SAM_ST : DM_SAM_SB;
    return DM_NONE;
}

// frames handled by one front launch: one wave covers a channel's launch block
static int front_frames(int N, int R) { return N < FRONT_WAVE * R ? N : FRONT_WAVE * R; }

// N == 0: support query.  want: outputs per lane, 8 by default (more waves per batch, and its
// 8+ lanes per channel prefetch whole history rows) or 16 (uhsdr_rx_set_front_block); strict:
// only that R, else the nearest the call size admits.
static const FrontVariant* find_front(const uhsdr_rx_plan& p, int N = 0, int want = 8, bool strict = false)
{
    const int t1 = p.use_decimated_iq ? p.dec_taps : p.hilbert_taps;
    const int t2 = p.use_decimated_iq ? p.hilbert_taps : p.dec_taps;
    const int st = p.stereo == 1 || p.stereo == 2;       // SAM stereo splits in the demodulator
    const FrontVariant* best = nullptr;
    for (const FrontVariant& v : kFront)
        if (v.t1 == t1 && v.t2 == t2 && v.m == p.decimation_rate && v.decim_first == p.use_decimated_iq && v.st == st)
        {
            if (N && (N % v.R || front_frames(N, v.R) / v.R < 4)) continue;   // >= 4 lanes per channel
            if (strict && v.R != want) continue;
            if (!best || (v.R == want && best->R != want)) best = &v;
        }
    return best;
}

static const ChainVariant* find_chain(const uhsdr_rx_plan& p, const BackVariant* bv)
{
    if (!bv || bv->dm != DM_NONE || p.stereo || p.notch_enabled || p.dmod_mode == UHSDR_DEMOD_FM) return nullptr;
    const int t1 = p.use_decimated_iq ? p.dec_taps : p.hilbert_taps;
    const int t2 = p.use_decimated_iq ? p.hilbert_taps : p.dec_taps;
    for (const ChainVariant& v : kChain)
        if (v.t1 == t1 && v.t2 == t2 && v.m == p.decimation_rate && v.decim_first == p.use_decimated_iq &&
            v.pre == bv->pre && v.aa == bv->aa && v.L == bv->L && v.ph == bv->ph && v.w == bv->w)
            return &v;
    return nullptr;
}

static const NotchVariant* find_notch(const uhsdr_rx_plan& p)
{
    if (!p.notch_enabled) return nullptr;
    for (const NotchVariant& v : kNotch)
        if (v.L == p.decimation_rate && v.dm == plan_dm(p)) return &v;
    return nullptr;
}

// with the notch on, the demodulator runs in rx_notch and rx_back takes its DM_NONE variant
static const BackVariant* find_back(const uhsdr_rx_plan& p)
{
    if (p.dmod_mode == UHSDR_DEMOD_FM) return p.sq_stages == 6 ? &kBackFm : nullptr;
    const int dm = p.notch_enabled ? DM_NONE : plan_dm(p);
    if (p.stereo)
    {
        for (const BackVariant& v : kBackStereo)
            if (v.pre == p.pre_stages && v.aa == p.aa_stages && v.L == p.interp_L && v.ph == p.interp_phase &&
                v.w == p.agc.attack_buffsize && v.dm == dm)
                return &v;
        return nullptr;
    }
    for (const BackVariant& v : kBack)
        if (v.pre == p.pre_stages && v.aa == p.aa_stages && v.L == p.interp_L && v.ph == p.interp_phase &&
            v.w == p.agc.attack_buffsize && v.dm == dm)
            return &v;
    return nullptr;
}

// ------------------------------------------------------------------------------------
// host runtime

constexpr int TAPS2_MAX = (UHSDR_MAX_FIR_TAPS + 7) & ~7;   // taps per pair table
constexpr int BACK_FUSED_MIN_CHANNELS = 131072;   // measured crossover (64-frame calls)

// pipelined mode: hand-off buffers in rotation, so rx_front runs ahead of rx_back and the side
// stream's wait on it is already satisfied when rx_back gets there.  The buffers' reuse is
// ordered per group of PIPE_GROUP calls, not per call: rx_back records a completion event at
// the end of each group, and the first rx_front of a group waits for the group two before it
// (PIPE_BUFS = 2 PIPE_GROUP buffers).  With the front's and back's events folded into their
// launches (hipExtLaunchKernelGGL) a call costs the host 2 launches + 1 stream wait (+1 per
// group) instead of 2 launches + 2 records + 2 waits: C2's host submission, 22-25 us per call,
// was as long as the GPU's, and the GPU idled between calls (rocprofv3 kernel trace, r03).
#ifndef UHSDR_PIPE_GROUP
#define UHSDR_PIPE_GROUP 4
#endif
constexpr int PIPE_GROUP = UHSDR_PIPE_GROUP;
#ifndef UHSDR_BACK_SKEW
#define UHSDR_BACK_SKEW 1
#endif
constexpr int PIPE_BUFS = 2 * PIPE_GROUP;

struct uhsdr_rx_s
{
    uhsdr_rx_plan plan;
    uhsdr_rx_plan* d_plan;
    const FrontVariant* fv;
    const BackVariant* bv;
    const NotchVariant* nv;  // LMS auto notch kernel (null: notch off)
    const ChainVariant* cv;  // rx_chain instance of the path (null: none)
    int C, N, Nd, Nf;        // Nf: frames per front launch (N split into N / Nf launches)
    int lw;                  // front LDS window pitch (floats)
    int schedule;            // resolved UHSDR_SCHEDULE_SPLIT_PIPE / _SPLIT_FUSED / _CHAIN
    int precision;           // UHSDR_PRECISION_EXACT / _FMA (front FIR MACs)
    int T1, T2;
    hipStream_t stream;
    // front state
    float *hist1, *hist2, *teta, *osc, *adec, *adec_q;
    uint16_t* d_lanemap;     // [2][2][64] the front's lane maps for R = 8 / 16, pass 1 / 2 (g << 8 | b)
    uint16_t lmap[2][2][64]; // host copies (front_window_pitch's choice)
    int* tp;                 // [5][C] twin-peaks detector state
    unsigned* clip;          // user output (uhsdr_rx_set_clip_output)
    float* d_taps2;          // FIR pair tables: [2][2 * TAPS2_MAX] (pass 1, pass 2)
    // back state
    BackState bs;
    void* arena;
    size_t arena_bytes;
    long long dec_samples;   // decimated samples processed (AGC ring phase)
    int cw_count;            // CW decoder sample_counter (uniform over channels)
    int cw_bmax, cw_blocks_last;
    int beep_left;           // key beep: 32-frame calls still to get the tone (uhsdr_rx_key_beep)
    uint32_t beep_acc;       // its softdds accumulator at the next beep frame
    uint8_t* cw_signal;      // user outputs (uhsdr_rx_set_cw_outputs)
    float* cw_energy;
    long long calls_done;
    long long front_launches; // oscillator ping-pong parity
    // pipelined mode (uhsdr_rx_set_pipelined): rx_back on a side stream, decimated hand-off
    // rotated over PIPE_BUFS buffers so the next calls' rx_front overlaps this call's rx_back
    int pipelined;
    hipStream_t side;
    hipEvent_t ev_front, ev_join, ev_back[2];  // ev_back[g % 2]: end of group g's rx_back
    hipEvent_t ev_switch;    // uhsdr_rx_set_stream: new stream after the old one's work
    float *adecp[PIPE_BUFS - 1], *adec_qp[PIPE_BUFS - 1];  // the pipelined mode's other hand-off buffers
    long long calls_issued;  // process() calls
    long long pipe_calls;    // calls since the pipelined mode was entered (buffer index, group)
    int side_dirty;          // back-end work on the side stream not yet joined by a one-kernel call
    // per-kernel timing (uhsdr_rx_enable_timing)
    int timing;               // 0 off, else every timing-th call is bracketed
    int tsample;              // the call being enqueued is a timed one
    long long tcalls;         // calls since timing was enabled
    int nev;
    int nev_cap;
    hipEvent_t* ev;          // [cap][NKERN kernels][start, stop]
    uint8_t* evmask;         // [cap] kernels recorded in each timed call
    float total_ms[4];
    int launches[4];
    // failure contract of the bounded device-side polls: fail_host is host-mapped coherent memory
    // (fail_dev its device address) that a poll giving up sets to 1; process / join / synchronize
    // return UHSDR_TIMEOUT while it is set, uhsdr_rx_reset clears it
    volatile unsigned* fail_host;
    unsigned* fail_dev;
    unsigned spin_max;       // polls before a give-up (uhsdr_rx_set_handoff_bound; default 2^24)
    // pipelined device hand-off (uhsdr_rx_set_pipelined 2): rx_back polls the arrival counters the
    // front waves of its group bump (FrontArgs::gcnt) instead of waiting on a cross-stream event
    int dflag;
    unsigned* gcnt;          // [PIPE_BUFS][groups][CNT_PITCH] arrival counters, one row per hand-off buffer
    unsigned fills[PIPE_BUFS];   // counted front launches into each buffer since reset
    int* skew;               // BackSched: per group, the wave pipeline ended a launch skewed (arena)
    float* bnd;              // BackSched: the roles' pending input sub-calls (arena)
    int dflag_grid;          // largest rx_back grid it is used for (half the CUs: the polling
                             // workgroups never crowd out the front they wait for)
    int back_attr;           // rx_back's LDS attribute raised for the reserved launch (1), failed (-1)
    // persistent back end (uhsdr_rx_set_pipelined 3, PersistCtl): pmem = host-mapped coherent memory,
    // PC_WORDS control words then DESC_RING call descriptors (pmem_dev: its device address); plive:
    // a launch may still take the next grant; plast: the last call granted; pprev: the previous call
    // ran on it (else the next one starts a new run: both streams synchronised, the words reset)
    int pers;
    unsigned* pmem;
    unsigned* pmem_dev;
    unsigned* pdec;          // device memory: group 0's decision per call (BackArgs::pdec)
    int plive, pprev;
    unsigned plast;
    unsigned pepoch;         // the running (or last) launch's epoch (BackArgs::pepoch)
    unsigned plaunches;      // persistent launches since creation (uhsdr_rx_debug_persist)
    int main_back;           // back-end state was last written on the handle's stream (a one-kernel
                             // schedule, a serial call, a reset): the next side-stream rx_back waits
                             // on ev_front, which orders it after that work; the device hand-off
                             // orders it after the front only
};

// kernel slots of the timing API: a call runs rx_front + rx_back (any back-end kernel) or rx_chain
enum { K_FRONT = 0, K_BACK = 1, K_CHAIN = 2, NKERN = 3 };
static const char* kKernelNames[NKERN] = { "rx_front", "rx_back", "rx_chain" };

static bool side_mode(const uhsdr_rx_s* h) { return h->pipelined; }
static hipStream_t back_stream(const uhsdr_rx_s* h) { return side_mode(h) ? h->side : h->stream; }

static void time_mark(uhsdr_rx_s* h, int k, int which)
{
    if (!h->tsample) return;
    (void)hipEventRecord(h->ev[((size_t)h->nev * NKERN + k) * 2 + which], k == K_BACK ? back_stream(h) : h->stream);
    if (which) h->evmask[h->nev] |= (uint8_t)(1u << k);
}

// the persistent back end's running launch gets no more grants (PersistCtl: the next call goes to a
// new launch of the next epoch); it ends after the calls granted so far
static void pers_close(uhsdr_rx_s* h)
{
    h->plive = 0;
}

// every call enqueued so far, on both streams, has finished
static hipError_t sync_all(uhsdr_rx_s* h)
{
    pers_close(h);
    hipError_t e = hipStreamSynchronize(h->stream);
    if (e == hipSuccess && h->side) e = hipStreamSynchronize(h->side);
    return e;
}

static void time_harvest(uhsdr_rx_s* h)
{
    if (!h->nev) return;
    (void)sync_all(h);
    for (int i = 0; i < h->nev; ++i)
        for (int k = 0; k < NKERN; ++k)
        {
            float ms = 0.0f;
            const size_t e = ((size_t)i * NKERN + k) * 2;
            if ((h->evmask[i] >> k & 1) && hipEventElapsedTime(&ms, h->ev[e], h->ev[e + 1]) == hipSuccess)
            {
                h->total_ms[k] += ms;
                h->launches[k] += 1;
            }
        }
    h->nev = 0;
}

#define HIPCHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { uhsdr_set_error("%s: %s", #x, hipGetErrorString(e_)); return UHSDR_DEVICE_ERROR; } } while (0)

// LDS window pitch per channel: room for every pass (T-1 history + new samples + tail),
// a multiple of 4 floats, chosen among 16 candidates for the fewest ds_read bank conflicts
// Pass 1 is always a FIR pair over an interleaved window (2 floats per sample); pass 2 is the
// scalar audio decimator (Hilbert-first paths) or the Hilbert pair (decimate-first paths).
static size_t front_lds_extra(const uhsdr_rx_s* h);
constexpr size_t LDS_PER_CU = 160 * 1024;           // MI355X_MICROARCH.md §LDS

// waves per CU a kernel's register allocation allows (MI355X_MICROARCH.md §Register files:
// granule 8, 512 VGPRs + AGPRs per lane per SIMD, at most 8 waves per SIMD)
static int kernel_waves_per_cu(const void* fn)
{
    hipFuncAttributes at;
    if (hipFuncGetAttributes(&at, fn) != hipSuccess || at.numRegs <= 0) return 16;
    const int alloc = (at.numRegs + 7) & ~7;
    const int w = 512 / alloc;
    return 4 * (w > 8 ? 8 : w);
}
// floats after the last window that the FIRs' over-read may touch (FRONT_TAIL pairs)
constexpr int FRONT_SLACK = 2 * FRONT_TAIL;

// the front's window pitch and lane maps: the most waves per CU (LDS per wave sets them: the
// front is occupancy-sensitive), then the fewest modeled LDS-array cycles of the window traffic
// (front_lds_pass1 / _pass2) over the pitches from the data's length up and, per pass, the lane
// maps front_lane (runs of consecutive blocks, for the pass's window stride) and interleaved.
// (At 1M x 64 P48 the occupancy-only choice lw = 320 = 0 mod 64 put every channel's window on
// the same banks: 74 % of the LDS cycles were conflicts, PMC r03.)
static int front_window_pitch(const uhsdr_rx_s* h, uint16_t (&lm1_out)[64], uint16_t (&lm2_out)[64])
{
    const int N = h->Nf, R = h->fv->R, M = h->plan.decimation_rate;
    const bool df = h->plan.use_decimated_iq;
    const bool pair2 = df || h->fv->st;                  // pass 2 is a FIR pair over {x0, x1}
    const int nb = N / R, cpw = FRONT_WAVE / nb;
    const int n2 = df ? N / M : N;
    const int pb1 = front_pad1(R, h->fv->decim_first != 0, h->fv->m);
    // a padded pass-1 window holds its FIRs' over-read (FRONT_TAIL pairs) inside the pitch
    int need = pb1 ? pwin_off<4>(h->T1 - 1 + N + FRONT_TAIL) : 2 * (h->T1 - 1 + N);   // pb1: 0 or 4
    const int need2 = h->T2 ? (pair2 ? 2 : 1) * (h->T2 - 1 + n2) : 0;
    need = ((need > need2 ? need : need2) + 3) & ~3;
    const int RD = R / M;
    const int NV2 = df ? RD : R, RD2 = df ? RD : RD, M2 = df ? 1 : M;   // pass 2 (front_body)
    const int S2 = (pair2 ? 2 : 1) * NV2;                 // pass-2 window floats per lane
    const size_t extra = front_lds_extra(h) + FRONT_SLACK;
    const int vgpr_waves = kernel_waves_per_cu((const void*)h->fv->fn);
    // candidate maps: front_lane for the pass-1 stride, for the pass-2 stride, interleaved
    uint16_t maps[3][64];
    int nmaps = 0;
    for (int m = 0; m < 3; ++m)
    {
        bool ok = true;
        for (int l = 0; l < 64 && ok; ++l)
        {
            int g = 0, b = 0;
            if (m == 0) front_lane(l, nb, 2 * R, g, b);
            else if (m == 1) { ok = S2 <= 64; if (ok) front_lane(l, nb, S2, g, b); }
            else ok = front_lane_interleaved(l, nb, g, b);
            maps[nmaps][l] = (uint16_t)(g << 8 | b);
        }
        if (ok) ++nmaps;
    }
    int best = need, best_cost = 1 << 30, best_waves = 0, best1 = 0, best2 = 0;
    for (int lw = need; lw < need + 64; lw += 4)
    {
        int waves = (int)(LDS_PER_CU / (sizeof(float) * ((size_t)cpw * lw + extra)));
        waves = waves > vgpr_waves ? vgpr_waves : waves;
        // history rows: pair rows (hist_stride / 2 float4s per channel), or the mono decimator's
        const int hist_cost = front_lds_hist(lw, cpw, hist_p4(h->T1), 2 * N) +
                              (h->T2 ? (pair2 ? front_lds_hist(lw, cpw, hist_p4(h->T2), 2 * (df ? N / M : N))
                                              : front_lds_hist(lw, cpw, hist_stride(h->T2) / 4, N)) : 0);
        for (int m1 = 0; m1 < nmaps; ++m1)
            for (int m2 = 0; m2 < (h->T2 ? nmaps : 1); ++m2)
            {
                int cost = front_lds_pass1(lw, maps[m1], cpw, h->T1, R, pb1) + hist_cost;
                if (h->T2) cost += front_lds_pass2(lw, maps[m1], maps[m2], cpw, h->T2, pair2, NV2, RD2, M2);
                if (waves > best_waves || (waves == best_waves && cost < best_cost))
                {
                    best_cost = cost; best = lw; best_waves = waves; best1 = m1; best2 = h->T2 ? m2 : m1;
                }
            }
    }
    memcpy(lm1_out, maps[best1], sizeof lm1_out);
    memcpy(lm2_out, maps[best2], sizeof lm2_out);
    return best;
}

// interleaved tap pairs {c0[k], c1[k]} for fir_block2, zero-padded to a multiple of 8 taps
static void pair_taps(float* dst, const float* c0, const float* c1, int T)
{
    const int n = (T + 7) & ~7;
    for (int k = 0; k < n; ++k)
    {
        dst[2 * k] = k < T ? c0[k] : 0.0f;
        dst[2 * k + 1] = k < T ? c1[k] : 0.0f;
    }
}

// LDS of one front workgroup (one wave): must match the carve-up in rx_front
// floats after the windows: auto-IQ factors, oscillator trajectory, FM exchange
static size_t front_lds_extra(const uhsdr_rx_s* h)
{
    const int N = h->Nf;
    const int cpw = FRONT_WAVE / (N / h->fv->R);
    size_t f = 0;
    if (h->plan.iq_auto_correction) f += 2 * cpw * (N / BLK);
    if (h->plan.freq_shift_hz != 0 && h->plan.shift_kind == 2) f += 2 * N;
    if (h->fv->m == 1) f += 2 * FRONT_WAVE;              // FM: per-lane last {I, Q} exchange
    return f;
}

static size_t front_lds(const uhsdr_rx_s* h)
{
    const int N = h->Nf;
    const int cpw = FRONT_WAVE / (N / h->fv->R);
    size_t f = (size_t)cpw * h->lw + front_lds_extra(h) + FRONT_SLACK;
    return f * sizeof(float);
}

// rx_chain's LDS: the front region (also the back end's output staging) + the decimated hand-off
static size_t chain_front_floats(const uhsdr_rx_s* h)
{
    const size_t f = front_lds(h) / sizeof(float), ys = (size_t)BACK_CH * FUSED_YPITCH;
    return ((f > ys ? f : ys) + 3) & ~(size_t)3;
}
static size_t chain_lds(const uhsdr_rx_s* h)
{
    return sizeof(float) * (chain_front_floats(h) + (size_t)h->Nd * CHAIN_ADP);
}

// front variant with R outputs per lane for the handle's call size (strict: exactly R)
static uhsdr_status configure_front(uhsdr_rx_s* h, int R, bool strict)
{
    const FrontVariant* fv = find_front(h->plan, h->N, R, strict);
    if (!fv) { uhsdr_set_error("no front kernel with %d outputs per lane for %d-frame calls", R, h->N); return UHSDR_UNSUPPORTED; }
    const FrontVariant* old = h->fv;
    const int oNf = h->Nf, olw = h->lw;
    h->fv = fv;
    h->T1 = fv->t1; h->T2 = fv->t2;
    h->Nf = front_frames(h->N, fv->R);
    uint16_t lm[2][64];
    h->lw = front_window_pitch(h, lm[0], lm[1]);
    uhsdr_status st = UHSDR_OK;
    if (h->N % h->Nf) { uhsdr_set_error("frames_per_call %d not a multiple of %d", h->N, h->Nf); st = UHSDR_LENGTH_ERROR; }
    else if (front_lds(h) > 64 * 1024) { uhsdr_set_error("frames_per_call too long for LDS"); st = UHSDR_LENGTH_ERROR; }
    if (st != UHSDR_OK && old) { h->fv = old; h->T1 = old->t1; h->T2 = old->t2; h->Nf = oNf; h->lw = olw; }
    if (st == UHSDR_OK)
    {
        // the map for this block size (a deterministic function of the handle's shape: a launch
        // still in flight with this slot reads the same values)
        const int k = fv->R == 16 ? 1 : 0;
        memcpy(h->lmap[k], lm, sizeof lm);
        if (h->d_lanemap && hipMemcpy(h->d_lanemap + 128 * k, lm, sizeof lm, hipMemcpyHostToDevice) != hipSuccess)
        {
            uhsdr_set_error("lane map upload failed");
            st = UHSDR_DEVICE_ERROR;
        }
    }
    return st;
}

// can the handle run rx_chain: a chain instance, one front pass per call, LDS within a workgroup's
static bool chain_ok(const uhsdr_rx_s* h)
{
    // (the chain's back end has no DC removal: its paths are SSB / CW / DIGI, no notch)
    return h->cv && h->fv->R == h->cv->R && h->Nf == h->N && chain_lds(h) <= 64 * 1024 && !h->plan.agc.remove_dc;
}

static size_t back_lds(const uhsdr_rx_s* h);

// AUTO: batches of BACK_FUSED_MIN_CHANNELS channels and more run rx_front + rx_back_fused
// (SPLIT_FUSED), smaller ones rx_front + the back-end wave pipeline (SPLIT_PIPE); rx_chain (CHAIN)
// runs only when asked for (measured slower at 1M x 64).
// Measured and dropped: the fused back end split in two at the interpolator (decimated-rate stages
// / 48 ksps stages, half the registers each): 0.225 vs 0.211 ms at 1M x 64, and slower on C3 / C5
// too -- more waves did not raise the VALU issue rate.
static int resolve_schedule(const uhsdr_rx_s* h, int want)
{
    if (want == UHSDR_SCHEDULE_AUTO)
    {
        if (h->C < BACK_FUSED_MIN_CHANNELS) return UHSDR_SCHEDULE_SPLIT_PIPE;
        return h->bv->fused ? UHSDR_SCHEDULE_SPLIT_FUSED : UHSDR_SCHEDULE_SPLIT_PIPE;
    }
    if (want == UHSDR_SCHEDULE_CHAIN) return chain_ok(h) ? want : -1;
    if (want == UHSDR_SCHEDULE_SPLIT_FUSED) return h->bv->fused ? want : -1;
    if (want == UHSDR_SCHEDULE_SPLIT_PIPE) return want;
    return -1;
}

// the fused back-end kernel of a launch: FORM 1 (one body, 3 waves per SIMD) when the AGC is on,
// no DC removal and no CW decoder front end (only the L == 4 bodies carry one); else the kernel
// that dispatches the AGC / CW flags itself
static back_fn fused_back_fn(const uhsdr_rx_s* h)
{
    const BackVariant* bv = h->bv;
    if (h->plan.agc.remove_dc || !bv->fused_nodc) return bv->fused;
    if (bv->fused_ssb && h->plan.agc.mode != 5 && (!h->plan.cw_enabled || bv->L != 4)) return bv->fused_ssb;
    return bv->fused_nodc;
}

static size_t back_lds(const uhsdr_rx_s* h)
{
    if (h->bv->dm == DM_FM) return sizeof(float) * (size_t)BACK_CH * 2 * (BLK + 1);
    return sizeof(float) * (size_t)back_lds_floats(BLK / h->plan.interp_L);
}

extern "C" int uhsdr_rx_plan_supported(const uhsdr_rx_plan* p)
{
    return p && uhsdr_rx_mode_supported(p) && find_front(*p) && find_back(*p) && (!p->notch_enabled || find_notch(*p));
}

// FMA acceptance (north_star: within 1e-5 normwise), from the sweep of every Hilbert-first
// (path, demodulator, stereo) against the oracle (tools/fma_sweep.py, profiles/r03_fma_sweep.jsonl):
//   FM (paths 1-3)                          max 1.4e-6
//   12 ksps wide paths (48-54, decimation 4) max 5.0e-6
//   24 ksps wide paths (55-65, decimation 2) 7.6e-6 .. 1.22e-5: at the bound, refused
// Decimate-first families (narrow SSB / CW, AM, SAM) exceed it (P35 1.7e-5, P70 AM 1.8e-5 /
// SAM 1.3e-5, P4 CW 1.3e-5), refused.  Accepted cases sit at half the bound or less.
extern "C" int uhsdr_rx_plan_fma_ok(const uhsdr_rx_plan* p)
{
    if (!p || p->use_decimated_iq) return 0;
    return p->dmod_mode == UHSDR_DEMOD_FM || p->decimation_rate == 4;
}

extern "C" uhsdr_status uhsdr_rx_reset(uhsdr_rx_handle h)
{
    if (!h) return UHSDR_ARGUMENT_ERROR;
    HIPCHK(sync_all(h));
    HIPCHK(hipMemsetAsync(h->arena, 0, h->arena_bytes, h->stream));
    // oscillator starts at {I=0, Q=1} (freq_shift.c:48-49); both ping-pong copies
    const float osc0[4] = { 0.0f, 1.0f, 0.0f, 1.0f };
    HIPCHK(hipMemcpyAsync(h->osc, osc0, sizeof osc0, hipMemcpyHostToDevice, h->stream));
    // ts.twinpeaks_tested = TWINPEAKS_WAIT at boot (src/uhsdr_main.c:339); the statics start at 0
    HIPCHK(hipMemsetD32Async((hipDeviceptr_t)h->tp, UHSDR_TWINPEAKS_WAIT, (size_t)h->C, h->stream));
    // the device hand-off's arrival counters restart with fills; a poll's give-up is cleared (the
    // state it poisoned was zeroed above)
    HIPCHK(hipMemsetAsync(h->gcnt, 0, sizeof(unsigned) * CNT_PITCH * PIPE_BUFS * (((size_t)h->C + BACK_CH - 1) / BACK_CH), h->stream));
    *h->fail_host = 0;
    memset(h->fills, 0, sizeof h->fills);
    h->main_back = 1;
    h->pprev = 0;
    if (h->bs.cw)
    {
        // old_siglevel starts at 0.001 (function static, cw_decoder.c:189)
        float* v = (float*)malloc(sizeof(float) * h->C);
        for (int i = 0; i < h->C; ++i) v[i] = 0.001f;
        HIPCHK(hipMemcpyAsync(h->bs.cw + 2 * (size_t)h->C, v, sizeof(float) * h->C, hipMemcpyHostToDevice, h->stream));
        HIPCHK(hipStreamSynchronize(h->stream));
        free(v);
    }
    HIPCHK(hipStreamSynchronize(h->stream));
    h->dec_samples = 0;
    h->calls_done = 0;
    h->front_launches = 0;
    h->calls_issued = 0;
    h->cw_count = 0;
    h->cw_blocks_last = 0;
    h->beep_left = 0;
    h->beep_acc = 0;
    return UHSDR_OK;
}

extern "C" uhsdr_status uhsdr_rx_key_beep(uhsdr_rx_handle h, int32_t calls)
{
    if (!h || calls < 0) { uhsdr_set_error("bad argument"); return UHSDR_ARGUMENT_ERROR; }
    h->beep_acc = 0;          // AudioManagement_KeyBeep: ads.beep.acc = 0 (audio_management.c:372)
    h->beep_left = calls;
    return UHSDR_OK;
}

extern "C" uhsdr_status uhsdr_rx_create(const uhsdr_rx_config* cfg, int32_t C, int32_t N, void* stream,
                                        uhsdr_rx_handle* out)
{
    if (!cfg || !out || C <= 0 || N <= 0) { uhsdr_set_error("bad argument"); return UHSDR_ARGUMENT_ERROR; }
    if (N % BLK) { uhsdr_set_error("frames_per_call %d not a multiple of %d", N, BLK); return UHSDR_LENGTH_ERROR; }
    *out = nullptr;
    uhsdr_rx_s* h = (uhsdr_rx_s*)calloc(1, sizeof(uhsdr_rx_s));
    uhsdr_status bst = uhsdr_rx_plan_build(cfg, &h->plan);
    if (bst != UHSDR_OK) { free(h); return bst; }
    const uhsdr_rx_plan& p = h->plan;
    // 8 FIR outputs per lane, or 16 for the narrow (decimate-first SSB / CW / DIGI) family on large
    // batches, whose 199-tap Hilbert pair at the decimated rate then gets 4 outputs per register
    // window instead of 2 (C5, 131072 x 256: 0.394 -> 0.359 ms per call; the wide, AM / SAM and
    // FM families measured slower at 16: 1M x 64 P48 0.695 vs 0.573 ms front, C3 SAM 0.129 vs
    // 0.115, C4 FM 0.108 vs 0.094; uhsdr_rx_set_front_block overrides)
    const bool narrow = p.use_decimated_iq && p.hilbert_taps > 0;     // the front's pass 2 is the Hilbert pair
    h->fv = find_front(p, N, narrow && C >= 65536 ? 16 : 8);
    h->bv = find_back(p);
    h->nv = find_notch(p);
    h->cv = find_chain(p, h->bv);
    if (!uhsdr_rx_mode_supported(&p) || !h->fv || !h->bv || (p.notch_enabled && !h->nv))
    {
        free(h);
        uhsdr_set_error("demodulation mode %d / filter path %d not implemented on the device", cfg->dmod_mode,
                        cfg->filter_path);
        return UHSDR_UNSUPPORTED;
    }
    h->C = C; h->N = N; h->Nd = N / p.decimation_rate;
    h->stream = (hipStream_t)stream;
    {
        const int R = h->fv->R;
        h->fv = nullptr;
        const uhsdr_status fs = configure_front(h, R, true);
        if (fs != UHSDR_OK) { free(h); return fs; }
    }
    const int W = h->bv->w;
    h->schedule = resolve_schedule(h, UHSDR_SCHEDULE_AUTO);

    size_t fl = 0;
    auto take = [&](size_t n) { size_t o = fl; fl += (n + 63) & ~(size_t)63; return o; };
    const size_t hs1 = (h->T1 - 1 + 3) & ~3, hs2 = (h->T2 - 1 + 3) & ~3;   // padded history rows
    const size_t o_h1 = take((size_t)2 * C * hs1);     // pair rows {I, Q}
    const size_t o_h2 = take((size_t)2 * C * hs2);     // pair rows, or the scalar decimator row
    const size_t o_teta = take((size_t)3 * C), o_osc = take(4), o_tp = take((size_t)5 * C);
    const size_t o_pre = take((size_t)10 * C), o_aa = take((size_t)10 * C), o_bq1 = take((size_t)16 * C);
    const size_t o_bq2 = take((size_t)4 * C), o_ip = take((size_t)15 * C), o_ring = take(W > 0 ? (size_t)(W - 1) * C : 0);
    const size_t o_agc = take((size_t)(8 + AGC_Q) * C), o_agci = take((size_t)3 * C);
    const bool am = plan_dm(p) != DM_NONE;             // AM / SAM / FM demodulator state
    const bool st = p.stereo != 0;                      // second audio channel
    const size_t o_sam = take(am ? (size_t)(7 + 96 + 2) * C : 0), o_adq = take(am || st ? (size_t)C * h->Nd : 0);
    const size_t o_ring1 = take(st && W > 0 ? (size_t)(W - 1) * C : 0);
    const size_t o_pre1 = take(st ? (size_t)10 * C : 0), o_aa1 = take(st ? (size_t)10 * C : 0);
    const size_t o_bq1_1 = take(st ? (size_t)16 * C : 0), o_bq2_1 = take(st ? (size_t)4 * C : 0);
    const size_t o_ip1 = take(st ? (size_t)15 * C : 0);
    const size_t o_notch = take(h->nv ? (size_t)(2 * NOTCH_TAPS + 2 + NOTCH_DELAY) * C : 0);
    const bool cw = p.cw_enabled && p.decimation_rate == 4;
    const size_t o_cw = take(cw ? (size_t)5 * C : 0);
    // the wave pipeline's running ahead (BackSched): per group its skew word, per channel the roles'
    // pending input sub-calls
    const bool skewable = h->bv->dm == DM_NONE && !st && p.interp_L > 0;
    const size_t bnd_rows = skewable ? (size_t)6 * (BLK / p.interp_L) + 2 * BLK : 0;
    const size_t o_skew = take(skewable ? (size_t)(C + BACK_CH - 1) / BACK_CH : 0);
    const size_t o_bnd = take(skewable ? bnd_rows * C : 0);
    h->arena_bytes = fl * sizeof(float);
    if (hipMalloc(&h->arena, h->arena_bytes) != hipSuccess ||
        hipMalloc((void**)&h->adec, sizeof(float) * (size_t)C * h->Nd) != hipSuccess ||
        hipMalloc((void**)&h->d_plan, sizeof(uhsdr_rx_plan)) != hipSuccess ||
        hipMalloc((void**)&h->d_taps2, sizeof(float) * 4 * TAPS2_MAX) != hipSuccess ||
        hipMalloc((void**)&h->d_lanemap, sizeof(uint16_t) * 4 * 64) != hipSuccess ||
        hipMalloc((void**)&h->gcnt, sizeof(unsigned) * CNT_PITCH * PIPE_BUFS * (((size_t)C + BACK_CH - 1) / BACK_CH)) != hipSuccess ||
        hipHostMalloc((void**)&h->fail_host, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer((void**)&h->fail_dev, (void*)h->fail_host, 0) != hipSuccess)
    {
        uhsdr_set_error("hipMalloc failed (%zu bytes state)", h->arena_bytes);
        (void)uhsdr_rx_destroy(h);
        return UHSDR_DEVICE_ERROR;
    }
    *h->fail_host = 0;
    h->spin_max = DFLAG_SPIN_MAX;
    float* A = (float*)h->arena;
    h->hist1 = A + o_h1; h->hist2 = A + o_h2;
    h->teta = A + o_teta; h->osc = A + o_osc; h->tp = (int*)(A + o_tp);
    h->bs.pre = A + o_pre; h->bs.aa = A + o_aa; h->bs.bq1 = A + o_bq1; h->bs.bq2 = A + o_bq2;
    h->bs.interp = A + o_ip; h->bs.ring = A + o_ring; h->bs.agc = A + o_agc; h->bs.agci = (int*)(A + o_agci);
    h->bs.sam = am ? A + o_sam : nullptr;
    h->bs.cw = cw ? A + o_cw : nullptr;
    h->skew = skewable ? (int*)(A + o_skew) : nullptr;
    h->bnd = skewable ? A + o_bnd : nullptr;
    h->bs.notch = h->nv ? A + o_notch : nullptr;
    h->bs.ring1 = st ? A + o_ring1 : nullptr;
    h->bs.pre1 = st ? A + o_pre1 : nullptr; h->bs.aa1 = st ? A + o_aa1 : nullptr;
    h->bs.bq1_1 = st ? A + o_bq1_1 : nullptr; h->bs.bq2_1 = st ? A + o_bq2_1 : nullptr;
    h->bs.interp1 = st ? A + o_ip1 : nullptr;
    {
        // blocks per call: one completes at the end of every ceil(blocksize / NDC)-th call
        const int ndc = BLK / p.decimation_rate, cpb = (p.cw_blocksize + ndc - 1) / ndc;
        h->cw_bmax = cw ? (N / BLK + cpb - 1) / cpb : 0;
    }
    h->adec_q = am || st ? A + o_adq : nullptr;
    {
        // pass 1: the Hilbert / low-pass pair (Hilbert-first and FM), or the I and Q decimators
        // (DECIMATE_RX_I / _Q: the same table for SSB, the path's I and Q tables for AM / SAM);
        // pass 2 (decimate-first SSB): the Hilbert pair at the decimated rate
        float t2[4 * TAPS2_MAX];
        memset(t2, 0, sizeof t2);
        if (p.use_decimated_iq)
        {
            const bool amq = plan_dm(p) != DM_NONE;
            pair_taps(t2, p.dec, amq ? p.dec_q : p.dec, p.dec_taps);
            if (h->T2) pair_taps(t2 + 2 * TAPS2_MAX, p.hilbert_i, p.hilbert_q, p.hilbert_taps);
        }
        else
        {
            pair_taps(t2, p.hilbert_i, p.hilbert_q, p.hilbert_taps);
            // stereo Hilbert-first: DECIMATE_RX_I / _Q (the same table) as a pair
            // the audio decimator as duplicated pairs {dec, dec}: the stereo decimator pair
            // (DECIMATE_RX_I / _Q, the same table) and the mono decimator's packed output pairs
            pair_taps(t2 + 2 * TAPS2_MAX, p.dec, p.dec, p.dec_taps);
        }
        if (hipMemcpy(h->d_taps2, t2, sizeof t2, hipMemcpyHostToDevice) != hipSuccess)
        {
            uhsdr_set_error("tap upload failed");
            (void)uhsdr_rx_destroy(h);
            return UHSDR_DEVICE_ERROR;
        }
    }
    {
        // the front's lane -> (channel, block) maps (configure_front)
        const uint16_t (&lm)[2][2][64] = h->lmap;
        if (hipMemcpy(h->d_lanemap, lm, sizeof lm, hipMemcpyHostToDevice) != hipSuccess)
        {
            uhsdr_set_error("lane map upload failed");
            (void)uhsdr_rx_destroy(h);
            return UHSDR_DEVICE_ERROR;
        }
    }
    if (hipMemcpy(h->d_plan, &h->plan, sizeof(uhsdr_rx_plan), hipMemcpyHostToDevice) != hipSuccess)
    {
        uhsdr_set_error("plan upload failed");
        (void)uhsdr_rx_destroy(h);
        return UHSDR_DEVICE_ERROR;
    }
    const uhsdr_status rs = uhsdr_rx_reset(h);
    if (rs != UHSDR_OK) { (void)uhsdr_rx_destroy(h); return rs; }
    *out = h;
    return UHSDR_OK;
}

extern "C" uhsdr_status uhsdr_rx_set_cw_outputs(uhsdr_rx_handle h, uint8_t* signal, float* energy)
{
    if (!h) return UHSDR_ARGUMENT_ERROR;
    h->cw_signal = signal;
    h->cw_energy = energy;
    return UHSDR_OK;
}

extern "C" uhsdr_status uhsdr_rx_set_clip_output(uhsdr_rx_handle h, uint32_t* clip)
{
    if (!h) return UHSDR_ARGUMENT_ERROR;
    h->clip = clip;
    return UHSDR_OK;
}

__global__ void twinpeaks_rearm(int* st, int C)
{
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c < C && st[c] == UHSDR_TWINPEAKS_CODEC_RESTART) st[c] = UHSDR_TWINPEAKS_WAIT;
}

extern "C" uhsdr_status uhsdr_rx_twinpeaks_state(uhsdr_rx_handle h, int32_t* state)
{
    if (!h || !state) return UHSDR_ARGUMENT_ERROR;
    HIPCHK(hipMemcpyAsync(state, h->tp, sizeof(int32_t) * (size_t)h->C, hipMemcpyDeviceToDevice, h->stream));
    return UHSDR_OK;
}

extern "C" uhsdr_status uhsdr_rx_twinpeaks_rearm(uhsdr_rx_handle h)
{
    if (!h) return UHSDR_ARGUMENT_ERROR;
    hipLaunchKernelGGL(twinpeaks_rearm, dim3((h->C + 255) / 256), dim3(256), 0, h->stream, h->tp, h->C);
    HIPCHK(hipGetLastError());
    return UHSDR_OK;
}

extern "C" int32_t uhsdr_rx_cw_blocks_max(uhsdr_rx_handle h) { return h ? h->cw_bmax : 0; }
extern "C" int32_t uhsdr_rx_cw_blocks_last(uhsdr_rx_handle h) { return h ? h->cw_blocks_last : 0; }

extern "C" uhsdr_status uhsdr_rx_set_stream(uhsdr_rx_handle h, void* stream)
{
    if (!h) return UHSDR_ARGUMENT_ERROR;
    if ((hipStream_t)stream == h->stream) return UHSDR_OK;
    // the next call's kernels read and write the state the calls already queued on the old
    // stream (and, pipelined, on the side stream) are still using: order the new stream after them
    if (h->pipelined)
    {
        const uhsdr_status st = uhsdr_rx_join(h);
        if (st != UHSDR_OK) return st;
    }
    if (!h->ev_switch) HIPCHK(hipEventCreateWithFlags(&h->ev_switch, hipEventDisableTiming));
    HIPCHK(hipEventRecord(h->ev_switch, h->stream));
    HIPCHK(hipStreamWaitEvent((hipStream_t)stream, h->ev_switch, 0));
    h->stream = (hipStream_t)stream;
    return UHSDR_OK;
}

static uhsdr_status rx_process(uhsdr_rx_handle h, const int32_t* iq, float* audio, float* audio0, int32_t* dst);

extern "C" uhsdr_status uhsdr_rx_process(uhsdr_rx_handle h, const int32_t* iq, float* audio, int32_t* dst)
{
    return rx_process(h, iq, audio, nullptr, dst);
}

extern "C" uhsdr_status uhsdr_rx_process_stereo(uhsdr_rx_handle h, const int32_t* iq, float* audio, float* audio0,
                                                int32_t* dst)
{
    return rx_process(h, iq, audio, audio0, dst);
}

// demodulator of rx_front's Hilbert pair (FRONT_COMB_*)
static int front_comb_of(const uhsdr_rx_plan& p)
{
    if (p.stereo == 1) return FRONT_COMB_SSB_ST;
    if (p.stereo == 2) return FRONT_COMB_IQ_ST;
    if (p.dmod_mode == UHSDR_DEMOD_IQ) return FRONT_COMB_I;
    return p.lsb ? FRONT_COMB_LSB : FRONT_COMB_USB;
}

// rx_front's arguments for the launch covering frames f0 .. f0 + Nf of the call
static FrontArgs front_args(const uhsdr_rx_s* h, const int32_t* iq, int f0, float* adec, float* adec_q)
{
    FrontArgs fa;
    fa.plan = h->d_plan;
    fa.iq = (const int2*)iq + f0;
    fa.hist1 = h->hist1; fa.hist2 = h->hist2;
    fa.nb = h->Nf / h->fv->R;
    fa.cpw = FRONT_WAVE / fa.nb;
    fa.lanemap = h->d_lanemap + (h->fv->R == 16 ? 128 : 0);
    fa.lanemap2 = fa.lanemap + 64;
    fa.teta = h->teta;
    fa.tp = h->tp;
    fa.clip = h->clip;
    fa.osc_in = h->osc + 2 * (h->front_launches & 1);     // ping-pong: read one copy, write the other
    fa.osc_out = h->osc + 2 * ((h->front_launches + 1) & 1);
    fa.adec = adec ? adec + f0 / h->plan.decimation_rate : nullptr;
    fa.adec_q = adec_q ? adec_q + f0 / h->plan.decimation_rate : nullptr;
    fa.C = h->C; fa.N = h->Nf; fa.ld = h->N; fa.ldd = h->Nd;
    fa.lw = h->lw;
    fa.taps2a = h->d_taps2;
    fa.taps2b = h->d_taps2 + 2 * TAPS2_MAX;
    fa.comb = front_comb_of(h->plan);
    fa.gcnt = nullptr;
    fa.fm_prev = h->bs.sam;                          // FM: fields 0, 1 of rx_fm's state
    return fa;
}

// the back end's arguments of this call; advances the host-side per-call counters (key beep,
// CW decoder sample counter)
static BackArgs back_args(uhsdr_rx_s* h, float* adec, float* adec_q, float* audio, float* audio0, int32_t* dst)
{
    BackArgs ba;
    ba.plan = h->d_plan;
    ba.adec = adec;
    ba.adec_q = adec_q;
    ba.audio = audio;
    ba.audio0 = h->plan.stereo || h->plan.single_channel ? audio0 : nullptr;   // stereo / mcHF: a_buffer[0]
    ba.mchf = h->plan.single_channel != 0;
    ba.dst = (int2*)dst;
    ba.s = h->bs;
    ba.C = h->C; ba.N = h->N; ba.Nd = h->Nd;
    ba.ring_phase = (int)(h->calls_done % (h->bv->dm == DM_FM ? 200 : AGC_Q));   // FM: fm_data.count phase
    ba.cw_signal = h->bs.cw ? h->cw_signal : nullptr;
    ba.cw_energy = h->bs.cw ? h->cw_energy : nullptr;
    ba.cw_count0 = h->cw_count;
    ba.cw_bmax = h->cw_bmax;
    {
        const int slots = NOTCH_DELAY / (BLK / h->plan.decimation_rate);
        ba.notch_slot0 = (int)(h->calls_done % slots);
        ba.notch_first = h->calls_done == 0;
    }
    ba.tone_phase = (int)(h->calls_done % 400);
    ba.dwait = nullptr;
    ba.dtarget = 0;
    ba.spin_max = h->spin_max;
    ba.fail = h->fail_dev;
    ba.adec_next = nullptr;
    ba.dwait_next = nullptr;
    ba.dnext = 0;
    ba.fcpw = 1;
    ba.skew = h->skew;
    ba.bnd = h->bnd;
    ba.bnd_mid = h->bnd ? 6 * (BLK / h->plan.interp_L) : 0;   // (FM has no interpolator: interp_L 0)
    ba.pctl = nullptr;
    ba.pdesc = nullptr;
    ba.pdec = nullptr;
    ba.seq0 = 0;
    ba.pepoch = 0;
    {
        // key beep: frames [0, beep_n1) of this launch while calls are left (uhsdr_rx_key_beep)
        const int calls = h->N / BLK;
        const int bc = h->plan.beep_step ? (h->beep_left < calls ? h->beep_left : calls) : 0;
        ba.beep_n0 = 0;
        ba.beep_n1 = bc * BLK;
        ba.beep_acc = h->beep_acc;
        h->beep_acc += (uint32_t)ba.beep_n1 * h->plan.beep_step;
        h->beep_left -= bc;
    }
    if (h->bs.cw)
    {
        const int ndc = BLK / h->plan.decimation_rate;
        int blocks = 0;
        for (int k = 0; k < h->N / BLK; ++k)
        {
            h->cw_count += ndc;
            if (h->cw_count >= h->plan.cw_blocksize) { h->cw_count = 0; ++blocks; }
        }
        h->cw_blocks_last = blocks;
    }
    return ba;
}


// the failure word a bounded device-side poll sets when it gives up (BackArgs::fail)
static uhsdr_status check_fail(const uhsdr_rx_s* h)
{
    if (!*h->fail_host) return UHSDR_OK;
    uhsdr_set_error("the pipelined device hand-off gave up waiting for rx_front (a poll bound of %u polls): the "
                    "outputs of that call are poisoned (NaN audio) and the handle's state is invalid until "
                    "uhsdr_rx_reset", h->spin_max);
    return UHSDR_TIMEOUT;
}

static uhsdr_status rx_process(uhsdr_rx_handle h, const int32_t* iq, float* audio, float* audio0, int32_t* dst)
{
    if (!h || !iq) { uhsdr_set_error("null argument"); return UHSDR_ARGUMENT_ERROR; }
    {
        const uhsdr_status fs = check_fail(h);
        if (fs != UHSDR_OK) return fs;
    }
    if (h->timing && h->nev >= h->nev_cap) time_harvest(h);
    h->tsample = h->timing && (h->tcalls++ % h->timing) == 0;
    if (h->tsample) h->evmask[h->nev] = 0;
    const bool fma = h->precision == UHSDR_PRECISION_FMA;
    if (h->schedule == UHSDR_SCHEDULE_CHAIN)
    {
        // one kernel: front passes and back end per 64 channels, the hand-off in LDS
        // after every back end still running on the pipelined mode's side stream (state it writes)
        if (side_mode(h) && h->side_dirty)
        {
            HIPCHK(hipEventRecord(h->ev_join, h->side));
            HIPCHK(hipStreamWaitEvent(h->stream, h->ev_join, 0));
            h->side_dirty = 0;
        }
        const FrontArgs fa = front_args(h, iq, 0, nullptr, nullptr);
        const BackArgs ba = back_args(h, nullptr, nullptr, audio, audio0, dst);
        time_mark(h, K_CHAIN, 0);
        hipLaunchKernelGGL(fma ? h->cv->fn_fma : h->cv->fn, dim3((h->C + BACK_CH - 1) / BACK_CH), dim3(FRONT_WAVE),
                           chain_lds(h), h->stream, fa, ba, (int)chain_front_floats(h));
        HIPCHK(hipGetLastError());
        time_mark(h, K_CHAIN, 1);
        h->main_back = 1;
        h->front_launches += 1;
    }
    else
    {
        // hand-off buffers of this call; pipelined: rotate, and at the start of a group wait
        // until the rx_back of the group two before it (the last readers of its buffers) is done
        const long long pk = h->pipe_calls;
        const int par = h->pipelined ? (int)(pk % PIPE_BUFS) : 0;
        const int grp = (int)((pk / PIPE_GROUP) & 1);
        const bool group_end = h->pipelined && pk % PIPE_GROUP == PIPE_GROUP - 1;
        float* adec = par ? h->adecp[par - 1] : h->adec;
        float* adec_q = par ? h->adec_qp[par - 1] : h->adec_q;
        const int cpw = FRONT_WAVE / (h->Nf / h->fv->R);
        const size_t lds = front_lds(h);
        const bool side = side_mode(h);
        const bool fused = h->schedule == UHSDR_SCHEDULE_SPLIT_FUSED || h->plan.stereo;
        // device hand-off: rx_back (the wave pipeline, adec its only input from the front) polls
        // the arrival counters its group's front waves bump (FrontArgs::gcnt) instead of waiting on
        // ev_front: no barrier packet on the side stream, whose back ends then run back to back,
        // and no signal kernel between the fronts (round 5's rx_handoff_signal: ~4.7 us of the
        // handle stream per call)
        const int bgroups = (h->C + BACK_CH - 1) / BACK_CH;
        // (rx_fm measured slower with it: C4 FM 0.131-0.133 vs 0.115-0.117 ms, its 512 polling
        // workgroups beside the fronts; profiles/r05_fm_handoff_ab.txt)
        const bool dfl = side && h->dflag && !h->main_back && !fused && !h->nv && !h->fv->st &&
                         h->bv->dm == DM_NONE && bgroups <= h->dflag_grid;
        unsigned* const gc = h->gcnt + (size_t)par * bgroups * CNT_PITCH;
        // persistent back end (PersistCtl): the wave pipeline's skewed form, calls of 8+ sub-calls
        const bool pm = dfl && h->pers && h->skew && UHSDR_BACK_SKEW && h->N / BLK >= 2 * BACK_SKEW && !h->bs.cw &&
                        bgroups <= PC_MAX_GROUPS && h->bv->fn_pers;
        const unsigned seq = (unsigned)pk;
        unsigned* const pw = h->pmem;
        if (!pm && h->plive) HIPCHK(sync_all(h));     // leaving it: its launch ends, and everything completes
        if (pm && !h->pprev)
        {
            // a new run: the buffers are free once everything enqueued has completed
            HIPCHK(sync_all(h));
            // no call's decision yet (ordered before the run's first launch on the side stream)
            HIPCHK(hipMemsetAsync(h->pdec, 0xFF, sizeof(unsigned) * DESC_RING * PDEC_PITCH, h->side));
            for (int g = 0; g < bgroups; ++g) __atomic_store_n(pw + PC_CONSUMED + g, seq, __ATOMIC_SEQ_CST);
            __atomic_store_n(pw + PC_GRANT, 0u, __ATOMIC_SEQ_CST);
            __atomic_store_n(pw + PC_EXIT, seq - 2, __ATOMIC_SEQ_CST);
            __atomic_store_n(pw + PC_DECIDED, ((seq - 2) << 1) | 1u, __ATOMIC_SEQ_CST);
        }
        h->pprev = pm;
        if (pm)
        {
            // the buffer (and descriptor) of call seq - PIPE_BUFS is refilled once the back end has
            // read it: the host waits (seconds at most: a give-up still moves the word on)
            const unsigned need = seq - (PIPE_BUFS - 1);
            auto behind = [&]() {
                for (int g = 0; g < bgroups; ++g)
                    if ((int)(__atomic_load_n(pw + PC_CONSUMED + g, __ATOMIC_ACQUIRE) - need) < 0) return true;
                return false;
            };
            if (behind())
            {
                const auto t0 = std::chrono::steady_clock::now();
                while (behind())
                {
                    if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(30))
                    {
                        uhsdr_set_error("persistent back end: call %u's hand-off buffer not released within 30 s", seq);
                        return UHSDR_TIMEOUT;
                    }
                }
            }
        }
        // (Measured and dropped in round 6, profiles/r06_c2_ab_group.txt: skipping this wait when a
        // host query finds the event complete, and groups of 8 or 16 calls: no gain at 20 steps,
        // 0.0229-0.0235 vs 0.0221 ms at 1000 steps for the larger rotations)
        else if (side_mode(h) && pk % PIPE_GROUP == 0)
            HIPCHK(hipStreamWaitEvent(h->stream, h->ev_back[grp], 0));
        time_mark(h, K_FRONT, 0);
        for (int f0 = 0; f0 < h->N; f0 += h->Nf)
        {
            FrontArgs fa = front_args(h, iq, f0, adec, adec_q);
            if (dfl)
            {
                fa.gcnt = gc;
                h->fills[par] += 1;
            }
            const auto fn = fma ? h->fv->fn_fma : h->fv->fn;
            const dim3 grid((h->C + cpw - 1) / cpw), block(FRONT_WAVE);
            // pipelined: the call's last front launch records ev_front as it completes
            if (side && !dfl && f0 + h->Nf >= h->N)
                hipExtLaunchKernelGGL(fn, grid, block, lds, h->stream, nullptr, h->ev_front, 0, fa);
            else
                hipLaunchKernelGGL(fn, grid, block, lds, h->stream, fa);
            HIPCHK(hipGetLastError());
            h->front_launches += 1;
        }
        time_mark(h, K_FRONT, 1);

        // (the mcHF output stage runs inline in every back end: the wave pipeline's tail waves,
        // line_out4; round 5's finishing pass rx_line_out_mchf and its [C][N] scratch are gone)
        BackArgs bk = back_args(h, adec, adec_q, audio, audio0, dst);
        if (dfl)
        {
            bk.dwait = gc;
            bk.dtarget = h->fills[par];
            bk.fcpw = cpw;
            // BackSched: run ahead into the next call if it has arrived by then.  The next buffer
            // of the rotation is filled next by the next call only (its later reuse waits for this
            // launch: ev_back), and its counters move only with a device hand-off front -- whose
            // call's back end is then this same kernel on this stream (a mode change in between
            // joins the side stream first, so no later front starts before this launch ends).  Not
            // with the CW decoder (its per-call outputs belong to the launch's own call) or calls of
            // fewer than BACK_SKEW 32-frame blocks.
            if (UHSDR_BACK_SKEW && h->skew && h->N / BLK >= BACK_SKEW && !h->bs.cw)
            {
                const int parn = (int)((pk + 1) % PIPE_BUFS);
                bk.adec_next = parn ? h->adecp[parn - 1] : h->adec;
                bk.dwait_next = h->gcnt + (size_t)parn * bgroups * CNT_PITCH;
                bk.dnext = h->fills[parn] + (unsigned)((h->N + h->Nf - 1) / h->Nf);
            }
        }
        bool plaunch = true;
        if (pm)
        {
            // the call's descriptor, then its grant; a running launch takes it unless it is closing
            // after the previous call (PC_EXIT): then its decision tells (PersistCtl)
            BackDesc* d = (BackDesc*)(pw + PC_WORDS) + seq % DESC_RING;
            d->adec = adec;
            d->cnt = gc;
            d->audio = bk.audio;
            d->audio0 = bk.audio0;
            d->dst = bk.dst;
            d->target = h->fills[par];
            d->beep_n0 = bk.beep_n0;
            d->beep_n1 = bk.beep_n1;
            d->beep_acc = bk.beep_acc;
            __atomic_store_n(&d->seq, seq, __ATOMIC_RELEASE);
            auto grant = [&]() { return h->pepoch << 24 | (seq & 0xFFFFFFu); };
            if (h->plive)
            {
                __atomic_store_n(pw + PC_GRANT, grant(), __ATOMIC_SEQ_CST);
                plaunch = false;
                if (__atomic_load_n(pw + PC_EXIT, __ATOMIC_SEQ_CST) == seq - 1)
                {
                    const unsigned want = (seq - 1) & 0x7FFFFFFFu;
                    const auto t0 = std::chrono::steady_clock::now();
                    unsigned dv;
                    while (((dv = __atomic_load_n(pw + PC_DECIDED, __ATOMIC_ACQUIRE)) >> 1) != want)
                    {
                        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(30))
                        {
                            uhsdr_set_error("persistent back end: no decision after call %u within 30 s", seq - 1);
                            return UHSDR_TIMEOUT;
                        }
                    }
                    plaunch = dv & 1u;               // it closed: a new launch takes this call
                }
            }
            h->plast = seq;
            if (plaunch)
            {
                // a new launch, of the next epoch: grants of the old one's epoch no longer reach it
                h->pepoch = (h->pepoch + 1) & 0xFFu;
                __atomic_store_n(pw + PC_GRANT, grant(), __ATOMIC_SEQ_CST);
                bk.pepoch = h->pepoch;
                bk.pctl = h->pmem_dev;
                bk.pdesc = (const BackDesc*)(h->pmem_dev + PC_WORDS);
                bk.pdec = h->pdec;
                bk.seq0 = seq;
                bk.adec_next = nullptr;
                bk.dwait_next = nullptr;
                h->plive = 1;
                h->plaunches += 1;
            }
        }
        const hipStream_t bst = back_stream(h);
        if (side && !dfl) HIPCHK(hipStreamWaitEvent(bst, h->ev_front, 0));
        time_mark(h, K_BACK, 0);
        if (h->nv)
        {
            hipLaunchKernelGGL(h->nv->fn, dim3((h->C + BACK_CH - 1) / BACK_CH), dim3(BACK_CH), 0, bst, bk);
            HIPCHK(hipGetLastError());
        }
        const back_fn bfn = fused ? fused_back_fn(h) : pm ? h->bv->fn_pers : h->bv->fn;
        // (the wave pipeline: its role waves and BACK_TAILS tail waves; rx_fm: its two; the fused kernels: one)
        const int bwaves = fused ? 1 : h->bv->dm == DM_FM ? back_roles(DM_FM) : back_roles(h->bv->dm) + back_tails(h->bv->dm);
        const dim3 bgrid((h->C + BACK_CH - 1) / BACK_CH), bblock(bwaves * BACK_CH);
#ifndef UHSDR_FUSED_LDS_PAD
#define UHSDR_FUSED_LDS_PAD 0
#endif
#ifndef UHSDR_BACK_RESERVE
#define UHSDR_BACK_RESERVE 1
#endif
        // (UHSDR_FUSED_LDS_PAD: unused dynamic LDS per fused workgroup, an occupancy cap for A/B)
        size_t blds = fused ? (size_t)UHSDR_FUSED_LDS_PAD : back_lds(h);
        // device hand-off: rx_back takes nearly all of a CU's LDS, so no rx_front workgroup of the
        // next calls shares its SIMDs (the role waves are latency-bound; a front wave beside them
        // stretches every step).  At most half the CUs (dflag_grid); C2 0.0263 -> 0.0257 ms at
        // 1000 steps, 20 steps unchanged (profiles/r05_c2_back_reserve_ab.txt)
        if (UHSDR_BACK_RESERVE && dfl)
        {
            if (!h->back_attr)
            {
                h->back_attr = hipFuncSetAttribute((const void*)h->bv->fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                                   (int)LDS_PER_CU) == hipSuccess ? 1 : -1;
                if (h->back_attr > 0 && h->bv->fn_pers &&
                    hipFuncSetAttribute((const void*)h->bv->fn_pers, hipFuncAttributeMaxDynamicSharedMemorySize,
                                        (int)LDS_PER_CU) != hipSuccess)
                    h->back_attr = -1;
                (void)hipGetLastError();
            }
            if (h->back_attr > 0) blds = LDS_PER_CU - 4096;
        }
        // pipelined: the group's last rx_back records ev_back[grp] as it completes (the persistent
        // back end: a launch only to start a run of calls; the buffers' reuse waits on PC_CONSUMED)
        if (pm)
        {
            if (plaunch) hipLaunchKernelGGL(bfn, bgrid, bblock, blds, bst, bk);
        }
        else if (side && group_end)
            hipExtLaunchKernelGGL(bfn, bgrid, bblock, blds, bst, nullptr, h->ev_back[grp], 0, bk);
        else
            hipLaunchKernelGGL(bfn, bgrid, bblock, blds, bst, bk);
        HIPCHK(hipGetLastError());
        time_mark(h, K_BACK, 1);
        if (h->pipelined) h->pipe_calls += 1;
        if (side) h->side_dirty = 1;
        h->main_back = !side;
    }
    h->calls_issued += 1;
    if (h->tsample) h->nev++;
    h->tsample = 0;
    h->dec_samples += h->Nd;
    h->calls_done += h->N / BLK;
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
    if (st == UHSDR_OK) st = uhsdr_rx_join(h);
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

extern "C" uhsdr_status uhsdr_rx_synchronize(uhsdr_rx_handle h)
{
    if (!h) return UHSDR_ARGUMENT_ERROR;
    HIPCHK(sync_all(h));
    return check_fail(h);
}

extern "C" uhsdr_status uhsdr_rx_set_precision(uhsdr_rx_handle h, int32_t precision)
{
    if (!h) return UHSDR_ARGUMENT_ERROR;
    if (precision != UHSDR_PRECISION_EXACT && precision != UHSDR_PRECISION_FMA)
    {
        uhsdr_set_error("unknown precision %d", (int)precision);
        return UHSDR_ARGUMENT_ERROR;
    }
    if (precision == UHSDR_PRECISION_FMA && !uhsdr_rx_plan_fma_ok(&h->plan))
    {
        uhsdr_set_error("FMA precision not within 1e-5 on filter path %d, demodulator %d%s: EXACT only",
                        (int)h->plan.filter_path, (int)h->plan.dmod_mode, h->plan.stereo ? " (stereo)" : "");
        return UHSDR_UNSUPPORTED;
    }
    h->precision = precision;
    return UHSDR_OK;
}

extern "C" int32_t uhsdr_rx_get_precision(uhsdr_rx_handle h) { return h ? h->precision : -1; }

extern "C" uhsdr_status uhsdr_rx_set_schedule(uhsdr_rx_handle h, int32_t schedule)
{
    if (!h) return UHSDR_ARGUMENT_ERROR;
    if (schedule < UHSDR_SCHEDULE_AUTO || schedule > UHSDR_SCHEDULE_CHAIN)
    {
        uhsdr_set_error("schedule %d: not a UHSDR_SCHEDULE_*", (int)schedule);
        return UHSDR_ARGUMENT_ERROR;
    }
    const int s = resolve_schedule(h, schedule);
    if (s < 0)
    {
        uhsdr_set_error("schedule %d not available on filter path %d with %d-frame calls", (int)schedule,
                        (int)h->plan.filter_path, h->N);
        return UHSDR_UNSUPPORTED;
    }
    h->schedule = s;
    return UHSDR_OK;
}

extern "C" int32_t uhsdr_rx_get_schedule(uhsdr_rx_handle h) { return h ? h->schedule : -1; }

extern "C" int32_t uhsdr_rx_handoff_timeouts(uhsdr_rx_handle h)
{
    if (!h || sync_all(h) != hipSuccess) return -1;
    return (int32_t)*h->fail_host;
}

extern "C" uhsdr_status uhsdr_rx_set_handoff_bound(uhsdr_rx_handle h, uint32_t polls)
{
    if (!h) return UHSDR_ARGUMENT_ERROR;
    if (polls == 0) { uhsdr_set_error("handoff bound: at least one poll"); return UHSDR_ARGUMENT_ERROR; }
    h->spin_max = polls;
    return UHSDR_OK;
}

extern "C" uhsdr_status uhsdr_rx_set_front_block(uhsdr_rx_handle h, int32_t outputs_per_lane)
{
    if (!h) return UHSDR_ARGUMENT_ERROR;
    if (outputs_per_lane != 8 && outputs_per_lane != 16)
    {
        uhsdr_set_error("front block %d: 8 or 16 outputs per lane", (int)outputs_per_lane);
        return UHSDR_ARGUMENT_ERROR;
    }
    const uhsdr_status st = configure_front(h, outputs_per_lane, true);
    if (st != UHSDR_OK) return st;
    // a CHAIN schedule needs the chain's block: fall back to the split kernels otherwise
    if (h->schedule == UHSDR_SCHEDULE_CHAIN && !chain_ok(h))
        h->schedule = h->bv->fused ? UHSDR_SCHEDULE_SPLIT_FUSED : UHSDR_SCHEDULE_SPLIT_PIPE;
    return UHSDR_OK;
}

// test hook: the persistent back end's control words (PC_GRANT, the epoch, PC_EXIT, PC_DECIDED,
// PC_CONSUMED) and the host's plive / plast / plaunches
extern "C" uhsdr_status uhsdr_rx_debug_persist(uhsdr_rx_handle h, uint32_t* out)
{
    if (!h || !out) return UHSDR_ARGUMENT_ERROR;
    if (!h->pmem) return UHSDR_UNSUPPORTED;
    const int w[5] = { PC_GRANT, -1, PC_EXIT, PC_DECIDED, PC_CONSUMED };
    for (int i = 0; i < 5; ++i) out[i] = w[i] < 0 ? h->pepoch : __atomic_load_n(h->pmem + w[i], __ATOMIC_SEQ_CST);   // (group 0's PC_CONSUMED)
    out[5] = (uint32_t)h->plive;
    out[6] = h->plast;
    out[7] = h->plaunches;
    return UHSDR_OK;
}

extern "C" uhsdr_status uhsdr_rx_join(uhsdr_rx_handle h)
{
    if (!h) return UHSDR_ARGUMENT_ERROR;
    pers_close(h);                                     // the persistent back end ends after the last call
    if (side_mode(h))
    {
        HIPCHK(hipEventRecord(h->ev_join, h->side));
        HIPCHK(hipStreamWaitEvent(h->stream, h->ev_join, 0));
    }
    return check_fail(h);
}

extern "C" uhsdr_status uhsdr_rx_set_pipelined(uhsdr_rx_handle h, int32_t enable)
{
    if (!h) return UHSDR_ARGUMENT_ERROR;
    if (enable < 0 || enable > 3)
    {
        uhsdr_set_error("pipelined mode %d: 0 (off), 1 (event hand-off), 2 (device hand-off) or 3 (persistent "
                        "back end)", (int)enable);
        return UHSDR_ARGUMENT_ERROR;
    }
    if (enable == 3 && !h->pmem)
    {
        HIPCHK(hipHostMalloc((void**)&h->pmem, PC_BYTES, hipHostMallocCoherent | hipHostMallocMapped));
        memset(h->pmem, 0, PC_BYTES);
        HIPCHK(hipHostGetDevicePointer((void**)&h->pmem_dev, h->pmem, 0));
        HIPCHK(hipMalloc((void**)&h->pdec, sizeof(unsigned) * DESC_RING * PDEC_PITCH));
    }
    // into or out of the persistent back end: everything enqueued completes first
    if ((enable == 3) != (h->pers != 0)) HIPCHK(sync_all(h));
    if (enable && !h->side)
    {
        const size_t nd = (size_t)h->C * h->Nd;
        HIPCHK(hipStreamCreateWithFlags(&h->side, hipStreamNonBlocking));
        // ev_front / ev_back are recorded by hipExtLaunchKernel as their kernels complete
        HIPCHK(hipEventCreate(&h->ev_front));
        HIPCHK(hipEventCreateWithFlags(&h->ev_join, hipEventDisableTiming));
        for (int i = 0; i < 2; ++i) HIPCHK(hipEventCreate(&h->ev_back[i]));
        for (int i = 0; i < PIPE_BUFS - 1; ++i)
        {
            HIPCHK(hipMalloc((void**)&h->adecp[i], sizeof(float) * nd));
            if (h->adec_q) HIPCHK(hipMalloc((void**)&h->adec_qp[i], sizeof(float) * nd));
        }
    }
    if (h->timing) time_harvest(h);
    // leaving the mode: the side stream's work completes before the handle stream goes on
    if (!enable && h->pipelined)
    {
        const uhsdr_status st = uhsdr_rx_join(h);
        if (st != UHSDR_OK) return st;
    }
    if (enable && !h->pipelined)
    {
        // entering it: the side stream starts after the handle stream's work (the state the first
        // rx_back reads), and both group events start out complete
        HIPCHK(hipEventRecord(h->ev_join, h->stream));
        HIPCHK(hipStreamWaitEvent(h->side, h->ev_join, 0));
        for (int i = 0; i < 2; ++i) HIPCHK(hipEventRecord(h->ev_back[i], h->side));
        h->pipe_calls = 0;
    }
    h->pipelined = enable != 0;
    h->dflag = enable >= 2;
    h->pers = enable == 3;
    h->pprev = 0;
    if (h->dflag && !h->dflag_grid)
    {
        int dev = 0, cus = 0;
        if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess)
            h->dflag_grid = cus / 2;
    }
    return UHSDR_OK;
}

extern "C" void* uhsdr_device_alloc(uint64_t bytes)
{
    void* p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) { uhsdr_set_error("hipMalloc(%llu) failed", (unsigned long long)bytes); return nullptr; }
    return p;
}

extern "C" void uhsdr_device_free(void* p) { if (p) (void)hipFree(p); }

extern "C" uhsdr_status uhsdr_copy_to_device(void* dst, const void* src, uint64_t bytes)
{
    if (!dst || !src) return UHSDR_ARGUMENT_ERROR;
    HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
    return UHSDR_OK;
}

extern "C" uhsdr_status uhsdr_copy_to_host(void* dst, const void* src, uint64_t bytes)
{
    if (!dst || !src) return UHSDR_ARGUMENT_ERROR;
    HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
    return UHSDR_OK;
}

extern "C" uhsdr_status uhsdr_rx_get_plan(uhsdr_rx_handle h, uhsdr_rx_plan* plan)
{
    if (!h || !plan) return UHSDR_ARGUMENT_ERROR;
    memcpy(plan, &h->plan, sizeof *plan);
    return UHSDR_OK;
}

extern "C" int32_t uhsdr_rx_kernel_count(uhsdr_rx_handle h) { return h ? NKERN : 0; }

extern "C" uhsdr_status uhsdr_rx_enable_timing(uhsdr_rx_handle h, int32_t enable)
{
    if (!h) return UHSDR_ARGUMENT_ERROR;
    if (enable && !h->ev)
    {
        h->nev_cap = 1024;
        h->ev = (hipEvent_t*)calloc((size_t)h->nev_cap * NKERN * 2, sizeof(hipEvent_t));
        h->evmask = (uint8_t*)calloc((size_t)h->nev_cap, 1);
        for (int i = 0; i < h->nev_cap * NKERN * 2; ++i) HIPCHK(hipEventCreate(&h->ev[i]));
    }
    if (h->timing) time_harvest(h);
    h->timing = enable > 0 ? enable : 0;
    h->tsample = 0;
    h->tcalls = 0;
    h->nev = 0;
    for (int k = 0; k < NKERN; ++k) { h->total_ms[k] = 0.0f; h->launches[k] = 0; }
    return UHSDR_OK;
}

extern "C" int32_t uhsdr_rx_kernel_times(uhsdr_rx_handle h, float* total_ms, int32_t* launches, int32_t max_kernels)
{
    if (!h) return 0;
    time_harvest(h);
    const int n = max_kernels < NKERN ? max_kernels : NKERN;
    for (int k = 0; k < n; ++k)
    {
        if (total_ms) total_ms[k] = h->total_ms[k];
        if (launches) launches[k] = h->launches[k];
    }
    return n;
}

extern "C" const char* uhsdr_rx_kernel_name(int32_t index) { return (index >= 0 && index < NKERN) ? kKernelNames[index] : ""; }

extern "C" uhsdr_status uhsdr_rx_destroy(uhsdr_rx_handle h)
{
    if (!h) return UHSDR_ARGUMENT_ERROR;
    (void)sync_all(h);
    if (h->side)
    {
        (void)hipEventDestroy(h->ev_front);
        (void)hipEventDestroy(h->ev_join);
        for (int i = 0; i < 2; ++i) (void)hipEventDestroy(h->ev_back[i]);
        (void)hipStreamDestroy(h->side);
        for (int i = 0; i < PIPE_BUFS - 1; ++i)
        {
            (void)hipFree(h->adecp[i]);
            if (h->adec_qp[i]) (void)hipFree(h->adec_qp[i]);
        }
    }
    if (h->ev)
    {
        for (int i = 0; i < h->nev_cap * NKERN * 2; ++i) (void)hipEventDestroy(h->ev[i]);
        free(h->ev);
        free(h->evmask);
    }
    if (h->ev_switch) (void)hipEventDestroy(h->ev_switch);
    if (h->arena) (void)hipFree(h->arena);
    if (h->adec) (void)hipFree(h->adec);
    if (h->d_plan) (void)hipFree(h->d_plan);
    if (h->d_taps2) (void)hipFree(h->d_taps2);
    if (h->d_lanemap) (void)hipFree(h->d_lanemap);
    if (h->gcnt) (void)hipFree(h->gcnt);
    if (h->fail_host) (void)hipHostFree((void*)h->fail_host);
    if (h->pmem) (void)hipHostFree(h->pmem);
    if (h->pdec) (void)hipFree(h->pdec);
    free(h);
    return UHSDR_OK;
}
