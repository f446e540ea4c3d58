// MI355X (gfx950) SSB transmit chain of the UHSDR firmware, batched over channels.
//
// One uhsdr_tx_process() call == N/32 consecutive TX-mode AudioDriver_I2SCallback invocations
// (drivers/audio/audio_driver.c:3010-3036 -> TxProcessor_Run, drivers/audio/tx_processor.c:891-1078)
// on each of C independent channels.  Two kernels:
//
//  tx_voice  (sequential per channel: lane == channel)
//      codec frame -> f32, mic gain                     tx_processor.c:339-405
//      TX band-pass lattice, bass/treble biquads        :416-429
//      ALC compressor + 9-call look-ahead delay         :173-242
//    -> compressed audio txa[C][N] (= adb.a_buffer[0]) in HBM; delay ring [10][32][C] in HBM
//
//  tx_iq     (time-parallel within a channel, the rx_front scheme)
//      201-tap Hilbert pair (one LDS window, two FIR blocks)   :467-483
//      FreqShift (Fs/4 exchange or recursive oscillator)       :484-487, freq_shift.c:219-334
//      I/Q gain + phase, float -> int32 DAC frames             :282-330
//
// Arithmetic: the reference's binary32 operation sequence (-ffp-contract=off): outputs are
// bit-identical to the firmware built for x86 (tests/test_gpu_tx.py).

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
#include <math.h>
#include "uhsdr_internal.h"
#include "uhsdr_dsp.h"

#define TX_DELAY_SLOTS (UHSDR_TX_DELAY / BLK)   // 10 blocks of 32
#define TX_T UHSDR_TX_HILBERT_TAPS

struct TxVoiceArgs
{
    const uhsdr_tx_plan* plan;
    const int2* audio;      // [C][N] codec frames {l, r}
    float* txa;             // [C][N] compressed audio out
    float* a0;              // optional copy of txa for the caller (adb.a_buffer[0])
    float* lat;             // [10][C]
    float* bq;              // [12][C]
    float* alc;             // [C]
    float* delay;           // [10][32][C]
    uint32_t* fm;           // FM: [4][C] hpf_prev_a, hpf_prev_b (f32 bits), fm_mod_accum, sub-audible dds acc
    int2* iq;               // FM: DAC frames [C][N] written here (no tx_iq)
    int C, N;
    int delay_phase;        // alc_delay_inbuf / 32 before this launch
    // softdds tones common to all channels (accumulators at frame 0 of this launch):
    // tune 0 off, 1 single (dbldds[0]), 2 two-tone (dbldds[0] + [1]); burst: FM tone burst on
    int tune, burst;
    uint32_t tune_acc0, tune_acc1, burst_acc;
};

// softdds_runIQ(a, a, n) (softdds.c:152-163): with both outputs in one buffer the quadrature
// sample, written second, stays -- DDS_TABLE[k + 768] single, or the two-tone integer mean
__device__ __forceinline__ float tune_tone(const TxVoiceArgs& a, const uhsdr_tx_plan* __restrict__ P, int n)
{
    const uint32_t k0 = ((a.tune_acc0 + (uint32_t)n * P->tune_step[0]) >> 22) % 1024u;
    const int q0 = P->dds_table[(k0 + 768u) % 1024u];
    if (a.tune == 1) return (float)q0;
    const uint32_t k1 = ((a.tune_acc1 + (uint32_t)n * P->tune_step[1]) >> 22) % 1024u;
    return (float)((q0 + (int)P->dds_table[(k1 + 768u) % 1024u]) / 2);
}

__device__ __forceinline__ int tx_to_int32(float f)
{
    return (f > -2147483904.0f && f < 2147483648.0f) ? (int)f : INT32_MIN;
}

// The ALC's double-precision steps that binary32 reproduces exactly (exhaustive over all binary32
// inputs, tools/alc_check.c): (float)((double)q - 1.0) is q - 1.0f, and (double)a < 0.001 is
// a < 0.001f; the 0.1 attack step stays in double.
// x / 30000 in binary32 (ALC_KNEE, tx_processor.c:202) without the IEEE division sequence:
// q0 = x * (1/30000) and one FMA residual correction give the correctly rounded quotient for
// every normal quotient (exhaustive over all binary32 x: tools/div_check.c); tiny, huge, inf and
// NaN inputs take the division itself
__device__ __forceinline__ float alc_knee_div(float x)
{
    constexpr float y = 30000.0f, z = 1.0f / 30000.0f;
    const float q0 = x * z;
    float q = __builtin_fmaf(__builtin_fmaf(-q0, y, x), z, q0);
    if (!(x >= 0x1.0p-100f && x <= 0x1.0p+127f)) q = x / y;
    return q;
}

// TxProcessor_AudioBufferFill + _FilterAudio + _VoiceCompressor, one lane per channel; with FM
// also TxProcessor_FM (tx_processor.c:534-588) and TxProcessor_IqFinalProcessing (:282-330)
template <int S, bool FM>
__global__ void __launch_bounds__(64) tx_voice(TxVoiceArgs a)
{
    // raised issue priority: in the pipelined mode tx_iq of the previous call shares these SIMDs,
    // and this one-lane-per-channel recursion is the call's critical path
    __builtin_amdgcn_s_setprio(3);
    const uhsdr_tx_plan* __restrict__ P = a.plan;
    const int c = blockIdx.x * 64 + threadIdx.x;
    const bool live = c < a.C;
    const int cl = live ? c : a.C - 1;
    const int C = a.C;
    float lk[S], lv[S + 1], g[S], bc[15], bq[12];
#pragma unroll
    for (int i = 0; i < S; ++i) lk[i] = P->lat_k[i];
#pragma unroll
    for (int i = 0; i <= S; ++i) lv[i] = P->lat_v[i];
#pragma unroll
    for (int i = 0; i < 15; ++i) bc[i] = P->biquad[i];
#pragma unroll
    for (int i = 0; i < S; ++i) g[i] = a.lat[i * C + cl];
#pragma unroll
    for (int i = 0; i < 12; ++i) bq[i] = a.bq[i * C + cl];
    float alc_val = a.alc[cl];
    const bool right = P->audio_source == UHSDR_TX_AUDIO_LINEIN_R;
    // TUNE: the tone replaces the input, no gain, no filters, no post-filter gain (tx_processor.c:344,444,179)
    const bool tune = a.tune != 0;
    const bool apply_gain = P->apply_in_gain && !tune, run_lat = P->run_lattice && !tune, run_bq = P->run_biquad && !tune;
    const bool comp = P->comp_on;
    const float in_gain = P->in_gain, post = P->postfilt_gain, decay = P->alc_decay, gscale = P->alc_gain_scaling;
    const int calls = a.N / BLK;
    float hpf_a = 0.0f, hpf_b = 0.0f;
    uint32_t fm_acc = 0, sub_acc = 0;
    if constexpr (FM)
    {
        hpf_a = __uint_as_float(a.fm[cl]); hpf_b = __uint_as_float(a.fm[C + cl]);
        fm_acc = a.fm[2 * C + cl]; sub_acc = a.fm[3 * C + cl];
    }
    for (int k = 0; k < calls; ++k)
    {
        float x[BLK];
        const int4* src = (const int4*)(a.audio + (size_t)cl * a.N + k * BLK);
#pragma unroll
        for (int j = 0; j < BLK / 2; ++j)
        {
            const int4 v = src[j];
            x[2 * j] = (float)(right ? v.y : v.x);
            x[2 * j + 1] = (float)(right ? v.w : v.z);
        }
        if (tune)
        {
#pragma unroll
            for (int m = 0; m < BLK; ++m) x[m] = tune_tone(a, P, k * BLK + m);
        }
        const int slot_in = (a.delay_phase + k + 1) % TX_DELAY_SLOTS;   // alc_delay_inbuf after += 32
        const int slot_out = (a.delay_phase + k + 2) % TX_DELAY_SLOTS;  // alc_delay_outbuf
        float dly[BLK];
        if (comp)
        {
            const float* dr = a.delay + ((size_t)slot_out * BLK) * C + cl;
#pragma unroll
            for (int m = 0; m < BLK; ++m) dly[m] = dr[(size_t)m * C];
        }
#pragma unroll
        for (int m = 0; m < BLK; ++m)
        {
            float v = x[m];
            if (apply_gain) v = v * in_gain;
            // the packed lattice (uhsdr_dsp.h), pairing by the sample's parity
            if (run_lat) v = (m & 1) ? lattice_step_pk<S, 1>(v, g, lk, lv) : lattice_step_pk<S, 0>(v, g, lk, lv);
            if (run_bq)
            {
#pragma unroll
                for (int st = 0; st < 3; ++st)
                    v = biquad_step(v, bq[4 * st], bq[4 * st + 1], bq[4 * st + 2], bq[4 * st + 3], bc + 5 * st);
            }
            x[m] = v;
        }
        if (comp)
        {
            float* dw = a.delay + ((size_t)slot_in * BLK) * C + c;
#pragma unroll
            for (int m = 0; m < BLK; ++m)
            {
                const float v = tune ? x[m] : x[m] * post;
                // ALC (tx_processor.c:197-221)
                const float alc_var = alc_knee_div(fabsf(v * alc_val)) - 1.0f;   // == (float)((double)q - 1.0)
                // both branches evaluated and selected: lanes of a wave no longer split
                const float dec = alc_val - alc_val * decay * alc_var;
                float att = (float)((double)alc_val - (double)alc_val * 0.1 * (double)alc_var);
                att = (att < 0.001f) ? 0.001f : att;                 // == (double)att < 0.001
                alc_val = (alc_var < 0) ? dec : att;
                if (alc_val > 1) alc_val = 1;
                if (live) dw[(size_t)m * C] = v;                        // into the delay buffer
                x[m] = dly[m] * (alc_val * gscale);                     // delayed audio x ALC gain
            }
        }
        if (live)
        {
            float* d0 = a.a0 ? a.a0 + (size_t)c * a.N + k * BLK : nullptr;
            float* dst = FM ? nullptr : a.txa + (size_t)c * a.N + k * BLK;
#pragma unroll
            for (int m = 0; m < BLK; m += 4)
            {
                const float4 v = make_float4(x[m], x[m + 1], x[m + 2], x[m + 3]);
                if (!FM) *(float4*)(dst + m) = v;
                if (d0) *(float4*)(d0 + m) = v;
            }
        }
        if constexpr (FM)
        {
            const int16_t* __restrict__ dds = P->dds_table;
            // the sub-audible tone pauses during a tone burst (tx_processor.c:555-564)
            const bool sub = P->fm_sub_on && !a.burst, swap = P->fm_swap;
            const bool burst = a.burst != 0;
            const float burst_scale = P->tone_burst_scale;
            const float mult = P->fm_mod_mult, sub_scale = P->fm_sub_scale;
            const uint32_t word = P->fm_word, step = P->fm_sub_step;
            const float gi = P->final_i_gain, gq = P->final_q_gain, ph = P->phase_balance;
            int out[2 * BLK];
#pragma unroll
            for (int m = 0; m < BLK; ++m)
            {
                const float av = x[m];
                hpf_b = (float)(0.05 * (double)(hpf_b + av - hpf_a));    // FM_TX_HPF_ALPHA pre-emphasis
                hpf_a = av;
                float a1 = hpf_b;
                if (sub)
                {
                    // softdds_addSingleTone (softdds.c:113-119): index (acc >> 22) % 1024, then acc += step
                    const uint32_t idx = (sub_acc >> 22) % 1024u;
                    sub_acc += step;
                    a1 += (float)dds[idx] * sub_scale;
                }
                if (burst)
                {
                    const uint32_t idx = ((a.burst_acc + (uint32_t)(k * BLK + m) * P->tone_burst_step) >> 22) % 1024u;
                    a1 += (float)dds[idx] * burst_scale;
                }
                // fm_mod_accum += word + a1 * FM_MOD_SCALING * mult; as on x86, the float sum is
                // truncated through a 64-bit integer (cvttss2si) into the uint32 accumulator
                const float t = word + (a1 * 16 * mult);
                const float sum = (float)fm_acc + t;
                fm_acc = (uint32_t)(long long)sum;
                fm_acc %= 65536u;
                const uint32_t idx = fm_acc >> 6;                            // FM_MOD_DDS_ACC_SHIFT
                const float vi = dds[idx], vq = dds[(idx + 768u) % 1024u];
                float I = swap ? vq : vi, Q = swap ? vi : vq;
                I = I * gi;
                Q = Q * gq;
                if (ph < 0) { const float e = I * ph; Q = Q + e; }
                else if (ph > 0) { const float e = Q * ph; I = I + e; }
                out[2 * m] = tx_to_int32(I);
                out[2 * m + 1] = tx_to_int32(Q);
            }
            if (live)
            {
                int4* dq = (int4*)(a.iq + (size_t)c * a.N + k * BLK);
#pragma unroll
                for (int j = 0; j < BLK / 2; ++j) dq[j] = make_int4(out[4 * j], out[4 * j + 1], out[4 * j + 2], out[4 * j + 3]);
            }
        }
    }
    if (FM && live)
    {
        a.fm[c] = __float_as_uint(hpf_a); a.fm[C + c] = __float_as_uint(hpf_b);
        a.fm[2 * C + c] = fm_acc; a.fm[3 * C + c] = sub_acc;
    }
    if (live)
    {
#pragma unroll
        for (int i = 0; i < S; ++i) a.lat[i * C + c] = g[i];
#pragma unroll
        for (int i = 0; i < 12; ++i) a.bq[i * C + c] = bq[i];
        a.alc[c] = alc_val;
    }
}

// tx_voice for SSB / AM as a two-wave pipeline over the launch's 32-frame calls (the RX back end's
// scheme): wave 0 runs the input (codec frame / TUNE tone), the mic gain and the TX band-pass
// lattice of call s while wave 1 runs the three biquads, the ALC with its look-ahead delay and
// the stores of call s - 1; the call's 32 samples per channel cross in LDS (double-buffered,
// 65-float pitch), one LDS-only barrier per call.  Per lane the same operations on the same
// operands in the same order as tx_voice: bit-identical.  Two waves per 64 channels halve the
// per-call critical path of this one-lane-per-channel recursion.
constexpr int TXV_PITCH = 65;
template <int S>
__global__ void __launch_bounds__(128) tx_voice2(TxVoiceArgs a)
{
    __builtin_amdgcn_s_setprio(3);
    __shared__ float hand[2][BLK * TXV_PITCH];
    const uhsdr_tx_plan* __restrict__ P = a.plan;
    const int role = __builtin_amdgcn_readfirstlane(threadIdx.x / 64);
    const int lane = threadIdx.x & 63;
    const int c = blockIdx.x * 64 + lane;
    const bool live = c < a.C;
    const int cl = live ? c : a.C - 1;
    const int C = a.C;
    const int calls = a.N / BLK;
    const bool tune = a.tune != 0;
    if (role == 0)
    {
        float lk[S], lv[S + 1], g[S];
#pragma unroll
        for (int i = 0; i < S; ++i) lk[i] = P->lat_k[i];
#pragma unroll
        for (int i = 0; i <= S; ++i) lv[i] = P->lat_v[i];
#pragma unroll
        for (int i = 0; i < S; ++i) g[i] = a.lat[i * C + cl];
        const bool right = P->audio_source == UHSDR_TX_AUDIO_LINEIN_R;
        const bool apply_gain = P->apply_in_gain && !tune, run_lat = P->run_lattice && !tune;
        const float in_gain = P->in_gain;
        const int4* src = (const int4*)(a.audio + (size_t)cl * a.N);
        int4 nxt[BLK / 2];
#pragma unroll
        for (int j = 0; j < BLK / 2; ++j) nxt[j] = src[j];
        for (int k = 0; k < calls; ++k)
        {
            float x[BLK];
#pragma unroll
            for (int j = 0; j < BLK / 2; ++j)
            {
                const int4 v = nxt[j];
                x[2 * j] = (float)(right ? v.y : v.x);
                x[2 * j + 1] = (float)(right ? v.w : v.z);
            }
            if (k + 1 < calls)
            {
#pragma unroll
                for (int j = 0; j < BLK / 2; ++j) nxt[j] = src[(k + 1) * (BLK / 2) + j];
            }
            if (tune)
            {
#pragma unroll
                for (int m = 0; m < BLK; ++m) x[m] = tune_tone(a, P, k * BLK + m);
            }
            float* hb = hand[k & 1] + lane;
#pragma unroll
            for (int m = 0; m < BLK; ++m)
            {
                float v = x[m];
                if (apply_gain) v = v * in_gain;
                if (run_lat) v = (m & 1) ? lattice_step_pk<S, 1>(v, g, lk, lv) : lattice_step_pk<S, 0>(v, g, lk, lv);
                hb[m * TXV_PITCH] = v;
            }
            lds_barrier();
        }
        if (live)
        {
#pragma unroll
            for (int i = 0; i < S; ++i) a.lat[i * C + c] = g[i];
        }
        return;
    }
    float bc[15], bq[12];
#pragma unroll
    for (int i = 0; i < 15; ++i) bc[i] = P->biquad[i];
#pragma unroll
    for (int i = 0; i < 12; ++i) bq[i] = a.bq[i * C + cl];
    float alc_val = a.alc[cl];
    const bool run_bq = P->run_biquad && !tune;
    const bool comp = P->comp_on;
    const float post = P->postfilt_gain, decay = P->alc_decay, gscale = P->alc_gain_scaling;
    float dnext[BLK];
    if (comp)
    {
        const float* dr = a.delay + ((size_t)((a.delay_phase + 2) % TX_DELAY_SLOTS) * BLK) * C + cl;
#pragma unroll
        for (int m = 0; m < BLK; ++m) dnext[m] = dr[(size_t)m * C];
    }
    for (int k = 0; k < calls; ++k)
    {
        float dly[BLK];
#pragma unroll
        for (int m = 0; m < BLK; ++m) dly[m] = dnext[m];
        const int slot_in = (a.delay_phase + k + 1) % TX_DELAY_SLOTS;   // alc_delay_inbuf after += 32
        if (comp && k + 1 < calls)
        {
            // the next call's delayed samples: its slot_out (k + 3) is not this call's slot_in (k + 1)
            const float* dr = a.delay + ((size_t)((a.delay_phase + k + 3) % TX_DELAY_SLOTS) * BLK) * C + cl;
#pragma unroll
            for (int m = 0; m < BLK; ++m) dnext[m] = dr[(size_t)m * C];
        }
        lds_barrier();
        float x[BLK];
        const float* hb = hand[k & 1] + lane;
#pragma unroll
        for (int m = 0; m < BLK; ++m) x[m] = hb[m * TXV_PITCH];
        if (run_bq)
        {
#pragma unroll
            for (int m = 0; m < BLK; ++m)
            {
                float v = x[m];
#pragma unroll
                for (int st = 0; st < 3; ++st)
                    v = biquad_step(v, bq[4 * st], bq[4 * st + 1], bq[4 * st + 2], bq[4 * st + 3], bc + 5 * st);
                x[m] = v;
            }
        }
        if (comp)
        {
            float* dw = a.delay + ((size_t)slot_in * BLK) * C + c;
#pragma unroll
            for (int m = 0; m < BLK; ++m)
            {
                const float v = tune ? x[m] : x[m] * post;
                const float alc_var = alc_knee_div(fabsf(v * alc_val)) - 1.0f;   // == (float)((double)q - 1.0)
                const float dec = alc_val - alc_val * decay * alc_var;
                float att = (float)((double)alc_val - (double)alc_val * 0.1 * (double)alc_var);
                att = (att < 0.001f) ? 0.001f : att;                 // == (double)att < 0.001
                alc_val = (alc_var < 0) ? dec : att;
                if (alc_val > 1) alc_val = 1;
                if (live) dw[(size_t)m * C] = v;
                x[m] = dly[m] * (alc_val * gscale);
            }
        }
        if (live)
        {
            float* d0 = a.a0 ? a.a0 + (size_t)c * a.N + k * BLK : nullptr;
            float* dst = a.txa + (size_t)c * a.N + k * BLK;
#pragma unroll
            for (int m = 0; m < BLK; m += 4)
            {
                const float4 v = make_float4(x[m], x[m + 1], x[m + 2], x[m + 3]);
                *(float4*)(dst + m) = v;
                if (d0) *(float4*)(d0 + m) = v;
            }
        }
    }
    if (live)
    {
#pragma unroll
        for (int i = 0; i < 12; ++i) a.bq[i * C + c] = bq[i];
        a.alc[c] = alc_val;
    }
}

struct TxIqArgs
{
    const uhsdr_tx_plan* plan;
    const float* txa;        // [C][ld] compressed audio, frame 0 of this launch
    float* hist;             // [C][200] Hilbert history (shared by the I and Q filters: same input)
    const float* osc_in;     // [2] oscillator {I, Q} at launch start
    float* osc_out;          // [2]
    int2* iq;                // [C][ld] DAC frames, frame 0 of this launch
    const float* taps2;      // Hilbert pair {hilbert_i[k], hilbert_q[k]} interleaved (fir_block2)
    int C, N, ld, lw;
};

// F: UHSDR_PRECISION_FMA (uhsdr_tx_set_precision): the Hilbert pair's MACs fused (v_pk_fma_f32)
template <int R, bool F>
__global__ void __launch_bounds__(64) tx_iq(TxIqArgs a)
{
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const uhsdr_tx_plan* __restrict__ P = a.plan;
    const int N = a.N, C = a.C;
    const int lane = threadIdx.x;
    const int nb = N / R;
    const int CPW = 64 / nb;
    int g, b;
    front_lane(lane, nb, 2 * R, g, b);               // lane map for the pair window (2R floats per lane)
    const int c = blockIdx.x * CPW + g;
    const bool act = g < CPW;
    const bool live = act && c < C;
    const int gs = act ? g : 0;
    const int cl = c < C ? c : C - 1;
    constexpr int HQ = hist_q(TX_T);
    float* W = smem + gs * a.lw;
    float* osc = smem + CPW * a.lw;                 // [2N] oscillator trajectory (shift kind 2)

    float xv[R];
    {
        const float4* src = (const float4*)(a.txa + (size_t)cl * a.ld + b * R);
#pragma unroll
        for (int j = 0; j < R / 4; ++j)
        {
            const float4 v = src[j];
            xv[4 * j] = v.x; xv[4 * j + 1] = v.y; xv[4 * j + 2] = v.z; xv[4 * j + 3] = v.w;
        }
    }
    vf4 hA[HQ];
    front_load_row<TX_T>(a.hist, cl, b, nb, hA);
    const int shift = P->freq_shift_hz != 0 ? P->shift_kind : 0;
    if (shift == 2 && lane == 0)
    {
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
        if (blockIdx.x == 0) { a.osc_out[0] = vi; a.osc_out[1] = vq; }
    }
    // the Hilbert pair as one packed FIR pair over the window {x[n], x[n]} (fir_block2)
    v2f x2[R];
#pragma unroll
    for (int j = 0; j < R; ++j) x2[j] = v2f{ xv[j], xv[j] };
    front_fill2<TX_T, HQ, true>(W, a.hist, a.hist, c, act, live, b, nb, hA, hA, x2, R);
    v2f h2[R];
    fir_block2<TX_T, R, 1, F>(W + 2 * b * R, as_taps2(a.taps2), h2);
    float hi[R], hq[R];
#pragma unroll
    for (int r = 0; r < R; ++r) { hi[r] = h2[r].x; hq[r] = h2[r].y; }
    const bool up = P->shift_up;
    const float gi = P->final_i_gain, gq = P->final_q_gain, ph = P->phase_balance;
    int out[2 * R];
    const bool am = P->am;
#pragma unroll
    for (int r = 0; r < R; ++r)
    {
        const int n = b * R + r;
        float I = hi[r], Q = hq[r];
        if (am)
        {
            // TxProcessor_AM (tx_processor.c:780-788): both sidebands and the carrier,
            // 2 * AM_CARRIER_LEVEL (audio_driver.h:429) as the float the int constant converts to
            const float i_am = (I - Q) + 10200.0f;
            const float q_am = (Q - I) - 10200.0f;
            I = i_am;
            Q = q_am;
        }
        if (shift)
        {
            float ib = up ? I : Q, qb = up ? Q : I;
            if (shift == 1)
            {
                const float iv = ib, qv = qb;
                switch (n & 3)
                {
                case 0: break;
                case 1: ib = qv; qb = -iv; break;
                case 2: ib = -iv; qb = -qv; break;
                default: ib = -qv; qb = iv; break;
                }
            }
            else
            {
                const float oq = osc[2 * n], oi = osc[2 * n + 1];
                const float qt = qb, it = ib;
                qb = (qt * oq) - (it * oi);
                ib = (it * oq) + (qt * oi);
            }
            I = up ? ib : qb;
            Q = up ? qb : ib;
        }
        I = I * gi;
        Q = Q * gq;
        if (ph < 0) { const float e = I * ph; Q = Q + e; }
        else if (ph > 0) { const float e = Q * ph; I = I + e; }
        out[2 * r] = tx_to_int32(I);
        out[2 * r + 1] = tx_to_int32(Q);
    }
    if (live)
    {
        int4* dst = (int4*)(a.iq + (size_t)c * a.ld + b * R);
#pragma unroll
        for (int j = 0; j < R / 2; ++j) dst[j] = make_int4(out[4 * j], out[4 * j + 1], out[4 * j + 2], out[4 * j + 3]);
    }
}

// TX_AUDIO_DIGIQ (tx_processor.c:950-961): the USB I/Q frames, int32 -> f32, straight to
// TxProcessor_IqFinalProcessing (:282-330) with iq_gain_comp 1.0; two frames per lane
__global__ void __launch_bounds__(256) tx_digiq(const uhsdr_tx_plan* plan, const int4* src, int4* dst, long long pairs)
{
    const long long k = (long long)blockIdx.x * 256 + threadIdx.x;
    if (k >= pairs) return;
    const uhsdr_tx_plan* __restrict__ P = plan;
    const float gi = P->digiq_i_gain, gq = P->digiq_q_gain, ph = P->phase_balance;
    const int4 v = src[k];
    float I[2] = { (float)v.x, (float)v.z }, Q[2] = { (float)v.y, (float)v.w };
#pragma unroll
    for (int j = 0; j < 2; ++j)
    {
        I[j] = I[j] * gi;
        Q[j] = Q[j] * gq;
        if (ph < 0) { const float e = I[j] * ph; Q[j] = Q[j] + e; }
        else if (ph > 0) { const float e = Q[j] * ph; I[j] = I[j] + e; }
    }
    dst[k] = make_int4(tx_to_int32(I[0]), tx_to_int32(Q[0]), tx_to_int32(I[1]), tx_to_int32(Q[1]));
}

// ------------------------------------------------------------------------------------
// host runtime

struct uhsdr_tx_s
{
    uhsdr_tx_plan plan;
    uhsdr_tx_plan* d_plan;
    float* d_taps2;          // Hilbert pair, interleaved for fir_block2
    int C, N, Nf, R, lw;
    hipStream_t stream;
    float *lat, *bq, *alc, *delay, *hist, *osc, *txa;
    uint32_t* fm;            // FM modulator state [4][C] (null for SSB)
    void* arena;
    size_t arena_bytes;
    long long calls_done, iq_launches;
    int tune, burst;                 // uhsdr_tx_set_tune / _set_tone_burst
    uint32_t tune_acc[2], burst_acc; // softdds accumulators (dbldds[0..1], tone_burst_dds) at the next frame
    // pipelined mode (uhsdr_tx_set_pipelined): tx_iq on a side stream, the compressed-audio
    // hand-off txa in two buffers, so tx_voice of call k+1 overlaps tx_iq of call k
    int pipelined;
    long long calls_issued;
    hipStream_t side;
    hipEvent_t ev_voice, ev_join, ev_iq[2];
    float* txa2;                     // the second hand-off buffer [C][N]
    int precision;                   // uhsdr_tx_set_precision
};

#define HIPCHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { uhsdr_set_error("%s: %s", #x, hipGetErrorString(e_)); return UHSDR_DEVICE_ERROR; } } while (0)

static int tx_pitch(int Nf, int R)
{
    const int nb = Nf / R, cpw = 64 / nb;
    const int need = (2 * (TX_T - 1 + Nf + FRONT_TAIL) + 3) & ~3;   // pair window {x, x}
    uint16_t lm[64];
    for (int l = 0; l < 64; ++l)
    {
        int g, b;
        front_lane(l, nb, 2 * R, g, b);
        lm[l] = (uint16_t)(g << 8 | b);
    }
    int best = need, best_cost = 1 << 30;
    for (int lw = need; lw < need + 64; lw += 4)
    {
        const int cost = window_conflicts(lw, lm, cpw, 2 * R);
        if (cost < best_cost) { best_cost = cost; best = lw; }
    }
    return best;
}

// the side stream's work (tx_iq of pipelined calls) ordered before the handle's stream
static uhsdr_status tx_join(uhsdr_tx_s* h)
{
    if (h->pipelined)
    {
        HIPCHK(hipEventRecord(h->ev_join, h->side));
        HIPCHK(hipStreamWaitEvent(h->stream, h->ev_join, 0));
    }
    return UHSDR_OK;
}

extern "C" uhsdr_status uhsdr_tx_reset(uhsdr_tx_handle h)
{
    if (!h) return UHSDR_ARGUMENT_ERROR;
    if (tx_join(h) != UHSDR_OK) return UHSDR_DEVICE_ERROR;
    HIPCHK(hipMemsetAsync(h->arena, 0, h->arena_bytes, h->stream));
    // ads.alc_val = 1 (TxProcessor_Init, tx_processor.c:137); oscillator {I=0, Q=1} (freq_shift.c:48-49)
    float* ones = (float*)malloc(sizeof(float) * h->C);
    for (int i = 0; i < h->C; ++i) ones[i] = 1.0f;
    HIPCHK(hipMemcpyAsync(h->alc, ones, sizeof(float) * h->C, hipMemcpyHostToDevice, h->stream));
    const float osc0[4] = { 0.0f, 1.0f, 0.0f, 1.0f };
    HIPCHK(hipMemcpyAsync(h->osc, osc0, sizeof osc0, hipMemcpyHostToDevice, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    free(ones);
    // TxProcessor_Init -> AudioManagement_LoadToneBurstMode: tone burst DDS from phase 0
    h->burst_acc = 0;
    h->tune_acc[0] = h->tune_acc[1] = 0;
    h->calls_done = 0;
    h->iq_launches = 0;
    h->calls_issued = 0;
    return UHSDR_OK;
}

extern "C" uhsdr_status uhsdr_tx_set_tune(uhsdr_tx_handle h, int32_t tune)
{
    if (!h || tune < UHSDR_TUNE_OFF || tune > UHSDR_TUNE_TWO) { uhsdr_set_error("bad argument"); return UHSDR_ARGUMENT_ERROR; }
    // AudioManagement_SetSidetoneForDemodMode -> softdds_configRunIQ(freq, rate, smooth = 0): both
    // accumulators restart at 0, on entering and on leaving TUNE (audio_management.c:377-404)
    h->tune = tune;
    h->tune_acc[0] = h->tune_acc[1] = 0;
    return UHSDR_OK;
}

extern "C" uhsdr_status uhsdr_tx_set_tone_burst(uhsdr_tx_handle h, int32_t active)
{
    if (!h) return UHSDR_ARGUMENT_ERROR;
    h->burst = active != 0;    // the tone burst DDS keeps its phase between bursts
    return UHSDR_OK;
}

extern "C" uhsdr_status uhsdr_tx_prepare_run(uhsdr_tx_handle h)
{
    if (!h) return UHSDR_ARGUMENT_ERROR;
    // TxProcessor_PrepareRun (tx_processor.c:63-66): arm_fill_f32(0, audio_delay_buffer, ...)
    HIPCHK(hipMemsetAsync(h->delay, 0, sizeof(float) * UHSDR_TX_DELAY * (size_t)h->C, h->stream));
    return UHSDR_OK;
}

extern "C" uhsdr_status uhsdr_tx_create(const uhsdr_tx_config* cfg, int32_t C, int32_t N, void* stream,
                                        uhsdr_tx_handle* out)
{
    if (!cfg || !out || C <= 0 || N <= 0) { uhsdr_set_error("bad argument"); return UHSDR_ARGUMENT_ERROR; }
    if (N % BLK) { uhsdr_set_error("frames_per_call %d not a multiple of %d", N, BLK); return UHSDR_LENGTH_ERROR; }
    *out = nullptr;
    uhsdr_tx_s* h = (uhsdr_tx_s*)calloc(1, sizeof(uhsdr_tx_s));
    uhsdr_status st = uhsdr_tx_plan_build(cfg, &h->plan);
    if (st != UHSDR_OK) { free(h); return st; }
    if (h->plan.lat_stages != 10) { free(h); uhsdr_set_error("TX lattice with %d stages", h->plan.lat_stages); return UHSDR_UNSUPPORTED; }
    h->C = C; h->N = N;
    h->stream = (hipStream_t)stream;
    h->R = 8;
    h->Nf = N < 64 * h->R ? N : 64 * h->R;
    if (h->Nf / h->R < 4) { h->R = 8; }
    if (N % h->Nf || h->Nf % h->R || h->Nf / h->R < 4)
    { free(h); uhsdr_set_error("frames_per_call %d: need a multiple of 32 of at least 32", N); return UHSDR_LENGTH_ERROR; }
    h->lw = tx_pitch(h->Nf, h->R);
    size_t fl = 0;
    auto take = [&](size_t n) { size_t o = fl; fl += (n + 63) & ~(size_t)63; return o; };
    const size_t o_lat = take((size_t)10 * C), o_bq = take((size_t)12 * C), o_alc = take((size_t)C);
    const size_t o_dly = take((size_t)UHSDR_TX_DELAY * C), o_hist = take((size_t)hist_stride(TX_T) * C);
    const size_t o_osc = take(4), o_txa = take(h->plan.fm ? 0 : (size_t)C * N);
    const size_t o_fm = take(h->plan.fm ? (size_t)4 * C : 0);
    h->arena_bytes = fl * sizeof(float);
    constexpr int T2N = (TX_T + 7) & ~7;
    if (hipMalloc(&h->arena, h->arena_bytes) != hipSuccess || hipMalloc((void**)&h->d_plan, sizeof(uhsdr_tx_plan)) != hipSuccess ||
        hipMalloc((void**)&h->d_taps2, sizeof(float) * 2 * T2N) != hipSuccess)
    {
        uhsdr_set_error("hipMalloc failed (%zu bytes state)", h->arena_bytes);
        if (h->arena) (void)hipFree(h->arena);
        free(h);
        return UHSDR_DEVICE_ERROR;
    }
    float* A = (float*)h->arena;
    h->lat = A + o_lat; h->bq = A + o_bq; h->alc = A + o_alc; h->delay = A + o_dly;
    h->hist = A + o_hist; h->osc = A + o_osc; h->txa = A + o_txa;
    h->fm = h->plan.fm ? (uint32_t*)(A + o_fm) : nullptr;
    {
        float t2[2 * T2N];
        for (int k = 0; k < T2N; ++k)
        {
            t2[2 * k] = k < TX_T ? h->plan.hilbert_i[k] : 0.0f;
            t2[2 * k + 1] = k < TX_T ? h->plan.hilbert_q[k] : 0.0f;
        }
        if (hipMemcpy(h->d_taps2, t2, sizeof t2, hipMemcpyHostToDevice) != hipSuccess)
        {
            uhsdr_set_error("tap upload failed");
            return UHSDR_DEVICE_ERROR;
        }
    }
    if (hipMemcpy(h->d_plan, &h->plan, sizeof(uhsdr_tx_plan), hipMemcpyHostToDevice) != hipSuccess)
    {
        uhsdr_set_error("plan upload failed");
        return UHSDR_DEVICE_ERROR;
    }
    *out = h;
    return uhsdr_tx_reset(h);
}

extern "C" uhsdr_status uhsdr_tx_process(uhsdr_tx_handle h, const int32_t* audio, int32_t* iq, float* a0)
{
    if (!h || !audio || !iq) { uhsdr_set_error("null argument"); return UHSDR_ARGUMENT_ERROR; }
    if (h->plan.digiq && !h->tune)
    {
        // USB I/Q source: no voice chain, no modulator state advances, a0 (adb.a_buffer[0]) untouched.
        // Pipelined: the handle's stream first waits for the side stream (the DAC frames of the
        // voice calls before it), then tx_digiq runs on the handle's stream itself, so the input
        // buffer is read in stream order exactly as in serial mode
        const long long pairs = (long long)h->C * h->N / 2;
        const hipStream_t st = h->stream;
        if (tx_join(h) != UHSDR_OK) return UHSDR_DEVICE_ERROR;
        hipLaunchKernelGGL(tx_digiq, dim3((unsigned)((pairs + 255) / 256)), dim3(256), 0, st, h->d_plan,
                           (const int4*)audio, (int4*)iq, pairs);
        HIPCHK(hipGetLastError());
        return UHSDR_OK;
    }
    if ((h->plan.am || h->plan.fm) && h->plan.freq_shift_hz == 0)
    {
        // DIGIQ source with TUNE in AM / FM without frequency translation: the reference's AM / FM
        // branch does nothing (tx_processor.c:996-1016), signal_active stays false and the zeroed
        // I/Q goes through the final stage (:1021-1025, :282-330): all-zero DAC frames, no state
        // advances, a0 untouched
        if (tx_join(h) != UHSDR_OK) return UHSDR_DEVICE_ERROR;
        HIPCHK(hipMemsetAsync(iq, 0, sizeof(int32_t) * 2 * (size_t)h->C * h->N, h->stream));
        return UHSDR_OK;
    }
    // pipelined: this call's hand-off buffer, free once the tx_iq that read it two calls ago is done
    const int par = h->pipelined ? (int)(h->calls_issued & 1) : 0;
    float* const txa = par ? h->txa2 : h->txa;
    if (h->pipelined && !h->plan.fm) HIPCHK(hipStreamWaitEvent(h->stream, h->ev_iq[par], 0));
    TxVoiceArgs va;
    va.plan = h->d_plan; va.audio = (const int2*)audio; va.txa = txa; va.a0 = a0;
    va.lat = h->lat; va.bq = h->bq; va.alc = h->alc; va.delay = h->delay;
    va.fm = h->fm; va.iq = (int2*)iq;
    va.C = h->C; va.N = h->N;
    va.delay_phase = (int)(h->calls_done % TX_DELAY_SLOTS);
    va.tune = h->tune;
    va.tune_acc0 = h->tune_acc[0];
    va.tune_acc1 = h->tune_acc[1];
    va.burst = h->plan.fm && h->burst;
    va.burst_acc = h->burst_acc;
    if (h->tune)
    {
        h->tune_acc[0] += (uint32_t)h->N * h->plan.tune_step[0];
        if (h->tune == 2) h->tune_acc[1] += (uint32_t)h->N * h->plan.tune_step[1];
    }
    if (va.burst) h->burst_acc += (uint32_t)h->N * h->plan.tone_burst_step;
    if (h->plan.fm)
    {
        // FM: the modulator is sequential per channel and finishes in tx_voice
        hipLaunchKernelGGL((tx_voice<10, true>), dim3((h->C + 63) / 64), dim3(64), 0, h->stream, va);
        HIPCHK(hipGetLastError());
        h->calls_done += h->N / BLK;
        return UHSDR_OK;
    }
    hipLaunchKernelGGL(tx_voice2<10>, dim3((h->C + 63) / 64), dim3(128), 0, h->stream, va);
    HIPCHK(hipGetLastError());
    const hipStream_t ist = h->pipelined ? h->side : h->stream;
    if (h->pipelined)
    {
        HIPCHK(hipEventRecord(h->ev_voice, h->stream));
        HIPCHK(hipStreamWaitEvent(ist, h->ev_voice, 0));
    }
    const int cpw = 64 / (h->Nf / h->R);
    const size_t lds = sizeof(float) * ((size_t)cpw * h->lw + (h->plan.shift_kind == 2 ? 2 * h->Nf : 0));
    void (*const iq_fn)(TxIqArgs) = h->precision == UHSDR_PRECISION_FMA ? tx_iq<8, true> : tx_iq<8, false>;
    for (int f0 = 0; f0 < h->N; f0 += h->Nf)
    {
        TxIqArgs ia;
        ia.plan = h->d_plan; ia.txa = txa + f0; ia.hist = h->hist;
        ia.osc_in = h->osc + 2 * (h->iq_launches & 1);
        ia.osc_out = h->osc + 2 * ((h->iq_launches + 1) & 1);
        ia.iq = (int2*)iq + f0;
        ia.C = h->C; ia.N = h->Nf; ia.ld = h->N; ia.lw = h->lw;
        ia.taps2 = h->d_taps2;
        hipLaunchKernelGGL(iq_fn, dim3((h->C + cpw - 1) / cpw), dim3(64), lds, ist, ia);
        HIPCHK(hipGetLastError());
        h->iq_launches += 1;
    }
    if (h->pipelined) HIPCHK(hipEventRecord(h->ev_iq[par], ist));
    h->calls_issued += 1;
    h->calls_done += h->N / BLK;
    return UHSDR_OK;
}

extern "C" uhsdr_status uhsdr_tx_set_precision(uhsdr_tx_handle h, int32_t precision)
{
    if (!h) return UHSDR_ARGUMENT_ERROR;
    if (precision != UHSDR_PRECISION_EXACT && precision != UHSDR_PRECISION_FMA)
    {
        uhsdr_set_error("unknown precision %d", (int)precision);
        return UHSDR_ARGUMENT_ERROR;
    }
    h->precision = precision;
    return UHSDR_OK;
}

extern "C" int32_t uhsdr_tx_get_precision(uhsdr_tx_handle h) { return h ? h->precision : -1; }

extern "C" uhsdr_status uhsdr_tx_join(uhsdr_tx_handle h)
{
    if (!h) return UHSDR_ARGUMENT_ERROR;
    return tx_join(h);
}

extern "C" uhsdr_status uhsdr_tx_set_pipelined(uhsdr_tx_handle h, int32_t enable)
{
    if (!h) return UHSDR_ARGUMENT_ERROR;
    if (enable && !h->side)
    {
        HIPCHK(hipStreamCreateWithFlags(&h->side, hipStreamNonBlocking));
        HIPCHK(hipEventCreateWithFlags(&h->ev_voice, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&h->ev_join, hipEventDisableTiming));
        for (int i = 0; i < 2; ++i) HIPCHK(hipEventCreateWithFlags(&h->ev_iq[i], hipEventDisableTiming));
        // no call has run on the side stream yet: the events start complete
        for (int i = 0; i < 2; ++i) HIPCHK(hipEventRecord(h->ev_iq[i], h->side));
    }
    if (enable && !h->txa2 && !h->plan.fm)
        HIPCHK(hipMalloc((void**)&h->txa2, sizeof(float) * (size_t)h->C * h->N));
    if (!enable && h->pipelined && tx_join(h) != UHSDR_OK) return UHSDR_DEVICE_ERROR;
    if (enable && !h->pipelined)
    {
        // the side stream starts after everything the handle's stream has queued (state it reads)
        HIPCHK(hipEventRecord(h->ev_voice, h->stream));
        HIPCHK(hipStreamWaitEvent(h->side, h->ev_voice, 0));
        for (int i = 0; i < 2; ++i) HIPCHK(hipEventRecord(h->ev_iq[i], h->side));
        h->calls_issued = 0;
    }
    h->pipelined = enable != 0;
    return UHSDR_OK;
}

extern "C" int32_t uhsdr_tx_get_pipelined(uhsdr_tx_handle h) { return h ? h->pipelined : 0; }

extern "C" uhsdr_status uhsdr_tx_get_plan(uhsdr_tx_handle h, uhsdr_tx_plan* plan)
{
    if (!h || !plan) return UHSDR_ARGUMENT_ERROR;
    memcpy(plan, &h->plan, sizeof *plan);
    return UHSDR_OK;
}

extern "C" uhsdr_status uhsdr_tx_destroy(uhsdr_tx_handle h)
{
    if (!h) return UHSDR_ARGUMENT_ERROR;
    (void)hipStreamSynchronize(h->stream);
    if (h->side)
    {
        (void)hipStreamSynchronize(h->side);
        (void)hipStreamDestroy(h->side);
        (void)hipEventDestroy(h->ev_voice);
        (void)hipEventDestroy(h->ev_join);
        for (int i = 0; i < 2; ++i) (void)hipEventDestroy(h->ev_iq[i]);
    }
    if (h->txa2) (void)hipFree(h->txa2);
    (void)hipFree(h->arena);
    (void)hipFree(h->d_plan);
    (void)hipFree(h->d_taps2);
    free(h);
    return UHSDR_OK;
}
