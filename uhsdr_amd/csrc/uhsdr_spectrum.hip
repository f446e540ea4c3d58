// MI355X (gfx950) spectrum display of the UHSDR firmware, batched over channels.
//
// Per channel and per fft_len input samples (one display frame), bit-identical to the firmware
// built for x86:
//   producer  convert x 2^-16, I/Q correction (manual / auto)   audio_driver.c:2660-2685, 2254-2316
//             into the interleaved [Q, I] ring                    audio_driver.c:1811-1851
//   consumer  Hann window per float of the ring                  ui_spectrum.c:402-414
//             arm_cfft_f32 forward + bit reversal                CMSIS arm_cfft_f32.c:574-632,
//                                                                arm_cfft_radix8_f32.c:130-383,
//                                                                arm_bitreversal2.S:136-180
//             arm_cmplx_mag_f32, IIR average clamped at 1        ui_spectrum.c:1405, 1432-1446
//
// One wave per channel (four per workgroup, no workgroup barrier): the frame lives in LDS
// (2 * fft_len floats), every FFT stage is one pass of independent butterflies over it, the
// running average sits in registers (fft_len / 64 bins per lane) for the whole launch.  Frames
// that straddle calls are carried in HBM.  HBM traffic per sample: 8 B I/Q in + 4 B per output
// array written; the state (average, carry) moves once per launch.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
#include <math.h>
#include "uhsdr_internal.h"
#include "uhsdr_dsp.h"

namespace {

constexpr int SPEC_WAVES = 4;

struct SpecArgs
{
    const uhsdr_spectrum_plan* plan;
    const int2* iq;          // [C][ld] IqSample_t
    float* teta;             // [3][C] auto I/Q correction low-pass state
    float* avg_state;        // [C][L] sd.FFT_AVGData
    float* carry;            // [C][2L] windowed ring of an incomplete frame (positions < fill)
    float* mag;              // optional [C][F][L]
    float* avg;              // optional [C][F][L]
    int C, N, ld, F, fill0, lds_pitch;
};

__device__ __forceinline__ float sign_new(float x) { return (x < 0) ? -1.0f : ((x > 0) ? 1.0f : 0.0f); }

// arm_radix8_butterfly_f32 butterfly on the 8 complex values x[base + k*stride] (LDS): the
// reference's two loop bodies share one sequence of adds for the eight outputs X_k; the twiddled
// groups then rotate X_k, k >= 1, by twiddle[k * tstep] as (c*re + s*im, c*im - s*re).
__device__ __forceinline__ void bfly8(float* __restrict__ x, int base, int stride, const float* __restrict__ tw, int tstep)
{
    const float C81 = 0.70710678118f;
    float re[8], im[8];
#pragma unroll
    for (int k = 0; k < 8; ++k)
    {
        const float2 v = *(const float2*)(x + 2 * (base + k * stride));
        re[k] = v.x;
        im[k] = v.y;
    }
    float sr[4], dr[4], si[4], di[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
    {
        sr[k] = re[k] + re[k + 4];
        dr[k] = re[k] - re[k + 4];
        si[k] = im[k] + im[k + 4];
        di[k] = im[k] - im[k + 4];
    }
    float Xr[8], Xi[8];
    const float a = sr[0] - sr[2], b = sr[0] + sr[2], cc = sr[1] - sr[3], d = sr[1] + sr[3];
    const float ai = si[0] - si[2], bi = si[0] + si[2], ci = si[1] - si[3], dd = si[1] + si[3];
    Xr[0] = b + d;   Xi[0] = bi + dd;
    Xr[4] = b - d;   Xi[4] = bi - dd;
    Xr[2] = a + ci;  Xi[2] = ai - cc;
    Xr[6] = a - ci;  Xi[6] = ai + cc;
    const float u = (dr[1] - dr[3]) * C81, v = (dr[1] + dr[3]) * C81;
    const float ui = (di[1] - di[3]) * C81, vi = (di[1] + di[3]) * C81;
    const float e0 = dr[0] - u, e1 = dr[0] + u, f0 = dr[2] - v, f1 = dr[2] + v;
    const float g0 = di[0] - ui, g1 = di[0] + ui, h0 = di[2] - vi, h1 = di[2] + vi;
    Xr[1] = e1 + h1; Xi[1] = g1 - f1;
    Xr[7] = e1 - h1; Xi[7] = g1 + f1;
    Xr[5] = e0 + h0; Xi[5] = g0 - f0;
    Xr[3] = e0 - h0; Xi[3] = g0 + f0;
    if (tstep)
    {
#pragma unroll
        for (int k = 1; k < 8; ++k)
        {
            const float2 t = *(const float2*)(tw + 2 * k * tstep);
            const float p1 = t.x * Xr[k], p2 = t.y * Xi[k], p3 = t.x * Xi[k], p4 = t.y * Xr[k];
            Xr[k] = p1 + p2;
            Xi[k] = p3 - p4;
        }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) *(float2*)(x + 2 * (base + k * stride)) = make_float2(Xr[k], Xi[k]);
}

// arm_radix8_butterfly_f32 stages on NSUB sub-arrays of n points each (contiguous), twiddle
// modifier TM0; butterflies of a stage are independent, spread over the wave's lanes
template <int n, int NSUB, int TM0>
__device__ __forceinline__ void radix8_stages(float* x, const float* tw, int lane)
{
#pragma unroll
    for (int span = n, tm = TM0; span >= 8; span >>= 3, tm <<= 3)
    {
        const int stride = span >> 3;
        constexpr int per_sub = n / 8;
        for (int q = lane; q < NSUB * per_sub; q += 64)
        {
            const int sub = q / per_sub, r = q % per_sub;
            const int j = r % stride, g = j + span * (r / stride);
            bfly8(x + 2 * n * sub, g, stride, tw, j * tm);
        }
        wave_sync();
    }
}

__device__ __forceinline__ float2 rot_fwd(float xr, float xi, float c, float s)
{
    const float m0 = xr * c, m1 = xi * s, m2 = xi * c, m3 = xr * s;
    return make_float2(m0 + m1, m2 - m3);
}

// arm_cfft_radix8by2_f32 (arm_cfft_f32.c:207-317) radix-2 split, n = 1024
template <int n>
__device__ __forceinline__ void split_by2(float* x, const float* tw, int lane)
{
    constexpr int H = n / 2, Q = n / 4;
    for (int a = lane; a < Q; a += 64)
    {
        float2* p1 = (float2*)x + a;
        float2* p3 = (float2*)x + a + Q;
        float2* p2 = (float2*)x + a + H;
        float2* p4 = (float2*)x + a + H + Q;
        const float2 x1 = *p1, x2 = *p2, x3 = *p3, x4 = *p4;
        const float t2r = x1.x - x2.x, t2i = x1.y - x2.y;
        const float t4r = x4.x - x3.x, t4i = x4.y - x3.y;
        *p1 = make_float2(x1.x + x2.x, x1.y + x2.y);
        *p3 = make_float2(x3.x + x4.x, x3.y + x4.y);
        const float2 t = *(const float2*)(tw + 2 * a);
        *p2 = rot_fwd(t2r, t2i, t.x, t.y);
        const float m0 = t4r * t.y, m1 = t4i * t.x, m2 = t4i * t.y, m3 = t4r * t.x;
        *p4 = make_float2(m0 - m1, m2 + m3);
    }
    wave_sync();
}

// arm_cfft_radix8by4_f32 (arm_cfft_f32.c:319-557) radix-4 split, n = 256: lanes 0..Q/2 take
// the top rows t (t = 0 untwiddled, t = Q/2 the reference's MIDDLE block), lanes Q/2+1.. the
// bottom rows Q - t with the mirrored twiddles of t
template <int n>
__device__ __forceinline__ void split_by4(float* x, const float* tw, int lane)
{
    constexpr int Q = n / 4;
    static_assert(Q == 64, "one row per lane");
    const bool top = lane <= Q / 2;
    const int t = top ? lane : lane - Q / 2;
    const int row = top ? t : Q - t;
    float2* p1 = (float2*)x + row;
    float2* p2 = p1 + Q;
    float2* p3 = p1 + 2 * Q;
    float2* p4 = p1 + 3 * Q;
    const float2 x1 = *p1, x2 = *p2, x3 = *p3, x4 = *p4;
    const float s13r = x1.x + x3.x, d13r = x1.x - x3.x;
    const float s13i = x1.y + x3.y, d13i = x1.y - x3.y;
    const float2 w2 = *(const float2*)(tw + 2 * t), w3 = *(const float2*)(tw + 4 * t), w4 = *(const float2*)(tw + 6 * t);
    if (top)
    {
        const float t2r = d13r + x2.y - x4.y, t2i = d13i - x2.x + x4.x;
        const float t3r = s13r - x2.x - x4.x, t3i = s13i - x2.y - x4.y;
        const float t4r = d13r - x2.y + x4.y, t4i = d13i + x2.x - x4.x;
        *p1 = make_float2(s13r + x2.x + x4.x, s13i + x2.y + x4.y);
        if (t == 0)
        {
            *p2 = make_float2(t2r, t2i);
            *p3 = make_float2(t3r, t3i);
            *p4 = make_float2(t4r, t4i);
        }
        else
        {
            *p2 = rot_fwd(t2r, t2i, w2.x, w2.y);
            *p3 = rot_fwd(t3r, t3i, w3.x, w3.y);
            *p4 = rot_fwd(t4r, t4i, w4.x, w4.y);
        }
    }
    else
    {
        const float u2r = x2.y - x4.y + d13r;
        const float u2i = x1.y - x3.y - x2.x + x4.x;
        const float u3r = s13r - x2.x - x4.x;
        const float u3i = s13i - x2.y - x4.y;
        const float u4r = x2.y - x4.y - d13r;
        const float u4i = x4.x - x2.x - d13i;
        *p1 = make_float2(s13r + x2.x + x4.x, s13i + x2.y + x4.y);
        {
            const float m0 = u2i * w2.y, m1 = u2r * w2.x, m2 = u2r * w2.y, m3 = u2i * w2.x;
            *p2 = make_float2(m2 + m3, m0 - m1);
        }
        {
            const float m0 = -u3i * w3.x, m1 = u3r * w3.y, m2 = u3r * w3.x, m3 = u3i * w3.y;
            *p3 = make_float2(m3 - m2, m0 - m1);
        }
        {
            const float m0 = u4i * w4.y, m1 = u4r * w4.x, m2 = u4r * w4.y, m3 = u4i * w4.x;
            *p4 = make_float2(m2 + m3, m0 - m1);
        }
    }
    wave_sync();
}

template <int L>
__device__ __forceinline__ void cfft(float* x, const float* tw, int lane)
{
    if constexpr (L == 1024)
    {
        split_by2<L>(x, tw, lane);
        radix8_stages<L / 2, 2, 2>(x, tw, lane);
    }
    else if constexpr (L == 512)
    {
        radix8_stages<L, 1, 1>(x, tw, lane);
    }
    else
    {
        split_by4<L>(x, tw, lane);
        radix8_stages<L / 4, 4, 4>(x, tw, lane);
    }
}

template <int L>
__global__ void __launch_bounds__(64 * SPEC_WAVES) spectrum_frames(SpecArgs a)
{
    extern __shared__ __attribute__((aligned(16))) float smem[];
    constexpr int NB = L / 64;                   // bins per lane
    constexpr int NCALL = L / BLK;               // 32-frame calls per display frame
    const uhsdr_spectrum_plan* __restrict__ P = a.plan;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = blockIdx.x * SPEC_WAVES + w;
    if (c >= a.C) return;                        // whole wave; no workgroup barrier below
    float* X = smem + w * a.lds_pitch;           // the frame, [re = Q, im = I] interleaved
    float* T = X + 2 * L;                        // auto I/Q: per-call sums, then factors [3][NCALL]
    const float* __restrict__ tw = P->twiddle;
    const float* __restrict__ win = P->window;
    const bool formula = P->window_formula;
    const bool iq_auto = P->iq_auto_correction;
    const float gi = P->iq_gain_i, gq = P->iq_gain_q, ph = P->iq_phase_balance, f = P->filt_factor;
    const int C = a.C, N = a.N;

    int fill = a.fill0;
    for (int i = lane; i < 2 * fill; i += 64) X[i] = a.carry[(size_t)c * 2 * L + i];
    float av[NB];
#pragma unroll
    for (int m = 0; m < NB; ++m) av[m] = a.avg_state[(size_t)c * L + lane + 64 * m];
    float o1 = 0.0f, o2 = 0.0f, o3 = 0.0f;
    if (iq_auto) { o1 = a.teta[c]; o2 = a.teta[C + c]; o3 = a.teta[2 * C + c]; }
    const int2* __restrict__ src = a.iq + (size_t)c * a.ld;
    int frame = 0;
    for (int n0 = 0; n0 < N;)
    {
        const int seg = min(L - fill, N - n0);   // multiple of 32
        // ---- convert into the ring ----
        for (int i = lane; i < seg; i += 64)
        {
            const int2 v = src[n0 + i];
            float I = (float)v.x, Q = (float)v.y;
            I = I * IQ_BIT_SCALE_DOWN;
            Q = Q * IQ_BIT_SCALE_DOWN;
            *(float2*)(X + 2 * (fill + i)) = make_float2(Q, I);
        }
        wave_sync();
        // ---- auto I/Q correction factors per 32-frame call (audio_driver.c:2274-2313) ----
        if (iq_auto)
        {
            const int ncall = seg / BLK;
            if (lane < ncall)
            {
                float t1 = 0.0f, t2 = 0.0f, t3 = 0.0f;
                const float* s = X + 2 * (fill + lane * BLK);
                for (int i = 0; i < BLK; ++i)
                {
                    const float Q = s[2 * i], I = s[2 * i + 1];
                    t1 += sign_new(I) * Q;
                    t2 += sign_new(I) * I;
                    t3 += sign_new(Q) * Q;
                }
                T[lane] = t1; T[NCALL + lane] = t2; T[2 * NCALL + lane] = t3;
            }
            wave_sync();
            float m1v = 0.0f, m2v = 0.0f;
            for (int j = 0; j < ncall; ++j)           // the low-pass recursion, uniform in all lanes
            {
                float t1 = T[j], t2 = T[NCALL + j], t3 = T[2 * NCALL + j];
                t1 = (float)(-0.003 * (double)(t1 / (float)BLK) + 0.997 * (double)o1);
                t2 = (float)(0.003 * (double)(t2 / (float)BLK) + 0.997 * (double)o2);
                t3 = (float)(0.003 * (double)(t3 / (float)BLK) + 0.997 * (double)o3);
                const float M_c1 = (t2 != 0.0f) ? t1 / t2 : 0.0f;
                float help = (t2 * t2);
                if (help > 0.0f) help = (t3 * t3 - t1 * t1) / help;
                const float M_c2 = (help > 0.0f) ? sqrtf(help) : 1.0f;
                o1 = t1; o2 = t2; o3 = t3;
                if (j == lane) { m1v = M_c1; m2v = M_c2; }
            }
            wave_sync();
            if (lane < ncall) { T[lane] = m1v; T[NCALL + lane] = m2v; }
            wave_sync();
        }
        // ---- correction + window, in place ----
        for (int i = lane; i < seg; i += 64)
        {
            const int p = fill + i;
            const float2 v = *(const float2*)(X + 2 * p);
            float Q = v.x, I = v.y;
            if (!iq_auto)
            {
                I = I * gi;
                Q = Q * gq;
                if (ph < 0) { const float e3 = I * ph; Q = Q + e3; }
                else if (ph > 0) { const float e3 = Q * ph; I = I + e3; }
            }
            else
            {
                const int j = i / BLK;
                Q += T[j] * I;
                I = I * T[NCALL + j];
            }
            const float2 wv = *(const float2*)(win + 2 * p);
            float wq, wi;
            if (formula) { wq = 0.5f * (wv.x * Q); wi = 0.5f * (wv.y * I); }
            else { wq = Q * wv.x; wi = I * wv.y; }
            *(float2*)(X + 2 * p) = make_float2(wq, wi);
        }
        wave_sync();
        fill += seg;
        n0 += seg;
        if (fill < L) break;                     // frame continues in the next call
        // ---- one display frame ----
        cfft<L>(X, tw, lane);
        float* mo = a.mag ? a.mag + ((size_t)c * a.F + frame) * L : nullptr;
        float* ao = a.avg ? a.avg + ((size_t)c * a.F + frame) * L : nullptr;
#pragma unroll
        for (int m = 0; m < NB; ++m)
        {
            const int k = lane + 64 * m;
            const float2 v = *(const float2*)(X + 2 * (int)P->perm[k]);
            const float mg = sqrtf((v.x * v.x) + (v.y * v.y));
            float s = av[m];
            const float old = s * f;
            s = s - old;
            const float add = mg * f;
            s = add + s;
            if (s < 1) s = 1;
            av[m] = s;
            if (mo) mo[k] = mg;
            if (ao) ao[k] = s;
        }
        wave_sync();
        ++frame;
        fill = 0;
    }
    for (int i = lane; i < 2 * fill; i += 64) a.carry[(size_t)c * 2 * L + i] = X[i];
#pragma unroll
    for (int m = 0; m < NB; ++m) a.avg_state[(size_t)c * L + lane + 64 * m] = av[m];
    if (iq_auto && lane == 0) { a.teta[c] = o1; a.teta[C + c] = o2; a.teta[2 * C + c] = o3; }
}

} // namespace

struct uhsdr_spectrum_s
{
    uhsdr_spectrum_plan plan;
    uhsdr_spectrum_plan* d_plan;
    int C, N, L, F, fill;
    hipStream_t stream;
    float *teta, *avg, *carry;
    void* arena;
    size_t arena_bytes;
};

#define HIPCHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { uhsdr_set_error("%s: %s", #x, hipGetErrorString(e_)); return UHSDR_DEVICE_ERROR; } } while (0)

static int spec_pitch(int L) { return 2 * L + 3 * (L / BLK) + 4; }

extern "C" uhsdr_status uhsdr_spectrum_reset(uhsdr_spectrum_handle h)
{
    if (!h) return UHSDR_ARGUMENT_ERROR;
    HIPCHK(hipMemsetAsync(h->arena, 0, h->arena_bytes, h->stream));   // sd.FFT_AVGData / iq_corr start zeroed
    HIPCHK(hipStreamSynchronize(h->stream));
    h->fill = 0;
    return UHSDR_OK;
}

extern "C" uhsdr_status uhsdr_spectrum_create(const uhsdr_spectrum_config* cfg, int32_t C, int32_t N, void* stream,
                                              uhsdr_spectrum_handle* out)
{
    if (!cfg || !out || C <= 0 || N <= 0) { uhsdr_set_error("bad argument"); return UHSDR_ARGUMENT_ERROR; }
    *out = nullptr;
    uhsdr_spectrum_s* h = (uhsdr_spectrum_s*)calloc(1, sizeof(uhsdr_spectrum_s));
    uhsdr_status st = uhsdr_spectrum_plan_build(cfg, &h->plan);
    if (st != UHSDR_OK) { free(h); return st; }
    const int L = h->plan.fft_len;
    if (N % BLK || (N % L && L % N))
    {
        free(h);
        uhsdr_set_error("frames_per_call %d: need a multiple of %d that is a multiple or a divisor of fft_len %d", N, BLK, L);
        return UHSDR_LENGTH_ERROR;
    }
    h->C = C; h->N = N; h->L = L;
    h->F = N >= L ? N / L : 1;
    h->stream = (hipStream_t)stream;
    size_t fl = 0;
    auto take = [&](size_t n) { size_t o = fl; fl += (n + 63) & ~(size_t)63; return o; };
    const size_t o_teta = take((size_t)3 * C), o_avg = take((size_t)C * L), o_carry = take(N < L ? (size_t)C * 2 * L : 0);
    h->arena_bytes = fl * sizeof(float);
    if (hipMalloc(&h->arena, h->arena_bytes) != hipSuccess ||
        hipMalloc((void**)&h->d_plan, sizeof(uhsdr_spectrum_plan)) != hipSuccess)
    {
        uhsdr_set_error("hipMalloc failed (%zu bytes state)", h->arena_bytes);
        if (h->arena) (void)hipFree(h->arena);
        free(h);
        return UHSDR_DEVICE_ERROR;
    }
    float* A = (float*)h->arena;
    h->teta = A + o_teta; h->avg = A + o_avg; h->carry = A + o_carry;
    if (hipMemcpy(h->d_plan, &h->plan, sizeof(uhsdr_spectrum_plan), hipMemcpyHostToDevice) != hipSuccess)
    {
        uhsdr_set_error("plan upload failed");
        return UHSDR_DEVICE_ERROR;
    }
    *out = h;
    return uhsdr_spectrum_reset(h);
}

extern "C" uhsdr_status uhsdr_spectrum_process(uhsdr_spectrum_handle h, const int32_t* iq, float* mag, float* avg,
                                               int32_t* frames)
{
    if (!h || !iq) { uhsdr_set_error("null argument"); return UHSDR_ARGUMENT_ERROR; }
    SpecArgs sa;
    sa.plan = h->d_plan; sa.iq = (const int2*)iq;
    sa.teta = h->teta; sa.avg_state = h->avg; sa.carry = h->carry;
    sa.mag = mag; sa.avg = avg;
    sa.C = h->C; sa.N = h->N; sa.ld = h->N; sa.F = h->F; sa.fill0 = h->fill;
    sa.lds_pitch = spec_pitch(h->L);
    const size_t lds = sizeof(float) * (size_t)SPEC_WAVES * sa.lds_pitch;
    const dim3 grid((h->C + SPEC_WAVES - 1) / SPEC_WAVES), block(64 * SPEC_WAVES);
    switch (h->L)
    {
    case 256: hipLaunchKernelGGL(spectrum_frames<256>, grid, block, lds, h->stream, sa); break;
    case 512: hipLaunchKernelGGL(spectrum_frames<512>, grid, block, lds, h->stream, sa); break;
    default: hipLaunchKernelGGL(spectrum_frames<1024>, grid, block, lds, h->stream, sa); break;
    }
    HIPCHK(hipGetLastError());
    const int done = (h->fill + h->N) / h->L;
    h->fill = (h->fill + h->N) % h->L;
    if (frames) *frames = done;
    return UHSDR_OK;
}

extern "C" uhsdr_status uhsdr_spectrum_get_plan(uhsdr_spectrum_handle h, uhsdr_spectrum_plan* plan)
{
    if (!h || !plan) return UHSDR_ARGUMENT_ERROR;
    memcpy(plan, &h->plan, sizeof *plan);
    return UHSDR_OK;
}

extern "C" uhsdr_status uhsdr_spectrum_destroy(uhsdr_spectrum_handle h)
{
    if (!h) return UHSDR_ARGUMENT_ERROR;
    (void)hipStreamSynchronize(h->stream);
    (void)hipFree(h->arena);
    (void)hipFree(h->d_plan);
    free(h);
    return UHSDR_OK;
}
