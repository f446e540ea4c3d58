// CMSIS-DSP signature shims on the MI355X (include/uhsdr_cmsis.h, libuhsdr_cmsis.so).
//
// Same symbols, instance layouts and state conventions as CMSIS-DSP V1.4.5
// (basesw/ovi40/Drivers/CMSIS/Include/arm_math.h); every processing call packs the instance's
// carried state and the block into one device buffer, runs one kernel on a per-thread HIP
// stream, and returns the outputs and the new state to the caller's host arrays.  Arithmetic
// is the reference's binary32 sequence (compiled -ffp-contract=off):
//   arm_fir_f32 / arm_fir_decimate_f32  y[m] = sum_{k<T} c[k] x[Mm + k] from +0.0f in tap order
//                                       (FilteringFunctions/arm_fir_f32.c:482-560,
//                                       arm_fir_decimate_f32.c), one lane per output
//   arm_fir_interpolate_f32             output j of input n: sum_{t<ph} x[n+t] c[(L-1-j) + tL]
//                                       (arm_fir_interpolate_f32.c:482-575), one lane per output
//   arm_iir_lattice_f32                 lattice_step per sample (arm_iir_lattice_f32.c:348-447)
//   arm_biquad_cascade_df1_f32          b0 x + b1 x1 + b2 x2 + a1 y1 + a2 y2 per stage
//                                       (arm_biquad_cascade_df1_f32.c:178-418)
//   arm_cfft_f32                        cfft_core (uhsdr_cfft.h) with the wrapper's input
//                                       conjugation, bit reversal and 1/L scaling
//                                       (TransformFunctions/arm_cfft_f32.c:574-628)
//   arm_cmplx_mag_f32                   sqrtf(re * re + im * im) (arm_cmplx_mag_f32.c:84-170)
// The recursive filters (lattice, biquad) are sequential in time: one lane runs the block.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
#include <math.h>
#include "uhsdr_internal.h"
#include "uhsdr_dsp.h"
#include "uhsdr_cfft.h"
#include "../../include/uhsdr_cmsis.h"

namespace {

constexpr int SHIM_THREADS = 256;
constexpr int MAX_LATTICE_STAGES = 256;

__global__ void __launch_bounds__(SHIM_THREADS) shim_fir(const float* __restrict__ x, const float* __restrict__ c,
                                                         float* __restrict__ y, int T, int nout, int M)
{
    const int m = blockIdx.x * SHIM_THREADS + threadIdx.x;
    if (m >= nout) return;
    const float* w = x + (size_t)M * m;
    float acc = 0.0f;
    for (int k = 0; k < T; ++k) acc += w[k] * c[k];
    y[m] = acc;
}

__global__ void __launch_bounds__(SHIM_THREADS) shim_interp(const float* __restrict__ x, const float* __restrict__ c,
                                                            float* __restrict__ y, int L, int ph, int B)
{
    const int o = blockIdx.x * SHIM_THREADS + threadIdx.x;
    if (o >= B * L) return;
    const int n = o / L, j = o % L;
    const float* w = x + n;
    const float* cc = c + (L - 1 - j);
    float sum = 0.0f;
    for (int t = 0; t < ph; ++t) sum += w[t] * cc[t * L];
    y[o] = sum;
}

// g: the S delayed values (pState[0..S-1]) in, the state after the block out
__global__ void shim_lattice(const float* __restrict__ x, float* __restrict__ y, const float* __restrict__ kc,
                             const float* __restrict__ vc, float* __restrict__ g_io, int S, int B)
{
    __shared__ float g[MAX_LATTICE_STAGES], gn[MAX_LATTICE_STAGES];
    if (threadIdx.x != 0) return;
    for (int i = 0; i < S; ++i) g[i] = g_io[i];
    for (int n = 0; n < B; ++n)
    {
        float fcurr = x[n], fnext = 0.0f, acc = 0.0f;
        for (int i = 0; i < S; ++i)
        {
            const float gcurr = g[i];
            fnext = fcurr - (kc[i] * gcurr);
            const float gnext = (fnext * kc[i]) + gcurr;
            acc += (gnext * vc[i]);
            gn[i] = gnext;
            fcurr = fnext;
        }
        acc += (fnext * vc[S]);
        for (int i = 0; i + 1 < S; ++i) g[i] = gn[i + 1];
        if (S > 0) g[S - 1] = fnext;
        y[n] = acc;
    }
    for (int i = 0; i < S; ++i) g_io[i] = g[i];
}

// st: {x[n-1], x[n-2], y[n-1], y[n-2]} per stage, in and out; y doubles as the stage buffer
__global__ void shim_biquad(const float* __restrict__ x, float* __restrict__ y, const float* __restrict__ c,
                            float* __restrict__ st, int S, int B)
{
    if (threadIdx.x != 0) return;
    const float* in = x;
    for (int s = 0; s < S; ++s)
    {
        float x1 = st[4 * s], x2 = st[4 * s + 1], y1 = st[4 * s + 2], y2 = st[4 * s + 3];
        const float* cs = c + 5 * s;
        for (int n = 0; n < B; ++n) y[n] = biquad_step(in[n], x1, x2, y1, y2, cs);
        st[4 * s] = x1; st[4 * s + 1] = x2; st[4 * s + 2] = y1; st[4 * s + 3] = y2;
        in = y;
    }
}

__global__ void __launch_bounds__(SHIM_THREADS) shim_mag(const float* __restrict__ x, float* __restrict__ y, int n)
{
    const int i = blockIdx.x * SHIM_THREADS + threadIdx.x;
    if (i >= n) return;
    const float re = x[2 * i], im = x[2 * i + 1];
    const float in = (re * re) + (im * im);
    y[i] = (in >= 0.0f) ? sqrtf(in) : 0.0f;      // arm_sqrt_f32 (arm_math.h:5745-5771)
}

// one wave: p1 (interleaved complex, L points) in place
template <int L>
__global__ void __launch_bounds__(64) shim_cfft(float* __restrict__ p1, const uhsdr_spectrum_plan* __restrict__ P,
                                                int ifft, int bitrev)
{
    using G = SpecGeom<L>;
    constexpr int K = G::K, NBF = G::NBF, R3 = G::R3;
    __shared__ __attribute__((aligned(16))) float S[G::FRAME];
    const int lane = threadIdx.x;
    float2 z[K];
#pragma unroll
    for (int k = 0; k < K; ++k)
    {
        const float2 v = ((const float2*)p1)[lane + 64 * k];
        z[k] = ifft ? make_float2(v.x, -v.y) : v;          // conjugate input (arm_cfft_f32.c:583-592)
    }
    float2 y[R3][8];
    cfft_core<L>(z, (float2*)S, P->twiddle, &P->tw_lane[0][0][0], lane, y);
    wave_sync();                                          // every lane has read the frame
    const float invL = 1.0f / (float)L;
#pragma unroll
    for (int r = 0; r < R3; ++r)
    {
        const int q = lane + 64 * r;
        if (q < NBF)
        {
#pragma unroll
            for (int k = 0; k < 8; ++k)
            {
                const int pos = 8 * q + k;
                const int dst = bitrev ? (int)P->iperm[pos] : pos;
                float2 v = y[r][k];
                if (ifft)                                 // conjugate and scale (:616-627)
                {
                    v.x = v.x * invL;
                    v.y = -(v.y) * invL;
                }
                ((float2*)p1)[dst] = v;
            }
        }
    }
}

// ---- per-thread device context ----
struct ShimCtx
{
    hipStream_t stream = nullptr;
    void* buf = nullptr;
    size_t cap = 0;
    uhsdr_spectrum_plan* plans[3] = { nullptr, nullptr, nullptr };   // 256, 512, 1024
};

thread_local ShimCtx t_ctx;
thread_local int32_t t_status = 0;

int fail(int32_t st, const char* what, hipError_t e)
{
    t_status = st;
    uhsdr_set_error("%s: %s", what, e == hipSuccess ? "invalid argument" : hipGetErrorString(e));
    return -1;
}

// device scratch of at least n floats
float* scratch(size_t n)
{
    ShimCtx& c = t_ctx;
    if (!c.stream && hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking) != hipSuccess) return nullptr;
    const size_t bytes = n * sizeof(float);
    if (bytes > c.cap)
    {
        if (c.buf) (void)hipFree(c.buf);
        c.buf = nullptr;
        c.cap = 0;
        size_t want = bytes < (1u << 20) ? (1u << 20) : bytes;
        if (hipMalloc(&c.buf, want) != hipSuccess) return nullptr;
        c.cap = want;
    }
    return (float*)c.buf;
}

// copy the host segments into one device buffer: returns the device base (segments at the
// offsets given, in floats), or null
struct Seg { const float* src; size_t n; };

float* upload(const Seg* segs, int nseg, size_t total, size_t* offs)
{
    float* d = scratch(total);
    if (!d) return nullptr;
    size_t o = 0;
    for (int i = 0; i < nseg; ++i)
    {
        offs[i] = o;
        if (segs[i].n && segs[i].src &&
            hipMemcpyAsync(d + o, segs[i].src, segs[i].n * sizeof(float), hipMemcpyHostToDevice, t_ctx.stream) != hipSuccess)
            return nullptr;
        o += (segs[i].n + 3) & ~(size_t)3;           // 16-byte aligned segments
    }
    return d;
}

size_t seg_total(const Seg* segs, int nseg)
{
    size_t t = 0;
    for (int i = 0; i < nseg; ++i) t += (segs[i].n + 3) & ~(size_t)3;
    return t;
}

bool finish(float* host, const float* dev, size_t n)
{
    if (n && hipMemcpyAsync(host, dev, n * sizeof(float), hipMemcpyDeviceToHost, t_ctx.stream) != hipSuccess)
        return false;
    return hipStreamSynchronize(t_ctx.stream) == hipSuccess;
}

unsigned grid(size_t n) { return (unsigned)((n + SHIM_THREADS - 1) / SHIM_THREADS); }

// FIR / decimator body: window = the T-1 carried samples + the block; new carried samples =
// the window's last T-1 (written to pState[0..T-2] as CMSIS leaves them)
void fir_run(float* pState, const float* pCoeffs, const float* pSrc, float* pDst, int T, int B, int M)
{
    t_status = 0;
    if (!pState || !pCoeffs || !pSrc || !pDst || T <= 0 || M <= 0) { fail(UHSDR_ARGUMENT_ERROR, "arm_fir", hipSuccess); return; }
    const int nout = B / M;
    if (B <= 0) return;
    // device layout: the window [T-1 carried samples | block] (contiguous), taps, outputs
    const size_t coff = ((size_t)T - 1 + B + 3) & ~(size_t)3, yoff = coff + (((size_t)T + 3) & ~(size_t)3);
    float* d = scratch(yoff + (size_t)nout);
    if (!d) { fail(UHSDR_DEVICE_ERROR, "arm_fir scratch", hipGetLastError()); return; }
    hipError_t e = hipSuccess;
    if (T > 1) e = hipMemcpyAsync(d, pState, sizeof(float) * (T - 1), hipMemcpyHostToDevice, t_ctx.stream);
    if (e == hipSuccess) e = hipMemcpyAsync(d + T - 1, pSrc, sizeof(float) * B, hipMemcpyHostToDevice, t_ctx.stream);
    if (e == hipSuccess) e = hipMemcpyAsync(d + coff, pCoeffs, sizeof(float) * T, hipMemcpyHostToDevice, t_ctx.stream);
    float* dy = d + yoff;
    if (e != hipSuccess) { fail(UHSDR_DEVICE_ERROR, "arm_fir upload", e); return; }
    hipLaunchKernelGGL(shim_fir, dim3(grid(nout)), dim3(SHIM_THREADS), 0, t_ctx.stream, d, d + coff, dy, T, nout, M);
    e = hipGetLastError();
    // carried samples for the next call: the last T-1 of the device window [history | block],
    // which still holds this call's input -- the reference decimates and filters in place
    // (pSrc == pDst, audio_driver.c:2744-2745, 2751-2752, 2803), so pSrc may already hold outputs
    // once finish() has copied them back
    if (e == hipSuccess && T > 1)
        e = hipMemcpyAsync(pState, d + B, sizeof(float) * (T - 1), hipMemcpyDeviceToHost, t_ctx.stream);
    if (e != hipSuccess || !finish(pDst, dy, nout)) { fail(UHSDR_DEVICE_ERROR, "arm_fir", e); return; }
}

template <int L>
int cfft_run(float* p1, int ifft, int bitrev)
{
    ShimCtx& c = t_ctx;
    const int idx = L == 256 ? 0 : L == 512 ? 1 : 2;
    float* d = scratch(2 * L);
    if (!d) return fail(UHSDR_DEVICE_ERROR, "arm_cfft_f32 scratch", hipGetLastError());
    if (!c.plans[idx])
    {
        uhsdr_spectrum_config cfg;
        uhsdr_spectrum_config_default(&cfg);
        cfg.fft_len = L;
        uhsdr_spectrum_plan* hp = (uhsdr_spectrum_plan*)malloc(sizeof(uhsdr_spectrum_plan));
        if (!hp || uhsdr_spectrum_plan_build(&cfg, hp) != UHSDR_OK) { free(hp); return fail(UHSDR_UNSUPPORTED, "arm_cfft_f32 plan", hipSuccess); }
        void* dp = nullptr;
        const hipError_t e = hipMalloc(&dp, sizeof(uhsdr_spectrum_plan));
        if (e != hipSuccess || hipMemcpy(dp, hp, sizeof(uhsdr_spectrum_plan), hipMemcpyHostToDevice) != hipSuccess)
        {
            free(hp);
            if (dp) (void)hipFree(dp);
            return fail(UHSDR_DEVICE_ERROR, "arm_cfft_f32 plan upload", e);
        }
        free(hp);
        c.plans[idx] = (uhsdr_spectrum_plan*)dp;
    }
    hipError_t e = hipMemcpyAsync(d, p1, sizeof(float) * 2 * L, hipMemcpyHostToDevice, c.stream);
    if (e != hipSuccess) return fail(UHSDR_DEVICE_ERROR, "arm_cfft_f32 upload", e);
    hipLaunchKernelGGL(shim_cfft<L>, dim3(1), dim3(64), 0, c.stream, d, c.plans[idx], ifft, bitrev);
    if ((e = hipGetLastError()) != hipSuccess || !finish(p1, d, 2 * L)) return fail(UHSDR_DEVICE_ERROR, "arm_cfft_f32", e);
    return 0;
}

} // namespace

extern "C" {

int32_t uhsdr_cmsis_last_status(void) { return t_status; }

void arm_fir_init_f32(arm_fir_instance_f32* S, uint16_t numTaps, float32_t* pCoeffs, float32_t* pState,
                      uint32_t blockSize)
{
    S->numTaps = numTaps;
    S->pCoeffs = pCoeffs;
    S->pState = pState;
    memset(pState, 0, (numTaps + (blockSize - 1u)) * sizeof(float32_t));
}

void arm_fir_f32(const arm_fir_instance_f32* S, float32_t* pSrc, float32_t* pDst, uint32_t blockSize)
{
    if (!S) { fail(UHSDR_ARGUMENT_ERROR, "arm_fir_f32", hipSuccess); return; }
    fir_run(S->pState, S->pCoeffs, pSrc, pDst, S->numTaps, (int)blockSize, 1);
}

arm_status arm_fir_decimate_init_f32(arm_fir_decimate_instance_f32* S, uint16_t numTaps, uint8_t M,
                                     float32_t* pCoeffs, float32_t* pState, uint32_t blockSize)
{
    if (M == 0 || (blockSize % M) != 0u) return ARM_MATH_LENGTH_ERROR;
    S->numTaps = numTaps;
    S->pCoeffs = pCoeffs;
    memset(pState, 0, (numTaps + (blockSize - 1u)) * sizeof(float32_t));
    S->pState = pState;
    S->M = M;
    return ARM_MATH_SUCCESS;
}

void arm_fir_decimate_f32(const arm_fir_decimate_instance_f32* S, float32_t* pSrc, float32_t* pDst,
                          uint32_t blockSize)
{
    if (!S) { fail(UHSDR_ARGUMENT_ERROR, "arm_fir_decimate_f32", hipSuccess); return; }
    fir_run(S->pState, S->pCoeffs, pSrc, pDst, S->numTaps, (int)blockSize, S->M);
}

arm_status arm_fir_interpolate_init_f32(arm_fir_interpolate_instance_f32* S, uint8_t L, uint16_t numTaps,
                                        float32_t* pCoeffs, float32_t* pState, uint32_t blockSize)
{
    if (L == 0 || (numTaps % L) != 0u) return ARM_MATH_LENGTH_ERROR;
    S->L = L;
    S->pCoeffs = pCoeffs;
    S->phaseLength = numTaps / L;
    memset(pState, 0, (blockSize + ((uint32_t)S->phaseLength - 1u)) * sizeof(float32_t));
    S->pState = pState;
    return ARM_MATH_SUCCESS;
}

void arm_fir_interpolate_f32(const arm_fir_interpolate_instance_f32* S, float32_t* pSrc, float32_t* pDst,
                             uint32_t blockSize)
{
    t_status = 0;
    if (!S || !S->pState || !S->pCoeffs || !pSrc || !pDst || !S->L || !S->phaseLength)
    { fail(UHSDR_ARGUMENT_ERROR, "arm_fir_interpolate_f32", hipSuccess); return; }
    const int L = S->L, ph = S->phaseLength, B = (int)blockSize;
    if (B <= 0) return;
    const size_t nw = (size_t)ph - 1 + B, woff = 0, coff = (nw + 3) & ~(size_t)3, yoff = coff + (((size_t)L * ph + 3) & ~(size_t)3);
    float* d = scratch(yoff + (size_t)B * L);
    if (!d) { fail(UHSDR_DEVICE_ERROR, "arm_fir_interpolate_f32 scratch", hipGetLastError()); return; }
    hipError_t e = hipSuccess;
    if (ph > 1) e = hipMemcpyAsync(d + woff, S->pState, sizeof(float) * (ph - 1), hipMemcpyHostToDevice, t_ctx.stream);
    if (e == hipSuccess) e = hipMemcpyAsync(d + woff + ph - 1, pSrc, sizeof(float) * B, hipMemcpyHostToDevice, t_ctx.stream);
    if (e == hipSuccess) e = hipMemcpyAsync(d + coff, S->pCoeffs, sizeof(float) * L * ph, hipMemcpyHostToDevice, t_ctx.stream);
    if (e != hipSuccess) { fail(UHSDR_DEVICE_ERROR, "arm_fir_interpolate_f32 upload", e); return; }
    hipLaunchKernelGGL(shim_interp, dim3(grid((size_t)B * L)), dim3(SHIM_THREADS), 0, t_ctx.stream, d + woff, d + coff,
                       d + yoff, L, ph, B);
    e = hipGetLastError();
    // carried samples: the last phaseLength-1 of the device window (pSrc may alias pDst)
    if (e == hipSuccess && ph > 1)
        e = hipMemcpyAsync(S->pState, d + woff + B, sizeof(float) * (ph - 1), hipMemcpyDeviceToHost, t_ctx.stream);
    if (e != hipSuccess || !finish(pDst, d + yoff, (size_t)B * L))
    { fail(UHSDR_DEVICE_ERROR, "arm_fir_interpolate_f32", e); return; }
}

void arm_iir_lattice_init_f32(arm_iir_lattice_instance_f32* S, uint16_t numStages, float32_t* pkCoeffs,
                              float32_t* pvCoeffs, float32_t* pState, uint32_t blockSize)
{
    S->numStages = numStages;
    S->pkCoeffs = pkCoeffs;
    S->pvCoeffs = pvCoeffs;
    memset(pState, 0, (numStages + blockSize) * sizeof(float32_t));
    S->pState = pState;
}

void arm_iir_lattice_f32(const arm_iir_lattice_instance_f32* S, float32_t* pSrc, float32_t* pDst, uint32_t blockSize)
{
    t_status = 0;
    if (!S || !S->pState || !S->pkCoeffs || !S->pvCoeffs || !pSrc || !pDst || S->numStages > MAX_LATTICE_STAGES)
    { fail(UHSDR_ARGUMENT_ERROR, "arm_iir_lattice_f32", hipSuccess); return; }
    const int NS = S->numStages, B = (int)blockSize;
    if (B <= 0) return;
    const Seg segs[5] = { { pSrc, (size_t)B }, { nullptr, (size_t)B }, { S->pkCoeffs, (size_t)NS },
                          { S->pvCoeffs, (size_t)NS + 1 }, { S->pState, (size_t)NS } };
    size_t offs[5];
    float* d = upload(segs, 5, seg_total(segs, 5), offs);
    if (!d) { fail(UHSDR_DEVICE_ERROR, "arm_iir_lattice_f32 upload", hipGetLastError()); return; }
    hipLaunchKernelGGL(shim_lattice, dim3(1), dim3(64), 0, t_ctx.stream, d + offs[0], d + offs[1], d + offs[2],
                       d + offs[3], d + offs[4], NS, B);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess && NS) e = hipMemcpyAsync(S->pState, d + offs[4], sizeof(float) * NS, hipMemcpyDeviceToHost, t_ctx.stream);
    if (e != hipSuccess || !finish(pDst, d + offs[1], B)) { fail(UHSDR_DEVICE_ERROR, "arm_iir_lattice_f32", e); return; }
}

void arm_biquad_cascade_df1_init_f32(arm_biquad_casd_df1_inst_f32* S, uint8_t numStages, float32_t* pCoeffs,
                                     float32_t* pState)
{
    S->numStages = numStages;
    S->pCoeffs = pCoeffs;
    memset(pState, 0, (4u * (uint32_t)numStages) * sizeof(float32_t));
    S->pState = pState;
}

void arm_biquad_cascade_df1_f32(const arm_biquad_casd_df1_inst_f32* S, float32_t* pSrc, float32_t* pDst,
                                uint32_t blockSize)
{
    t_status = 0;
    if (!S || !S->pState || !S->pCoeffs || !pSrc || !pDst) { fail(UHSDR_ARGUMENT_ERROR, "arm_biquad_cascade_df1_f32", hipSuccess); return; }
    const int NS = (int)S->numStages, B = (int)blockSize;
    if (B <= 0 || NS <= 0) return;
    const Seg segs[4] = { { pSrc, (size_t)B }, { nullptr, (size_t)B }, { S->pCoeffs, (size_t)5 * NS },
                          { S->pState, (size_t)4 * NS } };
    size_t offs[4];
    float* d = upload(segs, 4, seg_total(segs, 4), offs);
    if (!d) { fail(UHSDR_DEVICE_ERROR, "arm_biquad_cascade_df1_f32 upload", hipGetLastError()); return; }
    hipLaunchKernelGGL(shim_biquad, dim3(1), dim3(64), 0, t_ctx.stream, d + offs[0], d + offs[1], d + offs[2],
                       d + offs[3], NS, B);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpyAsync(S->pState, d + offs[3], sizeof(float) * 4 * NS, hipMemcpyDeviceToHost, t_ctx.stream);
    if (e != hipSuccess || !finish(pDst, d + offs[1], B)) { fail(UHSDR_DEVICE_ERROR, "arm_biquad_cascade_df1_f32", e); return; }
}

void arm_cfft_f32(const arm_cfft_instance_f32* S, float32_t* p1, uint8_t ifftFlag, uint8_t bitReverseFlag)
{
    t_status = 0;
    if (!S || !p1) { fail(UHSDR_ARGUMENT_ERROR, "arm_cfft_f32", hipSuccess); return; }
    const int ifft = ifftFlag == 1u, bitrev = bitReverseFlag != 0;
    switch (S->fftLen)
    {
    case 256: cfft_run<256>(p1, ifft, bitrev); break;
    case 512: cfft_run<512>(p1, ifft, bitrev); break;
    case 1024: cfft_run<1024>(p1, ifft, bitrev); break;
    default: fail(UHSDR_UNSUPPORTED, "arm_cfft_f32: fftLen not 256 / 512 / 1024", hipSuccess); break;
    }
}

void arm_cmplx_mag_f32(float32_t* pSrc, float32_t* pDst, uint32_t numSamples)
{
    t_status = 0;
    if (!pSrc || !pDst) { fail(UHSDR_ARGUMENT_ERROR, "arm_cmplx_mag_f32", hipSuccess); return; }
    const int n = (int)numSamples;
    if (n <= 0) return;
    const Seg segs[2] = { { pSrc, 2 * (size_t)n }, { nullptr, (size_t)n } };
    size_t offs[2];
    float* d = upload(segs, 2, seg_total(segs, 2), offs);
    if (!d) { fail(UHSDR_DEVICE_ERROR, "arm_cmplx_mag_f32 upload", hipGetLastError()); return; }
    hipLaunchKernelGGL(shim_mag, dim3(grid(n)), dim3(SHIM_THREADS), 0, t_ctx.stream, d + offs[0], d + offs[1], n);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess || !finish(pDst, d + offs[1], n)) { fail(UHSDR_DEVICE_ERROR, "arm_cmplx_mag_f32", e); return; }
}

} // extern "C"
