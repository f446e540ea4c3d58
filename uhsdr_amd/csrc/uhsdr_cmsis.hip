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
//   arm_lms_norm_f32                    per sample: energy -= x0 x0, += in in; y = sum_k x[n+k] w[k]
//                                       in tap order; e = d - y; w[k] += (e mu / (energy + eps))
//                                       x[n+k]; x0 = x[n] (arm_lms_norm_f32.c:205-300)
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

// one wave: the dot product runs in lane 0 in tap order (the reference's sum), the coefficient
// update is split over the lanes (each w[k] is updated independently); w lives in LDS for the
// block.  win: [T-1 carried | B new] samples; ex: {energy, x0} in and out; w_io: coefficients in
// and out.
constexpr int MAX_LMS_TAPS = 8192;

__global__ void __launch_bounds__(64) shim_lms_norm(const float* __restrict__ win, const float* __restrict__ ref,
                                                    float* __restrict__ out, float* __restrict__ err,
                                                    float* __restrict__ w_io, float* __restrict__ ex, float mu,
                                                    int T, int B)
{
    __shared__ float w[MAX_LMS_TAPS];
    __shared__ float step;
    const int lane = threadIdx.x;
    for (int k = lane; k < T; k += 64) w[k] = w_io[k];
    float energy = ex[0], x0 = ex[1];
    __syncthreads();
    for (int n = 0; n < B; ++n)
    {
        const float* x = win + n;
        if (lane == 0)
        {
            const float in = x[T - 1];
            energy -= x0 * x0;
            energy += in * in;
            float sum = 0.0f;
            for (int k = 0; k < T; ++k) sum += x[k] * w[k];
            out[n] = sum;
            const float e = ref[n] - sum;
            err[n] = e;
            step = (e * mu) / (energy + 0.000000119209289f);
            x0 = x[0];
        }
        __syncthreads();
        const float wf = step;
        for (int k = lane; k < T; k += 64) w[k] += wf * x[k];
        __syncthreads();
    }
    for (int k = lane; k < T; k += 64) w_io[k] = w[k];
    if (lane == 0) { ex[0] = energy; ex[1] = x0; }
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

// ---- arm_cfft_f32 for the lengths the spectrum kernels do not specialise (16, 32, 64, 128, 2048,
//      4096), on the instance's own tables: one workgroup, the frame in LDS, one thread per
//      butterfly of a stage (the butterflies of a stage touch disjoint points), the binary32
//      sequence of CMSIS's arm_cfft_radix8by2_f32 / _by4_f32 (arm_cfft_f32.c:207-557) and
//      arm_radix8_butterfly_f32 (arm_cfft_radix8_f32.c:130-282) per butterfly ----
__device__ __forceinline__ void gcf_radix8(float* x, int base, int stride, const float* __restrict__ tw, int tstep)
{
    const float C81 = 0.70710678118f;
    float re[8], im[8];
#pragma unroll
    for (int k = 0; k < 8; k++) { re[k] = x[2 * (base + k * stride)]; im[k] = x[2 * (base + k * stride) + 1]; }
    float sr[4], dr[4], si[4], di[4];
#pragma unroll
    for (int k = 0; k < 4; k++)
    {
        sr[k] = re[k] + re[k + 4]; dr[k] = re[k] - re[k + 4];
        si[k] = im[k] + im[k + 4]; di[k] = im[k] - im[k + 4];
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
#pragma unroll
    for (int k = 0; k < 8; k++)
    {
        float yr = Xr[k], yi = Xi[k];
        if (tstep && k)
        {
            const float c = tw[2 * k * tstep], s = tw[2 * k * tstep + 1];
            const float p1 = c * Xr[k], p2 = s * Xi[k], p3 = c * Xi[k], p4 = s * Xr[k];
            yr = p1 + p2;
            yi = p3 - p4;
        }
        x[2 * (base + k * stride)] = yr;
        x[2 * (base + k * stride) + 1] = yi;
    }
}

// radix-8 stages over `parts` sub-arrays of n points each, twiddle modifier tm
__device__ __forceinline__ void gcf_stages(float* x, int parts, int n, const float* __restrict__ tw, int tm)
{
    for (int span = n; span >= 8; span >>= 3, tm <<= 3)
    {
        const int stride = span >> 3, nbf = n / 8;
        for (int t = threadIdx.x; t < parts * nbf; t += blockDim.x)
        {
            const int part = t / nbf, r = t % nbf, j = r % stride, g = j + (r / stride) * span;
            gcf_radix8(x + 2 * part * n, g, stride, tw, j * tm);
        }
        __syncthreads();
    }
}

__global__ void __launch_bounds__(SHIM_THREADS) shim_cfft_generic(float* __restrict__ p1, const float* __restrict__ tw,
                                                                  const uint16_t* __restrict__ perm, int L, int ifft)
{
    extern __shared__ float x[];                      // 2L floats
    for (int i = threadIdx.x; i < L; i += blockDim.x)
    {
        const float2 v = ((const float2*)p1)[i];
        x[2 * i] = v.x;
        x[2 * i + 1] = ifft ? -v.y : v.y;             // conjugate input (arm_cfft_f32.c:583-592)
    }
    __syncthreads();
    const bool by2 = L == 16 || L == 128 || L == 1024 || L == 8192;
    const bool by4 = L == 32 || L == 256 || L == 2048;
    if (by2)
    {
        // arm_cfft_radix8by2_f32 (arm_cfft_f32.c:207-317)
        const int H = L / 2, Q = L / 4;
        for (int a = threadIdx.x; a < Q; a += blockDim.x)
        {
            float* q1 = x + 2 * a;
            float* q3 = x + 2 * (a + Q);
            float* q2 = x + 2 * (a + H);
            float* q4 = x + 2 * (a + H + Q);
            const float t2r = q1[0] - q2[0], t2i = q1[1] - q2[1];
            const float t4r = q4[0] - q3[0], t4i = q4[1] - q3[1];
            q1[0] = q1[0] + q2[0];
            q1[1] = q1[1] + q2[1];
            q3[0] = q3[0] + q4[0];
            q3[1] = q3[1] + q4[1];
            const float c = tw[2 * a], s = tw[2 * a + 1];
            {
                const float m0 = t2r * c, m1 = t2i * s, m2 = t2i * c, m3 = t2r * s;
                q2[0] = m0 + m1;
                q2[1] = m2 - m3;
            }
            {
                const float m0 = t4r * s, m1 = t4i * c, m2 = t4i * s, m3 = t4r * c;
                q4[0] = m0 - m1;
                q4[1] = m2 + m3;
            }
        }
        __syncthreads();
        gcf_stages(x, 2, H, tw, 2);
    }
    else if (by4)
    {
        // arm_cfft_radix8by4_f32 (arm_cfft_f32.c:319-557): top rows t = 0 .. Q/2, bottom rows
        // Q - t for t = 1 .. Q/2 - 1 with the mirrored twiddles of t
        const int Q = L / 4;
        float* c1 = x;
        float* c2 = x + 2 * Q;
        float* c3 = x + 4 * Q;
        float* c4 = x + 6 * Q;
        for (int w = threadIdx.x; w < Q; w += blockDim.x)
        {
            if (w <= Q / 2)
            {
                const int t = w;
                float* q1 = c1 + 2 * t;
                float* q2 = c2 + 2 * t;
                float* q3 = c3 + 2 * t;
                float* q4 = c4 + 2 * t;
                const float s13r = q1[0] + q3[0], d13r = q1[0] - q3[0];
                const float s13i = q1[1] + q3[1], d13i = q1[1] - q3[1];
                const float t2r = d13r + q2[1] - q4[1], t2i = d13i - q2[0] + q4[0];
                const float t3r = s13r - q2[0] - q4[0], t3i = s13i - q2[1] - q4[1];
                const float t4r = d13r - q2[1] + q4[1], t4i = d13i + q2[0] - q4[0];
                q1[0] = s13r + q2[0] + q4[0];
                q1[1] = s13i + q2[1] + q4[1];
                if (t == 0)
                {
                    q2[0] = t2r; q2[1] = t2i;
                    q3[0] = t3r; q3[1] = t3i;
                    q4[0] = t4r; q4[1] = t4i;
                }
                else
                {
                    const float* tt[3] = { tw + 2 * t, tw + 4 * t, tw + 6 * t };
                    float* qq[3] = { q2, q3, q4 };
                    const float xr[3] = { t2r, t3r, t4r }, xi[3] = { t2i, t3i, t4i };
#pragma unroll
                    for (int k = 0; k < 3; ++k)
                    {
                        const float c = tt[k][0], s = tt[k][1];
                        const float m0 = xr[k] * c, m1 = xi[k] * s, m2 = xi[k] * c, m3 = xr[k] * s;
                        qq[k][0] = m0 + m1;
                        qq[k][1] = m2 - m3;
                    }
                }
            }
            else
            {
                const int t = Q - w, b = w;            // w = Q - t for t = 1 .. Q/2 - 1
                float* q1 = c1 + 2 * b;
                float* q2 = c2 + 2 * b;
                float* q3 = c3 + 2 * b;
                float* q4 = c4 + 2 * b;
                const float s13r = q1[0] + q3[0], d13r = q1[0] - q3[0];
                const float s13i = q1[1] + q3[1], d13i = q1[1] - q3[1];
                const float u2r = q2[1] - q4[1] + d13r;
                const float u2i = q1[1] - q3[1] - q2[0] + q4[0];
                const float u3r = s13r - q2[0] - q4[0];
                const float u3i = s13i - q2[1] - q4[1];
                const float u4r = q2[1] - q4[1] - d13r;
                const float u4i = q4[0] - q2[0] - d13i;
                q1[1] = s13i + q2[1] + q4[1];
                q1[0] = s13r + q2[0] + q4[0];
                {
                    const float c = tw[2 * t], s = tw[2 * t + 1];
                    const float m0 = u2i * s, m1 = u2r * c, m2 = u2r * s, m3 = u2i * c;
                    q2[1] = m0 - m1;
                    q2[0] = m2 + m3;
                }
                {
                    const float c = tw[4 * t], s = tw[4 * t + 1];
                    const float m0 = -u3i * c, m1 = u3r * s, m2 = u3r * c, m3 = u3i * s;
                    q3[1] = m0 - m1;
                    q3[0] = m3 - m2;
                }
                {
                    const float c = tw[6 * t], s = tw[6 * t + 1];
                    const float m0 = u4i * s, m1 = u4r * c, m2 = u4r * s, m3 = u4i * c;
                    q4[1] = m0 - m1;
                    q4[0] = m2 + m3;
                }
            }
        }
        __syncthreads();
        gcf_stages(x, 4, Q, tw, 4);
    }
    else
        gcf_stages(x, 1, L, tw, 1);                   // arm_radix8_butterfly_f32(p1, L, pTwiddle, 1)
    // bit reversal as the permutation the reference's swap sequence composes (host-built, perm null
    // without bitReverseFlag): point i of the output is point perm[i] of the transform
    const float invL = 1.0f / (float)L;
    for (int i = threadIdx.x; i < L; i += blockDim.x)
    {
        const int src = perm ? perm[i] : i;
        float re = x[2 * src], im = x[2 * src + 1];
        if (ifft)
        {
            re = re * invL;                           // arm_cfft_f32.c:617-628
            im = -im * invL;
        }
        ((float2*)p1)[i] = make_float2(re, im);
    }
}

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

// the other CMSIS lengths: the instance's twiddle (twiddleCoef_L: L complex;
// the first radix-8 stage reads up to index 7 (L/8 - 1)) and bit-reversal tables go up with
// the frame (CMSIS keeps them in the caller's arm_cfft_sR_f32_lenL instance)
int cfft_run_generic(const arm_cfft_instance_f32* S, float* p1, int ifft, int bitrev)
{
    const int L = S->fftLen;
    if (!S->pTwiddle || (bitrev && !S->pBitRevTable))
        return fail(UHSDR_ARGUMENT_ERROR, "arm_cfft_f32: instance without twiddle / bit-reversal tables", hipSuccess);
    const size_t ntw = 2 * (size_t)L, nperm = bitrev ? ((size_t)L + 1) / 2 : 0;   // uint16 pairs per float
    float* d = scratch(2 * (size_t)L + ntw + nperm);
    if (!d) return fail(UHSDR_DEVICE_ERROR, "arm_cfft_f32 scratch", hipGetLastError());
    float* dtw = d + 2 * L;
    uint16_t* dperm = bitrev ? (uint16_t*)(dtw + ntw) : nullptr;
    hipError_t e = hipMemcpyAsync(d, p1, sizeof(float) * 2 * L, hipMemcpyHostToDevice, t_ctx.stream);
    if (e == hipSuccess) e = hipMemcpyAsync(dtw, S->pTwiddle, sizeof(float) * ntw, hipMemcpyHostToDevice, t_ctx.stream);
    if (e == hipSuccess && bitrev)
    {
        // arm_bitreversal_32 (arm_bitreversal2.S:136-180): (len + 1) >> 2 iterations of two swaps of
        // the complex values at the table's byte offsets, in order -- cycles of the permutation
        // share points between swaps, so the sequence is composed here into one gather
        uint16_t* perm = (uint16_t*)malloc(sizeof(uint16_t) * L);
        if (!perm) return fail(UHSDR_DEVICE_ERROR, "arm_cfft_f32 table", hipSuccess);
        for (int i = 0; i < L; ++i) perm[i] = (uint16_t)i;
        const int it = (S->bitRevLength + 1) >> 2;
        for (int k = 0; k < 2 * it && 2 * k + 1 < S->bitRevLength; ++k)
        {
            const int ia = S->pBitRevTable[2 * k] >> 3, ib = S->pBitRevTable[2 * k + 1] >> 3;
            if (ia >= L || ib >= L) { free(perm); return fail(UHSDR_ARGUMENT_ERROR, "arm_cfft_f32: bit-reversal table", hipSuccess); }
            const uint16_t t = perm[ia]; perm[ia] = perm[ib]; perm[ib] = t;
        }
        e = hipMemcpyAsync(dperm, perm, sizeof(uint16_t) * L, hipMemcpyHostToDevice, t_ctx.stream);
        if (e == hipSuccess) e = hipStreamSynchronize(t_ctx.stream);
        free(perm);
    }
    if (e != hipSuccess) return fail(UHSDR_DEVICE_ERROR, "arm_cfft_f32 upload", e);
    hipLaunchKernelGGL(shim_cfft_generic, dim3(1), dim3(SHIM_THREADS), sizeof(float) * 2 * L, t_ctx.stream, d, dtw, dperm,
                       L, ifft);
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
    case 16: case 32: case 64: case 128: case 2048: case 4096: cfft_run_generic(S, p1, ifft, bitrev); break;
    default: fail(UHSDR_UNSUPPORTED, "arm_cfft_f32: fftLen not 16 / 32 / ... / 4096", hipSuccess); break;
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

void arm_lms_norm_init_f32(arm_lms_norm_instance_f32* S, uint16_t numTaps, float32_t* pCoeffs, float32_t* pState,
                           float32_t mu, uint32_t blockSize)
{
    S->numTaps = numTaps;
    S->pCoeffs = pCoeffs;
    memset(pState, 0, (numTaps + (blockSize - 1u)) * sizeof(float32_t));
    S->pState = pState;
    S->mu = mu;
    S->energy = 0.0f;
    S->x0 = 0.0f;
}

void arm_lms_norm_f32(arm_lms_norm_instance_f32* S, float32_t* pSrc, float32_t* pRef, float32_t* pOut,
                      float32_t* pErr, uint32_t blockSize)
{
    t_status = 0;
    if (!S || !S->pState || !S->pCoeffs || !pSrc || !pRef || !pOut || !pErr || !S->numTaps || S->numTaps > MAX_LMS_TAPS)
    { fail(UHSDR_ARGUMENT_ERROR, "arm_lms_norm_f32", hipSuccess); return; }
    const int T = S->numTaps, B = (int)blockSize;
    if (B <= 0) return;
    const float ex[2] = { S->energy, S->x0 };
    // the window [T-1 carried | block] must be contiguous: carried state and block are separate
    // host segments, so the window is one segment built from both
    const size_t nwin = (size_t)T - 1 + B;
    const Seg segs[6] = { { nullptr, nwin }, { pRef, (size_t)B }, { nullptr, (size_t)B }, { nullptr, (size_t)B },
                          { S->pCoeffs, (size_t)T }, { ex, 2 } };
    size_t offs[6];
    float* d = upload(segs, 6, seg_total(segs, 6), offs);
    hipError_t e = hipSuccess;
    if (d && T > 1) e = hipMemcpyAsync(d + offs[0], S->pState, sizeof(float) * (T - 1), hipMemcpyHostToDevice, t_ctx.stream);
    if (d && e == hipSuccess) e = hipMemcpyAsync(d + offs[0] + T - 1, pSrc, sizeof(float) * B, hipMemcpyHostToDevice, t_ctx.stream);
    if (!d || e != hipSuccess) { fail(UHSDR_DEVICE_ERROR, "arm_lms_norm_f32 upload", d ? e : hipGetLastError()); return; }
    hipLaunchKernelGGL(shim_lms_norm, dim3(1), dim3(64), 0, t_ctx.stream, d + offs[0], d + offs[1], d + offs[2],
                       d + offs[3], d + offs[4], d + offs[5], S->mu, T, B);
    e = hipGetLastError();
    // carried samples: the window's last T-1 (pErr may alias pSrc, so they come from the device)
    if (e == hipSuccess && T > 1)
        e = hipMemcpyAsync(S->pState, d + offs[0] + B, sizeof(float) * (T - 1), hipMemcpyDeviceToHost, t_ctx.stream);
    if (e == hipSuccess) e = hipMemcpyAsync(S->pCoeffs, d + offs[4], sizeof(float) * T, hipMemcpyDeviceToHost, t_ctx.stream);
    if (e == hipSuccess) e = hipMemcpyAsync(pOut, d + offs[2], sizeof(float) * B, hipMemcpyDeviceToHost, t_ctx.stream);
    float exo[2];
    if (e == hipSuccess) e = hipMemcpyAsync(exo, d + offs[5], sizeof(float) * 2, hipMemcpyDeviceToHost, t_ctx.stream);
    if (e != hipSuccess || !finish(pErr, d + offs[3], B)) { fail(UHSDR_DEVICE_ERROR, "arm_lms_norm_f32", e); return; }
    S->energy = exo[0];
    S->x0 = exo[1];
}

} // extern "C"
