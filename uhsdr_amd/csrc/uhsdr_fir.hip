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
//                    K = T + 15 rounded up to 4 (+3 % MACs at 513 taps), on
//                    v_mfma_f32_16x16x4_f32.  That instruction is an fmaf chain in k order
//                    (cdna_hip_programming.md §3), so every output is the reference's tap-ordered
//                    sum with each multiply-add fused: within ~1e-7 * sum|c x| of it, not
//                    bit-identical (tests/test_gpu_fir.py: 1e-5 relative, north_star's bar).
//
// Layout: one wave owns FIR_CPW = 4 channels (4 independent MFMA accumulators hide the
// 40-cycle dependent latency); each channel's window [T-1 carried | B new | 32 zero] sits in
// LDS with one pad word per 16 (fpad), so the 16 rows of an A fragment (stride 16 samples)
// land in distinct banks; the taps sit once per workgroup in LDS with 16 zeros on each side,
// so the B fragment c[k - i] is one LDS read per lane.  B % 256 == 0; a channel's block is
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
constexpr int FIR_CPW = 4;      // channels per wave
constexpr int FIR_TAIL = 32;    // zero samples after a window (K round-up, EXACT chunk over-read)

typedef float f32x4 __attribute__((ext_vector_type(4)));

__host__ __device__ constexpr int fpad(int i) { return i + (i >> 4); }

struct FirArgs
{
    const float* taps;   // [T]
    float* hist;         // [C][T-1] carried samples (oldest first)
    const float* src;    // [C][B]
    float* dst;          // [C][B]
    int C, B, T, K;      // K: MFMA depth, T + 15 rounded up to 4
    int lw;              // LDS floats per channel window
    int cp;              // LDS floats of the padded tap copy
};

// the tiles of one channel group from its LDS windows Wb (4 channels from c0)
template <bool MFMA>
__device__ __forceinline__ void fir_group(const FirArgs& a, const float* Wb, const float* cp, int c0, int lane)
{
    const int r = lane & 15, kq = lane >> 4;
    for (int t = 0; t < a.B / FIR_TILE; ++t)
    {
        const int base = FIR_TILE * t;
        if constexpr (MFMA)
        {
            // A[m = r][k] = w[base + 16r + k0 + kq]; B[k][i = r] = c[k0 + kq - r]
            f32x4 acc[FIR_CPW];
#pragma unroll
            for (int j = 0; j < FIR_CPW; ++j) acc[j] = f32x4{ 0.0f, 0.0f, 0.0f, 0.0f };
            const float* bp = cp + 16 + kq - r;
            const int ab = base + 16 * r + kq;
            // fpad(ab + k0) for k0 = 16q + s, s in {0, 4, 8, 12}: kq + s < 16, so the padded
            // address is a0 + 17q + s -- per 16-deep chunk one pointer step, the four k-steps
            // and the four channels as immediate LDS offsets
            const float* ap = Wb + fpad(ab);
            const int nq = a.K / 16;
            for (int q = 0; q < nq; ++q, ap += 17, bp += 16)
            {
#pragma unroll
                for (int s = 0; s < 16; s += 4)
                {
                    const float bv = bp[s];
#pragma unroll
                    for (int j = 0; j < FIR_CPW; ++j)
                        acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(ap[j * a.lw + s], bv, acc[j], 0, 0, 0);
                }
            }
            for (int k0 = 16 * nq; k0 < a.K; k0 += 4)      // K % 16 tail
            {
                const float bv = cp[16 + kq - r + k0];
#pragma unroll
                for (int j = 0; j < FIR_CPW; ++j)
                    acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(Wb[j * a.lw + fpad(ab + k0)], bv, acc[j], 0, 0, 0);
            }
            // D[row = 4 kq + i][col = r] is output 16 row + col of the tile
#pragma unroll
            for (int j = 0; j < FIR_CPW; ++j)
            {
                const int c = c0 + j;
                if (c >= a.C) continue;
                float* d = a.dst + (size_t)c * a.B + base + 64 * kq + r;
#pragma unroll
                for (int i = 0; i < 4; ++i) d[16 * i] = acc[j][i];
            }
        }
        else
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

// One group per wave, windows filled straight from HBM (EXACT: VALU-bound, the fill hides behind
// the other waves; the persistent form's prefetch registers cost it 20 %)
template <bool MFMA>
__global__ void __launch_bounds__(256) fir_batch_direct(FirArgs a)
{
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const int H = a.T - 1, n = H + a.B;
    float* cp = sm;
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
    fir_group<MFMA>(a, Wb, cp, c0, lane);
}

// floats of a channel's window each lane carries in registers between groups (n <= 64 * FIR_NPL)
constexpr int FIR_NPL = 16;

// Persistent: each wave walks channel groups g = wave, wave + waves in grid, ...  The next
// group's window (carried samples + block) is loaded into registers while the current group's
// tiles run from LDS, then written into the wave's LDS windows -- the HBM latency of the fill
// hides behind the MFMA (or VALU) chain instead of stalling the wave between groups.
template <bool MFMA>
__global__ void __launch_bounds__(256) fir_batch(FirArgs a)
{
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const int H = a.T - 1, n = H + a.B;
    float* cp = sm;                                   // cp[16 + k] = c[k], zeros around
    for (int i = threadIdx.x; i < a.cp; i += blockDim.x)
        cp[i] = (i >= 16 && i < 16 + a.T) ? a.taps[i - 16] : 0.0f;
    float* Wb = sm + a.cp + (size_t)w * FIR_CPW * a.lw;
    // windows: [carried samples | block | zero tail]; the tail is written once
#pragma unroll
    for (int j = 0; j < FIR_CPW; ++j)
        for (int i = n + lane; i < n + FIR_TAIL; i += 64) Wb[j * a.lw + fpad(i)] = 0.0f;
    __syncthreads();                                  // taps (whole workgroup) ready
    const int ng = (a.C + FIR_CPW - 1) / FIR_CPW;
    const int nwt = gridDim.x * nw;
    float pf[FIR_CPW][FIR_NPL];
    auto fetch = [&](int g) {
#pragma unroll
        for (int j = 0; j < FIR_CPW; ++j)
        {
            const int c = g * FIR_CPW + j;
            const int cl = c < a.C ? c : a.C - 1;     // loads clamped: no exec-masked load branches
            const float* h = a.hist + (size_t)cl * H;
            const float* s = a.src + (size_t)cl * a.B;
#pragma unroll
            for (int k = 0; k < FIR_NPL; ++k)
            {
                const int i = lane + 64 * k;
                const int is = i - H < a.B ? i - H : a.B - 1;
                pf[j][k] = *(i < H ? h + i : s + is);
            }
        }
    };
    int g = blockIdx.x * nw + w;
    if (g < ng) fetch(g);
    for (; g < ng; g += nwt)
    {
        wave_sync();                                  // every lane is done with the last group's windows
#pragma unroll
        for (int j = 0; j < FIR_CPW; ++j)
#pragma unroll
            for (int k = 0; k < FIR_NPL; ++k)
            {
                const int i = lane + 64 * k;
                if (i < n) Wb[j * a.lw + fpad(i)] = pf[j][k];
            }
        wave_sync();
        if (g + nwt < ng) fetch(g + nwt);             // in flight while this group computes
        const int c0 = g * FIR_CPW;
        // the next call's carried samples: the window's last T-1
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
        fir_group<MFMA>(a, Wb, cp, c0, lane);
    }
}

} // namespace

struct uhsdr_fir_s
{
    int C, B, T, K, mode, lw, cp, waves, grid;
    hipStream_t stream;
    float* taps;
    float* hist;
};

#define HIPCHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { uhsdr_set_error("%s: %s", #x, hipGetErrorString(e_)); return UHSDR_DEVICE_ERROR; } } while (0)

static size_t fir_lds(const uhsdr_fir_s* h, int waves)
{
    return sizeof(float) * ((size_t)h->cp + (size_t)waves * FIR_CPW * h->lw);
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
    if (waves != 1 && waves != 2 && waves != 4)
    {
        uhsdr_set_error("waves per workgroup %d not 1, 2 or 4", waves);
        return UHSDR_ARGUMENT_ERROR;
    }
    if (!strict)
        while (waves > 1 && fir_lds(h, waves) > 64 * 1024) waves /= 2;
    if (fir_lds(h, waves) > 64 * 1024 || h->T - 1 + h->B > 64 * FIR_NPL)
    {
        uhsdr_set_error("num_taps - 1 + block_size %d too long for %d waves per workgroup", h->T - 1 + h->B, waves);
        return UHSDR_LENGTH_ERROR;
    }
    // persistent grid: as many workgroups as the CUs hold at once (LDS-limited), each wave
    // walking channel groups
    int dev = 0, cus = 256;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
        cus = prop.multiProcessorCount;
    const size_t lds = fir_lds(h, waves);
    int per_cu = (int)((160 * 1024) / lds);
    const int thread_cap = 2048 / (64 * waves);
    if (per_cu > thread_cap) per_cu = thread_cap;
    if (per_cu < 1) per_cu = 1;
    const int groups = (h->C + FIR_CPW - 1) / FIR_CPW;
    const int need = (groups + waves - 1) / waves;
    // MFMA: persistent (C5 0.69 -> 0.40 ms per call); EXACT: fir_batch_direct, one
    // group per wave (0.99 ms; 1.20 in the persistent form)
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
    h->K = (num_taps + 15 + 3) & ~3;
    h->stream = (hipStream_t)stream;
    h->lw = (fpad(num_taps - 1 + block_size + FIR_TAIL) + 4) & ~3;
    h->cp = (h->K + 16 + 16 + 3) & ~3;
    // waves per workgroup: EXACT 2 (one group per wave, more resident waves per CU: C5 513-tap
    // 1.048 -> 0.927 ms per call), MFMA 4 (persistent; 0.395 ms vs 0.497 at 2);
    // uhsdr_fir_set_waves picks 1, 2 or 4 explicitly
    const uhsdr_status st = fir_configure(h, mode == UHSDR_FIR_MFMA ? 4 : 2, false);
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
    a.C = h->C; a.B = h->B; a.T = h->T; a.K = h->K; a.lw = h->lw; a.cp = h->cp;
    const dim3 grid(h->grid), block(64 * h->waves);
    if (h->mode == UHSDR_FIR_MFMA)
        hipLaunchKernelGGL(fir_batch<true>, grid, block, fir_lds(h, h->waves), h->stream, a);
    else
        hipLaunchKernelGGL(fir_batch_direct<false>, grid, block, fir_lds(h, h->waves), h->stream, a);
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
