// Exhaustive device check of a short division for atanf's reduction quotient (uhsdr_libm.h
// ul_atanf_pos): for every binary32 a in [7/16, 2^25) -- the operands that reach the division --
// num = fma(ka, a, -kb) and den = kb a + ka as ul_atanf_pos forms them, and
//   q = fma(fma(-den, num * r, num), r, num * r),  r = v_rcp_f32(den)
// against the IEEE quotient num / den.  Prints the number of operands where the bits differ.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/micro/atan_div_check tools/micro/atan_div_check.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>

__device__ __forceinline__ float short_div(float num, float den)
{
    const float r = __builtin_amdgcn_rcpf(den);
    const float q0 = num * r;
    const float e = fmaf(-den, q0, num);
    return fmaf(e, r, q0);
}

__global__ void check(uint32_t lo, uint32_t n, unsigned* bad, uint32_t* first)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t ia = lo + i;
    const float a = __uint_as_float(ia);
    const int lo2 = ia < 0x3f980000u, i0 = ia < 0x3f300000u, i2 = ia < 0x401c0000u;
    const float ka = i0 ? 2.0f : (i2 ? 1.0f : 0.0f);
    const float kb = (!lo2 && i2) ? 1.5f : 1.0f;
    const float num = fmaf(ka, a, -kb);
    const float den = kb * a + ka;
    const float q = num / den;
    const float s = short_div(num, den);
    if (__float_as_uint(q) != __float_as_uint(s))
    {
        atomicAdd(bad, 1u);
        atomicMin(first, ia);
    }
}

int main()
{
    const uint32_t lo = 0x3ee00000u, hi = 0x4c000000u, n = hi - lo;
    unsigned* bad; uint32_t* first;
    hipMalloc(&bad, 4); hipMalloc(&first, 4);
    hipMemset(bad, 0, 4);
    const uint32_t ff = 0xffffffffu;
    hipMemcpy(first, &ff, 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(check, dim3((n + 255) / 256), dim3(256), 0, 0, lo, n, bad, first);
    unsigned hb = 0; uint32_t hf = 0;
    hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
    hipMemcpy(&hf, first, 4, hipMemcpyDeviceToHost);
    if (hipGetLastError() != hipSuccess) { printf("hip error\n"); return 2; }
    float fa; memcpy(&fa, &hf, 4);
    printf("operands %u, differing %u, first 0x%08x (%g)\n", n, hb, hf, hb ? fa : 0.0f);
    return 0;
}
