// Microbenchmark: VALU issue rate of packed f32 (v_pk_mul_f32 / v_pk_add_f32) vs scalar
// v_mul_f32 / v_add_f32 on gfx950, many waves per SIMD, independent chains.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float v2 __attribute__((ext_vector_type(2)));
constexpr int ITERS = 4096;

__global__ void k_scalar(float* out, float m, float a)
{
    float x[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = threadIdx.x + i;
    for (int it = 0; it < ITERS; ++it)
    {
#pragma unroll
        for (int i = 0; i < 16; ++i)
        {
            asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x[i]) : "s"(m));
        }
#pragma unroll
        for (int i = 0; i < 16; ++i)
        {
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[i]) : "s"(a));
        }
    }
    float s = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_packed(float* out, float m, float a)
{
    v2 x[8];
    v2 ms = v2{m, a}, as = v2{a, m};
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = v2{(float)threadIdx.x + i, (float)i};
    for (int it = 0; it < ITERS; ++it)
    {
#pragma unroll
        for (int i = 0; i < 8; ++i)
        {
            asm volatile("v_pk_mul_f32 %0, %0, %1 op_sel_hi:[1,0]" : "+v"(x[i]) : "s"(ms));
        }
#pragma unroll
        for (int i = 0; i < 8; ++i)
        {
            asm volatile("v_pk_add_f32 %0, %0, %1 op_sel_hi:[1,0]" : "+v"(x[i]) : "s"(as));
        }
    }
    float s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += x[i].x + x[i].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// packed with 64-bit VGPR second operand (per-lane coefficient pair)
__global__ void k_packed_vv(float* out, float m, float a)
{
    v2 x[8];
    v2 mm = v2{m, m * 0.5f + threadIdx.x * 1e-9f}, aa = v2{a, a};
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = v2{(float)threadIdx.x + i, (float)i};
    for (int it = 0; it < ITERS; ++it)
    {
#pragma unroll
        for (int i = 0; i < 8; ++i)
        {
            asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(x[i]) : "v"(mm));
        }
#pragma unroll
        for (int i = 0; i < 8; ++i)
        {
            asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(x[i]) : "v"(aa));
        }
    }
    float s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += x[i].x + x[i].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main()
{
    float* out;
    const int blocks = 256 * 4 * 8, threads = 256;   // 8 waves of 256-thread blocks per SIMD... oversubscribed
    hipMalloc(&out, (size_t)blocks * threads * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    for (int rep = 0; rep < 2; ++rep)
    for (int w = 0; w < 3; ++w)
    {
        hipEventRecord(e0);
        if (w == 0) k_scalar<<<blocks, threads>>>(out, 0.999f, 0.5f);
        else if (w == 1) k_packed<<<blocks, threads>>>(out, 0.999f, 0.5f);
        else k_packed_vv<<<blocks, threads>>>(out, 0.999f, 0.5f);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        double lane_flops = (double)blocks * threads * ITERS * 32.0;  // 16 mul+16 add per iter
        double winstr = (double)blocks * threads / 64 * ITERS * (w == 0 ? 32 : 16);
        printf("%s: %.3f ms  %.1f Tflop/s (lane ops)  %.2f cycles/instr/SIMD @2.4GHz\n",
               w == 0 ? "scalar v_mul+v_add" : (w == 1 ? "packed (sgpr)" : "packed (vgpr)"), ms,
               lane_flops / ms / 1e9, ms * 1e-3 * 2.4e9 * 1024 / winstr);
    }
    return 0;
}
