// Microbenchmark: issue rate of VOP2 (32-bit encoded) vs VOP3 / VOP3P f32 instructions on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float v2 __attribute__((ext_vector_type(2)));
constexpr int ITERS = 4096;

#define KERNEL(name, BODY)                                                   \
__global__ void name(float* out, float m, float a)                           \
{                                                                            \
    float x[16]; v2 y[8];                                                     \
    v2 ms = v2{m, a};                                                        \
    _Pragma("unroll") for (int i = 0; i < 16; ++i) x[i] = threadIdx.x + i;   \
    _Pragma("unroll") for (int i = 0; i < 8; ++i) y[i] = v2{(float)threadIdx.x, (float)i}; \
    for (int it = 0; it < ITERS; ++it) { BODY }                              \
    float s = 0;                                                             \
    _Pragma("unroll") for (int i = 0; i < 16; ++i) s += x[i];                \
    _Pragma("unroll") for (int i = 0; i < 8; ++i) s += y[i].x + y[i].y;      \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;                          \
}

KERNEL(k_vop2_s, _Pragma("unroll") for (int i = 0; i < 16; ++i) asm volatile("v_mul_f32_e32 %0, %1, %0" : "+v"(x[i]) : "s"(m));
                 _Pragma("unroll") for (int i = 0; i < 16; ++i) asm volatile("v_add_f32_e32 %0, %1, %0" : "+v"(x[i]) : "s"(a));)
KERNEL(k_vop3_s, _Pragma("unroll") for (int i = 0; i < 16; ++i) asm volatile("v_mul_f32_e64 %0, %0, %1" : "+v"(x[i]) : "s"(m));
                 _Pragma("unroll") for (int i = 0; i < 16; ++i) asm volatile("v_add_f32_e64 %0, %0, %1" : "+v"(x[i]) : "s"(a));)
KERNEL(k_vop2_v, _Pragma("unroll") for (int i = 0; i < 16; ++i) asm volatile("v_mul_f32_e32 %0, %1, %0" : "+v"(x[i]) : "v"(x[(i + 1) & 15]));
                 _Pragma("unroll") for (int i = 0; i < 16; ++i) asm volatile("v_add_f32_e32 %0, %1, %0" : "+v"(x[i]) : "v"(x[(i + 3) & 15]));)
KERNEL(k_pk_s,   _Pragma("unroll") for (int i = 0; i < 8; ++i) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(y[i]) : "s"(ms));
                 _Pragma("unroll") for (int i = 0; i < 8; ++i) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(y[i]) : "s"(ms));)
KERNEL(k_pk_v,   _Pragma("unroll") for (int i = 0; i < 8; ++i) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(y[i]) : "v"(y[(i + 1) & 7]));
                 _Pragma("unroll") for (int i = 0; i < 8; ++i) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(y[i]) : "v"(y[(i + 3) & 7]));)
KERNEL(k_mov,    _Pragma("unroll") for (int i = 0; i < 16; ++i) asm volatile("v_mov_b32_e32 %0, %1" : "=v"(x[i]) : "v"(x[(i + 1) & 15]));
                 _Pragma("unroll") for (int i = 0; i < 16; ++i) asm volatile("v_mov_b32_e32 %0, %1" : "=v"(x[i]) : "v"(x[(i + 5) & 15]));)

int main()
{
    float* out;
    const int blocks = 256 * 4 * 8, threads = 256;
    (void)hipMalloc(&out, (size_t)blocks * threads * 4);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    const char* names[] = { "vop2 sgpr (v_mul/v_add_e32)", "vop3 sgpr (_e64)", "vop2 vgpr", "pk sgpr", "pk vgpr", "v_mov_b32" };
    for (int rep = 0; rep < 2; ++rep)
        for (int w = 0; w < 6; ++w)
        {
            (void)hipEventRecord(e0);
            switch (w)
            {
            case 0: k_vop2_s<<<blocks, threads>>>(out, 0.999f, 0.5f); break;
            case 1: k_vop3_s<<<blocks, threads>>>(out, 0.999f, 0.5f); break;
            case 2: k_vop2_v<<<blocks, threads>>>(out, 0.999f, 0.5f); break;
            case 3: k_pk_s<<<blocks, threads>>>(out, 0.999f, 0.5f); break;
            case 4: k_pk_v<<<blocks, threads>>>(out, 0.999f, 0.5f); break;
            default: k_mov<<<blocks, threads>>>(out, 0.999f, 0.5f); break;
            }
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms; (void)hipEventElapsedTime(&ms, e0, e1);
            const double winstr = (double)blocks * threads / 64 * ITERS * (w == 3 || w == 4 ? 16 : 32);
            printf("%-30s %.3f ms  %.2f cycles/instr/SIMD @2.4GHz\n", names[w], ms, ms * 1e-3 * 2.4e9 * 1024 / winstr);
        }
    return 0;
}
