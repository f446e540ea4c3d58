// Microbenchmark: cycles per VALU instruction for K independent dependent chains of v_add_f32 /
// v_mul_f32 per wave, with W waves per SIMD (one workgroup of 64*W lanes per CU, 4 SIMDs).
// Build: hipcc --offload-arch=gfx950 -O3 tools/micro/dep_latency.hip -o tools/micro/dep_latency
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int K, bool VY>
__global__ void chain(float* out, float ys, int iters, long long* cyc)
{
    float y = ys;
    if (VY) asm volatile("v_mov_b32 %0, %1" : "=v"(y) : "s"(ys));   // operand in a VGPR
    float x[K];
#pragma unroll
    for (int k = 0; k < K; ++k) x[k] = threadIdx.x * 1e-3f + k;
    const long long t0 = wall_clock64(), c0 = clock64();
    for (int i = 0; i < iters; ++i)
    {
#pragma unroll
        for (int r = 0; r < 32; ++r)
#pragma unroll
            for (int k = 0; k < K; ++k) x[k] = x[k] * y + y;   // mul + add (no contraction: -ffp-contract=off)
    }
    const long long c1 = clock64();
    float s = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) s += x[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = c1 - c0;
    (void)t0;
}

template <int K, bool VY>
void run(int waves)
{
    float* out; long long* cyc;
    const int blocks = 256, iters = 2000;
    hipMalloc(&out, sizeof(float) * blocks * 64 * waves * 4);
    hipMalloc(&cyc, sizeof(long long) * blocks);
    hipLaunchKernelGGL((chain<K, VY>), dim3(blocks), dim3(64 * 4 * waves), 0, 0, out, 0.999f, 10, cyc);
    hipDeviceSynchronize();
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL((chain<K, VY>), dim3(blocks), dim3(64 * 4 * waves), 0, 0, out, 0.999f, iters, cyc);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    long long c[1]; hipMemcpy(c, cyc, sizeof(long long), hipMemcpyDeviceToHost);
    const double instr_per_wave = (double)iters * 32 * K * 2;
    printf("%s K=%d waves/SIMD=%d: %.2f cycles per instr per wave (clock64), SIMD-wide %.2f; %.3f ms\n", VY ? "vgpr" : "sgpr", K, waves,
           (double)c[0] / instr_per_wave, (double)c[0] / instr_per_wave / waves, ms);
    hipFree(out); hipFree(cyc);
}

int main()
{
    for (int w : { 1, 2, 3, 4, 8 })
    {
        run<1, false>(w); run<2, false>(w); run<4, false>(w); run<8, false>(w);
        run<1, true>(w); run<2, true>(w); run<4, true>(w); run<8, true>(w);
    }
    return 0;
}
