// Microbenchmark: does a launch with hipExtAnyOrderLaunch (AQL barrier bit clear) start before
// the previous kernel on the same stream has finished on gfx950?  Kernel A spins ~200 us on the
// wall clock and records its start / end; kernel B records its start; kernel C (default launch)
// records its start.  B.start < A.end means B overlapped A on one stream.
// Build: hipcc --offload-arch=gfx950 -O3 tools/micro/any_order.hip -o tools/micro/any_order
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdio.h>

__global__ void spin(long long* t, int slot, long long ticks)
{
    if (threadIdx.x != 0) return;
    const long long t0 = wall_clock64();
    long long t1 = t0;
    while (t1 - t0 < ticks) t1 = wall_clock64();   // bounded: ticks of the 100 MHz wall clock
    t[2 * slot] = t0;
    t[2 * slot + 1] = t1;
}

static void run(unsigned flags_b)
{
    long long* t;
    hipMalloc(&t, 8 * sizeof(long long));
    hipMemset(t, 0, 8 * sizeof(long long));
    hipStream_t s;
    hipStreamCreate(&s);
    hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s, t, 3, 10LL);   // warm-up
    hipStreamSynchronize(s);
    hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s, t, 0, 20000LL);           // A: 200 us
    hipError_t e = hipSuccess;
    hipExtLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s, nullptr, nullptr, flags_b, t, 1, 10LL);   // B
    e = hipGetLastError();
    hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s, t, 2, 10LL);              // C
    hipStreamSynchronize(s);
    long long h[8];
    hipMemcpy(h, t, sizeof h, hipMemcpyDeviceToHost);
    printf("flags=%u launch=%s: A [0, %lld] B start %lld  C start %lld (wall ticks from A.start) -> B %s A\n",
           flags_b, hipGetErrorString(e), h[1] - h[0], h[2] - h[0], h[4] - h[0],
           h[2] < h[1] ? "OVERLAPPED" : "after");
    hipStreamDestroy(s);
    hipFree(t);
}

int main()
{
    run(0);
    run(hipExtAnyOrderLaunch);
    return 0;
}
