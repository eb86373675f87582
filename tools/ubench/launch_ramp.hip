// Micro-benchmark: how fast does the chip fill with one 1024-thread
// workgroup per CU (the persistent T-table claim kernels' shape)?  Each wave
// records s_memrealtime (100 MHz) when it starts; printed: the spread of
// the start times over 256 workgroups, with and without 128 KiB of dynamic
// LDS, at a small and a large VGPR budget, and the 256-thread shape of the
// bitsliced kernel for comparison.  Question it answers: is the 0-47 us
// start ramp of the persistent T-table kernel (profiles/r6/claim_tail/)
// set by the workgroup shape, its LDS, or its registers?
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

template <int VG>
__global__ __launch_bounds__(1024) void k_ramp(unsigned long long *t, unsigned *sink)
{
    extern __shared__ unsigned lds[];
    const unsigned long long now = __builtin_amdgcn_s_memrealtime();
    unsigned v[VG];
#pragma unroll
    for (int i = 0; i < VG; ++i) v[i] = threadIdx.x * (i + 1);
#pragma unroll
    for (int i = 0; i < VG; ++i) asm volatile("" : "+v"(v[i]));
    unsigned r = 0;
#pragma unroll
    for (int i = 0; i < VG; ++i) r ^= v[i];
    if ((threadIdx.x & 63) == 0) t[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = now;
    if (r == 0xdeadbeefu) { lds[threadIdx.x] = r; sink[0] = lds[(threadIdx.x + 1) & 1023]; }
}

static void run(const char *name, void (*k)(unsigned long long *, unsigned *), int wgs, int threads, size_t lds,
                unsigned long long *t, unsigned *sink)
{
    if (lds) (void)hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(k, dim3(wgs), dim3(threads), lds, 0, t, sink); /* warm */
    (void)hipDeviceSynchronize();
    const int n = wgs * threads / 64;
    std::vector<unsigned long long> h(n);
    double med_spread = 0, max_spread = 0;
    for (int rep = 0; rep < 5; ++rep) {
        hipLaunchKernelGGL(k, dim3(wgs), dim3(threads), lds, 0, t, sink);
        if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed %s\n", name); return; }
        (void)hipMemcpy(h.data(), t, n * sizeof h[0], hipMemcpyDeviceToHost);
        std::sort(h.begin(), h.end());
        med_spread += (h[n / 2] - h[0]) / 100.0 / 5;  /* 100 MHz ticks -> us */
        max_spread += (h[n - 1] - h[0]) / 100.0 / 5;
    }
    printf("{\"shape\": \"%s\", \"wgs\": %d, \"threads\": %d, \"lds\": %zu, \"waves\": %d, \"start_median_us\": %.2f, "
           "\"start_max_us\": %.2f}\n", name, wgs, threads, lds, n, med_spread, max_spread);
}

int main()
{
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0) != hipSuccess) return 1;
    unsigned long long *t;
    unsigned *sink;
    if (hipMalloc(&t, (size_t)cus * 64 * sizeof *t) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) return 1;
    run("1024thr_vg16_nolds", k_ramp<16>, cus, 1024, 0, t, sink);
    run("1024thr_vg16_lds128k", k_ramp<16>, cus, 1024, 128 << 10, t, sink);
    run("1024thr_vg80_nolds", k_ramp<80>, cus, 1024, 0, t, sink);
    run("1024thr_vg80_lds128k", k_ramp<80>, cus, 1024, 128 << 10, t, sink);
    run("1024thr_vg80_lds160k", k_ramp<80>, cus, 1024, 160 << 10, t, sink);
    run("256thr_vg16_x4_nolds", k_ramp<16>, cus * 4, 256, 0, t, sink);
    return 0;
}
