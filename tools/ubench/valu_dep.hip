// Micro-benchmark: issue rate of gfx950 VALU bit ops for 1/2/4/8 independent
// chains at 1..8 waves per SIMD (256 CUs x 4 SIMDs): v_bitop3_b32 with three
// VGPR sources, with two VGPRs + one SGPR, and v_xor_b32 (two VGPRs).
// Question it answers for the bitsliced AES kernel: what a wave and a SIMD
// can issue, and how much a chain-shaped (minimum-register) order costs.
// Prints cycles per VALU instruction per SIMD over the whole grid (span of
// s_memtime from the first wave start to the last wave end: one wave's own
// time is biased, since the SIMD's issue arbiter favours older waves).
#include <hip/hip_runtime.h>
#include <cstdio>

template <int CHAINS, int OP>
__global__ __launch_bounds__(256) void k_chain(unsigned *out, int iters, unsigned sk, unsigned long long *cyc)
{
    unsigned a[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = threadIdx.x * (2 * j + 1);
    const unsigned b = threadIdx.x ^ 0x1234u, c = threadIdx.x ^ 0x9876u;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < 16 / CHAINS; ++k) {
#pragma unroll
            for (int j = 0; j < CHAINS; ++j) {
                if (OP == 0) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a[j]) : "v"(b), "v"(c));
                if (OP == 1) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a[j]) : "v"(b), "s"(sk));
                if (OP == 2) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[j]) : "v"(b));
            }
        }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    unsigned r = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) r ^= a[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
    if ((threadIdx.x & 63) == 0) { /* s_memtime is per XCD: span per XCD (workgroups go round-robin) */
        atomicMin(&cyc[2 * (blockIdx.x & 7)], t0);
        atomicMax(&cyc[2 * (blockIdx.x & 7) + 1], t1);
    }
}

template <int C, int OP>
void run(int cus, int wps, unsigned *out, unsigned long long *cyc)
{
    const int iters = 20000;
    dim3 g(cus * wps), b(256); /* 256 threads = one wave per SIMD per workgroup */
    unsigned long long init[16];
    for (int x = 0; x < 8; ++x) { init[2 * x] = ~0ull; init[2 * x + 1] = 0ull; }
    hipLaunchKernelGGL((k_chain<C, OP>), g, b, 0, 0, out, iters, 0x5555u, cyc);
    hipDeviceSynchronize();
    hipMemcpy(cyc, init, 128, hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL((k_chain<C, OP>), g, b, 0, 0, out, iters, 0x5555u, cyc);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned long long hc[16];
    hipMemcpy(hc, cyc, 128, hipMemcpyDeviceToHost);
    double span = 0;
    for (int x = 0; x < 8; ++x) span += (double)(hc[2 * x + 1] - hc[2 * x]) / 8;
    const double n = (double)iters * 16 * wps; /* wave-instructions per SIMD */
    static const char *nm[] = {"bitop3_vvv", "bitop3_vvs", "xor_vv"};
    printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"chains\": %d, \"simd_cycles_per_instr\": %.3f, "
           "\"tick_ghz\": %.3f, \"ms\": %.3f}\n", nm[OP], wps, C, span / n, span / (ms * 1e6), ms);
}

template <int OP>
void sweep(int cus, unsigned *out, unsigned long long *cyc)
{
    for (int wps : {1, 2, 3, 4, 6, 8}) {
        run<1, OP>(cus, wps, out, cyc);
        run<2, OP>(cus, wps, out, cyc);
        run<4, OP>(cus, wps, out, cyc);
        run<8, OP>(cus, wps, out, cyc);
    }
}

int main()
{
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0) != hipSuccess) return 1;
    unsigned *out;
    unsigned long long *cyc;
    if (hipMalloc(&out, (size_t)cus * 8 * 256 * 4) != hipSuccess || hipMalloc(&cyc, 128) != hipSuccess) return 1;
    sweep<0>(cus, out, cyc);
    sweep<1>(cus, out, cyc);
    sweep<2>(cus, out, cyc);
    return 0;
}
