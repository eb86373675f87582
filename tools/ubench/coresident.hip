// Co-residency probe for the claimed splits: can a workgroup of kernel B
// start on a CU while a workgroup of kernel A (persistent, one per CU) runs
// there?  The splits (csrc/hip/engine.cpp split_claim) assume a T-table
// workgroup (1024 threads, 128 KiB LDS, 4 waves per SIMD) and one bitsliced
// wave per SIMD share every CU; a claim-counter readback showed the bitsliced
// side taking no unit when the T-table kernel holds every CU.
//
// A: AT threads, LDS_A bytes of LDS, ~VA VGPRs (a clobbered high register),
//    waits (s_sleep) until the host sets *stop or ~0.5 s pass (wall clock),
//    so a probe never hangs the GPU.
// B: 256 threads (one wave per SIMD), ~VB VGPRs, no LDS: every workgroup
//    adds 1 to *started and exits.
// Host: A on stream 1 (grid = CUs), 20 ms later B on stream 2 (grid = CUs),
// 20 ms later read *started (pinned host memory, system-scope atomics), then
// release A.  Prints one JSON line per configuration.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <thread>

#define CHK(x)                                                                                    \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) {                                                                   \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                              \
            return 1;                                                                             \
        }                                                                                         \
    } while (0)

template <int VA>
__device__ __forceinline__ void clobber()
{
    if constexpr (VA >= 160) asm volatile("" ::: "v159");
    else if constexpr (VA >= 88) asm volatile("" ::: "v87");
    else if constexpr (VA >= 64) asm volatile("" ::: "v63");
    else asm volatile("" ::: "v31");
}

template <int S>
__device__ __forceinline__ void sclobber()
{
    if constexpr (S >= 100) asm volatile("" ::: "s99");
}

/* BUSY: instead of sleeping, A's waves run LDS lookups + VALU (the T-table
 * kernel's mix) between their stop-flag polls */
template <int AT, int LDS_A, int VA, int SA = 0, bool BUSY = false>
__global__ __launch_bounds__(AT) void k_a(unsigned *started, const unsigned *stop, unsigned *sink)
{
    extern __shared__ unsigned dyn[];
    if (LDS_A) {
        for (int i = threadIdx.x; i < LDS_A / 4; i += AT) dyn[i] = i * 2654435761u;
        __syncthreads();
    }
    clobber<VA>();
    sclobber<SA>();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(started, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const unsigned long long t0 = wall_clock64();
    unsigned x = threadIdx.x, acc = 0;
    while (!__hip_atomic_load(stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) && wall_clock64() - t0 < 50000000ull) {
        if (BUSY && LDS_A) {
#pragma unroll 1
            for (int k = 0; k < 256; ++k) {
                const unsigned a = dyn[(x & 0xFFu) << 5 | (threadIdx.x & 31)];
                const unsigned b = dyn[((x >> 8) & 0xFFu) << 5 | (threadIdx.x & 31)];
                x = __builtin_amdgcn_bitop3_b32(a, b, x, 0x96) + k;
                acc ^= x;
            }
        } else {
            __builtin_amdgcn_s_sleep(100);
        }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

template <int VB, int SB = 0>
__global__ __launch_bounds__(256) void k_b(unsigned *started)
{
    clobber<VB>();
    sclobber<SB>();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(started, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

/* how B is issued: 0 = A on s1, B on s2 20 ms later; 1 = A on the NULL
 * stream, B right after on a non-blocking stream that first waits on an
 * event recorded on the NULL stream before A (the library's fork); 2 = the
 * same with A on a non-blocking stream */
template <int AT, int LDS_A, int VA, int VB, int SA = 0, int SB = 0, int HOW = 0, bool BUSY = false>
static int probe(int cus, unsigned *h)
{
    hipStream_t s1, s2;
    CHK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CHK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    hipEvent_t fork;
    CHK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
    if (HOW == 1 || HOW == 3) s1 = nullptr;
    /* HOW 3: as 1 with three more streams alive, each given a kernel so its
     * hardware queue is created (GPU_MAX_HW_QUEUES = 4 on the box) */
    hipStream_t extra[3] = {nullptr, nullptr, nullptr};
    if (HOW == 3)
        for (auto &x : extra) {
            CHK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
            hipLaunchKernelGGL((k_b<32, 0>), dim3(1), dim3(64), 0, x, &h[3]);
            CHK(hipStreamSynchronize(x));
        }
    for (int i = 0; i < 4; ++i) __atomic_store_n(&h[i], 0u, __ATOMIC_SEQ_CST);
    if (LDS_A) CHK(hipFuncSetAttribute((const void *)k_a<AT, LDS_A, VA, SA, BUSY>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_A));
    if (HOW) {
        CHK(hipEventRecord(fork, s1));
        CHK(hipStreamWaitEvent(s2, fork, 0));
    }
    hipLaunchKernelGGL((k_a<AT, LDS_A, VA, SA, BUSY>), dim3(cus), dim3(AT), LDS_A, s1, &h[0], &h[2], &h[4]);
    CHK(hipGetLastError());
    if (!HOW) std::this_thread::sleep_for(std::chrono::milliseconds(20));
    hipLaunchKernelGGL((k_b<VB, SB>), dim3(cus), dim3(256), 0, s2, &h[1]);
    CHK(hipGetLastError());
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
    const unsigned a = __atomic_load_n(&h[0], __ATOMIC_SEQ_CST), b = __atomic_load_n(&h[1], __ATOMIC_SEQ_CST);
    __atomic_store_n(&h[2], 1u, __ATOMIC_SEQ_CST);
    CHK(hipStreamSynchronize(s1));
    CHK(hipStreamSynchronize(s2));
    printf("{\"busy\": %d, \"how\": %d, \"a_threads\": %d, \"a_lds\": %d, \"a_vgpr\": %d, \"b_vgpr\": %d, \"a_sgpr\": %d, \"b_sgpr\": %d, "
           "\"cus\": %d, \"a_started\": %u, \"b_started_beside_a\": %u, \"b_total\": %u}\n",
           (int)BUSY, HOW, AT, LDS_A, VA, VB, SA, SB, cus, a, b, __atomic_load_n(&h[1], __ATOMIC_SEQ_CST));
    fflush(stdout);
    if (s1) CHK(hipStreamDestroy(s1));
    for (auto x : extra)
        if (x) CHK(hipStreamDestroy(x));
    CHK(hipStreamDestroy(s2));
    CHK(hipEventDestroy(fork));
    return 0;
}

int main()
{
    int cus = 0;
    CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    unsigned *h = nullptr;
    CHK(hipHostMalloc((void **)&h, 64, hipHostMallocDefault));
    int r = 0;
    r |= probe<1024, 131072, 88, 160, 100, 100, 1, true>(cus, h); /* A busy with LDS + VALU, the library's sequence */
    r |= probe<1024, 131072, 88, 160, 100, 100, 0, true>(cus, h); /* A busy, B 20 ms later */
    r |= probe<1024, 131072, 88, 160, 100, 100, 3>(cus, h); /* ... with every hardware queue in use */
    r |= probe<1024, 131072, 88, 160, 100, 100, 1>(cus, h); /* the library's launch sequence */
    r |= probe<1024, 131072, 88, 160, 100, 100, 2>(cus, h);
    r |= probe<1024, 131072, 88, 160>(cus, h); /* the ECB split's shape */
    r |= probe<1024, 131072, 88, 160, 100, 100>(cus, h); /* ... with ~100 SGPRs per wave, as the real kernels */
    r |= probe<1024, 131072, 32, 32, 100, 100>(cus, h);
    r |= probe<1024, 131072, 32, 32, 0, 100>(cus, h);
    r |= probe<1024, 131072, 32, 32, 100, 0>(cus, h);
    r |= probe<1024, 0, 88, 160>(cus, h);      /* without A's LDS */
    r |= probe<1024, 131072, 32, 32>(cus, h);  /* small registers on both sides */
    r |= probe<1024, 65536, 32, 32>(cus, h);
    r |= probe<512, 131072, 32, 32>(cus, h);   /* 2 waves per SIMD in A */
    r |= probe<256, 131072, 32, 32>(cus, h);
    r |= probe<256, 0, 32, 32>(cus, h);
    CHK(hipHostFree(h));
    return r;
}
