// Micro-benchmark: how long does a 1024-thread workgroup take to build the
// T-table kernels' 128 KiB replicated LDS table (aes_tt.hip fill_tbl4: 8192
// ds_write_b128, each of a rotated word of a 1 KiB global table)?  256
// workgroups (one per CU), each wave records s_memrealtime at entry and
// after the fill + barrier; printed: entry->ready median / max over waves.
// Forms: the shipped loop (one 4-byte global load per 16-byte store); the
// same with the values made from the index (no global load: the store side
// alone); the table loaded once per wave (one 16-byte load per lane = the
// whole 1 KiB) and spread with ds_bpermute.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

__device__ __forceinline__ uint32_t rot(uint32_t t, int k) { return k ? ((t << (8 * k)) | (t >> (32 - 8 * k))) : t; }

template <int FORM>
__global__ __launch_bounds__(1024) void k_fill(const uint32_t *te0, unsigned long long *t, unsigned *sink)
{
    extern __shared__ uint4 l4[];
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    if (FORM == 0) { /* shipped */
        for (int q = threadIdx.x; q < 8192; q += 1024) {
            const int r = q >> 12, x = (q >> 4) & 255, half = (q >> 3) & 1;
            const uint32_t v = rot(te0[x], 2 * r + half);
            l4[q] = make_uint4(v, v, v, v);
        }
    } else if (FORM == 1) { /* no global loads */
        for (int q = threadIdx.x; q < 8192; q += 1024) {
            const int r = q >> 12, x = (q >> 4) & 255, half = (q >> 3) & 1;
            const uint32_t v = rot(x * 0x01030507u, 2 * r + half);
            l4[q] = make_uint4(v, v, v, v);
        }
    } else { /* one 1 KiB load per wave, ds_bpermute */
        const uint32_t lane = threadIdx.x & 63u;
        const uint4 w = reinterpret_cast<const uint4 *>(te0)[lane];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int q = threadIdx.x + 1024 * k;
            const int r = q >> 12, x = (q >> 4) & 255, half = (q >> 3) & 1;
            const int src = (x >> 2) << 2; /* byte address of lane x/4 */
            const uint32_t c0 = __builtin_amdgcn_ds_bpermute(src, w.x), c1 = __builtin_amdgcn_ds_bpermute(src, w.y);
            const uint32_t c2 = __builtin_amdgcn_ds_bpermute(src, w.z), c3 = __builtin_amdgcn_ds_bpermute(src, w.w);
            const int c = x & 3;
            const uint32_t tv = c == 0 ? c0 : c == 1 ? c1 : c == 2 ? c2 : c3;
            const uint32_t v = rot(tv, 2 * r + half);
            l4[q] = make_uint4(v, v, v, v);
        }
    }
    __syncthreads();
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63) == 0) {
        const int w = blockIdx.x * 16 + threadIdx.x / 64;
        t[2 * w] = t0;
        t[2 * w + 1] = t1;
    }
    if (l4[(threadIdx.x * 7) & 8191].x == 0xdeadbeefu) sink[0] = 1;
}

template <int FORM>
static void run(const char *name, int cus, const uint32_t *te0, unsigned long long *t, unsigned *sink)
{
    (void)hipFuncSetAttribute((const void *)k_fill<FORM>, hipFuncAttributeMaxDynamicSharedMemorySize, 128 << 10);
    const int n = cus * 16;
    std::vector<unsigned long long> h(2 * n);
    std::vector<double> d(n);
    for (int rep = 0; rep < 4; ++rep) {
        hipLaunchKernelGGL(k_fill<FORM>, dim3(cus), dim3(1024), 128 << 10, 0, te0, t, sink);
        if (hipDeviceSynchronize() != hipSuccess) { printf("failed %s\n", name); return; }
        if (rep == 0) continue; /* cold */
        (void)hipMemcpy(h.data(), t, h.size() * sizeof h[0], hipMemcpyDeviceToHost);
        for (int i = 0; i < n; ++i) d[i] = (h[2 * i + 1] - h[2 * i]) / 100.0;
        std::sort(d.begin(), d.end());
        printf("{\"form\": \"%s\", \"rep\": %d, \"fill_us_median\": %.2f, \"fill_us_max\": %.2f}\n", name, rep, d[n / 2],
               d[n - 1]);
    }
}

int main()
{
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0) != hipSuccess) return 1;
    uint32_t *te0;
    unsigned long long *t;
    unsigned *sink;
    std::vector<uint32_t> host(256);
    for (int i = 0; i < 256; ++i) host[i] = 0x9E3779B9u * (i + 1);
    if (hipMalloc(&te0, 1024) != hipSuccess || hipMalloc(&t, (size_t)cus * 32 * 8) != hipSuccess ||
        hipMalloc(&sink, 64) != hipSuccess)
        return 1;
    (void)hipMemcpy(te0, host.data(), 1024, hipMemcpyHostToDevice);
    run<0>("shipped_global_per_store", cus, te0, t, sink);
    run<1>("no_global_loads", cus, te0, t, sink);
    run<2>("wave_load_bpermute", cus, te0, t, sink);
    return 0;
}
