// Micro-benchmark: relative issue cost of the gfx950 VALU instructions a
// bitsliced AES kernel can build its S-box, MixColumns and bit-matrix
// transposes from.  Every op runs as 8 independent dependency chains per
// wave at 4 waves per SIMD (the whole chip), so latency is hidden and the
// time measures issue cost.  Printed: ns per launch and the cost relative to
// v_xor_b32 (1.0 = same issue rate).  Question it answers: which transpose /
// linear-layer forms are cheaper than their instruction count suggests.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

enum {
    OP_XOR,
    OP_BITOP3,
    OP_BFI,
    OP_PERM,
    OP_LSHL,
    OP_LSHL_OR,
    OP_ALIGNBIT,
    OP_AND_OR,
    OP_LSHL_B64,
    OP_PK_MOV,
    OP_PERMLANE32,
    OP_PERMLANE16,
    OP_XOR_DPP,
    OP_N
};
static const char *names[OP_N] = {"v_xor_b32",        "v_bitop3_b32",      "v_bfi_b32",         "v_perm_b32",
                                  "v_lshlrev_b32",    "v_lshl_or_b32",     "v_alignbit_b32",    "v_and_or_b32",
                                  "v_lshlrev_b64",    "v_pk_mov_b32",      "v_permlane32_swap", "v_permlane16_swap",
                                  "v_xor_b32_dpp_row_shr1"};

template <int OP>
__global__ __launch_bounds__(256) void k_op(unsigned *out, int iters)
{
    unsigned a[8];
    uint64_t q[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        a[j] = threadIdx.x * (2 * j + 1);
        q[j] = (uint64_t)a[j] * 0x9E3779B97F4A7C15ull;
    }
    const unsigned b = threadIdx.x ^ 0x1234u, c = threadIdx.x ^ 0x9876u;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < 2; ++k) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if (OP == OP_XOR) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[j]) : "v"(b));
                if (OP == OP_BITOP3) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a[j]) : "v"(b), "v"(c));
                if (OP == OP_BFI) asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(a[j]) : "v"(b), "v"(c));
                if (OP == OP_PERM) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b), "v"(c));
                if (OP == OP_LSHL) asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(a[j]));
                if (OP == OP_LSHL_OR) asm volatile("v_lshl_or_b32 %0, %0, 3, %1" : "+v"(a[j]) : "v"(b));
                if (OP == OP_ALIGNBIT) asm volatile("v_alignbit_b32 %0, %0, %1, 4" : "+v"(a[j]) : "v"(b));
                if (OP == OP_AND_OR) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b), "v"(c));
                if (OP == OP_LSHL_B64) asm volatile("v_lshlrev_b64 %0, 3, %0" : "+v"(q[j]));
                if (OP == OP_PK_MOV) asm volatile("v_pk_mov_b32 %0, %0, %0 op_sel:[1,0]" : "+v"(q[j]));
                if (OP == OP_PERMLANE32) {
                    if (j & 1) continue;
                    asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(a[j]), "+v"(a[j + 1]));
                }
                if (OP == OP_PERMLANE16) {
                    if (j & 1) continue;
                    asm volatile("v_permlane16_swap_b32 %0, %1" : "+v"(a[j]), "+v"(a[j + 1]));
                }
                if (OP == OP_XOR_DPP)
                    asm volatile("v_xor_b32_dpp %0, %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(a[j]) : "v"(b));
            }
        }
    }
    unsigned r = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) r ^= a[j] ^ (unsigned)q[j] ^ (unsigned)(q[j] >> 32);
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int OP>
double run(int cus, unsigned *out)
{
    const int iters = 20000;
    dim3 g(cus * 4), b(256); /* 4 waves per SIMD */
    hipLaunchKernelGGL(k_op<OP>, g, b, 0, 0, out, iters);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
        hipEventRecord(e0);
        hipLaunchKernelGGL(k_op<OP>, g, b, 0, 0, out, iters);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    /* instructions issued per wave: permlane ops issue 8 per 16 slots */
    const double per = (OP == OP_PERMLANE32 || OP == OP_PERMLANE16) ? 8.0 : 16.0;
    return best / per;
}

template <int OP>
void all(int cus, unsigned *out, double *r)
{
    r[OP] = run<OP>(cus, out);
    if constexpr (OP + 1 < OP_N) all<OP + 1>(cus, out, r);
}

int main()
{
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0) != hipSuccess) return 1;
    unsigned *out;
    if (hipMalloc(&out, (size_t)cus * 4 * 256 * 4) != hipSuccess) return 1;
    double r[OP_N];
    all<0>(cus, out, r);
    for (int o = 0; o < OP_N; ++o)
        printf("{\"op\": \"%s\", \"ms_per_16_slots\": %.4f, \"cost_vs_xor\": %.3f}\n", names[o], r[o] * 16.0,
               r[o] / r[OP_XOR]);
    return 0;
}
