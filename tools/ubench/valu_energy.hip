// Micro-benchmark: VALU throughput of one instruction form run for a fixed
// wall time over the whole chip (8 independent chains per wave, 4 waves per
// SIMD), so that scripts/energy_probe.sh can sample socket power and clocks
// (amd-smi) while it runs and derive energy per wave-instruction.
//
//   valu_energy OP SECONDS      OP in: xor_vv bitop3_vvv bitop3_vvs and_vv
//                               bfi_vvv perm_vvv lshl_vi and_or_vvv ds_read_b32 ds_read_u8
//                               ds_addr nop
// Prints one JSON line: wave-instructions per second of the chip.
// Question it answers for the bitsliced AES kernel (power-limited): does a
// 3-VGPR-operand v_bitop3_b32 cost more energy than a 2-operand v_xor_b32,
// i.e. is the LUT3 cover (fewer, wider ops) also the lower-energy circuit?
// Round 4 adds ds_read_u8 (the same conflict-free lookups, one byte each) and
// ds_addr (their address arithmetic alone, no LDS access) to split a T-table
// lookup's energy into LDS access and VALU, and to price a byte-table (S-box
// in LDS, MixColumns in VALU) AES against the 32-bit T-table.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

enum { XOR_VV, BITOP3_VVV, BITOP3_VVS, AND_VV, BFI_VVV, PERM_VVV, LSHL_VI, AND_OR_VVV, DS_READ, DS_READ_U8, DS_ADDR,
       NOP, NOPS };
static const char *names[NOPS] = {"xor_vv",  "bitop3_vvv", "bitop3_vvs", "and_vv",      "bfi_vvv",    "perm_vvv",
                                  "lshl_vi", "and_or_vvv", "ds_read_b32", "ds_read_u8", "ds_addr",    "nop"};

template <int OP>
__global__ __launch_bounds__(256) void k_op(unsigned *out, int iters, unsigned sk)
{
    unsigned a[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = threadIdx.x * (2 * j + 1) + blockIdx.x;
    const unsigned b = threadIdx.x ^ 0x1234u, c = threadIdx.x ^ 0x9876u;
    /* ds_read_b32: 32 KiB per workgroup, lane l reads bank l mod 32 of a
     * data-dependent row (conflict-free, like the T-table kernel's lookups) */
    __shared__ unsigned lds[8192];
    if (OP == DS_READ || OP == DS_READ_U8) {
        for (int q = threadIdx.x; q < 8192; q += 256) lds[q] = q * 2654435761u;
        __syncthreads();
    }
    const unsigned lane_off = threadIdx.x & 31u;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if (OP == XOR_VV) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[j]) : "v"(b));
                if (OP == BITOP3_VVV) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a[j]) : "v"(b), "v"(c));
                if (OP == BITOP3_VVS) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a[j]) : "v"(b), "s"(sk));
                if (OP == AND_VV) asm volatile("v_and_b32 %0, %0, %1" : "+v"(a[j]) : "v"(b));
                if (OP == BFI_VVV) asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(a[j]) : "v"(b), "v"(c));
                if (OP == PERM_VVV) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b), "v"(c));
                if (OP == LSHL_VI) asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(a[j]));
                if (OP == AND_OR_VVV) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b), "v"(c));
                if (OP == DS_READ) /* 8 chains in flight, one wait per round of them (hipcc) */
                    a[j] = lds[((a[j] & 0xFFu) << 5) | lane_off];
                if (OP == DS_READ_U8) /* byte (a >> 8) & 3 of the same dword: same bank, one byte */
                    a[j] = ((const unsigned char *)lds)[((((a[j] & 0xFFu) << 5) | lane_off) << 2) | ((a[j] >> 8) & 3u)] +
                           (a[j] << 8);
                if (OP == DS_ADDR) { /* the ds_read_b32 chain's address arithmetic alone */
                    unsigned ad = ((a[j] & 0xFFu) << 5) | lane_off;
                    asm volatile("" : "+v"(ad));
                    a[j] = ad ^ (a[j] >> 3);
                }
                if (OP == NOP) asm volatile("s_nop 0" : "+v"(a[j]));
            }
        }
    }
    unsigned r = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) r ^= a[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int OP>
static double run(int cus, unsigned *out, double seconds)
{
    const int iters = 4000; /* 128k wave-instructions per wave per launch */
    dim3 g(cus * 4), b(256);
    hipLaunchKernelGGL(k_op<OP>, g, b, 0, 0, out, iters, 0x5555u);
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    long launches = 0;
    const auto t0 = std::chrono::steady_clock::now();
    double el = 0;
    while (el < seconds) {
        for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(k_op<OP>, g, b, 0, 0, out, iters, 0x5555u);
        if (hipDeviceSynchronize() != hipSuccess) return -1;
        launches += 20;
        el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    }
    const double waves = (double)cus * 16; /* 4 workgroups of 4 waves per CU */
    return launches * waves * iters * 32.0 / el;
}

int main(int argc, char **argv)
{
    if (argc < 3) {
        fprintf(stderr, "usage: valu_energy OP SECONDS\n");
        return 2;
    }
    int op = -1;
    for (int i = 0; i < NOPS; ++i)
        if (!strcmp(argv[1], names[i])) op = i;
    const double secs = atof(argv[2]);
    int cus = 0;
    if (op < 0 || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0) != hipSuccess) return 2;
    unsigned *out;
    if (hipMalloc(&out, (size_t)cus * 4 * 256 * 4) != hipSuccess) return 1;
    double r = -1;
    switch (op) {
    case XOR_VV: r = run<XOR_VV>(cus, out, secs); break;
    case BITOP3_VVV: r = run<BITOP3_VVV>(cus, out, secs); break;
    case BITOP3_VVS: r = run<BITOP3_VVS>(cus, out, secs); break;
    case AND_VV: r = run<AND_VV>(cus, out, secs); break;
    case BFI_VVV: r = run<BFI_VVV>(cus, out, secs); break;
    case PERM_VVV: r = run<PERM_VVV>(cus, out, secs); break;
    case LSHL_VI: r = run<LSHL_VI>(cus, out, secs); break;
    case AND_OR_VVV: r = run<AND_OR_VVV>(cus, out, secs); break;
    case DS_READ: r = run<DS_READ>(cus, out, secs); break;
    case DS_READ_U8: r = run<DS_READ_U8>(cus, out, secs); break;
    case DS_ADDR: r = run<DS_ADDR>(cus, out, secs); break;
    case NOP: r = run<NOP>(cus, out, secs); break;
    }
    if (r < 0) return 1;
    printf("{\"op\": \"%s\", \"seconds\": %.1f, \"wave_instr_per_s\": %.4e}\n", names[op], secs, r);
    return 0;
}
