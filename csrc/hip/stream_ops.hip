/*
 * stream_ops.hip -- byte-stream kernels for gfx950:
 *   * k_xor        : the device arc4_crypt combiner, out = in ^ keystream
 *                    (reference arc4.c:101-112 / test.c:44-58 did this with
 *                    pthreads); 16 B per lane, grid-stride, HBM-bound.
 *   * k_rc4_multi  : many independent RC4 streams, one per lane, S-box in LDS
 *                    (the "P3 many-stream" design of SURVEY.md section 2.4:
 *                    RC4's PRGA is serial per stream, so GPU throughput comes
 *                    from thousands of concurrent streams).
 *   * k_fill_random / k_checksum: synthetic data + verification helpers.
 *
 * RC4 LDS layout: byte x of lane l's permutation lives in dword
 * (x >> 2) * 64 + l, byte (x & 3) -- i.e. byte address
 * ((x >> 2) << 8) | (l << 2) | (x & 3).  Every lane owns one bank (l mod 32),
 * so the data-dependent S[j] / S[S[i]+S[j]] reads of a wave never conflict.
 * 16 KiB per wave; one wave per workgroup, up to 10 workgroups per CU.
 */
#include <hip/hip_runtime.h>

#include "otc_device.h"
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

namespace {

/* One 16-byte load of each input per lane per trip: the stream already runs
 * at the HBM rate a read-read-write stream reaches here (~5 TB/s of traffic);
 * 2-8 loads per trip, 4-32 workgroups per CU and non-temporal accesses all
 * measured within noise (profiles/r1/otbench_xor_variants.jsonl). */
typedef uint32_t xu32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_xor_kernel(const uint8_t *a, const uint8_t *b, uint8_t *o, uint64_t n)
{
    const uint64_t n16 = n / 16;
    const xu32x4 *A = reinterpret_cast<const xu32x4 *>(a);
    const xu32x4 *B = reinterpret_cast<const xu32x4 *>(b);
    xu32x4 *O = reinterpret_cast<xu32x4 *>(o);
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) O[i] = A[i] ^ B[i];
    if (blockIdx.x == 0 && threadIdx.x < (n & 15)) {
        const uint64_t j = n16 * 16 + threadIdx.x;
        o[j] = a[j] ^ b[j];
    }
}

__device__ __forceinline__ uint64_t splitmix(uint64_t z)
{
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void k_fill_kernel(uint8_t *p, uint64_t n, uint64_t seed)
{
    const uint64_t n16 = n / 16;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t s = splitmix(seed);
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) {
        uint64_t a = splitmix(s ^ (2 * i)), b = splitmix(s ^ (2 * i + 1));
        reinterpret_cast<uint4 *>(p)[i] = make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32));
    }
    if (blockIdx.x == 0 && threadIdx.x < (n & 15)) {
        const uint64_t j = n16 * 16 + threadIdx.x;
        p[j] = (uint8_t)splitmix(s ^ (0xFFFFull << 48) ^ j);
    }
}

__global__ __launch_bounds__(256) void k_checksum_kernel(const uint64_t *p, uint64_t nw, unsigned long long *out)
{
    uint64_t acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nw; i += stride)
        acc ^= p[i] * (0x9E3779B97F4A7C15ull | 1) + (i << 1); /* position-dependent fold */
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc ^= __shfl_xor(acc, o, 64);
    if ((threadIdx.x & 63) == 0) atomicXor(out, (unsigned long long)acc);
}

/* ---- RC4 many-stream --------------------------------------------------- */
__device__ __forceinline__ uint32_t sbox_addr(uint32_t x, uint32_t lane4)
{
    /* ((x & 0xFC) << 6) | (x & 3) | lane4 ; bits of x above 7 are ignored */
    uint32_t t = (x << 6) & 0x3F00u;
    return t | (x & 3u) | lane4;
}

/* RC4 S-box address: byte x of lane l at ((x>>2)<<8) | l<<2 | (x&3) -- every
 * lane owns a bank (conflict-free for any data).  A byte-interleaved layout
 * ((x<<6) | l, fewer VALU per address, ~2-way conflicts) measured slower
 * (profiles/r1/otbench_rc4_bytelayout_negative.jsonl). */
__device__ __forceinline__ uint32_t rc4_addr(uint32_t x, uint32_t lane4) { return sbox_addr(x, lane4); }

/* The aligned PRGA's two byte indices per step (j and S[i] + S[j]) in three
 * VALU each instead of five: the sum masked to a byte by SDWA (dst BYTE_0,
 * zero pad), then t = x | x << 6 (bits 0-1 = x0-1, bits 8-13 = x2-7) and one
 * bit-field insert of the lane term into bits 2-7 (mask 0x3F03 in an SGPR).
 * The PRGA issues ~21 instructions per byte with the LDS pipe 25% busy
 * (profiles/r5/rc4/): +1-3% over the five-VALU form
 * (profiles/r5/rc4/ab_addr3_vs_addr5.jsonl). */
__device__ __forceinline__ uint32_t add8(uint32_t a, uint32_t b)
{
    uint32_t r;
    asm("v_add_u32_sdwa %0, %1, %2 dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:DWORD"
        : "=v"(r)
        : "v"(a), "v"(b));
    return r;
}
/* x < 256 */
__device__ __forceinline__ uint32_t rc4_addr8(uint32_t x, uint32_t lane4)
{
    uint32_t t, r;
    asm("v_lshl_or_b32 %0, %1, 6, %1" : "=v"(t) : "v"(x));
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "s"(0x3F03u), "v"(t), "v"(lane4));
    return r;
}

/* Output modes: RC4_KS = keystream only (no input); RC4_VEC = input, in/out
 * 16-byte aligned and len a multiple of 16 (host-checked), so every lane
 * uses 16-byte accesses and the input chunk is loaded one chunk ahead;
 * RC4_ANY = input with arbitrary alignment. */
enum { RC4_KS = 0, RC4_VEC = 1, RC4_ANY = 2 };

__device__ __forceinline__ void rc4_emit(const uint8_t *in, uint8_t *out, uint64_t pos, uint32_t kb, bool live)
{
    if (live) out[pos] = in ? (uint8_t)(in[pos] ^ kb) : (uint8_t)kb;
}

__device__ __forceinline__ uint4 rc4_ld16(const uint8_t *p)
{
    return *reinterpret_cast<const uint4 *>(p);
}

__device__ __forceinline__ void rc4_st16x(uint8_t *p, const uint32_t (&w)[4], uint4 x, bool live)
{
    if (live) *reinterpret_cast<uint4 *>(p) = make_uint4(w[0] ^ x.x, w[1] ^ x.y, w[2] ^ x.z, w[3] ^ x.w);
}

/* RC4_KS / RC4_ANY: 16 bytes at pos, 16-byte access where both pointers allow */
__device__ __forceinline__ void rc4_store16_any(const uint8_t *in, uint8_t *out, uint64_t pos, const uint32_t (&w)[4],
                                                bool live)
{
    if (!live) return;
    if ((((uintptr_t)(out + pos) | (in ? (uintptr_t)(in + pos) : 0)) & 15u) == 0) {
        rc4_st16x(out + pos, w, in ? rc4_ld16(in + pos) : make_uint4(0, 0, 0, 0), true);
    } else {
#pragma unroll
        for (int q = 0; q < 16; ++q) rc4_emit(in, out, pos + q, (w[q >> 2] >> (8 * (q & 3))) & 0xFFu, true);
    }
}

/* Main loop over 16-byte chunks while m + LIM <= len.  RC4_VEC: the input
 * chunk of the NEXT 16 bytes is loaded (unconditionally, at a clamped,
 * always-valid address) while the current ones are generated, in two
 * alternating registers -- a load issued at store time exposes the whole HBM
 * latency once per 16 bytes, and a register copy of a just-loaded value
 * waits for it. */
#define RC4_MAIN_LOOP(LIM, GEN16)                                                                              \
    if constexpr (MODE == RC4_VEC) {                                                                           \
        uint4 xa = make_uint4(0, 0, 0, 0), xb;                                                                 \
        if (m + (LIM) <= len) xa = rc4_ld16(in + base + m);                                                    \
        while (m + (LIM) <= len) {                                                                             \
            xb = rc4_ld16(in + base + (m + 16 < len - 16 ? m + 16 : len - 16));                                \
            {                                                                                                  \
                uint32_t w[4] = {0, 0, 0, 0};                                                                  \
                GEN16(w);                                                                                      \
                rc4_st16x(out + base + m, w, xa, live);                                                        \
            }                                                                                                  \
            m += 16;                                                                                           \
            if (m + (LIM) > len) break;                                                                        \
            xa = rc4_ld16(in + base + (m + 16 < len - 16 ? m + 16 : len - 16));                                \
            {                                                                                                  \
                uint32_t w[4] = {0, 0, 0, 0};                                                                  \
                GEN16(w);                                                                                      \
                rc4_st16x(out + base + m, w, xb, live);                                                        \
            }                                                                                                  \
            m += 16;                                                                                           \
        }                                                                                                      \
    } else {                                                                                                   \
        while (m + (LIM) <= len) {                                                                             \
            uint32_t w[4] = {0, 0, 0, 0};                                                                      \
            GEN16(w);                                                                                          \
            rc4_store16_any(in, out, base + m, w, live);                                                       \
            m += 16;                                                                                           \
        }                                                                                                      \
    }

/* PRGA: the loop of arc4_prep (reference arc4.c:72-97), one stream per lane.
 * Measured and rejected (profiles/r1/otbench_rc4_prefetch_pipe_ab.jsonl,
 * rocprof/rc4_counters.txt): a software-pipelined variant that writes each
 * swap two iterations late and corrects the reads issued before it in
 * registers (no LDS round trip left in the j chain) -- 4-8% slower: a wave
 * issues at most one instruction per 4 cycles, and the corrections add half
 * again to the ~27 instructions per byte, which bound the loop with 2 waves
 * per SIMD more than the LDS latency does. */
/* i-aligned PRGA main loop (drop % 16 == 0): every 16-byte chunk starts at
 * i = 16k, so S[i] of step q (i = 16k + q + 1) sits at a compile-time byte
 * offset from one per-chunk lane address -- the i side of every step becomes a
 * ds_read_u8 / ds_write_b8 immediate offset, with no SALU index arithmetic and
 * no VALU address op (the loop is issue-bound at ~2 waves per SIMD). */
__device__ __forceinline__ constexpr uint32_t rc4_ioff(int m) { return ((uint32_t)(m >> 2) << 8) | (uint32_t)(m & 3); }

/* AL: i-aligned loops with the S[i+1] read-ahead (drop % 16 == 0, the
 * default; +5-7% over the generic loop, profiles/r1/otbench_rc4_readahead_ab.jsonl) */
template <int MODE, bool AL>
__device__ __forceinline__ void rc4_prga(uint8_t *S, uint32_t lane4, uint32_t &i, uint32_t &j, uint64_t len,
                                               const uint8_t *in, uint8_t *out, uint64_t base, bool live)
{
#define RC4_STEP(O)                                                                                            \
    do {                                                                                                       \
        i = (i + 1) & 0xFFu;                                                                                   \
        const uint32_t ai_ = rc4_addr(i, lane4);                                                              \
        const uint32_t a_ = S[ai_];                                                                            \
        j = (j + a_) & 0xFFu;                                                                                  \
        const uint32_t aj_ = rc4_addr(j, lane4);                                                              \
        const uint32_t b_ = S[aj_];                                                                            \
        S[ai_] = (uint8_t)b_;                                                                                  \
        S[aj_] = (uint8_t)a_;                                                                                  \
        O = S[rc4_addr(a_ + b_, lane4)];                                                                      \
    } while (0)
#define RC4_GEN16(w)                                                                                           \
    _Pragma("unroll") for (int q = 0; q < 16; ++q)                                                             \
    {                                                                                                          \
        uint32_t o;                                                                                            \
        RC4_STEP(o);                                                                                           \
        w[q >> 2] |= o << (8 * (q & 3));                                                                       \
    }
    /* AL: S[i+1] read ahead together with S[j], before the swap writes, and
     * corrected when the swap moved it (i + 1 == j -> a), so the j chain
     * carries one LDS round trip per byte instead of two. */
#define RC4_GEN16P(w)                                                                                          \
    {                                                                                                          \
        uint8_t *Sk = S + ((k << 10) | lane4);                                                                 \
        const uint32_t ib = k << 4;                                                                            \
        k = (k + 1) & 15u;                                                                                     \
        uint8_t *Sn = S + ((k << 10) | lane4);                                                                 \
        const uint32_t nb = k << 4;                                                                            \
        _Pragma("unroll") for (int q = 0; q < 16; ++q)                                                         \
        {                                                                                                      \
            uint8_t *si_ = q < 15 ? Sk + rc4_ioff(q + 1) : Sn;                                                 \
            uint8_t *sp_ = q < 14 ? Sk + rc4_ioff(q + 2) : (q == 14 ? Sn : Sn + rc4_ioff(1));                            \
            const uint32_t a_ = an;                                                                            \
            j = add8(j, a_);                                                                                   \
            const uint32_t aj_ = rc4_addr8(j, lane4);                                                          \
            const uint32_t b_ = S[aj_];                                                                        \
            const uint32_t pn_ = *sp_;                                                                         \
            const uint32_t inx_ = q < 14 ? ib + (uint32_t)(q + 2) : nb + (uint32_t)(q - 14);                   \
            an = (j == inx_) ? a_ : pn_;                                                                       \
            *si_ = (uint8_t)b_;                                                                                \
            S[aj_] = (uint8_t)a_;                                                                              \
            const uint32_t o_ = S[rc4_addr8(add8(a_, b_), lane4)];                                            \
            w[q >> 2] |= o_ << (8 * (q & 3));                                                                  \
        }                                                                                                      \
    }
    uint64_t m = 0;
    if constexpr (AL) {
        uint32_t k = (i >> 4) & 15u; /* i % 16 == 0 here (host checks drop % 16) */
        uint32_t an = S[((k << 10) | lane4) + rc4_ioff(1)]; /* S[i + 1] */
        RC4_MAIN_LOOP(16, RC4_GEN16P)
        i = k << 4;
    } else {
        RC4_MAIN_LOOP(16, RC4_GEN16)
    }
    for (; m < len; ++m) {
        uint32_t o;
        RC4_STEP(o);
        rc4_emit(in, out, base + m, o, live);
    }
#undef RC4_GEN16P
#undef RC4_GEN16
#undef RC4_STEP
}

#undef RC4_MAIN_LOOP

template <int MODE, bool AL>
__global__ __launch_bounds__(64) void k_rc4_kernel(const uint8_t *keys, int keylen, uint64_t nstreams, uint64_t len,
                                                   uint64_t drop, const uint8_t *in, uint8_t *out)
{
    __shared__ __attribute__((aligned(16))) uint8_t S[64 * 256];
    const uint32_t lane = threadIdx.x;
    const uint32_t lane4 = lane << 2; /* lane term of rc4_addr */
    const uint64_t sid = (uint64_t)blockIdx.x * 64 + lane;
    const bool live = sid < nstreams;

    /* identity permutation: dword q of lane l = bytes 4q..4q+3 */
    for (uint32_t q = 0; q < 64; ++q)
        *reinterpret_cast<uint32_t *>(S + ((q << 8) | lane4)) = 0x03020100u + 0x04040404u * q;

    /* KSA (reference arc4.c:43-67) */
    const uint8_t *key = keys + (live ? sid : 0) * (uint64_t)keylen;
    uint32_t j = 0;
    if ((keylen == 1 || keylen == 2 || keylen == 4 || keylen == 8 || keylen == 16 || keylen == 32)) {
        /* key lengths dividing 32: the key is loaded once into registers (one
         * byte per VGPR, all loads in flight together) instead of one
         * dependent global byte load per KSA step, and i runs in 16-step
         * chunks whose S[i] accesses are LDS immediate offsets (+7-27%,
         * profiles/r1/otbench_rc4_ksa16_ab.jsonl). */
#define RC4_KSA_CHUNK(C, KB)                                                                                   \
    {                                                                                                          \
        uint8_t *Sc = S + (((uint32_t)(C) << 10) | lane4);                                                     \
        uint8_t *Sn = S + (((((uint32_t)(C) + 1u) & 15u) << 10) | lane4);                                      \
        const uint32_t ib = (uint32_t)(C) << 4;                                                                \
        _Pragma("unroll") for (int q = 0; q < 16; ++q)                                                         \
        {                                                                                                      \
            if constexpr (AL) { /* S[i+1] read ahead, fixed up when the swap moved it */                 \
                const uint32_t a = an;                                                                         \
                j = (j + a + (KB)[q]) & 0xFFu;                                                                 \
                const uint32_t aj = rc4_addr(j, lane4);                                                    \
                const uint32_t b = S[aj];                                                                      \
                const uint32_t pn = q < 15 ? Sc[rc4_ioff(q + 1)] : Sn[0];                                  \
                an = (j == ((ib + (uint32_t)q + 1u) & 0xFFu)) ? a : pn;                                        \
                Sc[rc4_ioff(q)] = (uint8_t)b;                                                              \
                S[aj] = (uint8_t)a;                                                                            \
            } else {                                                                                           \
                const uint32_t a = Sc[rc4_ioff(q)];                                                        \
                j = (j + a + (KB)[q]) & 0xFFu;                                                                 \
                const uint32_t aj = rc4_addr(j, lane4);                                                    \
                const uint32_t b = S[aj];                                                                      \
                Sc[rc4_ioff(q)] = (uint8_t)b;                                                              \
                S[aj] = (uint8_t)a;                                                                            \
            }                                                                                                  \
        }                                                                                                      \
    }
        uint32_t an = S[lane4]; /* S[0] */
        (void)an;
        if (keylen == 32) {
            uint32_t kb[32];
#pragma unroll
            for (int q = 0; q < 32; ++q) kb[q] = key[q];
            for (uint32_t c = 0; c < 16; c += 2) {
                RC4_KSA_CHUNK(c, kb)
                RC4_KSA_CHUNK(c + 1, kb + 16)
            }
        } else {
            const uint32_t km = (uint32_t)keylen - 1u;
            uint32_t kb[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) kb[q] = key[(uint32_t)q & km];
            for (uint32_t c = 0; c < 16; ++c) RC4_KSA_CHUNK(c, kb)
        }
#undef RC4_KSA_CHUNK
    } else {
        int kpos = 0;
        for (uint32_t i = 0; i < 256; ++i) {
            const uint32_t ai = rc4_addr(i, lane4);
            const uint32_t a = S[ai];
            j = (j + a + key[kpos]) & 0xFFu;
            if (++kpos == keylen) kpos = 0;
            const uint32_t aj = rc4_addr(j, lane4);
            const uint32_t b = S[aj];
            S[ai] = (uint8_t)b;
            S[aj] = (uint8_t)a;
        }
    }

    /* RC4-drop: discard the first `drop` keystream bytes */
    uint32_t i = 0;
    j = 0;
    uint64_t n = 0;
    if constexpr (AL) {
        /* drop % 16 == 0 here (host): 16-step chunks, i = 16c + q + 1, S[i]
         * at immediate offsets (the last step of a chunk wraps into c + 1) */
        uint32_t an = S[lane4 + rc4_ioff(1)]; /* S[1] */
        (void)an;
        for (uint32_t c = 0; n < drop; n += 16, c = (c + 1) & 15u) {
            uint8_t *Sc = S + ((c << 10) | lane4);
            uint8_t *Sn = S + ((((c + 1) & 15u) << 10) | lane4);
            const uint32_t ib = c << 4, nb = ((c + 1) & 15u) << 4;
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                uint8_t *si = q < 15 ? Sc + rc4_ioff(q + 1) : Sn;
                {
                    uint8_t *sp = q < 14 ? Sc + rc4_ioff(q + 2) : (q == 14 ? Sn : Sn + rc4_ioff(1));
                    const uint32_t a = an;
                    j = (j + a) & 0xFFu;
                    const uint32_t aj = rc4_addr(j, lane4);
                    const uint32_t b = S[aj];
                    const uint32_t pn = *sp;
                    const uint32_t inx = q < 14 ? ib + (uint32_t)(q + 2) : nb + (uint32_t)(q - 14);
                    an = (j == inx) ? a : pn;
                    *si = (uint8_t)b;
                    S[aj] = (uint8_t)a;
                }
            }
        }
        i = (uint32_t)(drop & 0xFFu);
    }
    for (; n < drop; ++n) {
        i = (i + 1) & 0xFFu;
        const uint32_t ai = rc4_addr(i, lane4);
        const uint32_t a = S[ai];
        j = (j + a) & 0xFFu;
        const uint32_t aj = rc4_addr(j, lane4);
        const uint32_t b = S[aj];
        S[ai] = (uint8_t)b;
        S[aj] = (uint8_t)a;
    }
    const uint64_t base = (live ? sid : 0) * len;
    const uint8_t *src = MODE == RC4_KS ? nullptr : in;
    rc4_prga<MODE, AL>(S, lane4, i, j, len, src, out, base, live);
}

/* Resumable rc4.h streams (struct rc4_state, /root/reference/rc4.h:43-50):
 * lane s continues stream s from its saved permutation and indices, runs the
 * PRGA over its len bytes with the same LDS layout and loops as
 * k_rc4_kernel (generic i: a resumed state can be anywhere in the period),
 * and writes the state back -- rc4_crypt for many states in one launch. */
struct Rc4StateDev {
    uint32_t perm[64]; /* char perm[256] */
    int32_t index1, index2;
};
static_assert(sizeof(Rc4StateDev) == 264, "struct rc4_state layout");

template <int MODE>
__global__ __launch_bounds__(64) void k_rc4_state_kernel(Rc4StateDev *st, uint64_t nstreams, uint64_t len,
                                                         const uint8_t *in, uint8_t *out)
{
    __shared__ __attribute__((aligned(16))) uint8_t S[64 * 256];
    const uint32_t lane = threadIdx.x;
    const uint32_t lane4 = lane << 2;
    const uint64_t sid = (uint64_t)blockIdx.x * 64 + lane;
    const bool live = sid < nstreams;
    Rc4StateDev *my = st + (live ? sid : 0);
    for (uint32_t q = 0; q < 64; ++q) *reinterpret_cast<uint32_t *>(S + ((q << 8) | lane4)) = my->perm[q];
    uint32_t i = (uint32_t)my->index1 & 0xFFu, j = (uint32_t)my->index2 & 0xFFu;
    const uint64_t base = (live ? sid : 0) * len;
    rc4_prga<MODE, false>(S, lane4, i, j, len, in, out, base, live);
    if (live) {
        for (uint32_t q = 0; q < 64; ++q) my->perm[q] = *reinterpret_cast<const uint32_t *>(S + ((q << 8) | lane4));
        my->index1 = (int32_t)i;
        my->index2 = (int32_t)j;
    }
}

int grid_stream(uint64_t items, int per_cu)
{
    uint64_t need = (items + 255) / 256;
    uint64_t cap = (uint64_t)otc_dev::device_cus() * per_cu;
    if (need < 1) need = 1;
    return (int)(need < cap ? need : cap);
}

/* Clock probe: one wave stamps s_memtime (shader clock) and s_memrealtime
 * (constant 100 MHz) around a window of `ticks` real-time ticks that starts
 * `delay` ticks after launch, sleeping in between so it takes no issue slots
 * from co-resident waves.  Launched on a side stream beside a workload, it
 * reads the clock the chip holds under that load (MI355X_MICROARCH: the chip
 * lowers its clock under load; cycles/byte at the nominal 2.4 GHz overstate
 * the cycle count).  out[0] = shader cycles, out[1] = real-time ticks. */
__global__ __launch_bounds__(64) void k_clock_probe(unsigned long long *out, uint64_t delay, uint64_t ticks)
{
    uint64_t r = __builtin_amdgcn_s_memrealtime();
    const uint64_t start = r + delay;
    while (r < start) {
        __builtin_amdgcn_s_sleep(32);
        r = __builtin_amdgcn_s_memrealtime();
    }
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
    do {
        __builtin_amdgcn_s_sleep(32);
        r = __builtin_amdgcn_s_memrealtime();
    } while (r - r0 < ticks);
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        out[0] = t1 - t0;
        out[1] = r1 - r0;
    }
}

} // namespace

namespace otc_impl {

hipError_t k_clock(uint64_t *out, uint64_t delay_ticks, uint64_t ticks, hipStream_t st)
{
    hipLaunchKernelGGL(k_clock_probe, dim3(1), dim3(64), 0, st, (unsigned long long *)out, delay_ticks, ticks);
    return hipGetLastError();
}

hipError_t k_xor(const void *a, const void *b, void *out, size_t n, hipStream_t st)
{
    hipLaunchKernelGGL(k_xor_kernel, dim3(grid_stream(n / 16, 8)), dim3(256), 0, st, (const uint8_t *)a,
                       (const uint8_t *)b, (uint8_t *)out, (uint64_t)n);
    return hipGetLastError();
}

hipError_t k_fill_random(void *p, size_t n, uint64_t seed, hipStream_t st)
{
    hipLaunchKernelGGL(k_fill_kernel, dim3(grid_stream(n / 16, 8)), dim3(256), 0, st, (uint8_t *)p, (uint64_t)n, seed);
    return hipGetLastError();
}

hipError_t k_checksum(const void *p, size_t n, uint64_t *out, hipStream_t st)
{
    hipError_t e = hipMemsetAsync(out, 0, sizeof(uint64_t), st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_checksum_kernel, dim3(grid_stream(n / 8, 8)), dim3(256), 0, st, (const uint64_t *)p,
                       (uint64_t)(n / 8), (unsigned long long *)out);
    return hipGetLastError();
}

hipError_t k_rc4_states(void *states, size_t nstreams, size_t len, const void *in, void *out, hipStream_t st)
{
    const uint64_t wgs = (nstreams + 63) / 64;
    const bool vec = ((((uintptr_t)in | (uintptr_t)out) & 15u) == 0 && len % 16 == 0);
    auto kern = vec ? k_rc4_state_kernel<RC4_VEC> : k_rc4_state_kernel<RC4_ANY>;
    hipLaunchKernelGGL(kern, dim3((unsigned)wgs), dim3(64), 0, st, (Rc4StateDev *)states, (uint64_t)nstreams,
                       (uint64_t)len, (const uint8_t *)in, (uint8_t *)out);
    return hipGetLastError();
}

hipError_t k_rc4_multi(const uint8_t *keys, int keylen, size_t nstreams, size_t len, size_t drop, const void *in,
                       void *out, hipStream_t st)
{
    const uint64_t wgs = (nstreams + 63) / 64;
    const int mode = !in ? RC4_KS
                     : ((((uintptr_t)in | (uintptr_t)out) & 15u) == 0 && len % 16 == 0) ? RC4_VEC : RC4_ANY;
    const bool al = drop % 16 == 0; /* i-aligned loops with the S[i+1] read-ahead */
    auto kern = al ? (mode == RC4_KS    ? k_rc4_kernel<RC4_KS, true>
                      : mode == RC4_VEC ? k_rc4_kernel<RC4_VEC, true>
                                        : k_rc4_kernel<RC4_ANY, true>)
                   : (mode == RC4_KS    ? k_rc4_kernel<RC4_KS, false>
                      : mode == RC4_VEC ? k_rc4_kernel<RC4_VEC, false>
                                        : k_rc4_kernel<RC4_ANY, false>);
    /* Resident-workgroup cap per CU, by reserving unused dynamic LDS (each
     * workgroup holds 16 KiB of S-boxes; 160 KiB per CU).  Measured
     * (profiles/r1/otbench_rc4_wgcap_ab.jsonl, otbench_rc4_cap10_ab.jsonl):
     * a launch that would put all 10 per CU in one round runs 563 GB/s, the
     * same work in two rounds of <= 6 per CU 690 GB/s; every other shape is
     * best uncapped. */
    const uint64_t cus = (uint64_t)otc_dev::device_cus();
    const int wg_cap = (wgs > 9 * cus && wgs <= 10 * cus) ? 6 : 0;
    size_t dyn_lds = 0;
    if (wg_cap >= 1 && wg_cap < 10) {
        const size_t per_wg = (160u * 1024u / (size_t)wg_cap) & ~(size_t)1023;
        dyn_lds = per_wg - 64u * 256u;
    }
    hipLaunchKernelGGL(kern, dim3((unsigned)wgs), dim3(64), dyn_lds, st, keys, keylen, (uint64_t)nstreams, (uint64_t)len,
                       (uint64_t)drop, (const uint8_t *)in, (uint8_t *)out);
    return hipGetLastError();
}

} // namespace otc_impl
