/*
 * otc_device.h -- device-side helpers shared by the gfx950 kernels.
 *
 * AES tables are generated at COMPILE time (constexpr, FIPS-197 definition)
 * into __device__ read-only globals; each workgroup replicates what it needs
 * into LDS at kernel start (csrc/hip/aes_tt.hip).  Nothing is uploaded per
 * launch, unlike the reference which re-copied the key schedule and kept the
 * tables in uncached global memory (/root/reference/aes-gpu/Source/AES.tab:689,
 * AES.cu:222).
 */
#ifndef OTC_DEVICE_H
#define OTC_DEVICE_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>

#include "otc.h"

namespace otc_dev {

struct AesTables {
    uint8_t sb[256];
    uint8_t isb[256];
    uint32_t te0[256];
    uint32_t td0[256];
    uint32_t is4[256]; /* inverse S-box byte replicated into all 4 bytes */
};

constexpr uint8_t xt(uint8_t a) { return (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0)); }
constexpr uint8_t gmul(uint8_t a, uint8_t b)
{
    uint8_t r = 0;
    for (int i = 0; i < 8; ++i) {
        if (b & 1) r ^= a;
        a = xt(a);
        b >>= 1;
    }
    return r;
}

constexpr AesTables make_tables()
{
    AesTables t{};
    uint8_t ex[256]{}, lg[256]{};
    uint8_t v = 1;
    for (int i = 0; i < 255; ++i) {
        ex[i] = v;
        lg[v] = (uint8_t)i;
        v = (uint8_t)(v ^ xt(v));
    }
    for (int a = 0; a < 256; ++a) {
        uint8_t inv = a ? ex[(255 - lg[a]) % 255] : 0;
        uint8_t s = inv, r = inv;
        for (int k = 0; k < 4; ++k) {
            r = (uint8_t)((r << 1) | (r >> 7));
            s ^= r;
        }
        s ^= 0x63;
        t.sb[a] = s;
        t.isb[s] = (uint8_t)a;
    }
    for (int a = 0; a < 256; ++a) {
        uint8_t s = t.sb[a];
        t.te0[a] = (uint32_t)gmul(s, 2) | ((uint32_t)s << 8) | ((uint32_t)s << 16) |
                   ((uint32_t)gmul(s, 3) << 24);
        uint8_t u = t.isb[a];
        t.td0[a] = (uint32_t)gmul(u, 14) | ((uint32_t)gmul(u, 9) << 8) |
                   ((uint32_t)gmul(u, 13) << 16) | ((uint32_t)gmul(u, 11) << 24);
        t.is4[a] = (uint32_t)u * 0x01010101u;
    }
    return t;
}

/* byte swap via v_perm_b32 (one VALU op) */
__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_amdgcn_perm(x, x, 0x00010203u); }
/* 3-input XOR in one v_bitop3_b32 (gfx950 has no v_xor3_b32; hipcc does not
 * fuse pure XOR chains by itself) */
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c)
{
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t rotl8(uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 24); }
__device__ __forceinline__ uint32_t rotl16(uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 16); }
__device__ __forceinline__ uint32_t rotl24(uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 8); }

/* 128-bit counter value (numeric, big-endian semantics) */
struct Ctr128 {
    uint64_t hi, lo;
};

/* counter + idx; `wrap64` keeps the carry out of the high half (RFC 3686 /
 * AES-NI layout of the reference, aesni.c:139-143). */
__device__ __forceinline__ void ctr_words(const Ctr128 &c, uint64_t idx, bool wrap64, uint32_t &w0,
                                          uint32_t &w1, uint32_t &w2, uint32_t &w3)
{
    uint64_t lo = c.lo + idx;
    uint64_t hi = c.hi + ((!wrap64 && lo < c.lo) ? 1ull : 0ull);
    w0 = bswap32((uint32_t)(hi >> 32));
    w1 = bswap32((uint32_t)hi);
    w2 = bswap32((uint32_t)(lo >> 32));
    w3 = bswap32((uint32_t)lo);
}

/* Bitsliced kernel modes (aes_bs.hip): BS_ECB: ECB encryption; BS_ECB_DEC /
 * BS_CBC_DEC: the inverse cipher through the forward S-box (S^-1 = L S L,
 * otc_invmix.h) with a decryption key; BS_CFB_DEC: CFB128 decryption, P_i =
 * E(C_{i-1}) ^ C_i -- the forward cipher on the input shifted back one block,
 * XORed with the input */
enum : int { BS_CTR = 0, BS_ECB = 1, BS_ECB_DEC = 2, BS_CBC_DEC = 3, BS_CFB_DEC = 4,
              /* CBC / CFB decryption of independent power-of-two segments:
               * block i of a segment start takes IV_s = iv0 + s (128-bit BE)
               * instead of block i-1 */
              BS_CBC_DEC_SEG = 5, BS_CFB_DEC_SEG = 6 };

/* Work claiming of a co-resident split (engine.cpp split_claim): the T-table
 * and the bitsliced kernel take units of ONE buffer from a shared 64-bit
 * counter -- the bitsliced kernel from the front (count in the low 32 bits),
 * the T-table kernel from the back (high 32 bits) -- so both run until the
 * buffer is done and finish together, whatever rate each gets on the box.
 * Every claim is one atomic add on the whole word, valid iff front + back
 * units claimed before it < nunits, so the two ends never overlap and a
 * failed claim (nothing left) hides nothing.  A T-table claim adds one unit;
 * a front claim adds one unit too.
 * Units: 2048 blocks for the whole-buffer modes (one bitsliced task; 1024-
 * block units and a reserve left to the T-table measured 1-11% slower and
 * were removed, profiles/r4/claim_unit/); 64 segments for the persistent
 * segment-encryption kernel (one T-table wave, back claims only).
 * A wave claims with one lane (a vector-memory atomic) and broadcasts.
 * First units without a claim: the host hands the first pf units to the
 * bitsliced waves (wave j < pf starts on unit j) and the last pb units to the
 * T-table waves (wave w < pb starts on unit nunits - 1 - w); the claim word
 * covers the units between.  Otherwise every wave's FIRST claim lands on the
 * word at once -- 4096 T-table waves queue ~45 us on one address (~90 atomics
 * per us), the last of them idle that long (docs/PERF.md round 6). */
constexpr uint32_t CLAIM_UNIT = 2048u;
struct SplitClaim {
    unsigned long long *ctr; /* zeroed (stream-ordered) before the launches */
    uint32_t nunits;         /* full units */
    uint32_t wgs;            /* host side: workgroups of the kernel given this claim (0: one per CU) */
    uint32_t pf = 0;         /* units [0, pf): the bitsliced waves' first units, unclaimed */
    uint32_t pb = 0;         /* units [nunits - pb, nunits): the T-table waves' first units, unclaimed */
};

/* lane id from the exec-mask count: nothing to keep live across a loop
 * (threadIdx.x lives in v0 from kernel entry; read in every trip of a long
 * loop body, hipcc keeps it -- and spills it) */
/* 16-byte global load / store with an optional non-temporal hint (the NT
 * bit: the line is not kept in L2 / MALL).  Streaming data that is read once
 * and written once -- every byte of a 64 GiB CTR call -- does not benefit
 * from being cached, and the hint cut the headline kernel's J/GB by 2-3% and
 * raised its rate 1.7-1.8% under the power cap (round 6,
 * profiles/r6/nt_ab/).  The builtins take native vector types, not HIP's
 * uint4 struct. */
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ uint4 ld_u4(const void *p)
{
    if constexpr (NT) {
        const u32x4 v = __builtin_nontemporal_load((const u32x4 *)p);
        return make_uint4(v.x, v.y, v.z, v.w);
    } else {
        return *(const uint4 *)p;
    }
}
template <bool NT>
__device__ __forceinline__ void st_u4(void *p, uint4 v)
{
    if constexpr (NT) {
        const u32x4 w = {v.x, v.y, v.z, v.w};
        __builtin_nontemporal_store(w, (u32x4 *)p);
    } else {
        *(uint4 *)p = v;
    }
}

__device__ __forceinline__ uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

/* one atomic add of `inc` on the claim word; returns the old value (wave-uniform) */
__device__ __forceinline__ uint64_t claim_add(const SplitClaim &c, unsigned long long inc)
{
    unsigned long long old = 0;
    if (lane_id() == 0) {
        /* built per claim: hoisted out of a caller's loop, the operand pair
         * would stay live (and spill) across the whole loop body */
        asm volatile("" : "+v"(inc));
        old = __hip_atomic_fetch_add(c.ctr, inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    const uint32_t f = __builtin_amdgcn_readfirstlane((uint32_t)old);
    const uint32_t b = __builtin_amdgcn_readfirstlane((uint32_t)(old >> 32));
    return (uint64_t)b << 32 | f;
}

/* back: a unit index; front: the next unit index from the front; -1 when
 * nothing is left for this side (wave-uniform) */
__device__ __forceinline__ int64_t claim_unit(const SplitClaim &c, bool back)
{
    const uint64_t old = claim_add(c, back ? (1ull << 32) : 1ull);
    const uint32_t f = (uint32_t)old, b = (uint32_t)(old >> 32);
    if ((uint64_t)f + b + c.pf + c.pb >= c.nunits) return -1;
    return back ? (int64_t)(c.nunits - c.pb - 1u - b) : (int64_t)(c.pf + f);
}

/* a wave's first unit: its pre-assigned one (w: the wave's index among its
 * kernel's waves, wave-uniform), else its first claim */
__device__ __forceinline__ int64_t first_unit(const SplitClaim &c, bool back, uint32_t w)
{
    if (back ? w < c.pb : w < c.pf) return back ? (int64_t)(c.nunits - 1u - w) : (int64_t)w;
    return claim_unit(c, back);
}

/* Wave-start trace of the splits (a diagnostic build: make variant
 * VFLAGS=-DOTC_SPLIT_TRACE=1): lane 0 of a wave appends {s_memrealtime,
 * tag << 32 | HW_ID} to a per-code-object buffer; otc_split_trace reads it
 * back.  Off (no code) in the shipped build. */
#ifndef OTC_SPLIT_TRACE
#define OTC_SPLIT_TRACE 0
#endif
constexpr unsigned STRACE_MAX = 16384;
#if OTC_SPLIT_TRACE
static __device__ unsigned long long g_strace[2 * STRACE_MAX];
static __device__ unsigned int g_strace_n;
__device__ __forceinline__ void strace(uint32_t tag)
{
    if (lane_id() == 0) {
        /* the clock first: thousands of waves queue on the slot counter's
         * atomic (~90 per us on one word), and a time read after it measured
         * that queue -- a 45-55 us "start ramp" the chip does not have
         * (tools/ubench/launch_ramp.hip: 256 x 1024-thread workgroups with
         * 128 KiB LDS start within 2.3 us) */
        const unsigned long long now = __builtin_amdgcn_s_memrealtime();
        const unsigned i = atomicAdd(&g_strace_n, 1u);
        if (i < STRACE_MAX) {
            uint32_t hw;
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
            g_strace[2 * i] = now;
            g_strace[2 * i + 1] = (unsigned long long)tag << 32 | hw;
        }
    }
}
/* host: copy out this code object's records (and reset the count) */
#define OTC_STRACE_READER(NAME)                                                                   \
    int NAME(unsigned long long *buf, int max)                                                    \
    {                                                                                             \
        unsigned n = 0;                                                                           \
        if (hipMemcpyFromSymbol(&n, HIP_SYMBOL(g_strace_n), sizeof n) != hipSuccess) return -1;   \
        if (n > STRACE_MAX) n = STRACE_MAX;                                                       \
        if ((int)n > max) n = (unsigned)max;                                                      \
        if (n && hipMemcpyFromSymbol(buf, HIP_SYMBOL(g_strace), 16ull * n) != hipSuccess) return -1; \
        const unsigned z = 0;                                                                     \
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_strace_n), &z, sizeof z);                            \
        return (int)n;                                                                            \
    }
#else
__device__ __forceinline__ void strace(uint32_t) {}
#define OTC_STRACE_READER(NAME)                                                                   \
    int NAME(unsigned long long *, int) { return -1; }
#endif

/* Allocation fault injection, a test hook (otc_fault_inject_alloc): true
 * when the runtime allocation about to be made should fail.  One atomic
 * countdown; off (no cost beyond a relaxed load) unless armed. */
bool alloc_fault();

/* Host: CU count of the calling thread's current device, cached per device.
 * Thread-safe (the multi-GPU paths launch from one host thread per GPU): the
 * attribute is immutable, so a relaxed atomic cache is enough. */
inline int device_cus()
{
    static std::atomic<int> cache[64];
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::atomic<int> &slot = cache[(unsigned)dev & 63u];
    int v = slot.load(std::memory_order_relaxed);
    if (v <= 0) {
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
        slot.store(v, std::memory_order_relaxed);
    }
    return v;
}

} // namespace otc_dev

#endif
