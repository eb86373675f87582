/*
 * aes_bs8.hip -- the VALU half of the chained segment-encryption split:
 * CBC / CFB128 encryption of independent segments (IV_s = iv0 + s), 8 chains
 * per lane in the row-sliced layout of otc_bs8.h.
 *
 * The T-table segment kernel (aes_tt.hip k_aes_seg_enc_tt_claim) is LDS-bound
 * with the VALU two-thirds idle and the socket ~40% under its power limit
 * (profiles/r4/energy_table: CBC-enc-seg-256 972 GB/s, PPT active 56%).  This
 * kernel runs beside it on every CU, one wave per SIMD, no LDS, and takes
 * work from the same claim counter (otc_device.h): 64-segment units, the
 * T-table one per wave from the back, this kernel 8 per wave (lane l, chain
 * k = segment (u0 + k) * 64 + l) from the front.
 *
 * Chain step, with F = the cipher output before the last round key:
 *   CBC  c_j = E(p_j ^ c_{j-1})  = F_j ^ k_NR,  F_j = R(F_{j-1} ^ p_j, k_0 ^ k_NR)
 *   CFB  c_j = p_j ^ E(c_{j-1})  = Y_j ^ k_NR,  Y_j = R(Y_{j-1}, k_0 ^ k_NR) ^ p_j
 * where R(x, k) runs the rounds with k as the first round key.  So the
 * state stays in planes, the plaintext XOR happens in word form between the
 * two transposes that every step needs anyway (planes -> words for the store,
 * words -> planes for the next rounds), and k_NR is added only to stored words
 * (an SGPR operand).  Both chains start from IV_s ^ k_NR.
 *
 * Per step (8 KiB per wave): two transposes (512 VALU) and NR rounds of
 * 387 -- AES-256 ~5.9k VALU, 1.06x the wide ECB kernel's work per byte.
 */
#include <hip/hip_runtime.h>

#include <utility>

#include "otc_bs8.h"
#include "otc_device.h"

using namespace otc_dev;
using namespace otc_bs;

namespace {

constexpr uint32_t SEG_UNIT = 64;  /* segments per claim unit (one T-table wave) */
constexpr uint32_t TASK_UNITS = 8; /* units per bs8 task: 8 chains per lane */

struct Bs8Params {
    const uint8_t *in;
    uint8_t *out;
    uint64_t seg_blocks;  /* blocks per segment */
    uint32_t seg_bytes;   /* lane stride: segment bytes (< 8 MiB, host-checked) */
    uint32_t chain_bytes; /* chain stride: 64 segments */
    Ctr128 iv0;           /* IV of segment 0 (numeric BE) */
    const uint32_t *ktab; /* key terms: [round][row] x OTC_BS_KT_STRIDE words */
    uint32_t klast[4];    /* k_NR as LE words */
    SplitClaim cl;        /* 64-segment units from the front */
};

/* key-term table: one thread per (round j, row r); round 0 is k_0 ^ k_NR */
__global__ __launch_bounds__(64) void k_bs8_key_table(otc_aes_key K, uint32_t *tab)
{
    const int e = (int)threadIdx.x;
    if (e >= K.nr * 4) return;
    W t[OTC_SBOX_KEY_TERMS];
    otc_bs8::key_terms(K.rk, K.nr, e >> 2, e & 3, true, t);
    uint32_t *o = tab + e * OTC_BS_KT_STRIDE;
#pragma unroll
    for (int j = 0; j < OTC_SBOX_KEY_TERMS; ++j) o[j] = t[j];
    o[OTC_SBOX_KEY_TERMS] = 0;
}

using ktab_ptr = const __attribute__((address_space(4))) uint32_t *;

/* key terms of (round j, row r) by scalar loads from the table */
struct Bs8Terms {
    ktab_ptr tp;
    __device__ __forceinline__ void operator()(int j, int r, W *t) const
    {
        ktab_ptr q = tp;
        asm volatile("" : "+s"(q)); /* loaded next to its S-box, not all hoisted */
#pragma unroll
        for (int i = 0; i < OTC_SBOX_KEY_TERMS; ++i) t[i] = q[(j * 4 + r) * OTC_BS_KT_STRIDE + i];
    }
};

/* f(integral_constant<int, T>) for each T, in order */
template <int... T, class F>
__device__ __forceinline__ void for_each_c(std::integer_sequence<int, T...>, F f)
{
    (f(std::integral_constant<int, T>{}), ...);
}

using gptr = __attribute__((address_space(1))) uint8_t *;
using gcptr = const __attribute__((address_space(1))) uint8_t *;

/* One task: chains k < n (n = 8 unless FULL is false) of lane l are segments
 * (u0 + k) * 64 + l.  Block j of chain k lives at
 *   base + j * 16 + k * chain_bytes + l * seg_bytes
 * (uniform 64-bit base + 32-bit offsets: global loads / stores with an SGPR
 * base and one VGPR offset). */
/* plaintext blocks per chain per load burst: 2 and 4 (32-64 contiguous bytes
 * per cache-line visit) measured no faster (profiles/r5/seg_split/bs8_burst.jsonl) */
constexpr int BURST = 1;

template <int NR, bool CFB, bool FULL>
__device__ __forceinline__ void bs8_task(const Bs8Params &P, uint64_t u0, uint32_t n)
{
    uint32_t lane = lane_id();
    asm volatile("" : "+v"(lane)); /* opaque per task: nothing lane-derived hoisted out of the claim loop */
    const uint32_t lo = lane * P.seg_bytes;
    const uint64_t tbase = u0 * SEG_UNIT * (uint64_t)P.seg_bytes;
    gcptr gib = (gcptr)P.in + tbase;
    gptr gob = (gptr)P.out + tbase;
    asm volatile("" : "+s"(gib), "+s"(gob));
    /* generic pointers derived from global ones: hipcc still emits global_ ops */
    const uint8_t *ib = (const uint8_t *)gib;
    uint8_t *ob = (uint8_t *)gob;
    const uint32_t cb = P.chain_bytes;
    /* chains past the claim (a partial last task) load chain 0's blocks and store nothing */
    auto kk = [&](int k) -> uint32_t { return (FULL || (uint32_t)k < n) ? (uint32_t)k : 0u; };
    const uint32_t kl0 = P.klast[0], kl1 = P.klast[1], kl2 = P.klast[2], kl3 = P.klast[3];
    const Bs8Terms kt{(ktab_ptr)P.ktab};

    W s[32];
    /* IV_s ^ k_NR as words, then planes */
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const uint64_t seg = (u0 + (uint64_t)kk(k)) * SEG_UNIT + lane;
        uint32_t w0, w1, w2, w3;
        ctr_words(P.iv0, seg, false, w0, w1, w2, w3);
        s[k] = w0 ^ kl0;
        s[8 + k] = w1 ^ kl1;
        s[16 + k] = w2 ^ kl2;
        s[24 + k] = w3 ^ kl3;
    }
    transpose32(s);
    pin_n(s, 32);

    const uint64_t sb = P.seg_blocks;
    /* plaintext in bursts of BURST blocks per chain (32-64 contiguous bytes
     * instead of 16 per cache line visit), loaded right after the last add of
     * the previous burst: the rounds of one step cover the latency */
    uint4 pt[BURST][8];
    auto load = [&](uint64_t j0) {
#pragma unroll
        for (int t = 0; t < BURST; ++t) {
            const uint64_t j = j0 + t < sb ? j0 + t : sb - 1; /* a short last burst re-reads a valid block */
#pragma unroll
            for (int k = 0; k < 8; ++k) pt[t][k] = *(const uint4 *)(ib + j * 16 + kk(k) * cb + lo);
        }
    };
    /* CBC stores c_{j-1} = F_{j-1} ^ k_NR after adding p_j (s = F_{j-1} ^ p_j,
     * so c_{j-1} = s ^ p_j ^ k_NR, one v_bitop3 per word): the stores then
     * follow the plaintext wait instead of preceding it -- in the other order
     * hipcc waits for the stores too (vmcnt(0) per step, the loop's merged
     * counts).  CFB stores y_j ^ k_NR. */
    auto store = [&](uint64_t j, int t) {
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (FULL || (uint32_t)k < n) {
                uint4 v = make_uint4(s[k] ^ kl0, s[8 + k] ^ kl1, s[16 + k] ^ kl2, s[24 + k] ^ kl3);
                if (!CFB) {
                    v.x ^= pt[t][k].x;
                    v.y ^= pt[t][k].y;
                    v.z ^= pt[t][k].z;
                    v.w ^= pt[t][k].w;
                }
                *(uint4 *)(ob + j * 16 + k * cb + lo) = v;
            }
    };
    auto add_pt = [&](int t) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            s[k] ^= pt[t][k].x;
            s[8 + k] ^= pt[t][k].y;
            s[16 + k] ^= pt[t][k].z;
            s[24 + k] ^= pt[t][k].w;
        }
    };
    /* one loop shape for both modes: planes -> words, add the plaintext,
     * store, words -> planes, (prefetch), rounds.  CBC adds p_j to F_{j-1}
     * before the rounds of step j; CFB adds p_j to F_j after them, so its
     * rounds run one step ahead (the first before the loop, none after the
     * last block) */
    load(0);
    if (CFB) {
        otc_bs8::rounds<NR>(s, kt);
        pin_n(s, 32);
        sched_fence();
    }
    /* step t of a burst, t a compile-time constant (pt[t] in registers; a
     * "#pragma unroll" loop over t was left rolled at AES-256 -- pt to scratch) */
    auto step = [&](uint64_t j0, auto tc) {
        constexpr int t = decltype(tc)::value;
        const uint64_t j = j0 + t;
        if (BURST == 1 || j < sb) {
            transpose32(s);
            add_pt(t);
            if (CFB) store(j, t);
            else if (j > 0) store(j - 1, t);
            if (!CFB || j + 1 < sb) {
                transpose32(s);
                pin_n(s, 32);
                sched_fence();
                if (t == BURST - 1 && j + 1 < sb) load(j + 1);
                sched_fence();
                otc_bs8::rounds<NR>(s, kt);
                pin_n(s, 32);
                sched_fence();
            }
        }
    };
    for (uint64_t j0 = 0; j0 < sb; j0 += BURST)
        for_each_c(std::make_integer_sequence<int, BURST>{}, [&](auto tc) { step(j0, tc); });
    if (!CFB) {
        transpose32(s);
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (FULL || (uint32_t)k < n)
                *(uint4 *)(ob + (sb - 1) * 16 + k * cb + lo) =
                    make_uint4(s[k] ^ kl0, s[8 + k] ^ kl1, s[16 + k] ^ kl2, s[24 + k] ^ kl3);
    }
}

/* one workgroup per CU beside the T-table claim kernel: one wave per SIMD
 * beside its four (<= 72 VGPRs each at 4-block bursts), so up to 224 VGPRs
 * (tests/test_isa_cpu.py::test_bs8_segment_pair_shares_a_simd).  Only a
 * minimum occupancy: a maximum (waves_per_eu(2, 2)) makes hipcc pad the
 * descriptor to 169 VGPRs (176 allocated) to enforce it. */
template <int NR, bool CFB>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void k_aes_bs8_seg_claim(Bs8Params P)
{
    strace(3);
    for (;;) {
        uint32_t n = 0;
        const int64_t u = claim_front(P.cl, TASK_UNITS, &n);
        if (u < 0) break;
        if (n == TASK_UNITS)
            bs8_task<NR, CFB, true>(P, (uint64_t)u, n);
        else
            bs8_task<NR, CFB, false>(P, (uint64_t)u, n);
    }
}

} // namespace

namespace otc_impl {

OTC_STRACE_READER(strace_read_bs8)

/* The bitsliced half of the segment-encryption split: units of 64 segments
 * from the front of `cl`, cl.wgs workgroups (default one per CU).  seg_blocks
 * * 16 < 8 MiB (the engine checks). */
hipError_t bs8_seg_encrypt_claim(bool cfb, const void *in, void *out, uint64_t seg_blocks, const otc_aes_key &K,
                                 Ctr128 iv0, SplitClaim cl, hipStream_t st)
{
    if (seg_blocks == 0 || seg_blocks * 16 * SEG_UNIT * TASK_UNITS > 0xFFFFFFFFull) return hipErrorInvalidValue;
    uint32_t *tab = nullptr;
    const size_t words = (size_t)K.nr * 4 * OTC_BS_KT_STRIDE;
    hipError_t e = alloc_fault() ? hipErrorOutOfMemory : hipMallocAsync((void **)&tab, words * 4, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_bs8_key_table, dim3(1), dim3(64), 0, st, K, tab);
    Bs8Params P{};
    P.in = (const uint8_t *)in;
    P.out = (uint8_t *)out;
    P.seg_blocks = seg_blocks;
    P.seg_bytes = (uint32_t)(seg_blocks * 16);
    P.chain_bytes = (uint32_t)(seg_blocks * 16 * SEG_UNIT);
    P.iv0 = iv0;
    P.ktab = tab;
    for (int i = 0; i < 4; ++i) P.klast[i] = K.rk[4 * K.nr + i];
    P.cl = cl;
    const dim3 g(cl.wgs ? cl.wgs : (unsigned)device_cus()), b(256);
    switch (K.nr) {
    case 10:
        if (cfb) hipLaunchKernelGGL((k_aes_bs8_seg_claim<10, true>), g, b, 0, st, P);
        else hipLaunchKernelGGL((k_aes_bs8_seg_claim<10, false>), g, b, 0, st, P);
        break;
    case 12:
        if (cfb) hipLaunchKernelGGL((k_aes_bs8_seg_claim<12, true>), g, b, 0, st, P);
        else hipLaunchKernelGGL((k_aes_bs8_seg_claim<12, false>), g, b, 0, st, P);
        break;
    case 14:
        if (cfb) hipLaunchKernelGGL((k_aes_bs8_seg_claim<14, true>), g, b, 0, st, P);
        else hipLaunchKernelGGL((k_aes_bs8_seg_claim<14, false>), g, b, 0, st, P);
        break;
    default: e = hipErrorInvalidValue;
    }
    if (e == hipSuccess) e = hipGetLastError();
    const hipError_t f = hipFreeAsync(tab, st);
    return e != hipSuccess ? e : f;
}

} // namespace otc_impl
