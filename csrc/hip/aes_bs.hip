/*
 * aes_bs.hip -- wave-level bitsliced AES encryption (CTR / ECB-encrypt) on
 * the gfx950 VALU.
 *
 * Each lane holds 32 blocks as 128 bit-planes (one VGPR per state bit, see
 * include/otc_bitslice.h); a wave therefore processes 64 x 32 = 2048 blocks
 * (32 KiB) per task.  Slot k of lane l is block task*2048 + 64*k + l, so every
 * plaintext load / ciphertext store of one slot is a coalesced 1 KiB
 * dwordx4 wave access.
 *
 * CTR never transposes its input: task boundaries are aligned to the counter
 * (the first task starts (ctr0 mod 2048) blocks "early" with those slots
 * masked), so inside a task the counter of slot (k, l) is C + 64k + l with no
 * carry out of bit 10.  Counter plane n is then
 *     n < 6   : bit n of the lane id        (per lane)
 *     6..10   : 0xAAAAAAAA, 0xCCCCCCCC, ... (a constant pattern over slots)
 *     n >= 11 : bit n of C                  (wave uniform -> SGPR)
 * and hipcc's uniformity analysis keeps the uniform planes on the scalar ALU:
 * in round 1 only state byte 15 is per-lane, in round 2 only column 0, so
 * ~27 of the 160 S-box evaluations of AES-128 cost no VALU at all ("counter
 * mode caching", done by the compiler instead of by hand).
 *
 * The last round key is folded into the output XOR (ks ^ rk ^ pt as one
 * v_bitop3 per word) after the single output transpose.
 *
 * No reference counterpart (the reference has only a T-table CUDA kernel,
 * /root/reference/aes-gpu/Source/AES.cu:284-392).
 */
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "otc_bitslice.h"
#include "otc_device.h"

using namespace otc_dev;
using namespace otc_bs;

namespace {

struct BsParams {
    const uint8_t *in;
    uint8_t *out;
    uint64_t nblocks;   /* full blocks */
    uint32_t tail;      /* CTR: trailing partial block bytes */
    uint32_t wrap64;    /* CTR: 64-bit counter increment */
    uint64_t shift;     /* CTR: ctr0.lo mod 2048 (virtual index = i + shift) */
    Ctr128 cbase;       /* CTR: ctr0 with the low 11 bits cleared */
    uint32_t stagger;   /* 100 MHz ticks of start delay per residency slot (0: none) */
    uint32_t cus;       /* CUs (residency slot of workgroup b = b / cus) */
};

/* Start-time stagger for the first resident round of workgroups: slot
 * b / cus (0, 1, 2 on a 3-wave build) waits slot * stagger ticks, so the
 * waves sharing a SIMD do not run their memory phases in lockstep.  Later
 * workgroups replace finished ones and inherit the offsets. */
__device__ __forceinline__ void stagger_start(const BsParams &P, uint32_t slots)
{
    if (P.stagger == 0 || blockIdx.x >= slots * P.cus) return;
    const uint64_t wait = (uint64_t)(blockIdx.x / P.cus) * P.stagger;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < wait) __builtin_amdgcn_s_sleep(8);
}

enum : int { BS_CTR = 0, BS_ECB = 1 };

__device__ __forceinline__ W lane_mask(uint32_t lane, int n) { return (W)(0u - ((lane >> n) & 1u)); }

/* CTR: the plaintext of slots 0..LS-1 is copied into LDS by the DMA path
 * (global_load_lds_dwordx4, no VGPRs) when the task starts and lands while the
 * ~60 us of rounds run; layout [wave][slot][lane] x 16 B is exactly the
 * lane-linear image glds writes, and each lane reads its own 16 B back with a
 * conflict-free ds_read_b128. */
template <int NR, int MODE, bool CACHE, int PF, int LS>
__device__ __forceinline__ void aes_bs_task(const BsParams &P, const otc_aes_key &K, uint4 *stage)
{
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t gwave = (uint64_t)blockIdx.x * 4u + wave;
    const uint64_t shift = (MODE == BS_CTR) ? P.shift : 0;
    const uint64_t vtotal = P.nblocks + shift; /* full blocks only; the host
                                                  routes a trailing partial block
                                                  to the T-table kernel */

    /* One 2048-block task per wave, no grid-stride loop: a loop lets hipcc
     * hoist loop-invariant plane/mask values out of it, which costs more
     * registers than the 128-plane state leaves. */
    {
        const uint64_t task = gwave;
        if (task * 2048u >= vtotal) return;
        const uint64_t vbase = task * 2048u;
        /* block index of slot k = vbase - shift + 64k + lane (may be out of range) */
        const bool full = vbase >= shift && vbase + 2048u - shift <= P.nblocks; /* uniform */
        W s[128];

        if (MODE == BS_CTR && LS > 0) {
            const int64_t t0 = (int64_t)vbase - (int64_t)shift;
            const uint8_t *ib0 = P.in + t0 * 16 + lane * 16u;
            /* branch-free (a per-slot branch splits the kernel's one basic
             * block and costs ~70 VGPRs): lanes outside the buffer load block 0
             * instead, and their slots are never stored */
#pragma unroll
            for (int k = 0; k < LS; ++k) {
                const int64_t si = t0 + (int64_t)lane + 64 * k;
                const bool ok = full || (si >= 0 && (uint64_t)si < P.nblocks);
                __builtin_amdgcn_global_load_lds((const void *)(ok ? ib0 + 1024u * k : P.in),
                                                 (__attribute__((address_space(3))) void *)&stage[(wave * LS + k) * 64],
                                                 16, 0, 0);
            }
        }
        if (MODE == BS_CTR) {
            /* C = cbase + vbase (128-bit, or 64-bit wrap) */
            uint64_t clo = P.cbase.lo + vbase;
            uint64_t chi = P.cbase.hi + ((!P.wrap64 && clo < P.cbase.lo) ? 1u : 0u);
#pragma unroll
            for (int b = 0; b < 16; ++b) {
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const int n = 8 * (15 - b) + i; /* numeric counter bit */
                    W v;
                    if (n < 6) {
                        v = lane_mask(lane, n);
                    } else if (n < 11) {
                        constexpr W pat[5] = {0xAAAAAAAAu, 0xCCCCCCCCu, 0xF0F0F0F0u, 0xFF00FF00u, 0xFFFF0000u};
                        v = pat[n - 6];
                    } else if (n < 64) {
                        v = (W)(0u - (uint32_t)((clo >> n) & 1u));
                    } else {
                        v = (W)(0u - (uint32_t)((chi >> (n - 64)) & 1u));
                    }
                    s[8 * b + i] = v;
                }
            }
        } else {
            /* ECB: load 32 blocks (uniform task base + 32-bit lane offsets:
             * 64-bit per-slot addresses would be CSE'd with the stores and
             * kept live across the rounds) and transpose each word column */
            const uint8_t *tb = P.in + vbase * 16;
            const uint32_t lo = lane * 16u;
            uint4 blk[32];
#pragma unroll
            for (int k = 0; k < 32; ++k) {
                const uint64_t i = vbase + lane + 64u * k;
                blk[k] = (full || i < P.nblocks) ? *(const uint4 *)(tb + lo + 1024u * k) : make_uint4(0, 0, 0, 0);
            }
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                W m[32];
#pragma unroll
                for (int k = 0; k < 32; ++k) m[k] = w == 0 ? blk[k].x : w == 1 ? blk[k].y : w == 2 ? blk[k].z : blk[k].w;
                transpose32(m);
                pin_n(m, 32);
#pragma unroll
                for (int q = 0; q < 32; ++q) s[32 * w + q] = m[q];
                sched_fence();
            }
        }

        sched_fence();
        /* Round keys are laundered through an empty asm so hipcc materialises
         * each key mask next to its use instead of all 128*NR up front. */
        uint32_t rk[4 * (NR + 1)];
#pragma unroll
        for (int q = 0; q < 4 * (NR + 1); ++q) {
            uint32_t v = K.rk[q];
            asm volatile("" : "+s"(v));
            rk[q] = v;
        }
        /* rounds (AddRoundKey folded into the S-boxes; last key folded below) */
        encrypt_planes<NR, MODE == BS_CTR && CACHE>(s, [&](int r, int p) -> W {
            /* plane p = 32*w + q  <->  bit q of round-key word w */
            return (W)(0u - ((rk[4 * r + (p >> 5)] >> (p & 31)) & 1u));
        });

        pin_n(s, 128);
        sched_fence();

        /* uniform task base (may point before the buffer for the first CTR
         * task; those slots are masked) + 32-bit per-lane offsets */
        const int64_t tstart = (int64_t)vbase - (int64_t)shift;
        const uint8_t *ib = P.in + tstart * 16;
        uint8_t *ob = P.out + tstart * 16;
        uint32_t lo = lane * 16u;
        /* ordered after the pin above (volatile asms keep their order), so
         * the loads below cannot be hoisted into the round phase */
        asm volatile("" : "+v"(lo));
        auto slot_ok = [&](int k) {
            const int64_t si = tstart + (int64_t)lane + 64 * k;
            return full || (si >= 0 && (uint64_t)si < P.nblocks);
        };
        /* CTR plaintext is software-pipelined PF slots ahead: after the
         * output transposes the first PF loads are issued, then each group of
         * 4 slots issues the loads of the group PF/4 ahead (PF = 0: each group
         * loads and waits for its own slots).  Issuing the first loads before
         * the transposes instead pushes the kernel past 256 VGPRs. */
        uint4 pt[32];
        sched_fence();
        /* planes -> blocks (keystream / ciphertext without the last key) */
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            transpose32(s + 32 * w);
            pin_n(s + 32 * w, 32);
            sched_fence();
        }

        if (MODE == BS_CTR) {
#pragma unroll
            for (int k = LS; k < LS + PF && k < 32; ++k)
                pt[k] = slot_ok(k) ? *(const uint4 *)(ib + lo + 1024u * k) : make_uint4(0, 0, 0, 0);
        }
        const uint32_t k0 = rk[4 * NR + 0], k1 = rk[4 * NR + 1], k2 = rk[4 * NR + 2],
                       k3 = rk[4 * NR + 3];
#pragma unroll
        for (int k = 0; k < 32; ++k) {
            if ((k & 3) == 0) {
                sched_fence();
                if (MODE == BS_CTR) {
#pragma unroll
                    for (int j = (k + PF > LS + PF ? k + PF : LS + PF); j < k + PF + 4 && j < 32; ++j)
                        pt[j] = slot_ok(j) ? *(const uint4 *)(ib + lo + 1024u * j) : make_uint4(0, 0, 0, 0);
                }
            }
            const uint32_t off = lo + 1024u * k;
            if (slot_ok(k)) {
                uint4 o;
                if (MODE == BS_CTR) {
                    /* lane index from the laundered offset: keeps the LDS
                     * reads below the round phase (else hoisted, +70 VGPRs) */
                    const uint4 x = k < LS ? stage[(wave * LS + k) * 64 + (lo >> 4)] : pt[k];
                    o.x = x3(x.x, s[k], k0);
                    o.y = x3(x.y, s[32 + k], k1);
                    o.z = x3(x.z, s[64 + k], k2);
                    o.w = x3(x.w, s[96 + k], k3);
                } else {
                    o = make_uint4(s[k] ^ k0, s[32 + k] ^ k1, s[64 + k] ^ k2, s[96 + k] ^ k3);
                }
                *(uint4 *)(ob + off) = o;
            }
        }
    }
}

/* Same task with a ROLLED round loop: the fully unrolled kernel is ~150 KB
 * of code (AES-128), larger than the instruction cache, so every wave streams
 * the whole kernel from L2 (SQ_IFETCH ~4800 x 32 B per wave).  Here rounds
 * 0..NR-2 are one ~14 KB loop body (round keys read per round from the
 * kernel-argument segment by scalar loads), the final round is peeled.
 * MIXT: low-register MixColumns (mix_column_t). */
template <int NR, int MODE, bool MIXT, int LS, bool ZEROKEY = false, int FENCE = 2>
__device__ __forceinline__ void aes_bs_task_loop(const BsParams &P, const otc_aes_key &K, uint4 *stage)
{
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t gwave = (uint64_t)blockIdx.x * 4u + wave;
    const uint64_t shift = (MODE == BS_CTR) ? P.shift : 0;
    const uint64_t vtotal = P.nblocks + shift;
    const uint64_t task = gwave;
    if (task * 2048u >= vtotal) return;
    const uint64_t vbase = task * 2048u;
    const bool full = vbase >= shift && vbase + 2048u - shift <= P.nblocks;
    W s[128];
    if (MODE == BS_CTR && LS > 0) {
        /* plaintext of slots 0..LS-1 straight into LDS (no VGPRs): lands
         * while the rounds run; the rounds issue no vector memory op, so no
         * vmcnt wait before the output phase depends on it */
        const int64_t t0 = (int64_t)vbase - (int64_t)P.shift;
        const uint8_t *ib0 = P.in + t0 * 16 + lane * 16u;
#pragma unroll
        for (int k = 0; k < LS; ++k) {
            const int64_t si = t0 + (int64_t)lane + 64 * k;
            const bool ok = full || (si >= 0 && (uint64_t)si < P.nblocks);
            __builtin_amdgcn_global_load_lds((const void *)(ok ? ib0 + 1024u * k : P.in),
                                             (__attribute__((address_space(3))) void *)&stage[(wave * LS + k) * 64],
                                             16, 0, 0);
        }
    }
    if (MODE == BS_CTR) {
        uint64_t clo = P.cbase.lo + vbase;
        uint64_t chi = P.cbase.hi + ((!P.wrap64 && clo < P.cbase.lo) ? 1u : 0u);
#pragma unroll
        for (int b = 0; b < 16; ++b) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int n = 8 * (15 - b) + i;
                W v;
                if (n < 6) {
                    v = lane_mask(lane, n);
                } else if (n < 11) {
                    constexpr W pat[5] = {0xAAAAAAAAu, 0xCCCCCCCCu, 0xF0F0F0F0u, 0xFF00FF00u, 0xFFFF0000u};
                    v = pat[n - 6];
                } else if (n < 64) {
                    v = (W)(0u - (uint32_t)((clo >> n) & 1u));
                } else {
                    v = (W)(0u - (uint32_t)((chi >> (n - 64)) & 1u));
                }
                s[8 * b + i] = v;
            }
        }
        /* the counter planes are uniform except 11 per-lane ones: make them
         * VGPRs now (the loop needs one register layout for every round) */
#pragma unroll
        for (int q = 0; q < 128; ++q) asm volatile("" : "+v"(s[q]));
    } else {
        const uint8_t *tb = P.in + vbase * 16;
        const uint32_t lo = lane * 16u;
        uint4 blk[32];
#pragma unroll
        for (int k = 0; k < 32; ++k) {
            const uint64_t i = vbase + lane + 64u * k;
            blk[k] = (full || i < P.nblocks) ? *(const uint4 *)(tb + lo + 1024u * k) : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            W m[32];
#pragma unroll
            for (int k = 0; k < 32; ++k) m[k] = w == 0 ? blk[k].x : w == 1 ? blk[k].y : w == 2 ? blk[k].z : blk[k].w;
            transpose32(m);
            pin_n(m, 32);
#pragma unroll
            for (int q = 0; q < 32; ++q) s[32 * w + q] = m[q];
            sched_fence();
        }
    }
    sched_fence();
#pragma nounroll
    for (int r = 0; r < NR - 1; ++r) {
        uint32_t kw[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) kw[j] = K.rk[4 * r + j];
        auto kz = [&](int p) -> W { return (W)0; };
        auto kr = [&](int p) -> W { return (W)(0u - ((kw[p >> 5] >> (p & 31)) & 1u)); };
        if (ZEROKEY) /* measurement only: key masks folded away (wrong output) */
            round_step<MIXT, decltype(kz), FENCE>(s, kz);
        else
            round_step<MIXT, decltype(kr), FENCE>(s, kr);
        pin_n(s, 128);
    }
    {
        uint32_t kw[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) kw[j] = K.rk[4 * (NR - 1) + j];
        round_final(s, [&](int p) -> W { return (W)(0u - ((kw[p >> 5] >> (p & 31)) & 1u)); });
    }
    pin_n(s, 128);
    sched_fence();

    const int64_t tstart = (int64_t)vbase - (int64_t)shift;
    const uint8_t *ib = P.in + tstart * 16;
    uint8_t *ob = P.out + tstart * 16;
    uint32_t lo = lane * 16u;
    asm volatile("" : "+v"(lo));
    auto slot_ok = [&](int k) {
        const int64_t si = tstart + (int64_t)lane + 64 * k;
        return full || (si >= 0 && (uint64_t)si < P.nblocks);
    };
    /* register-loaded plaintext (slots LS..31): all issued before the
     * transposes, none after a store -- vmcnt is in order on gfx9, so a load
     * issued behind stores would also wait for them */
    uint4 pt[32];
    if (MODE == BS_CTR) {
#pragma unroll
        for (int k = LS; k < 32; ++k)
            pt[k] = slot_ok(k) ? *(const uint4 *)(ib + lo + 1024u * k) : make_uint4(0, 0, 0, 0);
    }
    sched_fence();
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        transpose32(s + 32 * w);
        pin_n(s + 32 * w, 32);
        sched_fence();
    }
    const uint32_t k0 = K.rk[4 * NR + 0], k1 = K.rk[4 * NR + 1], k2 = K.rk[4 * NR + 2], k3 = K.rk[4 * NR + 3];
#pragma unroll
    for (int k = 0; k < 32; ++k) {
        const uint32_t off = lo + 1024u * k;
        if (slot_ok(k)) {
            uint4 o;
            if (MODE == BS_CTR) {
                const uint4 x = k < LS ? stage[(wave * LS + k) * 64 + (lo >> 4)] : pt[k];
                o.x = x3(x.x, s[k], k0);
                o.y = x3(x.y, s[32 + k], k1);
                o.z = x3(x.z, s[64 + k], k2);
                o.w = x3(x.w, s[96 + k], k3);
            } else {
                o = make_uint4(s[k] ^ k0, s[32 + k] ^ k1, s[64 + k] ^ k2, s[96 + k] ^ k3);
            }
            *(uint4 *)(ob + off) = o;
        }
    }
}

template <int NR, int MODE, bool MIXT, int LS, bool ZK = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3, 3))) void k_aes_bs_loop3(BsParams P,
                                                                                                 otc_aes_key K)
{
    __shared__ uint4 stage[LS > 0 ? 4 * LS * 64 : 1];
    stagger_start(P, 3);
    aes_bs_task_loop<NR, MODE, MIXT, LS, ZK>(P, K, stage);
}

template <int NR, int MODE, bool MIXT, int LS, bool ZK = false, int FENCE = 2>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_aes_bs_loop2(BsParams P,
                                                                                                 otc_aes_key K)
{
    __shared__ uint4 stage[LS > 0 ? 4 * LS * 64 : 1];
    stagger_start(P, 2);
    aes_bs_task_loop<NR, MODE, MIXT, LS, ZK, FENCE>(P, K, stage);
}

template <int NR, int MODE, bool CACHE, int PF, int LS>
__global__ __launch_bounds__(256) void k_aes_bs(BsParams P, otc_aes_key K)
{
    __shared__ uint4 stage[LS > 0 ? 4 * LS * 64 : 1];
    aes_bs_task<NR, MODE, CACHE, PF, LS>(P, K, stage);
}

/* Same task at 3 waves per SIMD (<= 168 VGPRs, ~32 values spilled to
 * scratch): the default (OTC_BS_W3=0 selects k_aes_bs).  LS > 0 (12 slots, 3
 * workgroups x 48 KiB) measured slower: more spills than latency saved. */
template <int NR, int MODE, int LS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3, 3))) void k_aes_bs_w3(BsParams P,
                                                                                             otc_aes_key K)
{
    __shared__ uint4 stage[LS > 0 ? 4 * LS * 64 : 1];
    stagger_start(P, 3);
    aes_bs_task<NR, MODE, false, 0, LS>(P, K, stage);
}

template <int NR, int MODE>
hipError_t launch_nr(const BsParams &P, const otc_aes_key &K, hipStream_t st)
{
    const uint64_t vt = P.nblocks + (MODE == BS_CTR ? P.shift : 0);
    const uint64_t tasks = (vt + 2047) / 2048;
    uint64_t wgs = (tasks + 3) / 4;
    if (wgs < 1) wgs = 1;
    if (wgs > 0xFFFFFFFFull) return hipErrorInvalidValue;
    static const bool cache = getenv("OTC_BS_CTR_CACHE") && atoi(getenv("OTC_BS_CTR_CACHE")) != 0;
    /* 2-wave builds (OTC_BS_W3=0), AES-128 CTR options: LS = 20 plaintext
     * slots prefetched into LDS at task start (OTC_BS_LDS=1, measured +5% on
     * the 2-wave build) and PF = 8 slots pipelined in registers (OTC_BS_PF=1,
     * +1%).  Off by default: the 3-wave build beats both, and with the current
     * transpose they push the 2-wave build past 256 VGPRs. */
    static const bool pf = getenv("OTC_BS_PF") && atoi(getenv("OTC_BS_PF")) != 0;
    const dim3 g((unsigned)wgs), b(256);
    /* Default: 3 waves per SIMD (<= 168 VGPRs with ~32 values in scratch):
     * +9..15% over the 2-wave builds below in every mode and key size, whose
     * register-hungry plaintext prefetches (PF, LDS) it makes unnecessary
     * (measured: docs/PERF.md).  OTC_BS_W3=0 selects the 2-wave builds. */
    static const bool w3 = !getenv("OTC_BS_W3") || atoi(getenv("OTC_BS_W3")) != 0;
    static const bool lds = getenv("OTC_BS_LDS") && atoi(getenv("OTC_BS_LDS")) != 0;
    /* OTC_BS_LOOP=1|2|3: rolled round loop (1: 3 waves + low-register
     * MixColumns, 2: 2 waves, 3: 3 waves + classic MixColumns);
     * OTC_BS_STAGGER=ticks: start stagger per residency slot (A/B knobs) */
    static const int loop = getenv("OTC_BS_LOOP") ? atoi(getenv("OTC_BS_LOOP")) : 0;
    BsParams Q = P;
    Q.stagger = getenv("OTC_BS_STAGGER") ? (uint32_t)atoi(getenv("OTC_BS_STAGGER")) : 0u;
    Q.cus = (uint32_t)device_cus();
    if (loop == 1) {
        hipLaunchKernelGGL((k_aes_bs_loop3<NR, MODE, true, 0>), g, b, 0, st, Q, K);
    } else if (loop == 2) {
        hipLaunchKernelGGL((k_aes_bs_loop2<NR, MODE, true, 0>), g, b, 0, st, Q, K);
    } else if (loop == 4) { /* 2 waves, 20 LDS-prefetched slots (2 x 80 KiB per CU) */
        hipLaunchKernelGGL((k_aes_bs_loop2<NR, MODE, true, (MODE == BS_CTR ? 20 : 0)>), g, b, 0, st, Q, K);
    } else if (loop == 5) { /* 2 waves, 16 LDS slots */
        hipLaunchKernelGGL((k_aes_bs_loop2<NR, MODE, true, (MODE == BS_CTR ? 16 : 0)>), g, b, 0, st, Q, K);
    } else if (loop == 7) { /* measurement only: 3 waves, zero key */
        hipLaunchKernelGGL((k_aes_bs_loop3<NR, MODE, true, 0, true>), g, b, 0, st, Q, K);
    } else if (loop == 8) { /* measurement only: 2 waves, zero key, LDS prefetch */
        hipLaunchKernelGGL((k_aes_bs_loop2<NR, MODE, true, (MODE == BS_CTR ? 20 : 0), true>), g, b, 0, st, Q, K);
    } else if (loop == 9) { /* 2 waves, LDS prefetch, pins only */
        hipLaunchKernelGGL((k_aes_bs_loop2<NR, MODE, true, (MODE == BS_CTR ? 20 : 0), false, 1>), g, b, 0, st, Q, K);
    } else if (loop == 10) { /* 2 waves, LDS prefetch, no fences */
        hipLaunchKernelGGL((k_aes_bs_loop2<NR, MODE, true, (MODE == BS_CTR ? 20 : 0), false, 0>), g, b, 0, st, Q, K);
    } else if (loop == 6) { /* 3 waves, 12 LDS slots (3 x 48 KiB per CU) */
        hipLaunchKernelGGL((k_aes_bs_loop3<NR, MODE, true, (MODE == BS_CTR ? 12 : 0)>), g, b, 0, st, Q, K);
    } else if (w3 && !(MODE == BS_CTR && cache)) {
        hipLaunchKernelGGL((k_aes_bs_w3<NR, MODE, 0>), g, b, 0, st, Q, K);
    } else if (MODE == BS_CTR && cache) {
        hipLaunchKernelGGL((k_aes_bs<NR, MODE, true, 0, 0>), g, b, 0, st, P, K);
    } else if constexpr (MODE == BS_CTR && NR == 10) {
        if (lds && pf)
            hipLaunchKernelGGL((k_aes_bs<NR, MODE, false, 8, 20>), g, b, 0, st, P, K);
        else if (lds)
            hipLaunchKernelGGL((k_aes_bs<NR, MODE, false, 0, 20>), g, b, 0, st, P, K);
        else if (pf)
            hipLaunchKernelGGL((k_aes_bs<NR, MODE, false, 8, 0>), g, b, 0, st, P, K);
        else
            hipLaunchKernelGGL((k_aes_bs<NR, MODE, false, 0, 0>), g, b, 0, st, P, K);
    } else {
        hipLaunchKernelGGL((k_aes_bs<NR, MODE, false, 0, 0>), g, b, 0, st, P, K);
    }
    return hipGetLastError();
}

template <int MODE>
hipError_t launch(const BsParams &P, const otc_aes_key &K, hipStream_t st)
{
    switch (K.nr) {
    case 10: return launch_nr<10, MODE>(P, K, st);
#ifndef OTC_BS_ONLY_NR10
    case 12: return launch_nr<12, MODE>(P, K, st);
    case 14: return launch_nr<14, MODE>(P, K, st);
#endif
    default: return hipErrorInvalidValue;
    }
}

} // namespace

namespace otc_impl {

hipError_t tt_ctr(const void *, void *, size_t, const otc_aes_key &, Ctr128, bool, hipStream_t, int);

hipError_t bs_ctr(const void *in, void *out, size_t nbytes, const otc_aes_key &K, Ctr128 c, bool wrap64,
                  hipStream_t st)
{
    if (nbytes % 16) {
        /* trailing partial block: T-table kernel, same counter stream */
        const size_t full = nbytes - nbytes % 16;
        Ctr128 ct = c;
        ct.lo = c.lo + full / 16;
        if (!wrap64 && ct.lo < c.lo) ct.hi += 1;
        hipError_t e = tt_ctr((const uint8_t *)in + full, (uint8_t *)out + full, nbytes % 16, K, ct, wrap64, st, 2);
        if (e != hipSuccess) return e;
        nbytes = full;
        if (nbytes == 0) return hipSuccess;
    }
    BsParams P{};
    P.in = (const uint8_t *)in;
    P.out = (uint8_t *)out;
    P.nblocks = nbytes / 16;
    P.tail = (uint32_t)(nbytes % 16);
    P.wrap64 = wrap64 ? 1u : 0u;
    P.shift = c.lo & 2047u;
    P.cbase.lo = c.lo & ~(uint64_t)2047u;
    P.cbase.hi = c.hi;
    return launch<BS_CTR>(P, K, st);
}

hipError_t bs_ecb_encrypt(const void *in, void *out, uint64_t nblocks, const otc_aes_key &K, hipStream_t st)
{
    BsParams P{};
    P.in = (const uint8_t *)in;
    P.out = (uint8_t *)out;
    P.nblocks = nblocks;
    return launch<BS_ECB>(P, K, st);
}

} // namespace otc_impl
