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
 *     n >= 11 : bit n of C                  (wave uniform)
 *
 * Default kernel (k_aes_bs_t3), built for 3 waves per SIMD (<= 168 VGPRs):
 *   - CTR counter caching (otc_bitslice.h): bytes 0..13 of the 2048 counters
 *     of a task are constant, so rounds 1-2 reduce to table reads (round-2
 *     S-box outputs per (group, lane) and per task, k_bs_ctr_table) and one
 *     partial MixColumns -- 32 of the 160 AES-128 S-boxes and 2 MixColumns
 *     rounds disappear;
 *   - the S-box's key-dependent terms (11 words per round byte, see
 *     sbox_key_terms) come from a per-call table written by k_bs_key_table
 *     and read with scalar loads next to each S-box: no SALU mask arithmetic
 *     and no round-key SGPRs live across the kernel;
 *   - a 77-LUT3 S-box (tools/sbox_choices.py: ILP cover over structural
 *     choices of the circuit) in minimum-live-plane order
 *     (tools/sbox_schedule.py) and a 55-node MixColumns column
 *     (tools/mixcol_search.py; the textbook forms take 76-80);
 *   - CTR: the plaintext of the first 8 slots goes straight to LDS by the
 *     DMA path (no VGPRs) once rounds 1-2 have consumed the counter-cache
 *     table loads, and lands while the other rounds run; the other slots are
 *     loaded 8 slots ahead of their use in groups of 4;
 *   - a bulk launch compiled for full tasks only, whose load / store
 *     phases are straight-line code with exact vmcnt waits, plus a
 *     one-workgroup launch for a partial first / last task (BS_FULL_ONLY /
 *     BS_EDGE_ONLY);
 *   - the last round key is folded into the output XOR (ks ^ rk ^ pt as one
 *     v_bitop3 per word) after the single output transpose.
 * Measurements (and the round-1 kernel this replaced): docs/PERF.md,
 * profiles/r2/bitslice.
 *
 * No reference counterpart (the reference has only a T-table CUDA kernel,
 * /root/reference/aes-gpu/Source/AES.cu:284-392).
 */
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <type_traits>

#include "otc_bitslice.h"
#include "otc_device.h"

using namespace otc_dev;
using namespace otc_bs;

namespace {

struct BsParams {
    const uint8_t *in;
    uint8_t *out;
    uint64_t nblocks;     /* full blocks */
    uint32_t tail;        /* CTR: trailing partial block bytes */
    uint32_t wrap64;      /* CTR: 64-bit counter increment */
    uint64_t shift;       /* CTR: ctr0.lo mod 2048 (virtual index = i + shift) */
    Ctr128 cbase;         /* CTR: ctr0 with the low 11 bits cleared */
    const uint32_t *ktab; /* key-term table (key_term_table layout) */
    const uint32_t *ctab; /* CTR counter caching: round-3 key terms per group */
    const uint32_t *e0tab; /* CTR counter caching: E0 words per (group, lane) */
    const uint32_t *e1tab; /* CTR counter caching: E1 plane words per task */
    uint64_t tasks;       /* 2048-block tasks of the call */
    uint32_t part;        /* BS_FULL_ONLY or BS_EDGE_ONLY */
    uint32_t iv[4];       /* CBC / CFB decrypt: IV as LE words (block 0's predecessor) */
    SplitClaim cl;        /* k_aes_bs_claim: units taken from the front of the buffer */
    Ctr128 iv0;           /* *_SEG: IV of segment 0 (numeric BE; IV_s = iv0 + s) */
    uint32_t seg_shift;   /* *_SEG: log2(blocks per segment) */
};

/* mode families: the CBC / CFB decryptions, whole-stream or per segment */
template <int MODE> constexpr bool is_cbcd = MODE == BS_CBC_DEC || MODE == BS_CBC_DEC_SEG;
template <int MODE> constexpr bool is_cfbd = MODE == BS_CFB_DEC || MODE == BS_CFB_DEC_SEG;
template <int MODE> constexpr bool is_seg = MODE == BS_CBC_DEC_SEG || MODE == BS_CFB_DEC_SEG;

/* Which tasks a launch runs.  The bulk launch (BS_FULL_ONLY) takes only tasks
 * whose 2048 slots are all in range and is compiled knowing it: its load and
 * store phases are single basic blocks, where hipcc's waitcnt pass keeps
 * precise vmcnt(N) counts -- per-slot range branches made it fall back to
 * vmcnt(0) around nearly every slot.  A one-workgroup launch (BS_EDGE_ONLY)
 * runs the first and the last task (wave 0 / wave 1) if they are partial. */
enum : uint32_t { BS_FULL_ONLY = 1, BS_EDGE_ONLY = 2 };

/* the modes BS_CTR .. BS_CFB_DEC: otc_device.h (engine.cpp names them too) */

__device__ __forceinline__ W lane_mask(uint32_t lane, int n) { return (W)(0u - ((lane >> n) & 1u)); }

/* v, or the IV where `first`: an explicit per-word blend after an unconditional
 * load from a valid address -- written as a select of the IV and the loaded
 * block, hipcc made a 16-byte private copy of the IV and loaded through a
 * pointer select (scratch traffic in every task) */
__device__ __forceinline__ uint4 blend_iv(uint4 v, bool first, const BsParams &P)
{
    const uint32_t m = 0u - (uint32_t)first;
    v.x = (v.x & ~m) | (P.iv[0] & m);
    v.y = (v.y & ~m) | (P.iv[1] & m);
    v.z = (v.z & ~m) | (P.iv[2] & m);
    v.w = (v.w & ~m) | (P.iv[3] & m);
    return v;
}

/* *_SEG: the block a slot reads one block back, or -- for lanes at a segment
 * start -- its own block with IV_s blended in.  The IV is built only when a
 * lane of the wave is at a segment start in this slot (a uniform branch: with
 * segments of >= 64 blocks, one slot in seg/64). */
template <int MODE>
__device__ __forceinline__ uint4 seg_prev(const BsParams &P, const uint8_t *own, uint64_t i, bool ok)
{
    const bool first = (i & ((1ull << P.seg_shift) - 1)) == 0;
    uint4 v = ok ? *(const uint4 *)(own - (first ? 0 : 16)) : make_uint4(0, 0, 0, 0);
    if (__builtin_amdgcn_ballot_w64(first)) {
        uint32_t w0, w1, w2, w3;
        ctr_words(P.iv0, i >> P.seg_shift, false, w0, w1, w2, w3);
        const uint32_t m = 0u - (uint32_t)first;
        v.x = (v.x & ~m) | (w0 & m);
        v.y = (v.y & ~m) | (w1 & m);
        v.z = (v.z & ~m) | (w2 & m);
        v.w = (v.w & ~m) | (w3 & m);
    }
    return v;
}

/* Waves per workgroup of the CTR launches (k_aes_bs_t3; the claim kernel
 * keeps 4): each wave is an independent 2048-block task, so the workgroup
 * only sets how many waves the dispatcher must place at once -- a 4-wave
 * group needs a free slot on all four SIMDs and its 32 KiB of staging LDS.
 * Smaller groups LOSE: AES-128 CTR 64 GiB 1705-1712 (1 wave) and 1710-1714
 * (2) vs 1726-1752 GB/s (4), AES-256 and 4 GiB alike, same held clock
 * (profiles/r6/wpg/, 3 interleaved reps). */
#ifndef OTC_BS_WPG
#define OTC_BS_WPG 4
#endif
constexpr uint32_t BS_WPG = OTC_BS_WPG;

/* Task geometry shared by both kernels. */
struct Task {
    uint32_t lane, wave;
    uint64_t vbase; /* virtual block index of slot 0, lane 0 */
    bool full;      /* every slot of the task is in range (uniform) */
};

template <int MODE>
__device__ __forceinline__ bool task_of(const BsParams &P, Task &t, int64_t claimed)
{
    if (claimed >= 0) {
        /* k_aes_bs_claim loops over tasks: the lane from mbcnt, opaque per
         * task, keeps hipcc from hoisting lane-derived values out of the loop
         * (live across the rounds, they spill); no staging slots, no wave */
        t.lane = lane_id();
        asm volatile("" : "+v"(t.lane));
        /* CTR stages its plaintext in per-wave LDS slots */
        t.wave = MODE == BS_CTR ? __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) : 0;
    } else {
        t.lane = threadIdx.x & 63u;
        t.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    }
    const uint64_t shift = (MODE == BS_CTR) ? P.shift : 0;
    /* one 2048-block task per wave, no grid-stride loop: a loop lets hipcc
     * hoist loop-invariant plane/mask values out of it, which costs more
     * registers than the 128-plane state leaves.  Full blocks only; the host
     * routes a trailing partial CTR block to the T-table kernel. */
    const uint32_t gw = (uint32_t)blockIdx.x * BS_WPG + t.wave; /* the wave's index in the launch */
    uint64_t task = claimed >= 0 ? (uint64_t)claimed : (uint64_t)gw;
    if (P.part == BS_EDGE_ONLY) {
        if (gw > 1 || (gw == 1 && P.tasks < 2)) return false;
        task = gw == 0 ? 0 : P.tasks - 1;
    }
    t.vbase = task * 2048u;
    if (t.vbase >= P.nblocks + shift) return false;
    t.full = t.vbase >= shift && t.vbase + 2048u - shift <= P.nblocks;
    if (P.part == BS_FULL_ONLY && !t.full) return false;
    if (P.part == BS_EDGE_ONLY && t.full) return false;
    return true;
}

/* Streaming cache policy (otc_device.h ld_u4 / st_u4).  OTC_BS_NT (default
 * 1): the non-temporal bit on every block this kernel reads or writes once --
 * the CTR plaintext loads (LDS DMA and register slots), the ECB / decryption
 * plane loads, the CBC / CFB XOR-block loads, every ciphertext store.  Round
 * 6 A/B, 64 GiB in place, 3 reps (profiles/r6/nt_ab/): AES-128 CTR 1705-1717
 * vs 1677-1687 GB/s at 0.795-0.803 vs 0.814-0.818 J/GB, AES-256 1275-1279 vs
 * 1248-1260 at 1.061-1.062 vs 1.088-1.095; the splits' bitsliced halves with
 * the T-table's streaming forms (aes_tt.hip OTC_TT_NT): +0.8-1.5%
 * (profiles/r6/ntall_ab/). */
#ifndef OTC_BS_NT
#define OTC_BS_NT 1
#endif
constexpr bool BS_NT = OTC_BS_NT != 0;
constexpr bool BS_NT_IN = BS_NT;
constexpr int BS_LDS_AUX = BS_NT ? 2 : 0; /* CPol: NT (SLC) bit of the LDS DMA loads */
__device__ __forceinline__ uint4 ld_stream(const uint8_t *p) { return ld_u4<BS_NT>(p); }
__device__ __forceinline__ void st_stream(uint8_t *p, uint4 v) { st_u4<BS_NT>(p, v); }

/* ECB input: load 32 blocks (uniform task base + 32-bit lane offsets: 64-bit
 * per-slot addresses would be CSE'd with the stores and kept live across the
 * rounds) and transpose each word column into 32 planes.  CFB decryption
 * enciphers the block before each output block: the same loads one block back,
 * with the IV in front of block 0 of a whole-stream call. */
template <int MODE>
__device__ __forceinline__ void ecb_load_planes(const BsParams &P, const Task &t, W *s, bool full)
{
    constexpr int64_t BACK = MODE == BS_CFB_DEC ? 16 : 0; /* the segment form reads through seg_prev */
    const uint8_t *tb = P.in + (int64_t)(t.vbase * 16) - BACK;
    const uint32_t lo = t.lane * 16u;
    uint4 blk[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) {
        const uint64_t i = t.vbase + t.lane + 64u * k;
        if constexpr (MODE == BS_CFB_DEC_SEG) {
            blk[k] = seg_prev<MODE>(P, tb + lo + 1024u * k, i, full || i < P.nblocks);
        } else if (MODE == BS_CFB_DEC && k == 0) {
            /* only slot 0 of lane 0 of task 0 can be block 0: it loads block 0
             * itself (a valid address) and takes the IV instead */
            const bool first = i == 0;
            const uint8_t *src = P.in + (int64_t)(t.vbase * 16) + lo - (first ? 0 : 16);
            blk[k] = blend_iv((full || i < P.nblocks) ? *(const uint4 *)src : make_uint4(0, 0, 0, 0), first, P);
        } else {
            blk[k] = (full || i < P.nblocks) ? ld_u4<BS_NT_IN>(tb + lo + 1024u * k) : make_uint4(0, 0, 0, 0);
        }
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

/* Key-term table of the schedule (otc_bs::key_term_table on the device):
 * one thread per (round, byte); written once per call into a stream-ordered
 * buffer, then read by every wave with scalar loads. */
template <bool DEC>
__global__ __launch_bounds__(256) void k_bs_key_table(otc_aes_key K, uint32_t *tab)
{
    const int e = (int)threadIdx.x; /* r * 16 + b */
    if (e >= K.nr * 16) return;
    const int r = e >> 4, b = e & 15;
    uint32_t byte = (K.rk[4 * r + (b >> 2)] >> (8 * (b & 3))) & 0xFFu;
    if (DEC) byte = dec_round_key_byte(byte, r); /* S-box input key of S^-1 = L S L */
    W k[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) k[i] = ((byte >> i) & 1u) ? ~0u : 0u;
    W t[OTC_SBOX_KEY_TERMS];
    sbox_key_terms(k[0], k[1], k[2], k[3], k[4], k[5], k[6], k[7], t);
    uint32_t *o = tab + e * OTC_BS_KT_STRIDE;
#pragma unroll
    for (int j = 0; j < OTC_SBOX_KEY_TERMS; ++j) o[j] = t[j];
    o[OTC_SBOX_KEY_TERMS] = 0;
}

using ktab_ptr = const __attribute__((address_space(4))) uint32_t *;

/* key terms of round R, byte b, by scalar loads from the table: no SALU
 * mask arithmetic (3.5k SALU instructions per 2048-block task otherwise) */
template <int R>
struct TableTerms {
    ktab_ptr tp;
    __device__ __forceinline__ void operator()(int b, W *t) const
    {
        ktab_ptr q = tp;
        asm volatile("" : "+s"(q)); /* loaded next to its S-box, not all hoisted */
#pragma unroll
        for (int j = 0; j < OTC_SBOX_KEY_TERMS; ++j) t[j] = q[(R * 16 + b) * OTC_BS_KT_STRIDE + j];
    }
};

/* Rounds unrolled at compile time (template recursion: a #pragma unroll
 * over this loop exceeds LLVM's unroll threshold; a rolled loop measured
 * slower -- its back edge permutes 128 planes and spills), low-register
 * MixColumns, S-box fence level 2 (per-S-box fences: LUT-level pins cost an
 * s_nop per asm boundary). */
/* key terms of the counter-cached round 3 from the task's group entry */
template <int BASE>
struct GroupTerms {
    ktab_ptr gp;
    __device__ __forceinline__ void operator()(int b, W *t) const
    {
        ktab_ptr q = gp;
        asm volatile("" : "+s"(q));
#pragma unroll
        for (int j = 0; j < OTC_SBOX_KEY_TERMS; ++j) t[j] = q[(BASE + b) * OTC_BS_KT_STRIDE + j];
    }
};

/* CTR counter-caching tables of one call (otc_bitslice.h, "CTR counter
 * caching"), one thread per entry: threads [0, ngroups) the round-3 key terms
 * of each group, then one per (group, lane) for E0, then one per task for E1.
 * Group g's counter prefix is (cbase with bits 0-15 cleared) + g * 2^16 with
 * the kernel's carry rule (128-bit, or 64-bit wrap); task t has group
 * ((cbase >> 11 & 31) + t) >> 5 and u5 = (cbase >> 11) + t mod 32, as in the
 * kernel.  The byte S-box comes from a 256-entry LDS table built per block. */
__global__ __launch_bounds__(256) void k_bs_ctr_table(otc_aes_key K, Ctr128 cbase, uint32_t wrap64,
                                                      uint64_t ngroups, uint64_t tasks, uint32_t *gtab,
                                                      uint32_t *e0tab, uint32_t *e1tab)
{
    __shared__ uint32_t sbt[256];
    sbt[threadIdx.x] = sbox_value(threadIdx.x);
    __syncthreads();
    const auto sb = [&](uint32_t v) { return sbt[v & 0xFFu]; };
    const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    auto rk0b = [&](int b) -> uint32_t { return (K.rk[b >> 2] >> (8 * (b & 3))) & 0xFFu; };
    uint64_t g;
    int kind;
    if (i < ngroups) {
        g = i;
        kind = 0;
    } else if (i < ngroups * 65) {
        g = (i - ngroups) >> 6;
        kind = 1;
    } else if (i < ngroups * 65 + tasks) {
        g = (((cbase.lo >> 11) & 31u) + (i - ngroups * 65)) >> 5;
        kind = 2;
    } else {
        return;
    }
    uint8_t pre[14];
    ctr_group_prefix(cbase.lo, cbase.hi, wrap64 != 0, g, pre);
    uint32_t c8[8];
    if (kind == 0) {
        ctr_group_consts(pre, K.rk, sb, c8, gtab + g * OTC_BS_CTR_GRP_WORDS);
    } else if (kind == 1) {
        ctr_group_consts(pre, K.rk, sb, c8, (uint32_t *)nullptr);
        const uint32_t lane = (uint32_t)(i - ngroups) & 63u;
        ctr_e0_lane(c8, rk0b(15), lane, sb, e0tab + (g * 64 + lane) * 8);
    } else {
        ctr_group_consts(pre, K.rk, sb, c8, (uint32_t *)nullptr);
        const uint64_t t = i - ngroups * 65;
        const uint32_t u5 = (uint32_t)((cbase.lo >> 11) + t) & 31u;
        ctr_e1_task(c8, rk0b(14), u5, sb, e1tab + t * OTC_BS_CTR_E1_WORDS);
    }
}

template <int R, int NR, int MIX, bool DEC = false>
__device__ __forceinline__ void rounds_table(W *s, ktab_ptr tp)
{
    if constexpr (R < NR - 1) {
        round_step_kt<MIX, TableTerms<R>, 2, DEC>(s, TableTerms<R>{tp});
        pin_n(s, 128);
        rounds_table<R + 1, NR, MIX, DEC>(s, tp);
    } else {
        round_final_kt<TableTerms<NR - 1>, DEC>(s, TableTerms<NR - 1>{tp});
    }
}

/* Default task.  LS: CTR plaintext slots prefetched into LDS (layout
 * [wave][slot][lane] x 16 B, exactly the lane-linear image the DMA writes;
 * each lane reads its own 16 B back with a conflict-free ds_read_b128).
 * PRE: register slots issued before the output transposes, whose ~1k VALU
 * ops cover their latency.  D: the other register slots are loaded D slots
 * ahead of use, in groups of 4, as the keystream of consumed slots frees
 * registers (loading all of them up front spills at 3 waves). */
/* register plaintext slots issued before the output transposes (2: with the
 * 81-LUT S-box (27 live planes at its peak) 4 early slots spilled in the
 * output phase; with the 79-LUT one (24) they no longer spill but measured
 * 1-1.5% slower, profiles/r3/sbox79; the 77-LUT one peaks at 23) */
#ifndef OTC_BS_CBC_D
#define OTC_BS_CBC_D 4
#endif
#ifndef OTC_BS_CFB_D
#define OTC_BS_CFB_D 2
#endif
#ifndef OTC_BS_PRE
#define OTC_BS_PRE 2
#endif
template <int NR, int MODE, int LS, bool CACHE, bool FO, int MIX = 2, int PRE = OTC_BS_PRE, int D = 8>
__device__ __forceinline__ void aes_bs_task(const BsParams &P, const otc_aes_key &K, uint4 *stage,
                                            int64_t claimed = -1)
{
    Task t;
    if (!task_of<MODE>(P, t, claimed)) return;
    const uint32_t lane = t.lane, wave = t.wave;
    const uint64_t shift = (MODE == BS_CTR) ? P.shift : 0;
    const bool full = FO || t.full; /* FO: a BS_FULL_ONLY launch */
    W s[128];
    /* with counter caching: issued after rounds 1-2 have consumed the
     * per-lane table loads -- vmcnt retires in order and hipcc waits for a
     * vector load queued behind LDS DMA with vmcnt(0), so a DMA issued first
     * put its whole latency in front of every task's round 1 */
    auto prefetch = [&]() {
    if (MODE == BS_CTR && LS > 0) {
        /* branch-free (a per-slot branch splits the kernel's one basic block
         * and costs registers): lanes outside the buffer load block 0 instead,
         * and their slots are never stored.  The rounds issue no vector memory
         * op, so no vmcnt wait before the output phase depends on these. */
        const int64_t t0 = (int64_t)t.vbase - (int64_t)shift;
        const uint8_t *ib0 = P.in + t0 * 16 + lane * 16u;
#pragma unroll
        for (int k = 0; k < LS; ++k) {
            const int64_t si = t0 + (int64_t)lane + 64 * k;
            const bool ok = full || (si >= 0 && (uint64_t)si < P.nblocks);
            __builtin_amdgcn_global_load_lds((const void *)(ok ? ib0 + 1024u * k : P.in),
                                             (__attribute__((address_space(3))) void *)&stage[(wave * LS + k) * 64],
                                             16, 0, BS_LDS_AUX);
        }
    }
    };
    if (!(MODE == BS_CTR && CACHE)) prefetch();
    if (MODE == BS_CTR && CACHE) {
        /* counter caching: rounds 1-2 from the per-group / per-task tables */
        const uint64_t task = t.vbase >> 11;
        const uint64_t g = (((P.cbase.lo >> 11) & 31u) + task) >> 5;
        const uint4 *q0 = (const uint4 *)(P.e0tab + (g * 64u + lane) * 8u);
        const uint4 a = q0[0], b = q0[1];
        const W ew[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
        W e0[32];
#pragma unroll
        for (int p = 0; p < 32; ++p) e0[p] = rep_byte(ew[p >> 2], p & 3);
        const ktab_ptr e1p = (ktab_ptr)P.e1tab + task * OTC_BS_CTR_E1_WORDS;
        W e1[32];
#pragma unroll
        for (int p = 0; p < 32; ++p) e1[p] = e1p[p];
        const ktab_ptr gp = (ktab_ptr)P.ctab + g * OTC_BS_CTR_GRP_WORDS;
        ctr_round2_mix(e0, e1, s);
        pin_n(s, 128);
        sched_fence();
        prefetch();
        sched_fence();
        round_step_kt<MIX, GroupTerms<0>, 2>(s, GroupTerms<0>{gp});
        pin_n(s, 128);
        sched_fence();
        rounds_table<3, NR, MIX>(s, (ktab_ptr)P.ktab);
    } else if (MODE == BS_CTR) {
        const uint64_t clo = P.cbase.lo + t.vbase;
        const uint64_t chi = P.cbase.hi + ((!P.wrap64 && clo < P.cbase.lo) ? 1u : 0u);
        /* the four counter words as VGPRs, so the 117 uniform counter planes
         * are made by VALU bit extracts straight into their VGPRs instead of
         * 117 live SGPRs first (SGPR spills otherwise) */
        uint32_t cw[4] = {(uint32_t)clo, (uint32_t)(clo >> 32), (uint32_t)chi, (uint32_t)(chi >> 32)};
#pragma unroll
        for (int j = 0; j < 4; ++j) asm volatile("" : "+v"(cw[j]));
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
                } else {
                    v = (W)(0u - ((cw[n >> 5] >> (n & 31)) & 1u));
                }
                s[8 * b + i] = v;
            }
        }
#pragma unroll
        for (int q = 0; q < 128; ++q) asm volatile("" : "+v"(s[q]));
    } else {
        ecb_load_planes<MODE>(P, t, s, full);
    }
    constexpr bool DEC = MODE == BS_ECB_DEC || is_cbcd<MODE>;
    if (DEC) {
        dec_premap(s); /* L on every ciphertext byte */
        pin_n(s, 128);
    }
    if (!(MODE == BS_CTR && CACHE)) {
        sched_fence();
        rounds_table<0, NR, MIX, DEC>(s, (ktab_ptr)P.ktab);
    }
    pin_n(s, 128);
    sched_fence();

    const int64_t tstart = (int64_t)t.vbase - (int64_t)shift;
    const uint8_t *ib = P.in + tstart * 16;
    uint8_t *ob = P.out + tstart * 16;
    uint32_t lo = lane * 16u;
    /* ordered after the pins above (volatile asms keep their order), so the
     * loads below cannot be hoisted into the round phase */
    asm volatile("" : "+v"(lo));
    auto slot_ok = [&](int k) {
        const int64_t si = tstart + (int64_t)lane + 64 * k;
        return full || (si >= 0 && (uint64_t)si < P.nblocks);
    };
    /* register-loaded plaintext (slots LS..31); none is issued behind a
     * store -- vmcnt is in order on gfx9, so such a load would also wait for
     * the stores */
    /* the block XORed into the output: CTR the plaintext, CBC decrypt the
     * previous ciphertext block (the IV for block 0 of a whole-stream call),
     * CFB decrypt the ciphertext block itself */
    constexpr bool XIN = MODE == BS_CTR || is_cbcd<MODE> || is_cfbd<MODE>;
    constexpr int XOFF = MODE == BS_CBC_DEC ? -16 : 0;
    uint4 pt[32];
    auto issue = [&](int j) {
        if (XIN && j >= LS && j < 32) {
            if constexpr (MODE == BS_CBC_DEC_SEG) {
                pt[j] = seg_prev<MODE>(P, ib + lo + 1024u * j, (uint64_t)(tstart + lane + 64 * j),
                                       slot_ok(j));
            } else if (MODE == BS_CBC_DEC && j == 0) {
                /* block 0 of a whole-stream call XORs with the IV: it loads
                 * itself (a valid address) and blends the IV in */
                const bool first = tstart + lane == 0;
                const uint4 v = slot_ok(j) ? *(const uint4 *)(ib + lo + (first ? 0 : XOFF)) : make_uint4(0, 0, 0, 0);
                pt[j] = blend_iv(v, first, P);
            } else {
                pt[j] = slot_ok(j) ? ld_stream(ib + lo + 1024u * j + XOFF) : make_uint4(0, 0, 0, 0);
            }
        }
    };
    /* CBC / CFB decrypt load all 32 XOR blocks into registers (CTR stages 8 in
     * LDS): few slots ahead (CBC 4, CFB 2: 163 VGPRs, no scratch; 4 spills),
     * none early, or the output phase spills */
    constexpr bool REG_XIN = is_cbcd<MODE> || is_cfbd<MODE>;
    constexpr int PRE_ = REG_XIN ? 0 : PRE, D_ = is_cfbd<MODE> ? OTC_BS_CFB_D : REG_XIN ? OTC_BS_CBC_D : D;
#pragma unroll
    for (int j = 0; j < LS + PRE_; ++j) issue(j);
    sched_fence();
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        transpose32(s + 32 * w);
        pin_n(s + 32 * w, 32);
        sched_fence();
    }
    /* last round key; decryption adds the 0x05 the post-map L leaves */
    constexpr uint32_t KD = DEC ? 0x05050505u : 0u;
    const uint32_t k0 = K.rk[4 * NR + 0] ^ KD, k1 = K.rk[4 * NR + 1] ^ KD, k2 = K.rk[4 * NR + 2] ^ KD,
                   k3 = K.rk[4 * NR + 3] ^ KD;
    auto ks_xor = [&](int k, uint4 x) {
        uint4 o;
        o.x = x3(x.x, s[k], k0);
        o.y = x3(x.y, s[32 + k], k1);
        o.z = x3(x.z, s[64 + k], k2);
        o.w = x3(x.w, s[96 + k], k3);
        return o;
    };
#pragma unroll
    for (int k = 0; k < 32; ++k) {
        if ((k & 3) == 0) {
            sched_fence();
#pragma unroll
            for (int j = LS + PRE_; j < 32; ++j)
                if ((j - D_ < 0 ? 0 : ((j - D_) & ~3)) == k) issue(j);
        }
        if (slot_ok(k)) {
            const uint4 o = XIN ? ks_xor(k, k < LS ? stage[(wave * LS + k) * 64 + (lo >> 4)] : pt[k])
                                : make_uint4(s[k] ^ k0, s[32 + k] ^ k1, s[64 + k] ^ k2, s[96 + k] ^ k3);
            st_stream(ob + lo + 1024u * k, o);
        }
    }
}

/* CTR: 8 LDS slots (4 waves x 8 x 1 KiB = 32 KiB per workgroup, 3
 * workgroups per CU); ECB loads its whole input before the rounds. */
#ifndef OTC_BS_LS
#define OTC_BS_LS 8
#endif
constexpr int BS_LS = OTC_BS_LS;


template <int NR, int MODE, int LS, bool CACHE, bool FO>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3, 3))) void k_aes_bs_t3(BsParams P,
                                                                                             otc_aes_key K)
{
    __shared__ uint4 stage[LS > 0 ? BS_WPG * LS * 64 : 1];
    aes_bs_task<NR, MODE, LS, CACHE, FO>(P, K, stage);
}

/* The bitsliced half of a claimed co-resident split (otc_device.h
 * SplitClaim): each wave takes whole 2048-block tasks from the front of the
 * buffer until none are left.  No LDS, so it fits beside the 160 KiB
 * decryption T-table; the loop is the only one in a bitsliced kernel (the
 * task body is unchanged: no hoisted state, same VGPRs -- tests/test_isa_cpu.py). */
template <int NR, int MODE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3, 3))) void k_aes_bs_claim(BsParams P,
                                                                                               otc_aes_key K)
{
    strace(3);
    const uint32_t w = blockIdx.x * 4u + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (int64_t u = first_unit(P.cl, false, w); u >= 0; u = claim_unit(P.cl, false)) {
        /* the buffers opaque per task, as the lane (task_of): nothing derived
         * from them is hoisted; laundered as global pointers, or the loads and
         * stores become flat ones */
        BsParams Q = P;
        auto gin = (__attribute__((address_space(1))) const uint8_t *)P.in;
        auto gout = (__attribute__((address_space(1))) uint8_t *)P.out;
        asm volatile("" : "+s"(gin), "+s"(gout));
        Q.in = (const uint8_t *)gin;
        Q.out = (uint8_t *)gout;
        aes_bs_task<NR, MODE, 0, false, true>(Q, K, nullptr, u);
    }
}

template <int NR, int MODE>
hipError_t launch_nr(const BsParams &P, const otc_aes_key &K, hipStream_t st)
{
    const uint64_t vt = P.nblocks + (MODE == BS_CTR ? P.shift : 0);
    const uint64_t tasks = (vt + 2047) / 2048;
    uint64_t wgs = (tasks + BS_WPG - 1) / BS_WPG;
    if (wgs < 1) wgs = 1;
    if (wgs > 0xFFFFFFFFull) return hipErrorInvalidValue;
    const dim3 g((unsigned)wgs), b(64 * BS_WPG);
    /* CTR counter caching (+34% over no caching, profiles/r2/bitslice) */
    bool cache = MODE == BS_CTR;
    const uint64_t ngroups = cache ? (((P.cbase.lo >> 11) & 31u) + tasks + 31) >> 5 : 0;
    const size_t ctab_words =
        cache ? ngroups * (OTC_BS_CTR_GRP_WORDS + OTC_BS_CTR_E0_WORDS) + tasks * OTC_BS_CTR_E1_WORDS : 0;
    const size_t kt_words = (size_t)NR * 16 * OTC_BS_KT_STRIDE;
    /* per-call tables, stream-ordered: written by small kernels, freed behind
     * the main kernel (the pool recycles the memory).  The counter-caching
     * tables are ~0.6% of the data (2.8 KiB per 1 MiB group + 128 B per
     * 32 KiB task); if they do not fit beside a near-full HBM, CTR runs
     * without counter caching rather than failing. */
    uint32_t *tab = nullptr;
    hipError_t e = hipErrorOutOfMemory;
    if (cache) {
        e = alloc_fault() ? hipErrorOutOfMemory : hipMallocAsync((void **)&tab, (kt_words + ctab_words) * 4, st);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            cache = false;
        }
    }
    if (!cache) e = alloc_fault() ? hipErrorOutOfMemory : hipMallocAsync((void **)&tab, kt_words * 4, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_bs_key_table<MODE == BS_ECB_DEC || is_cbcd<MODE>>, dim3(1), dim3(256), 0, st, K, tab);
    BsParams Q = P;
    Q.ktab = tab;
    Q.tasks = tasks;
    constexpr int LS = MODE == BS_CTR ? BS_LS : 0;
    /* Split launch: a bulk launch compiled for full tasks only (straight-line
     * load / store phases with exact vmcnt waits) + a one-workgroup launch
     * for a partial first / last task.  One launch with per-slot range checks
     * measured slower for both modes: ECB 1178 vs 1240 GB/s (4 GiB,
     * profiles/r2/bitslice_out), CTR (64 GiB, with the key-term prefetch)
     * 1547/1551 vs 1606/1606 (profiles/r3/split). */
    if constexpr (MODE != BS_CTR) {
        /* ECB and the decryptions run only as claim kernels: beside the
         * T-table (the split: one workgroup per CU), or alone (impl
         * "bitslice": cl.wgs = 3 per CU, the T-table claim kernel does the
         * blocks past the last unit) */
        (void)g;
        if (!P.cl.ctr) {
            (void)hipFreeAsync(tab, st);
            return hipErrorInvalidValue;
        }
        hipLaunchKernelGGL((k_aes_bs_claim<NR, MODE>),
                           dim3(P.cl.wgs ? P.cl.wgs : (unsigned)otc_dev::device_cus()), dim3(256), 0, st, Q, K);
    } else {
        const bool edge = P.shift != 0 || vt % 2048 != 0;
        auto run = [&](auto cachec) {
            constexpr bool C = decltype(cachec)::value;
            Q.part = BS_FULL_ONLY;
            hipLaunchKernelGGL((k_aes_bs_t3<NR, MODE, LS, C, true>), g, b, 0, st, Q, K);
            if (edge) {
                Q.part = BS_EDGE_ONLY;
                hipLaunchKernelGGL((k_aes_bs_t3<NR, MODE, LS, C, false>), dim3((2 + BS_WPG - 1) / BS_WPG), b, 0, st,
                                   Q, K);
            }
        };
        if (cache) {
            uint32_t *gt = tab + kt_words, *e0 = gt + ngroups * OTC_BS_CTR_GRP_WORDS,
                     *e1 = e0 + ngroups * OTC_BS_CTR_E0_WORDS;
            Q.ctab = gt;
            Q.e0tab = e0;
            Q.e1tab = e1;
            const uint64_t n = ngroups * 65 + tasks;
            hipLaunchKernelGGL(k_bs_ctr_table, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, K, P.cbase,
                               P.wrap64, ngroups, tasks, gt, e0, e1);
        }
        if (cache)
            run(std::true_type{});
        else
            run(std::false_type{});
    }
    e = hipGetLastError();
    const hipError_t f = hipFreeAsync(tab, st);
    return e != hipSuccess ? e : f;
}

template <int MODE>
hipError_t launch(const BsParams &P, const otc_aes_key &K, hipStream_t st)
{
    switch (K.nr) {
    case 10: return launch_nr<10, MODE>(P, K, st);
    case 12: return launch_nr<12, MODE>(P, K, st);
    case 14: return launch_nr<14, MODE>(P, K, st);
    default: return hipErrorInvalidValue;
    }
}

} // namespace

namespace otc_impl {

OTC_STRACE_READER(strace_read_bs)

hipError_t tt_ctr(const void *, void *, size_t, const otc_aes_key &, Ctr128, bool, hipStream_t);

hipError_t bs_ctr(const void *in, void *out, size_t nbytes, const otc_aes_key &K, Ctr128 c, bool wrap64,
                  hipStream_t st)
{
    if (nbytes % 16) {
        /* trailing partial block: T-table kernel, same counter stream */
        const size_t full = nbytes - nbytes % 16;
        Ctr128 ct = c;
        ct.lo = c.lo + full / 16;
        if (!wrap64 && ct.lo < c.lo) ct.hi += 1;
        hipError_t e = tt_ctr((const uint8_t *)in + full, (uint8_t *)out + full, nbytes % 16, K, ct, wrap64, st);
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

/* One-time warm-up of the split's bitsliced half (engine.cpp aux_take, when
 * a device's first auxiliary stream is created): the runtime loads this
 * file's code object at the first lookup of one of its kernels, and a first
 * split call otherwise paid for that after its T-table half had started --
 * which then took every unit (profiles/r6/coresidency/matrix.jsonl). */
hipError_t bs_preload()
{
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, reinterpret_cast<const void *>(&k_aes_bs_claim<14, BS_ECB>));
}

/* The bitsliced halves of a claimed split: the whole buffer (block 0's
 * predecessor is iv_le), units from the front of `cl` */
hipError_t bs_claim(int mode, const void *in, void *out, uint64_t nblocks, const otc_aes_key &K,
                    const uint32_t iv_le[4], SplitClaim cl, hipStream_t st)
{
    BsParams P{};
    P.in = (const uint8_t *)in;
    P.out = (uint8_t *)out;
    P.nblocks = nblocks;
    for (int i = 0; i < 4; ++i) P.iv[i] = iv_le ? iv_le[i] : 0u;
    P.cl = cl;
    switch (mode) {
    case BS_ECB: return launch<BS_ECB>(P, K, st);
    case BS_ECB_DEC: return launch<BS_ECB_DEC>(P, K, st);
    case BS_CBC_DEC: return launch<BS_CBC_DEC>(P, K, st);
    case BS_CFB_DEC: return launch<BS_CFB_DEC>(P, K, st);
    default: return hipErrorInvalidValue;
    }
}

/* ... and of a claimed split over independent segments of 2^seg_shift
 * blocks, segment s chained from IV_s = iv0 + s */
hipError_t bs_claim_seg(int mode, const void *in, void *out, uint64_t nblocks, const otc_aes_key &K, Ctr128 iv0,
                        uint32_t seg_shift, SplitClaim cl, hipStream_t st)
{
    BsParams P{};
    P.in = (const uint8_t *)in;
    P.out = (uint8_t *)out;
    P.nblocks = nblocks;
    P.iv0 = iv0;
    P.seg_shift = seg_shift;
    P.cl = cl;
    switch (mode) {
    case BS_CBC_DEC_SEG: return launch<BS_CBC_DEC_SEG>(P, K, st);
    case BS_CFB_DEC_SEG: return launch<BS_CFB_DEC_SEG>(P, K, st);
    default: return hipErrorInvalidValue;
    }
}

} // namespace otc_impl
