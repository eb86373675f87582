/*
 * aes_tt.hip -- AES T-table kernels for gfx950 with the table resident in LDS.
 *
 * Reference counterpart: AES_encrypt / AES_decrypt
 * (/root/reference/aes-gpu/Source/AES.cu:284-502), one CUDA thread per block
 * with four T tables in uncached global memory, a __shared__ state shared by
 * the whole block (data race) and a launch that asked for the whole buffer as
 * dynamic shared memory (never ran).  This file is a gfx950-first design:
 *
 *  * T0..T3 (T_k = rotl(T0, 8k)) each replicated 32 ways in 128 KiB of LDS:
 *    entry x of table k for lane l lives at byte
 *    (k >> 1) << 16 | x << 8 | (k & 1) << 7 | (l & 31) << 2, so the two
 *    32-lane groups of a ds_read_b32 each hit 32 distinct banks --
 *    conflict free for any data.
 *  * The LDS address of a lookup is ONE v_perm_b32: byte 1 <- the state byte,
 *    bytes 0 and 2 <- a per-lane, per-table constant.  A round costs per block
 *    16 ds_read_b32 + 16 v_perm + 8 v_xor3 (issued all lookups first).
 *  * Last round reuses the T tables: S[x] is one byte of each T_k[x]; two
 *    v_perm + one xor3 assemble a column with the last round key.
 *  * Round keys arrive BY VALUE in the kernel arguments (otc_aes_key), i.e.
 *    they are wave-uniform SGPR operands of the v_xor3s.
 *  * Each lane carries B independent blocks (ILP across LDS latency); block
 *    index = chunk + wave*64*B + b*64 + lane, so every global access is a
 *    fully coalesced 1 KiB dwordx4 wave access.  Persistent grid-stride loop
 *    amortises the table fill.
 *  * CTR: counter-mode caching (k_aes_ctr_tt_cached): bytes 0..14 of a wave's
 *    counters are uniform, so rounds 1-2 need 5 instead of 32 lookups/block.
 *  * Decryption keeps Td0..Td3 (128 KiB) + the inverse S-box replicated as
 *    words (32 KiB) = the whole 160 KiB LDS, same one-op v_perm addressing.
 * Measurements and rejected variants (1-table layout, non-temporal accesses,
 * other shapes): docs/PERF.md.
 */
#include <hip/hip_runtime.h>

#include <algorithm>

#include <atomic>
#include <cstdio>
#include <cstdlib>

#include "otc_device.h"

using namespace otc_dev;

/* compile-time A/B switches (make variant NAME=x VFLAGS=-D...; docs/PERF.md) */
#ifndef OTC_SEG_G
#define OTC_SEG_G 8 /* blocks per load burst, grouped segment encryption (A/B knob) */
#endif
/* the segment claim kernel: single-buffered 8-block bursts (60-65 VGPRs; 3-5%
 * faster than double-buffered 4-block ones, non-temporal loads / stores far
 * slower: profiles/r5/seg_split/tt_claim_ab.jsonl, tt_sb_ab.jsonl) */
constexpr int SEG_CLAIM_G = 8;
#ifndef OTC_TT_CTR_B
#define OTC_TT_CTR_B 4 /* blocks per lane, bulk CTR kernel (A/B knob: 2 fits a bitsliced wave beside it) */
#endif
#ifndef OTC_TT_ENC_B
#define OTC_TT_ENC_B 4 /* blocks per lane, bulk ECB-encrypt / CFB-decrypt kernel */
#endif
#ifndef OTC_TT_DEC_B
#define OTC_TT_DEC_B 4 /* blocks per lane, bulk ECB / CBC decrypt kernel */
#endif

namespace {

__device__ const AesTables g_tab = make_tables();



/* second table (byte 2 of the address taken from lane word byte 2 = 1) */
constexpr uint32_t SEL_HI(int k) { return 0x0c020000u | ((uint32_t)(4 + k) << 8); }

__device__ __forceinline__ uint32_t lds_at(const uint32_t *tbl, uint32_t byte_addr)
{
    return *(const uint32_t *)((const char *)tbl + byte_addr);
}

/* The claim kernels' tables live in dynamic LDS (tt_lds below), which starts
 * at address 0 -- those kernels declare no static LDS (tests/test_isa_cpu.py
 * checks their descriptors' fixed group segment size is 0).  hipcc learns the
 * dynamic base only after instruction selection, so addressing through the
 * extern array adds it to every lookup (v_add_u32 v, 0, v: +1792 VALU per
 * AES-256 ECB claim-loop iteration, +36% instructions, ~8-10% slower).  Their
 * lookups take the integer LDS address instead. */
struct DynTbl {
};

/* Negative control for the co-residency test (tests/test_gpu_queues.py):
 * `make variant NAME=padclaim VFLAGS=-DOTC_DIAG_PAD_CLAIM` pads the T-table
 * claim kernels' register descriptors to a 4-waves-per-SIMD budget -- what the
 * round-4 static-LDS build did by accident -- so no bitsliced wave fits beside
 * them and the split's halves run one after the other.  Never in the release
 * build. */
#ifdef OTC_DIAG_PAD_CLAIM
#define OTC_CLAIM_ATTR __attribute__((amdgpu_waves_per_eu(4, 4)))
#else
#define OTC_CLAIM_ATTR
#endif
__device__ __forceinline__ uint32_t lds_at(DynTbl, uint32_t byte_addr)
{
    return *(const __attribute__((address_space(3))) uint32_t *)(uintptr_t)byte_addr;
}

/* LDS address of table k's entry for byte k of state word w: byte 1 <- that
 * byte, bytes 0 / 2 <- the per-lane, per-table constant lkk (whose bytes 1
 * and 3 are zero).  For k = 1 the byte is already in place, so the address is
 * one bit-field insert (v_bfi_b32, ~0.75 nJ per wave-instruction) instead of
 * a v_perm_b32 (~1.03 nJ, profiles/r3/energy/): a quarter of all lookups. */
__device__ __forceinline__ uint32_t tt_addr(uint32_t w, uint32_t lkk, int k)
{
    if (k == 1) {
        /* written out: hipcc turns the C form into v_and_or_b32 (0.83 nJ,
         * and a costlier VOP3 issue than v_perm) */
        uint32_t r;
        asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "s"(0x0000FF00u), "v"(w), "v"(lkk));
        return r;
    }
    return __builtin_amdgcn_perm(w, lkk, SEL_HI(k));
}

/* 4-table layout (TBL4): T_k (k = 0..3, T_k = rotl(T0, 8k)) each replicated
 * 32 ways.  Row x of region r (r = k >> 1, 64 KiB each) holds T_{2r} for lanes
 * 0..31 in bytes 0..127 and T_{2r+1} in bytes 128..255:
 *   addr(k, x, lane) = (k >> 1) << 16 | x << 8 | (k & 1) << 7 | (lane & 31) << 2
 * so again one v_perm per lookup (byte 1 <- x, bytes 0/2 <- a per-lane,
 * per-table constant) and no rotations: 16 perm + 8 bitop3 per round instead
 * of 16 + 12 + 8.  Bank = lane & 31 for every lookup -> conflict free. */
template <int THREADS>
__device__ __forceinline__ void fill_tbl4(uint32_t *lds, const uint32_t *te0)
{
    uint4 *l4 = reinterpret_cast<uint4 *>(lds);
    for (int q = threadIdx.x; q < 8192; q += THREADS) {
        const int r = q >> 12, x = (q >> 4) & 255, half = (q >> 3) & 1;
        const int k = 2 * r + half;
        const uint32_t t = te0[x];
        const uint32_t v = k ? ((t << (8 * k)) | (t >> (32 - 8 * k))) : t;
        l4[q] = make_uint4(v, v, v, v);
    }
}

__device__ __forceinline__ void tbl4_lane_consts(uint32_t lane, uint32_t (&lk)[4])
{
#pragma unroll
    for (int k = 0; k < 4; ++k) lk[k] = ((uint32_t)(k >> 1) << 16) | ((uint32_t)(k & 1) << 7) | ((lane & 31u) << 2);
}

/* Per round, issue every lookup of all B blocks before combining any of
 * them (+0..1.6%, profiles/r1/otbench_issue_all_ab.jsonl).  hipcc otherwise consumes each ds_read right away (1-3 LDS ops
 * in flight per wave); with at most 16 waves per CU (the 128 KiB table allows
 * one workgroup) that starves the LDS pipe.  gfx9 lgkmcnt still caps a wave at
 * 15 outstanding LDS ops. */
template <int R0, int NR, int B, class TBL>
__device__ __forceinline__ void enc_rounds4_from(TBL tbl, const uint32_t (&lk)[4], const otc_aes_key &K,
                                                 uint32_t (&s)[B][4])
{
#pragma unroll
    for (int r = R0; r < NR; ++r) {
        uint32_t t[B][4];
        uint32_t a[B][4][4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int b = 0; b < B; ++b)
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    a[b][j][k] = lds_at(tbl, tt_addr(s[b][(j + k) & 3], lk[k], k));
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int b = 0; b < B; ++b)
                t[b][j] = xor3(xor3(a[b][j][0], a[b][j][1], a[b][j][2]), a[b][j][3], K.rk[4 * r + j]);
#pragma unroll
        for (int b = 0; b < B; ++b)
#pragma unroll
            for (int j = 0; j < 4; ++j) s[b][j] = t[b][j];
    }
    uint32_t t[B][4];
    uint32_t a[B][4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int b = 0; b < B; ++b)
#pragma unroll
            for (int k = 0; k < 4; ++k)
                a[b][j][k] = lds_at(tbl, tt_addr(s[b][(j + k) & 3], lk[k], k));
#pragma unroll
    for (int b = 0; b < B; ++b) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            /* S[x] sits in byte 1 of T0, byte 2 of T1, byte 3 of T2, byte 0 of T3 */
            uint32_t lo = __builtin_amdgcn_perm(a[b][j][1], a[b][j][0], 0x0c0c0601u);
            uint32_t hi = __builtin_amdgcn_perm(a[b][j][3], a[b][j][2], 0x04030c0cu);
            t[b][j] = xor3(lo, hi, K.rk[4 * NR + j]);
        }
    }
#pragma unroll
    for (int b = 0; b < B; ++b)
#pragma unroll
        for (int j = 0; j < 4; ++j) s[b][j] = t[b][j];
}

/* Decryption 4-table layout: Td0..Td3 as above (128 KiB) plus the inverse
 * S-box replicated 32 ways as byte-splatted words at 0x20000 + x*128 + lane*4
 * (32 KiB): 160 KiB, the whole LDS of a CU.  The final-round address is one
 * v_perm + one shift: perm gives 0x40000 | x << 8 | lane*8, >> 1 gives the
 * row-128 address. */
template <int THREADS>
__device__ __forceinline__ void fill_dtbl4(uint32_t *lds, const uint32_t *td0, const uint32_t *is4)
{
    uint4 *l4 = reinterpret_cast<uint4 *>(lds);
    for (int q = threadIdx.x; q < 8192 + 2048; q += THREADS) {
        uint32_t v;
        if (q < 8192) {
            const int r = q >> 12, x = (q >> 4) & 255, half = (q >> 3) & 1;
            const int k = 2 * r + half;
            const uint32_t t = td0[x];
            v = k ? ((t << (8 * k)) | (t >> (32 - 8 * k))) : t;
        } else {
            v = is4[(q - 8192) >> 3]; /* 8 uint4 (32 dwords) per 128-byte row */
        }
        l4[q] = make_uint4(v, v, v, v);
    }
}

template <int NR, int B, class TBL>
__device__ __forceinline__ void dec_rounds4(TBL tbl, const uint32_t (&lk)[4], uint32_t lk_is2,
                                            const otc_aes_key &K, uint32_t (&s)[B][4])
{
#pragma unroll
    for (int r = 1; r < NR; ++r) {
        uint32_t t[B][4];
#pragma unroll
        for (int b = 0; b < B; ++b) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                uint32_t a0 = lds_at(tbl, tt_addr(s[b][j], lk[0], 0));
                uint32_t a1 = lds_at(tbl, tt_addr(s[b][(j + 3) & 3], lk[1], 1));
                uint32_t a2 = lds_at(tbl, tt_addr(s[b][(j + 2) & 3], lk[2], 2));
                uint32_t a3 = lds_at(tbl, tt_addr(s[b][(j + 1) & 3], lk[3], 3));
                t[b][j] = xor3(xor3(a0, a1, a2), a3, K.rk[4 * r + j]);
            }
        }
#pragma unroll
        for (int b = 0; b < B; ++b)
#pragma unroll
            for (int j = 0; j < 4; ++j) s[b][j] = t[b][j];
    }
    uint32_t t[B][4];
#pragma unroll
    for (int b = 0; b < B; ++b) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            uint32_t a0 = lds_at(tbl, tt_addr(s[b][j], lk_is2, 0) >> 1);
            uint32_t a1 = lds_at(tbl, tt_addr(s[b][(j + 3) & 3], lk_is2, 1) >> 1);
            uint32_t a2 = lds_at(tbl, tt_addr(s[b][(j + 2) & 3], lk_is2, 2) >> 1);
            uint32_t a3 = lds_at(tbl, tt_addr(s[b][(j + 1) & 3], lk_is2, 3) >> 1);
            uint32_t lo = __builtin_amdgcn_perm(a1, a0, 0x0c0c0400u);
            uint32_t hi = __builtin_amdgcn_perm(a3, a2, 0x04000c0cu);
            t[b][j] = xor3(lo, hi, K.rk[4 * NR + j]);
        }
    }
#pragma unroll
    for (int b = 0; b < B; ++b)
#pragma unroll
        for (int j = 0; j < 4; ++j) s[b][j] = t[b][j];
}

__device__ __forceinline__ uint4 ld16(const uint8_t *p, uint64_t blk) { return ld_u4<false>(p + 16 * blk); }
__device__ __forceinline__ void st16(uint8_t *p, uint64_t blk, uint4 v) { st_u4<false>(p + 16 * blk, v); }
/* Streaming forms (otc_device.h ld_u4 / st_u4) for the kernels whose wave
 * loads / stores 1 KiB of consecutive blocks per instruction -- ECB, CTR, the
 * CFB / CBC decryptions and their claim forms: the non-temporal bit
 * (OTC_TT_NT, default 1).  Round 6 A/B (profiles/r6/ntall_ab/, AES-256, 2
 * reps): the splits +0.8-1.5% (CBC-dec 8 GiB 1205-1208 vs 1188-1194), ECB-dec
 * +1%, T-table CTR even.  NOT the serial segment chains: there each lane
 * walks its own segment 16 B at a time, the next block sits in the line just
 * read, and without the line in cache every block refetches it -- CBC
 * segment encryption fell from 1114-1120 to 472-476 GB/s with the bit. */
#ifndef OTC_TT_NT
#define OTC_TT_NT 1
#endif
__device__ __forceinline__ uint4 lds16(const uint8_t *p, uint64_t blk) { return ld_u4<OTC_TT_NT != 0>(p + 16 * blk); }
__device__ __forceinline__ void sts16(uint8_t *p, uint64_t blk, uint4 v) { st_u4<OTC_TT_NT != 0>(p + 16 * blk, v); }
enum : int { E_ECB = 0, E_CFB_DEC = 2, E_CFB_DEC_SEG = 3 };
enum : int { D_ECB = 0, D_CBC = 1, D_CBC_SEG = 2 };

struct EncParams {
    const uint8_t *in;
    uint8_t *out;
    uint64_t nfull;   /* full 16-byte blocks */
    Ctr128 ctr;       /* CFB_DEC_SEG: IV of segment 0 (IV_s = ctr + s) */
    uint32_t iv[4];   /* CFB: IV as LE words */
    uint64_t seg_blocks; /* CFB_DEC_SEG: blocks per segment */
    uint32_t seg_shift;  /* CFB_DEC_SEG: log2(seg_blocks), or 64 if not a power of two */
    SplitClaim cl;       /* CLAIM kernels: units taken from the back of the buffer */
};

struct DecParams {
    const uint8_t *in;
    uint8_t *out;
    uint64_t nfull;
    uint32_t seg_shift; /* D_CBC_SEG: log2(blocks per segment) */
    uint32_t pad;
    Ctr128 iv;          /* CBC: IV (numeric BE); CBC_SEG: IV of segment 0 */
    SplitClaim cl;      /* CLAIM kernels: units taken from the back of the buffer */
};

/* ---------------------------------------------------------------------------
 * Encryption-direction kernel: ECB-enc, CFB128-dec (CTR has its own
 * counter-caching kernel below)
 * ------------------------------------------------------------------------- */
/* The T tables in LDS.  The claim kernels (CLAIM / DYN) take them as dynamic
 * LDS, sized at launch (launch_dyn below): with a static 128 / 160 KiB array
 * hipcc knows the workgroup fills the CU and pads the kernel descriptor's
 * register count up to the occupancy the LDS allows (4 waves per SIMD: 97
 * VGPRs -> 104 allocated, whatever the kernel uses), and then no bitsliced
 * wave (160-176 registers) fits beside the 4 T-table waves, so the "split"
 * ran its halves one after the other (split wave-start trace,
 * profiles/r5/coresidency/).  Dynamic LDS leaves the descriptor at the
 * registers actually used (tests/test_isa_cpu.py checks the granule). */

template <bool DYN, uint32_t WORDS>
__device__ __forceinline__ uint32_t *tt_lds()
{
    if constexpr (DYN) {
        extern __shared__ __attribute__((aligned(16))) uint32_t tt_dyn_lds[];
        return tt_dyn_lds;
    } else {
        __shared__ __attribute__((aligned(16))) uint32_t tt_static_lds[WORDS];
        return tt_static_lds;
    }
}
/* what the lookups address: the static array, or dynamic LDS by integer */
template <bool DYN>
__device__ __forceinline__ auto tt_ref(const uint32_t *p)
{
    if constexpr (DYN)
        return DynTbl{};
    else
        return p;
}

/* CLAIM: the T-table half of a co-resident split (otc_device.h SplitClaim):
 * workgroup 0 first runs the blocks past the last full 2048-block unit, then
 * every wave takes units from the back of the buffer until none are left. */
template <int NR, int MODE, int B, int THREADS, bool CLAIM>
__device__ __forceinline__ void enc_tt_body(const EncParams &P, const otc_aes_key &K)
{
    uint32_t *tbl = tt_lds<CLAIM, 2 * 256 * 64>();
    fill_tbl4<THREADS>(tbl, g_tab.te0);
    __syncthreads();

    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = threadIdx.x >> 6;
    uint32_t lk[4];
    tbl4_lane_consts(lane, lk);
    constexpr uint64_t PER = (uint64_t)THREADS * B;

    /* B blocks per lane: i0 + 64 b, b < B; `full`: all below lim (wave-uniform) */
    auto chunk = [&](uint64_t i0, bool full, uint64_t lim) {
        uint32_t s[B][4];
        uint4 x[B];
#pragma unroll
        for (int b = 0; b < B; ++b) {
            const uint64_t i = i0 + 64u * b;
            const bool ok = full || i < lim;
            if (MODE == E_ECB) {
                uint4 v = ok ? lds16(P.in, i) : make_uint4(0, 0, 0, 0);
                s[b][0] = v.x; s[b][1] = v.y; s[b][2] = v.z; s[b][3] = v.w;
            } else if (MODE == E_CFB_DEC) { /* cipher input is the previous ciphertext */
                x[b] = ok ? lds16(P.in, i) : make_uint4(0, 0, 0, 0);
                uint4 v = (i == 0) ? make_uint4(P.iv[0], P.iv[1], P.iv[2], P.iv[3])
                                   : (ok ? lds16(P.in, i - 1) : make_uint4(0, 0, 0, 0));
                s[b][0] = v.x; s[b][1] = v.y; s[b][2] = v.z; s[b][3] = v.w;
            } else { /* CFB decrypt of independent segments: IV_s at segment starts */
                x[b] = ok ? lds16(P.in, i) : make_uint4(0, 0, 0, 0);
                const uint64_t sg = P.seg_shift < 64 ? (i >> P.seg_shift) : i / P.seg_blocks;
                if (i == sg * P.seg_blocks) {
                    ctr_words(P.ctr, sg, false, s[b][0], s[b][1], s[b][2], s[b][3]);
                } else {
                    uint4 v = ok ? lds16(P.in, i - 1) : make_uint4(0, 0, 0, 0);
                    s[b][0] = v.x; s[b][1] = v.y; s[b][2] = v.z; s[b][3] = v.w;
                }
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) s[b][j] ^= K.rk[j];
        }

        enc_rounds4_from<1, NR, B>(tt_ref<CLAIM>(tbl), lk, K, s);

#pragma unroll
        for (int b = 0; b < B; ++b) {
            const uint64_t i = i0 + 64u * b;
            uint4 o;
            if (MODE == E_ECB) {
                o = make_uint4(s[b][0], s[b][1], s[b][2], s[b][3]);
            } else {
                o = make_uint4(x[b].x ^ s[b][0], x[b].y ^ s[b][1], x[b].z ^ s[b][2], x[b].w ^ s[b][3]);
            }
            if (full || i < lim) sts16(P.out, i, o);
        }
    };

    if constexpr (CLAIM) {
        strace(1);
        /* the blocks past the last unit: workgroup 0, first */
        const uint64_t done = (uint64_t)P.cl.nunits * CLAIM_UNIT;
        if (blockIdx.x == 0) {
            for (uint64_t base = done; base < P.nfull; base += PER)
                chunk(base + (uint64_t)wave * 64u * B + lane, false, P.nfull);
        }
        const uint32_t wg = blockIdx.x * (THREADS / 64u) + __builtin_amdgcn_readfirstlane(wave);
        for (int64_t u = first_unit(P.cl, true, wg); u >= 0; u = claim_unit(P.cl, true)) {
            const uint64_t u0 = (uint64_t)u * CLAIM_UNIT;
#pragma unroll 1
            for (uint32_t it = 0; it < CLAIM_UNIT / (64u * B); ++it) chunk(u0 + it * 64u * B + lane, true, 0);
        }
        strace(5); /* trace builds: when the wave ran out of units (the claim tail) */
        return;
    }
    for (uint64_t base = (uint64_t)blockIdx.x * PER; base < P.nfull; base += (uint64_t)gridDim.x * PER)
        chunk(base + (uint64_t)wave * 64u * B + lane, base + PER <= P.nfull, P.nfull);
}

template <int NR, int MODE, int B, int THREADS>
__global__ __launch_bounds__(THREADS) void k_aes_enc_tt(EncParams P, otc_aes_key K)
{
    enc_tt_body<NR, MODE, B, THREADS, false>(P, K);
}

/* Claimed split: a bitsliced wave per SIMD (156-168 registers) must fit
 * beside the workgroup's 4 T-table waves in the 512-register file, which
 * leaves each T-table wave 80-88.  hipcc will not cap a kernel whose LDS
 * already limits it to 4 waves per SIMD (amdgpu_num_vgpr is ignored,
 * waves_per_eu "fails to meet" the target), so the blocks per lane are the
 * lever: ECB encryption at B = 4 takes 82 (88 allocated + 160 = 512); the
 * chained CFB decryption needs B = 2 (61; at 4: 101). */
#ifndef OTC_TT_CLAIM_B
#define OTC_TT_CLAIM_B 2
#endif
#ifndef OTC_TT_ECB_CLAIM_B
#define OTC_TT_ECB_CLAIM_B OTC_TT_ENC_B
#endif
template <int NR>
__global__ __launch_bounds__(1024) OTC_CLAIM_ATTR void k_aes_ecb_tt_claim(EncParams P, otc_aes_key K)
{
    enc_tt_body<NR, E_ECB, OTC_TT_ECB_CLAIM_B, 1024, true>(P, K);
}
template <int NR>
__global__ __launch_bounds__(1024) OTC_CLAIM_ATTR void k_aes_cfb_tt_claim(EncParams P, otc_aes_key K)
{
    enc_tt_body<NR, E_CFB_DEC, OTC_TT_CLAIM_B, 1024, true>(P, K);
}
template <int NR>
__global__ __launch_bounds__(1024) OTC_CLAIM_ATTR void k_aes_cfbseg_tt_claim(EncParams P, otc_aes_key K)
{
    enc_tt_body<NR, E_CFB_DEC_SEG, OTC_TT_CLAIM_B, 1024, true>(P, K);
}

/* ---------------------------------------------------------------------------
 * CTR with counter-mode caching.
 *
 * Chunks are aligned to the counter (virtual index v = i + shift, shift =
 * ctr0 mod PER; the first chunk starts `shift` blocks early with those blocks
 * masked), so within one wave-iteration the counter of block (b, lane) is
 * C + 64b + lane with no carry out of the low byte: bytes 0..14 of the counter
 * block are WAVE-UNIFORM.  Hence in round 1 only the T3 lookup of byte 15
 * differs between lanes, and in round 2 only the four lookups fed by column 0.
 * The 15 + 12 uniform lookups are done once per wave-iteration on the scalar
 * unit (s_load from the constant table); LDS reads per AES-128 block drop from
 * 160 to 133.
 * ------------------------------------------------------------------------- */
struct CtrParams {
    const uint8_t *in;
    uint8_t *out;
    uint64_t nfull;   /* full blocks */
    uint32_t tail;    /* trailing partial block bytes */
    uint32_t wrap64;
    uint64_t shift;   /* ctr0.lo mod PER */
    Ctr128 cbase;     /* ctr0 - shift (low log2(PER) bits zero) */
    SplitClaim cl;    /* k_aes_ctr_tt_persist: 2048-block units of the virtual range */
};

__device__ __forceinline__ uint32_t te_u(uint32_t idx) { return g_tab.te0[idx & 0xFFu]; } /* uniform lookup */

/* one wave-iteration: the 64 x B blocks from virtual block vw (uniform,
 * a multiple of 64 x B) */
template <int NR, int B>
__device__ __forceinline__ void ctr_cached_iter(const CtrParams &P, const otc_aes_key &K, const uint32_t *tbl,
                                                const uint32_t (&lk)[4], uint32_t lane, uint64_t vw)
{
    /* uniform counter C = cbase + vw */
    uint64_t clo = P.cbase.lo + vw;
    uint64_t chi = P.cbase.hi + ((!P.wrap64 && clo < P.cbase.lo) ? 1u : 0u);
    const uint32_t w0 = bswap32((uint32_t)(chi >> 32)) ^ K.rk[0];
    const uint32_t w1 = bswap32((uint32_t)chi) ^ K.rk[1];
    const uint32_t w2 = bswap32((uint32_t)(clo >> 32)) ^ K.rk[2];
    const uint32_t w3u = bswap32((uint32_t)clo) ^ K.rk[3]; /* byte 15 (top byte) patched per block */
    /* round 1, uniform parts */
    const uint32_t U0 = te_u(w0) ^ rotl8(te_u(w1 >> 8)) ^ rotl16(te_u(w2 >> 16)) ^ K.rk[4];
    const uint32_t t1 = te_u(w1) ^ rotl8(te_u(w2 >> 8)) ^ rotl16(te_u(w3u >> 16)) ^ rotl24(te_u(w0 >> 24)) ^ K.rk[5];
    const uint32_t t2 = te_u(w2) ^ rotl8(te_u(w3u >> 8)) ^ rotl16(te_u(w0 >> 16)) ^ rotl24(te_u(w1 >> 24)) ^ K.rk[6];
    const uint32_t t3 = te_u(w3u) ^ rotl8(te_u(w0 >> 8)) ^ rotl16(te_u(w1 >> 16)) ^ rotl24(te_u(w2 >> 24)) ^ K.rk[7];
    /* round 2, uniform parts */
    const uint32_t V0 = rotl8(te_u(t1 >> 8)) ^ rotl16(te_u(t2 >> 16)) ^ rotl24(te_u(t3 >> 24)) ^ K.rk[8];
    const uint32_t V1 = te_u(t1) ^ rotl8(te_u(t2 >> 8)) ^ rotl16(te_u(t3 >> 16)) ^ K.rk[9];
    const uint32_t V2 = te_u(t2) ^ rotl8(te_u(t3 >> 8)) ^ rotl24(te_u(t1 >> 24)) ^ K.rk[10];
    const uint32_t V3 = te_u(t3) ^ rotl16(te_u(t1 >> 16)) ^ rotl24(te_u(t2 >> 24)) ^ K.rk[11];
    const uint32_t b15 = (uint32_t)(clo & 0xFFu); /* low byte of C (low 6+log2(B) bits are 0) */

    const int64_t i0 = (int64_t)vw - (int64_t)P.shift + lane; /* real block index of (b=0, lane) */
    const bool full = vw >= P.shift && vw - P.shift + 64u * B <= P.nfull; /* uniform */
    uint32_t s[B][4];
    uint4 x[B];
#pragma unroll
    for (int b = 0; b < B; ++b) {
        const int64_t i = i0 + 64 * b;
        const bool ok = full || (i >= 0 && (uint64_t)i < P.nfull);
        x[b] = ok ? lds16(P.in, (uint64_t)i) : make_uint4(0, 0, 0, 0);
        /* round 1: only T3[byte 15] varies */
        const uint32_t c15 = (b15 | (uint32_t)(64 * b) | lane) ^ (K.rk[3] >> 24);
        const uint32_t s0 = U0 ^ lds_at(tbl, (c15 << 8) | lk[3]);
        /* round 2: the four lookups fed by s0 */
        s[b][0] = V0 ^ lds_at(tbl, tt_addr(s0, lk[0], 0));
        s[b][1] = V1 ^ lds_at(tbl, tt_addr(s0, lk[3], 3));
        s[b][2] = V2 ^ lds_at(tbl, tt_addr(s0, lk[2], 2));
        s[b][3] = V3 ^ lds_at(tbl, tt_addr(s0, lk[1], 1));
    }
    /* rounds 3..NR */
    enc_rounds4_from<3, NR, B>(tbl, lk, K, s);

#pragma unroll
    for (int b = 0; b < B; ++b) {
        const int64_t i = i0 + 64 * b;
        const bool ok = full || (i >= 0 && (uint64_t)i < P.nfull);
        if (ok) {
            sts16(P.out, (uint64_t)i,
                 make_uint4(x[b].x ^ s[b][0], x[b].y ^ s[b][1], x[b].z ^ s[b][2], x[b].w ^ s[b][3]));
        } else if (i >= 0 && (uint64_t)i == P.nfull && P.tail) {
            const uint32_t ks[4] = {s[b][0], s[b][1], s[b][2], s[b][3]};
            for (uint32_t n = 0; n < P.tail; ++n)
                P.out[16 * (uint64_t)i + n] = P.in[16 * (uint64_t)i + n] ^ (uint8_t)(ks[n >> 2] >> (8 * (n & 3)));
        }
    }
}

template <int NR, int B, int THREADS>
__global__ __launch_bounds__(THREADS) void k_aes_ctr_tt_cached(CtrParams P, otc_aes_key K)
{
    __shared__ __attribute__((aligned(16))) uint32_t tbl[2 * 256 * 64];
    fill_tbl4<THREADS>(tbl, g_tab.te0);
    __syncthreads();

    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint32_t lk[4];
    tbl4_lane_consts(lane, lk);
    constexpr uint64_t PER = (uint64_t)THREADS * B;
    const uint64_t vtotal = P.nfull + (P.tail ? 1u : 0u) + P.shift;
    for (uint64_t vbase = (uint64_t)blockIdx.x * PER; vbase < vtotal; vbase += (uint64_t)gridDim.x * PER)
        ctr_cached_iter<NR, B>(P, K, tbl, lk, lane, vbase + (uint64_t)wave * 64u * B);
}

/* The same cipher as a persistent claim kernel (one 1024-thread workgroup
 * per CU, engine.cpp routes CTR calls from tt_persistent_min() to the T-table
 * here): every wave takes 2048-block units of the virtual range -- its first
 * one handed out (otc_device.h first_unit), the rest claimed from the back --
 * so a call ends when the work does, not when the CU with the most static
 * chunks does.  Blocks outside [0, nfull] are masked per iteration, as in
 * the grid kernel.  It never runs beside the bitsliced kernel, so it keeps
 * the grid kernel's static table (not a "_claim" kernel of the splits). */
template <int NR>
__global__ __launch_bounds__(1024) void k_aes_ctr_tt_persist(CtrParams P, otc_aes_key K)
{
    constexpr int B = OTC_TT_CTR_B;
    __shared__ __attribute__((aligned(16))) uint32_t tbl[2 * 256 * 64];
    fill_tbl4<1024>(tbl, g_tab.te0);
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint32_t lk[4];
    tbl4_lane_consts(lane, lk);
    for (int64_t u = first_unit(P.cl, true, blockIdx.x * 16u + wave); u >= 0; u = claim_unit(P.cl, true)) {
#pragma unroll 1
        for (uint32_t it = 0; it < CLAIM_UNIT / (64u * B); ++it)
            ctr_cached_iter<NR, B>(P, K, tbl, lk, lane, (uint64_t)u * CLAIM_UNIT + it * 64u * B);
    }
}

/* ---------------------------------------------------------------------------
 * Decryption-direction kernel: ECB-dec, CBC-dec (single stream or power-of-2
 * segments with per-segment IVs)
 * ------------------------------------------------------------------------- */
template <int NR, int MODE, int B, int THREADS, bool CLAIM>
__device__ __forceinline__ void dec_tt_body(const DecParams &P, const otc_aes_key &K)
{
    uint32_t *tbl = tt_lds<CLAIM, 2 * 256 * 64 + 256 * 32>(); /* 160 KiB */
    fill_dtbl4<THREADS>(tbl, g_tab.td0, g_tab.is4);
    __syncthreads();

    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = threadIdx.x >> 6;
    uint32_t lk[4];
    tbl4_lane_consts(lane, lk);
    const uint32_t lk_is2 = 0x40000u | ((lane & 31u) << 3);
    constexpr uint64_t PER = (uint64_t)THREADS * B;

    auto chunk = [&](uint64_t i0, bool full) {
        uint32_t s[B][4];
        uint4 prev[B];
#pragma unroll
        for (int b = 0; b < B; ++b) {
            const uint64_t i = i0 + 64u * b;
            const bool ok = full || i < P.nfull;
            uint4 v = ok ? lds16(P.in, i) : make_uint4(0, 0, 0, 0);
            s[b][0] = v.x ^ K.rk[0]; s[b][1] = v.y ^ K.rk[1];
            s[b][2] = v.z ^ K.rk[2]; s[b][3] = v.w ^ K.rk[3];
            if (MODE == D_CBC || MODE == D_CBC_SEG) {
                bool first;
                Ctr128 ivv = P.iv;
                if (MODE == D_CBC) {
                    first = (i == 0);
                } else {
                    first = (i & ((1ull << P.seg_shift) - 1)) == 0;
                    const uint64_t seg = i >> P.seg_shift;
                    ivv.lo = P.iv.lo + seg;
                    ivv.hi = P.iv.hi + (ivv.lo < P.iv.lo ? 1 : 0);
                }
                if (first) {
                    uint32_t w0, w1, w2, w3;
                    ctr_words(ivv, 0, false, w0, w1, w2, w3);
                    prev[b] = make_uint4(w0, w1, w2, w3);
                } else {
                    prev[b] = ok ? lds16(P.in, i - 1) : make_uint4(0, 0, 0, 0);
                }
            }
        }

        dec_rounds4<NR, B>(tt_ref<CLAIM>(tbl), lk, lk_is2, K, s);

#pragma unroll
        for (int b = 0; b < B; ++b) {
            const uint64_t i = i0 + 64u * b;
            uint4 o = make_uint4(s[b][0], s[b][1], s[b][2], s[b][3]);
            if (MODE != D_ECB) {
                o.x ^= prev[b].x; o.y ^= prev[b].y; o.z ^= prev[b].z; o.w ^= prev[b].w;
            }
            if (full || i < P.nfull) sts16(P.out, i, o);
        }
    };

    if constexpr (CLAIM) { /* as k_aes_enc_tt */
        strace(1);
        const uint64_t done = (uint64_t)P.cl.nunits * CLAIM_UNIT;
        if (blockIdx.x == 0)
            for (uint64_t base = done; base < P.nfull; base += PER) chunk(base + (uint64_t)wave * 64u * B + lane, false);
        const uint32_t wg = blockIdx.x * (THREADS / 64u) + __builtin_amdgcn_readfirstlane(wave);
        for (int64_t u = first_unit(P.cl, true, wg); u >= 0; u = claim_unit(P.cl, true)) {
#pragma unroll 1
            for (uint32_t it = 0; it < CLAIM_UNIT / (64u * B); ++it) chunk((uint64_t)u * CLAIM_UNIT + it * 64u * B + lane, true);
        }
        strace(5);
        return;
    }
    for (uint64_t base = (uint64_t)blockIdx.x * PER; base < P.nfull; base += (uint64_t)gridDim.x * PER)
        chunk(base + (uint64_t)wave * 64u * B + lane, base + PER <= P.nfull);
}

template <int NR, int MODE, int B, int THREADS>
__global__ __launch_bounds__(THREADS) void k_aes_dec_tt(DecParams P, otc_aes_key K)
{
    dec_tt_body<NR, MODE, B, THREADS, false>(P, K);
}

/* Claimed split: the bitsliced inverse-cipher kernels take 168 registers,
 * leaving 80 per T-table wave: B = 2 (ECB 51, CBC 66; at 4: 83 / 106) */
template <int NR, int MODE>
__global__ __launch_bounds__(1024) OTC_CLAIM_ATTR void k_aes_dec_tt_claim(DecParams P, otc_aes_key K)
{
    dec_tt_body<NR, MODE, OTC_TT_CLAIM_B, 1024, true>(P, K);
}

/* ---------------------------------------------------------------------------
 * CBC / CFB128 encryption over independent contiguous segments: one segment
 * per lane slot, B segments per lane for ILP.  IV_s = iv0 + s.  Next
 * plaintext block is prefetched one step ahead.  Both modes are serial chains
 * (reference aes-modes/aes.c:801-812 CBC, :822-862 CFB); per block
 *   CBC:  c = E(p ^ c)          out = c
 *   CFB:  c = p ^ E(c)          out = c
 * so one kernel body serves both (template flag CFB).
 * ------------------------------------------------------------------------- */
struct CbcSegParams {
    const uint8_t *in;
    uint8_t *out;
    uint64_t seg_blocks;
    uint64_t nseg;
    Ctr128 iv0;
    SplitClaim cl; /* k_aes_seg_enc_tt_claim: 64-segment units from the back */
};

/* chain step on B lanes: s = cipher input ^ rk0 from the chain value c and
 * the plaintext p; after the rounds, chain_out gives the new c (= output) */
template <bool CFB>
__device__ __forceinline__ void chain_in(const uint4 &p, const uint32_t (&c)[4], const otc_aes_key &K, uint32_t (&s)[4])
{
    if (CFB) {
        s[0] = c[0] ^ K.rk[0]; s[1] = c[1] ^ K.rk[1]; s[2] = c[2] ^ K.rk[2]; s[3] = c[3] ^ K.rk[3];
    } else {
        s[0] = p.x ^ c[0] ^ K.rk[0]; s[1] = p.y ^ c[1] ^ K.rk[1]; s[2] = p.z ^ c[2] ^ K.rk[2];
        s[3] = p.w ^ c[3] ^ K.rk[3];
    }
}
template <bool CFB>
__device__ __forceinline__ void chain_out(const uint4 &p, const uint32_t (&s)[4], uint32_t (&c)[4])
{
    if (CFB) {
        c[0] = s[0] ^ p.x; c[1] = s[1] ^ p.y; c[2] = s[2] ^ p.z; c[3] = s[3] ^ p.w;
    } else {
        c[0] = s[0]; c[1] = s[1]; c[2] = s[2]; c[3] = s[3];
    }
}

template <int NR, int B, int THREADS, bool CFB = false>
__global__ __launch_bounds__(THREADS) void k_aes_cbc_enc_seg(CbcSegParams P, otc_aes_key K)
{
    __shared__ __attribute__((aligned(16))) uint32_t tbl[2 * 256 * 64];
    fill_tbl4<THREADS>(tbl, g_tab.te0);
    __syncthreads();

    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = threadIdx.x >> 6;
    uint32_t lk[4];
    tbl4_lane_consts(lane, lk);
    constexpr uint64_t PER = (uint64_t)THREADS * B;

    for (uint64_t base = (uint64_t)blockIdx.x * PER; base < P.nseg; base += (uint64_t)gridDim.x * PER) {
        uint64_t seg[B];
        bool live[B];
        uint32_t c[B][4];
        uint4 nxt[B];
#pragma unroll
        for (int b = 0; b < B; ++b) {
            seg[b] = base + (uint64_t)wave * 64u * B + 64u * b + lane;
            live[b] = seg[b] < P.nseg;
            Ctr128 ivv;
            ivv.lo = P.iv0.lo + seg[b];
            ivv.hi = P.iv0.hi + (ivv.lo < P.iv0.lo ? 1 : 0);
            ctr_words(ivv, 0, false, c[b][0], c[b][1], c[b][2], c[b][3]);
            nxt[b] = (live[b] && P.seg_blocks) ? ld16(P.in, seg[b] * P.seg_blocks) : make_uint4(0, 0, 0, 0);
        }
        for (uint64_t j = 0; j < P.seg_blocks; ++j) {
            uint32_t s[B][4];
            uint4 p[B];
#pragma unroll
            for (int b = 0; b < B; ++b) {
                p[b] = nxt[b];
                chain_in<CFB>(p[b], c[b], K, s[b]);
                nxt[b] = (live[b] && j + 1 < P.seg_blocks) ? ld16(P.in, seg[b] * P.seg_blocks + j + 1)
                                                           : make_uint4(0, 0, 0, 0);
            }
            enc_rounds4_from<1, NR, B>(tbl, lk, K, s);
#pragma unroll
            for (int b = 0; b < B; ++b) {
                chain_out<CFB>(p[b], s[b], c[b]);
                if (live[b]) st16(P.out, seg[b] * P.seg_blocks + j, make_uint4(c[b][0], c[b][1], c[b][2], c[b][3]));
            }
        }
    }
}

/* Same job, grouped memory access: each lane loads and stores the next G
 * blocks of its segment back to back (one burst per cache line) instead of
 * one block per block-time.  Lanes are a segment apart (4 KiB for disk
 * sectors), so every wave access touches 64 lines; spread over G block-times,
 * the ~2048 live segments per CU evict those lines from L2 between uses and
 * each 16-byte block re-fetches a whole line.  Group g+1 is prefetched while
 * group g is encrypted; ciphertext overwrites the plaintext registers and is
 * stored as a burst at the end of the group.  One segment per lane (two, with
 * 4- or 8-block bursts, measured 1-27% slower: profiles/r4/seg_ab/). */
template <int NR, int G, bool CFB, bool DB = true, class TBL = const uint32_t *>
__device__ __forceinline__ void seg_chain_g(const CbcSegParams &P, const otc_aes_key &K, TBL tbl,
                                            const uint32_t (&lk)[4], uint64_t seg, bool live)
{
    const uint64_t sb = P.seg_blocks;
    const uint64_t ng = sb / G;
    const uint64_t first = seg * sb; /* block index of the segment's first block */
    uint32_t c[4];
    uint4 cur[G], nxt[DB ? G : 1];
    Ctr128 ivv;
    ivv.lo = P.iv0.lo + seg;
    ivv.hi = P.iv0.hi + (ivv.lo < P.iv0.lo ? 1 : 0);
    ctr_words(ivv, 0, false, c[0], c[1], c[2], c[3]);
#pragma unroll
    for (int t = 0; t < G; ++t) cur[t] = (live && ng) ? ld16(P.in, first + t) : make_uint4(0, 0, 0, 0);
    for (uint64_t g = 0; g < ng; ++g) {
        const bool more = g + 1 < ng;
        if constexpr (DB) {
#pragma unroll
            for (int t = 0; t < G; ++t)
                nxt[t] = (live && more) ? ld16(P.in, first + (g + 1) * G + t) : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int t = 0; t < G; ++t) {
            uint32_t s[1][4];
            chain_in<CFB>(cur[t], c, K, s[0]);
            enc_rounds4_from<1, NR, 1>(tbl, lk, K, s);
            chain_out<CFB>(cur[t], s[0], c);
            cur[t] = make_uint4(c[0], c[1], c[2], c[3]);
        }
#pragma unroll
        for (int t = 0; t < G; ++t) {
            if (live) st16(P.out, first + g * G + t, cur[t]);
            if constexpr (DB) cur[t] = nxt[t];
        }
        if constexpr (!DB) {
            /* single buffer: the next group is loaded behind this group's
             * stores; the other waves of the SIMD cover its latency */
#pragma unroll
            for (int t = 0; t < G; ++t)
                cur[t] = (live && more) ? ld16(P.in, first + (g + 1) * G + t) : make_uint4(0, 0, 0, 0);
        }
    }
    /* remaining sb % G blocks, one at a time */
    for (uint64_t j = ng * G; j < sb; ++j) {
        uint32_t s[1][4];
        const uint4 p = live ? ld16(P.in, first + j) : make_uint4(0, 0, 0, 0);
        chain_in<CFB>(p, c, K, s[0]);
        enc_rounds4_from<1, NR, 1>(tbl, lk, K, s);
        chain_out<CFB>(p, s[0], c);
        if (live) st16(P.out, first + j, make_uint4(c[0], c[1], c[2], c[3]));
    }
}

/* One chain per thread; the workgroup size is chosen at launch (a multiple
 * of 64 up to THREADS): with fewer chains than CUs x THREADS the launch
 * shrinks the workgroups so that every CU gets chains, instead of filling
 * nseg / THREADS CUs and leaving the rest idle (launch_seg_nr). */
template <int NR, int THREADS, int G, bool CFB = false>
__global__ __launch_bounds__(THREADS) void k_aes_cbc_enc_seg_g(CbcSegParams P, otc_aes_key K)
{
    __shared__ __attribute__((aligned(16))) uint32_t tbl[2 * 256 * 64];
    const uint32_t nt = blockDim.x;
    if (nt == THREADS) {
        fill_tbl4<THREADS>(tbl, g_tab.te0);
    } else {
        uint4 *l4 = reinterpret_cast<uint4 *>(tbl);
        for (uint32_t q = threadIdx.x; q < 8192; q += nt) {
            const uint32_t r = q >> 12, x = (q >> 4) & 255, half = (q >> 3) & 1, k = 2 * r + half;
            const uint32_t t = g_tab.te0[x];
            const uint32_t v = k ? ((t << (8 * k)) | (t >> (32 - 8 * k))) : t;
            l4[q] = make_uint4(v, v, v, v);
        }
    }
    __syncthreads();
    uint32_t lk[4];
    tbl4_lane_consts(threadIdx.x & 63u, lk);
    for (uint64_t base = (uint64_t)blockIdx.x * nt; base < P.nseg; base += (uint64_t)gridDim.x * nt) {
        const uint64_t seg = base + threadIdx.x;
        seg_chain_g<NR, G, CFB>(P, K, tbl, lk, seg, seg < P.nseg);
    }
}

/* The T-table half of the chained segment encryption split (engine.cpp
 * seg_enc_run): a claim unit is 64 segments, one per lane of a wave, taken
 * from the back; workgroup 0 first runs the segments past the last full unit.
 * It runs alone (engine.cpp seg_enc_run): no VALU half claims from the front. */
constexpr uint32_t SEG_UNIT = 64;
template <int NR, int G, bool CFB>
__global__ __launch_bounds__(1024) OTC_CLAIM_ATTR void k_aes_seg_enc_tt_claim(CbcSegParams P, otc_aes_key K)
{
    uint32_t *tbl = tt_lds<true, 2 * 256 * 64>();
    fill_tbl4<1024>(tbl, g_tab.te0);
    __syncthreads();
    uint32_t lk[4];
    tbl4_lane_consts(threadIdx.x & 63u, lk);
    strace(1);
    const uint64_t done = (uint64_t)P.cl.nunits * SEG_UNIT;
    if (blockIdx.x == 0 && done + (threadIdx.x & ~63u) < P.nseg) { /* the remainder (< 64 segments): wave 0 */
        const uint64_t seg = done + threadIdx.x;
        seg_chain_g<NR, G, CFB, false>(P, K, DynTbl{}, lk, seg, seg < P.nseg);
    }
    const uint32_t wg = blockIdx.x * 16u + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (int64_t u = first_unit(P.cl, true, wg); u >= 0; u = claim_unit(P.cl, true))
        seg_chain_g<NR, G, CFB, false>(P, K, DynTbl{}, lk, (uint64_t)u * SEG_UNIT + lane_id(), true);
}

/* CBC-decrypt over segments of ANY length: the plain CBC kernel XORs every
 * block with its predecessor; this fix-up swaps that predecessor for IV_s at
 * each segment start s >= 1 (touches nseg blocks only). */
__global__ __launch_bounds__(256) void k_cbc_seg_fixup(const uint8_t *in, uint8_t *out, uint64_t seg_blocks,
                                                       uint64_t nseg, Ctr128 iv0)
{
    const uint64_t s = 1 + (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (s >= nseg) return;
    const uint64_t i = s * seg_blocks;
    Ctr128 ivv;
    ivv.lo = iv0.lo + s;
    ivv.hi = iv0.hi + (ivv.lo < iv0.lo ? 1 : 0);
    uint32_t w0, w1, w2, w3;
    ctr_words(ivv, 0, false, w0, w1, w2, w3);
    const uint4 prev = ld16(in, i - 1);
    uint4 o = ld16(out, i);
    o.x ^= prev.x ^ w0; o.y ^= prev.y ^ w1; o.z ^= prev.z ^ w2; o.w ^= prev.w ^ w3;
    st16(out, i, o);
}

/* ---------------------------------------------------------------------------
 * CTR over a body whose data pointer is NOT 16-byte aligned (the resumable
 * stream API after a partial block: nc_off != 0 leaves the next call's data at
 * body = in + head).  Keystream block b still covers data bytes
 * [16b, 16b + 16); the memory is processed in ALIGNED 16-byte chunks J, and
 * with a = body & 15 chunk J holds data bytes [16J - a, 16J - a + 16), i.e.
 * the last a bytes of keystream block J-1 and the first 16 - a of block J.
 * Lane l of a wave encrypts block J0 + l - 1, takes block J0 + l - 2 from lane
 * l - 1 (one cross-lane shuffle per word) and funnel-shifts the two
 * (v_alignbyte) into the chunk's keystream: 63 chunks per wave, dwordx4 loads
 * and stores, byte accesses only for the two edge chunks.  In and out must
 * share the misalignment (in place always does).
 * ------------------------------------------------------------------------- */
struct CtrShiftParams {
    const uint8_t *in; /* aligned base: body - a */
    uint8_t *out;
    uint64_t len;      /* body bytes */
    uint32_t a;        /* misalignment 1..15 */
    uint32_t pad;
    Ctr128 ctr;        /* counter of the body's keystream block 0 */
};

template <int NR, int THREADS>
__global__ __launch_bounds__(THREADS) void k_aes_ctr_shift(CtrShiftParams P, otc_aes_key K)
{
    __shared__ __attribute__((aligned(16))) uint32_t tbl[2 * 256 * 64];
    fill_tbl4<THREADS>(tbl, g_tab.te0);
    __syncthreads();

    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = threadIdx.x >> 6;
    uint32_t lk[4];
    tbl4_lane_consts(lane, lk);
    constexpr uint64_t WPB = THREADS / 64;
    const uint64_t nchunks = (P.a + P.len + 15) / 16;
    const uint32_t d = 16u - P.a, dq = d >> 2, db = d & 3u;

    for (uint64_t w = (uint64_t)blockIdx.x * WPB + wave; w * 63u < nchunks; w += (uint64_t)gridDim.x * WPB) {
        const uint64_t J0 = w * 63u;
        /* block J0 - 1 for lane 0 (wraps to the counter's predecessor for the
         * very first wave: computed, never used) */
        uint32_t s[1][4];
        ctr_words(P.ctr, J0 + lane - 1u, false, s[0][0], s[0][1], s[0][2], s[0][3]);
#pragma unroll
        for (int j = 0; j < 4; ++j) s[0][j] ^= K.rk[j];
        enc_rounds4_from<1, NR, 1>(tbl, lk, K, s);
        uint32_t cat[8];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            cat[j] = (uint32_t)__shfl_up((int)s[0][j], 1);
            cat[4 + j] = s[0][j];
        }
        const uint64_t J = J0 + lane - 1u;
        if (lane == 0 || J >= nchunks) continue;
        /* chunk byte t = concatenated keystream byte d + t */
        uint32_t ks[4];
#define OTC_KS_SHIFT(Q)                                                                  \
    for (int k = 0; k < 4; ++k) ks[k] = __builtin_amdgcn_alignbyte(cat[(Q) + k + 1], cat[(Q) + k], db);
        switch (dq) {
        case 0: OTC_KS_SHIFT(0) break;
        case 1: OTC_KS_SHIFT(1) break;
        case 2: OTC_KS_SHIFT(2) break;
        default: OTC_KS_SHIFT(3) break;
        }
#undef OTC_KS_SHIFT
        const int64_t lo = (int64_t)(16u * J) - (int64_t)P.a; /* data index of the chunk's byte 0 */
        if (J >= 1 && lo + 16 <= (int64_t)P.len) {
            const uint4 x = ld16(P.in, J);
            st16(P.out, J, make_uint4(x.x ^ ks[0], x.y ^ ks[1], x.z ^ ks[2], x.w ^ ks[3]));
        } else { /* edge chunk: only the bytes inside the body */
            for (int t = 0; t < 16; ++t) {
                const int64_t i = lo + t;
                if (i >= 0 && i < (int64_t)P.len)
                    P.out[16u * J + t] = P.in[16u * J + t] ^ (uint8_t)(ks[t >> 2] >> (8 * (t & 3)));
            }
        }
    }
}

/* Tiny XOR with up to 16 keystream bytes passed by value (head of a resumed
 * CTR stream: the bytes of the context's stream_block) */
struct SmallXor {
    uint8_t ks[16];
};
__global__ __launch_bounds__(64) void k_xor_small(const uint8_t *in, uint8_t *out, uint32_t n, SmallXor k)
{
    const uint32_t t = threadIdx.x;
    if (t < n) out[t] = in[t] ^ k.ks[t];
}

/* ---------------------------------------------------------------------------
 * Batched CTR (otc_aes_ctr_batch): many independent messages, each with its
 * own buffers, key and counter, in ONE launch.  Work unit: a wave tile of
 * 64 x B blocks of one message; tile t belongs to message tile_msg[t] at local
 * tile t - tile_first[m] (host planner).  The descriptor and the message's
 * round keys are wave-uniform: loaded once per tile and moved to SGPRs with
 * readfirstlane, so the rounds are the same code as the single-message kernel
 * (round keys as SGPR operands of the v_bitop3s).  The LDS 4-table image is
 * key independent, so one persistent workgroup per CU serves every message.
 * No counter caching here: tiles start at arbitrary counters.
 * ------------------------------------------------------------------------- */
struct BatchParams {
    const otc_ctr_msg *msgs;
    const otc_aes_key *keys;
    const uint32_t *tile_msg;
    const uint64_t *tile_first;
    uint64_t ntiles;
    SplitClaim cl; /* ctr != nullptr: BATCH_UNIT-tile units, first handed out, the rest claimed */
};
constexpr uint64_t BATCH_UNIT = 8; /* tiles per claimed unit (8 x 4 KiB at B = 4) */

__device__ __forceinline__ uint32_t ufl(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

/* load through the constant address space (wave-uniform address -> s_load) */
typedef const __attribute__((address_space(4))) uint32_t *cptr32;
typedef const __attribute__((address_space(4))) uint64_t *cptr64;
__device__ __forceinline__ uint32_t cld32(const uint32_t *p) { return *(cptr32)p; }
__device__ __forceinline__ uint64_t cld64(const uint64_t *p) { return *(cptr64)p; }
/* message buffers come from descriptors as plain addresses: access them as
 * GLOBAL memory, or hipcc emits flat_* ops, which count against lgkmcnt and
 * make every LDS wait also wait for HBM */
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) u32x4 g_u32x4;
typedef __attribute__((address_space(1))) uint8_t g_u8;
/* OTC_BATCH_NT (default 1): the non-temporal bit on the message loads /
 * stores -- each tile is read and written once, lane-linear.  Round 6 A/B,
 * 3 reps (profiles/r6/batch_nt/): 1024 x 1 MiB packed 1484-1492 vs 1446-1460
 * GB/s, 16384 x 4 KiB packed 1156-1164 vs 1136-1144, 262144 x 4 KiB
 * 1191-1212 vs 1173-1192, 65536 x 1504 B even. */
#ifndef OTC_BATCH_NT
#define OTC_BATCH_NT 1
#endif
__device__ __forceinline__ uint4 gld16(const uint8_t *p, uint64_t blk)
{
    const g_u32x4 *q = (const g_u32x4 *)(p + 16 * blk);
    const u32x4 v = OTC_BATCH_NT ? __builtin_nontemporal_load(q) : *q;
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void gst16(uint8_t *p, uint64_t blk, uint4 v)
{
    g_u32x4 *q = (g_u32x4 *)(p + 16 * blk);
    const u32x4 w = {v.x, v.y, v.z, v.w};
    if (OTC_BATCH_NT) __builtin_nontemporal_store(w, q);
    else *q = w;
}

template <int NR, int B, int THREADS>
__global__ __launch_bounds__(THREADS) void k_aes_ctr_batch_tt(BatchParams P)
{
    __shared__ __attribute__((aligned(16))) uint32_t tbl[2 * 256 * 64];
    fill_tbl4<THREADS>(tbl, g_tab.te0);
    __syncthreads();

    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = ufl(threadIdx.x >> 6);
    uint32_t lk[4];
    tbl4_lane_consts(lane, lk);
    constexpr uint32_t WAVES = THREADS / 64;
    constexpr uint64_t TILE = 64u * B;

    /* each wave walks a CONTIGUOUS run of tiles: consecutive tiles share
     * tile-map / descriptor cache lines (and usually the message), so the
     * dependent scalar loads at a tile start hit the scalar cache */
    const uint64_t nw = (uint64_t)gridDim.x * WAVES, wid = (uint64_t)blockIdx.x * WAVES + wave;
    /* large batches (P.cl.ctr set, engine.cpp): runs of BATCH_UNIT tiles,
     * the first handed out, the rest claimed, so the batch ends when the
     * work does -- a static split left CUs idle behind the slowest share, as
     * the T-table CTR grid did (docs/PERF.md round 6) */
    const bool claimed = P.cl.ctr != nullptr;
    uint64_t t = wid * P.ntiles / nw, t_end = (wid + 1) * P.ntiles / nw;
    if (claimed) {
        const int64_t u = first_unit(P.cl, true, (uint32_t)wid);
        t = u < 0 ? 0 : (uint64_t)u * BATCH_UNIT;
        t_end = u < 0 ? 0 : min((uint64_t)(u + 1) * BATCH_UNIT, P.ntiles);
    }
    for (;; ++t) {
        if (t >= t_end) {
            if (!claimed) break;
            const int64_t u = claim_unit(P.cl, true);
            if (u < 0) break;
            t = (uint64_t)u * BATCH_UNIT;
            t_end = min((uint64_t)(u + 1) * BATCH_UNIT, P.ntiles);
        }
        /* descriptor, tile base and round keys through the constant address
         * space: wave-uniform addresses -> scalar loads (s_load_dwordx*) into
         * SGPRs, no VGPRs and no per-lane memory traffic */
        const uint32_t m = cld32(P.tile_msg + t);
        const uint64_t *D = (const uint64_t *)(P.msgs + m);
        const uint8_t *in = (const uint8_t *)cld64(D + 0);
        uint8_t *out = (uint8_t *)cld64(D + 1);
        const uint64_t nbytes = cld64(D + 2);
        const Ctr128 c = {cld64(D + 3), cld64(D + 4)};
        const uint64_t kw = cld64(D + 5); /* key index | align word << 32 */
        const uint32_t *Kg = P.keys[0].rk + (sizeof(otc_aes_key) / 4) * (uint32_t)kw;
        const uint32_t align = (uint32_t)(kw >> 32);
        otc_aes_key K;
#pragma unroll
        for (int q = 0; q < 4 * (NR + 1); ++q) K.rk[q] = cld32(Kg + q);
        const uint64_t nfull = nbytes >> 4;
        const uint32_t tail = (uint32_t)(nbytes & 15u);
        const uint64_t vb = (t - cld64(P.tile_first + m)) * TILE; /* tile base (virtual block) */

        uint32_t s[B][4];
        uint4 x[B];
        int64_t i0;
        if (align & OTC_BATCH_ALIGNED) {
            /* counter-aligned tiles (large messages): virtual block v = real
             * block + shift with shift = ctr0.lo mod TILE, so within a tile the
             * counters are C + 64b + lane with no carry out of the low byte
             * and the bulk kernel's counter-mode caching applies: rounds 1-2
             * cost 1 + 4 LDS lookups per block instead of 32 (133 vs 160) */
            const uint64_t shift = align & 0xFFFFu;
            const uint64_t cb = c.lo - shift; /* no borrow: shift <= ctr0.lo mod TILE */
            const uint64_t clo = cb + vb;
            const uint64_t chi = c.hi + (clo < cb ? 1u : 0u);
            const uint32_t w0 = bswap32((uint32_t)(chi >> 32)) ^ K.rk[0];
            const uint32_t w1 = bswap32((uint32_t)chi) ^ K.rk[1];
            const uint32_t w2 = bswap32((uint32_t)(clo >> 32)) ^ K.rk[2];
            const uint32_t w3u = bswap32((uint32_t)clo) ^ K.rk[3];
            const uint32_t U0 = te_u(w0) ^ rotl8(te_u(w1 >> 8)) ^ rotl16(te_u(w2 >> 16)) ^ K.rk[4];
            const uint32_t t1 = te_u(w1) ^ rotl8(te_u(w2 >> 8)) ^ rotl16(te_u(w3u >> 16)) ^ rotl24(te_u(w0 >> 24)) ^ K.rk[5];
            const uint32_t t2 = te_u(w2) ^ rotl8(te_u(w3u >> 8)) ^ rotl16(te_u(w0 >> 16)) ^ rotl24(te_u(w1 >> 24)) ^ K.rk[6];
            const uint32_t t3 = te_u(w3u) ^ rotl8(te_u(w0 >> 8)) ^ rotl16(te_u(w1 >> 16)) ^ rotl24(te_u(w2 >> 24)) ^ K.rk[7];
            const uint32_t V0 = rotl8(te_u(t1 >> 8)) ^ rotl16(te_u(t2 >> 16)) ^ rotl24(te_u(t3 >> 24)) ^ K.rk[8];
            const uint32_t V1 = te_u(t1) ^ rotl8(te_u(t2 >> 8)) ^ rotl16(te_u(t3 >> 16)) ^ K.rk[9];
            const uint32_t V2 = te_u(t2) ^ rotl8(te_u(t3 >> 8)) ^ rotl24(te_u(t1 >> 24)) ^ K.rk[10];
            const uint32_t V3 = te_u(t3) ^ rotl16(te_u(t1 >> 16)) ^ rotl24(te_u(t2 >> 24)) ^ K.rk[11];
            const uint32_t b15 = (uint32_t)(clo & 0xFFu);
            i0 = (int64_t)vb - (int64_t)shift + lane;
#pragma unroll
            for (int b = 0; b < B; ++b) {
                const int64_t i = i0 + 64 * b;
                x[b] = (i >= 0 && (uint64_t)i < nfull) ? gld16(in, (uint64_t)i) : make_uint4(0, 0, 0, 0);
                const uint32_t c15 = (b15 | (uint32_t)(64 * b) | lane) ^ (K.rk[3] >> 24);
                const uint32_t s0 = U0 ^ lds_at(tbl, (c15 << 8) | lk[3]);
                s[b][0] = V0 ^ lds_at(tbl, tt_addr(s0, lk[0], 0));
                s[b][1] = V1 ^ lds_at(tbl, tt_addr(s0, lk[3], 3));
                s[b][2] = V2 ^ lds_at(tbl, tt_addr(s0, lk[2], 2));
                s[b][3] = V3 ^ lds_at(tbl, tt_addr(s0, lk[1], 1));
            }
            enc_rounds4_from<3, NR, B>(tbl, lk, K, s);
        } else {
            i0 = (int64_t)vb + lane;
#pragma unroll
            for (int b = 0; b < B; ++b) {
                const uint64_t i = (uint64_t)i0 + 64u * b;
                ctr_words(c, i, false, s[b][0], s[b][1], s[b][2], s[b][3]);
                x[b] = i < nfull ? gld16(in, i) : make_uint4(0, 0, 0, 0);
#pragma unroll
                for (int j = 0; j < 4; ++j) s[b][j] ^= K.rk[j];
            }
            enc_rounds4_from<1, NR, B>(tbl, lk, K, s);
        }
#pragma unroll
        for (int b = 0; b < B; ++b) {
            const int64_t i = i0 + 64 * b;
            if (i < 0) continue;
            if ((uint64_t)i < nfull) {
                gst16(out, (uint64_t)i,
                      make_uint4(x[b].x ^ s[b][0], x[b].y ^ s[b][1], x[b].z ^ s[b][2], x[b].w ^ s[b][3]));
            } else if ((uint64_t)i == nfull && tail) {
                const uint32_t ks[4] = {s[b][0], s[b][1], s[b][2], s[b][3]};
                const g_u8 *gi = (const g_u8 *)in;
                g_u8 *go = (g_u8 *)out;
                for (uint32_t n = 0; n < tail; ++n)
                    go[16 * (uint64_t)i + n] = gi[16 * (uint64_t)i + n] ^ (uint8_t)(ks[n >> 2] >> (8 * (n & 3)));
            }
        }
    }
}

constexpr int BATCH_THREADS = 1024;
static_assert(64 * 4 == OTC_BATCH_TILE_BLOCKS, "largest tile must match otc.h");

/* ---------------------------------------------------------------------------
 * Host-side launch helpers
 * ------------------------------------------------------------------------- */
inline int num_cus() { return otc_dev::device_cus(); }

/* launch a claim kernel with `lds` bytes of dynamic LDS for its tables
 * (tt_lds); the opt-in above 64 KiB is made once per kernel and device */
template <auto KERN, typename... A>
hipError_t launch_dyn(dim3 g, dim3 b, uint32_t lds, hipStream_t st, A... args)
{
    static std::atomic<uint64_t> opted{0};
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    const uint64_t bit = 1ull << (dev & 63);
    if (!(opted.load(std::memory_order_acquire) & bit)) {
        e = hipFuncSetAttribute((const void *)KERN, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        opted.fetch_or(bit, std::memory_order_acq_rel);
    }
    hipLaunchKernelGGL(KERN, g, b, lds, st, args...);
    return hipGetLastError();
}
constexpr uint32_t ENC_LDS = 2 * 256 * 64 * 4, DEC_LDS = (2 * 256 * 64 + 256 * 32) * 4;

int grid_for(uint64_t work_items, uint64_t per_wg, int wg_per_cu)
{
    uint64_t need = (work_items + per_wg - 1) / per_wg;
    uint64_t cap = (uint64_t)num_cus() * (uint64_t)wg_per_cu;
    if (need < 1) need = 1;
    return (int)(need < cap ? need : cap);
}

/* Small inputs: a persistent 1024 x 4 workgroup takes 4096 blocks per step,
 * so a 1 MiB message (65536 blocks) occupies only 16 CUs and takes as long as
 * one CU needs for 4096 blocks (~10 us).  Below these sizes the launch uses
 * smaller steps so that (up to) every CU gets work: 256 threads x 1 block per
 * lane up to 256 x 256 blocks (1 MiB), 1024 x 1 up to 256 x 1024 (4 MiB).
 * Mid sizes: the busiest CU does ceil(steps / CUs) steps, so 10 MiB (160
 * steps of 4096 blocks) leaves 96 CUs idle and 100 MiB (1600 steps) runs 7
 * rounds for 6.25 rounds of work; 1024-block steps are used whenever they cut
 * the busiest CU's block count by 5% or more. */
enum SmallShape { SHAPE_BULK = 0, SHAPE_256x1 = 1, SHAPE_1024x1 = 2 };
inline uint64_t busiest_cu_blocks(uint64_t nblocks, uint64_t step)
{
    const uint64_t cus = (uint64_t)num_cus();
    return ((nblocks + step - 1) / step + cus - 1) / cus * step;
}
inline SmallShape small_shape(uint64_t nblocks)
{
    if (nblocks <= 256ull * 256) return SHAPE_256x1;
    if (nblocks <= 256ull * 1024) return SHAPE_1024x1;
    if (busiest_cu_blocks(nblocks, 1024) * 20 <= busiest_cu_blocks(nblocks, 4096) * 19)
        return SHAPE_1024x1;
    return SHAPE_BULK;
}

constexpr int ENC_THREADS = 1024; /* measured best of 256..1024 x B=1..4 (docs/PERF.md) */
constexpr int ENC_B = OTC_TT_ENC_B;
constexpr int DEC_THREADS = 1024;
constexpr int DEC_B = OTC_TT_DEC_B;
constexpr int SEG_THREADS = 1024;
constexpr int SEG_B = 2;

template <int NR, int MODE, int T, int B>
hipError_t launch_enc_tb(const EncParams &P, const otc_aes_key &K, hipStream_t st)
{
    int grid = grid_for(P.nfull, (uint64_t)T * B, 1); /* 128 KiB LDS: one workgroup per CU */
    hipLaunchKernelGGL((k_aes_enc_tt<NR, MODE, B, T>), dim3(grid), dim3(T), 0, st, P, K);
    return hipGetLastError();
}

template <int NR, int MODE>
hipError_t launch_enc_nr(const EncParams &P, const otc_aes_key &K, hipStream_t st)
{
    switch (small_shape(P.nfull)) {
    case SHAPE_256x1: return launch_enc_tb<NR, MODE, 256, 1>(P, K, st);
    case SHAPE_1024x1: return launch_enc_tb<NR, MODE, 1024, 1>(P, K, st);
    default: return launch_enc_tb<NR, MODE, ENC_THREADS, ENC_B>(P, K, st);
    }
}

template <int MODE>
hipError_t launch_enc(const EncParams &P, const otc_aes_key &K, hipStream_t st)
{
    switch (K.nr) {
    case 10: return launch_enc_nr<10, MODE>(P, K, st);
    case 12: return launch_enc_nr<12, MODE>(P, K, st);
    case 14: return launch_enc_nr<14, MODE>(P, K, st);
    default: return hipErrorInvalidValue;
    }
}

template <int NR, int MODE>
hipError_t launch_dec_nr(const DecParams &P, const otc_aes_key &K, hipStream_t st)
{
    switch (small_shape(P.nfull)) {
    case SHAPE_256x1:
        hipLaunchKernelGGL((k_aes_dec_tt<NR, MODE, 1, 256>), dim3(grid_for(P.nfull, 256, 1)), dim3(256), 0, st, P, K);
        break;
    case SHAPE_1024x1:
        hipLaunchKernelGGL((k_aes_dec_tt<NR, MODE, 1, 1024>), dim3(grid_for(P.nfull, 1024, 1)), dim3(1024), 0, st, P,
                           K);
        break;
    default:
        hipLaunchKernelGGL((k_aes_dec_tt<NR, MODE, DEC_B, DEC_THREADS>),
                           dim3(grid_for(P.nfull, (uint64_t)DEC_THREADS * DEC_B, 1)), dim3(DEC_THREADS), 0, st, P, K);
    }
    return hipGetLastError();
}

template <int MODE>
hipError_t launch_dec(const DecParams &P, const otc_aes_key &K, hipStream_t st)
{
    switch (K.nr) {
    case 10: return launch_dec_nr<10, MODE>(P, K, st);
    case 12: return launch_dec_nr<12, MODE>(P, K, st);
    case 14: return launch_dec_nr<14, MODE>(P, K, st);
    default: return hipErrorInvalidValue;
    }
}

/* the T-table half of a claimed split: one persistent workgroup per CU */
template <int MODE>
hipError_t launch_enc_claim(const EncParams &P, const otc_aes_key &K, hipStream_t st)
{
    const dim3 g(P.cl.wgs ? P.cl.wgs : (unsigned)num_cus()), b(ENC_THREADS);
    auto go = [&](auto nr) {
        constexpr int NR = decltype(nr)::value;
        if constexpr (MODE == E_ECB) return launch_dyn<k_aes_ecb_tt_claim<NR>>(g, b, ENC_LDS, st, P, K);
        else if constexpr (MODE == E_CFB_DEC) return launch_dyn<k_aes_cfb_tt_claim<NR>>(g, b, ENC_LDS, st, P, K);
        else return launch_dyn<k_aes_cfbseg_tt_claim<NR>>(g, b, ENC_LDS, st, P, K);
    };
    switch (K.nr) {
    case 10: return go(std::integral_constant<int, 10>{});
    case 12: return go(std::integral_constant<int, 12>{});
    case 14: return go(std::integral_constant<int, 14>{});
    default: return hipErrorInvalidValue;
    }
}

template <int MODE>
hipError_t launch_dec_claim(const DecParams &P, const otc_aes_key &K, hipStream_t st)
{
    const dim3 g(P.cl.wgs ? P.cl.wgs : (unsigned)num_cus()), b(DEC_THREADS);
    switch (K.nr) {
    case 10: return launch_dyn<k_aes_dec_tt_claim<10, MODE>>(g, b, DEC_LDS, st, P, K);
    case 12: return launch_dyn<k_aes_dec_tt_claim<12, MODE>>(g, b, DEC_LDS, st, P, K);
    case 14: return launch_dyn<k_aes_dec_tt_claim<14, MODE>>(g, b, DEC_LDS, st, P, K);
    default: return hipErrorInvalidValue;
    }
}

template <int NR, bool CFB>
hipError_t launch_seg_nr(const CbcSegParams &P, const otc_aes_key &K, hipStream_t st)
{
    int grid = grid_for(P.nseg, (uint64_t)SEG_THREADS * SEG_B, 1);
    /* 8-block load/store bursts per segment (+119% over one block at a time,
     * profiles/r1/otbench_cbcenc_group_ab.jsonl); B = 1: two 8-block buffers
     * per segment fit without spills.  Segments shorter than 8 blocks take the
     * per-block kernel. */
    if (P.seg_blocks >= OTC_SEG_G) {
        /* fewer chains than CUs x SEG_THREADS: smaller workgroups on every CU
         * (e.g. 768 MiB of 4 KiB segments: 256 x 768 threads, not 192 x 1024) */
        uint64_t nt = SEG_THREADS;
        const uint64_t cus = (uint64_t)num_cus();
#ifndef OTC_SEG_FIXED_WG /* A/B arm: 1024-thread workgroups at every size */
        if (P.nseg < cus * SEG_THREADS) nt = std::max<uint64_t>(64, ((P.nseg + cus - 1) / cus + 63) / 64 * 64);
#endif
        hipLaunchKernelGGL((k_aes_cbc_enc_seg_g<NR, SEG_THREADS, OTC_SEG_G, CFB>), dim3(grid_for(P.nseg, nt, 1)),
                           dim3((unsigned)nt), 0, st, P, K);
    } else
        hipLaunchKernelGGL((k_aes_cbc_enc_seg<NR, SEG_B, SEG_THREADS, CFB>), dim3(grid), dim3(SEG_THREADS), 0, st, P,
                           K);
    return hipGetLastError();
}

template <int NR, int B>
hipError_t launch_ctr_batch_nrb(const BatchParams &P, hipStream_t st)
{
    /* one workgroup per CU (128 KiB LDS), 16 tiles per workgroup step */
    const int grid = grid_for(P.ntiles, BATCH_THREADS / 64, 1);
    hipLaunchKernelGGL((k_aes_ctr_batch_tt<NR, B, BATCH_THREADS>), dim3(grid), dim3(BATCH_THREADS), 0, st, P);
    return hipGetLastError();
}

template <int NR>
hipError_t launch_ctr_batch_nr(const BatchParams &P, int tile_blocks, hipStream_t st)
{
    switch (tile_blocks) {
    case 64: return launch_ctr_batch_nrb<NR, 1>(P, st);
    case 128: return launch_ctr_batch_nrb<NR, 2>(P, st);
    case 256: return launch_ctr_batch_nrb<NR, 4>(P, st);
    default: return hipErrorInvalidValue;
    }
}

} // namespace

/* ---- internal entry points used by engine.cpp ---------------------------- */
namespace otc_impl {

OTC_STRACE_READER(strace_read_tt)

uint64_t tt_ctr_batch_units(uint64_t ntiles) { return (ntiles + BATCH_UNIT - 1) / BATCH_UNIT; }

hipError_t tt_ctr_batch(const otc_ctr_msg *msgs, const otc_aes_key *keys, const uint32_t *tile_msg,
                        const uint64_t *tile_first, uint64_t ntiles, int tile_blocks, int nr, hipStream_t st,
                        const SplitClaim *cl)
{
    BatchParams P{msgs, keys, tile_msg, tile_first, ntiles};
    if (cl) P.cl = *cl;
    switch (nr) {
    case 10: return launch_ctr_batch_nr<10>(P, tile_blocks, st);
    case 12: return launch_ctr_batch_nr<12>(P, tile_blocks, st);
    case 14: return launch_ctr_batch_nr<14>(P, tile_blocks, st);
    default: return hipErrorInvalidValue;
    }
}

hipError_t tt_ecb_encrypt(const void *in, void *out, uint64_t nblocks, const otc_aes_key &K, hipStream_t st)
{
    EncParams P{};
    P.in = (const uint8_t *)in;
    P.out = (uint8_t *)out;
    P.nfull = nblocks;
    return launch_enc<E_ECB>(P, K, st);
}

/* one 1024- or 256-thread workgroup per CU (the 128 KiB 4-table image) */
template <int NR, int T, int B>
hipError_t launch_ctr_cached_tb(CtrParams P, const otc_aes_key &K, uint64_t ctr_lo, hipStream_t st)
{
    constexpr uint64_t PER = (uint64_t)T * B;
    P.shift = ctr_lo & (PER - 1);
    P.cbase.lo = ctr_lo - P.shift;
    const uint64_t vt = P.nfull + (P.tail ? 1 : 0) + P.shift;
    hipLaunchKernelGGL((k_aes_ctr_tt_cached<NR, B, T>), dim3(grid_for(vt, PER, 1)), dim3(T), 0, st, P, K);
    return hipGetLastError();
}

template <int NR>
hipError_t launch_ctr_cached(CtrParams P, const otc_aes_key &K, uint64_t ctr_lo, hipStream_t st)
{
    switch (small_shape(P.nfull + (P.tail ? 1 : 0))) {
    case SHAPE_256x1: return launch_ctr_cached_tb<NR, 256, 1>(P, K, ctr_lo, st);
    case SHAPE_1024x1: return launch_ctr_cached_tb<NR, 1024, 1>(P, K, ctr_lo, st);
    default: return launch_ctr_cached_tb<NR, 1024, OTC_TT_CTR_B>(P, K, ctr_lo, st);
    }
}

hipError_t tt_ctr(const void *in, void *out, size_t nbytes, const otc_aes_key &K, Ctr128 c, bool wrap64,
                  hipStream_t st)
{
    CtrParams P{};
    P.in = (const uint8_t *)in;
    P.out = (uint8_t *)out;
    P.nfull = nbytes / 16;
    P.tail = (uint32_t)(nbytes % 16);
    P.wrap64 = wrap64 ? 1u : 0u;
    P.cbase.hi = c.hi;
    switch (K.nr) {
    case 10: return launch_ctr_cached<10>(P, K, c.lo, st);
    case 12: return launch_ctr_cached<12>(P, K, c.lo, st);
    case 14: return launch_ctr_cached<14>(P, K, c.lo, st);
    default: return hipErrorInvalidValue;
    }
}

/* the persistent claim form of tt_ctr: its virtual range (the blocks plus
 * ctr0 mod 4096 in front) in 2048-block units */
uint64_t tt_ctr_claim_units(size_t nbytes, uint64_t ctr_lo)
{
    return (nbytes / 16 + (nbytes % 16 ? 1 : 0) + (ctr_lo & 4095u) + CLAIM_UNIT - 1) / CLAIM_UNIT;
}

hipError_t tt_ctr_claim(const void *in, void *out, size_t nbytes, const otc_aes_key &K, Ctr128 c, bool wrap64,
                        SplitClaim cl, hipStream_t st)
{
    CtrParams P{};
    P.in = (const uint8_t *)in;
    P.out = (uint8_t *)out;
    P.nfull = nbytes / 16;
    P.tail = (uint32_t)(nbytes % 16);
    P.wrap64 = wrap64 ? 1u : 0u;
    P.cbase.hi = c.hi;
    P.shift = c.lo & 4095u; /* as the grid kernel's bulk shape (PER = 1024 x 4) */
    P.cbase.lo = c.lo - P.shift;
    P.cl = cl;
    const dim3 g(cl.wgs ? cl.wgs : (unsigned)num_cus()), b(1024);
    switch (K.nr) {
    case 10: hipLaunchKernelGGL(k_aes_ctr_tt_persist<10>, g, b, 0, st, P, K); break;
    case 12: hipLaunchKernelGGL(k_aes_ctr_tt_persist<12>, g, b, 0, st, P, K); break;
    case 14: hipLaunchKernelGGL(k_aes_ctr_tt_persist<14>, g, b, 0, st, P, K); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t tt_cfb_decrypt(const void *in, void *out, uint64_t nblocks, const otc_aes_key &K,
                          const uint32_t iv_le[4], hipStream_t st)
{
    EncParams P{};
    P.in = (const uint8_t *)in;
    P.out = (uint8_t *)out;
    P.nfull = nblocks;
    for (int i = 0; i < 4; ++i) P.iv[i] = iv_le[i];
    return launch_enc<E_CFB_DEC>(P, K, st);
}

hipError_t tt_ecb_decrypt(const void *in, void *out, uint64_t nblocks, const otc_aes_key &K, hipStream_t st)
{
    DecParams P{};
    P.in = (const uint8_t *)in;
    P.out = (uint8_t *)out;
    P.nfull = nblocks;
    return launch_dec<D_ECB>(P, K, st);
}

hipError_t tt_cbc_decrypt(const void *in, void *out, uint64_t nblocks, const otc_aes_key &K, Ctr128 iv,
                          hipStream_t st)
{
    DecParams P{};
    P.in = (const uint8_t *)in;
    P.out = (uint8_t *)out;
    P.nfull = nblocks;
    P.iv = iv;
    return launch_dec<D_CBC>(P, K, st);
}

/* The T-table halves of a claimed co-resident split (engine.cpp): the whole
 * buffer, units from the back of `cl`, plus the blocks past its last unit. */
hipError_t tt_ecb_encrypt_claim(const void *in, void *out, uint64_t nblocks, const otc_aes_key &K, SplitClaim cl,
                                hipStream_t st)
{
    EncParams P{};
    P.in = (const uint8_t *)in;
    P.out = (uint8_t *)out;
    P.nfull = nblocks;
    P.cl = cl;
    return launch_enc_claim<E_ECB>(P, K, st);
}

hipError_t tt_cfb_decrypt_claim(const void *in, void *out, uint64_t nblocks, const otc_aes_key &K,
                                const uint32_t iv_le[4], SplitClaim cl, hipStream_t st)
{
    EncParams P{};
    P.in = (const uint8_t *)in;
    P.out = (uint8_t *)out;
    P.nfull = nblocks;
    for (int i = 0; i < 4; ++i) P.iv[i] = iv_le[i];
    P.cl = cl;
    return launch_enc_claim<E_CFB_DEC>(P, K, st);
}

hipError_t tt_ecb_decrypt_claim(const void *in, void *out, uint64_t nblocks, const otc_aes_key &K, SplitClaim cl,
                                hipStream_t st)
{
    DecParams P{};
    P.in = (const uint8_t *)in;
    P.out = (uint8_t *)out;
    P.nfull = nblocks;
    P.cl = cl;
    return launch_dec_claim<D_ECB>(P, K, st);
}

hipError_t tt_cbc_decrypt_claim(const void *in, void *out, uint64_t nblocks, const otc_aes_key &K, Ctr128 iv,
                                SplitClaim cl, hipStream_t st)
{
    DecParams P{};
    P.in = (const uint8_t *)in;
    P.out = (uint8_t *)out;
    P.nfull = nblocks;
    P.iv = iv;
    P.cl = cl;
    return launch_dec_claim<D_CBC>(P, K, st);
}

/* the T-table halves of a claimed split over power-of-two segments
 * (2^seg_shift blocks, IV_s = iv0 + s) */
hipError_t tt_cbc_decrypt_seg_claim(const void *in, void *out, uint64_t nblocks, const otc_aes_key &K, Ctr128 iv0,
                                    uint32_t seg_shift, SplitClaim cl, hipStream_t st)
{
    DecParams P{};
    P.in = (const uint8_t *)in;
    P.out = (uint8_t *)out;
    P.nfull = nblocks;
    P.iv = iv0;
    P.seg_shift = seg_shift;
    P.cl = cl;
    return launch_dec_claim<D_CBC_SEG>(P, K, st);
}

hipError_t tt_cfb_decrypt_seg_claim(const void *in, void *out, uint64_t nblocks, const otc_aes_key &K, Ctr128 iv0,
                                    uint32_t seg_shift, SplitClaim cl, hipStream_t st)
{
    EncParams P{};
    P.in = (const uint8_t *)in;
    P.out = (uint8_t *)out;
    P.nfull = nblocks;
    P.ctr = iv0;
    P.seg_blocks = 1ull << seg_shift;
    P.seg_shift = seg_shift;
    P.cl = cl;
    return launch_enc_claim<E_CFB_DEC_SEG>(P, K, st);
}

hipError_t tt_cbc_decrypt_seg(const void *in, void *out, uint64_t seg_blocks, uint64_t nseg,
                              const otc_aes_key &K, Ctr128 iv0, hipStream_t st)
{
    DecParams P{};
    P.in = (const uint8_t *)in;
    P.out = (uint8_t *)out;
    P.nfull = seg_blocks * nseg;
    P.iv = iv0;
    if (seg_blocks && (seg_blocks & (seg_blocks - 1)) == 0) { /* power of two: in-kernel IVs */
        uint32_t sh = 0;
        while ((1ull << sh) < seg_blocks) ++sh;
        P.seg_shift = sh;
        return launch_dec<D_CBC_SEG>(P, K, st);
    }
    hipError_t e = launch_dec<D_CBC>(P, K, st);
    if (e != hipSuccess || nseg < 2) return e;
    const uint64_t nfix = nseg - 1;
    hipLaunchKernelGGL(k_cbc_seg_fixup, dim3((unsigned)((nfix + 255) / 256)), dim3(256), 0, st,
                       (const uint8_t *)in, (uint8_t *)out, seg_blocks, nseg, iv0);
    return hipGetLastError();
}

template <bool CFB>
static hipError_t chain_encrypt_seg(const void *in, void *out, uint64_t seg_blocks, uint64_t nseg,
                                    const otc_aes_key &K, Ctr128 iv0, hipStream_t st)
{
    CbcSegParams P{};
    P.in = (const uint8_t *)in;
    P.out = (uint8_t *)out;
    P.seg_blocks = seg_blocks;
    P.nseg = nseg;
    P.iv0 = iv0;
    switch (K.nr) {
    case 10: return launch_seg_nr<10, CFB>(P, K, st);
    case 12: return launch_seg_nr<12, CFB>(P, K, st);
    case 14: return launch_seg_nr<14, CFB>(P, K, st);
    default: return hipErrorInvalidValue;
    }
}

hipError_t tt_cbc_encrypt_seg(const void *in, void *out, uint64_t seg_blocks, uint64_t nseg,
                              const otc_aes_key &K, Ctr128 iv0, hipStream_t st)
{
    return chain_encrypt_seg<false>(in, out, seg_blocks, nseg, K, iv0, st);
}

hipError_t tt_ctr_shift(const void *body_in, void *body_out, size_t len, const otc_aes_key &K, Ctr128 c,
                        hipStream_t st)
{
    const uint32_t a = (uint32_t)((uintptr_t)body_in & 15u);
    if (a == 0 || a != ((uintptr_t)body_out & 15u)) return hipErrorInvalidValue;
    if (len == 0) return hipSuccess;
    CtrShiftParams P{};
    P.in = (const uint8_t *)body_in - a;
    P.out = (uint8_t *)body_out - a;
    P.len = len;
    P.a = a;
    P.ctr = c;
    constexpr int T = 1024;
    const uint64_t waves = ((a + len + 15) / 16 + 62) / 63;
    const int grid = grid_for(waves, T / 64, 1);
    switch (K.nr) {
    case 10: hipLaunchKernelGGL((k_aes_ctr_shift<10, T>), dim3(grid), dim3(T), 0, st, P, K); break;
    case 12: hipLaunchKernelGGL((k_aes_ctr_shift<12, T>), dim3(grid), dim3(T), 0, st, P, K); break;
    case 14: hipLaunchKernelGGL((k_aes_ctr_shift<14, T>), dim3(grid), dim3(T), 0, st, P, K); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t xor_small(const void *in, void *out, uint32_t n, const uint8_t *ks, hipStream_t st)
{
    if (n == 0) return hipSuccess;
    if (n > 16) return hipErrorInvalidValue;
    SmallXor k{};
    for (uint32_t i = 0; i < n; ++i) k.ks[i] = ks[i];
    hipLaunchKernelGGL(k_xor_small, dim3(1), dim3(64), 0, st, (const uint8_t *)in, (uint8_t *)out, n, k);
    return hipGetLastError();
}

hipError_t tt_cfb_encrypt_seg(const void *in, void *out, uint64_t seg_blocks, uint64_t nseg,
                              const otc_aes_key &K, Ctr128 iv0, hipStream_t st)
{
    return chain_encrypt_seg<true>(in, out, seg_blocks, nseg, K, iv0, st);
}

/* the T-table half of the chained segment-encryption split: 64-segment
 * units from the back of `cl` (cl.wgs workgroups, default one per CU) */
hipError_t tt_seg_encrypt_claim(bool cfb, const void *in, void *out, uint64_t seg_blocks, uint64_t nseg,
                                const otc_aes_key &K, Ctr128 iv0, SplitClaim cl, hipStream_t st)
{
    CbcSegParams P{};
    P.in = (const uint8_t *)in;
    P.out = (uint8_t *)out;
    P.seg_blocks = seg_blocks;
    P.nseg = nseg;
    P.iv0 = iv0;
    P.cl = cl;
    const dim3 g(cl.wgs ? cl.wgs : (unsigned)num_cus()), b(1024);
    constexpr int G = SEG_CLAIM_G;
    auto go = [&](auto nr) {
        constexpr int NR = decltype(nr)::value;
        return cfb ? launch_dyn<k_aes_seg_enc_tt_claim<NR, G, true>>(g, b, ENC_LDS, st, P, K)
                   : launch_dyn<k_aes_seg_enc_tt_claim<NR, G, false>>(g, b, ENC_LDS, st, P, K);
    };
    switch (K.nr) {
    case 10: return go(std::integral_constant<int, 10>{});
    case 12: return go(std::integral_constant<int, 12>{});
    case 14: return go(std::integral_constant<int, 14>{});
    default: return hipErrorInvalidValue;
    }
}

hipError_t tt_cfb_decrypt_seg(const void *in, void *out, uint64_t seg_blocks, uint64_t nseg,
                              const otc_aes_key &K, Ctr128 iv0, hipStream_t st)
{
    EncParams P{};
    P.in = (const uint8_t *)in;
    P.out = (uint8_t *)out;
    P.nfull = seg_blocks * nseg;
    P.ctr = iv0;
    P.seg_blocks = seg_blocks;
    P.seg_shift = 64;
    if ((seg_blocks & (seg_blocks - 1)) == 0) {
        uint32_t sh = 0;
        while ((1ull << sh) < seg_blocks) ++sh;
        P.seg_shift = sh;
    }
    return launch_enc<E_CFB_DEC_SEG>(P, K, st);
}

} // namespace otc_impl
