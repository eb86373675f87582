/*
 * otc_bitslice.h -- bitsliced AES round functions, shared by the gfx950 HIP
 * kernels (csrc/hip/aes_bs.hip) and the host unit test (csrc/cpu/bs_selftest.cpp).
 *
 * Representation: one 32-bit word per (state byte, bit) "plane".  Bit k of
 * plane[8*b + i] is bit i of AES state byte b (b = row + 4*col, FIPS-197
 * order) of block slot k, so one lane processes 32 blocks with 128 VGPRs of
 * state.  ShiftRows is free (compile-time renaming under full unrolling);
 * SubBytes is the Boyar-Peralta depth-16 circuit (113 XOR/XNOR/AND gates) which
 * hipcc fuses into gfx950's 3-input v_bitop3_b32 / v_xor3_b32; MixColumns is
 * the xtime formulation out_r = xt(a_r ^ a_{r+1}) ^ (a0^a1^a2^a3) ^ a_r.
 *
 * No reference counterpart: the reference's only GPU code is a T-table kernel
 * (/root/reference/aes-gpu/Source/AES.cu:284-392).  This is the "wave-level
 * bitsliced VALU path" of BASELINE.json's north star.
 */
#ifndef OTC_BITSLICE_H
#define OTC_BITSLICE_H

#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define OTC_HD __host__ __device__ __forceinline__
#else
#define OTC_HD inline
#endif



namespace otc_bs {

typedef uint32_t W;

/* Forward S-box on 8 planes x[0..7] (x[i] = bit i, i = 0 is the LSB). */
OTC_HD void sbox(W &x0, W &x1, W &x2, W &x3, W &x4, W &x5, W &x6, W &x7)
{
    /* Boyar-Peralta naming: U0 is the most significant bit. */
    const W U0 = x7, U1 = x6, U2 = x5, U3 = x4, U4 = x3, U5 = x2, U6 = x1, U7 = x0;
    const W T1 = U0 ^ U3, T2 = U0 ^ U5, T3 = U0 ^ U6, T4 = U3 ^ U5, T5 = U4 ^ U6;
    const W T6 = T1 ^ T5, T7 = U1 ^ U2, T8 = U7 ^ T6, T9 = U7 ^ T7, T10 = T6 ^ T7;
    const W T11 = U1 ^ U5, T12 = U2 ^ U5, T13 = T3 ^ T4, T14 = T6 ^ T11, T15 = T5 ^ T11;
    const W T16 = T5 ^ T12, T17 = T9 ^ T16, T18 = U3 ^ U7, T19 = T7 ^ T18, T20 = T1 ^ T19;
    const W T21 = U6 ^ U7, T22 = T7 ^ T21, T23 = T2 ^ T22, T24 = T2 ^ T10, T25 = T20 ^ T17;
    const W T26 = T3 ^ T16, T27 = T1 ^ T12;

    const W M1 = T13 & T6, M2 = T23 & T8, M3 = T14 ^ M1, M4 = T19 & U7, M5 = M4 ^ M1;
    const W M6 = T3 & T16, M7 = T22 & T9, M8 = T26 ^ M6, M9 = T20 & T17, M10 = M9 ^ M6;
    const W M11 = T1 & T15, M12 = T4 & T27, M13 = M12 ^ M11, M14 = T2 & T10, M15 = M14 ^ M11;
    const W M16 = M3 ^ M2, M17 = M5 ^ T24, M18 = M8 ^ M7, M19 = M10 ^ M15, M20 = M16 ^ M13;
    const W M21 = M17 ^ M15, M22 = M18 ^ M13, M23 = M19 ^ T25, M24 = M22 ^ M23, M25 = M22 & M20;
    const W M26 = M21 ^ M25, M27 = M20 ^ M21, M28 = M23 ^ M25, M29 = M28 & M27, M30 = M26 & M24;
    const W M31 = M20 & M23, M32 = M27 & M31, M33 = M27 ^ M25, M34 = M21 & M22, M35 = M24 & M34;
    const W M36 = M24 ^ M25, M37 = M21 ^ M29, M38 = M32 ^ M33, M39 = M23 ^ M30, M40 = M35 ^ M36;
    const W M41 = M38 ^ M40, M42 = M37 ^ M39, M43 = M37 ^ M38, M44 = M39 ^ M40, M45 = M42 ^ M41;
    const W M46 = M44 & T6, M47 = M40 & T8, M48 = M39 & U7, M49 = M43 & T16, M50 = M38 & T9;
    const W M51 = M37 & T17, M52 = M42 & T15, M53 = M45 & T27, M54 = M41 & T10, M55 = M44 & T13;
    const W M56 = M40 & T23, M57 = M39 & T19, M58 = M43 & T3, M59 = M38 & T22, M60 = M37 & T20;
    const W M61 = M42 & T1, M62 = M45 & T4, M63 = M41 & T2;

    const W L0 = M61 ^ M62, L1 = M50 ^ M56, L2 = M46 ^ M48, L3 = M47 ^ M55, L4 = M54 ^ M58;
    const W L5 = M49 ^ M61, L6 = M62 ^ L5, L7 = M46 ^ L3, L8 = M51 ^ M59, L9 = M52 ^ M53;
    const W L10 = M53 ^ L4, L11 = M60 ^ L2, L12 = M48 ^ M51, L13 = M50 ^ L0, L14 = M52 ^ M61;
    const W L15 = M55 ^ L1, L16 = M56 ^ L0, L17 = M57 ^ L1, L18 = M58 ^ L8, L19 = M63 ^ L4;
    const W L20 = L0 ^ L1, L21 = L1 ^ L7, L22 = L3 ^ L12, L23 = L18 ^ L2, L24 = L15 ^ L9;
    const W L25 = L6 ^ L10, L26 = L7 ^ L9, L27 = L8 ^ L10, L28 = L11 ^ L14, L29 = L11 ^ L17;

    const W S0 = L6 ^ L24, S1 = ~(L16 ^ L26), S2 = ~(L19 ^ L28), S3 = L6 ^ L21;
    const W S4 = L20 ^ L22, S5 = L25 ^ L29, S6 = ~(L13 ^ L27), S7 = ~(L6 ^ L23);
    x7 = S0; x6 = S1; x5 = S2; x4 = S3; x3 = S4; x2 = S5; x1 = S6; x0 = S7;
}

OTC_HD void sub_bytes(W *s)
{
#pragma unroll
    for (int b = 0; b < 16; ++b)
        sbox(s[8 * b + 0], s[8 * b + 1], s[8 * b + 2], s[8 * b + 3], s[8 * b + 4], s[8 * b + 5],
             s[8 * b + 6], s[8 * b + 7]);
}

/* Scheduling fence on the device: keeps hipcc's machine scheduler from
 * interleaving independent S-boxes / columns, which otherwise blows the live
 * register set far past the 128-plane state (1 wave/SIMD + spills). */
OTC_HD void sched_fence()
{
#if defined(__HIP_DEVICE_COMPILE__)
    __builtin_amdgcn_sched_barrier(0);
#endif
}

/* Pin values in VGPRs at this program point: an empty volatile asm that
 * "modifies" them.  Volatile asms keep their relative order and everything
 * computed from a pinned value must follow it, so this orders whole phases
 * for the SelectionDAG scheduler too (sched_barrier only binds the machine
 * scheduler; pure ALU ops float across it in the DAG). */
OTC_HD void pin8(W *x)
{
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]));
#else
    (void)x;
#endif
}
OTC_HD void pin_n(W *x, int n)
{
    for (int i = 0; i + 8 <= n; i += 8) pin8(x + i);
}

/* Wait for the current S-box's key terms BEFORE the next S-box's scalar
 * loads are issued: scalar loads return out of order, so the only wait the
 * compiler can emit for them is lgkmcnt(0) -- placed at their first use inside
 * the S-box it would also wait for the prefetch just issued.  An empty asm
 * reading the terms puts that wait here. */
/* lists t[0..10]: OTC_SBOX_KEY_TERMS (otc_sbox_lut3.h) is pinned to 11 below */
OTC_HD void kt_ready(const W *t)
{
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" ::"s"(t[0]), "s"(t[1]), "s"(t[2]), "s"(t[3]), "s"(t[4]), "s"(t[5]), "s"(t[6]), "s"(t[7]),
                 "s"(t[8]), "s"(t[9]), "s"(t[10]));
#else
    (void)t;
#endif
}

/* 3-input XOR.  VEC: one v_bitop3_b32 on gfx950 (hipcc does not fuse pure
 * XOR chains itself).  !VEC: plain C, so hipcc can keep wave-uniform planes
 * on the scalar ALU. */
template <bool VEC>
OTC_HD W xx3(W a, W b, W c)
{
#if defined(__HIP_DEVICE_COMPILE__)
    if (VEC) return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#endif
    return a ^ b ^ c;
}

/* S-box of (x ^ k) with the round-key masks k0..k7 (wave-uniform, 0 or ~0)
 * folded into the top linear layer: every first-level XOR of two inputs
 * becomes a 3-input XOR with the uniform constant k_a ^ k_b (free: the third
 * bitop3 operand is an SGPR), and only U7, used raw by two ANDs, needs an
 * explicit XOR.  AddRoundKey thus costs 1 VALU op per S-box instead of 8. */
template <bool VEC>
OTC_HD void sbox_k(W &x0, W &x1, W &x2, W &x3, W &x4, W &x5, W &x6, W &x7, W k0, W k1, W k2, W k3,
                   W k4, W k5, W k6, W k7)
{
    const W U0 = x7, U1 = x6, U2 = x5, U3 = x4, U4 = x3, U5 = x2, U6 = x1, U7 = x0;
    const W K0 = k7, K1 = k6, K2 = k5, K3 = k4, K4 = k3, K5 = k2, K6 = k1, K7 = k0;
    const W U7k = U7 ^ K7;
    const W T1 = xx3<VEC>(U0, U3, K0 ^ K3), T2 = xx3<VEC>(U0, U5, K0 ^ K5);
    const W T3 = xx3<VEC>(U0, U6, K0 ^ K6), T4 = xx3<VEC>(U3, U5, K3 ^ K5);
    const W T5 = xx3<VEC>(U4, U6, K4 ^ K6);
    const W T6 = T1 ^ T5, T7 = xx3<VEC>(U1, U2, K1 ^ K2), T8 = U7k ^ T6, T9 = U7k ^ T7, T10 = T6 ^ T7;
    const W T11 = xx3<VEC>(U1, U5, K1 ^ K5), T12 = xx3<VEC>(U2, U5, K2 ^ K5), T13 = T3 ^ T4;
    const W T14 = T6 ^ T11, T15 = T5 ^ T11;
    const W T16 = T5 ^ T12, T17 = T9 ^ T16, T18 = xx3<VEC>(U3, U7, K3 ^ K7), T19 = T7 ^ T18,
            T20 = T1 ^ T19;
    const W T21 = xx3<VEC>(U6, U7, K6 ^ K7), T22 = T7 ^ T21, T23 = T2 ^ T22, T24 = T2 ^ T10,
            T25 = T20 ^ T17;
    const W T26 = T3 ^ T16, T27 = T1 ^ T12;

    const W M1 = T13 & T6, M2 = T23 & T8, M3 = T14 ^ M1, M4 = T19 & U7k, M5 = M4 ^ M1;
    const W M6 = T3 & T16, M7 = T22 & T9, M8 = T26 ^ M6, M9 = T20 & T17, M10 = M9 ^ M6;
    const W M11 = T1 & T15, M12 = T4 & T27, M13 = M12 ^ M11, M14 = T2 & T10, M15 = M14 ^ M11;
    const W M16 = M3 ^ M2, M17 = M5 ^ T24, M18 = M8 ^ M7, M19 = M10 ^ M15, M20 = M16 ^ M13;
    const W M21 = M17 ^ M15, M22 = M18 ^ M13, M23 = M19 ^ T25, M24 = M22 ^ M23, M25 = M22 & M20;
    const W M26 = M21 ^ M25, M27 = M20 ^ M21, M28 = M23 ^ M25, M29 = M28 & M27, M30 = M26 & M24;
    const W M31 = M20 & M23, M32 = M27 & M31, M33 = M27 ^ M25, M34 = M21 & M22, M35 = M24 & M34;
    const W M36 = M24 ^ M25, M37 = M21 ^ M29, M38 = M32 ^ M33, M39 = M23 ^ M30, M40 = M35 ^ M36;
    const W M41 = M38 ^ M40, M42 = M37 ^ M39, M43 = M37 ^ M38, M44 = M39 ^ M40, M45 = M42 ^ M41;
    const W M46 = M44 & T6, M47 = M40 & T8, M48 = M39 & U7k, M49 = M43 & T16, M50 = M38 & T9;
    const W M51 = M37 & T17, M52 = M42 & T15, M53 = M45 & T27, M54 = M41 & T10, M55 = M44 & T13;
    const W M56 = M40 & T23, M57 = M39 & T19, M58 = M43 & T3, M59 = M38 & T22, M60 = M37 & T20;
    const W M61 = M42 & T1, M62 = M45 & T4, M63 = M41 & T2;

    const W L0 = M61 ^ M62, L1 = M50 ^ M56, L2 = M46 ^ M48, L3 = M47 ^ M55, L4 = M54 ^ M58;
    const W L5 = M49 ^ M61, L6 = M62 ^ L5, L7 = M46 ^ L3, L8 = M51 ^ M59, L9 = M52 ^ M53;
    const W L10 = M53 ^ L4, L11 = M60 ^ L2, L12 = M48 ^ M51, L13 = M50 ^ L0, L14 = M52 ^ M61;
    const W L15 = M55 ^ L1, L16 = M56 ^ L0, L17 = M57 ^ L1, L18 = M58 ^ L8, L19 = M63 ^ L4;
    const W L20 = L0 ^ L1, L21 = L1 ^ L7, L22 = L3 ^ L12, L23 = L18 ^ L2, L24 = L15 ^ L9;
    const W L25 = L6 ^ L10, L26 = L7 ^ L9, L27 = L8 ^ L10, L28 = L11 ^ L14, L29 = L11 ^ L17;

    x7 = L6 ^ L24;
    x6 = ~(L16 ^ L26);
    x5 = ~(L19 ^ L28);
    x4 = L6 ^ L21;
    x3 = L20 ^ L22;
    x2 = L25 ^ L29;
    x1 = ~(L13 ^ L27);
    x0 = ~(L6 ^ L23);
}

/* MixColumns of one column (bytes a0..a3 = 4 x 8 planes, rows 0..3):
 * d_r = a_r ^ a_{r+1};  out_r = xtime(d_r) ^ a_{r+1} ^ d_{r+2}
 * (= 2a_r ^ 3a_{r+1} ^ a_{r+2} ^ a_{r+3}); 76 ops with 3-input XORs. */
template <bool VEC>
OTC_HD void mix_column(const W *in, W *out)
{
    /* Register-frugal order: d_0..d_3 first (the inputs a_r stay live only
     * for the a_{r+1} term), then rows 0..3 -- row r is the last reader of
     * a_{r+1}, so each finished row frees 8 input planes. */
    W d[4][8];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int i = 0; i < 8; ++i) d[r][i] = in[8 * r + i] ^ in[8 * ((r + 1) & 3) + i];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const W *an = in + 8 * ((r + 1) & 3);
        const W *dr = d[r], *d2 = d[(r + 2) & 3];
        W *o = out + 8 * r;
        o[0] = xx3<VEC>(dr[7], an[0], d2[0]);
        o[1] = xx3<VEC>(dr[0], dr[7], an[1] ^ d2[1]);
        o[2] = xx3<VEC>(dr[1], an[2], d2[2]);
        o[3] = xx3<VEC>(dr[2], dr[7], an[3] ^ d2[3]);
        o[4] = xx3<VEC>(dr[3], dr[7], an[4] ^ d2[4]);
        o[5] = xx3<VEC>(dr[4], an[5], d2[5]);
        o[6] = xx3<VEC>(dr[5], an[6], d2[6]);
        o[7] = xx3<VEC>(dr[6], an[7], d2[7]);
    }
}

/* Low-register MixColumns of one column: t = a0^a1^a2^a3 first, then rows
 * in order, out_r[i] = xt(a_r ^ a_{r+1})[i] ^ t[i] ^ a_r[i] computed bit by
 * bit (only d7 = a_r[7] ^ a_{r+1}[7] is kept), so besides the 32 inputs only
 * t and one row of outputs are live (vs the 32 d_r planes of mix_column):
 * 80 ops instead of 76, ~20 fewer live registers at the mix peak. */
template <bool VEC>
OTC_HD void mix_column_t(const W *in, W *out)
{
    W t[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) t[i] = xx3<VEC>(in[i], in[8 + i], in[16 + i]) ^ in[24 + i];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const W *ar = in + 8 * r, *an = in + 8 * ((r + 1) & 3);
        W *o = out + 8 * r;
        const W d7 = ar[7] ^ an[7];
        o[0] = xx3<VEC>(d7, t[0], ar[0]);
#pragma unroll
        for (int i = 1; i < 8; ++i) {
            const bool fb = (i == 1 || i == 3 || i == 4); /* x^8 = x^4+x^3+x+1 feedback */
            const W u = fb ? xx3<VEC>(ar[i - 1], an[i - 1], d7) : xx3<VEC>(ar[i - 1], an[i - 1], t[i]);
            o[i] = fb ? xx3<VEC>(u, t[i], ar[i]) : (u ^ ar[i]);
        }
    }
}

/* ShiftRows: new byte (r,c) = old byte (r, c+r mod 4). */
OTC_HD void shift_rows(const W *in, W *out)
{
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int i = 0; i < 8; ++i) out[8 * (r + 4 * c) + i] = in[8 * (r + 4 * ((c + r) & 3)) + i];
}

/* 3-input XOR: one v_bitop3_b32 on gfx950 (hipcc does not fuse XOR chains). */
OTC_HD W x3(W a, W b, W c)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#else
    return a ^ b ^ c;
#endif
}

/* MixColumns on a ShiftRows'd state `in`, result into `out`, with the round
 * key folded in: kf(p) returns the 0 / ~0 mask of plane p.  Per column:
 * t = a0^a1^a2^a3, d_r = a_r ^ a_{r+1}, out_r = xtime(d_r) ^ t ^ a_r ^ k. */
template <class KF>
OTC_HD void mix_columns_ark(const W *in, W *out, KF kf)
{
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const W *a0 = in + 32 * c, *a1 = a0 + 8, *a2 = a0 + 16, *a3 = a0 + 24;
        W t[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) t[i] = x3(a0[i], a1[i], a2[i]) ^ a3[i];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const W *ar = in + 32 * c + 8 * r;
            const W *an = in + 32 * c + 8 * ((r + 1) & 3);
            W d[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) d[i] = ar[i] ^ an[i];
            W *o = out + 32 * c + 8 * r;
            const int p = 32 * c + 8 * r;
            /* u_i = t_i ^ a_r,i ^ k_i  (a_r ^ t = a_{r+1} ^ a_{r+2} ^ a_{r+3}) */
            o[0] = x3(d[7], x3(t[0], ar[0], kf(p + 0)), 0);
            o[1] = x3(d[0], d[7], x3(t[1], ar[1], kf(p + 1)));
            o[2] = x3(d[1], t[2], ar[2]) ^ kf(p + 2);
            o[3] = x3(d[2], d[7], x3(t[3], ar[3], kf(p + 3)));
            o[4] = x3(d[3], d[7], x3(t[4], ar[4], kf(p + 4)));
            o[5] = x3(d[4], t[5], ar[5]) ^ kf(p + 5);
            o[6] = x3(d[5], t[6], ar[6]) ^ kf(p + 6);
            o[7] = x3(d[6], t[7], ar[7]) ^ kf(p + 7);
        }
    }
}

} /* namespace otc_bs */
#include "otc_sbox_lut3.h"
static_assert(OTC_SBOX_KEY_TERMS == 11, "kt_ready lists t[0..10]: update its operand list with the S-box header");
#include "otc_mixcol.h"
#include "otc_invmix.h"
namespace otc_bs {

template <bool CTR_CACHE, int R, class KF>
OTC_HD void sbox_byte(W *s, int b, KF &kf)
{
    W *x = s + 8 * b;
    const int p = 8 * b;
    /* which S-boxes see per-lane data under CTR caching:
     * round 0: only byte 15; round 1: bytes 0..3 (column 0) */
    const bool vec = !CTR_CACHE || R >= 2 || (R == 0 && b == 15) || (R == 1 && b < 4);
    if (vec) /* 86-LUT3 mapping of the same circuit (tools/sbox_lut3.py) */
        sbox_lut3(x[0], x[1], x[2], x[3], x[4], x[5], x[6], x[7], kf(R, p), kf(R, p + 1), kf(R, p + 2),
                  kf(R, p + 3), kf(R, p + 4), kf(R, p + 5), kf(R, p + 6), kf(R, p + 7));
    else
        sbox_k<false>(x[0], x[1], x[2], x[3], x[4], x[5], x[6], x[7], kf(R, p), kf(R, p + 1), kf(R, p + 2),
                      kf(R, p + 3), kf(R, p + 4), kf(R, p + 5), kf(R, p + 6), kf(R, p + 7));
    if (vec) pin8(x); /* uniform (SALU) bytes must not be forced into VGPRs */
}

/* One AES round on the planes.  Streaming order per OUTPUT column c:
 * S-box the four bytes that ShiftRows brings into column c, then MixColumns
 * them into a fresh array.  Each input byte feeds exactly one output column,
 * so the live set stays ~128 planes + one column of temporaries (keeps the
 * kernel at 2 waves/SIMD; the textbook SubBytes -> ShiftRows -> MixColumns
 * order keeps old and new state live together). */
template <int R, int NR, bool CTR_CACHE, class KF>
OTC_HD void encrypt_round(W *s, KF &kf)
{
    if constexpr (R + 1 < NR) {
        W ns[128];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            W col[32];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int b = r + 4 * ((c + r) & 3); /* ShiftRows source byte */
                sbox_byte<CTR_CACHE, R>(s, b, kf);
#pragma unroll
                for (int i = 0; i < 8; ++i) col[8 * r + i] = s[8 * b + i];
            }
            if (CTR_CACHE && R == 0)
                mix_column<false>(col, ns + 32 * c);
            else
                mix_column<true>(col, ns + 32 * c);
        }
#pragma unroll
        for (int q = 0; q < 128; ++q) s[q] = ns[q];
        /* explicit compile-time recursion: a `#pragma unroll` loop over rounds
         * exceeds LLVM's pragma-unroll size threshold and is left rolled
         * (dynamic key indexing, spills) */
        encrypt_round<R + 1, NR, CTR_CACHE>(s, kf);
    } else {
#pragma unroll
        for (int b = 0; b < 16; ++b) sbox_byte<CTR_CACHE, R>(s, b, kf);
        W t[128];
        shift_rows(s, t);
#pragma unroll
        for (int q = 0; q < 128; ++q) s[q] = t[q];
    }
}

/* One non-final round as a self-contained step: S-box every byte with the
 * round key folded in, ShiftRows by renaming, MixColumns (MIX 0: the d-form
 * mix_column, 1: the low-register t-form, 2: the searched 55-node circuit
 * mix_column_g), result back in s[] in the canonical layout, in the
 * streaming column order of encrypt_round.
 *
 * The key comes as S-box key TERMS: kt(b, t) fills the OTC_SBOX_KEY_TERMS
 * values of byte b (sbox_key_terms of its 8 plane masks) -- computed from the
 * round key on the fly (KeyMasks) or read from a precomputed table. */
template <int MIX, class KT, int FENCE = 2, bool DEC = false>
OTC_HD void round_step_kt(W *s, KT kt)
{
    W ns[128];
    /* S-box i of the round (streaming order) is byte r + 4((c + r) & 3) with
     * c = i / 4, r = i % 4 (ShiftRows brings it into column c); decryption:
     * r + 4((c - r) & 3) (InvShiftRows) */
    constexpr int SG = DEC ? -1 : 1;
    /* the key terms of the NEXT S-box are loaded (scalar loads) before the
     * current one runs, so their latency hides under its ~83 VALU ops instead
     * of an s_waitcnt lgkmcnt(0) in front of every S-box */
    W tn[OTC_SBOX_KEY_TERMS];
    kt(0, tn);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        W col[32];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int b = r + 4 * ((c + SG * r) & 3);
            W *x = s + 8 * b;
            W t[OTC_SBOX_KEY_TERMS];
#pragma unroll
            for (int j = 0; j < OTC_SBOX_KEY_TERMS; ++j) t[j] = tn[j];
            kt_ready(t);
            const int i = 4 * c + r + 1;
            if (i < 16) kt((i & 3) + 4 * (((i >> 2) + SG * (i & 3)) & 3), tn);
            sched_fence(); /* the loads issue here, not next to their use */
            /* FENCE 3: every LUT output pinned in the low-pressure order of
             * tools/sbox_schedule.py; 2: pin + scheduling barrier per S-box;
             * 1: pin only; 0: the scheduler may interleave S-boxes (more ILP,
             * more registers) */
            sbox_lut3_c<(FENCE >= 3)>(x[0], x[1], x[2], x[3], x[4], x[5], x[6], x[7], t[0], t[1], t[2], t[3], t[4],
                                      t[5], t[6], t[7], t[8], t[9], t[10]);
            if (FENCE >= 1) pin8(x);
            if (FENCE >= 2) sched_fence();
#pragma unroll
            for (int i = 0; i < 8; ++i) col[8 * r + i] = x[i];
        }
        if (DEC)
            inv_mix_column_g(col, ns + 32 * c); /* L o InvMixColumns o L (otc_invmix.h) */
        else if (MIX == 2)
            mix_column_g(col, ns + 32 * c);
        else if (MIX == 1)
            mix_column_t<true>(col, ns + 32 * c);
        else
            mix_column<true>(col, ns + 32 * c);
        if (FENCE >= 2) {
            pin_n(ns + 32 * c, 32);
            sched_fence();
        }
    }
#pragma unroll
    for (int q = 0; q < 128; ++q) s[q] = ns[q];
}

/* Final round: S-box with the key folded in + ShiftRows (the last round key
 * is left to the caller's output XOR, as in encrypt_planes).  Decryption:
 * InvShiftRows, then L on every byte (the post-map of S^-1 = L S L). */
template <class KT, bool DEC = false>
OTC_HD void round_final_kt(W *s, KT kt)
{
    W tn[OTC_SBOX_KEY_TERMS];
    kt(0, tn);
#pragma unroll
    for (int b = 0; b < 16; ++b) {
        W *x = s + 8 * b;
        W t[OTC_SBOX_KEY_TERMS];
#pragma unroll
        for (int j = 0; j < OTC_SBOX_KEY_TERMS; ++j) t[j] = tn[j];
        kt_ready(t);
        if (b + 1 < 16) kt(b + 1, tn);
        sched_fence();
        sbox_lut3_c(x[0], x[1], x[2], x[3], x[4], x[5], x[6], x[7], t[0], t[1], t[2], t[3], t[4], t[5], t[6], t[7],
                    t[8], t[9], t[10]);
        pin8(x);
    }
    W t[128];
    if (DEC) {
        /* new byte (r, c) = L(old byte (r, c - r)) */
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int r = 0; r < 4; ++r) lmap_byte(s + 8 * (r + 4 * ((c - r) & 3)), t + 8 * (r + 4 * c));
    } else {
        shift_rows(s, t);
    }
#pragma unroll
    for (int q = 0; q < 128; ++q) s[q] = t[q];
}

/* Decryption pre-map: L on every byte of the loaded ciphertext planes */
OTC_HD void dec_premap(W *s)
{
#pragma unroll
    for (int b = 0; b < 16; ++b) {
        W t[8];
        lmap_byte(s + 8 * b, t);
#pragma unroll
        for (int i = 0; i < 8; ++i) s[8 * b + i] = t[i];
    }
}

/* Byte value of L = M^-1 (bit i <- bits i+2, i+5, i+7 mod 8) and the
 * S-box input key of decryption round r from the equivalent-inverse-cipher
 * round-key byte k (otc_invmix.h): L(k) ^ 0x05, and ^ L(0x05) = 0x63 after
 * the first round (the constant the previous round's L o InvMixColumns o L
 * leaves behind). */
OTC_HD uint32_t lmap_value(uint32_t v)
{
    uint32_t o = 0;
    for (int i = 0; i < 8; ++i)
        o |= (((v >> ((i + 2) & 7)) ^ (v >> ((i + 5) & 7)) ^ (v >> ((i + 7) & 7))) & 1u) << i;
    return o;
}
OTC_HD uint32_t dec_round_key_byte(uint32_t k, int r) { return lmap_value(k) ^ 0x05u ^ (r > 0 ? 0x63u : 0u); }

/* key terms from a plane-mask functor kf(p) */
template <class KF>
struct KeyMasks {
    KF kf;
    OTC_HD void operator()(int b, W *t) const
    {
        const int p = 8 * b;
        sbox_key_terms(kf(p), kf(p + 1), kf(p + 2), kf(p + 3), kf(p + 4), kf(p + 5), kf(p + 6), kf(p + 7), t);
    }
};

template <int MIX, class KF, int FENCE = 2>
OTC_HD void round_step(W *s, KF kf)
{
    round_step_kt<MIX, KeyMasks<KF>, FENCE>(s, KeyMasks<KF>{kf});
}

template <class KF>
OTC_HD void round_final(W *s, KF kf)
{
    round_final_kt(s, KeyMasks<KF>{kf});
}

/* Precomputed key-term table of a whole key schedule: for round r (0..NR-1,
 * the key folded into that round's S-boxes) and byte b, OTC_BS_KT_STRIDE
 * words at ((r * 16 + b) * OTC_BS_KT_STRIDE): the 11 terms + 1 pad word (so
 * a byte's terms are 3 aligned 16-byte scalar loads). */
#define OTC_BS_KT_STRIDE 12
OTC_HD void key_term_table(const uint32_t *rk, int nr, uint32_t *tab)
{
    for (int r = 0; r < nr; ++r)
        for (int b = 0; b < 16; ++b) {
            const uint32_t byte = (rk[4 * r + (b >> 2)] >> (8 * (b & 3))) & 0xFFu;
            W k[8];
            for (int i = 0; i < 8; ++i) k[i] = ((byte >> i) & 1u) ? ~0u : 0u;
            uint32_t *t = tab + (r * 16 + b) * OTC_BS_KT_STRIDE;
            sbox_key_terms(k[0], k[1], k[2], k[3], k[4], k[5], k[6], k[7], t);
            t[OTC_SBOX_KEY_TERMS] = 0;
        }
}

/* ---- CTR counter caching -----------------------------------------------
 * The bitsliced CTR kernel (csrc/hip/aes_bs.hip) gives each wave ("task") the
 * 2048 counters C + 64k + l (slot k < 32, lane l < 64, C = 0 mod 2048).  So
 * counter byte 15 (bits 0-7) = lane bits 0-5 + slot bits 0-1, byte 14 = slot
 * bits 2-4 + the task's counter bits 11-15 ("u5"), and bytes 0..13 (bits 16+)
 * are a prefix shared by a GROUP of 32 consecutive tasks.  Rounds 1 and 2
 * then leave nothing per lane but table reads:
 *   round 1: only S(byte 15) and S(byte 14) vary; ShiftRows/MixColumns take
 *            them into columns 0 and 1 as (1,1,3,2)*S15 and (1,3,2,1)*S14 on
 *            top of a group constant (c8: ctr_group_consts);
 *   round 2: the S-box outputs of bytes 0..3 ("E0") are then a function of
 *            the group and byte 15 alone: per (group, lane) 4 values per
 *            plane (slot bits 0-1), stored as 32 bytes -- byte 8j+i = that
 *            4-bit pattern of plane i of byte j, doubled to 8 bits -- which
 *            the kernel widens to plane words with one v_perm_b32 each.  Those
 *            of bytes 4..7 ("E1") are a function of the task alone (u5 + slot
 *            bits 2-4): 32 wave-uniform plane words per task, read with scalar
 *            loads.  Bytes 8..15 are group constants;
 *   round 3: input = MixColumns of E0 / E1 (ctr_round2_mix) + a group
 *            constant (round 2's constant bytes through MixColumns, plus rk2)
 *            that becomes the round-3 S-box key: 16 key-term sets per group.
 * Rounds 1-2 thus cost ~190 VALU ops (32 widenings + the MixColumns of the 8
 * varying bytes) instead of 32 S-boxes + 4 MixColumns (round 2 of this
 * scheme computed the 8 varying S-boxes in the kernel, +650 ops per task).
 * Table layout of a call (aes_bs.hip): group terms [ngroups][GRP_WORDS], E0
 * [ngroups][64 lanes][8 words], E1 [tasks][32 words]. */
#define OTC_BS_CTR_GRP_WORDS (16 * OTC_BS_KT_STRIDE)
#define OTC_BS_CTR_E0_WORDS (64 * 8)
#define OTC_BS_CTR_E1_WORDS 32

/* S-box of one byte value through the bitsliced circuit (table-free, so
 * the device precompute and the host tests share it) */
OTC_HD uint32_t sbox_value(uint32_t v)
{
    W x[8];
    for (int i = 0; i < 8; ++i) x[i] = (v >> i) & 1u;
    sbox(x[0], x[1], x[2], x[3], x[4], x[5], x[6], x[7]);
    uint32_t r = 0;
    for (int i = 0; i < 8; ++i) r |= (x[i] & 1u) << i;
    return r;
}
OTC_HD uint32_t xtime_value(uint32_t a) { return ((a << 1) ^ ((a & 0x80u) ? 0x1Bu : 0u)) & 0xFFu; }
/* GF(2^8) product c * a for the MixColumns coefficients c = 1, 2, 3 */
OTC_HD uint32_t gmul123(uint32_t c, uint32_t a) { return c == 1 ? a : c == 2 ? xtime_value(a) : xtime_value(a) ^ a; }

/* MixColumns of one column of byte values a[row] */
OTC_HD void mix_column_bytes(const uint32_t *a, uint32_t *o)
{
    for (int r = 0; r < 4; ++r) {
        const uint32_t a0 = a[r], a1 = a[(r + 1) & 3], a2 = a[(r + 2) & 3], a3 = a[(r + 3) & 3];
        o[r] = xtime_value(a0) ^ xtime_value(a1) ^ a1 ^ a2 ^ a3;
    }
}

/* ShiftRows + MixColumns of 16 byte values (state byte b = row + 4*col) */
OTC_HD void shift_mix_bytes(const uint32_t *in, uint32_t *out)
{
    for (int c = 0; c < 4; ++c) {
        uint32_t col[4];
        for (int r = 0; r < 4; ++r) col[r] = in[r + 4 * ((c + r) & 3)];
        mix_column_bytes(col, out + 4 * c);
    }
}

/* key terms (+ pad word) of one key byte */
OTC_HD void key_terms_of_byte(uint32_t byte, uint32_t *t)
{
    W k[8];
    for (int i = 0; i < 8; ++i) k[i] = ((byte >> i) & 1u) ? ~0u : 0u;
    sbox_key_terms(k[0], k[1], k[2], k[3], k[4], k[5], k[6], k[7], t);
    t[OTC_SBOX_KEY_TERMS] = 0;
}

/* Counter bytes 0..13 of group g: (cbase with bits 0-15 cleared) + g * 2^16,
 * carried into the high word unless the counter wraps at 64 bits. */
OTC_HD void ctr_group_prefix(uint64_t cbase_lo, uint64_t cbase_hi, bool wrap64, uint64_t g, uint8_t *pre)
{
    const uint64_t base = cbase_lo & ~(uint64_t)0xFFFF;
    const uint64_t lo = base + (g << 16);
    const uint64_t hi = cbase_hi + ((!wrap64 && lo < base) ? 1u : 0u);
    for (int b = 0; b < 8; ++b) pre[b] = (uint8_t)(hi >> (8 * (7 - b)));
    for (int b = 0; b < 6; ++b) pre[8 + b] = (uint8_t)(lo >> (8 * (7 - b)));
}

/* Group constants: pre[0..13] = counter bytes 0..13 of the group, rk = the
 * LE round-key words (aes_export_rk32), sb = a byte S-box.  c8[b] (b < 8) =
 * constant part of the round-2 S-box input of byte b (round 1 with S14 =
 * S15 = 0, plus rk1).  terms (if non-null): OTC_BS_CTR_GRP_WORDS words, the
 * key terms of the 16 round-3 bytes. */
template <class SB>
OTC_HD void ctr_group_consts(const uint8_t *pre, const uint32_t *rk, SB sb, uint32_t *c8, uint32_t *terms)
{
    auto rkb = [&](int r, int b) -> uint32_t { return (rk[4 * r + (b >> 2)] >> (8 * (b & 3))) & 0xFFu; };
    uint32_t a[16], B[16];
    for (int b = 0; b < 14; ++b) a[b] = sb(pre[b] ^ rkb(0, b));
    a[14] = a[15] = 0; /* varying */
    shift_mix_bytes(a, B);
    for (int b = 0; b < 8; ++b) c8[b] = B[b] ^ rkb(1, b);
    if (terms) {
        uint32_t d[16], Q[16];
        for (int b = 0; b < 8; ++b) d[b] = 0; /* varying: E0 / E1 */
        for (int b = 8; b < 16; ++b) d[b] = sb(B[b] ^ rkb(1, b));
        shift_mix_bytes(d, Q);
        for (int b = 0; b < 16; ++b) key_terms_of_byte(Q[b] ^ rkb(2, b), terms + b * OTC_BS_KT_STRIDE);
    }
}

/* E0 entry of (group, lane): out[8] words = 32 bytes, byte 8j+i (j < 4) has
 * at bit q (and q + 4) bit i of the round-2 S-box output of byte j for the
 * counter byte 15 = lane + 64q (slot bits 0-1 = q).  k15 = rk0 byte 15. */
template <class SB>
OTC_HD void ctr_e0_lane(const uint32_t *c8, uint32_t k15, uint32_t lane, SB sb, uint32_t *out)
{
    /* built in registers, stored once (out is global memory on the device) */
    const uint32_t cf[4] = {1, 1, 3, 2};
    uint32_t e[4][4];
#pragma unroll
    for (uint32_t q = 0; q < 4; ++q) {
        const uint32_t s15 = sb((lane | (q << 6)) ^ k15);
#pragma unroll
        for (int j = 0; j < 4; ++j) e[q][j] = sb(c8[j] ^ gmul123(cf[j], s15));
    }
#pragma unroll
    for (int w = 0; w < 8; ++w) {
        uint32_t v = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int p = 4 * w + b, j = p >> 3, i = p & 7;
            uint32_t nib = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) nib |= ((e[q][j] >> i) & 1u) << q;
            v |= (nib | (nib << 4)) << (8 * b);
        }
        out[w] = v;
    }
}

/* E1 entry of a task with counter bits 11-15 = u5: out[32] plane words, bit k
 * of word 8j+i = bit i of the round-2 S-box output of byte 4+j for counter
 * byte 14 = (k >> 2) | u5 << 3.  k14 = rk0 byte 14. */
template <class SB>
OTC_HD void ctr_e1_task(const uint32_t *c8, uint32_t k14, uint32_t u5, SB sb, uint32_t *out)
{
    /* built in registers, stored once (out is global memory on the device) */
    const uint32_t cf[4] = {1, 3, 2, 1};
    uint32_t e[8][4];
#pragma unroll
    for (uint32_t w = 0; w < 8; ++w) {
        const uint32_t s14 = sb((w | (u5 << 3)) ^ k14);
#pragma unroll
        for (int j = 0; j < 4; ++j) e[w][j] = sb(c8[4 + j] ^ gmul123(cf[j], s14));
    }
#pragma unroll
    for (int p = 0; p < 32; ++p) {
        uint32_t v = 0;
#pragma unroll
        for (uint32_t w = 0; w < 8; ++w) v |= ((e[w][p >> 3] >> (p & 7)) & 1u) * (0xFu << (4 * w));
        out[p] = v;
    }
}

/* plane word of E0 byte p: byte p & 3 of word x replicated (one v_perm_b32) */
OTC_HD W rep_byte(W x, int b)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_perm(x, x, 0x01010101u * (uint32_t)b);
#else
    return ((x >> (8 * b)) & 0xFFu) * 0x01010101u;
#endif
}

/* xtime on 8 planes */
OTC_HD void xt8(const W *a, W *o)
{
    o[0] = a[7];
    o[1] = a[0] ^ a[7];
    o[2] = a[1];
    o[3] = a[2] ^ a[7];
    o[4] = a[3] ^ a[7];
    o[5] = a[4];
    o[6] = a[5];
    o[7] = a[6];
}

/* MixColumns of a column whose only non-zero rows are i (a) and j (b):
 * out_r = M[r][i] a ^ M[r][j] b, M[r][j] = (2,3,1,1)[(j - r) mod 4]; one
 * 3-input XOR per output plane for the row pairs that occur here. */
OTC_HD void mix_column2(const W *a, int i, const W *b, int j, W *out)
{
    W a2[8], b2[8];
    xt8(a, a2);
    xt8(b, b2);
    const int cf[4] = {2, 3, 1, 1};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int ca = cf[(i - r) & 3], cb = cf[(j - r) & 3];
#pragma unroll
        for (int p = 0; p < 8; ++p) {
            W v;
            if (ca == 3 && cb == 3)
                v = x3(a[p], a2[p], b[p]) ^ b2[p];
            else if (ca == 3)
                v = x3(a[p], a2[p], cb == 1 ? b[p] : b2[p]);
            else if (cb == 3)
                v = x3(b[p], b2[p], ca == 1 ? a[p] : a2[p]);
            else
                v = (ca == 1 ? a[p] : a2[p]) ^ (cb == 1 ? b[p] : b2[p]);
            out[8 * r + p] = v;
        }
    }
}

/* Round 2's ShiftRows + MixColumns on its 8 varying S-box outputs: e0[32] =
 * planes of bytes 0..3, e1[32] = bytes 4..7.  Result in s[128]: the round-3
 * S-box input WITHOUT its key (the group's round-3 terms carry that).  The
 * varying bytes land at col0 rows 0,1 (bytes 0,5), col1 rows 0,3 (4,3), col2
 * rows 2,3 (2,7), col3 rows 1,2 (1,6). */
OTC_HD void ctr_round2_mix(const W *e0, const W *e1, W *s)
{
    mix_column2(e0 + 0, 0, e1 + 8, 1, s);
    mix_column2(e1 + 0, 0, e0 + 24, 3, s + 32);
    mix_column2(e0 + 16, 2, e1 + 24, 3, s + 64);
    mix_column2(e0 + 8, 1, e1 + 16, 2, s + 96);
}

/* Rounds 1..NR of AES on bitsliced planes s[128] (AddRoundKey r folded into
 * the S-box of round r+1; the LAST round key is NOT applied -- callers fold it
 * into their output XOR).  kf(r, p) returns the mask of plane p of round key r.
 * CTR_CACHE: the caller guarantees bytes 0..14 of the input are wave-uniform
 * (counter-mode caching) so rounds 1 and 2 evaluate their uniform S-boxes and
 * columns with plain C ops that hipcc keeps on the scalar ALU. */
template <int NR, bool CTR_CACHE, class KF>
OTC_HD void encrypt_planes(W *s, KF kf)
{
    encrypt_round<0, NR, CTR_CACHE>(s, kf);
}

/* Expand one 16-byte round key (4 LE words, as produced by aes_export_rk32)
 * into 128 plane masks. */
OTC_HD void key_masks(const uint32_t *rk4, W *k)
{
#pragma unroll
    for (int b = 0; b < 16; ++b) {
        uint32_t byte = (rk4[b >> 2] >> (8 * (b & 3))) & 0xffu;
#pragma unroll
        for (int i = 0; i < 8; ++i) k[8 * b + i] = ((byte >> i) & 1u) ? ~0u : 0u;
    }
}

/* Full-round helper for host tests: s <- MixColumns(ShiftRows(SubBytes(s))) ^ k */
struct ArrayKey {
    const W *k;
    OTC_HD W operator()(int p) const { return k[p]; }
};

OTC_HD void round_full(W *s, const W *k)
{
    W t[128];
    sub_bytes(s);
    shift_rows(s, t);
    mix_columns_ark(t, s, ArrayKey{k});
}

OTC_HD void round_last(W *s, const W *k)
{
    W t[128];
    sub_bytes(s);
    shift_rows(s, t);
#pragma unroll
    for (int p = 0; p < 128; ++p) s[p] = t[p] ^ k[p];
}

/* Transpose 32 blocks (blk[k][0..3] = 4 LE words of block slot k) into planes,
 * and back.  Plane 8*b+i, bit k  <->  block k, byte b, bit i, i.e. word
 * w = b/4, bit 8*(b%4)+i of blk[k][w].  Each word-column w is an independent
 * 32x32 bit-matrix transpose. */
/* v_perm_b32 (byte select from {hi, lo}; selector bytes 0-3 = lo, 4-7 = hi),
 * emulated on the host. */
OTC_HD W perm_b(W hi, W lo, uint32_t sel)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_perm(hi, lo, sel);
#else
    W r = 0;
    for (int i = 0; i < 4; ++i) {
        const uint32_t s = (sel >> (8 * i)) & 0xFFu;
        const W byte = s < 4 ? (lo >> (8 * s)) & 0xFFu : (hi >> (8 * (s - 4))) & 0xFFu;
        r |= byte << (8 * i);
    }
    return r;
#endif
}

/* bit select: m ? x : y  (v_bfi_b32 / v_bitop3_b32) */
OTC_HD W bsel(W m, W x, W y) { return (x & m) | (y & ~m); }

/* one bit-level block-swap stage of transpose32 (J = 4, 2, 1; a template so
 * the stage is fully unrolled -- a rolled loop puts m[] in scratch).  The
 * selects compile to v_bfi_b32.  Measured alternatives (profiles/r3/
 * round2_tables): the selects as v_bitop3_b32 -- which issue at ~0.65x the
 * cost of v_bfi_b32 in tools/ubench/valu_ops.hip -- ran at the same speed
 * (the kernel is power-, not issue-bound); two pairs per 64-bit shift made
 * hipcc add a v_mov_b64 per shift (the operands are never in adjacent VGPRs)
 * and spill. */
template <int J>
OTC_HD void transpose_bits(W *m, W mk)
{
#pragma unroll
    for (int k = 0; k < 32; ++k) {
        if (k & J) continue;
        const W a = m[k], b = m[k | J];
        m[k] = bsel(mk << J, b << J, a);
        m[k | J] = bsel(mk, a >> J, b);
    }
}

OTC_HD void transpose32(W *m)
{
    /* in-place 32x32 transpose: m[r] bit c  ->  m[c] bit r.  Classic 5-stage
     * block swap; the 16- and 8-bit stages only move bytes, so each output
     * word is one v_perm_b32 (2 ops per pair instead of 5); the 4/2/1-bit
     * stages are a shift and a bit select per word (transpose_bits). */
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const W a = m[k], b = m[k | 16];
        m[k] = perm_b(b, a, 0x05040100u);      /* [b1 b0 a1 a0] */
        m[k | 16] = perm_b(b, a, 0x07060302u); /* [b3 b2 a3 a2] */
    }
#pragma unroll
    for (int k = 0; k < 32; ++k) {
        if (k & 8) continue;
        const W a = m[k], b = m[k | 8];
        m[k] = perm_b(b, a, 0x06020400u);     /* [b2 a2 b0 a0] */
        m[k | 8] = perm_b(b, a, 0x07030501u); /* [b3 a3 b1 a1] */
    }
    transpose_bits<4>(m, 0x0F0F0F0Fu);
    transpose_bits<2>(m, 0x33333333u);
    transpose_bits<1>(m, 0x55555555u);
}

/* Reference transpose (host tests). */
inline void transpose32_ref(W *m)
{
    W t[32] = {0};
    for (int r = 0; r < 32; ++r)
        for (int c = 0; c < 32; ++c) t[c] |= ((m[r] >> c) & 1u) << r;
    for (int i = 0; i < 32; ++i) m[i] = t[i];
}

} /* namespace otc_bs */

#endif
