/*
 * otc_bs8.h -- row-sliced AES: 8 blocks per lane in 32 planes, the VALU
 * kernel of the serial-chain segment modes (CBC / CFB128 encryption of
 * independent sectors, csrc/hip/aes_bs8.hip).  Shared with the host test
 * (csrc/cpu/bs_selftest.cpp, otc_bs8_selftest).
 *
 * Why a second slicing.  The 32-block-per-lane bitslice (otc_bitslice.h)
 * needs 2048 independent inputs per wave; a chained mode has one block per
 * chain in flight, so it would carry 2048 chains (sectors) per wave -- a
 * quarter GiB of live cache lines across the chip and multi-millisecond
 * tasks.  Here a lane holds 8 chains, 512 per wave:
 *
 *   plane s[8r + b]  (row r = 0..3, bit b = 0..7) is a 32-bit word whose
 *   byte c (column c = 0..3) holds, in bit k, bit b of state byte (r, c) of
 *   chain k (k = 0..7).
 *
 * That is exactly what transpose32 (otc_bitslice.h) makes of the 32 words
 * m[8c + k] = word c of chain k's block: word-to-plane and back are the same
 * 256-op transpose.  In this layout
 *   - SubBytes is the same 77-LUT3 circuit on the 8 planes of a row (32
 *     bytes at a time: 4 S-boxes per round for 8 blocks, 38.5 LUTs a block,
 *     as the wide layout), with the round key folded into its input: the key
 *     planes are per-column byte masks, still wave-uniform (SGPR operands);
 *   - ShiftRows rotates row r's planes by r bytes: one v_perm_b32 per plane,
 *     24 per round;
 *   - MixColumns combines the four rows byte for byte: the wide layout's
 *     55-node column circuit (otc_mixcol.h) on the 32 planes does all four
 *     columns of all 8 blocks at once.
 * Per round and 8 blocks: 308 + 24 + 55 = 387 VALU, 48.4 a block (the wide
 * layout: ~45 plus its transposes).  No reference counterpart: the reference
 * runs these chains one block at a time on the CPU
 * (/root/reference/aes-modes/aes.c:801-812 CBC, :822-862 CFB128).
 */
#ifndef OTC_BS8_H
#define OTC_BS8_H

#include "otc_bitslice.h" /* also the 77-LUT S-box and the 55-node MixColumns column */

namespace otc_bs8 {

using otc_bs::W;

/* row r's rotation: new byte c = old byte (c + r) mod 4 */
OTC_HD W rot_row(W x, int r)
{
    return otc_bs::perm_b(x, x, r == 1 ? 0x00030201u : r == 2 ? 0x01000302u : 0x02010003u);
}

/* key planes of round key j, row r (byte c = key byte (r, c) spread to a
 * mask per bit) -> the S-box's 11 key terms.  chain: round 0 takes
 * k_0 ^ k_NR (the chained kernels carry the state without the last round key,
 * see aes_bs8.hip). */
OTC_HD void key_terms(const uint32_t *rk, int nr, int j, int r, bool chain, W *t)
{
    W k[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int c = 0; c < 4; ++c) {
        uint32_t kb = (rk[4 * j + c] >> (8 * r)) & 0xFFu;
        if (chain && j == 0) kb ^= (rk[4 * nr + c] >> (8 * r)) & 0xFFu;
        for (int i = 0; i < 8; ++i)
            if ((kb >> i) & 1u) k[i] |= 0xFFu << (8 * c);
    }
    otc_bs::sbox_key_terms(k[0], k[1], k[2], k[3], k[4], k[5], k[6], k[7], t);
}

/* Round j of NR on the 32 planes: SubBytes with round key j folded in,
 * ShiftRows, MixColumns (not in the last round; the last round key is left
 * to the caller).  kt(j, r, t) gives the key terms of (round j, row r); the
 * terms of the next S-box are fetched before the current one runs (scalar
 * loads on the device: their latency hides under ~77 LUTs). */
template <int J, int NR, class KT>
OTC_HD void round_j(W *s, KT kt, W *tn)
{
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        W t[OTC_SBOX_KEY_TERMS];
#pragma unroll
        for (int q = 0; q < OTC_SBOX_KEY_TERMS; ++q) t[q] = tn[q];
        otc_bs::kt_ready(t);
        if (r < 3) kt(J, r + 1, tn);
        else if (J + 1 < NR) kt(J + 1, 0, tn);
        otc_bs::sched_fence();
        W *x = s + 8 * r;
        otc_bs::sbox_lut3_c(x[0], x[1], x[2], x[3], x[4], x[5], x[6], x[7], t[0], t[1], t[2], t[3], t[4], t[5],
                            t[6], t[7], t[8], t[9], t[10]);
        otc_bs::pin8(x);
        otc_bs::sched_fence();
    }
#pragma unroll
    for (int r = 1; r < 4; ++r)
#pragma unroll
        for (int b = 0; b < 8; ++b) s[8 * r + b] = rot_row(s[8 * r + b], r);
    if (J + 1 < NR) {
        W ns[32];
        otc_bs::mix_column_g(s, ns);
        otc_bs::pin_n(ns, 32);
        otc_bs::sched_fence();
#pragma unroll
        for (int q = 0; q < 32; ++q) s[q] = ns[q];
    }
}

template <int J, int NR, class KT>
OTC_HD void rounds_from(W *s, KT kt, W *tn)
{
    if constexpr (J < NR) {
        round_j<J, NR, KT>(s, kt, tn);
        rounds_from<J + 1, NR, KT>(s, kt, tn);
    }
}

/* all NR rounds (the last round key NOT added) */
template <int NR, class KT>
OTC_HD void rounds(W *s, KT kt)
{
    W tn[OTC_SBOX_KEY_TERMS];
    kt(0, 0, tn);
    rounds_from<0, NR, KT>(s, kt, tn);
}

/* key terms computed on the fly (host tests) */
struct HostKT {
    const uint32_t *rk;
    int nr;
    OTC_HD void operator()(int j, int r, W *t) const { key_terms(rk, nr, j, r, true, t); }
};

} /* namespace otc_bs8 */

#endif
