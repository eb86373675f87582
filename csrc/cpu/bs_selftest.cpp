/*
 * bs_selftest.cpp -- host-side validation of the bitsliced AES core
 * (include/otc_bitslice.h) against the table oracle (cpu/aes.c): exhaustive
 * S-box check plus full AES-128/192/256 encryption of 32 random blocks.
 * Exported as otc_bitslice_selftest() so both the C test binary and pytest
 * can call it without a GPU.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "aes.h"
#include "otc_bitslice.h"

using namespace otc_bs;

extern "C" int otc_bitslice_selftest(int verbose)
{
    const uint8_t *SB = aes_sbox();
    int fails = 0;
    /* S-box: 256 inputs as 8 batches of 32 slots */
    for (int batch = 0; batch < 8; ++batch) {
        W x[8] = {0};
        for (int k = 0; k < 32; ++k) {
            int v = batch * 32 + k;
            for (int i = 0; i < 8; ++i) x[i] |= (W)((v >> i) & 1) << k;
        }
        sbox(x[0], x[1], x[2], x[3], x[4], x[5], x[6], x[7]);
        for (int k = 0; k < 32; ++k) {
            int v = batch * 32 + k, o = 0;
            for (int i = 0; i < 8; ++i) o |= (int)((x[i] >> k) & 1) << i;
            if (o != SB[v]) {
                if (verbose) printf("  sbox mismatch at %02x: %02x vs %02x\n", v, o, SB[v]);
                ++fails;
            }
        }
    }
    /* key-folded S-box: sbox_k(x, k) == sbox(x ^ k) */
    for (int kv = 0; kv < 256; kv += 37) {
        W k[8], x[8] = {0}, y[8];
        for (int i = 0; i < 8; ++i) k[i] = ((kv >> i) & 1) ? ~0u : 0u;
        for (int slot = 0; slot < 32; ++slot)
            for (int i = 0; i < 8; ++i) x[i] |= (W)(((slot * 7 + kv) >> i) & 1) << slot;
        for (int i = 0; i < 8; ++i) y[i] = x[i] ^ k[i];
        sbox(y[0], y[1], y[2], y[3], y[4], y[5], y[6], y[7]);
        W z[8];
        for (int i = 0; i < 8; ++i) z[i] = x[i];
        sbox_k<false>(x[0], x[1], x[2], x[3], x[4], x[5], x[6], x[7], k[0], k[1], k[2], k[3], k[4], k[5], k[6], k[7]);
        sbox_lut3(z[0], z[1], z[2], z[3], z[4], z[5], z[6], z[7], k[0], k[1], k[2], k[3], k[4], k[5], k[6], k[7]);
        for (int i = 0; i < 8; ++i)
            if (x[i] != y[i] || z[i] != y[i]) {
                if (verbose) printf("  sbox_k/sbox_lut3 mismatch kv=%d bit %d\n", kv, i);
                ++fails;
            }
    }
    /* transpose32 (perm / bit-select stages) vs the bit-by-bit reference */
    for (int t = 0; t < 64; ++t) {
        W a[32], b[32];
        uint64_t z = 0x9E3779B97F4A7C15ull * (uint64_t)(t + 1);
        for (int i = 0; i < 32; ++i) {
            z ^= z << 13; z ^= z >> 7; z ^= z << 17;
            a[i] = b[i] = (W)(z >> 11);
        }
        transpose32(a);
        transpose32_ref(b);
        for (int i = 0; i < 32; ++i)
            if (a[i] != b[i]) {
                if (verbose) printf("  transpose32 mismatch (trial %d, word %d)\n", t, i);
                ++fails;
                break;
            }
    }
    /* full cipher */
    srand(7);
    for (int bits = 128; bits <= 256; bits += 64) {
        unsigned char key[32], pt[32][16], ref[32][16];
        for (int i = 0; i < 32; ++i) key[i] = (unsigned char)rand();
        for (int k = 0; k < 32; ++k)
            for (int i = 0; i < 16; ++i) pt[k][i] = (unsigned char)rand();
        aes_context ctx;
        aes_setkey_enc(&ctx, key, (unsigned)bits);
        for (int k = 0; k < 32; ++k) aes_crypt_ecb(&ctx, AES_ENCRYPT, pt[k], ref[k]);
        uint32_t rk[60];
        aes_export_rk32(&ctx, rk);
        W s[128];
        for (int w = 0; w < 4; ++w) {
            W m[32];
            for (int k = 0; k < 32; ++k) memcpy(&m[k], &pt[k][4 * w], 4);
            transpose32(m);
            for (int q = 0; q < 32; ++q) s[32 * w + q] = m[q];
        }
        W km[128];
        key_masks(rk, km);
        for (int p = 0; p < 128; ++p) s[p] ^= km[p];
        for (int r = 1; r < ctx.nr; ++r) {
            key_masks(rk + 4 * r, km);
            round_full(s, km);
        }
        key_masks(rk + 4 * ctx.nr, km);
        round_last(s, km);
        int bad = 0;
        for (int w = 0; w < 4; ++w) {
            W m[32];
            for (int q = 0; q < 32; ++q) m[q] = s[32 * w + q];
            transpose32(m);
            for (int k = 0; k < 32; ++k) bad += memcmp(&m[k], &ref[k][4 * w], 4) != 0;
        }
        if (verbose) printf("  bitsliced AES-%d (32 blocks): %s\n", bits, bad ? "failed" : "passed");
        fails += bad;

        /* kernel round structure (encrypt_planes, key folded into S-boxes) */
        for (int w = 0; w < 4; ++w) {
            W m[32];
            for (int k = 0; k < 32; ++k) memcpy(&m[k], &pt[k][4 * w], 4);
            transpose32(m);
            for (int q = 0; q < 32; ++q) s[32 * w + q] = m[q];
        }
        auto kf = [&](int r, int p) -> W { return (W)(0u - ((rk[4 * r + (p >> 5)] >> (p & 31)) & 1u)); };
        if (ctx.nr == 10) encrypt_planes<10, false>(s, kf);
        else if (ctx.nr == 12) encrypt_planes<12, false>(s, kf);
        else encrypt_planes<14, false>(s, kf);
        bad = 0;
        for (int w = 0; w < 4; ++w) {
            W m[32];
            for (int q = 0; q < 32; ++q) m[q] = s[32 * w + q];
            transpose32(m);
            for (int k = 0; k < 32; ++k) {
                uint32_t v = m[k] ^ rk[4 * ctx.nr + w];
                bad += memcmp(&v, &ref[k][4 * w], 4) != 0;
            }
        }
        if (verbose) printf("  bitsliced AES-%d kernel schedule: %s\n", bits, bad ? "failed" : "passed");
        fails += bad;

        /* rolled-loop round structure (round_step / round_final), all three
         * MixColumns forms */
        for (int mixt = 0; mixt < 3; ++mixt) {
            for (int w = 0; w < 4; ++w) {
                W m[32];
                for (int k = 0; k < 32; ++k) memcpy(&m[k], &pt[k][4 * w], 4);
                transpose32(m);
                for (int q = 0; q < 32; ++q) s[32 * w + q] = m[q];
            }
            for (int r = 0; r + 1 < ctx.nr; ++r) {
                auto kr = [&](int p) -> W { return kf(r, p); };
                if (mixt == 2) round_step<2>(s, kr);
                else if (mixt == 1) round_step<1>(s, kr);
                else round_step<0>(s, kr);
            }
            round_final(s, [&](int p) -> W { return kf(ctx.nr - 1, p); });
            bad = 0;
            for (int w = 0; w < 4; ++w) {
                W m[32];
                for (int q = 0; q < 32; ++q) m[q] = s[32 * w + q];
                transpose32(m);
                for (int k = 0; k < 32; ++k) {
                    uint32_t v = m[k] ^ rk[4 * ctx.nr + w];
                    bad += memcmp(&v, &ref[k][4 * w], 4) != 0;
                }
            }
            if (verbose)
                printf("  bitsliced AES-%d rolled rounds%s: %s\n", bits,
                       mixt == 2 ? " (searched 55-node MixColumns)" : mixt ? " (low-register MixColumns)" : "",
                       bad ? "failed" : "passed");
            fails += bad;
        }

        /* rounds reading the precomputed key-term table (the GPU kernel's
         * scalar-load key path) */
        {
            static uint32_t tab[14 * 16 * OTC_BS_KT_STRIDE];
            key_term_table(rk, ctx.nr, tab);
            for (int w = 0; w < 4; ++w) {
                W m[32];
                for (int k = 0; k < 32; ++k) memcpy(&m[k], &pt[k][4 * w], 4);
                transpose32(m);
                for (int q = 0; q < 32; ++q) s[32 * w + q] = m[q];
            }
            for (int r = 0; r + 1 < ctx.nr; ++r)
                round_step_kt<true>(s, [&](int b, W *t) {
                    for (int j = 0; j < OTC_SBOX_KEY_TERMS; ++j) t[j] = tab[(r * 16 + b) * OTC_BS_KT_STRIDE + j];
                });
            round_final_kt(s, [&](int b, W *t) {
                for (int j = 0; j < OTC_SBOX_KEY_TERMS; ++j) t[j] = tab[((ctx.nr - 1) * 16 + b) * OTC_BS_KT_STRIDE + j];
            });
            bad = 0;
            for (int w = 0; w < 4; ++w) {
                W m[32];
                for (int q = 0; q < 32; ++q) m[q] = s[32 * w + q];
                transpose32(m);
                for (int k = 0; k < 32; ++k) {
                    uint32_t v = m[k] ^ rk[4 * ctx.nr + w];
                    bad += memcmp(&v, &ref[k][4 * w], 4) != 0;
                }
            }
            if (verbose) printf("  bitsliced AES-%d key-term table rounds: %s\n", bits, bad ? "failed" : "passed");
            fails += bad;

            /* counter-cached CTR task (the GPU kernel's default CTR path):
             * round-3 key terms per group, E0 per (group, lane), E1 per task,
             * rounds 4.. from the table, for a few lanes of tasks with
             * different u5 / groups */
            bad = 0;
            for (int trial = 0; trial < 4; ++trial) {
                uint64_t hi = ((uint64_t)rand() << 32) ^ (uint64_t)rand();
                uint64_t lo = (((uint64_t)rand() << 32) ^ (uint64_t)rand()) & ~(uint64_t)2047u;
                if (trial == 3) lo = ~(uint64_t)0 << 11; /* all-ones bytes, u5 = 31 */
                const uint32_t u5 = (uint32_t)(lo >> 11) & 31u;
                uint8_t ctr[16];
                for (int b = 0; b < 8; ++b) ctr[b] = (uint8_t)(hi >> (8 * (7 - b)));
                for (int b = 0; b < 8; ++b) ctr[8 + b] = (uint8_t)(lo >> (8 * (7 - b)));
                /* the group prefix as the table kernel derives it (group 0 of
                 * a call whose cbase is this counter) */
                uint8_t pre[14];
                ctr_group_prefix(lo, hi, false, 0, pre);
                bad += memcmp(pre, ctr, 14) != 0;
                static uint32_t grp[OTC_BS_CTR_GRP_WORDS];
                uint32_t c8[8], e1w[OTC_BS_CTR_E1_WORDS];
                ctr_group_consts(pre, rk, sbox_value, c8, grp);
                const uint32_t k14 = (rk[3] >> 16) & 0xFFu, k15 = rk[3] >> 24;
                ctr_e1_task(c8, k14, u5, sbox_value, e1w);
                for (int lane = 0; lane < 64; lane += 21) {
                    uint32_t ent[8];
                    ctr_e0_lane(c8, k15, (uint32_t)lane, sbox_value, ent);
                    W e0[32], e1[32];
                    for (int p = 0; p < 32; ++p) {
                        e0[p] = rep_byte(ent[p >> 2], p & 3);
                        e1[p] = e1w[p];
                    }
                    ctr_round2_mix(e0, e1, s);
                    round_step_kt<true>(s, [&](int b, W *t) {
                        for (int j = 0; j < OTC_SBOX_KEY_TERMS; ++j) t[j] = grp[b * OTC_BS_KT_STRIDE + j];
                    });
                    for (int r = 3; r + 1 < ctx.nr; ++r)
                        round_step_kt<true>(s, [&](int b, W *t) {
                            for (int j = 0; j < OTC_SBOX_KEY_TERMS; ++j) t[j] = tab[(r * 16 + b) * OTC_BS_KT_STRIDE + j];
                        });
                    round_final_kt(s, [&](int b, W *t) {
                        for (int j = 0; j < OTC_SBOX_KEY_TERMS; ++j)
                            t[j] = tab[((ctx.nr - 1) * 16 + b) * OTC_BS_KT_STRIDE + j];
                    });
                    for (int w = 0; w < 4; ++w) {
                        W m[32];
                        for (int q = 0; q < 32; ++q) m[q] = s[32 * w + q];
                        transpose32(m);
                        for (int k = 0; k < 32; ++k) {
                            /* block (lane, slot k) encrypts counter C + 64k + lane */
                            uint8_t cb[16], ks[16];
                            memcpy(cb, ctr, 16);
                            const uint32_t add = 64u * (uint32_t)k + (uint32_t)lane; /* < 2048: bytes 14-15 */
                            cb[15] = (uint8_t)add;
                            cb[14] = (uint8_t)((u5 << 3) | (add >> 8));
                            aes_crypt_ecb(&ctx, AES_ENCRYPT, cb, ks);
                            uint32_t v = m[k] ^ rk[4 * ctx.nr + w];
                            bad += memcmp(&v, &ks[4 * w], 4) != 0;
                        }
                    }
                }
            }
            if (verbose) printf("  bitsliced AES-%d counter-cached CTR task: %s\n", bits, bad ? "failed" : "passed");
            fails += bad;
        }
    }
    return fails ? 1 : 0;
}
