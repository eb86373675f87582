/*
 * aesni.c -- AES-NI CPU baseline (see include/aesni.h).  Behavioural parity
 * with /root/reference/aes-modes/aesni.c:7-152; new implementation.
 */
#include "aesni.h"

#include <cpuid.h>
#include <immintrin.h>
#include <string.h>

int CheckAESSupport(void)
{
    unsigned a, b, c, d;
    if (!__get_cpuid(1, &a, &b, &c, &d)) return 0;
    return (c & bit_AES) ? 1 : 0;
}

#define KEYGEN(k, rc) _mm_aeskeygenassist_si128((k), (rc))

static inline __m128i fold(__m128i k)
{
    k = _mm_xor_si128(k, _mm_slli_si128(k, 4));
    k = _mm_xor_si128(k, _mm_slli_si128(k, 4));
    return _mm_xor_si128(k, _mm_slli_si128(k, 4));
}

void AES_128_Key_Expansion(const unsigned char *userkey, unsigned char *key)
{
    __m128i *rk = (__m128i *)key;
    __m128i k = _mm_loadu_si128((const __m128i *)userkey);
    _mm_storeu_si128(rk, k);
#define STEP128(i, rc)                                                   \
    k = _mm_xor_si128(fold(k), _mm_shuffle_epi32(KEYGEN(k, rc), 0xff)); \
    _mm_storeu_si128(rk + (i), k);
    STEP128(1, 0x01) STEP128(2, 0x02) STEP128(3, 0x04) STEP128(4, 0x08) STEP128(5, 0x10)
    STEP128(6, 0x20) STEP128(7, 0x40) STEP128(8, 0x80) STEP128(9, 0x1b) STEP128(10, 0x36)
#undef STEP128
}

/* 192/256-bit expansion done word-wise through the generic recurrence using
 * aeskeygenassist for SubWord/RotWord; stored as 16-byte round keys. */
static void expand_words(const unsigned char *userkey, unsigned char *key, int nk, int nr)
{
    unsigned w[60];
    memcpy(w, userkey, (size_t)nk * 4);
    unsigned rcon = 1;
    for (int i = nk; i < 4 * (nr + 1); ++i) {
        unsigned t = w[i - 1];
        if (i % nk == 0) {
            __m128i v = _mm_cvtsi32_si128((int)t);
            /* dword 1 of aeskeygenassist = RotWord(SubWord(X1)) ^ rcon, X1 = dword1 */
            v = _mm_shuffle_epi32(v, 0x00);
            t = (unsigned)_mm_extract_epi32(_mm_aeskeygenassist_si128(v, 0), 1) ^ rcon;
            rcon = (rcon << 1) ^ ((rcon & 0x80) ? 0x11b : 0);
        } else if (nk > 6 && i % nk == 4) {
            __m128i v = _mm_shuffle_epi32(_mm_cvtsi32_si128((int)t), 0x00);
            t = (unsigned)_mm_extract_epi32(_mm_aeskeygenassist_si128(v, 0), 0);
        }
        w[i] = w[i - nk] ^ t;
    }
    memcpy(key, w, (size_t)(4 * (nr + 1)) * 4);
}

void AES_192_Key_Expansion(const unsigned char *userkey, unsigned char *key) { expand_words(userkey, key, 6, 12); }
void AES_256_Key_Expansion(const unsigned char *userkey, unsigned char *key) { expand_words(userkey, key, 8, 14); }

void AES_Key_Expansion_Dec(const unsigned char *enc_key, unsigned char *dec_key, int nr)
{
    const __m128i *e = (const __m128i *)enc_key;
    __m128i *d = (__m128i *)dec_key;
    _mm_storeu_si128(d, _mm_loadu_si128(e + nr));
    for (int i = 1; i < nr; ++i) _mm_storeu_si128(d + i, _mm_aesimc_si128(_mm_loadu_si128(e + nr - i)));
    _mm_storeu_si128(d + nr, _mm_loadu_si128(e));
}

static inline __m128i enc1(__m128i b, const __m128i *rk, int nr)
{
    b = _mm_xor_si128(b, _mm_loadu_si128(rk));
    for (int j = 1; j < nr; ++j) b = _mm_aesenc_si128(b, _mm_loadu_si128(rk + j));
    return _mm_aesenclast_si128(b, _mm_loadu_si128(rk + nr));
}

void AES_ECB_encrypt(const unsigned char *in, unsigned char *out, unsigned long length,
                     const unsigned char *key, int nr)
{
    const __m128i *rk = (const __m128i *)key;
    unsigned long nb = length / 16, i = 0;
    for (; i + 4 <= nb; i += 4) { /* 4-way interleave to fill the AES pipe */
        __m128i b0 = _mm_loadu_si128((const __m128i *)in + i), b1 = _mm_loadu_si128((const __m128i *)in + i + 1);
        __m128i b2 = _mm_loadu_si128((const __m128i *)in + i + 2), b3 = _mm_loadu_si128((const __m128i *)in + i + 3);
        __m128i k = _mm_loadu_si128(rk);
        b0 = _mm_xor_si128(b0, k); b1 = _mm_xor_si128(b1, k); b2 = _mm_xor_si128(b2, k); b3 = _mm_xor_si128(b3, k);
        for (int j = 1; j < nr; ++j) {
            k = _mm_loadu_si128(rk + j);
            b0 = _mm_aesenc_si128(b0, k); b1 = _mm_aesenc_si128(b1, k); b2 = _mm_aesenc_si128(b2, k); b3 = _mm_aesenc_si128(b3, k);
        }
        k = _mm_loadu_si128(rk + nr);
        _mm_storeu_si128((__m128i *)out + i, _mm_aesenclast_si128(b0, k));
        _mm_storeu_si128((__m128i *)out + i + 1, _mm_aesenclast_si128(b1, k));
        _mm_storeu_si128((__m128i *)out + i + 2, _mm_aesenclast_si128(b2, k));
        _mm_storeu_si128((__m128i *)out + i + 3, _mm_aesenclast_si128(b3, k));
    }
    for (; i < nb; ++i) _mm_storeu_si128((__m128i *)out + i, enc1(_mm_loadu_si128((const __m128i *)in + i), rk, nr));
}

void AES_ECB_decrypt(const unsigned char *in, unsigned char *out, unsigned long length,
                     const char *key, int nr)
{
    const __m128i *rk = (const __m128i *)key;
    for (unsigned long i = 0; i < length / 16; ++i) {
        __m128i b = _mm_xor_si128(_mm_loadu_si128((const __m128i *)in + i), _mm_loadu_si128(rk));
        for (int j = 1; j < nr; ++j) b = _mm_aesdec_si128(b, _mm_loadu_si128(rk + j));
        _mm_storeu_si128((__m128i *)out + i, _mm_aesdeclast_si128(b, _mm_loadu_si128(rk + nr)));
    }
}

void AES_CTR_encrypt_at(const unsigned char *in, unsigned char *out, const unsigned char ivec[8],
                        const unsigned char nonce[4], unsigned long length,
                        const unsigned char *key, int nr, unsigned long long block_offset)
{
    const __m128i *rk = (const __m128i *)key;
    /* counter block: nonce[0..3] | ivec[0..7] | 00 00 00 01; the low 8 bytes
     * (ivec[4..7] | counter) are a 64-bit big-endian integer incremented per
     * block. */
    unsigned char hi[8];
    memcpy(hi, nonce, 4);
    memcpy(hi + 4, ivec, 4);
    unsigned long long lo = 0;
    for (int i = 4; i < 8; ++i) lo = (lo << 8) | ivec[i];
    lo = (lo << 32) | 1u;
    lo += block_offset;
    const __m128i bswap = _mm_setr_epi8(7, 6, 5, 4, 3, 2, 1, 0, 15, 14, 13, 12, 11, 10, 9, 8);
    unsigned long long hiw;
    memcpy(&hiw, hi, 8);
    unsigned long full = length / 16, i = 0;
    for (; i <= full; ++i) {
        unsigned long n = (i < full) ? 16 : (length % 16);
        if (n == 0) break;
        /* little-endian lane 1 holds bytes 8..15 -> store byte-swapped lo */
        __m128i c = _mm_set_epi64x((long long)(lo + i), 0);
        c = _mm_shuffle_epi8(c, bswap);
        c = _mm_insert_epi64(c, (long long)hiw, 0);
        __m128i ks = enc1(c, rk, nr);
        if (n == 16) {
            _mm_storeu_si128((__m128i *)(out + 16 * i),
                             _mm_xor_si128(ks, _mm_loadu_si128((const __m128i *)(in + 16 * i))));
        } else {
            unsigned char k[16];
            _mm_storeu_si128((__m128i *)k, ks);
            for (unsigned long b = 0; b < n; ++b) out[16 * i + b] = (unsigned char)(in[16 * i + b] ^ k[b]);
        }
    }
}

void AES_CTR_encrypt(const unsigned char *in, unsigned char *out, const unsigned char ivec[8],
                     const unsigned char nonce[4], unsigned long length,
                     const unsigned char *key, int nr)
{
    AES_CTR_encrypt_at(in, out, ivec, nonce, length, key, nr, 0);
}

/* Serial chains (one AES-NI pipe, latency bound): the host path for exact
 * single-stream CBC / CFB128 encryption, which no amount of GPU parallelism
 * can speed up (every block needs the previous ciphertext). */
void AES_CBC_encrypt(const unsigned char *in, unsigned char *out, unsigned char ivec[16], unsigned long length,
                     const unsigned char *key, int nr)
{
    const __m128i *rk = (const __m128i *)key;
    __m128i c = _mm_loadu_si128((const __m128i *)ivec);
    for (unsigned long i = 0; i < length / 16; ++i) {
        c = enc1(_mm_xor_si128(c, _mm_loadu_si128((const __m128i *)in + i)), rk, nr);
        _mm_storeu_si128((__m128i *)out + i, c);
    }
    _mm_storeu_si128((__m128i *)ivec, c);
}

void AES_CFB128_encrypt(const unsigned char *in, unsigned char *out, unsigned char ivec[16], unsigned long length,
                        const unsigned char *key, int nr)
{
    const __m128i *rk = (const __m128i *)key;
    __m128i c = _mm_loadu_si128((const __m128i *)ivec);
    unsigned long nb = length / 16;
    for (unsigned long i = 0; i < nb; ++i) {
        c = _mm_xor_si128(enc1(c, rk, nr), _mm_loadu_si128((const __m128i *)in + i));
        _mm_storeu_si128((__m128i *)out + i, c);
    }
    if (length % 16) { /* trailing partial block: keystream bytes of E(c) */
        unsigned char k[16];
        _mm_storeu_si128((__m128i *)k, enc1(c, rk, nr));
        for (unsigned long b = 0; b < length % 16; ++b) out[16 * nb + b] = (unsigned char)(in[16 * nb + b] ^ k[b]);
    }
    _mm_storeu_si128((__m128i *)ivec, c);
}
