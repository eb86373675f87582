/*
 * aes.h -- AES-128/192/256 block cipher, CPU reference ("oracle") API.
 *
 * Source-compatible with the reference's PolarSSL-derived API
 * (/root/reference/aes-modes/aes.h:31-161): same function names, argument
 * order, AES_ENCRYPT/AES_DECRYPT values, error codes and aes_context field
 * names (nr, rk, buf).  Implementation is new (csrc/cpu/aes.c) and differs
 * from the reference where the reference is defective:
 *   - table generation is thread safe (pthread_once), reference aes.c:448-452
 *     used an unsynchronised flag;
 *   - CFB128 and the self test are always compiled in (reference compiled
 *     them out, aes.c:818,903).
 *
 * Byte streams are FIPS-197 / SP 800-38A exact.  Round keys are kept as
 * little-endian 32-bit column words (byte 0 of the column in bits 0..7), one
 * word per `unsigned long` slot for source compatibility.
 */
#ifndef OTC_AES_H
#define OTC_AES_H

#include <stddef.h>
#include <stdint.h>
#include <string.h>

#define AES_ENCRYPT 1
#define AES_DECRYPT 0

#define POLARSSL_ERR_AES_INVALID_KEY_LENGTH   -0x0020
#define POLARSSL_ERR_AES_INVALID_INPUT_LENGTH -0x0022

typedef struct {
    int nr;                 /* number of rounds: 10, 12 or 14 */
    unsigned long *rk;      /* points into buf */
    unsigned long buf[68];  /* round-key words (low 32 bits used) */
} aes_context;

#ifdef __cplusplus
extern "C" {
#endif

int aes_setkey_enc(aes_context *ctx, const unsigned char *key, unsigned int keysize);
int aes_setkey_dec(aes_context *ctx, const unsigned char *key, unsigned int keysize);

int aes_crypt_ecb(aes_context *ctx, int mode,
                  const unsigned char input[16], unsigned char output[16]);

int aes_crypt_cbc(aes_context *ctx, int mode, size_t length, unsigned char iv[16],
                  const unsigned char *input, unsigned char *output);

int aes_crypt_cfb128(aes_context *ctx, int mode, size_t length, int *iv_off,
                     unsigned char iv[16], const unsigned char *input,
                     unsigned char *output);

int aes_crypt_ctr(aes_context *ctx, int length, int *nc_off,
                  unsigned char nonce_counter[16], unsigned char stream_block[16],
                  const unsigned char *input, unsigned char *output);

int aes_self_test(int verbose);

/* ---- extensions (not in the reference API) ------------------------------ */

/* Copy the (4*(nr+1)) round-key words into a packed uint32 array; returns the
 * word count.  This is the format uploaded to the GPU kernels. */
int aes_export_rk32(const aes_context *ctx, uint32_t *out);
/* Inverse of aes_export_rk32: a context over (4*(nr+1)) packed round-key
 * words (either direction's schedule). */
int aes_import_rk32(aes_context *ctx, const uint32_t *rk, int nr);

/* Multi-threaded bulk helpers used by the CPU-baseline harness and the tests.
 * Counter semantics = aes_crypt_ctr with nc_off == 0 (full 128-bit BE add). */
int aes_ctr_bulk(const aes_context *ctx, const unsigned char nonce_counter[16],
                 const unsigned char *input, unsigned char *output, size_t length,
                 int nthreads);
int aes_ecb_bulk(const aes_context *ctx, int mode, const unsigned char *input,
                 unsigned char *output, size_t length, int nthreads);

/* Monte-Carlo known-answer chains of the reference self-test
 * (aes-modes/aes.c:1084-1200): 10,000 chained operations from an all-zero
 * key / block / IV.  aes_monte_carlo writes the final block (CBC-enc: the last
 * ciphertext); aes_monte_carlo_expected returns the published value (hex). */
#define AES_MC_ECB_ENC 0
#define AES_MC_ECB_DEC 1
#define AES_MC_CBC_ENC 2
#define AES_MC_CBC_DEC 3
int aes_monte_carlo(int mode, int bits, unsigned char result[16]);
const char *aes_monte_carlo_expected(int mode, int bits);

/* 128-bit big-endian counter add: ctr += blocks. */
void aes_ctr128_add(unsigned char ctr[16], uint64_t blocks);

/* Raw tables (generated on first use), exposed for table-driven kernels and
 * tests: forward S-box, inverse S-box, forward T0 and inverse T0 tables. */
const uint8_t  *aes_sbox(void);
const uint8_t  *aes_inv_sbox(void);
const uint32_t *aes_te0(void);
const uint32_t *aes_td0(void);

#ifdef __cplusplus
}
#endif

#endif /* OTC_AES_H */
