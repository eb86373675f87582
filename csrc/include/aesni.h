/*
 * aesni.h -- x86 AES-NI CPU *baseline* (never used on the GPU path).
 *
 * API parity with /root/reference/aes-modes/aesni.h:11-32 (CheckAESSupport,
 * AES_256_Key_Expansion, AES_ECB_encrypt/decrypt, AES_CTR_encrypt with the
 * RFC 3686 nonce||ivec||BE32(1) counter block and a 64-bit big-endian
 * increment of its low 8 bytes).  Additions: 128/192-bit expansion and the
 * decryption (aesimc) schedule the reference never built, and exact tail
 * handling (the reference rounded the length up and over-read the input).
 * The header no longer depends on <wmmintrin.h> (reference aesni.h:1 did not
 * build on current compilers).
 */
#ifndef OTC_AESNI_H
#define OTC_AESNI_H

#if !defined(ALIGN16)
#define ALIGN16 __attribute__((aligned(16)))
#endif

#ifdef __cplusplus
extern "C" {
#endif

int CheckAESSupport(void);
void AES_128_Key_Expansion(const unsigned char *userkey, unsigned char *key);
void AES_192_Key_Expansion(const unsigned char *userkey, unsigned char *key);
void AES_256_Key_Expansion(const unsigned char *userkey, unsigned char *key);
/* Convert an encryption schedule (nr+1 round keys) into the aesdec schedule. */
void AES_Key_Expansion_Dec(const unsigned char *enc_key, unsigned char *dec_key, int number_of_rounds);

void AES_ECB_encrypt(const unsigned char *in, unsigned char *out, unsigned long length,
                     const unsigned char *key, int number_of_rounds);
void AES_ECB_decrypt(const unsigned char *in, unsigned char *out, unsigned long length,
                     const char *key, int number_of_rounds);
void AES_CTR_encrypt(const unsigned char *in, unsigned char *out, const unsigned char ivec[8],
                     const unsigned char nonce[4], unsigned long length,
                     const unsigned char *key, int number_of_rounds);
/* Same as AES_CTR_encrypt but starting `block_offset` blocks into the stream
 * (used to shard one stream over threads without keystream reuse). */
void AES_CTR_encrypt_at(const unsigned char *in, unsigned char *out, const unsigned char ivec[8],
                        const unsigned char nonce[4], unsigned long length,
                        const unsigned char *key, int number_of_rounds,
                        unsigned long long block_offset);

/* Serial CBC / CFB128 encryption chains (whole stream, one core): ivec is
 * updated to the last full ciphertext block, as a resumable IV.  CBC needs a
 * multiple of 16 bytes; CFB128 encrypts a trailing partial block too. */
void AES_CBC_encrypt(const unsigned char *in, unsigned char *out, unsigned char ivec[16], unsigned long length,
                     const unsigned char *key, int number_of_rounds);
void AES_CFB128_encrypt(const unsigned char *in, unsigned char *out, unsigned char ivec[16], unsigned long length,
                        const unsigned char *key, int number_of_rounds);

#ifdef __cplusplus
}
#endif

#endif
