/*
 * otc_aesni.h -- the AES-NI bulk API shapes of the reference
 * (/root/reference/aes-modes/aesni.h:11-32: AES_ECB_encrypt(in, out, length,
 * key, number_of_rounds), AES_ECB_decrypt, AES_CTR_encrypt(in, out, ivec,
 * nonce, length, key, number_of_rounds)) served by the gfx950 kernels.
 *
 * in / out are DEVICE buffers (16-byte aligned); `key` is the HOST expanded
 * schedule exactly as AES_{128,192,256}_Key_Expansion (encryption) or
 * AES_Key_Expansion_Dec (decryption) in aesni.h produce it: 16*(Nr+1) bytes,
 * round keys in FIPS byte order -- the same bytes as the PolarSSL word
 * schedule the kernels consume, so no conversion is needed.  Work is queued
 * on `stream` (hipStream_t; NULL = default stream).  Return 0 or an OTC_ERR_*
 * code (otc_last_error()).  CTR uses the RFC 3686 block nonce || ivec ||
 * BE32(1) with the reference's 64-bit increment (aesni.c:132-143).
 */
#ifndef OTC_AESNI_H
#define OTC_AESNI_H

#ifdef __cplusplus
extern "C" {
#endif

int otc_AES_ECB_encrypt(const unsigned char *in, unsigned char *out, unsigned long length,
                        const unsigned char *key, int number_of_rounds, void *stream);
int otc_AES_ECB_decrypt(const unsigned char *in, unsigned char *out, unsigned long length,
                        const unsigned char *key, int number_of_rounds, void *stream);
int otc_AES_CTR_encrypt(const unsigned char *in, unsigned char *out, const unsigned char ivec[8],
                        const unsigned char nonce[4], unsigned long length, const unsigned char *key,
                        int number_of_rounds, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* OTC_AESNI_H */
