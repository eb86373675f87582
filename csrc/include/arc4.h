/*
 * arc4.h -- ARCFOUR (RC4) stream cipher, CPU reference API.
 *
 * Source-compatible with /root/reference/arc4.h:35-77: arc4_context {x,y,m},
 * arc4_setup (KSA), arc4_prep (PRGA -> keystream buffer, resumable through
 * ctx->x/y/m), arc4_crypt (parallel XOR combiner) and arc4_self_test.
 * The reference splits RC4 into a serial producer (arc4_prep) and an
 * embarrassingly parallel consumer (arc4_crypt); the GPU path keeps that
 * split (device XOR combiner) and adds a many-stream RC4 kernel.
 */
#ifndef OTC_ARC4_H
#define OTC_ARC4_H

#include <stddef.h>
#include <string.h>

typedef struct {
    int x;                  /* permutation index i */
    int y;                  /* permutation index j */
    unsigned char m[256];   /* permutation S */
} arc4_context;

#ifdef __cplusplus
extern "C" {
#endif

void arc4_setup(arc4_context *ctx, const unsigned char *key, unsigned int keylen);

/* Generate `length` keystream bytes into `keystream`; ctx state advances so a
 * second call continues the stream.  Returns 0. */
int arc4_prep(arc4_context *ctx, size_t length, unsigned char *keystream);

/* output[i] = input[i] ^ keystream[i]; returns 0. */
int arc4_crypt(size_t length, const unsigned char *input, unsigned char *keystream,
               unsigned char *output);

/* Rescorla test vectors; verbose >= 1 prints one line per vector. */
int arc4_self_test(int verbose);

/* ---- extensions ---------------------------------------------------------- */
/* Multi-threaded XOR combiner (remainders are not dropped). */
int arc4_crypt_mt(size_t length, const unsigned char *input, const unsigned char *keystream,
                  unsigned char *output, int nthreads);

#ifdef __cplusplus
}
#endif

#endif
