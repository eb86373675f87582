/*
 * arc4.c -- CPU reference ARCFOUR.  API parity: /root/reference/arc4.c:43-183
 * (arc4_setup / arc4_prep / arc4_crypt / arc4_self_test).  New implementation.
 */
#include "arc4.h"

#include <pthread.h>
#include <stdint.h>
#include <stdio.h>

void arc4_setup(arc4_context *ctx, const unsigned char *key, unsigned int keylen)
{
    unsigned char *S = ctx->m;
    for (int i = 0; i < 256; ++i) S[i] = (unsigned char)i;
    unsigned j = 0;
    for (unsigned i = 0; i < 256; ++i) {
        unsigned char t = S[i];
        j = (j + t + (keylen ? key[i % keylen] : 0)) & 0xff;
        S[i] = S[j];
        S[j] = t;
    }
    ctx->x = 0;
    ctx->y = 0;
}

int arc4_prep(arc4_context *ctx, size_t length, unsigned char *keystream)
{
    unsigned i = (unsigned)ctx->x & 0xff, j = (unsigned)ctx->y & 0xff;
    unsigned char *S = ctx->m;
    for (size_t n = 0; n < length; ++n) {
        i = (i + 1) & 0xff;
        unsigned char a = S[i];
        j = (j + a) & 0xff;
        unsigned char b = S[j];
        S[i] = b;
        S[j] = a;
        keystream[n] = S[(unsigned char)(a + b)];
    }
    ctx->x = (int)i;
    ctx->y = (int)j;
    return 0;
}

int arc4_crypt(size_t length, const unsigned char *input, unsigned char *keystream,
               unsigned char *output)
{
    size_t n = 0;
    /* word-at-a-time main loop; memcpy keeps it alias/alignment safe */
    for (; n + 8 <= length; n += 8) {
        uint64_t a, k;
        memcpy(&a, input + n, 8);
        memcpy(&k, keystream + n, 8);
        a ^= k;
        memcpy(output + n, &a, 8);
    }
    for (; n < length; ++n) output[n] = (unsigned char)(input[n] ^ keystream[n]);
    return 0;
}

typedef struct {
    const unsigned char *in, *ks;
    unsigned char *out;
    size_t len;
} xor_job;

static void *xor_worker(void *p)
{
    xor_job *j = (xor_job *)p;
    arc4_crypt(j->len, j->in, (unsigned char *)j->ks, j->out);
    return NULL;
}

int arc4_crypt_mt(size_t length, const unsigned char *input, const unsigned char *keystream,
                  unsigned char *output, int nthreads)
{
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    if (nthreads == 1) return arc4_crypt(length, input, (unsigned char *)keystream, output);
    pthread_t th[256];
    xor_job jobs[256];
    size_t per = length / (size_t)nthreads, rem = length % (size_t)nthreads, off = 0;
    for (int t = 0; t < nthreads; ++t) {
        size_t n = per + ((size_t)t < rem ? 1 : 0);
        jobs[t].in = input + off;
        jobs[t].ks = keystream + off;
        jobs[t].out = output + off;
        jobs[t].len = n;
        off += n;
        pthread_create(&th[t], NULL, xor_worker, &jobs[t]);
    }
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    return 0;
}

/* Rescorla (sci.crypt, 1994) vectors */
static const unsigned char kat_key[3][8] = {
    {0x01, 0x23, 0x45, 0x67, 0x89, 0xAB, 0xCD, 0xEF},
    {0x01, 0x23, 0x45, 0x67, 0x89, 0xAB, 0xCD, 0xEF},
    {0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00}};
static const unsigned char kat_pt[3][8] = {
    {0x01, 0x23, 0x45, 0x67, 0x89, 0xAB, 0xCD, 0xEF},
    {0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00},
    {0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00}};
static const unsigned char kat_ct[3][8] = {
    {0x75, 0xB7, 0x87, 0x80, 0x99, 0xE0, 0xC5, 0x96},
    {0x74, 0x94, 0xC2, 0xE7, 0x10, 0x4B, 0x08, 0x79},
    {0xDE, 0x18, 0x89, 0x41, 0xA3, 0x37, 0x5D, 0x3A}};

int arc4_self_test(int verbose)
{
    int fails = 0;
    for (int v = 0; v < 3; ++v) {
        arc4_context ctx;
        unsigned char ks[8], out[8];
        if (verbose) printf("  ARC4 test #%d: ", v + 1);
        arc4_setup(&ctx, kat_key[v], 8);
        arc4_prep(&ctx, 8, ks);
        arc4_crypt(8, kat_pt[v], ks, out);
        int ok = memcmp(out, kat_ct[v], 8) == 0;
        if (verbose) printf("%s\n", ok ? "passed" : "failed");
        fails += !ok;
    }
    if (verbose) printf("\n");
    return fails ? 1 : 0;
}
