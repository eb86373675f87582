/*
 * rc4.c -- correct implementation of the rc4.h API (reference rc4.c:56-99 is
 * out-of-bounds for key bytes >= 0x80).  Output is identical to arc4.c.
 */
#include "rc4.h"

void rc4_init(struct rc4_state *const state, const char *key, int keylen)
{
    unsigned char *S = (unsigned char *)state->perm;
    const unsigned char *k = (const unsigned char *)key;
    for (int i = 0; i < 256; ++i) S[i] = (unsigned char)i;
    unsigned j = 0;
    for (int i = 0; i < 256; ++i) {
        unsigned char t = S[i];
        j = (j + t + (keylen > 0 ? k[i % keylen] : 0)) & 0xffu;
        S[i] = S[j];
        S[j] = t;
    }
    state->index1 = 0;
    state->index2 = 0;
}

void rc4_crypt(struct rc4_state *const state, const char *inbuf, char *outbuf, int buflen)
{
    unsigned char *S = (unsigned char *)state->perm;
    unsigned i = (unsigned)state->index1 & 0xffu, j = (unsigned)state->index2 & 0xffu;
    for (int n = 0; n < buflen; ++n) {
        i = (i + 1) & 0xffu;
        unsigned char a = S[i];
        j = (j + a) & 0xffu;
        unsigned char b = S[j];
        S[i] = b;
        S[j] = a;
        outbuf[n] = (char)((unsigned char)inbuf[n] ^ S[(unsigned char)(a + b)]);
    }
    state->index1 = (int)i;
    state->index2 = (int)j;
}
