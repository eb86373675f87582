/*
 * rc4.h -- one-call in-place RC4 API, source compatible with
 * /root/reference/rc4.h:43-50 (FreeBSD-derived).  The reference's
 * implementation indexed with a signed `char` and never masked its indices
 * (stack overflow under ASan, rc4.c:69-70); this implementation treats the
 * permutation as unsigned bytes and masks every index.
 */
#ifndef OTC_RC4_H
#define OTC_RC4_H

struct rc4_state {
    char perm[256];
    int index1;
    int index2;
};

#ifdef __cplusplus
extern "C" {
#endif
void rc4_crypt(struct rc4_state *const state, const char *inbuf, char *outbuf, int buflen);
void rc4_init(struct rc4_state *const state, const char *key, int keylen);
#ifdef __cplusplus
}
#endif

#endif
