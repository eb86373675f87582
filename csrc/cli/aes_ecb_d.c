/*
 * aes_ecb_d.c -> bin/aes_ecb_d KEYHEX CTHEX : ECB-decrypt one hex ciphertext
 * on the GPU and print the plaintext as uppercase hex.
 *
 * CLI parity with /root/reference/aes-gpu/Source/main_ecb_d.cu:10-40 (same
 * usage and error strings; the reference packed words big-endian (AES.cu:42)
 * and printed "%08X" words, which is byte-order hex -- reproduced here without
 * its sscanf("%02X") into a byte* UB, main_ecb_d.cu:47).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "otc.h"

static int hexnib(int c)
{
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
}

static size_t parse_hex(const char *s, unsigned char **out)
{
    size_t n = strlen(s) / 2;
    *out = malloc(n ? n : 1);
    for (size_t i = 0; i < n; ++i) {
        int hi = hexnib(s[2 * i]), lo = hexnib(s[2 * i + 1]);
        if (hi < 0 || lo < 0) return (size_t)-1;
        (*out)[i] = (unsigned char)(hi * 16 + lo);
    }
    return n;
}

int main(int argc, char **argv)
{
    if (argc < 3) {
        printf("USAGE: aes_ecb_d KEY PLAINTEXT [PLAINTEXT...]\n");
        return 1;
    }
    unsigned char *key, *ct;
    size_t klen = parse_hex(argv[1], &key);
    size_t clen = parse_hex(argv[2], &ct);
    if (klen != 16 && klen != 24 && klen != 32) {
        printf("Invalid AES key size.\n");
        return 1;
    }
    if (clen == (size_t)-1 || clen % 16 != 0) {
        printf("Plaintext size must be a multiple of AES block size.\n");
        return 1;
    }
    otc_aes_key k;
    if (otc_aes_key_init(&k, key, (int)klen * 8, OTC_DIR_DECRYPT)) {
        printf("Invalid AES key size.\n");
        return 1;
    }
    unsigned char *pt = malloc(clen ? clen : 1);
    void *d = otc_dev_malloc(clen);
    if (!d || otc_memcpy(d, ct, clen, OTC_H2D) || otc_aes_ecb(d, d, clen, &k, OTC_IMPL_AUTO, NULL) ||
        otc_memcpy(pt, d, clen, OTC_D2H)) {
        fprintf(stderr, "GPU error: %s\n", otc_last_error());
        return 1;
    }
    for (size_t i = 0; i < clen; ++i) printf("%02X", pt[i]);
    printf("\n");
    otc_dev_free(d);
    free(pt);
    free(key);
    free(ct);
    return 0;
}
