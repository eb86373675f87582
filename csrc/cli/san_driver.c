/*
 * san_driver.c -- exercises every multi-threaded and table-initialising path
 * of the CPU library under a sanitizer build (tests/test_sanitizers_cpu.py
 * builds it with -fsanitize=thread and with -fsanitize=address,undefined).
 *
 * Covers the reference's real races: the lazily built
 * AES tables (reference aes.c:359,448-452 set aes_init_done without any
 * synchronisation; here pthread_once) hit from many threads at once, and the
 * threaded CTR / ECB / XOR workers with remainders (reference test.c:50 and
 * aes-modes/test.c:33 drop them).  Every threaded result is compared with the
 * single-threaded one.  Exit code 0 = all equal.
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "aes.h"
#include "arc4.h"

#define NT 8

static unsigned char g_key[32];

static void *setkey_worker(void *arg)
{
    aes_context ctx;
    unsigned char blk[16] = {0}, out[16];
    int bits = 128 + 64 * (int)((size_t)arg % 3);
    if (aes_setkey_enc(&ctx, g_key, (unsigned)bits) != 0) return (void *)1;
    aes_crypt_ecb(&ctx, AES_ENCRYPT, blk, out);
    if (aes_setkey_dec(&ctx, g_key, (unsigned)bits) != 0) return (void *)1;
    aes_crypt_ecb(&ctx, AES_DECRYPT, out, blk);
    for (int i = 0; i < 16; ++i)
        if (blk[i]) return (void *)1;
    return NULL;
}

static int check(const char *what, const unsigned char *a, const unsigned char *b, size_t n)
{
    if (memcmp(a, b, n)) {
        fprintf(stderr, "MISMATCH %s\n", what);
        return 1;
    }
    return 0;
}

int main(void)
{
    int bad = 0;
    for (int i = 0; i < 32; ++i) g_key[i] = (unsigned char)(17 * i + 3);

    /* 1. first table use from NT threads at once */
    pthread_t th[NT];
    for (size_t i = 0; i < NT; ++i) pthread_create(&th[i], NULL, setkey_worker, (void *)i);
    for (int i = 0; i < NT; ++i) {
        void *r = NULL;
        pthread_join(th[i], &r);
        bad |= r != NULL;
    }

    /* 2. threaded bulk helpers vs one thread, odd length (remainders) */
    const size_t n = 3 * 4096 + 16 * 7 + 5, ne = n & ~(size_t)15;
    unsigned char *in = malloc(n), *o1 = malloc(n), *o8 = malloc(n), *ks = malloc(n);
    for (size_t i = 0; i < n; ++i) {
        in[i] = (unsigned char)(i * 131 + 7);
        ks[i] = (unsigned char)(i * 29 + 1);
    }
    unsigned char ctr0[16];
    memset(ctr0, 0xFF, 16);
    ctr0[0] = 0x12; /* forces a carry through 64-bit words mid-buffer */
    aes_context ctx;
    aes_setkey_enc(&ctx, g_key, 256);
    aes_ctr_bulk(&ctx, ctr0, in, o1, n, 1);
    aes_ctr_bulk(&ctx, ctr0, in, o8, n, NT);
    bad |= check("aes_ctr_bulk", o1, o8, n);
    aes_ecb_bulk(&ctx, AES_ENCRYPT, in, o1, ne, 1);
    aes_ecb_bulk(&ctx, AES_ENCRYPT, in, o8, ne, NT);
    bad |= check("aes_ecb_bulk", o1, o8, ne);
    arc4_crypt_mt(n, in, ks, o1, 1);
    arc4_crypt_mt(n, in, ks, o8, NT);
    bad |= check("arc4_crypt_mt", o1, o8, n);

    /* 3. self tests (both ciphers, every mode) */
    bad |= aes_self_test(0) != 0;
    bad |= arc4_self_test(0) != 0;

    free(in);
    free(o1);
    free(o8);
    free(ks);
    printf(bad ? "san_driver: FAIL\n" : "san_driver: OK\n");
    return bad;
}
