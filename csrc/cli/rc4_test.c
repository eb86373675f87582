/*
 * rc4_test.c -> bin/test : RC4 thread/GPU scaling harness.
 *
 * With no arguments it reproduces the reference sweep of /root/reference/test.c
 * (sizes 1/10/100/1000 MiB x threads 1/2/4/8 x 10 iterations, srand(1337),
 * 16-byte random key, keystream generated serially once per size, then the
 * XOR combiner timed 10 times) and its exact output format (results.* files):
 *     RC4, <bytes>, <threads>, \nGenerated a new key in <us>, \n<us>, ...x10\n
 * followed by arc4_self_test(2).  Fixes vs the reference: remainder bytes are
 * not dropped (test.c:50), buffers are freed (test.c:67,79).
 *
 * Extensions:  --device gpu   XOR combiner runs on the GPU (column 3 then
 *                             means GPUs instead of CPU threads; data resident)
 *              --sizes a,b,.. --threads a,b,.. --iters N --noselftest
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/time.h>

#include "arc4.h"
#ifdef OTC_WITH_GPU
#include "otc.h"
#endif

#define KEY_LENGTH_BYTES 16

static long long us_between(struct timeval a, struct timeval b)
{
    return (long long)(b.tv_sec - a.tv_sec) * 1000000LL + (b.tv_usec - a.tv_usec);
}

static int parse_list(const char *s, long long *out, int max)
{
    int n = 0;
    while (*s && n < max) {
        out[n++] = strtoll(s, (char **)&s, 10);
        if (*s == ',') ++s;
    }
    return n;
}

int main(int argc, char **argv)
{
    long long sizes[16] = {1048576, 10485760, 104857600, 1048576000};
    long long threads[16] = {1, 2, 4, 8};
    int nsizes = 4, nthreads = 4, iters = 10, gpu = 0, selftest = 1;
    for (int a = 1; a < argc; ++a) {
        if (!strcmp(argv[a], "--device") && a + 1 < argc) gpu = !strcmp(argv[++a], "gpu");
        else if (!strcmp(argv[a], "--sizes") && a + 1 < argc) nsizes = parse_list(argv[++a], sizes, 16);
        else if (!strcmp(argv[a], "--threads") && a + 1 < argc) nthreads = parse_list(argv[++a], threads, 16);
        else if (!strcmp(argv[a], "--iters") && a + 1 < argc) iters = atoi(argv[++a]);
        else if (!strcmp(argv[a], "--noselftest")) selftest = 0;
        else {
            fprintf(stderr, "usage: %s [--device cpu|gpu] [--sizes ..] [--threads ..] [--iters N]\n", argv[0]);
            return 2;
        }
    }
#ifndef OTC_WITH_GPU
    if (gpu) {
        fprintf(stderr, "built without GPU support\n");
        return 2;
    }
#endif
    srand(1337);
    for (int si = 0; si < nsizes; ++si) {
        for (int ti = 0; ti < nthreads; ++ti) {
            size_t len = (size_t)sizes[si];
            int nt = (int)threads[ti];
            printf("RC4, %zu, %d, ", len, nt);
            unsigned char *msg = malloc(len), *out = malloc(len), *ks = malloc(len);
            if (!msg || !out || !ks) {
                fprintf(stderr, "out of memory\n");
                return 1;
            }
            for (size_t i = 0; i < len; ++i) msg[i] = (unsigned char)(rand() % 255);
            unsigned char key[KEY_LENGTH_BYTES];
            for (int i = 0; i < KEY_LENGTH_BYTES; ++i) key[i] = (unsigned char)(rand() % 255);
            struct timeval t0, t1;
            arc4_context ctx;
            printf("\nGenerated a new key in ");
            gettimeofday(&t0, NULL);
            arc4_setup(&ctx, key, KEY_LENGTH_BYTES);
            arc4_prep(&ctx, len, ks);
            gettimeofday(&t1, NULL);
            printf("%lld, \n", us_between(t0, t1));
#ifdef OTC_WITH_GPU
            void *dm = NULL, *dk = NULL, *dout = NULL;
            if (gpu) {
                dm = otc_dev_malloc(len);
                dk = otc_dev_malloc(len);
                dout = otc_dev_malloc(len);
                if (!dm || !dk || !dout) {
                    fprintf(stderr, "device alloc failed: %s\n", otc_last_error());
                    return 1;
                }
                otc_memcpy(dm, msg, len, OTC_H2D);
                otc_memcpy(dk, ks, len, OTC_H2D);
            }
#endif
            for (int it = 0; it < iters; ++it) {
                gettimeofday(&t0, NULL);
#ifdef OTC_WITH_GPU
                if (gpu) {
                    otc_xor(dm, dk, dout, len, NULL);
                    otc_device_sync();
                } else
#endif
                    arc4_crypt_mt(len, msg, ks, out, nt);
                gettimeofday(&t1, NULL);
                printf("%lld, ", us_between(t0, t1));
            }
#ifdef OTC_WITH_GPU
            if (gpu) {
                otc_memcpy(out, dout, len, OTC_D2H);
                otc_dev_free(dm);
                otc_dev_free(dk);
                otc_dev_free(dout);
            }
#endif
            /* verify (outside the timed region) */
            for (size_t i = 0; i < len; i += 4093)
                if (out[i] != (unsigned char)(msg[i] ^ ks[i])) {
                    fprintf(stderr, "verification failed at %zu\n", i);
                    return 1;
                }
            free(msg);
            free(out);
            free(ks);
            printf("\n");
        }
    }
    if (selftest) return arc4_self_test(2);
    return 0;
}
