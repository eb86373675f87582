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
 * Extensions:  --device gpu   XOR combiner runs on the GPUs: column 3 then
 *                             counts GPUs instead of CPU threads (the buffers
 *                             are sharded over that many devices, data
 *                             resident; rows asking for more GPUs than the
 *                             node has are skipped)
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
#define MAX_GPUS 16

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
#ifdef OTC_WITH_GPU
    const int ndev = gpu ? otc_device_count() : 0;
#endif
    for (int si = 0; si < nsizes; ++si) {
        for (int ti = 0; ti < nthreads; ++ti) {
            size_t len = (size_t)sizes[si];
            int nt = (int)threads[ti];
#ifdef OTC_WITH_GPU
            if (gpu && (nt < 1 || nt > ndev || nt > MAX_GPUS)) continue; /* column 3 = GPUs actually used */
#endif
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
            /* GPU mode: the message and keystream are sharded over nt GPUs
             * (16-byte aligned contiguous shards, resident); each GPU runs the
             * combiner on its shard, all launched before any is waited for */
            void *dm[MAX_GPUS] = {0}, *dk[MAX_GPUS] = {0}, *dout[MAX_GPUS] = {0};
            size_t goff[MAX_GPUS + 1] = {0};
            if (gpu) {
                for (int g = 0; g < nt; ++g) goff[g] = (len / 16 * (size_t)g / (size_t)nt) * 16;
                goff[nt] = len;
                for (int g = 0; g < nt; ++g) {
                    const size_t n = goff[g + 1] - goff[g];
                    otc_set_device(g);
                    dm[g] = otc_dev_malloc(n);
                    dk[g] = otc_dev_malloc(n);
                    dout[g] = otc_dev_malloc(n);
                    if (!dm[g] || !dk[g] || !dout[g]) {
                        fprintf(stderr, "device alloc failed: %s\n", otc_last_error());
                        return 1;
                    }
                    otc_memcpy(dm[g], msg + goff[g], n, OTC_H2D);
                    otc_memcpy(dk[g], ks + goff[g], n, OTC_H2D);
                }
            }
#endif
            for (int it = 0; it < iters; ++it) {
                gettimeofday(&t0, NULL);
#ifdef OTC_WITH_GPU
                if (gpu) {
                    int rc = 0;
                    for (int g = 0; g < nt && !rc; ++g) {
                        otc_set_device(g);
                        rc = otc_xor(dm[g], dk[g], dout[g], goff[g + 1] - goff[g], NULL);
                    }
                    for (int g = 0; g < nt && !rc; ++g) {
                        otc_set_device(g);
                        rc = otc_device_sync();
                    }
                    if (rc) {
                        fprintf(stderr, "GPU error: %s\n", otc_last_error());
                        return 1;
                    }
                } else
#endif
                    arc4_crypt_mt(len, msg, ks, out, nt);
                gettimeofday(&t1, NULL);
                printf("%lld, ", us_between(t0, t1));
            }
#ifdef OTC_WITH_GPU
            if (gpu) {
                for (int g = 0; g < nt; ++g) {
                    otc_set_device(g);
                    otc_memcpy(out + goff[g], dout[g], goff[g + 1] - goff[g], OTC_D2H);
                    otc_dev_free(dm[g]);
                    otc_dev_free(dk[g]);
                    otc_dev_free(dout[g]);
                }
                otc_set_device(0);
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
