/*
 * aes_ecb_e.c -> bin/aes_ecb_e : GPU AES ECB benchmark with the output format
 * of /root/reference/aes-gpu/Source/main_ecb_e.cu:54-65
 *     AES ECB test, <bytes>: <us>, <us>, ... x10  Average <us>
 * for 1/10/100/1000 MiB, AES-256 random keys (main_ecb_e.cu:15).
 *
 * Timed region (reference methodology, main_ecb_e.cu:37-44): key expansion +
 * host->device + kernel + device->host, but through the pinned 3-stream
 * pipeline instead of per-call malloc/pageable copies.  --kernel-only times
 * the device kernel alone on resident data; --bits 128 for AES-128.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/time.h>

#include "otc.h"

static long long now_us(void)
{
    struct timeval t;
    gettimeofday(&t, NULL);
    return (long long)t.tv_sec * 1000000LL + t.tv_usec;
}

int main(int argc, char **argv)
{
    int bits = 256, kernel_only = 0, iters = 10, impl = OTC_IMPL_AUTO;
    long long sizes[4] = {1048576, 10485760, 104857600, 1048576000};
    for (int a = 1; a < argc; ++a) {
        if (!strcmp(argv[a], "--bits") && a + 1 < argc) bits = atoi(argv[++a]);
        else if (!strcmp(argv[a], "--kernel-only")) kernel_only = 1;
        else if (!strcmp(argv[a], "--iters") && a + 1 < argc) iters = atoi(argv[++a]);
        else if (!strcmp(argv[a], "--impl") && a + 1 < argc) {
            ++a;
            impl = !strcmp(argv[a], "bitslice") ? OTC_IMPL_BITSLICE : !strcmp(argv[a], "ttable") ? OTC_IMPL_TTABLE : 0;
        } else {
            fprintf(stderr, "usage: %s [--bits 128|192|256] [--kernel-only] [--iters N] [--impl ttable|bitslice]\n", argv[0]);
            return 2;
        }
    }
    srand(1337);
    otc_engine *eng = otc_engine_create(0, 64u << 20, 3);
    if (!eng) {
        fprintf(stderr, "engine: %s\n", otc_last_error());
        return 1;
    }
    for (int si = 0; si < 4; ++si) {
        size_t n = (size_t)sizes[si];
        unsigned char *pt = otc_host_alloc_pinned(n), *ct = otc_host_alloc_pinned(n);
        void *dpt = kernel_only ? otc_dev_malloc(n) : NULL, *dct = kernel_only ? otc_dev_malloc(n) : NULL;
        if (!pt || !ct || (kernel_only && (!dpt || !dct))) {
            fprintf(stderr, "alloc failed\n");
            return 1;
        }
        for (size_t i = 0; i < n; ++i) pt[i] = (unsigned char)rand();
        if (kernel_only) otc_memcpy(dpt, pt, n, OTC_H2D);
        printf("AES ECB test, %zu: ", n);
        long long sum = 0;
        for (int it = 0; it < iters; ++it) {
            unsigned char key[32];
            for (int i = 0; i < 32; ++i) key[i] = (unsigned char)rand();
            otc_aes_key k;
            long long t0 = now_us();
            otc_aes_key_init(&k, key, bits, OTC_DIR_ENCRYPT);
            int r;
            if (kernel_only) {
                r = otc_aes_ecb(dpt, dct, n, &k, impl, NULL);
                if (!r) r = otc_device_sync();
            } else {
                r = otc_engine_run(eng, OTC_MODE_ECB, pt, ct, n, &k, NULL, 0, impl, NULL);
            }
            long long t = now_us() - t0;
            if (r) {
                fprintf(stderr, "error: %s\n", otc_last_error());
                return 1;
            }
            sum += t;
            printf("%lld, ", t);
        }
        printf(" Average %lld\n", sum / iters);
        otc_host_free_pinned(pt);
        otc_host_free_pinned(ct);
        otc_dev_free(dpt);
        otc_dev_free(dct);
    }
    otc_engine_destroy(eng);
    return 0;
}
