/*
 * aes_test.c -> bin/aes_test : AES thread/GPU scaling harness.
 *
 * Output-format parity with /root/reference/aes-modes/test.c:46-446:
 *     <Label>, <bytes>, <threads>, <us>, ... x10
 * Labels: "Plain ECB", "Plain CTR", "AESNI ECB", "AESNI CTR" (CPU baselines),
 * plus "HIP ECB", "HIP CTR", "HIP CBC" (gfx950 kernels, device-resident data,
 * column 3 = GPUs).  With no arguments it runs what the reference main runs:
 * the AES-NI check line and the AESNI CTR sweep (AES-256, srand(1337)).
 * Fixed reference defects: "Plain CTR" really runs CTR (test.c:162 ran the
 * ECB worker), every thread gets its own counter offset (test.c:282 reused
 * one keystream), remainders are not dropped (test.c:33).
 *
 *   --suite plain-ecb,plain-ctr,aesni-ecb,aesni-ctr,hip-ecb,hip-ctr,hip-cbc
 *   --sizes a,b,..  --threads a,b,..  --iters N  --bits 128|192|256
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/time.h>

#include "aes.h"
#include "aesni.h"
#ifdef OTC_WITH_GPU
#include "otc.h"
#endif

#define MAX_GPUS 16

static size_t MSG_LEN;
static unsigned char *msg, *out;
static aes_context actx;
static ALIGN16 unsigned char ni_key[16 * 15];
static int g_nr;
static unsigned char ivec[8] = {'H', 'l', 'o', 'E', 'e', 'l', 'A', 'S'};
static unsigned char nonce[4] = {'3', '1', '5', 'A'};

typedef struct {
    int tid, nt;
    int kind; /* 0 plain ecb, 1 plain ctr, 2 aesni ecb, 3 aesni ctr */
} job_t;

static void shard(int tid, int nt, size_t *off, size_t *len)
{
    size_t nb = MSG_LEN / 16, per = nb / (size_t)nt, rem = nb % (size_t)nt;
    size_t b0 = (size_t)tid * per + ((size_t)tid < rem ? (size_t)tid : rem);
    size_t cnt = per + ((size_t)tid < rem ? 1 : 0);
    *off = b0 * 16;
    *len = cnt * 16;
    if (tid == nt - 1) *len = MSG_LEN - *off; /* trailing partial block */
}

static void *worker(void *p)
{
    job_t *j = (job_t *)p;
    size_t off, len;
    shard(j->tid, j->nt, &off, &len);
    switch (j->kind) {
    case 0:
        for (size_t i = 0; i + 16 <= len; i += 16) aes_crypt_ecb(&actx, AES_ENCRYPT, msg + off + i, out + off + i);
        break;
    case 1: {
        unsigned char nc[16] = {0}, sb[16];
        memcpy(nc, nonce, 4);
        memcpy(nc + 4, ivec, 8);
        nc[15] = 1;
        aes_ctr128_add(nc, off / 16);
        int o = 0;
        aes_crypt_ctr(&actx, (int)len, &o, nc, sb, msg + off, out + off);
        break;
    }
    case 2: AES_ECB_encrypt(msg + off, out + off, len, ni_key, g_nr); break;
    case 3: AES_CTR_encrypt_at(msg + off, out + off, ivec, nonce, len, ni_key, g_nr, off / 16); break;
    }
    return NULL;
}

static long long now_us(void)
{
    struct timeval t;
    gettimeofday(&t, NULL);
    return (long long)t.tv_sec * 1000000LL + t.tv_usec;
}

static int parse_list(const char *s, long long *o, int max)
{
    int n = 0;
    while (*s && n < max) {
        o[n++] = strtoll(s, (char **)&s, 10);
        if (*s == ',') ++s;
    }
    return n;
}

static const char *LABEL[] = {"Plain ECB", "Plain CTR", "AESNI ECB", "AESNI CTR", "HIP ECB", "HIP CTR", "HIP CBC"};
static const char *SUITE[] = {"plain-ecb", "plain-ctr", "aesni-ecb", "aesni-ctr", "hip-ecb", "hip-ctr", "hip-cbc"};

#ifdef OTC_WITH_GPU
/* Sample check of a HIP row (outside the timed region): the first 64 bytes of
 * every GPU's shard against the CPU oracle, with the shard's counter offset
 * (CTR) or halo IV (CBC decryption). */
static int verify_shards(int kind, const unsigned char *key, int bits, int nt, void **dout, const size_t *goff,
                         const size_t *glen)
{
    aes_context c;
    if (kind == 6)
        aes_setkey_dec(&c, key, (unsigned)bits);
    else
        aes_setkey_enc(&c, key, (unsigned)bits);
    unsigned char ctr0[16] = {0};
    memcpy(ctr0, nonce, 4);
    memcpy(ctr0 + 4, ivec, 8);
    ctr0[15] = 1;
    for (int g = 0; g < nt; ++g) {
        unsigned char got[64], exp[64];
        size_t n = glen[g] < 64 ? glen[g] : 64;
        if (kind != 5) n &= ~(size_t)15;
        if (!n) continue;
        otc_set_device(g);
        if (otc_memcpy(got, dout[g], n, OTC_D2H)) return 1;
        const unsigned char *m = msg + goff[g];
        if (kind == 4) {
            for (size_t i = 0; i < n; i += 16) aes_crypt_ecb(&c, AES_ENCRYPT, m + i, exp + i);
        } else if (kind == 5) {
            unsigned char nc[16], sb[16];
            memcpy(nc, ctr0, 16);
            aes_ctr128_add(nc, goff[g] / 16);
            int o = 0;
            aes_crypt_ctr(&c, (int)n, &o, nc, sb, m, exp);
        } else {
            unsigned char iv[16];
            memcpy(iv, goff[g] ? m - 16 : ctr0, 16);
            aes_crypt_cbc(&c, AES_DECRYPT, n, iv, m, exp);
        }
        if (memcmp(got, exp, n)) {
            fprintf(stderr, "%s: output of GPU %d does not match the CPU oracle\n", LABEL[kind], g);
            return 1;
        }
    }
    otc_set_device(0);
    return 0;
}
#endif

int main(int argc, char **argv)
{
    long long sizes[16] = {1048576, 10485760, 104857600, 1048576000};
    long long threads[16] = {1, 2, 4, 8};
    int nsizes = 4, nthreads = 4, iters = 10, bits = 256;
    int run[7] = {0, 0, 0, 1, 0, 0, 0};
    for (int a = 1; a < argc; ++a) {
        if (!strcmp(argv[a], "--sizes") && a + 1 < argc) nsizes = parse_list(argv[++a], sizes, 16);
        else if (!strcmp(argv[a], "--threads") && a + 1 < argc) nthreads = parse_list(argv[++a], threads, 16);
        else if (!strcmp(argv[a], "--iters") && a + 1 < argc) iters = atoi(argv[++a]);
        else if (!strcmp(argv[a], "--bits") && a + 1 < argc) bits = atoi(argv[++a]);
        else if (!strcmp(argv[a], "--suite") && a + 1 < argc) {
            memset(run, 0, sizeof run);
            const char *s = argv[++a];
            for (int k = 0; k < 7; ++k)
                if (strstr(s, SUITE[k])) run[k] = 1;
        } else {
            fprintf(stderr, "usage: %s [--suite ..] [--sizes ..] [--threads ..] [--iters N] [--bits B]\n", argv[0]);
            return 2;
        }
    }
    srand(1337);
    setbuf(stdout, NULL);
    g_nr = bits == 128 ? 10 : bits == 192 ? 12 : 14;
    int have_ni = CheckAESSupport();
    if (run[2] || run[3]) {
        if (have_ni)
            printf("## CPU Supports AES-NI instructions. Continuing...\n");
        else
            printf("## CPU Does Not Support AES-NI instructions. Skipping...\n");
    }
    for (int kind = 0; kind < 7; ++kind) {
        if (!run[kind]) continue;
        if ((kind == 2 || kind == 3) && !have_ni) continue;
#ifndef OTC_WITH_GPU
        if (kind >= 4) continue;
#endif
        for (int si = 0; si < nsizes; ++si) {
            for (int ti = 0; ti < nthreads; ++ti) {
                MSG_LEN = (size_t)sizes[si];
                int nt = (int)threads[ti];
#ifdef OTC_WITH_GPU
                if (kind >= 4 && (nt < 1 || nt > otc_device_count() || nt > MAX_GPUS)) continue;
#endif
                printf("%s, %zu, %d, ", LABEL[kind], MSG_LEN, nt);
                msg = malloc(MSG_LEN);
                out = malloc(MSG_LEN);
                for (size_t i = 0; i < MSG_LEN; ++i) msg[i] = (unsigned char)(rand() % 255);
#ifdef OTC_WITH_GPU
                /* HIP rows: column 3 = GPUs; shard g (same planner as the CPU
                 * threads) is resident on GPU g */
                void *dmsg[MAX_GPUS] = {0}, *dout[MAX_GPUS] = {0};
                size_t goff[MAX_GPUS], glen[MAX_GPUS];
                if (kind >= 4) {
                    for (int g = 0; g < nt; ++g) {
                        shard(g, nt, &goff[g], &glen[g]);
                        otc_set_device(g);
                        dmsg[g] = otc_dev_malloc(glen[g]);
                        dout[g] = otc_dev_malloc(glen[g]);
                        if (!dmsg[g] || !dout[g]) {
                            fprintf(stderr, "device alloc failed: %s\n", otc_last_error());
                            return 1;
                        }
                        otc_memcpy(dmsg[g], msg + goff[g], glen[g], OTC_H2D);
                    }
                }
#endif
                for (int it = 0; it < iters; ++it) {
                    unsigned char key[32];
                    for (int i = 0; i < 32; ++i) key[i] = (unsigned char)(rand() % 255);
                    aes_setkey_enc(&actx, key, (unsigned)bits);
                    if (bits == 128) AES_128_Key_Expansion(key, ni_key);
                    else if (bits == 192) AES_192_Key_Expansion(key, ni_key);
                    else AES_256_Key_Expansion(key, ni_key);
                    long long t0 = now_us();
                    if (kind < 4) {
                        pthread_t th[256];
                        job_t jobs[256];
                        for (int t = 0; t < nt; ++t) {
                            jobs[t].tid = t;
                            jobs[t].nt = nt;
                            jobs[t].kind = kind;
                            pthread_create(&th[t], NULL, worker, &jobs[t]);
                        }
                        for (int t = 0; t < nt; ++t) pthread_join(th[t], NULL);
                    }
#ifdef OTC_WITH_GPU
                    else {
                        otc_aes_key k;
                        unsigned char nc[16] = {0};
                        memcpy(nc, nonce, 4);
                        memcpy(nc + 4, ivec, 8);
                        nc[15] = 1;
                        otc_aes_key_init(&k, key, bits, kind == 6 ? OTC_DIR_DECRYPT : OTC_DIR_ENCRYPT);
                        int r = 0;
                        /* launch every shard, then wait for all GPUs */
                        for (int g = 0; g < nt && !r; ++g) {
                            otc_set_device(g);
                            if (kind == 4) {
                                r = otc_aes_ecb(dmsg[g], dout[g], glen[g] & ~(size_t)15, &k, OTC_IMPL_AUTO, NULL);
                            } else if (kind == 5) { /* counter offset of the shard */
                                r = otc_aes_ctr(dmsg[g], dout[g], glen[g], &k, nc, goff[g] / 16, OTC_IMPL_AUTO, NULL);
                            } else { /* CBC-dec halo: the ciphertext block before the shard */
                                const unsigned char *iv = goff[g] ? msg + goff[g] - 16 : nc;
                                r = otc_aes_cbc_decrypt(dmsg[g], dout[g], glen[g] & ~(size_t)15, &k, iv, NULL);
                            }
                        }
                        for (int g = 0; g < nt && !r; ++g) {
                            otc_set_device(g);
                            r = otc_device_sync();
                        }
                        if (r) {
                            fprintf(stderr, "GPU error: %s\n", otc_last_error());
                            return 1;
                        }
                    }
#endif
                    printf("%lld, ", now_us() - t0);
#ifdef OTC_WITH_GPU
                    if (kind >= 4 && it == iters - 1 && verify_shards(kind, key, bits, nt, dout, goff, glen)) return 1;
#endif
                }
#ifdef OTC_WITH_GPU
                if (kind >= 4) {
                    for (int g = 0; g < nt; ++g) {
                        otc_dev_free(dmsg[g]);
                        otc_dev_free(dout[g]);
                    }
                    otc_set_device(0);
                }
#endif
                free(msg);
                free(out);
                printf("\n");
            }
        }
    }
    return 0;
}
