/*
 * aes.c -- CPU reference implementation of AES-128/192/256 (FIPS-197) with
 * ECB / CBC / CFB128 / CTR modes (SP 800-38A).
 *
 * Role in this framework: the correctness oracle for the gfx950 HIP kernels
 * (csrc/hip/ kernels) and the CPU baseline for the harnesses.  API parity with
 * /root/reference/aes-modes/aes.h:62-161 (see include/aes.h).
 *
 * Design notes (new code, not derived from the reference's aes.c):
 *   - all tables (S-box, inverse S-box, Te0, Td0) are computed once from the
 *     GF(2^8) definition under pthread_once (thread safe; the reference's
 *     aes_gen_tables, aes.c:361-435, was guarded by a racy flag);
 *   - the other three T tables are byte rotations of T0 (the same trick the
 *     GPU kernel uses to fit one 64 KiB replicated table in LDS);
 *   - CFB128 and the self test are always built (reference: compiled out).
 */
#include "aes.h"

#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>

/* ---------------------------------------------------------------------------
 * Table generation
 * ------------------------------------------------------------------------- */
static uint8_t  g_sbox[256];
static uint8_t  g_isbox[256];
static uint32_t g_te0[256];
static uint32_t g_td0[256];
static uint32_t g_rcon[10];
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static inline uint32_t rotl32(uint32_t x, int n) { return (x << (n & 31)) | (x >> ((32 - n) & 31)); }
static inline uint8_t xt(uint8_t a) { return (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0x00)); }

static uint8_t gf_mul(uint8_t a, uint8_t b)
{
    uint8_t r = 0;
    while (b) {
        if (b & 1) r ^= a;
        a = xt(a);
        b >>= 1;
    }
    return r;
}

static void build_tables(void)
{
    uint8_t ex[256], lg[256];
    uint8_t v = 1;
    for (int i = 0; i < 255; ++i) {      /* generator 0x03 */
        ex[i] = v;
        lg[v] = (uint8_t)i;
        v = (uint8_t)(v ^ xt(v));
    }
    for (int a = 0; a < 256; ++a) {
        uint8_t inv = a ? ex[(255 - lg[a]) % 255] : 0;
        uint8_t s = inv;
        uint8_t r = inv;
        for (int k = 0; k < 4; ++k) {    /* affine map: b ^ rotl1..4(b) ^ 0x63 */
            r = (uint8_t)((r << 1) | (r >> 7));
            s ^= r;
        }
        s ^= 0x63;
        g_sbox[a] = s;
        g_isbox[s] = (uint8_t)a;
    }
    for (int a = 0; a < 256; ++a) {
        uint8_t s = g_sbox[a];
        g_te0[a] = (uint32_t)gf_mul(s, 2) | ((uint32_t)s << 8) | ((uint32_t)s << 16) |
                   ((uint32_t)gf_mul(s, 3) << 24);
        uint8_t t = g_isbox[a];
        g_td0[a] = (uint32_t)gf_mul(t, 14) | ((uint32_t)gf_mul(t, 9) << 8) |
                   ((uint32_t)gf_mul(t, 13) << 16) | ((uint32_t)gf_mul(t, 11) << 24);
    }
    uint8_t rc = 1;
    for (int i = 0; i < 10; ++i) {
        g_rcon[i] = rc;
        rc = xt(rc);
    }
}

static inline void ensure_tables(void) { pthread_once(&g_once, build_tables); }

const uint8_t *aes_sbox(void) { ensure_tables(); return g_sbox; }
const uint8_t *aes_inv_sbox(void) { ensure_tables(); return g_isbox; }
const uint32_t *aes_te0(void) { ensure_tables(); return g_te0; }
const uint32_t *aes_td0(void) { ensure_tables(); return g_td0; }

#define B0(x) ((x) & 0xff)
#define B1(x) (((x) >> 8) & 0xff)
#define B2(x) (((x) >> 16) & 0xff)
#define B3(x) ((x) >> 24)
#define TE(r, x) rotl32(g_te0[x], 8 * (r))
#define TD(r, x) rotl32(g_td0[x], 8 * (r))

static inline uint32_t load_le32(const unsigned char *p)
{
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
static inline void store_le32(unsigned char *p, uint32_t v)
{
    p[0] = (unsigned char)v;
    p[1] = (unsigned char)(v >> 8);
    p[2] = (unsigned char)(v >> 16);
    p[3] = (unsigned char)(v >> 24);
}

/* ---------------------------------------------------------------------------
 * Key schedule
 * ------------------------------------------------------------------------- */
static int expand_key(uint32_t *w, const unsigned char *key, unsigned int keysize, int *nr)
{
    int nk;
    switch (keysize) {
    case 128: nk = 4; *nr = 10; break;
    case 192: nk = 6; *nr = 12; break;
    case 256: nk = 8; *nr = 14; break;
    default: return POLARSSL_ERR_AES_INVALID_KEY_LENGTH;
    }
    int total = 4 * (*nr + 1);
    for (int i = 0; i < nk; ++i) w[i] = load_le32(key + 4 * i);
    for (int i = nk; i < total; ++i) {
        uint32_t t = w[i - 1];
        if (i % nk == 0) {
            t = (t >> 8) | (t << 24); /* RotWord on LE words */
            t = (uint32_t)g_sbox[B0(t)] | ((uint32_t)g_sbox[B1(t)] << 8) |
                ((uint32_t)g_sbox[B2(t)] << 16) | ((uint32_t)g_sbox[B3(t)] << 24);
            t ^= g_rcon[i / nk - 1];
        } else if (nk > 6 && i % nk == 4) {
            t = (uint32_t)g_sbox[B0(t)] | ((uint32_t)g_sbox[B1(t)] << 8) |
                ((uint32_t)g_sbox[B2(t)] << 16) | ((uint32_t)g_sbox[B3(t)] << 24);
        }
        w[i] = w[i - nk] ^ t;
    }
    return 0;
}

int aes_setkey_enc(aes_context *ctx, const unsigned char *key, unsigned int keysize)
{
    uint32_t w[60];
    ensure_tables();
    int ret = expand_key(w, key, keysize, &ctx->nr);
    if (ret) return ret;
    ctx->rk = ctx->buf;
    for (int i = 0; i < 4 * (ctx->nr + 1); ++i) ctx->buf[i] = w[i];
    return 0;
}

static inline uint32_t inv_mix_word(uint32_t x)
{
    /* Td includes the inverse S-box, so feed S-box(x) to cancel it. */
    return TD(0, g_sbox[B0(x)]) ^ TD(1, g_sbox[B1(x)]) ^ TD(2, g_sbox[B2(x)]) ^ TD(3, g_sbox[B3(x)]);
}

int aes_setkey_dec(aes_context *ctx, const unsigned char *key, unsigned int keysize)
{
    uint32_t w[60];
    ensure_tables();
    int nr;
    int ret = expand_key(w, key, keysize, &nr);
    if (ret) return ret;
    ctx->nr = nr;
    ctx->rk = ctx->buf;
    /* equivalent inverse cipher: reversed round keys, InvMixColumns on the
     * inner ones */
    for (int r = 0; r <= nr; ++r) {
        for (int c = 0; c < 4; ++c) {
            uint32_t k = w[4 * (nr - r) + c];
            ctx->buf[4 * r + c] = (r == 0 || r == nr) ? k : inv_mix_word(k);
        }
    }
    return 0;
}

int aes_export_rk32(const aes_context *ctx, uint32_t *out)
{
    int n = 4 * (ctx->nr + 1);
    for (int i = 0; i < n; ++i) out[i] = (uint32_t)ctx->rk[i];
    return n;
}

int aes_import_rk32(aes_context *ctx, const uint32_t *rk, int nr)
{
    if (nr != 10 && nr != 12 && nr != 14) return POLARSSL_ERR_AES_INVALID_KEY_LENGTH;
    ensure_tables();
    ctx->nr = nr;
    ctx->rk = ctx->buf;
    for (int i = 0; i < 4 * (nr + 1); ++i) ctx->buf[i] = rk[i];
    return 0;
}

/* ---------------------------------------------------------------------------
 * Block functions
 * ------------------------------------------------------------------------- */
static void encrypt_block(const aes_context *ctx, const unsigned char in[16], unsigned char out[16])
{
    const unsigned long *rk = ctx->rk;
    uint32_t s0 = load_le32(in) ^ (uint32_t)rk[0];
    uint32_t s1 = load_le32(in + 4) ^ (uint32_t)rk[1];
    uint32_t s2 = load_le32(in + 8) ^ (uint32_t)rk[2];
    uint32_t s3 = load_le32(in + 12) ^ (uint32_t)rk[3];
    for (int r = 1; r < ctx->nr; ++r) {
        rk += 4;
        uint32_t t0 = TE(0, B0(s0)) ^ TE(1, B1(s1)) ^ TE(2, B2(s2)) ^ TE(3, B3(s3)) ^ (uint32_t)rk[0];
        uint32_t t1 = TE(0, B0(s1)) ^ TE(1, B1(s2)) ^ TE(2, B2(s3)) ^ TE(3, B3(s0)) ^ (uint32_t)rk[1];
        uint32_t t2 = TE(0, B0(s2)) ^ TE(1, B1(s3)) ^ TE(2, B2(s0)) ^ TE(3, B3(s1)) ^ (uint32_t)rk[2];
        uint32_t t3 = TE(0, B0(s3)) ^ TE(1, B1(s0)) ^ TE(2, B2(s1)) ^ TE(3, B3(s2)) ^ (uint32_t)rk[3];
        s0 = t0; s1 = t1; s2 = t2; s3 = t3;
    }
    rk += 4;
#define FINAL_E(a, b, c, d) ((uint32_t)g_sbox[B0(a)] | ((uint32_t)g_sbox[B1(b)] << 8) | \
                             ((uint32_t)g_sbox[B2(c)] << 16) | ((uint32_t)g_sbox[B3(d)] << 24))
    store_le32(out, FINAL_E(s0, s1, s2, s3) ^ (uint32_t)rk[0]);
    store_le32(out + 4, FINAL_E(s1, s2, s3, s0) ^ (uint32_t)rk[1]);
    store_le32(out + 8, FINAL_E(s2, s3, s0, s1) ^ (uint32_t)rk[2]);
    store_le32(out + 12, FINAL_E(s3, s0, s1, s2) ^ (uint32_t)rk[3]);
#undef FINAL_E
}

static void decrypt_block(const aes_context *ctx, const unsigned char in[16], unsigned char out[16])
{
    const unsigned long *rk = ctx->rk;
    uint32_t s0 = load_le32(in) ^ (uint32_t)rk[0];
    uint32_t s1 = load_le32(in + 4) ^ (uint32_t)rk[1];
    uint32_t s2 = load_le32(in + 8) ^ (uint32_t)rk[2];
    uint32_t s3 = load_le32(in + 12) ^ (uint32_t)rk[3];
    for (int r = 1; r < ctx->nr; ++r) {
        rk += 4;
        uint32_t t0 = TD(0, B0(s0)) ^ TD(1, B1(s3)) ^ TD(2, B2(s2)) ^ TD(3, B3(s1)) ^ (uint32_t)rk[0];
        uint32_t t1 = TD(0, B0(s1)) ^ TD(1, B1(s0)) ^ TD(2, B2(s3)) ^ TD(3, B3(s2)) ^ (uint32_t)rk[1];
        uint32_t t2 = TD(0, B0(s2)) ^ TD(1, B1(s1)) ^ TD(2, B2(s0)) ^ TD(3, B3(s3)) ^ (uint32_t)rk[2];
        uint32_t t3 = TD(0, B0(s3)) ^ TD(1, B1(s2)) ^ TD(2, B2(s1)) ^ TD(3, B3(s0)) ^ (uint32_t)rk[3];
        s0 = t0; s1 = t1; s2 = t2; s3 = t3;
    }
    rk += 4;
#define FINAL_D(a, b, c, d) ((uint32_t)g_isbox[B0(a)] | ((uint32_t)g_isbox[B1(b)] << 8) | \
                             ((uint32_t)g_isbox[B2(c)] << 16) | ((uint32_t)g_isbox[B3(d)] << 24))
    store_le32(out, FINAL_D(s0, s3, s2, s1) ^ (uint32_t)rk[0]);
    store_le32(out + 4, FINAL_D(s1, s0, s3, s2) ^ (uint32_t)rk[1]);
    store_le32(out + 8, FINAL_D(s2, s1, s0, s3) ^ (uint32_t)rk[2]);
    store_le32(out + 12, FINAL_D(s3, s2, s1, s0) ^ (uint32_t)rk[3]);
#undef FINAL_D
}

int aes_crypt_ecb(aes_context *ctx, int mode, const unsigned char input[16], unsigned char output[16])
{
    if (mode == AES_ENCRYPT)
        encrypt_block(ctx, input, output);
    else
        decrypt_block(ctx, input, output);
    return 0;
}

/* ---------------------------------------------------------------------------
 * Modes of operation
 * ------------------------------------------------------------------------- */
int aes_crypt_cbc(aes_context *ctx, int mode, size_t length, unsigned char iv[16],
                  const unsigned char *input, unsigned char *output)
{
    if (length % 16) return POLARSSL_ERR_AES_INVALID_INPUT_LENGTH;
    unsigned char tmp[16];
    if (mode == AES_DECRYPT) {
        for (; length; length -= 16, input += 16, output += 16) {
            memcpy(tmp, input, 16);
            decrypt_block(ctx, input, output);
            for (int i = 0; i < 16; ++i) output[i] ^= iv[i];
            memcpy(iv, tmp, 16);
        }
    } else {
        for (; length; length -= 16, input += 16, output += 16) {
            for (int i = 0; i < 16; ++i) tmp[i] = input[i] ^ iv[i];
            encrypt_block(ctx, tmp, output);
            memcpy(iv, output, 16);
        }
    }
    return 0;
}

int aes_crypt_cfb128(aes_context *ctx, int mode, size_t length, int *iv_off,
                     unsigned char iv[16], const unsigned char *input, unsigned char *output)
{
    int n = *iv_off & 15;
    for (size_t i = 0; i < length; ++i) {
        if (n == 0) encrypt_block(ctx, iv, iv);
        unsigned char c;
        if (mode == AES_DECRYPT) {
            c = input[i];
            output[i] = (unsigned char)(c ^ iv[n]);
            iv[n] = c;
        } else {
            c = (unsigned char)(input[i] ^ iv[n]);
            output[i] = c;
            iv[n] = c;
        }
        n = (n + 1) & 15;
    }
    *iv_off = n;
    return 0;
}

void aes_ctr128_add(unsigned char ctr[16], uint64_t blocks)
{
    uint64_t carry = blocks;
    for (int i = 15; i >= 0 && carry; --i) {
        uint64_t v = (uint64_t)ctr[i] + (carry & 0xff);
        ctr[i] = (unsigned char)v;
        carry = (carry >> 8) + (v >> 8);
    }
}

int aes_crypt_ctr(aes_context *ctx, int length, int *nc_off, unsigned char nonce_counter[16],
                  unsigned char stream_block[16], const unsigned char *input, unsigned char *output)
{
    int n = *nc_off & 15;
    for (int i = 0; i < length; ++i) {
        if (n == 0) {
            encrypt_block(ctx, nonce_counter, stream_block);
            aes_ctr128_add(nonce_counter, 1);
        }
        output[i] = (unsigned char)(input[i] ^ stream_block[n]);
        n = (n + 1) & 15;
    }
    *nc_off = n;
    return 0;
}

/* ---------------------------------------------------------------------------
 * Multi-threaded bulk helpers (CPU baseline; remainders are NOT dropped and
 * every shard gets its own counter offset -- the reference's harness reused
 * one keystream across threads, aes-modes/test.c:282)
 * ------------------------------------------------------------------------- */
typedef struct {
    const aes_context *ctx;
    int mode;              /* AES_ENCRYPT / AES_DECRYPT for ECB, 2 for CTR */
    unsigned char ctr[16];
    const unsigned char *in;
    unsigned char *out;
    size_t len;
} bulk_job;

static void *bulk_worker(void *arg)
{
    bulk_job *j = (bulk_job *)arg;
    if (j->mode == 2) {
        unsigned char ks[16];
        size_t off = 0;
        while (off < j->len) {
            encrypt_block(j->ctx, j->ctr, ks);
            aes_ctr128_add(j->ctr, 1);
            size_t n = j->len - off < 16 ? j->len - off : 16;
            for (size_t i = 0; i < n; ++i) j->out[off + i] = (unsigned char)(j->in[off + i] ^ ks[i]);
            off += n;
        }
    } else {
        for (size_t off = 0; off + 16 <= j->len; off += 16) {
            if (j->mode == AES_ENCRYPT)
                encrypt_block(j->ctx, j->in + off, j->out + off);
            else
                decrypt_block(j->ctx, j->in + off, j->out + off);
        }
    }
    return NULL;
}

static int run_bulk(const aes_context *ctx, int mode, const unsigned char *nc,
                    const unsigned char *in, unsigned char *out, size_t len, int nthreads)
{
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    size_t nblocks = (len + 15) / 16;
    if ((size_t)nthreads > nblocks && nblocks > 0) nthreads = (int)nblocks;
    bulk_job jobs[256];
    pthread_t th[256];
    size_t per = nblocks / (size_t)nthreads, extra = nblocks % (size_t)nthreads;
    size_t blk = 0;
    for (int t = 0; t < nthreads; ++t) {
        size_t nb = per + ((size_t)t < extra ? 1 : 0);
        bulk_job *j = &jobs[t];
        j->ctx = ctx;
        j->mode = mode;
        if (nc) {
            memcpy(j->ctr, nc, 16);
            aes_ctr128_add(j->ctr, blk);
        }
        size_t start = blk * 16;
        size_t end = (blk + nb) * 16;
        if (end > len) end = len;
        j->in = in + start;
        j->out = out + start;
        j->len = end > start ? end - start : 0;
        blk += nb;
    }
    if (nthreads == 1) {
        bulk_worker(&jobs[0]);
        return 0;
    }
    for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, bulk_worker, &jobs[t]);
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    return 0;
}

int aes_ctr_bulk(const aes_context *ctx, const unsigned char nonce_counter[16],
                 const unsigned char *input, unsigned char *output, size_t length, int nthreads)
{
    return run_bulk(ctx, 2, nonce_counter, input, output, length, nthreads);
}

int aes_ecb_bulk(const aes_context *ctx, int mode, const unsigned char *input,
                 unsigned char *output, size_t length, int nthreads)
{
    if (length % 16) return POLARSSL_ERR_AES_INVALID_INPUT_LENGTH;
    return run_bulk(ctx, mode, NULL, input, output, length, nthreads);
}

/* ---------------------------------------------------------------------------
 * Self test: FIPS-197 appendix C, SP 800-38A F.1/F.2/F.3/F.5, RFC 3686 #1-#3,
 * and the 10,000-iteration Monte-Carlo ECB/CBC chains of the NIST
 * rijndael-vals set that the reference's self-test runs
 * (/root/reference/aes-modes/aes.c:912-950 vectors, loop :1084-1200).
 * ------------------------------------------------------------------------- */
static int hexval(char c)
{
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
}
static size_t unhex(const char *s, unsigned char *out)
{
    size_t n = 0;
    while (s[0] && s[1]) {
        out[n++] = (unsigned char)(hexval(s[0]) * 16 + hexval(s[1]));
        s += 2;
    }
    return n;
}

static const char *SP_PT =
    "6bc1bee22e409f96e93d7e117393172aae2d8a571e03ac9c9eb76fac45af8e51"
    "30c81c46a35ce411e5fbc1191a0a52eff69f2445df4f9b17ad2b417be66c3710";
static const char *SP_KEY[3] = {
    "2b7e151628aed2a6abf7158809cf4f3c",
    "8e73b0f7da0e6452c810f32b809079e562f8ead2522c6b7b",
    "603deb1015ca71be2b73aef0857d77811f352c073b6108d72d9810a30914dff4"};
static const char *SP_ECB[3] = {
    "3ad77bb40d7a3660a89ecaf32466ef97f5d3d58503b9699de785895a96fdbaaf"
    "43b1cd7f598ece23881b00e3ed0306887b0c785e27e8ad3f8223207104725dd4",
    "bd334f1d6e45f25ff712a214571fa5cc974104846d0ad3ad7734ecb3ecee4eef"
    "ef7afd2270e2e60adce0ba2face6444e9a4b41ba738d6c72fb16691603c18e0e",
    "f3eed1bdb5d2a03c064b5a7e3db181f8591ccb10d410ed26dc5ba74a31362870"
    "b6ed21b99ca6f4f9f153e7b1beafed1d23304b7a39f9f3ff067d8d8f9e24ecc7"};
static const char *SP_CBC[3] = {
    "7649abac8119b246cee98e9b12e9197d5086cb9b507219ee95db113a917678b2"
    "73bed6b8e3c1743b7116e69e222295163ff1caa1681fac09120eca307586e1a7",
    "4f021db243bc633d7178183a9fa071e8b4d9ada9ad7dedf4e5e738763f69145a"
    "571b242012fb7ae07fa9baac3df102e008b0e27988598881d920a9e64f5615cd",
    "f58c4c04d6e5f1ba779eabfb5f7bfbd69cfc4e967edb808d679f777bc6702c7d"
    "39f23369a9d9bacfa530e26304231461b2eb05e2c39be9fcda6c19078c6a9d1b"};
static const char *SP_CFB[3] = {
    "3b3fd92eb72dad20333449f8e83cfb4ac8a64537a0b3a93fcde3cdad9f1ce58b"
    "26751f67a3cbb140b1808cf187a4f4dfc04b05357c5d1c0eeac4c66f9ff7f2e6",
    "cdc80d6fddf18cab34c25909c99a417467ce7f7f81173621961a2b70171d3d7a"
    "2e1e8a1dd59b88b1c8e60fed1efac4c9c05f9f9ca9834fa042ae8fba584b09ff",
    "dc7e84bfda79164b7ecd8486985d386039ffed143b28b1c832113c6331e5407b"
    "df10132415e54b92a13ed0a8267ae2f975a385741ab9cef82031623d55b1e471"};
static const char *SP_CTR[3] = {
    "874d6191b620e3261bef6864990db6ce9806f66b7970fdff8617187bb9fffdff"
    "5ae4df3edbd5d35e5b4f09020db03eab1e031dda2fbe03d1792170a0f3009cee",
    "1abc932417521ca24f2b0459fe7e6e0b090339ec0aa6faefd5ccc2c6f4ce8e94"
    "1e36b26bd1ebc670d1bd1d665620abf74f78a7f6d29809585a97daec58c6b050",
    "601ec313775789a5b7a7f504bbf3d228f443e3ca4d62b59aca84e990cacaf5c5"
    "2b0930daa23de94ce87017ba2d84988ddfc9c58db67aada613c2dd08457941a6"};

/* RFC 3686: key, counter block (nonce||iv||00000001), plaintext, ciphertext */
static const char *RFC3686[3][4] = {
    {"ae6852f8121067cc4bf7a5765577f39e", "00000030000000000000000000000001",
     "53696e676c6520626c6f636b206d7367", "e4095d4fb7a7b3792d6175a3261311b8"},
    {"7e24067817fae0d743d6ce1f32539163", "006cb6dbc0543b59da48d90b00000001",
     "000102030405060708090a0b0c0d0e0f101112131415161718191a1b1c1d1e1f",
     "5104a106168a72d9790d41ee8edad388eb2e1efc46da57c8fce630df9141be28"},
    {"7691be035e5020a8ac6e618529f9a0dc", "00e0017b27777f3f4a1786f000000001",
     "000102030405060708090a0b0c0d0e0f101112131415161718191a1b1c1d1e1f20212223",
     "c1cf48a89f2ffdd9cf4652e9efdb72d74540a42bde6d7836d59a5ceaaef3105325b2072f"}};

static int report(int verbose, const char *name, int ok)
{
    if (verbose) printf("  %s: %s\n", name, ok ? "passed" : "failed");
    return ok ? 0 : 1;
}

/* Monte-Carlo results after 10,000 chained operations from an all-zero key
 * (128/192/256), block and IV (NIST rijndael-vals) */
static const char *MC_ECB_ENC[3] = {"c34c052cc0da8d73451afe5f03be297f", "f3f6752ae8d7831138f041560631b114",
                                    "8b79eecc93a0ee5dff30b4ea21636da4"};
static const char *MC_ECB_DEC[3] = {"44416ac2d1f53c583303917e6be9ebe0", "48e31e9e256718f29229319c19f15ba4",
                                    "058ccffdbbcb382d1f6f56585d8a4ade"};
static const char *MC_CBC_ENC[3] = {"8a05fc5e095af4848a08d328d3688e3d", "7bd966d53ad8c1bb85d2adfae87bb104",
                                    "fe3c53653e2f45b56fcd88b2cc898ff0"};
static const char *MC_CBC_DEC[3] = {"faca37e0b0c85373df706e73f7c9af86", "5df678dd17ba4e75b61768c6adef7c7b",
                                    "4804e1818fe6297519a3e88c57310413"};

int aes_monte_carlo(int mode, int bits, unsigned char result[16])
{
    unsigned char key[32] = {0}, buf[16] = {0}, iv[16] = {0}, prv[16] = {0};
    aes_context ctx;
    const int dec = (mode == AES_MC_ECB_DEC || mode == AES_MC_CBC_DEC);
    int r = dec ? aes_setkey_dec(&ctx, key, (unsigned)bits) : aes_setkey_enc(&ctx, key, (unsigned)bits);
    if (r) return r;
    for (int j = 0; j < 10000; ++j) {
        switch (mode) {
        case AES_MC_ECB_ENC: aes_crypt_ecb(&ctx, AES_ENCRYPT, buf, buf); break;
        case AES_MC_ECB_DEC: aes_crypt_ecb(&ctx, AES_DECRYPT, buf, buf); break;
        case AES_MC_CBC_DEC: aes_crypt_cbc(&ctx, AES_DECRYPT, 16, iv, buf, buf); break;
        case AES_MC_CBC_ENC: { /* the ciphertext becomes the next IV (in iv) and the
                                  previous ciphertext the next plaintext */
            unsigned char tmp[16];
            aes_crypt_cbc(&ctx, AES_ENCRYPT, 16, iv, buf, buf);
            memcpy(tmp, prv, 16);
            memcpy(prv, buf, 16);
            memcpy(buf, tmp, 16);
            break;
        }
        default: return POLARSSL_ERR_AES_INVALID_INPUT_LENGTH;
        }
    }
    memcpy(result, mode == AES_MC_CBC_ENC ? prv : buf, 16);
    return 0;
}

const char *aes_monte_carlo_expected(int mode, int bits)
{
    const int k = (bits - 128) / 64;
    if (k < 0 || k > 2 || bits % 64) return NULL;
    switch (mode) {
    case AES_MC_ECB_ENC: return MC_ECB_ENC[k];
    case AES_MC_ECB_DEC: return MC_ECB_DEC[k];
    case AES_MC_CBC_ENC: return MC_CBC_ENC[k];
    case AES_MC_CBC_DEC: return MC_CBC_DEC[k];
    default: return NULL;
    }
}

int aes_self_test(int verbose)
{
    int fails = 0;
    char name[64];
    unsigned char key[32], pt[64], ref[64], out[64], iv[16], sb[16];
    aes_context ctx;

    /* FIPS-197 appendix C: key 00..(n-1), pt 00112233..ff */
    static const char *fips_ct[3] = {"69c4e0d86a7b0430d8cdb78070b4c55a",
                                     "dda97ca4864cdfe06eaf70a0ec0d7191",
                                     "8ea2b7ca516745bfeafc49904b496089"};
    for (int k = 0; k < 3; ++k) {
        int bits = 128 + 64 * k;
        for (int i = 0; i < 32; ++i) key[i] = (unsigned char)i;
        unhex("00112233445566778899aabbccddeeff", pt);
        unhex(fips_ct[k], ref);
        aes_setkey_enc(&ctx, key, (unsigned)bits);
        aes_crypt_ecb(&ctx, AES_ENCRYPT, pt, out);
        snprintf(name, sizeof name, "FIPS-197 C.%d AES-%d (enc)", k + 1, bits);
        fails += report(verbose, name, memcmp(out, ref, 16) == 0);
        aes_setkey_dec(&ctx, key, (unsigned)bits);
        aes_crypt_ecb(&ctx, AES_DECRYPT, ref, out);
        snprintf(name, sizeof name, "FIPS-197 C.%d AES-%d (dec)", k + 1, bits);
        fails += report(verbose, name, memcmp(out, pt, 16) == 0);
    }

    unhex(SP_PT, pt);
    for (int k = 0; k < 3; ++k) {
        int bits = 128 + 64 * k;
        unhex(SP_KEY[k], key);

        /* ECB */
        unhex(SP_ECB[k], ref);
        aes_setkey_enc(&ctx, key, (unsigned)bits);
        for (int b = 0; b < 4; ++b) aes_crypt_ecb(&ctx, AES_ENCRYPT, pt + 16 * b, out + 16 * b);
        snprintf(name, sizeof name, "AES-ECB-%d (enc)", bits);
        fails += report(verbose, name, memcmp(out, ref, 64) == 0);
        aes_setkey_dec(&ctx, key, (unsigned)bits);
        for (int b = 0; b < 4; ++b) aes_crypt_ecb(&ctx, AES_DECRYPT, ref + 16 * b, out + 16 * b);
        snprintf(name, sizeof name, "AES-ECB-%d (dec)", bits);
        fails += report(verbose, name, memcmp(out, pt, 64) == 0);

        /* CBC */
        unhex(SP_CBC[k], ref);
        aes_setkey_enc(&ctx, key, (unsigned)bits);
        unhex("000102030405060708090a0b0c0d0e0f", iv);
        aes_crypt_cbc(&ctx, AES_ENCRYPT, 64, iv, pt, out);
        snprintf(name, sizeof name, "AES-CBC-%d (enc)", bits);
        fails += report(verbose, name, memcmp(out, ref, 64) == 0);
        aes_setkey_dec(&ctx, key, (unsigned)bits);
        unhex("000102030405060708090a0b0c0d0e0f", iv);
        aes_crypt_cbc(&ctx, AES_DECRYPT, 64, iv, ref, out);
        snprintf(name, sizeof name, "AES-CBC-%d (dec)", bits);
        fails += report(verbose, name, memcmp(out, pt, 64) == 0);

        /* CFB128 (byte-granular resume exercised by a 13/51 split) */
        unhex(SP_CFB[k], ref);
        aes_setkey_enc(&ctx, key, (unsigned)bits);
        int off = 0;
        unhex("000102030405060708090a0b0c0d0e0f", iv);
        aes_crypt_cfb128(&ctx, AES_ENCRYPT, 13, &off, iv, pt, out);
        aes_crypt_cfb128(&ctx, AES_ENCRYPT, 51, &off, iv, pt + 13, out + 13);
        snprintf(name, sizeof name, "AES-CFB128-%d (enc)", bits);
        fails += report(verbose, name, memcmp(out, ref, 64) == 0);
        off = 0;
        unhex("000102030405060708090a0b0c0d0e0f", iv);
        aes_crypt_cfb128(&ctx, AES_DECRYPT, 64, &off, iv, ref, out);
        snprintf(name, sizeof name, "AES-CFB128-%d (dec)", bits);
        fails += report(verbose, name, memcmp(out, pt, 64) == 0);

        /* CTR (resume across a 7/57 split) */
        unhex(SP_CTR[k], ref);
        unhex("f0f1f2f3f4f5f6f7f8f9fafbfcfdfeff", iv);
        off = 0;
        aes_crypt_ctr(&ctx, 7, &off, iv, sb, pt, out);
        aes_crypt_ctr(&ctx, 57, &off, iv, sb, pt + 7, out + 7);
        snprintf(name, sizeof name, "AES-CTR-%d (enc)", bits);
        fails += report(verbose, name, memcmp(out, ref, 64) == 0);
    }

    for (int v = 0; v < 3; ++v) {
        size_t kl = unhex(RFC3686[v][0], key);
        unhex(RFC3686[v][1], iv);
        size_t n = unhex(RFC3686[v][2], pt);
        unhex(RFC3686[v][3], ref);
        aes_setkey_enc(&ctx, key, (unsigned)(kl * 8));
        int off = 0;
        aes_crypt_ctr(&ctx, (int)n, &off, iv, sb, pt, out);
        snprintf(name, sizeof name, "RFC 3686 AES-CTR test vector #%d", v + 1);
        fails += report(verbose, name, memcmp(out, ref, n) == 0);
    }
    static const char *mc_name[4] = {"ECB", "ECB", "CBC", "CBC"};
    for (int mode = 0; mode < 4; ++mode)
        for (int k = 0; k < 3; ++k) {
            const int bits = 128 + 64 * k;
            unsigned char got[16];
            unhex(aes_monte_carlo_expected(mode, bits), ref);
            snprintf(name, sizeof name, "AES-%s-%d (%s) Monte-Carlo x10000", mc_name[mode], bits,
                     (mode & 1) ? "dec" : "enc");
            fails += report(verbose, name, aes_monte_carlo(mode, bits, got) == 0 && memcmp(got, ref, 16) == 0);
        }
    if (verbose) printf("\n");
    return fails ? 1 : 0;
}
