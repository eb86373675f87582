/*
 * otc_hostsim.cpp -- the subset of the otc.h device API that bin/otbench
 * uses, implemented on HOST memory with the C oracle.  Linked into
 * bin/otbench_hostsim, it lets the CPU test suite run otbench's own argument,
 * snapshot and verification logic without a GPU (tests/test_otbench_cpu.py):
 * in-place runs, every mode's oracle, the 2^32-byte boundary sample, and the
 * --corrupt-at hook that must turn "verified" false.  It is a harness double,
 * not a second implementation of the engine: the "device" op and the
 * verifier share the oracle, so what it proves is that otbench checks what it
 * claims to check.  SURVEY.md section 4 item 5 (fake device for the container).
 *
 * Buffers above OTC_HOSTSIM_MAX bytes are refused (this container has 64 GiB
 * of RAM); the >4 GiB sample logic is exercised with a sparse mapping.
 */
#include <sys/mman.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

extern "C" {
#include "aes.h"
#include "arc4.h"
#include "otc.h"
}

namespace {
thread_local std::string g_err;
int fail(int code, const char *m)
{
    g_err = m;
    return code;
}
aes_context ctx_of(const otc_aes_key *k)
{
    aes_context c;
    aes_import_rk32(&c, k->rk, k->nr);
    return c;
}
void be_add(uint8_t iv[16], uint64_t n) { aes_ctr128_add(iv, n); }
} // namespace

extern "C" {

const char *otc_last_error(void) { return g_err.c_str(); }

int otc_aes_key_init(otc_aes_key *k, const uint8_t *key, int bits, int dir)
{
    aes_context ctx;
    int r = dir == OTC_DIR_ENCRYPT ? aes_setkey_enc(&ctx, key, (unsigned)bits) : aes_setkey_dec(&ctx, key, (unsigned)bits);
    if (r) return fail(OTC_ERR_ARG, "invalid AES key size");
    memset(k, 0, sizeof *k);
    aes_export_rk32(&ctx, k->rk);
    k->nr = ctx.nr;
    k->dir = dir;
    k->bits = bits;
    return OTC_OK;
}

/* the host double runs the oracle: it reports the T-table family */
int otc_last_impl(void) { return OTC_IMPL_TTABLE; }
void otc_split_stats(int) {}
int otc_split_trace(int, unsigned long long *, int) { return -1; }
int otc_runtime_info(char *buf, size_t n)
{
    const int w = snprintf(buf, n, "{\"hip_runtime_version\": -1, \"host_simulation\": true}");
    return w < 0 || (size_t)w >= n ? OTC_ERR_ARG : OTC_OK;
}
int otc_split_last_units(uint64_t *f, uint64_t *b, uint64_t *n)
{
    *f = *b = *n = 0;
    return OTC_OK;
}

int otc_aes_ecb(const void *in, void *out, size_t n, const otc_aes_key *k, int, void *)
{
    if (n % 16) return fail(OTC_ERR_ARG, "ecb length");
    aes_context c = ctx_of(k);
    return aes_ecb_bulk(&c, k->dir == OTC_DIR_ENCRYPT ? AES_ENCRYPT : AES_DECRYPT, (const uint8_t *)in,
                        (uint8_t *)out, n, 8);
}

int otc_aes_ctr(const void *in, void *out, size_t n, const otc_aes_key *k, const uint8_t ctr0[16], uint64_t off, int,
                void *)
{
    aes_context c = ctx_of(k);
    uint8_t nc[16];
    memcpy(nc, ctr0, 16);
    be_add(nc, off);
    return aes_ctr_bulk(&c, nc, (const uint8_t *)in, (uint8_t *)out, n, 8);
}

int otc_aes_ctr_ctx_init(otc_aes_ctr_ctx *ctx, const uint8_t nc[16])
{
    memset(ctx, 0, sizeof *ctx);
    memcpy(ctx->nonce_counter, nc, 16);
    return OTC_OK;
}

int otc_aes_ctr_stream(otc_aes_ctr_ctx *ctx, const otc_aes_key *k, size_t n, const void *in, void *out, int, void *)
{
    aes_context c = ctx_of(k);
    int off = (int)ctx->nc_off;
    const uint8_t *pi = (const uint8_t *)in;
    uint8_t *po = (uint8_t *)out;
    while (n) { /* aes_crypt_ctr takes an int length */
        const size_t step = n < (1u << 30) ? n : (1u << 30);
        aes_crypt_ctr(&c, (int)step, &off, ctx->nonce_counter, ctx->stream_block, pi, po);
        pi += step;
        po += step;
        n -= step;
    }
    ctx->nc_off = (size_t)off;
    return OTC_OK;
}

int otc_aes_cbc_decrypt(const void *in, void *out, size_t n, const otc_aes_key *k, const uint8_t iv[16], void *);
int otc_aes_cbc_decrypt_impl(const void *in, void *out, size_t n, const otc_aes_key *k, const uint8_t iv[16], int,
                             void *st)
{
    return otc_aes_cbc_decrypt(in, out, n, k, iv, st);
}
int otc_aes_cbc_decrypt(const void *in, void *out, size_t n, const otc_aes_key *k, const uint8_t iv[16], void *)
{
    if (in == out) return fail(OTC_ERR_ARG, "cbc decrypt in place");
    aes_context c = ctx_of(k);
    uint8_t v[16];
    memcpy(v, iv, 16);
    return aes_crypt_cbc(&c, AES_DECRYPT, n, v, (const uint8_t *)in, (uint8_t *)out);
}

static int segs(int which, const void *in, void *out, size_t seg, size_t nseg, const otc_aes_key *k,
                const uint8_t iv0[16])
{
    aes_context c = ctx_of(k);
    for (size_t s = 0; s < nseg; ++s) {
        uint8_t iv[16];
        memcpy(iv, iv0, 16);
        be_add(iv, s);
        const uint8_t *pi = (const uint8_t *)in + s * seg;
        uint8_t *po = (uint8_t *)out + s * seg;
        int iv_off = 0;
        if (which == 0) aes_crypt_cbc(&c, AES_ENCRYPT, seg, iv, pi, po);
        else if (which == 3) aes_crypt_cbc(&c, AES_DECRYPT, seg, iv, pi, po);
        else aes_crypt_cfb128(&c, which == 1 ? AES_ENCRYPT : AES_DECRYPT, seg, &iv_off, iv, pi, po);
    }
    return OTC_OK;
}

int otc_aes_cbc_encrypt_segments(const void *in, void *out, size_t seg, size_t nseg, const otc_aes_key *k,
                                 const uint8_t iv0[16], void *)
{
    return segs(0, in, out, seg, nseg, k, iv0);
}
int otc_aes_cfb128_encrypt_segments(const void *in, void *out, size_t seg, size_t nseg, const otc_aes_key *k,
                                    const uint8_t iv0[16], void *)
{
    return segs(1, in, out, seg, nseg, k, iv0);
}
int otc_aes_cbc_encrypt_segments_impl(const void *in, void *out, size_t seg, size_t nseg, const otc_aes_key *k,
                                      const uint8_t iv0[16], int, void *st)
{
    return otc_aes_cbc_encrypt_segments(in, out, seg, nseg, k, iv0, st);
}
int otc_aes_cfb128_encrypt_segments_impl(const void *in, void *out, size_t seg, size_t nseg, const otc_aes_key *k,
                                         const uint8_t iv0[16], int, void *st)
{
    return otc_aes_cfb128_encrypt_segments(in, out, seg, nseg, k, iv0, st);
}
int otc_aes_cfb128_decrypt_segments(const void *in, void *out, size_t seg, size_t nseg, const otc_aes_key *k,
                                    const uint8_t iv0[16], void *)
{
    if (in == out) return fail(OTC_ERR_ARG, "cfb decrypt in place");
    return segs(2, in, out, seg, nseg, k, iv0);
}
int otc_aes_cfb128_decrypt_segments_impl(const void *in, void *out, size_t seg, size_t nseg, const otc_aes_key *k,
                                         const uint8_t iv0[16], int, void *st)
{
    return otc_aes_cfb128_decrypt_segments(in, out, seg, nseg, k, iv0, st);
}
int otc_aes_cbc_decrypt_segments_impl(const void *in, void *out, size_t seg, size_t nseg, const otc_aes_key *k,
                                      const uint8_t iv0[16], int, void *)
{
    if (in == out) return fail(OTC_ERR_ARG, "cbc decrypt in place");
    return segs(3, in, out, seg, nseg, k, iv0);
}

int otc_aes_cfb128_decrypt(const void *in, void *out, size_t n, const otc_aes_key *k, const uint8_t iv[16], void *);
int otc_aes_cfb128_decrypt_impl(const void *in, void *out, size_t n, const otc_aes_key *k, const uint8_t iv[16], int,
                                void *st)
{
    return otc_aes_cfb128_decrypt(in, out, n, k, iv, st);
}
int otc_aes_cfb128_decrypt(const void *in, void *out, size_t n, const otc_aes_key *k, const uint8_t iv[16], void *)
{
    if (in == out) return fail(OTC_ERR_ARG, "cfb decrypt in place");
    aes_context c = ctx_of(k);
    uint8_t v[16];
    memcpy(v, iv, 16);
    int iv_off = 0;
    return aes_crypt_cfb128(&c, AES_DECRYPT, n, &iv_off, v, (const uint8_t *)in, (uint8_t *)out);
}

int otc_xor(const void *a, const void *b, void *out, size_t n, void *)
{
    for (size_t i = 0; i < n; ++i) ((uint8_t *)out)[i] = ((const uint8_t *)a)[i] ^ ((const uint8_t *)b)[i];
    return OTC_OK;
}

int otc_rc4_multi(const uint8_t *keys, int keylen, size_t ns, size_t len, size_t drop, const void *in, void *out, void *)
{
    std::vector<uint8_t> ks(drop + len);
    for (size_t s = 0; s < ns; ++s) {
        arc4_context a;
        arc4_setup(&a, keys + s * keylen, (unsigned)keylen);
        arc4_prep(&a, ks.size(), ks.data());
        for (size_t i = 0; i < len; ++i)
            ((uint8_t *)out)[s * len + i] = (in ? ((const uint8_t *)in)[s * len + i] : 0) ^ ks[drop + i];
    }
    return OTC_OK;
}

int otc_fill_random(void *p, size_t n, uint64_t seed, void *)
{
    /* touches one byte per page: sparse mappings stay sparse, the sampled
     * pages still differ */
    uint64_t x = seed * 0x9E3779B97F4A7C15ull + 1;
    for (size_t i = 0; i < n; i += 4096) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        ((uint8_t *)p)[i] = (uint8_t)x;
    }
    return OTC_OK;
}

void *otc_dev_malloc(size_t n)
{
    void *p = mmap(nullptr, n ? n : 1, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
    return p == MAP_FAILED ? nullptr : p;
}
void otc_dev_free(void *) {} /* process exit unmaps; sizes are not tracked */
int otc_memcpy(void *d, const void *s, size_t n, int) { memcpy(d, s, n); return OTC_OK; }
int otc_device_sync(void) { return OTC_OK; }
void *otc_stream_create(void) { return (void *)1; }
void otc_stream_destroy(void *) {}
int otc_stream_join(void *, void *) { return OTC_OK; }

int otc_time_op(otc_op_fn op, void *arg, int iters, double *ms)
{
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < iters; ++i)
        if (int r = op(arg)) return r;
    *ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() / (iters ? iters : 1);
    return OTC_OK;
}
int otc_measure_clock(otc_op_fn, void *, double *ghz)
{
    *ghz = 0.0;
    return OTC_OK;
}
int otc_device_cus(int) { return 1; }
int otc_device_clock_khz(int) { return 1000000; }

void *otc_host_alloc_pinned(size_t n) { return otc_dev_malloc(n); }
void otc_host_free_pinned(void *) {}

struct otc_engine {
    int dummy;
};
otc_engine *otc_engine_create(int, size_t, int) { return new otc_engine{0}; }
void otc_engine_destroy(otc_engine *e) { delete e; }
int otc_engine_run(otc_engine *, int mode, const void *hin, void *hout, size_t n, const otc_aes_key *k,
                   const uint8_t iv[16], uint64_t off, int impl, otc_stream_stats *)
{
    if (mode == OTC_MODE_CTR) return otc_aes_ctr(hin, hout, n, k, iv, off, impl, nullptr);
    if (mode == OTC_MODE_CBC_DEC) return otc_aes_cbc_decrypt(hin, hout, n, k, iv, nullptr);
    if (mode == OTC_MODE_ECB) return otc_aes_ecb(hin, hout, n, k, impl, nullptr);
    return fail(OTC_ERR_ARG, "engine mode");
}
int otc_multi_run(int, int, int mode, const void *hin, void *hout, size_t n, const otc_aes_key *k,
                  const uint8_t iv[16], int impl, size_t, otc_multi_stats *)
{
    return otc_engine_run(nullptr, mode, hin, hout, n, k, iv, 0, impl, nullptr);
}

} // extern "C"
