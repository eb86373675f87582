/*
 * otbench.cpp -> bin/otbench : general benchmark / profiling driver for the
 * gfx950 kernels (the profiling target for rocprofv3).  Prints one JSON line
 * per configuration.
 *
 *   otbench --mode ctr|ecb|ecb-dec|cbc-dec|cbc-enc-seg|cfb-enc-seg|cfb-dec-seg|cbc-dec-seg|cfb-dec|ctr-stream|xor|rc4
 *                  |ecb-split|ecbdec-split|cbcdec-split|cfbdec-split|ctr-split
 *           [--bits 128] [--bytes 1G] [--iters 20] [--warmup 3]
 *           [--impl auto|ttable|bitslice|split] [--inplace] [--verify] [--clock]
 *           [--mark]                        "OTB_MARK start|end" on stderr around the timed loop
 *           [--strace]                      diagnostic builds (OTC_SPLIT_TRACE): wave start times of a split
 *           [--split-stats]                 one extra call after the loop: units each side of a
 *                                           split took ("split_units": [bitsliced, T-table, all])
 *           [--corrupt-at OFF]              test hook: flip output byte OFF after the
 *                                           verified op (verification must then fail)
 *           [--e2e --chunk 256M]            host-resident, pinned pipeline
 *           [--gpus N --strategy direct|rccl] single-process multi-GPU (e2e)
 *           [--seg 4096]                    CBC segment size
 *           [--share 0.2]                   *-split: the bitsliced kernel's share of the
 *                                           blocks, run CONCURRENTLY with the T-table kernel
 *                                           on the rest (two streams, co-resident per CU) --
 *                                           the library's impl "split" with an explicit share
 *           [--streams 65536 --len 4096 --keylen 16 --drop 0]    RC4 many-stream shape
 *
 * Kernel-only numbers come from hipEvents around `iters` back-to-back launches
 * on resident data (no allocation, no copies in the timed region: contrast the
 * reference's timing of malloc+pageable copies, main_ecb_e.cu:37-44).
 *
 * --verify checks the FIRST op of the run against the C oracle (whose own
 * tests pin it to FIPS-197, SP 800-38A, RFC 3686 and the reference's
 * Monte-Carlo KATs, /root/reference/aes-modes/aes.c:912-1078): before that op
 * the input of several samples (head, middle, tail, and the 2^32-byte boundary
 * of buffers above 4 GiB; whole segments / whole RC4 streams for the chained
 * modes) is copied to the host, so in-place runs are verified too.  Every mode
 * has an oracle; "verified" is true only when every sample matched, false when
 * one did not (exit 3), and null when --verify was not given.
 */
#include <algorithm>
#include <chrono>
#include <cinttypes>
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

static size_t parse_size(const char *s)
{
    char *e;
    double v = strtod(s, &e);
    switch (*e) {
    case 'k': case 'K': v *= 1024.0; break;
    case 'm': case 'M': v *= 1024.0 * 1024.0; break;
    case 'g': case 'G': v *= 1024.0 * 1024.0 * 1024.0; break;
    default: break;
    }
    return (size_t)v;
}

struct Cfg {
    std::string mode = "ctr";
    int bits = 128;
    size_t bytes = 1ull << 30;
    int iters = 20, warmup = 3;
    int impl = OTC_IMPL_AUTO;
    bool inplace = false, verify = false, e2e = false, clock = false, mark = false, split_stats = false, strace = false;
    long long corrupt_at = -1;
    size_t chunk = 256ull << 20;
    int gpus = 1, strategy = 0;
    size_t seg = 4096;
    double share = 0.2;
    size_t streams = 65536, len = 4096, keylen = 16, drop = 0;
};

struct OpArg {
    Cfg *c;
    void *in, *out;
    otc_aes_key *k;
    uint8_t iv[16];
    uint8_t *keys;
    void *sa, *sb; /* *-split: T-table / bitsliced streams */
    uint8_t prev[16]; /* cbcdec-split / cfbdec-split: ciphertext block before the bitsliced part */
};

static bool is_split(const std::string &m)
{
    return m == "ecb-split" || m == "ecbdec-split" || m == "cbcdec-split" || m == "cfbdec-split" || m == "ctr-split";
}

/* *-split: T-table bytes (the bitsliced part is whole 2048-block tasks, as
 * the library's split) */
static size_t split_nt(const Cfg &c)
{
    const size_t nb = (size_t)((double)(c.bytes / 16) * c.share) / 2048 * 2048;
    return c.bytes - 16 * std::min(nb, c.bytes / 16);
}

static int run_op(void *p)
{
    OpArg *a = (OpArg *)p;
    const Cfg &c = *a->c;
    if (c.mode == "ctr") return otc_aes_ctr(a->in, a->out, c.bytes, a->k, a->iv, 0, c.impl, nullptr);
    if (c.mode == "ecb" || c.mode == "ecb-dec") return otc_aes_ecb(a->in, a->out, c.bytes, a->k, c.impl, nullptr);
    if (is_split(c.mode)) {
        /* both streams are ordered with the default stream (otc_stream_create);
         * each call ends with a join (otc_stream_join), as the library's split
         * does -- without it the two parts of successive calls drift apart and
         * a badly balanced share hides its tail (profiles/r4/split_trace) */
        const size_t nt = split_nt(c);
        struct Join {
            const OpArg *a;
            ~Join() { (void)otc_stream_join(a->sa, a->sb); }
        } join{a};
        const uint8_t *bi = (const uint8_t *)a->in + nt;
        uint8_t *bo = (uint8_t *)a->out + nt;
        if (c.mode == "cbcdec-split") {
            if (int r = otc_aes_cbc_decrypt_impl(a->in, a->out, nt, a->k, a->iv, OTC_IMPL_TTABLE, a->sa)) return r;
            return otc_aes_cbc_decrypt_impl(bi, bo, c.bytes - nt, a->k, a->prev, OTC_IMPL_BITSLICE, a->sb);
        }
        if (c.mode == "ctr-split") { /* the bitsliced part continues the counter at block nt/16 */
            if (int r = otc_aes_ctr(a->in, a->out, nt, a->k, a->iv, 0, OTC_IMPL_TTABLE, a->sa)) return r;
            return otc_aes_ctr(bi, bo, c.bytes - nt, a->k, a->iv, nt / 16, OTC_IMPL_BITSLICE, a->sb);
        }
        if (c.mode == "cfbdec-split") {
            if (int r = otc_aes_cfb128_decrypt_impl(a->in, a->out, nt, a->k, a->iv, OTC_IMPL_TTABLE, a->sa)) return r;
            return otc_aes_cfb128_decrypt_impl(bi, bo, c.bytes - nt, a->k, a->prev, OTC_IMPL_BITSLICE, a->sb);
        }
        if (int r = otc_aes_ecb(a->in, a->out, nt, a->k, OTC_IMPL_TTABLE, a->sa)) return r;
        return otc_aes_ecb(bi, bo, c.bytes - nt, a->k, OTC_IMPL_BITSLICE, a->sb);
    }
    if (c.mode == "cbc-dec")
        return otc_aes_cbc_decrypt_impl(a->in, a->out, c.bytes, a->k, a->iv, c.impl, nullptr);
    if (c.mode == "cbc-enc-seg")
        return otc_aes_cbc_encrypt_segments_impl(a->in, a->out, c.seg, c.bytes / c.seg, a->k, a->iv, c.impl, nullptr);
    if (c.mode == "ctr-stream") { /* resumed mid-block: 1-byte head, then a body misaligned by 1 */
        otc_aes_ctr_ctx ctx;
        otc_aes_ctr_ctx_init(&ctx, a->iv);
        ctx.nc_off = 15;
        return otc_aes_ctr_stream(&ctx, a->k, c.bytes, a->in, a->out, c.impl, nullptr);
    }
    if (c.mode == "cfb-enc-seg")
        return otc_aes_cfb128_encrypt_segments_impl(a->in, a->out, c.seg, c.bytes / c.seg, a->k, a->iv, c.impl,
                                                    nullptr);
    if (c.mode == "cfb-dec-seg")
        return otc_aes_cfb128_decrypt_segments_impl(a->in, a->out, c.seg, c.bytes / c.seg, a->k, a->iv, c.impl, nullptr);
    if (c.mode == "cbc-dec-seg")
        return otc_aes_cbc_decrypt_segments_impl(a->in, a->out, c.seg, c.bytes / c.seg, a->k, a->iv, c.impl, nullptr);
    if (c.mode == "cfb-dec") return otc_aes_cfb128_decrypt_impl(a->in, a->out, c.bytes, a->k, a->iv, c.impl, nullptr);
    if (c.mode == "xor") return otc_xor(a->in, a->out, a->out, c.bytes, nullptr);
    if (c.mode == "rc4") return otc_rc4_multi(a->keys, (int)c.keylen, c.streams, c.len, c.drop, a->in, a->out, nullptr);
    return OTC_ERR_ARG;
}

/* ---- verification ---------------------------------------------------------
 * A Sample is an output range [off, off + len) plus everything the oracle
 * needs to recompute it, copied to the host BEFORE the verified op ran. */
struct Sample {
    size_t off = 0, len = 0;
    size_t pre = 0;              /* predecessor bytes in `in` before off (chained decrypts) */
    std::vector<uint8_t> in;     /* input [off - pre, off + len) */
    std::vector<uint8_t> old;    /* xor: output bytes before the op */
    std::vector<uint8_t> key;    /* rc4: the stream's key */
    uint64_t seg0 = 0;           /* segment modes: index of the first segment */
};

static bool is_seg_mode(const std::string &m)
{
    return m == "cbc-enc-seg" || m == "cfb-enc-seg" || m == "cfb-dec-seg" || m == "cbc-dec-seg";
}
static bool chained_dec(const std::string &m)
{
    return m == "cbc-dec" || m == "cfb-dec" || m == "cbcdec-split" || m == "cfbdec-split";
}

/* sample output ranges: head, middle, tail, and the 2^32-byte boundary (32-bit
 * byte-offset overflow) when the buffer is larger than 4 GiB */
static std::vector<std::pair<size_t, size_t>> sample_ranges(const Cfg &c)
{
    std::vector<std::pair<size_t, size_t>> r;
    if (c.mode == "rc4") { /* whole streams: first, middle, last */
        const size_t ss[3] = {0, c.streams / 2, c.streams - 1};
        for (size_t s : ss) r.push_back({s * c.len, c.len});
    } else if (is_seg_mode(c.mode)) { /* whole segments */
        const size_t nseg = c.bytes / c.seg, k = std::max<size_t>(1, std::min<size_t>(nseg, (64u << 10) / c.seg));
        const size_t s0[3] = {0, (nseg - k) / 2, nseg - k};
        for (size_t s : s0) r.push_back({s * c.seg, k * c.seg});
        if (c.bytes > (4ull << 30) + k * c.seg) r.push_back({((4ull << 30) / c.seg) * c.seg - c.seg, 2 * c.seg});
    } else {
        const size_t S = std::min<size_t>(c.bytes, 64 << 10);
        /* samples start on a block boundary of the mode: 16m, or 1 + 16m for
         * ctr-stream (its body starts after a 1-byte head) */
        const size_t b = c.mode == "ctr-stream" ? 1 : 0;
        auto down = [&](size_t o) { return o < b ? 0 : ((o - b) / 16) * 16 + b; };
        r.push_back({0, S});
        const size_t m = down((c.bytes - S) / 2);
        r.push_back({m, std::min(S, c.bytes - m)});
        const size_t t = down(c.bytes - S);
        r.push_back({t, c.bytes - t});
        if (c.bytes > (4ull << 30) + S) r.push_back({down((4ull << 30) - S / 2), S});
    }
    return r;
}

using CopyFn = int (*)(void *dst, const void *src, size_t n); /* from the buffers under test to the host */
static int copy_d2h(void *d, const void *s, size_t n) { return otc_memcpy(d, s, n, OTC_D2H); }
static int copy_h2h(void *d, const void *s, size_t n) { memcpy(d, s, n); return 0; }

static bool snapshot(const Cfg &c, const OpArg &a, CopyFn cp, std::vector<Sample> &out)
{
    for (auto [off, len] : sample_ranges(c)) {
        Sample s;
        s.off = off;
        s.len = len;
        s.pre = (chained_dec(c.mode) && off >= 16) ? 16 : 0;
        s.in.resize(s.pre + len);
        if (cp(s.in.data(), (const uint8_t *)a.in + off - s.pre, s.pre + len)) return false;
        if (c.mode == "xor") {
            s.old.resize(len);
            if (cp(s.old.data(), (const uint8_t *)a.out + off, len)) return false;
        }
        if (c.mode == "rc4") {
            s.key.resize(c.keylen);
            if (cp(s.key.data(), a.keys + (off / c.len) * c.keylen, c.keylen)) return false;
        }
        if (is_seg_mode(c.mode)) s.seg0 = off / c.seg;
        out.push_back(std::move(s));
    }
    return true;
}

/* the oracle's output for one sample; false if the mode has no oracle */
static bool oracle(const Cfg &c, const uint8_t key[32], const uint8_t iv0[16], const Sample &s, std::vector<uint8_t> &ref)
{
    ref.assign(s.len, 0);
    const uint8_t *in = s.in.data() + s.pre;
    aes_context ctx;
    const std::string &m = c.mode;
    if (m == "ctr" || m == "ctr-split") {
        aes_setkey_enc(&ctx, key, c.bits);
        uint8_t nc[16];
        memcpy(nc, iv0, 16);
        aes_ctr128_add(nc, s.off / 16);
        aes_ctr_bulk(&ctx, nc, in, ref.data(), s.len, 8);
    } else if (m == "ctr-stream") {
        /* the run's context: nc_off 15 with a zero stream block, so data byte 0
         * passes through and byte p >= 1 uses keystream byte (p - 1) of the
         * counter stream started at iv0; samples start at p = 0 or 1 + 16m */
        aes_setkey_enc(&ctx, key, c.bits);
        uint8_t nc[16], sb[16] = {0};
        memcpy(nc, iv0, 16);
        int nc_off = 15;
        if (s.off) {
            aes_ctr128_add(nc, (s.off - 1) / 16);
            nc_off = 0;
        }
        aes_crypt_ctr(&ctx, (int)s.len, &nc_off, nc, sb, in, ref.data());
    } else if (m == "ecb" || m == "ecb-split") {
        aes_setkey_enc(&ctx, key, c.bits);
        aes_ecb_bulk(&ctx, AES_ENCRYPT, in, ref.data(), s.len, 8);
    } else if (m == "ecb-dec" || m == "ecbdec-split") {
        aes_setkey_dec(&ctx, key, c.bits);
        aes_ecb_bulk(&ctx, AES_DECRYPT, in, ref.data(), s.len, 8);
    } else if (chained_dec(m)) {
        uint8_t iv[16];
        memcpy(iv, s.off ? s.in.data() : iv0, 16);
        if (m == "cbc-dec" || m == "cbcdec-split") {
            aes_setkey_dec(&ctx, key, c.bits);
            aes_crypt_cbc(&ctx, AES_DECRYPT, s.len, iv, in, ref.data());
        } else {
            aes_setkey_enc(&ctx, key, c.bits);
            int iv_off = 0;
            aes_crypt_cfb128(&ctx, AES_DECRYPT, s.len, &iv_off, iv, in, ref.data());
        }
    } else if (is_seg_mode(m)) {
        /* segment q: IV_q = iv0 + q (128-bit BE add), its own chain */
        if (m == "cbc-dec-seg")
            aes_setkey_dec(&ctx, key, c.bits);
        else
            aes_setkey_enc(&ctx, key, c.bits); /* CBC encrypt; CFB uses E() both ways */
        for (size_t q = 0; q < s.len / c.seg; ++q) {
            uint8_t iv[16];
            memcpy(iv, iv0, 16);
            aes_ctr128_add(iv, s.seg0 + q);
            const uint8_t *qi = in + q * c.seg;
            uint8_t *qo = ref.data() + q * c.seg;
            if (m == "cbc-enc-seg" || m == "cbc-dec-seg") {
                aes_crypt_cbc(&ctx, m == "cbc-enc-seg" ? AES_ENCRYPT : AES_DECRYPT, c.seg, iv, qi, qo);
            } else {
                int iv_off = 0;
                aes_crypt_cfb128(&ctx, m == "cfb-enc-seg" ? AES_ENCRYPT : AES_DECRYPT, c.seg, &iv_off, iv, qi, qo);
            }
        }
    } else if (m == "xor") {
        for (size_t i = 0; i < s.len; ++i) ref[i] = in[i] ^ s.old[i];
    } else if (m == "rc4") {
        arc4_context a4;
        arc4_setup(&a4, s.key.data(), (unsigned)c.keylen);
        std::vector<uint8_t> ks(c.drop + s.len);
        arc4_prep(&a4, ks.size(), ks.data());
        for (size_t i = 0; i < s.len; ++i) ref[i] = in[i] ^ ks[c.drop + i];
    } else {
        return false;
    }
    return true;
}

/* 1: every sample matched, 0: a mismatch (message on stderr), -1: no oracle
 * or a copy failed (reported as not verified) */
static int check_samples(const Cfg &c, const OpArg &a, CopyFn cp, const uint8_t key[32],
                         const std::vector<Sample> &samples)
{
    if (samples.empty()) return -1;
    for (const Sample &s : samples) {
        std::vector<uint8_t> got(s.len), ref;
        if (cp(got.data(), (const uint8_t *)a.out + s.off, s.len)) return -1;
        if (!oracle(c, key, a.iv, s, ref)) return -1;
        if (memcmp(got.data(), ref.data(), s.len) != 0) {
            size_t i = 0;
            while (got[i] == ref[i]) ++i;
            fprintf(stderr, "verify: %s mismatch at byte %zu (sample at %zu, %zu bytes)\n", c.mode.c_str(),
                    s.off + i, s.off, s.len);
            return 0;
        }
    }
    return 1;
}

/* test hook: flip one output byte (through the same copies as the check) */
static int corrupt(void *out, size_t off, bool device)
{
    uint8_t v;
    if (device) {
        if (otc_memcpy(&v, (uint8_t *)out + off, 1, OTC_D2H)) return 1;
        v ^= 0x5A;
        return otc_memcpy((uint8_t *)out + off, &v, 1, OTC_H2D);
    }
    ((uint8_t *)out)[off] ^= 0x5A;
    return 0;
}

/* the HIP runtime / RCCL this process is bound to (otc_runtime_info): every
 * record says which, so A/Bs across the /opt/rocm and torch runtimes are
 * never compared unawares */
static std::string runtime_json()
{
    char buf[1024];
    return otc_runtime_info(buf, sizeof buf) == OTC_OK ? std::string(buf) : std::string("null");
}

/* --mark lines, flushed at once: on the GPU box the runtime leaves stderr
 * buffered, and a mark that arrives late shrinks the power window */
static void mark(const char *what)
{
    fprintf(stderr, "OTB_MARK %s\n", what);
    fflush(stderr);
}

static const char *verdict(bool asked, int v) { return !asked ? "null" : v == 1 ? "true" : "false"; }

int main(int argc, char **argv)
{
    Cfg c;
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        auto nx = [&]() -> const char * { return i + 1 < argc ? argv[++i] : ""; };
        if (a == "--mode") c.mode = nx();
        else if (a == "--bits") c.bits = atoi(nx());
        else if (a == "--bytes") c.bytes = parse_size(nx());
        else if (a == "--iters") c.iters = atoi(nx());
        else if (a == "--warmup") c.warmup = atoi(nx());
        else if (a == "--impl") {
            std::string v = nx();
            if (v != "auto" && v != "ttable" && v != "bitslice" && v != "split") {
                fprintf(stderr, "--impl must be auto, ttable, bitslice or split\n");
                return 2;
            }
            c.impl = v == "ttable" ? OTC_IMPL_TTABLE : v == "bitslice" ? OTC_IMPL_BITSLICE
                   : v == "split"  ? OTC_IMPL_SPLIT  : OTC_IMPL_AUTO;
        } else if (a == "--inplace") c.inplace = true;
        else if (a == "--verify") c.verify = true;
        else if (a == "--clock") c.clock = true;
        else if (a == "--mark") c.mark = true;
        else if (a == "--split-stats") c.split_stats = true;
        else if (a == "--strace") c.strace = true;
        else if (a == "--corrupt-at") c.corrupt_at = atoll(nx());
        else if (a == "--e2e") c.e2e = true;
        else if (a == "--chunk") c.chunk = parse_size(nx());
        else if (a == "--gpus") c.gpus = atoi(nx());
        else if (a == "--strategy") c.strategy = std::string(nx()) == "rccl" ? 1 : 0;
        else if (a == "--seg") c.seg = parse_size(nx());
        else if (a == "--share") c.share = atof(nx());
        else if (a == "--streams") c.streams = parse_size(nx());
        else if (a == "--len") c.len = parse_size(nx());
        else if (a == "--keylen") c.keylen = parse_size(nx());
        else if (a == "--drop") c.drop = parse_size(nx());
        else {
            fprintf(stderr, "unknown option %s\n", a.c_str());
            return 2;
        }
    }
    static const char *modes[] = {"ctr", "ecb", "ecb-dec", "cbc-dec", "cbc-enc-seg", "cfb-enc-seg", "cfb-dec-seg",
                                  "cbc-dec-seg",
                                  "cfb-dec", "ctr-stream", "xor", "rc4", "ecb-split", "ecbdec-split", "cbcdec-split",
                                  "cfbdec-split", "ctr-split"};
    bool known = false;
    for (const char *m : modes) known |= c.mode == m;
    if (!known) {
        fprintf(stderr, "unknown mode %s\n", c.mode.c_str());
        return 2;
    }
    if (c.mode == "rc4") c.bytes = c.streams * c.len;
    if (c.mode != "ctr" && c.mode != "ctr-stream" && c.mode != "xor" && c.mode != "rc4") c.bytes &= ~(size_t)15;
    if (is_seg_mode(c.mode)) {
        if (c.seg == 0 || c.seg % 16) {
            fprintf(stderr, "--seg must be a positive multiple of 16\n");
            return 2;
        }
        c.bytes = (c.bytes / c.seg) * c.seg;
    }
    if (c.bytes == 0) {
        fprintf(stderr, "--bytes leaves nothing to process\n");
        return 2;
    }
    if (c.inplace && (chained_dec(c.mode) || c.mode == "cfb-dec-seg" || c.mode == "cbc-dec-seg")) {
        /* these read the previous ciphertext block: the library refuses in-place */
        fprintf(stderr, "%s cannot run in place\n", c.mode.c_str());
        return 2;
    }
    if (c.e2e && c.mode != "ctr" && c.mode != "ecb" && c.mode != "cbc-dec") {
        fprintf(stderr, "--e2e supports ctr, ecb and cbc-dec only\n");
        return 2;
    }

    uint8_t key[32];
    srand(1337);
    for (int i = 0; i < 32; ++i) key[i] = (uint8_t)rand();
    const bool dec = (c.mode == "ecb-dec" || c.mode == "cbc-dec" || c.mode == "ecbdec-split" ||
                      c.mode == "cbcdec-split" || c.mode == "cbc-dec-seg");
    otc_aes_key k;
    if (otc_aes_key_init(&k, key, c.bits, dec ? OTC_DIR_DECRYPT : OTC_DIR_ENCRYPT)) {
        fprintf(stderr, "key: %s\n", otc_last_error());
        return 1;
    }
    OpArg a{};
    a.c = &c;
    a.k = &k;
    for (int i = 0; i < 16; ++i) a.iv[i] = (uint8_t)(0xF0 + i);

    const int cus = otc_device_cus(0);
    const double clk_hz = otc_device_clock_khz(0) * 1e3;
    double ms = 0.0;

    if (c.e2e) {
        /* host-resident data through the pinned pipeline (1 GPU) or the
         * multi-GPU planner */
        uint8_t *hin = (uint8_t *)otc_host_alloc_pinned(c.bytes), *hout = (uint8_t *)otc_host_alloc_pinned(c.bytes);
        if (!hin || !hout) {
            fprintf(stderr, "pinned alloc failed\n");
            return 1;
        }
        for (size_t i = 0; i < c.bytes; i += 4096) hin[i] = (uint8_t)(i >> 12);
        a.in = hin;
        a.out = hout;
        std::vector<Sample> samples;
        if (c.verify && !snapshot(c, a, copy_h2h, samples)) return 1;
        int mode = c.mode == "ctr" ? OTC_MODE_CTR : c.mode == "cbc-dec" ? OTC_MODE_CBC_DEC : OTC_MODE_ECB;
        otc_engine *eng = (c.gpus > 1 || c.strategy == 1) ? nullptr : otc_engine_create(0, c.chunk, 3);
        int v = -1;
        for (int w = 0; w <= c.warmup; ++w) {
            if (c.mark && w == c.warmup) mark("start");
            auto t0 = std::chrono::steady_clock::now();
            int r;
            if (c.gpus > 1 || c.strategy == 1) {
                otc_multi_stats st{};
                r = otc_multi_run(c.gpus, c.strategy, mode, hin, hout, c.bytes, &k, a.iv, c.impl, c.chunk, &st);
            } else {
                r = eng ? otc_engine_run(eng, mode, hin, hout, c.bytes, &k, a.iv, 0, c.impl, nullptr) : OTC_ERR_NOMEM;
            }
            auto t1 = std::chrono::steady_clock::now();
            if (c.mark && w == c.warmup) mark("end");
            if (r) {
                fprintf(stderr, "run: %s\n", otc_last_error());
                return 1;
            }
            if (w == 0 && c.verify) { /* out of place: the input never changes */
                if (c.corrupt_at >= 0 && corrupt(hout, (size_t)c.corrupt_at, false)) return 1;
                v = check_samples(c, a, copy_h2h, key, samples);
            }
            ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
        }
        printf("{\"mode\": \"%s\", \"bits\": %d, \"bytes\": %zu, \"e2e\": true, \"gpus\": %d, \"strategy\": \"%s\", "
               "\"chunk\": %zu, \"ms\": %.3f, \"gbps\": %.3f, \"runtime\": %s, \"verified\": %s}\n",
               c.mode.c_str(), c.bits, c.bytes, c.gpus, c.strategy ? "rccl" : "direct", c.chunk, ms,
               c.bytes / (ms * 1e6), runtime_json().c_str(), verdict(c.verify, v));
        otc_engine_destroy(eng);
        otc_host_free_pinned(hin);
        otc_host_free_pinned(hout);
        return (c.verify && v != 1) ? 3 : 0;
    }

    if (is_split(c.mode)) {
        if (!(c.share >= 0.0 && c.share <= 1.0)) {
            fprintf(stderr, "--share must be in [0, 1]\n");
            return 2;
        }
        a.sa = otc_stream_create();
        a.sb = otc_stream_create();
        if (!a.sa || !a.sb) {
            fprintf(stderr, "stream: %s\n", otc_last_error());
            return 1;
        }
    }
    a.in = otc_dev_malloc(c.bytes);
    a.out = c.inplace ? a.in : otc_dev_malloc(c.bytes);
    if (!a.in || !a.out) {
        fprintf(stderr, "device alloc failed: %s\n", otc_last_error());
        return 1;
    }
    otc_fill_random(a.in, c.bytes, 42, nullptr);
    if (!c.inplace) otc_fill_random(a.out, c.bytes, 43, nullptr);
    if (c.mode == "rc4") {
        a.keys = (uint8_t *)otc_dev_malloc(c.streams * c.keylen);
        otc_fill_random(a.keys, c.streams * c.keylen, 44, nullptr);
    }
    otc_device_sync();
    if (c.mode == "cbcdec-split" || c.mode == "cfbdec-split") {
        /* the bitsliced part's IV: ciphertext block nt/16 - 1 (constant: out of place) */
        const size_t nt = split_nt(c);
        if (nt >= 16) {
            if (otc_memcpy(a.prev, (const uint8_t *)a.in + nt - 16, 16, OTC_D2H)) return 1;
        } else {
            memcpy(a.prev, a.iv, 16);
        }
    }
    int v = -1;
    if (c.verify) {
        /* the inputs of the samples are copied BEFORE the op: valid in place */
        std::vector<Sample> samples;
        if (!snapshot(c, a, copy_d2h, samples)) {
            fprintf(stderr, "verify snapshot: %s\n", otc_last_error());
            return 1;
        }
        if (run_op(&a) || otc_device_sync()) {
            fprintf(stderr, "op: %s\n", otc_last_error());
            return 1;
        }
        if (c.corrupt_at >= 0 && corrupt(a.out, (size_t)c.corrupt_at, true)) return 1;
        v = check_samples(c, a, copy_d2h, key, samples);
    }
    for (int w = 0; w < c.warmup; ++w)
        if (run_op(&a)) {
            fprintf(stderr, "op: %s\n", otc_last_error());
            return 1;
        }
    if (c.mark) {
        otc_device_sync();
        mark("start");
    }
    if (otc_time_op(run_op, &a, c.iters, &ms)) {
        fprintf(stderr, "timing: %s\n", otc_last_error());
        return 1;
    }
    if (c.mark) mark("end");
    char split_units[96] = "";
    if (c.strace) { /* diagnostic builds: when each kernel's waves started, one more call */
        std::vector<unsigned long long> rec(2 * 16384);
        for (int w = 0; w < 2; ++w) (void)otc_split_trace(w, rec.data(), 16384); /* reset */
        if (run_op(&a) || otc_device_sync()) return 1;
        unsigned long long t0 = ~0ull;
        std::vector<std::vector<unsigned long long>> st(2);
        std::vector<unsigned long long> ends; /* tag 5: a T-table claim wave out of units */
        for (int w = 0; w < 2; ++w) {
            const int n = otc_split_trace(w, rec.data(), 16384);
            for (int i = 0; i < n; ++i) {
                if ((rec[2 * i + 1] >> 32) == 5) {
                    ends.push_back(rec[2 * i]);
                    continue;
                }
                st[w].push_back(rec[2 * i]);
                if (w == 0) t0 = std::min(t0, rec[2 * i]);
            }
        }
        if (!ends.empty() && t0 != ~0ull) {
            std::sort(ends.begin(), ends.end());
            auto us = [&](unsigned long long t) { return ((double)t - (double)t0) / 100.0; };
            fprintf(stderr, "strace ttable ends: %zu waves, end (us after the first T-table wave) min %.1f p10 %.1f median %.1f p90 %.1f max %.1f\n",
                    ends.size(), us(ends.front()), us(ends[ends.size() / 10]), us(ends[ends.size() / 2]),
                    us(ends[ends.size() * 9 / 10]), us(ends.back()));
        }
        for (int w = 0; w < 2; ++w) {
            auto &v = st[w];
            if (v.empty()) continue;
            std::sort(v.begin(), v.end());
            auto us = [&](unsigned long long t) { return t0 == ~0ull ? 0.0 : ((double)t - (double)t0) / 100.0; };
            fprintf(stderr, "strace %s: %zu waves, start (us after the first T-table wave) min %.1f median %.1f p90 %.1f max %.1f\n",
                    w == 0 ? "ttable" : "bitslice", v.size(), us(v.front()), us(v[v.size() / 2]),
                    us(v[v.size() * 9 / 10]), us(v.back()));
        }
    }
    const double gbps = c.bytes / (ms * 1e6);
    if (c.split_stats) { /* one more call, after the timed loop: which side took how many units */
        uint64_t f = 0, b = 0, n = 0;
        otc_split_stats(1);
        const int rs = run_op(&a) || otc_split_last_units(&f, &b, &n);
        otc_split_stats(0);
        if (rs) {
            fprintf(stderr, "split stats: %s\n", otc_last_error());
            return 1;
        }
        snprintf(split_units, sizeof split_units, "\"split_units\": [%" PRIu64 ", %" PRIu64 ", %" PRIu64 "], ", f, b, n);
    }
    const double cpb = (ms * 1e-3) * clk_hz * cus / (double)c.bytes;
    double held = 0.0;
    if (c.clock && otc_measure_clock(run_op, &a, &held)) {
        fprintf(stderr, "clock: %s\n", otc_last_error());
        return 1;
    }
    char clk[320] = "";
    if (c.clock)
        snprintf(clk, sizeof clk, "\"held_clock_ghz\": %.3f, \"cycles_per_byte_per_cu_held\": %.3f, ", held,
                 (ms * 1e-3) * held * 1e9 * cus / (double)c.bytes);
    strncat(clk, split_units, sizeof clk - strlen(clk) - 1);
    if (c.mode.size() > 6 && c.mode.compare(c.mode.size() - 6, 6, "-split") == 0)
        snprintf(clk + strlen(clk), sizeof clk - strlen(clk), "\"share\": %.3f, ", c.share);
    const int ran = otc_last_impl(); /* what the last timed call ran (this thread) */
    printf("{\"mode\": \"%s\", \"bits\": %d, \"bytes\": %zu, \"impl\": \"%s\", \"ran\": \"%s\", \"inplace\": %s, "
           "\"iters\": %d, \"ms\": %.4f, \"gbps\": %.2f, \"cycles_per_byte_per_cu\": %.3f, \"cus\": %d, \"clock_mhz\": %.0f, %s"
           "\"runtime\": %s, \"verified\": %s}\n",
           c.mode.c_str(), c.bits, c.bytes,
           c.impl == OTC_IMPL_TTABLE ? "ttable" : c.impl == OTC_IMPL_BITSLICE ? "bitslice"
           : c.impl == OTC_IMPL_SPLIT    ? "split"  : "auto",
           ran == OTC_IMPL_TTABLE ? "ttable" : ran == OTC_IMPL_BITSLICE ? "bitslice" : ran == OTC_IMPL_SPLIT ? "split"
                                                                                                          : "auto",
           c.inplace ? "true" : "false", c.iters, ms, gbps, cpb, cus, clk_hz / 1e6, clk, runtime_json().c_str(),
           verdict(c.verify, v));
    otc_dev_free(a.in);
    if (!c.inplace) otc_dev_free(a.out);
    otc_dev_free(a.keys);
    otc_stream_destroy(a.sa);
    otc_stream_destroy(a.sb);
    return (c.verify && v != 1) ? 3 : 0;
}
