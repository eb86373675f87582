/*
 * engine.cpp -- host runtime of the MI355X cipher engine (C API in otc.h).
 *
 * Replaces the reference's BlockCipher/AES host class
 * (/root/reference/aes-gpu/Source/AES.cu:50-282), which did a synchronous
 * cudaMalloc -> pageable H2D -> launch -> D2H -> cudaFree per call, queried
 * device properties inside the timed region and never checked an error.
 * Here:
 *   - kernels are launched asynchronously on the caller's stream with the
 *     expanded key as a by-value kernel argument (no per-call copies);
 *   - the streaming engine (otc_engine_*) owns a pinned staging ring and three
 *     HIP streams per device, so H2D(k+1) | kernel(k) | D2H(k-1) overlap;
 *   - the multi-GPU path (otc_multi_*) shards one stream over devices, either
 *     by direct per-GPU ingest or by an RCCL scatter/gather over xGMI from a
 *     root GPU, with CTR counter offsets and CBC halos computed by the planner.
 */
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cstdint>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "aes.h"
#include "otc.h"
#include "otc_aesni.h"
#include "otc_device.h"

using otc_dev::Ctr128;

namespace otc_impl {
hipError_t tt_ecb_encrypt(const void *, void *, uint64_t, const otc_aes_key &, hipStream_t);
hipError_t tt_ecb_decrypt(const void *, void *, uint64_t, const otc_aes_key &, hipStream_t);
hipError_t tt_ctr(const void *, void *, size_t, const otc_aes_key &, Ctr128, bool, hipStream_t);
hipError_t tt_cfb_decrypt(const void *, void *, uint64_t, const otc_aes_key &, const uint32_t *, hipStream_t);
hipError_t tt_cbc_decrypt(const void *, void *, uint64_t, const otc_aes_key &, Ctr128, hipStream_t);
hipError_t tt_cbc_decrypt_seg(const void *, void *, uint64_t, uint64_t, const otc_aes_key &, Ctr128, hipStream_t);
hipError_t tt_cbc_encrypt_seg(const void *, void *, uint64_t, uint64_t, const otc_aes_key &, Ctr128, hipStream_t);
hipError_t bs_ctr(const void *, void *, size_t, const otc_aes_key &, Ctr128, bool, hipStream_t);
hipError_t bs_ecb_encrypt(const void *, void *, uint64_t, const otc_aes_key &, hipStream_t);
hipError_t tt_ctr_batch(const otc_ctr_msg *, const otc_aes_key *, const uint32_t *, const uint64_t *, uint64_t, int, int,
                        hipStream_t);
void tt_set_wg_per_cu(int);
hipError_t k_xor(const void *, const void *, void *, size_t, hipStream_t);
hipError_t k_fill_random(void *, size_t, uint64_t, hipStream_t);
hipError_t k_checksum(const void *, size_t, uint64_t *, hipStream_t);
hipError_t k_clock(uint64_t *, uint64_t, uint64_t, hipStream_t);
hipError_t k_rc4_multi(const uint8_t *, int, size_t, size_t, size_t, const void *, void *, hipStream_t);
} // namespace otc_impl

/* ------------------------------------------------------------------------- */
namespace {

thread_local std::string g_err;

int set_err(int code, const std::string &msg)
{
    g_err = msg;
    return code;
}

int hip_fail(hipError_t e, const char *what)
{
    return set_err(OTC_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

#define HIPCHK(expr)                                          \
    do {                                                      \
        hipError_t _e = (expr);                               \
        if (_e != hipSuccess) return hip_fail(_e, #expr);     \
    } while (0)

#define RCCLCHK(expr)                                                                      \
    do {                                                                                   \
        ncclResult_t _r = (expr);                                                          \
        if (_r != ncclSuccess)                                                             \
            return set_err(OTC_ERR_RCCL, std::string(#expr) + ": " + ncclGetErrorString(_r)); \
    } while (0)

Ctr128 ctr_from_bytes(const uint8_t c[16])
{
    Ctr128 v{0, 0};
    for (int i = 0; i < 8; ++i) v.hi = (v.hi << 8) | c[i];
    for (int i = 8; i < 16; ++i) v.lo = (v.lo << 8) | c[i];
    return v;
}

Ctr128 ctr_add(Ctr128 c, uint64_t n, bool wrap64)
{
    uint64_t lo = c.lo + n;
    if (!wrap64 && lo < c.lo) c.hi += 1;
    c.lo = lo;
    return c;
}

int pick_impl(int impl, int bits)
{
    if (impl == OTC_IMPL_TTABLE || impl == OTC_IMPL_BITSLICE || impl == OTC_IMPL_HYBRID) return impl;
    const char *env = getenv("OTC_IMPL");
    if (env) {
        if (!strcmp(env, "ttable")) return OTC_IMPL_TTABLE;
        if (!strcmp(env, "bitslice")) return OTC_IMPL_BITSLICE;
        if (!strcmp(env, "hybrid")) return OTC_IMPL_HYBRID;
    }
    (void)bits;
    return OTC_IMPL_TTABLE; /* default: the measured winner (see docs/PERF.md) */
}

int check_key(const otc_aes_key *k, int dir)
{
    if (!k) return set_err(OTC_ERR_ARG, "null key");
    if (k->nr != 10 && k->nr != 12 && k->nr != 14) return set_err(OTC_ERR_ARG, "bad key (nr)");
    if (k->dir != dir)
        return set_err(OTC_ERR_ARG, dir == OTC_DIR_ENCRYPT ? "key schedule is not an encryption schedule"
                                                           : "key schedule is not a decryption schedule");
    return OTC_OK;
}

/* roctx range for rocprofv3 --marker-trace (a no-op unless a tool is attached):
 * every public entry point is one named range, so traces show the API call
 * around its kernels and copies. */
struct Range {
    explicit Range(const char *name) { roctxRangePushA(name); }
    ~Range() { roctxRangePop(); }
    Range(const Range &) = delete;
    Range &operator=(const Range &) = delete;
};

/* Device buffers of the cipher ops: non-null, 16-byte aligned (every kernel
 * moves 16 B per lane with global_load/store_dwordx4), and either the same
 * buffer (in place, where the mode allows it) or disjoint -- a partial overlap
 * would race between workgroups. */
int check_bufs(const void *in, const void *out, size_t nbytes, bool inplace_ok, const char *what)
{
    if (nbytes == 0) return OTC_OK;
    if (!in || !out) return set_err(OTC_ERR_ARG, std::string(what) + ": null buffer");
    if (((uintptr_t)in | (uintptr_t)out) & 15u)
        return set_err(OTC_ERR_ARG, std::string(what) + ": device buffers must be 16-byte aligned");
    if (in == out) {
        if (!inplace_ok) return set_err(OTC_ERR_ARG, std::string(what) + ": in-place operation is not supported");
        return OTC_OK;
    }
    const uintptr_t a = (uintptr_t)in, b = (uintptr_t)out;
    if (a < b + nbytes && b < a + nbytes)
        return set_err(OTC_ERR_ARG, std::string(what) + ": input and output overlap partially");
    return OTC_OK;
}

} // namespace

/* ---- errors / keys ------------------------------------------------------ */
extern "C" const char *otc_last_error(void) { return g_err.c_str(); }

extern "C" int otc_aes_key_init(otc_aes_key *k, const uint8_t *key, int bits, int dir)
{
    if (!k || !key) return set_err(OTC_ERR_ARG, "null argument");
    aes_context ctx;
    int r = (dir == OTC_DIR_ENCRYPT) ? aes_setkey_enc(&ctx, key, (unsigned)bits)
                                     : aes_setkey_dec(&ctx, key, (unsigned)bits);
    if (r) return set_err(OTC_ERR_ARG, "invalid AES key size (must be 128/192/256)");
    memset(k, 0, sizeof *k);
    aes_export_rk32(&ctx, k->rk);
    k->nr = ctx.nr;
    k->dir = dir;
    k->bits = bits;
    return OTC_OK;
}

/* ---- device ops --------------------------------------------------------- */
extern "C" int otc_aes_ecb(const void *in, void *out, size_t nbytes, const otc_aes_key *k, int impl,
                           void *stream)
{
    Range rg("otc_aes_ecb");
    if (nbytes % 16) return set_err(OTC_ERR_ARG, "ECB length must be a multiple of 16");
    if (!k) return set_err(OTC_ERR_ARG, "null key");
    if (int r = check_bufs(in, out, nbytes, true, "aes_ecb")) return r;
    if (nbytes == 0) return OTC_OK;
    hipStream_t st = (hipStream_t)stream;
    hipError_t e;
    if (k->dir == OTC_DIR_ENCRYPT) {
        e = (pick_impl(impl, k->bits) == OTC_IMPL_BITSLICE) ? otc_impl::bs_ecb_encrypt(in, out, nbytes / 16, *k, st)
                                                            : otc_impl::tt_ecb_encrypt(in, out, nbytes / 16, *k, st);
    } else {
        e = otc_impl::tt_ecb_decrypt(in, out, nbytes / 16, *k, st);
    }
    if (e != hipSuccess) return hip_fail(e, "aes_ecb launch");
    return OTC_OK;
}

/* Hybrid CTR: the T-table kernel (LDS-bound, ~40% VALU) and the bitsliced
 * kernel (VALU-only) run CONCURRENTLY on two streams over disjoint ranges.
 * With OTC_TT_VARIANT=1024x2 (64 VGPRs x 4 waves) or 512x4 (112 x 2) each CU
 * hosts one T-table workgroup beside one 256-VGPR bitsliced wave per SIMD.
 * OTC_HYBRID_TT = fraction of blocks given to the T-table kernel.  Measured
 * slower than the T-table alone (docs/PERF.md): kept as an option. */
struct AuxStream {
    int dev = -1;
    hipStream_t s = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
};
thread_local AuxStream g_aux[16];

hipError_t hybrid_ctr(const void *in, void *out, size_t nbytes, const otc_aes_key &K, Ctr128 c, bool wrap64,
                      hipStream_t st)
{
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    AuxStream &a = g_aux[dev & 15];
    if (a.dev != dev) {
        if ((e = hipStreamCreateWithFlags(&a.s, hipStreamNonBlocking)) != hipSuccess) return e;
        if ((e = hipEventCreateWithFlags(&a.e0, hipEventDisableTiming)) != hipSuccess) return e;
        if ((e = hipEventCreateWithFlags(&a.e1, hipEventDisableTiming)) != hipSuccess) return e;
        a.dev = dev;
    }
    double frac = 0.6;
    if (const char *f = getenv("OTC_HYBRID_TT")) frac = atof(f);
    const uint64_t nblk = nbytes / 16;
    uint64_t ntt = (uint64_t)(nblk * frac);
    ntt -= ntt % 2048;
    if (ntt > nblk) ntt = nblk;
    const size_t tt_bytes = ntt * 16;
    /* order the aux stream after prior work on st */
    if ((e = hipEventRecord(a.e0, st)) != hipSuccess) return e;
    if ((e = hipStreamWaitEvent(a.s, a.e0, 0)) != hipSuccess) return e;
    Ctr128 c2 = c;
    c2.lo = c.lo + ntt;
    if (!wrap64 && c2.lo < c.lo) c2.hi += 1;
    /* persistent T-table grid (1 workgroup per CU) first, so its workgroups
     * are resident before the bitsliced waves fill the remaining VGPRs */
    if (tt_bytes) {
        /* the T-table variant for co-residency is chosen by OTC_TT_VARIANT
         * (B=2 keeps it at <= 64 VGPRs so a 256-VGPR bitsliced wave fits) */
        otc_impl::tt_set_wg_per_cu(1);
        e = otc_impl::tt_ctr(in, out, tt_bytes, K, c, wrap64, st);
        otc_impl::tt_set_wg_per_cu(2);
        if (e != hipSuccess) return e;
    }
    if (nbytes > tt_bytes) {
        e = otc_impl::bs_ctr((const uint8_t *)in + tt_bytes, (uint8_t *)out + tt_bytes, nbytes - tt_bytes, K, c2,
                             wrap64, a.s);
        if (e != hipSuccess) return e;
    }
    if ((e = hipEventRecord(a.e1, a.s)) != hipSuccess) return e;
    return hipStreamWaitEvent(st, a.e1, 0);
}

static int ctr_common(const void *in, void *out, size_t nbytes, const otc_aes_key *k, Ctr128 c, bool wrap64,
                      int impl, void *stream)
{
    int r = check_key(k, OTC_DIR_ENCRYPT);
    if (r) return r;
    if ((r = check_bufs(in, out, nbytes, true, "aes_ctr"))) return r;
    if (nbytes == 0) return OTC_OK;
    hipStream_t st = (hipStream_t)stream;
    const int im = pick_impl(impl, k->bits);
    hipError_t e = im == OTC_IMPL_BITSLICE ? otc_impl::bs_ctr(in, out, nbytes, *k, c, wrap64, st)
                   : im == OTC_IMPL_HYBRID ? hybrid_ctr(in, out, nbytes, *k, c, wrap64, st)
                                           : otc_impl::tt_ctr(in, out, nbytes, *k, c, wrap64, st);
    if (e != hipSuccess) return hip_fail(e, "aes_ctr launch");
    return OTC_OK;
}

extern "C" int otc_aes_ctr(const void *in, void *out, size_t nbytes, const otc_aes_key *k, const uint8_t ctr0[16],
                           uint64_t block_offset, int impl, void *stream)
{
    Range rg("otc_aes_ctr");
    if (!ctr0) return set_err(OTC_ERR_ARG, "null counter");
    return ctr_common(in, out, nbytes, k, ctr_add(ctr_from_bytes(ctr0), block_offset, false), false, impl, stream);
}

extern "C" int otc_aes_ctr_rfc3686(const void *in, void *out, size_t nbytes, const otc_aes_key *k,
                                   const uint8_t nonce[4], const uint8_t ivec[8], uint64_t block_offset, int impl,
                                   void *stream)
{
    Range rg("otc_aes_ctr_rfc3686");
    if (!nonce || !ivec) return set_err(OTC_ERR_ARG, "null nonce/ivec");
    uint8_t cb[16];
    memcpy(cb, nonce, 4);
    memcpy(cb + 4, ivec, 8);
    cb[12] = 0; cb[13] = 0; cb[14] = 0; cb[15] = 1;
    return ctr_common(in, out, nbytes, k, ctr_add(ctr_from_bytes(cb), block_offset, true), true, impl, stream);
}

extern "C" uint64_t otc_ctr_batch_plan(const otc_ctr_msg *msgs, size_t nmsg, int tile_blocks, uint32_t *tile_msg,
                                       uint64_t *tile_first)
{
    if (tile_blocks != 64 && tile_blocks != 128 && tile_blocks != 256) return 0;
    const uint64_t tile_bytes = 16ull * (uint64_t)tile_blocks;
    uint64_t t = 0;
    for (size_t m = 0; m < nmsg; ++m) {
        const uint64_t shift = (msgs[m].align & OTC_BATCH_ALIGNED) ? 16ull * (msgs[m].align & 0xFFFFu) : 0;
        const uint64_t nt = msgs[m].nbytes ? (msgs[m].nbytes + shift + tile_bytes - 1) / tile_bytes : 0;
        if (tile_first) tile_first[m] = t;
        if (tile_msg)
            for (uint64_t k = 0; k < nt; ++k) tile_msg[t + k] = (uint32_t)m;
        t += nt;
    }
    return t;
}

/* Descriptors live in device memory, so per-message checks (alignment,
 * overlap) are the planner's job on the host (our_tree_amd.ops.CtrBatch);
 * here only the launch arguments are validated. */
extern "C" int otc_aes_ctr_batch(const otc_ctr_msg *msgs, const otc_aes_key *keys, const uint32_t *tile_msg,
                                 const uint64_t *tile_first, uint64_t ntiles, int tile_blocks, int nr, void *stream)
{
    Range rg("otc_aes_ctr_batch");
    if (tile_blocks != 64 && tile_blocks != 128 && tile_blocks != 256)
        return set_err(OTC_ERR_ARG, "ctr_batch: tile_blocks must be 64, 128 or 256");
    if (ntiles == 0) return OTC_OK;
    if (!msgs || !keys || !tile_msg || !tile_first) return set_err(OTC_ERR_ARG, "ctr_batch: null array");
    if (nr != 10 && nr != 12 && nr != 14) return set_err(OTC_ERR_ARG, "ctr_batch: nr must be 10, 12 or 14");
    if ((((uintptr_t)msgs) | ((uintptr_t)keys) | ((uintptr_t)tile_first)) & 7u || ((uintptr_t)tile_msg & 3u))
        return set_err(OTC_ERR_ARG, "ctr_batch: misaligned descriptor arrays");
    hipError_t e = otc_impl::tt_ctr_batch(msgs, keys, tile_msg, tile_first, ntiles, tile_blocks, nr,
                                          (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "ctr_batch launch");
    return OTC_OK;
}

extern "C" int otc_aes_cbc_decrypt(const void *in, void *out, size_t nbytes, const otc_aes_key *k,
                                   const uint8_t iv[16], void *stream)
{
    Range rg("otc_aes_cbc_decrypt");
    int r = check_key(k, OTC_DIR_DECRYPT);
    if (r) return r;
    if (nbytes % 16) return set_err(OTC_ERR_ARG, "CBC length must be a multiple of 16");
    if (!iv) return set_err(OTC_ERR_ARG, "null iv");
    if ((r = check_bufs(in, out, nbytes, nbytes <= 16, "aes_cbc_decrypt"))) return r;
    if (nbytes == 0) return OTC_OK;
    hipError_t e = otc_impl::tt_cbc_decrypt(in, out, nbytes / 16, *k, ctr_from_bytes(iv), (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "cbc_decrypt launch");
    return OTC_OK;
}

extern "C" int otc_aes_cbc_encrypt_segments(const void *in, void *out, size_t seg_bytes, size_t nseg,
                                            const otc_aes_key *k, const uint8_t iv0[16], void *stream)
{
    Range rg("otc_aes_cbc_encrypt_segments");
    int r = check_key(k, OTC_DIR_ENCRYPT);
    if (r) return r;
    if (seg_bytes % 16) return set_err(OTC_ERR_ARG, "segment length must be a multiple of 16");
    if (!iv0) return set_err(OTC_ERR_ARG, "null iv");
    if (nseg && seg_bytes > SIZE_MAX / nseg) return set_err(OTC_ERR_ARG, "size overflow");
    if ((r = check_bufs(in, out, seg_bytes * nseg, true, "aes_cbc_encrypt_segments"))) return r;
    if (nseg == 0 || seg_bytes == 0) return OTC_OK;
    hipError_t e = otc_impl::tt_cbc_encrypt_seg(in, out, seg_bytes / 16, nseg, *k, ctr_from_bytes(iv0),
                                                (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "cbc_encrypt_segments launch");
    return OTC_OK;
}

extern "C" int otc_aes_cbc_decrypt_segments(const void *in, void *out, size_t seg_bytes, size_t nseg,
                                            const otc_aes_key *k, const uint8_t iv0[16], void *stream)
{
    Range rg("otc_aes_cbc_decrypt_segments");
    int r = check_key(k, OTC_DIR_DECRYPT);
    if (r) return r;
    if (seg_bytes % 16) return set_err(OTC_ERR_ARG, "segment length must be a multiple of 16");
    size_t sb = seg_bytes / 16;
    if (sb == 0) return set_err(OTC_ERR_ARG, "empty segments");
    if (!iv0) return set_err(OTC_ERR_ARG, "null iv");
    if (nseg && seg_bytes > SIZE_MAX / nseg) return set_err(OTC_ERR_ARG, "size overflow");
    if ((r = check_bufs(in, out, seg_bytes * nseg, false, "aes_cbc_decrypt_segments"))) return r;
    if (nseg == 0) return OTC_OK;
    hipError_t e = otc_impl::tt_cbc_decrypt_seg(in, out, sb, nseg, *k, ctr_from_bytes(iv0), (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "cbc_decrypt_segments launch");
    return OTC_OK;
}

extern "C" int otc_aes_cfb128_decrypt(const void *in, void *out, size_t nbytes, const otc_aes_key *k,
                                      const uint8_t iv[16], void *stream)
{
    Range rg("otc_aes_cfb128_decrypt");
    int r = check_key(k, OTC_DIR_ENCRYPT);
    if (r) return r;
    if (nbytes % 16) return set_err(OTC_ERR_ARG, "CFB128 device path needs a multiple of 16 bytes");
    if (!iv) return set_err(OTC_ERR_ARG, "null iv");
    if ((r = check_bufs(in, out, nbytes, nbytes <= 16, "aes_cfb128_decrypt"))) return r;
    if (nbytes == 0) return OTC_OK;
    uint32_t ivw[4];
    memcpy(ivw, iv, 16);
    hipError_t e = otc_impl::tt_cfb_decrypt(in, out, nbytes / 16, *k, ivw, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "cfb_decrypt launch");
    return OTC_OK;
}

extern "C" int otc_xor(const void *a, const void *b, void *out, size_t nbytes, void *stream)
{
    Range rg("otc_xor");
    if (int r = check_bufs(a, out, nbytes, true, "xor")) return r;
    if (int r = check_bufs(b, out, nbytes, true, "xor")) return r;
    if (nbytes == 0) return OTC_OK;
    hipError_t e = otc_impl::k_xor(a, b, out, nbytes, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "xor launch");
    return OTC_OK;
}

extern "C" int otc_rc4_multi(const uint8_t *keys, int keylen, size_t nstreams, size_t len, size_t drop,
                             const void *in, void *out, void *stream)
{
    Range rg("otc_rc4_multi");
    if (keylen < 1 || keylen > 256) return set_err(OTC_ERR_ARG, "RC4 key length must be 1..256");
    if (nstreams == 0 || len == 0) return OTC_OK;
    if (!keys || !out) return set_err(OTC_ERR_ARG, "rc4_multi: null buffer");
    if (len > SIZE_MAX / nstreams) return set_err(OTC_ERR_ARG, "size overflow");
    if (in && in != out) {
        const uintptr_t a = (uintptr_t)in, b = (uintptr_t)out, n = nstreams * len;
        if (a < b + n && b < a + n) return set_err(OTC_ERR_ARG, "rc4_multi: input and output overlap partially");
    }
    hipError_t e = otc_impl::k_rc4_multi(keys, keylen, nstreams, len, drop, in, out, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "rc4_multi launch");
    return OTC_OK;
}

extern "C" int otc_fill_random(void *p, size_t nbytes, uint64_t seed, void *stream)
{
    Range rg("otc_fill_random");
    if (nbytes == 0) return OTC_OK;
    if (int r = check_bufs(p, p, nbytes, true, "fill_random")) return r;
    hipError_t e = otc_impl::k_fill_random(p, nbytes, seed, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "fill_random launch");
    return OTC_OK;
}

extern "C" int otc_checksum(const void *p, size_t nbytes, uint64_t *out_dev, void *stream)
{
    Range rg("otc_checksum");
    if (nbytes % 8) return set_err(OTC_ERR_ARG, "checksum length must be a multiple of 8");
    if (!out_dev || (nbytes && !p)) return set_err(OTC_ERR_ARG, "checksum: null buffer");
    if (((uintptr_t)p | (uintptr_t)out_dev) & 7u) return set_err(OTC_ERR_ARG, "checksum: buffers must be 8-byte aligned");
    hipError_t e = otc_impl::k_checksum(p, nbytes, out_dev, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "checksum launch");
    return OTC_OK;
}

extern "C" int otc_clock_probe(uint64_t *out_dev, double delay_s, double window_s, void *stream)
{
    if (!out_dev || ((uintptr_t)out_dev & 7u)) return set_err(OTC_ERR_ARG, "clock_probe: bad output buffer");
    if (!(delay_s >= 0.0) || !(window_s > 0.0) || delay_s + window_s > 60.0)
        return set_err(OTC_ERR_ARG, "clock_probe: delay/window out of range (total <= 60 s)");
    const uint64_t hz = 100000000ull; /* s_memrealtime */
    hipError_t e = otc_impl::k_clock(out_dev, (uint64_t)(delay_s * hz), (uint64_t)(window_s * hz) + 1,
                                     (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "clock_probe launch");
    return OTC_OK;
}

/* ---- AES-NI-shaped bulk API (otc_aesni.h) ------------------------------- */
static int key_from_sched(otc_aes_key *k, const unsigned char *sched, int nr, int dir)
{
    if (!sched) return set_err(OTC_ERR_ARG, "null key schedule");
    if (nr != 10 && nr != 12 && nr != 14) return set_err(OTC_ERR_ARG, "number_of_rounds must be 10, 12 or 14");
    memset(k, 0, sizeof *k);
    memcpy(k->rk, sched, 16u * (unsigned)(nr + 1)); /* FIPS byte order = LE words on the host */
    k->nr = nr;
    k->dir = dir;
    k->bits = 32 * (nr - 6);
    return OTC_OK;
}

extern "C" int otc_AES_ECB_encrypt(const unsigned char *in, unsigned char *out, unsigned long length,
                                   const unsigned char *key, int number_of_rounds, void *stream)
{
    otc_aes_key k;
    if (int r = key_from_sched(&k, key, number_of_rounds, OTC_DIR_ENCRYPT)) return r;
    return otc_aes_ecb(in, out, length, &k, OTC_IMPL_AUTO, stream);
}

extern "C" int otc_AES_ECB_decrypt(const unsigned char *in, unsigned char *out, unsigned long length,
                                   const unsigned char *key, int number_of_rounds, void *stream)
{
    otc_aes_key k;
    if (int r = key_from_sched(&k, key, number_of_rounds, OTC_DIR_DECRYPT)) return r;
    return otc_aes_ecb(in, out, length, &k, OTC_IMPL_AUTO, stream);
}

extern "C" int otc_AES_CTR_encrypt(const unsigned char *in, unsigned char *out, const unsigned char ivec[8],
                                   const unsigned char nonce[4], unsigned long length, const unsigned char *key,
                                   int number_of_rounds, void *stream)
{
    otc_aes_key k;
    if (int r = key_from_sched(&k, key, number_of_rounds, OTC_DIR_ENCRYPT)) return r;
    return otc_aes_ctr_rfc3686(in, out, length, &k, nonce, ivec, 0, OTC_IMPL_AUTO, stream);
}

/* ---- device info -------------------------------------------------------- */
extern "C" int otc_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}
extern "C" int otc_device_cus(int dev)
{
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return -1;
    return v;
}
extern "C" int otc_device_clock_khz(int dev)
{
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeClockRate, dev) != hipSuccess) return -1;
    return v;
}
extern "C" int otc_set_device(int dev)
{
    HIPCHK(hipSetDevice(dev));
    return OTC_OK;
}
extern "C" int otc_device_sync(void)
{
    HIPCHK(hipDeviceSynchronize());
    return OTC_OK;
}

/* ---- device memory helpers --------------------------------------------- */
extern "C" void *otc_dev_malloc(size_t nbytes)
{
    void *p = nullptr;
    hipError_t e = hipMalloc(&p, nbytes ? nbytes : 16);
    if (e != hipSuccess) {
        hip_fail(e, "hipMalloc");
        return nullptr;
    }
    return p;
}
extern "C" void otc_dev_free(void *p)
{
    if (p) (void)hipFree(p);
}
extern "C" int otc_memcpy(void *dst, const void *src, size_t nbytes, int kind)
{
    hipMemcpyKind k = kind == OTC_H2D ? hipMemcpyHostToDevice : kind == OTC_D2H ? hipMemcpyDeviceToHost
                                                                                : hipMemcpyDeviceToDevice;
    HIPCHK(hipMemcpy(dst, src, nbytes, k));
    return OTC_OK;
}
extern "C" int otc_memset(void *p, int v, size_t nbytes)
{
    HIPCHK(hipMemset(p, v, nbytes));
    return OTC_OK;
}
struct EventPair {
    hipEvent_t a = nullptr, b = nullptr;
    ~EventPair()
    {
        if (a) (void)hipEventDestroy(a);
        if (b) (void)hipEventDestroy(b);
    }
};

extern "C" int otc_time_op(otc_op_fn op, void *arg, int iters, double *ms_per_iter)
{
    if (!op) return set_err(OTC_ERR_ARG, "null op");
    EventPair ev;
    HIPCHK(hipEventCreate(&ev.a));
    HIPCHK(hipEventCreate(&ev.b));
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipEventRecord(ev.a, nullptr));
    for (int i = 0; i < iters; ++i) {
        int r = op(arg);
        if (r) return r;
    }
    HIPCHK(hipEventRecord(ev.b, nullptr));
    HIPCHK(hipEventSynchronize(ev.b));
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, ev.a, ev.b));
    if (ms_per_iter) *ms_per_iter = iters > 0 ? ms / iters : 0.0;
    return OTC_OK;
}

/* Held clock under `op`: the clock probe on its own non-blocking stream,
 * beside >= 0.3 s of back-to-back ops on the default stream. */
extern "C" int otc_measure_clock(otc_op_fn op, void *arg, double *ghz)
{
    if (!op || !ghz) return set_err(OTC_ERR_ARG, "null argument");
    double ms = 0.0;
    if (int r = otc_time_op(op, arg, 1, &ms)) return r;
    const int n = std::max(3, (int)(300.0 / std::max(ms, 1e-3)) + 1);
    struct Res {
        hipStream_t s = nullptr;
        uint64_t *d = nullptr;
        ~Res()
        {
            if (d) (void)hipFree(d);
            if (s) (void)hipStreamDestroy(s);
        }
    } R;
    HIPCHK(hipStreamCreateWithFlags(&R.s, hipStreamNonBlocking));
    HIPCHK(hipMalloc(&R.d, 2 * sizeof(uint64_t)));
    HIPCHK(hipMemset(R.d, 0, 2 * sizeof(uint64_t)));
    if (int r = otc_clock_probe(R.d, 0.2 * n * ms * 1e-3, 0.6 * n * ms * 1e-3, R.s)) return r;
    for (int i = 0; i < n; ++i)
        if (int r = op(arg)) return r;
    HIPCHK(hipDeviceSynchronize());
    uint64_t h[2] = {0, 0};
    HIPCHK(hipMemcpy(h, R.d, sizeof h, hipMemcpyDeviceToHost));
    *ghz = h[1] ? 0.1 * (double)h[0] / (double)h[1] : 0.0;
    return OTC_OK;
}

/* ---- pinned host memory ------------------------------------------------- */
extern "C" int otc_host_register(void *p, size_t nbytes)
{
    HIPCHK(hipHostRegister(p, nbytes, hipHostRegisterDefault));
    return OTC_OK;
}
extern "C" int otc_host_unregister(void *p)
{
    HIPCHK(hipHostUnregister(p));
    return OTC_OK;
}
extern "C" void *otc_host_alloc_pinned(size_t nbytes)
{
    void *p = nullptr;
    if (hipHostMalloc(&p, nbytes, hipHostMallocDefault) != hipSuccess) return nullptr;
    return p;
}
extern "C" void otc_host_free_pinned(void *p)
{
    if (p) (void)hipHostFree(p);
}

/* ---- L3 streaming engine ------------------------------------------------ */
struct otc_engine {
    int device = 0;
    size_t chunk = 0;
    int depth = 0;                  /* ring slots */
    std::vector<void *> d_in, d_out; /* device ring */
    std::vector<void *> h_in, h_out; /* pinned staging ring */
    hipStream_t s_h2d = nullptr, s_k = nullptr, s_d2h = nullptr;
    std::vector<hipEvent_t> ev_h2d, ev_k, ev_d2h, ev_k0;
};

extern "C" otc_engine *otc_engine_create(int device, size_t chunk_bytes, int depth)
{
    if (chunk_bytes == 0) chunk_bytes = 256ull << 20;
    chunk_bytes = (chunk_bytes + 15) & ~(size_t)15;
    if (depth < 2) depth = 3;
    otc_engine *e = new otc_engine();
    e->device = device;
    e->chunk = chunk_bytes;
    e->depth = depth;
    if (hipSetDevice(device) != hipSuccess) { set_err(OTC_ERR_HIP, "hipSetDevice"); delete e; return nullptr; }
    bool ok = hipStreamCreateWithFlags(&e->s_h2d, hipStreamNonBlocking) == hipSuccess &&
              hipStreamCreateWithFlags(&e->s_k, hipStreamNonBlocking) == hipSuccess &&
              hipStreamCreateWithFlags(&e->s_d2h, hipStreamNonBlocking) == hipSuccess;
    e->d_in.assign(depth, nullptr);
    e->d_out.assign(depth, nullptr);
    e->h_in.assign(depth, nullptr);
    e->h_out.assign(depth, nullptr);
    e->ev_h2d.assign(depth, nullptr);
    e->ev_k.assign(depth, nullptr);
    e->ev_d2h.assign(depth, nullptr);
    e->ev_k0.assign(depth, nullptr);
    /* pinned staging (h_in/h_out) is allocated lazily, only for pageable
     * host buffers */
    for (int i = 0; ok && i < depth; ++i) {
        ok = hipMalloc(&e->d_in[i], chunk_bytes) == hipSuccess && hipMalloc(&e->d_out[i], chunk_bytes) == hipSuccess &&
             hipEventCreateWithFlags(&e->ev_h2d[i], hipEventDisableTiming) == hipSuccess &&
             hipEventCreate(&e->ev_k[i]) == hipSuccess &&
             hipEventCreateWithFlags(&e->ev_d2h[i], hipEventDisableTiming) == hipSuccess &&
             hipEventCreate(&e->ev_k0[i]) == hipSuccess;
    }
    if (!ok) {
        set_err(OTC_ERR_NOMEM, "engine allocation failed");
        otc_engine_destroy(e);
        return nullptr;
    }
    return e;
}

extern "C" void otc_engine_destroy(otc_engine *e)
{
    if (!e) return;
    (void)hipSetDevice(e->device);
    if (e->s_k) (void)hipStreamSynchronize(e->s_k);
    if (e->s_h2d) (void)hipStreamSynchronize(e->s_h2d);
    if (e->s_d2h) (void)hipStreamSynchronize(e->s_d2h);
    for (int i = 0; i < e->depth; ++i) {
        if (e->d_in[i]) (void)hipFree(e->d_in[i]);
        if (e->d_out[i]) (void)hipFree(e->d_out[i]);
        if (e->h_in[i]) (void)hipHostFree(e->h_in[i]);
        if (e->h_out[i]) (void)hipHostFree(e->h_out[i]);
        if (e->ev_h2d[i]) (void)hipEventDestroy(e->ev_h2d[i]);
        if (e->ev_k[i]) (void)hipEventDestroy(e->ev_k[i]);
        if (e->ev_d2h[i]) (void)hipEventDestroy(e->ev_d2h[i]);
        if (e->ev_k0[i]) (void)hipEventDestroy(e->ev_k0[i]);
    }
    if (e->s_h2d) (void)hipStreamDestroy(e->s_h2d);
    if (e->s_k) (void)hipStreamDestroy(e->s_k);
    if (e->s_d2h) (void)hipStreamDestroy(e->s_d2h);
    delete e;
}

static bool is_pinned(const void *p)
{
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

extern "C" int otc_ptr_kind(const void *p)
{
    if (!p) return OTC_PTR_HOST;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return OTC_PTR_HOST;
    }
    if (a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged) return OTC_PTR_DEVICE;
    if (a.type == hipMemoryTypeHost) return OTC_PTR_PINNED;
    return OTC_PTR_HOST;
}

/* Launch the cipher on one device chunk. `blk0` = block offset of the chunk
 * inside the whole stream; `prev` = for CBC-dec, the 16-byte ciphertext block
 * preceding the chunk (the halo), as counter-style numeric IV. */
/* Up-front validation of a host-streamed job (engine and multi-GPU), so a bad
 * call fails before any allocation or copy is issued. */
static int check_stream_args(int mode, const void *host_in, const void *host_out, size_t nbytes,
                             const otc_aes_key *k, const uint8_t ivc[16])
{
    if (mode != OTC_MODE_ECB && mode != OTC_MODE_CTR && mode != OTC_MODE_CBC_DEC)
        return set_err(OTC_ERR_ARG, "unsupported streaming mode");
    if (mode != OTC_MODE_CTR && nbytes % 16) return set_err(OTC_ERR_ARG, "length must be a multiple of 16");
    if (nbytes && (!host_in || !host_out)) return set_err(OTC_ERR_ARG, "null host buffer");
    if (!k) return set_err(OTC_ERR_ARG, "null key");
    if (mode == OTC_MODE_CTR || mode == OTC_MODE_CBC_DEC) {
        if (!ivc) return set_err(OTC_ERR_ARG, "null iv/counter");
        if (int r = check_key(k, mode == OTC_MODE_CTR ? OTC_DIR_ENCRYPT : OTC_DIR_DECRYPT)) return r;
    } else if (int r = check_key(k, k->dir)) {
        return r;
    }
    if (host_in != host_out && nbytes) {
        const uintptr_t a = (uintptr_t)host_in, b = (uintptr_t)host_out;
        if (a < b + nbytes && b < a + nbytes) return set_err(OTC_ERR_ARG, "input and output overlap partially");
    }
    return OTC_OK;
}

static int run_chunk(int mode, const void *din, void *dout, size_t n, const otc_aes_key *k, const uint8_t ivc[16],
                     uint64_t blk0, const uint8_t *halo, int impl, hipStream_t st)
{
    switch (mode) {
    case OTC_MODE_CTR: return otc_aes_ctr(din, dout, n, k, ivc, blk0, impl, st);
    case OTC_MODE_ECB: return otc_aes_ecb(din, dout, n, k, impl, st);
    case OTC_MODE_CBC_DEC: return otc_aes_cbc_decrypt(din, dout, n, k, halo ? halo : ivc, st);
    default: return set_err(OTC_ERR_ARG, "unsupported engine mode");
    }
}

extern "C" int otc_engine_run(otc_engine *e, int mode, const void *host_in, void *host_out, size_t nbytes,
                              const otc_aes_key *k, const uint8_t ivc[16], uint64_t block_offset, int impl,
                              otc_stream_stats *stats)
{
    Range rg("otc_engine_run");
    if (!e) return set_err(OTC_ERR_ARG, "null engine");
    if (int r = check_stream_args(mode, host_in, host_out, nbytes, k, ivc)) return r;
    if (mode == OTC_MODE_CBC_DEC && block_offset) return set_err(OTC_ERR_ARG, "CBC: pass the halo as iv instead");
    HIPCHK(hipSetDevice(e->device));
    auto t0 = std::chrono::steady_clock::now();
    const bool pin_in = is_pinned(host_in), pin_out = is_pinned(host_out);
    for (int i = 0; i < e->depth; ++i) {
        if (!pin_in && !e->h_in[i]) HIPCHK(hipHostMalloc(&e->h_in[i], e->chunk, hipHostMallocDefault));
        if (!pin_out && !e->h_out[i]) HIPCHK(hipHostMalloc(&e->h_out[i], e->chunk, hipHostMallocDefault));
    }
    const size_t C = e->chunk;
    const size_t nchunks = (nbytes + C - 1) / C;
    const uint8_t *hin = (const uint8_t *)host_in;
    uint8_t *hout = (uint8_t *)host_out;
    double kms = 0.0;
    std::vector<int> slot_used(e->depth, 0);

    for (size_t c = 0; c < nchunks; ++c) {
        const int s = (int)(c % e->depth);
        const size_t off = c * C;
        const size_t n = std::min(C, nbytes - off);
        /* slot reuse: wait until the D2H that last used this slot finished */
        if (slot_used[s]) {
            HIPCHK(hipEventSynchronize(e->ev_d2h[s]));
            float ms = 0.f;
            if (hipEventElapsedTime(&ms, e->ev_k0[s], e->ev_k[s]) == hipSuccess) kms += ms;
            if (!pin_out) {
                const size_t poff = (c - e->depth) * C;
                memcpy(hout + poff, e->h_out[s], std::min(C, nbytes - poff));
            }
        }
        const void *src = hin + off;
        if (!pin_in) {
            memcpy(e->h_in[s], hin + off, n);
            src = e->h_in[s];
        }
        HIPCHK(hipMemcpyAsync(e->d_in[s], src, n, hipMemcpyHostToDevice, e->s_h2d));
        HIPCHK(hipEventRecord(e->ev_h2d[s], e->s_h2d));
        HIPCHK(hipStreamWaitEvent(e->s_k, e->ev_h2d[s], 0));
        HIPCHK(hipEventRecord(e->ev_k0[s], e->s_k));
        uint8_t halo[16];
        const uint8_t *hp = nullptr;
        if (mode == OTC_MODE_CBC_DEC && off > 0) {
            memcpy(halo, hin + off - 16, 16); /* previous ciphertext block */
            hp = halo;
        }
        int r = run_chunk(mode, e->d_in[s], e->d_out[s], n, k, ivc, block_offset + off / 16, hp, impl, e->s_k);
        if (r) return r;
        HIPCHK(hipEventRecord(e->ev_k[s], e->s_k));
        HIPCHK(hipStreamWaitEvent(e->s_d2h, e->ev_k[s], 0));
        void *dst = pin_out ? (void *)(hout + off) : e->h_out[s];
        HIPCHK(hipMemcpyAsync(dst, e->d_out[s], n, hipMemcpyDeviceToHost, e->s_d2h));
        HIPCHK(hipEventRecord(e->ev_d2h[s], e->s_d2h));
        slot_used[s] = 1;
    }
    /* drain */
    for (size_t c = (nchunks > (size_t)e->depth ? nchunks - e->depth : 0); c < nchunks; ++c) {
        const int s = (int)(c % e->depth);
        HIPCHK(hipEventSynchronize(e->ev_d2h[s]));
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, e->ev_k0[s], e->ev_k[s]) == hipSuccess) kms += ms;
        if (!pin_out) {
            const size_t off = c * C;
            memcpy(hout + off, e->h_out[s], std::min(C, nbytes - off));
        }
    }
    auto t1 = std::chrono::steady_clock::now();
    if (stats) {
        stats->total_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
        stats->kernel_ms = kms;
        stats->h2d_ms = stats->d2h_ms = 0.0;
        stats->bytes = nbytes;
        stats->chunks = (int)nchunks;
    }
    return OTC_OK;
}

/* ---- L4 multi-GPU (single process) -------------------------------------- */
/* ---- RCCL root scatter / gather (otc_multi_run strategy 1) -----------------
 * Root GPU 0 ingests the host stream, ncclScatter deals equal S-byte pieces to
 * every GPU over xGMI, each GPU runs the cipher, ncclGather collects the
 * results at the root, which drains them to the host.  Two root buffer sets
 * are used in ping-pong: H2D of round r+1 (copy stream) and D2H of round r-1
 * (copy stream) overlap the scatter/compute/gather of round r, ordered by
 * events.  ncclScatter needs equal counts, so the last round is zero padded.
 *
 * Failure detection: waits poll hipStreamQuery and ncclCommGetAsyncError with a
 * watchdog (OTC_RCCL_TIMEOUT_S, default 600 s); on an async error or timeout
 * every communicator is aborted (ncclCommAbort) instead of destroyed, so a
 * hung peer cannot hang the caller.  All resources are owned by RcclJob and
 * released on every exit path. */
struct RcclJob {
    int n = 0;
    size_t S = 0;                         /* per-GPU bytes per round */
    std::vector<ncclComm_t> comms;
    std::vector<hipStream_t> st;          /* per GPU: scatter, cipher, gather */
    std::vector<void *> dsh, dsh_out;     /* per GPU S-byte piece (in / out) */
    hipStream_t h2d = nullptr, d2h = nullptr;  /* root copy streams */
    void *root_in[2] = {nullptr, nullptr}, *root_out[2] = {nullptr, nullptr};
    hipEvent_t ev_in[2] = {}, ev_scattered[2] = {}, ev_gathered[2] = {}, ev_drained[2] = {};
    bool failed = false;

    ~RcclJob()
    {
        for (int g = 0; g < n; ++g) {
            (void)hipSetDevice(g);
            if (!failed && st[g]) (void)hipStreamSynchronize(st[g]);
        }
        (void)hipSetDevice(0);
        if (!failed) {
            if (h2d) (void)hipStreamSynchronize(h2d);
            if (d2h) (void)hipStreamSynchronize(d2h);
        }
        for (int g = 0; g < n; ++g) {
            if (comms[g]) {
                if (failed) ncclCommAbort(comms[g]);
                else ncclCommDestroy(comms[g]);
            }
        }
        for (int g = 0; g < n; ++g) {
            (void)hipSetDevice(g);
            if (dsh[g]) (void)hipFree(dsh[g]);
            if (dsh_out[g]) (void)hipFree(dsh_out[g]);
            if (st[g]) (void)hipStreamDestroy(st[g]);
        }
        (void)hipSetDevice(0);
        for (int i = 0; i < 2; ++i) {
            if (root_in[i]) (void)hipFree(root_in[i]);
            if (root_out[i]) (void)hipFree(root_out[i]);
            for (hipEvent_t ev : {ev_in[i], ev_scattered[i], ev_gathered[i], ev_drained[i]})
                if (ev) (void)hipEventDestroy(ev);
        }
        if (h2d) (void)hipStreamDestroy(h2d);
        if (d2h) (void)hipStreamDestroy(d2h);
    }

    /* wait for `s` while watching every communicator */
    int wait(hipStream_t s, double timeout_s)
    {
        auto t0 = std::chrono::steady_clock::now();
        for (;;) {
            hipError_t q = hipStreamQuery(s);
            if (q == hipSuccess) return OTC_OK;
            if (q != hipErrorNotReady) {
                failed = true;
                return hip_fail(q, "hipStreamQuery (RCCL job)");
            }
            for (int g = 0; g < n; ++g) {
                ncclResult_t ae = ncclSuccess;
                if (ncclCommGetAsyncError(comms[g], &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress) {
                    failed = true;
                    return set_err(OTC_ERR_RCCL, std::string("RCCL async error on GPU ") + std::to_string(g) + ": " +
                                                     ncclGetErrorString(ae));
                }
            }
            if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s) {
                failed = true;
                return set_err(OTC_ERR_RCCL, "RCCL collective timed out (OTC_RCCL_TIMEOUT_S)");
            }
            std::this_thread::sleep_for(std::chrono::microseconds(50));
        }
    }
};

static int rccl_job_init(RcclJob &J, int ngpus, size_t S)
{
    J.n = ngpus;
    J.S = S;
    J.comms.assign(ngpus, nullptr);
    J.st.assign(ngpus, nullptr);
    J.dsh.assign(ngpus, nullptr);
    J.dsh_out.assign(ngpus, nullptr);
    std::vector<int> devs(ngpus);
    for (int g = 0; g < ngpus; ++g) devs[g] = g;
    RCCLCHK(ncclCommInitAll(J.comms.data(), ngpus, devs.data()));
    const size_t round = S * (size_t)ngpus;
    for (int g = 0; g < ngpus; ++g) {
        HIPCHK(hipSetDevice(g));
        HIPCHK(hipStreamCreateWithFlags(&J.st[g], hipStreamNonBlocking));
        HIPCHK(hipMalloc(&J.dsh[g], S));
        HIPCHK(hipMalloc(&J.dsh_out[g], S));
    }
    HIPCHK(hipSetDevice(0));
    HIPCHK(hipStreamCreateWithFlags(&J.h2d, hipStreamNonBlocking));
    HIPCHK(hipStreamCreateWithFlags(&J.d2h, hipStreamNonBlocking));
    for (int i = 0; i < 2; ++i) {
        HIPCHK(hipMalloc(&J.root_in[i], round));
        HIPCHK(hipMalloc(&J.root_out[i], round));
        for (hipEvent_t *ev : {&J.ev_in[i], &J.ev_scattered[i], &J.ev_gathered[i], &J.ev_drained[i]})
            HIPCHK(hipEventCreateWithFlags(ev, hipEventDisableTiming));
    }
    return OTC_OK;
}

/* The communicators, streams and buffers of the last job are cached across
 * calls (ncclCommInitAll + allocation cost ~0.4 s, more than streaming 8 GiB);
 * a different GPU count or round size rebuilds them, a failure aborts them,
 * otc_multi_release() frees them.  Never torn down by a static destructor:
 * at process exit the HIP runtime may already be gone. */
std::mutex g_rccl_mu;
RcclJob *g_rccl = nullptr;

/* strategy 0 (direct ingest): one cached pipeline engine per GPU */
std::mutex g_direct_mu;
std::vector<otc_engine *> g_direct;

static int rccl_job_run(RcclJob &J, int mode, const uint8_t *hin, uint8_t *hout, size_t nbytes,
                        const otc_aes_key *k, const uint8_t ivc[16], int impl, double timeout_s);

static int rccl_scatter_gather(int ngpus, int mode, const uint8_t *hin, uint8_t *hout, size_t nbytes,
                               const otc_aes_key *k, const uint8_t ivc[16], int impl, size_t chunk_bytes)
{
    const char *to = getenv("OTC_RCCL_TIMEOUT_S");
    const double timeout_s = to ? atof(to) : 600.0;
    size_t S = chunk_bytes ? chunk_bytes : (size_t)64 << 20; /* per-GPU bytes per round */
    S = (S + 15) & ~(size_t)15;
    std::lock_guard<std::mutex> lk(g_rccl_mu);
    if (g_rccl && (g_rccl->n != ngpus || g_rccl->S != S)) {
        delete g_rccl;
        g_rccl = nullptr;
    }
    if (!g_rccl) {
        RcclJob *J = new RcclJob;
        if (int r = rccl_job_init(*J, ngpus, S)) {
            delete J;
            return r;
        }
        g_rccl = J;
    }
    int rc = rccl_job_run(*g_rccl, mode, hin, hout, nbytes, k, ivc, impl, timeout_s);
    if (rc) { /* unknown state: abort the communicators, rebuild next time */
        g_rccl->failed = true;
        delete g_rccl;
        g_rccl = nullptr;
    }
    return rc;
}

static int rccl_job_run(RcclJob &J, int mode, const uint8_t *hin, uint8_t *hout, size_t nbytes,
                        const otc_aes_key *k, const uint8_t ivc[16], int impl, double timeout_s)
{
    const int ngpus = J.n;
    const size_t S = J.S, round = S * (size_t)ngpus;
    const size_t nrounds = (nbytes + round - 1) / round;
    for (size_t r = 0; r < nrounds; ++r) {
        const int b = (int)(r & 1);
        const size_t off = r * round, n = std::min(round, nbytes - off);
        HIPCHK(hipSetDevice(0));
        /* root_in[b] is free once round r-2's scatter has read it */
        if (r >= 2) HIPCHK(hipStreamWaitEvent(J.h2d, J.ev_scattered[b], 0));
        if (n < round) HIPCHK(hipMemsetAsync(J.root_in[b], 0, round, J.h2d));
        HIPCHK(hipMemcpyAsync(J.root_in[b], hin + off, n, hipMemcpyHostToDevice, J.h2d));
        HIPCHK(hipEventRecord(J.ev_in[b], J.h2d));
        HIPCHK(hipStreamWaitEvent(J.st[0], J.ev_in[b], 0));
        RCCLCHK(ncclGroupStart());
        for (int g = 0; g < ngpus; ++g)
            RCCLCHK(ncclScatter(J.root_in[b], J.dsh[g], S, ncclUint8, 0, J.comms[g], J.st[g]));
        RCCLCHK(ncclGroupEnd());
        HIPCHK(hipSetDevice(0));
        HIPCHK(hipEventRecord(J.ev_scattered[b], J.st[0]));
        for (int g = 0; g < ngpus; ++g) {
            const size_t goff = off + (size_t)g * S;
            if (goff >= nbytes) continue;
            HIPCHK(hipSetDevice(g));
            const size_t gn = std::min(S, nbytes - goff);
            uint8_t halo[16];
            const uint8_t *hp = nullptr;
            if (mode == OTC_MODE_CBC_DEC && goff > 0) {
                memcpy(halo, hin + goff - 16, 16);
                hp = halo;
            }
            if (int rr = run_chunk(mode, J.dsh[g], J.dsh_out[g], gn, k, ivc, goff / 16, hp, impl, J.st[g])) {
                J.failed = true;
                return rr;
            }
        }
        /* root_out[b] is free once round r-2's D2H has drained it */
        HIPCHK(hipSetDevice(0));
        if (r >= 2) HIPCHK(hipStreamWaitEvent(J.st[0], J.ev_drained[b], 0));
        RCCLCHK(ncclGroupStart());
        for (int g = 0; g < ngpus; ++g)
            RCCLCHK(ncclGather(J.dsh_out[g], J.root_out[b], S, ncclUint8, 0, J.comms[g], J.st[g]));
        RCCLCHK(ncclGroupEnd());
        HIPCHK(hipSetDevice(0));
        HIPCHK(hipEventRecord(J.ev_gathered[b], J.st[0]));
        HIPCHK(hipStreamWaitEvent(J.d2h, J.ev_gathered[b], 0));
        HIPCHK(hipMemcpyAsync(hout + off, J.root_out[b], n, hipMemcpyDeviceToHost, J.d2h));
        HIPCHK(hipEventRecord(J.ev_drained[b], J.d2h));
        /* every buffer reuse is ordered by the events above, so the host only
         * enqueues; it blocks in the copies when the host buffers are pageable
         * (pin them -- otc_host_register -- for H2D/D2H overlap) */
    }
    HIPCHK(hipSetDevice(0));
    if (int w = J.wait(J.st[0], timeout_s)) return w;
    if (int w = J.wait(J.d2h, timeout_s)) return w;
    return OTC_OK;
}

extern "C" void otc_multi_release(void)
{
    {
        std::lock_guard<std::mutex> lk(g_rccl_mu);
        delete g_rccl;
        g_rccl = nullptr;
    }
    std::lock_guard<std::mutex> lk(g_direct_mu);
    for (otc_engine *&e : g_direct) {
        otc_engine_destroy(e);
        e = nullptr;
    }
}

extern "C" int otc_multi_run(int ngpus, int strategy, int mode, const void *host_in, void *host_out, size_t nbytes,
                             const otc_aes_key *k, const uint8_t ivc[16], int impl, size_t chunk_bytes,
                             otc_multi_stats *stats)
{
    Range rg("otc_multi_run");
    if (int r = check_stream_args(mode, host_in, host_out, nbytes, k, ivc)) return r;
    int ndev = otc_device_count();
    if (ngpus < 1 || ngpus > ndev) return set_err(OTC_ERR_ARG, "ngpus out of range");
    const size_t nblk = (nbytes + 15) / 16;
    /* planner: contiguous block-aligned shards, remainder spread over the
     * first shards (nothing dropped, unlike reference test.c:50) */
    std::vector<size_t> boff(ngpus + 1, 0);
    for (int g = 0; g < ngpus; ++g) boff[g + 1] = boff[g] + nblk / ngpus + ((size_t)g < nblk % ngpus ? 1 : 0);
    auto t0 = std::chrono::steady_clock::now();
    int rc = OTC_OK;

    if (strategy == 0) {
        /* one host thread per GPU, each driving that GPU's cached pipeline
         * engine (pinned ring + 3 streams: created on first use, reused by
         * later calls with the same chunk size, freed by otc_multi_release).
         * Error messages are thread_local: a worker's is carried back so
         * otc_last_error() on the calling thread reports it. */
        std::lock_guard<std::mutex> lk(g_direct_mu);
        const size_t C = chunk_bytes ? ((chunk_bytes + 15) & ~(size_t)15) : (256ull << 20);
        if (g_direct.size() < (size_t)ngpus) g_direct.resize(ngpus, nullptr);
        std::vector<std::thread> th;
        std::vector<int> res(ngpus, 0);
        std::vector<std::string> msg(ngpus);
        for (int g = 0; g < ngpus; ++g) {
            th.emplace_back([&, g]() {
                const size_t b0 = std::min(boff[g] * 16, nbytes), b1 = std::min(boff[g + 1] * 16, nbytes);
                if (b1 <= b0) return;
                otc_engine *&e = g_direct[g];
                if (e && e->chunk != C) {
                    otc_engine_destroy(e);
                    e = nullptr;
                }
                if (!e) e = otc_engine_create(g, C, 3);
                if (!e) {
                    res[g] = OTC_ERR_NOMEM;
                    msg[g] = g_err;
                    return;
                }
                uint8_t iv_local[16];
                const uint8_t *ivp = ivc;
                uint64_t bo = 0;
                if (mode == OTC_MODE_CBC_DEC) {
                    if (b0 > 0) { memcpy(iv_local, (const uint8_t *)host_in + b0 - 16, 16); ivp = iv_local; }
                } else if (mode == OTC_MODE_CTR) {
                    bo = b0 / 16;
                }
                res[g] = otc_engine_run(e, mode, (const uint8_t *)host_in + b0, (uint8_t *)host_out + b0, b1 - b0, k,
                                        ivp, bo, impl, nullptr);
                if (res[g]) {
                    msg[g] = g_err;
                    otc_engine_destroy(e); /* unknown state: rebuild next time */
                    e = nullptr;
                }
            });
        }
        for (auto &t : th) t.join();
        for (int g = 0; g < ngpus; ++g)
            if (res[g]) {
                rc = res[g];
                set_err(rc, "GPU " + std::to_string(g) + ": " + msg[g]);
            }
    } else {
        rc = rccl_scatter_gather(ngpus, mode, (const uint8_t *)host_in, (uint8_t *)host_out, nbytes, k, ivc, impl,
                                 chunk_bytes);
    }
    auto t1 = std::chrono::steady_clock::now();
    if (stats) {
        stats->total_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
        stats->gbps = stats->total_ms > 0 ? (double)nbytes / (stats->total_ms * 1e6) : 0.0;
        stats->ngpus = ngpus;
        stats->strategy = strategy;
    }
    return rc;
}

extern "C" int otc_multi_ctr_resident(int ngpus, void *const *dev_bufs, size_t shard_bytes, const otc_aes_key *k,
                                      const uint8_t ctr0[16], int impl, double *elapsed_ms)
{
    Range rg("otc_multi_ctr_resident");
    if (ngpus < 1 || ngpus > otc_device_count()) return set_err(OTC_ERR_ARG, "ngpus out of range");
    if (shard_bytes % 16) return set_err(OTC_ERR_ARG, "shard must be a multiple of 16");
    std::vector<hipStream_t> st(ngpus);
    for (int g = 0; g < ngpus; ++g) {
        HIPCHK(hipSetDevice(g));
        HIPCHK(hipStreamCreateWithFlags(&st[g], hipStreamNonBlocking));
        HIPCHK(hipDeviceSynchronize());
    }
    auto t0 = std::chrono::steady_clock::now();
    for (int g = 0; g < ngpus; ++g) {
        HIPCHK(hipSetDevice(g));
        int r = otc_aes_ctr(dev_bufs[g], dev_bufs[g], shard_bytes, k, ctr0, (uint64_t)g * (shard_bytes / 16), impl, st[g]);
        if (r) return r;
    }
    for (int g = 0; g < ngpus; ++g) {
        HIPCHK(hipSetDevice(g));
        HIPCHK(hipStreamSynchronize(st[g]));
    }
    auto t1 = std::chrono::steady_clock::now();
    for (int g = 0; g < ngpus; ++g) {
        (void)hipSetDevice(g);
        (void)hipStreamDestroy(st[g]);
    }
    if (elapsed_ms) *elapsed_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
    return OTC_OK;
}

extern "C" const char *otc_build_info(void)
{
    return "otc: MI355X (gfx950) cipher engine; kernels: aes_tt (LDS T-table), aes_bs (bitsliced VALU), "
           "rc4_multi, xor; runtime: pinned 3-stream pipeline, RCCL multi-GPU";
}
