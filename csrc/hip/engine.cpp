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
#include "engine_internal.h"

using otc_dev::Ctr128;
using otc_dev::SplitClaim;
using otc_dev::BS_ECB;
using otc_dev::BS_ECB_DEC;
using otc_dev::BS_CBC_DEC;
using otc_dev::BS_CFB_DEC;
using otc_dev::BS_CBC_DEC_SEG;
using otc_dev::BS_CFB_DEC_SEG;

namespace otc_impl {
hipError_t tt_ecb_encrypt(const void *, void *, uint64_t, const otc_aes_key &, hipStream_t);
hipError_t tt_ecb_decrypt(const void *, void *, uint64_t, const otc_aes_key &, hipStream_t);
hipError_t tt_ctr(const void *, void *, size_t, const otc_aes_key &, Ctr128, bool, hipStream_t);
uint64_t tt_ctr_claim_units(size_t, uint64_t);
hipError_t tt_ctr_claim(const void *, void *, size_t, const otc_aes_key &, Ctr128, bool, SplitClaim, hipStream_t);
hipError_t tt_cfb_decrypt(const void *, void *, uint64_t, const otc_aes_key &, const uint32_t *, hipStream_t);
hipError_t tt_cbc_decrypt(const void *, void *, uint64_t, const otc_aes_key &, Ctr128, hipStream_t);
hipError_t tt_cbc_decrypt_seg(const void *, void *, uint64_t, uint64_t, const otc_aes_key &, Ctr128, hipStream_t);
hipError_t tt_cbc_encrypt_seg(const void *, void *, uint64_t, uint64_t, const otc_aes_key &, Ctr128, hipStream_t);
hipError_t tt_cfb_encrypt_seg(const void *, void *, uint64_t, uint64_t, const otc_aes_key &, Ctr128, hipStream_t);
hipError_t tt_cfb_decrypt_seg(const void *, void *, uint64_t, uint64_t, const otc_aes_key &, Ctr128, hipStream_t);
hipError_t tt_seg_encrypt_claim(bool, const void *, void *, uint64_t, uint64_t, const otc_aes_key &, Ctr128, SplitClaim,
                                hipStream_t);
int strace_read_tt(unsigned long long *, int);
int strace_read_bs(unsigned long long *, int);
hipError_t bs_ctr(const void *, void *, size_t, const otc_aes_key &, Ctr128, bool, hipStream_t);
hipError_t tt_ctr_shift(const void *, void *, size_t, const otc_aes_key &, Ctr128, hipStream_t);
hipError_t xor_small(const void *, void *, uint32_t, const uint8_t *, hipStream_t);
hipError_t bs_claim(int, const void *, void *, uint64_t, const otc_aes_key &, const uint32_t *, SplitClaim, hipStream_t);
hipError_t bs_preload();
hipError_t tt_ecb_encrypt_claim(const void *, void *, uint64_t, const otc_aes_key &, SplitClaim, hipStream_t);
hipError_t tt_cfb_decrypt_claim(const void *, void *, uint64_t, const otc_aes_key &, const uint32_t *, SplitClaim,
                                hipStream_t);
hipError_t tt_ecb_decrypt_claim(const void *, void *, uint64_t, const otc_aes_key &, SplitClaim, hipStream_t);
hipError_t tt_cbc_decrypt_claim(const void *, void *, uint64_t, const otc_aes_key &, Ctr128, SplitClaim, hipStream_t);
hipError_t bs_claim_seg(int, const void *, void *, uint64_t, const otc_aes_key &, Ctr128, uint32_t, SplitClaim,
                        hipStream_t);
hipError_t tt_cbc_decrypt_seg_claim(const void *, void *, uint64_t, const otc_aes_key &, Ctr128, uint32_t, SplitClaim,
                                    hipStream_t);
hipError_t tt_cfb_decrypt_seg_claim(const void *, void *, uint64_t, const otc_aes_key &, Ctr128, uint32_t, SplitClaim,
                                    hipStream_t);
hipError_t tt_ctr_batch(const otc_ctr_msg *, const otc_aes_key *, const uint32_t *, const uint64_t *, uint64_t, int, int,
                        hipStream_t, const SplitClaim *);
uint64_t tt_ctr_batch_units(uint64_t);
hipError_t k_xor(const void *, const void *, void *, size_t, hipStream_t);
hipError_t k_fill_random(void *, size_t, uint64_t, hipStream_t);
hipError_t k_checksum(const void *, size_t, uint64_t *, hipStream_t);
hipError_t k_clock(uint64_t *, uint64_t, uint64_t, hipStream_t);
hipError_t k_rc4_multi(const uint8_t *, int, size_t, size_t, size_t, const void *, void *, hipStream_t);
hipError_t k_rc4_states(void *, size_t, size_t, const void *, void *, hipStream_t);
} // namespace otc_impl

/* ------------------------------------------------------------------------- */
namespace otc_rt {

namespace {
thread_local std::string g_err;
}

int set_err(int code, const std::string &msg)
{
    g_err = msg;
    return code;
}

std::string last_err() { return g_err; }

int hip_fail(hipError_t e, const char *what)
{
    return set_err(OTC_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

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

int check_key(const otc_aes_key *k, int dir)
{
    if (!k) return set_err(OTC_ERR_ARG, "null key");
    if (k->nr != 10 && k->nr != 12 && k->nr != 14) return set_err(OTC_ERR_ARG, "bad key (nr)");
    if (k->dir != dir)
        return set_err(OTC_ERR_ARG, dir == OTC_DIR_ENCRYPT ? "key schedule is not an encryption schedule"
                                                           : "key schedule is not a decryption schedule");
    return OTC_OK;
}

} // namespace otc_rt

namespace otc_dev {
namespace {
std::atomic<long> g_fault_alloc{-1};
}
bool alloc_fault()
{
    /* armed with n >= 0: allocations n+1 from now fail once, then disarm */
    return g_fault_alloc.load(std::memory_order_relaxed) >= 0 &&
           g_fault_alloc.fetch_sub(1, std::memory_order_relaxed) == 0;
}
} // namespace otc_dev

extern "C" void otc_fault_inject_alloc(long after) { otc_dev::g_fault_alloc.store(after < 0 ? -1 : after); }

using namespace otc_rt;

namespace {

/* OTC_IMPL_AUTO: the measured winner (docs/PERF.md).  CTR calls of >= 2 GiB
 * (AES-256: >= 1 GiB) run bitsliced, the thresholds below; smaller CTR calls
 * (the bitsliced grid needs ~768 workgroups to fill the chip, plus two table
 * kernels per call) take the T-table.  ECB, CBC / CFB decryption: the
 * co-resident split (split_claim below) from split_min() bytes, the T-table
 * below that.  Segment encryption: T-table kernels only (seg_enc_run).
 * ctr_bytes = 0 for non-CTR calls.  OTC_IMPL=ttable|bitslice|split overrides
 * "auto" for the whole process, each where it applies: "split" for ECB and
 * the decryptions only (CTR keeps its auto choice), no override for segment
 * encryption (T-table only). */
int env_impl()
{
    static const int env = [] {
        const char *e = getenv("OTC_IMPL");
        if (!e || !*e || !strcmp(e, "auto")) return OTC_IMPL_AUTO;
        if (!strcmp(e, "ttable")) return OTC_IMPL_TTABLE;
        if (!strcmp(e, "bitslice")) return OTC_IMPL_BITSLICE;
        if (!strcmp(e, "split")) return OTC_IMPL_SPLIT;
        /* an old or mistyped value (e.g. the removed "hybrid") must not
         * silently select a different kernel: say so once */
        fprintf(stderr, "otc: ignoring OTC_IMPL=%s (expected auto, ttable, bitslice or split)\n", e);
        return OTC_IMPL_AUTO;
    }();
    return env;
}

int pick_impl(int impl, int bits, size_t ctr_bytes = 0)
{
    /* CTR has no split: "split" (per call, or OTC_IMPL=split set for the
     * whole process to get the ECB / decryption split) takes the auto choice
     * here.  The co-resident CTR split (bitsliced CTR claim + T-table CTR
     * claim kernels) lost to the bitsliced kernel alone on both HIP runtimes
     * -- AES-128 64 GiB 1600-1629 vs 1659-1669 GB/s, AES-256 16 GiB 1150-1220
     * vs 1222-1229, AES-256 64 GiB within +-2.5% -- and was removed in round
     * 6 (profiles/r6/ctr_split_rt/). */
    if (impl == OTC_IMPL_TTABLE || impl == OTC_IMPL_BITSLICE) return impl;
    const int env = impl == OTC_IMPL_SPLIT ? OTC_IMPL_AUTO : env_impl();
    if (env == OTC_IMPL_TTABLE || env == OTC_IMPL_BITSLICE) return env;
    /* measured crossover (profiles/r3/auto_impl/xover_after_round2_tables):
     * AES-128 2 GiB 1520 vs 1506 GB/s, 1 GiB 1353 vs 1360; AES-256 1 GiB
     * 1056 vs 1049.  AES-192 takes the AES-128 threshold (not measured at
     * 1 GiB; its margin lies between the two). */
    const size_t min_bs = bits == 256 ? ((size_t)1 << 30) : ((size_t)2 << 30);
    return ctr_bytes >= min_bs ? OTC_IMPL_BITSLICE : OTC_IMPL_TTABLE;
}

int check_impl(int impl)
{
    if (impl == OTC_IMPL_AUTO || impl == OTC_IMPL_TTABLE || impl == OTC_IMPL_BITSLICE || impl == OTC_IMPL_SPLIT)
        return OTC_OK;
    return set_err(OTC_ERR_ARG, "impl must be OTC_IMPL_AUTO, OTC_IMPL_TTABLE, OTC_IMPL_BITSLICE or OTC_IMPL_SPLIT");
}

/* ---- co-resident T-table + bitsliced split (ECB, CBC / CFB decryption) -----
 * The T-table kernels are LDS-bound (80% of the LDS array's cycles, 224
 * lookups per AES-256 block, VALU a third busy) and leave power on the table:
 * 1.23-1.29 kW with the package power limit active ~55-60% of the time, where
 * the VALU-bound bitsliced kernels hold the ~1.37 kW cap (profiles/r4/power).
 * A T-table workgroup (1024 threads = 4 waves per SIMD at 78-85 VGPRs, 128 or
 * 160 KiB LDS) leaves room for one bitsliced wave per SIMD (152-168 VGPRs, no
 * LDS).  So both kernels run at once on every CU over ONE buffer -- each on
 * a pooled CU-masked stream with a hardware queue of its own (fork / join
 * events with the caller's stream, aux_take) -- and take 2048-block units from a shared
 * counter, the bitsliced kernel from the front and the T-table from the back
 * (otc_device.h SplitClaim), so they finish together on any box: no share to
 * tune, no tail where one kernel runs alone.  Measured: docs/PERF.md
 * "Round 4" (the static shares this replaced: profiles/r4/ecb_split,
 * dec_split, cfb_split). */
struct AuxStream {
    int dev = -1;
    hipStream_t s = nullptr, t = nullptr; /* the bitsliced / the T-table half */
    hipEvent_t fork = nullptr, join = nullptr, join_t = nullptr;
};

/* pooled per device: a call takes one (creating it on first use), enqueues,
 * and returns it, so concurrent callers (one host thread per GPU in
 * otc_multi_run) never share the events they order on */
std::mutex g_aux_mu;
std::vector<AuxStream> g_aux_free;
/* AuxStreams created per device (in the pool or taken).  Each holds two
 * dedicated hardware queues, so the pool is capped: past AUX_MAX concurrent
 * split calls on one device a call runs the T-table alone and records why
 * (otc_split_fallback_reason) instead of taking more device queues. */
constexpr int AUX_MAX = 4;
int g_aux_live[64];
thread_local const char *g_split_fallback = "";

__global__ void k_aux_noop() {}

hipError_t aux_take(int dev, AuxStream &out, bool warm)
{
    {
        std::lock_guard<std::mutex> lk(g_aux_mu);
        for (size_t i = 0; i < g_aux_free.size(); ++i)
            if (g_aux_free[i].dev == dev) {
                out = g_aux_free[i];
                g_aux_free.erase(g_aux_free.begin() + (long)i);
                return hipSuccess;
            }
        if (dev < 0 || dev >= 64 || g_aux_live[dev] >= AUX_MAX) {
            g_split_fallback = "auxiliary stream pool exhausted (AUX_MAX concurrent split calls on this device)";
            return hipErrorOutOfMemory;
        }
        ++g_aux_live[dev]; /* reserved; released below if creation fails */
    }
    AuxStream a;
    a.dev = dev;
    /* both halves on streams with an all-CU mask: HIP gives a CU-masked
     * stream a hardware queue of its own.  On pooled queues (4 per process
     * here) a library stream can share one with the caller's stream or with
     * the other half, and then the two kernels run one after the other: in
     * bench.py, beside torch's and RCCL's streams, the CTR split ran at the
     * T-table's speed (1534 GB/s) */
#ifdef OTC_DIAG_POOLED_AUX
    /* A/B arm only (make variant NAME=pooledaux VFLAGS=-DOTC_DIAG_POOLED_AUX):
     * both halves on plain non-blocking streams, i.e. HIP's pooled queues */
    hipError_t e = hipStreamCreateWithFlags(&a.s, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&a.t, hipStreamNonBlocking);
#else
    hipError_t e = dedicated_stream_create(&a.s);
    if (e == hipSuccess) e = dedicated_stream_create(&a.t);
#endif
    if (e == hipSuccess) e = hipEventCreateWithFlags(&a.fork, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&a.join, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&a.join_t, hipEventDisableTiming);
    /* A new AuxStream's one-time costs, paid here and not inside the first
     * split (whose T-table half is already queued when the bitsliced half
     * launches -- engine.cpp split_claim): the bitsliced code object, and a
     * first submission on each queue.  Without this a process's first split
     * ran its halves one after the other (front 0 in 1 of 64 calls,
     * profiles/r6/coresidency/matrix.jsonl). */
    if (warm && e == hipSuccess && otc_impl::bs_preload() != hipSuccess)
        (void)hipGetLastError(); /* only a warm-up: the split works without it */
    /* not while the caller's stream is being captured into a graph: a
     * synchronisation there would invalidate the caller's capture */
    if (warm && e == hipSuccess) {
        hipLaunchKernelGGL(k_aux_noop, dim3(1), dim3(1), 0, a.s);
        hipLaunchKernelGGL(k_aux_noop, dim3(1), dim3(1), 0, a.t);
        if ((e = hipGetLastError()) == hipSuccess && (e = hipStreamSynchronize(a.s)) == hipSuccess)
            e = hipStreamSynchronize(a.t);
    }
    if (e != hipSuccess) {
        if (a.join_t) (void)hipEventDestroy(a.join_t);
        if (a.join) (void)hipEventDestroy(a.join);
        if (a.fork) (void)hipEventDestroy(a.fork);
        if (a.t) (void)hipStreamDestroy(a.t);
        if (a.s) (void)hipStreamDestroy(a.s);
        std::lock_guard<std::mutex> lk(g_aux_mu);
        --g_aux_live[dev];
        g_split_fallback = "auxiliary stream creation failed";
        return e;
    }
    out = a;
    return hipSuccess;
}

void aux_give(const AuxStream &a)
{
    std::lock_guard<std::mutex> lk(g_aux_mu);
    g_aux_free.push_back(a);
}

/* the smallest call that splits: 2 GiB.  Measured with the kernels truly
 * co-resident (round 5, profiles/r5/split_ab/remeasure_int_lds.jsonl,
 * split_thresholds/thresh2_int_lds.jsonl): against the grid T-table, AES-256
 * ECB wins 15% at 2 GiB, 24% at 4 and 64 GiB, CBC-dec 10% at 2 GiB and 21% at
 * 16 GiB, CFB-dec 26% at 16 GiB; at 1 GiB and below it is mixed (ECB 512 MiB
 * +3%, 1 GiB -13% on one box; CBC-dec 512 MiB -2%, 1 GiB +2%) and at 256 MiB
 * it loses 2-11%: each of the 4096 T-table waves then gets only one or two
 * 32 KiB units, and 256 x 128 KiB of LDS table fills plus the fork / join
 * are a fixed cost.  (Round 4's 896 MiB was measured while the halves ran one
 * after the other: docs/PERF.md round 5.) */
size_t split_min(int) { return (size_t)2 << 30; }

int pick_ecb_impl(int impl, int bits, size_t nbytes)
{
    if (impl == OTC_IMPL_TTABLE || impl == OTC_IMPL_BITSLICE || impl == OTC_IMPL_SPLIT) return impl;
    const int env = env_impl();
    if (env != OTC_IMPL_AUTO) return env;
    return nbytes >= split_min(bits) ? OTC_IMPL_SPLIT : OTC_IMPL_TTABLE;
}

int pick_dec_impl(int impl, int bits, size_t nbytes) { return pick_ecb_impl(impl, bits, nbytes); }

/* Split accounting (otc_split_stats): off by default -- one relaxed load
 * per split call.  On, each split call copies its claim word back and waits
 * for it (a profiling mode), so the caller can read how many units each side
 * took. */
std::atomic<int> g_split_stats{0};
__global__ void k_claim_snapshot(unsigned long long *ctr, unsigned long long *host)
{
    const unsigned long long v = __hip_atomic_fetch_add(ctr, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(host, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
thread_local uint64_t g_split_word = 0, g_split_nunits = 0, g_split_ttwaves = 0, g_split_pb = 0;

/* The split: tt(cl) launches the T-table claim kernel on st, bs(cl, aux) the
 * bitsliced claim kernel on the auxiliary stream, both over the whole buffer
 * (nunits claim units, the T-table kernel also runs what lies past the last
 * unit); plain() is the T-table alone (too few units, or no memory for the
 * counter / no auxiliary stream).  bs_only: impl "bitslice" -- the T-table
 * kernel's back counter starts full, so the bitsliced kernel (bs_wgs
 * workgroups) takes every unit and one T-table workgroup runs the rest.
 * *ran: the kernels actually used. */
template <class TT, class BS, class PLAIN>
hipError_t split_claim(uint64_t nunits, uint64_t min_units, bool bs_only, unsigned bs_wgs, hipStream_t st, int *ran,
                       TT tt, BS bs, PLAIN plain)
{
    *ran = OTC_IMPL_TTABLE;
    g_split_fallback = "";
    /* bs_wgs 0 (and not bs_only): the T-table claim kernel alone, no fork --
     * not a split request, so nothing to report if it runs plain() */
    const bool fork = bs_wgs != 0 || bs_only;
    if (nunits < (bs_only ? 1 : min_units) || nunits > 0x7FFFFFFFull) {
        if (fork) g_split_fallback = "too few claim units";
        return plain();
    }
    unsigned long long *ctr = nullptr;
    /* word 0: the shared claim word; word 1 (bs_only): the T-table kernel's
     * own word, preset to "every unit taken" */
    hipError_t e = otc_dev::alloc_fault() ? hipErrorOutOfMemory : hipMallocAsync((void **)&ctr, 2 * sizeof *ctr, st);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        if (fork) g_split_fallback = "no memory for the claim counter";
        return plain();
    }
    int dev = 0;
    AuxStream a;
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (fork && hipStreamIsCapturing(st, &cap) != hipSuccess) {
        (void)hipGetLastError();
        cap = hipStreamCaptureStatusActive; /* unknown: take the safe side */
    }
    if (fork && (hipGetDevice(&dev) != hipSuccess || aux_take(dev, a, cap == hipStreamCaptureStatusNone) != hipSuccess)) {
        /* no auxiliary stream: the T-table alone still gives the output */
        (void)hipGetLastError();
        (void)hipFreeAsync(ctr, st);
        return plain();
    }
    /* first units handed out without a claim (otc_device.h SplitClaim): the
     * last ones to the T-table waves (16 per workgroup, one workgroup per
     * CU), the first ones to the bitsliced waves (4 per workgroup) */
#ifndef OTC_CLAIM_NO_PREASSIGN /* A/B arm: every unit claimed (make variant VFLAGS=-DOTC_CLAIM_NO_PREASSIGN) */
    const uint32_t pb = bs_only ? 0u : (uint32_t)std::min<uint64_t>(nunits, 16ull * (uint64_t)otc_dev::device_cus());
    const uint32_t pf = (uint32_t)std::min<uint64_t>(nunits - pb, 4ull * bs_wgs);
#else
    const uint32_t pb = 0, pf = 0;
#endif
    SplitClaim cl{ctr, (uint32_t)nunits, bs_wgs};
    cl.pf = pf;
    cl.pb = pb;
    SplitClaim cl_tt{bs_only ? ctr + 1 : ctr, (uint32_t)nunits, bs_only ? 1u : 0u};
    cl_tt.pf = bs_only ? 0u : pf;
    cl_tt.pb = pb;
    /* word 0 zeroed; word 1 only where it is used (bs_only: the T-table's
     * word, all ones -- front + back far past nunits, so its claims fail;
     * hipMemsetD32Async at a 4-byte offset cost ~40 ms per call): one fill
     * kernel per call instead of two (no measurable rate change at 0.5-2 GiB,
     * profiles/r6/claim_tail/one_fill_ab.jsonl).  Then fork: the aux stream
     * starts after everything queued on st */
    if ((e = hipMemsetAsync(ctr, 0, sizeof *ctr, st)) == hipSuccess &&
        (!bs_only || (e = hipMemsetAsync(ctr + 1, 0xFF, sizeof *ctr, st)) == hipSuccess) &&
        (!fork || ((e = hipEventRecord(a.fork, st)) == hipSuccess && (e = hipStreamWaitEvent(a.s, a.fork, 0)) == hipSuccess &&
                   (e = hipStreamWaitEvent(a.t, a.fork, 0)) == hipSuccess)) &&
        (e = tt(cl_tt, fork ? a.t : st)) == hipSuccess) {
        /* The T-table half is enqueued first on purpose: its 1024-thread,
         * 128-160 KiB-LDS workgroups fit one per CU only when they are placed
         * before the bitsliced ones (two or three 168-VGPR bitsliced
         * workgroups on one CU leave no room for a T-table workgroup there).
         * The bitsliced half's one-time costs (its code object, a first
         * submission on each auxiliary queue) are therefore paid when the
         * AuxStream is created (aux_take), not here: paid here, they let a
         * process's first split call run the T-table half alone (front 0,
         * profiles/r6/coresidency/matrix.jsonl; with the warm-up the first
         * call co-runs, matrix_warm_aux.jsonl).
         * The bitsliced half failing (no memory for its key table) leaves the
         * T-table claim kernel to take every unit -- unless it was told to
         * take none (bs_only): then the T-table alone redoes the call.  The
         * join is recorded either way (a failure after its launch must still
         * be waited for). */
        const hipError_t eb = bs_wgs ? bs(cl, a.s) : hipSuccess;
        if (eb != hipSuccess) {
            (void)hipGetLastError();
            g_split_fallback = "the bitsliced half failed to launch";
        }
        if (fork && (e = hipEventRecord(a.join, a.s)) == hipSuccess && (e = hipEventRecord(a.join_t, a.t)) == hipSuccess &&
            (e = hipStreamWaitEvent(st, a.join, 0)) == hipSuccess)
            e = hipStreamWaitEvent(st, a.join_t, 0);
        if (e == hipSuccess) {
            if (eb == hipSuccess && bs_wgs) *ran = bs_only ? OTC_IMPL_BITSLICE : OTC_IMPL_SPLIT;
            else if (bs_only) e = plain();
            if (e == hipSuccess && g_split_stats.load(std::memory_order_relaxed)) {
                /* the counter's last value sits where the agent-scope atomics
                 * left it: read it with one (an ordinary copy can see a stale
                 * line) into pinned host memory */
                thread_local unsigned long long *snap = nullptr;
                if (!snap && hipHostMalloc((void **)&snap, sizeof *snap, hipHostMallocDefault) != hipSuccess) {
                    (void)hipGetLastError();
                    snap = nullptr;
                }
                if (snap) {
                    hipLaunchKernelGGL(k_claim_snapshot, dim3(1), dim3(1), 0, st, ctr, snap);
                    if ((e = hipGetLastError()) == hipSuccess) e = hipStreamSynchronize(st);
                }
                if (snap && e == hipSuccess) {
                    const uint64_t w = *(volatile unsigned long long *)snap;
                    g_split_word = bs_only ? (uint64_t)nunits : w; /* bs_only: the T-table has its own word */
                    g_split_nunits = nunits;
                    /* every T-table claim kernel runs 1024-thread workgroups,
                     * one per CU; each of their waves ends on one failed
                     * claim */
                    g_split_ttwaves = bs_only ? 0 : 16ull * (uint64_t)otc_dev::device_cus();
                    g_split_pb = pb; /* the T-table's units taken without a claim */
                }
            }
        } else if (fork) {
            /* no join on st: the counter must outlive both kernels */
            (void)hipStreamSynchronize(a.s);
            (void)hipStreamSynchronize(a.t);
        }
    }
    const hipError_t f = hipFreeAsync(ctr, st); /* after the join: both kernels are done with it */
    if (fork) aux_give(a); /* reusable as soon as the work is enqueued: stream order */
    return e != hipSuccess ? e : f;
}

/* The claimed forms of ECB and the decryptions: the co-resident split, the
 * bitsliced claim kernel alone (impl "bitslice"), or the persistent T-table
 * claim kernel alone -- one workgroup per CU, its LDS table filled once,
 * units claimed until none are left.  auto runs the last for the T-table
 * calls of [896 MiB, 2 GiB): against the grid kernel ECB-256 1000 MiB 1089
 * vs 1039, ECB-dec 1073 vs 966, CBC-dec 1049 vs 1017 (round 4's "split", which
 * was this kernel alone: profiles/r4/claim_split/mid_sizes.jsonl); 1 GiB
 * ECB-256 1026 vs 988, AES-128 1282 vs 1238 (profiles/r5/split_thresholds/);
 * round 5 at 1000 MiB (midsize_persistent_vs_grid.jsonl, 2 reps): ECB-256
 * 1068-1074 vs 1027-1031, ECB-dec-256 1053-1056 vs 872-911, CBC / CFB-dec
 * +1%, ECB-128 +2-9%; 1.5 GiB -4..+7%; at 512 MiB and below it ties or
 * loses.  Round 6, with the first claim units handed out (no first-claim
 * queue): from 512 MiB -- ECB-128 512 / 768 MiB +2.8 / +3.7%, ECB-256 +4.4 /
 * +4.4%, ECB-dec-256 +2.8 / +5.5%, CBC-dec-128 -1 / +2.7%; at 256 MiB mixed
 * (-4..+1.5%) (profiles/r6/xover/). */
enum { FORM_SPLIT = 0, FORM_BS = 1, FORM_TT = 2 };
/* OTC_TT_PERSISTENT_MIN_MIB / OTC_SEGENC_PERSISTENT_MIN_MIB: threshold
 * sweeps only (read once; unset = the measured defaults) */
size_t env_mib(const char *name, size_t dflt)
{
    const char *v = getenv(name);
    return v && *v ? (size_t)strtoull(v, nullptr, 10) << 20 : dflt;
}
/* CTR on the T-table: the persistent claim kernel from this size (A/B and
 * threshold sweeps: OTC_TT_CTR_PERSISTENT_MIN_MIB) */
size_t tt_ctr_persistent_min()
{
    static const size_t m = env_mib("OTC_TT_CTR_PERSISTENT_MIN_MIB", (size_t)512 << 20);
    return m;
}
size_t tt_persistent_min()
{
    static const size_t m = env_mib("OTC_TT_PERSISTENT_MIN_MIB", (size_t)512 << 20);
    return m;
}
int split_form(int picked, size_t nbytes)
{
    if (picked == OTC_IMPL_SPLIT) return FORM_SPLIT;
    if (picked == OTC_IMPL_BITSLICE) return FORM_BS;
    return nbytes >= tt_persistent_min() ? FORM_TT : -1;
}

/* bitsliced claim workgroups: one per CU beside the T-table (4 T-table waves
 * + 1 bitsliced wave per SIMD), three per CU alone (<= 168 VGPRs), none for
 * the T-table alone */
unsigned bs_wgs_for(int form)
{
    return form == FORM_TT ? 0u : (unsigned)otc_dev::device_cus() * (form == FORM_BS ? 3u : 1u);
}

hipError_t ecb_split(const void *in, void *out, uint64_t nblocks, const otc_aes_key &K, int form, hipStream_t st,
                     int *ran)
{
    const uint64_t nunits = nblocks / otc_dev::CLAIM_UNIT;
    if (K.dir == OTC_DIR_ENCRYPT)
        return split_claim(
            nunits, 2, form == FORM_BS, bs_wgs_for(form), st, ran,
            [&](SplitClaim cl, hipStream_t ts) { return otc_impl::tt_ecb_encrypt_claim(in, out, nblocks, K, cl, ts); },
            [&](SplitClaim cl, hipStream_t s) { return otc_impl::bs_claim(BS_ECB, in, out, nblocks, K, nullptr, cl, s); },
            [&]() { return otc_impl::tt_ecb_encrypt(in, out, nblocks, K, st); });
    return split_claim(
        nunits, 2, form == FORM_BS, bs_wgs_for(form), st, ran,
        [&](SplitClaim cl, hipStream_t ts) { return otc_impl::tt_ecb_decrypt_claim(in, out, nblocks, K, cl, ts); },
        [&](SplitClaim cl, hipStream_t s) { return otc_impl::bs_claim(BS_ECB_DEC, in, out, nblocks, K, nullptr, cl, s); },
        [&]() { return otc_impl::tt_ecb_decrypt(in, out, nblocks, K, st); });
}

hipError_t cbc_dec_split(const void *in, void *out, uint64_t nblocks, const otc_aes_key &K, const uint8_t iv[16],
                         int form, hipStream_t st, int *ran)
{
    uint32_t ivw[4];
    memcpy(ivw, iv, 16); /* the bitsliced kernel's IV: LE words of the bytes */
    const Ctr128 ivc = ctr_from_bytes(iv);
    return split_claim(
        nblocks / otc_dev::CLAIM_UNIT, 2, form == FORM_BS, bs_wgs_for(form), st, ran,
        [&](SplitClaim cl, hipStream_t ts) { return otc_impl::tt_cbc_decrypt_claim(in, out, nblocks, K, ivc, cl, ts); },
        [&](SplitClaim cl, hipStream_t s) { return otc_impl::bs_claim(BS_CBC_DEC, in, out, nblocks, K, ivw, cl, s); },
        [&]() { return otc_impl::tt_cbc_decrypt(in, out, nblocks, K, ivc, st); });
}

hipError_t cfb_dec_split(const void *in, void *out, uint64_t nblocks, const otc_aes_key &K, const uint32_t ivw[4],
                         int form, hipStream_t st, int *ran)
{
    return split_claim(
        nblocks / otc_dev::CLAIM_UNIT, 2, form == FORM_BS, bs_wgs_for(form), st, ran,
        [&](SplitClaim cl, hipStream_t ts) { return otc_impl::tt_cfb_decrypt_claim(in, out, nblocks, K, ivw, cl, ts); },
        [&](SplitClaim cl, hipStream_t s) { return otc_impl::bs_claim(BS_CFB_DEC, in, out, nblocks, K, ivw, cl, s); },
        [&]() { return otc_impl::tt_cfb_decrypt(in, out, nblocks, K, ivw, st); });
}

/* Segment decryption (CBC / CFB128 over independent segments of 2^shift
 * blocks, IV_s = iv0 + s): the same split, each kernel computing the segment
 * IVs itself.  Non-power-of-two segments and short calls: the T-table. */
int seg_shift_of(size_t seg_blocks)
{
    if (seg_blocks == 0 || (seg_blocks & (seg_blocks - 1))) return -1;
    int sh = 0;
    while (((size_t)1 << sh) < seg_blocks) ++sh;
    return sh;
}

int pick_seg_impl(int impl, int bits, size_t nbytes, size_t seg_blocks)
{
    if (seg_shift_of(seg_blocks) < 0) return OTC_IMPL_TTABLE;
    return pick_ecb_impl(impl, bits, nbytes);
}

hipError_t seg_dec_split(bool cfb, const void *in, void *out, size_t seg_blocks, size_t nseg, const otc_aes_key &K,
                         Ctr128 iv0, int form, hipStream_t st, int *ran)
{
    const uint64_t nblocks = (uint64_t)seg_blocks * nseg;
    const uint32_t sh = (uint32_t)seg_shift_of(seg_blocks);
    auto plain = [&]() {
        return cfb ? otc_impl::tt_cfb_decrypt_seg(in, out, seg_blocks, nseg, K, iv0, st)
                   : otc_impl::tt_cbc_decrypt_seg(in, out, seg_blocks, nseg, K, iv0, st);
    };
    return split_claim(
        nblocks / otc_dev::CLAIM_UNIT, 2, form == FORM_BS, bs_wgs_for(form), st, ran,
        [&](SplitClaim cl, hipStream_t ts) {
            return cfb ? otc_impl::tt_cfb_decrypt_seg_claim(in, out, nblocks, K, iv0, sh, cl, ts)
                       : otc_impl::tt_cbc_decrypt_seg_claim(in, out, nblocks, K, iv0, sh, cl, ts);
        },
        [&](SplitClaim cl, hipStream_t s) {
            return otc_impl::bs_claim_seg(cfb ? BS_CFB_DEC_SEG : BS_CBC_DEC_SEG, in, out, nblocks, K, iv0, sh, cl, s);
        },
        plain);
}

/* the kernel family the calling thread's last AES call ran (otc_last_impl) */
thread_local int g_last_impl = OTC_IMPL_AUTO;

/* Segment ENCRYPTION (CBC / CFB128, one serial chain per segment): T-table
 * kernels only, for every impl.  Two forms: the grid kernel, and the
 * persistent claim kernel (64-segment units from one counter, one workgroup
 * per CU, its LDS table filled once), from 2 GiB (from 1 GiB for segments <=
 * 1 KiB), where it beats the grid kernel by 4-15% (AES-256 4 KiB segments:
 * 2 GiB 1027 vs 986, 4 GiB 1040 vs 969, 32 GiB 1142 vs 995; 512 B at 1 GiB
 * 986 vs 951; AES-128 4 GiB 1383 vs 1267); below that the grid kernel (1 GiB
 * of 4 KiB segments: 916 vs 948; profiles/r5/split_thresholds/).  Round 6,
 * first claim units handed out: from 1 GiB for every segment size (AES-256
 * 4 KiB segments: 1 GiB 957-959 vs 948-950, 1.5 GiB 1036 vs 790-801 -- the
 * grid kernel's 384 workgroups there are 1.5 per CU; 512 MiB 542 vs 554-558;
 * profiles/r6/xover/).  A VALU
 * half for this mode (the row-sliced 8-chains-per-lane kernel of round 5)
 * lost at every size -- AES-256 4 GiB 775 vs 1040 GB/s for the claim kernel
 * alone (profiles/r5/split_ab/remeasure_int_lds.jsonl) -- and was removed
 * in round 6 (profiles/r6/retired/). */
constexpr uint64_t SEG_UNIT = 64;

int pick_segenc_impl(int, size_t, size_t) { return OTC_IMPL_TTABLE; }

bool segenc_persistent(size_t nbytes, size_t seg_bytes, size_t nseg)
{
    static const size_t env = env_mib("OTC_SEGENC_PERSISTENT_MIN_MIB", (size_t)1 << 30);
    const size_t min_bytes = env;
    (void)seg_bytes;
    return nbytes >= min_bytes && nseg / SEG_UNIT >= 16 && nseg / SEG_UNIT <= 0x7FFFFFFFull;
}

hipError_t seg_enc_run(bool cfb, const void *in, void *out, size_t seg_bytes, size_t nseg, const otc_aes_key &K,
                       Ctr128 iv0, hipStream_t st)
{
    const size_t seg_blocks = seg_bytes / 16;
    g_last_impl = OTC_IMPL_TTABLE;
    auto grid = [&]() {
        return cfb ? otc_impl::tt_cfb_encrypt_seg(in, out, seg_blocks, nseg, K, iv0, st)
                   : otc_impl::tt_cbc_encrypt_seg(in, out, seg_blocks, nseg, K, iv0, st);
    };
    if (!segenc_persistent(seg_bytes * nseg, seg_bytes, nseg)) return grid();
    return split_claim(
        nseg / SEG_UNIT, 16, false, 0u, st, &g_last_impl,
        [&](SplitClaim cl, hipStream_t ts) { return otc_impl::tt_seg_encrypt_claim(cfb, in, out, seg_blocks, nseg, K, iv0, cl, ts); },
        [&](SplitClaim, hipStream_t) { return hipErrorInvalidValue; /* no VALU half: bs_wgs = 0 never calls it */ },
        grid);
}


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
extern "C" const char *otc_last_error(void)
{
    thread_local std::string copy;
    copy = last_err();
    return copy.c_str();
}

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

/* mode: 1 CTR, 0 ECB encryption, 2 decryption (ECB / CBC), 3 CFB decryption, 4 segment decryption
 * (power-of-two segments), 5 segment encryption (segments < 8 MiB) */
extern "C" int otc_pick_impl(int impl, int bits, int mode, uint64_t nbytes)
{
    if (check_impl(impl)) return -1;
    if (mode == 0 || mode == 3) return pick_ecb_impl(impl, bits, (size_t)nbytes);
    if (mode == 2) return pick_dec_impl(impl, bits, (size_t)nbytes);
    if (mode == 4) return pick_seg_impl(impl, bits, (size_t)nbytes, 1);
    if (mode == 5) return pick_segenc_impl(impl, (size_t)nbytes, 16);
    if (mode == 1) return pick_impl(impl, bits, (size_t)nbytes);
    return -1;
}

/* the auxiliary streams of the split (otc_release_resources) */
void otc_rt::aux_release_all()
{
    std::lock_guard<std::mutex> lk(g_aux_mu);
    int cur = 0;
    (void)hipGetDevice(&cur);
    for (AuxStream &a : g_aux_free) {
        (void)hipSetDevice(a.dev);
        (void)hipStreamSynchronize(a.s);
        (void)hipStreamSynchronize(a.t);
        (void)hipEventDestroy(a.fork);
        (void)hipEventDestroy(a.join);
        (void)hipEventDestroy(a.join_t);
        (void)hipStreamDestroy(a.s);
        (void)hipStreamDestroy(a.t);
        if (a.dev >= 0 && a.dev < 64) --g_aux_live[a.dev];
    }
    g_aux_free.clear();
    (void)hipSetDevice(cur);
}

extern "C" int otc_last_impl(void) { return g_last_impl; }

/* which: 0 the T-table kernels' records, 1 the bitsliced (32-block) claim
 * kernels'; -1 in a build without OTC_SPLIT_TRACE */
extern "C" int otc_split_trace(int which, unsigned long long *buf, int max)
{
    if (!buf || max < 0) return set_err(OTC_ERR_ARG, "bad trace buffer");
    if (which != 0 && which != 1) return set_err(OTC_ERR_ARG, "which must be 0 (T-table) or 1 (bitsliced)");
    return which == 0 ? otc_impl::strace_read_tt(buf, max) : otc_impl::strace_read_bs(buf, max);
}

extern "C" const char *otc_split_fallback_reason(void) { return g_split_fallback; }

extern "C" void otc_split_stats(int on) { g_split_stats.store(on ? 1 : 0, std::memory_order_relaxed); }

extern "C" int otc_split_last_units(uint64_t *front, uint64_t *back, uint64_t *nunits)
{
    if (!front || !back || !nunits) return set_err(OTC_ERR_ARG, "null argument");
    /* every T-table wave ends on one failed back claim (+1 each), so the
     * back count less those, plus the units the T-table waves started on
     * without a claim, is what the T-table took; the front took the rest */
    const uint64_t b = g_split_word >> 32, n = g_split_nunits;
    *back = std::min(n, g_split_pb + (b > g_split_ttwaves ? b - g_split_ttwaves : 0));
    *front = n - *back;
    *nunits = n;
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
    if (int r = check_impl(impl)) return r;
    if (nbytes == 0) return OTC_OK;
    hipStream_t st = (hipStream_t)stream;
    hipError_t e;
    if (k->dir == OTC_DIR_ENCRYPT) {
        g_last_impl = pick_ecb_impl(impl, k->bits, nbytes);
    } else {
        g_last_impl = pick_dec_impl(impl, k->bits, nbytes);
    }
    if (const int form = split_form(g_last_impl, nbytes); form >= 0)
        e = ecb_split(in, out, nbytes / 16, *k, form, st, &g_last_impl);
    else if (k->dir == OTC_DIR_ENCRYPT)
        e = otc_impl::tt_ecb_encrypt(in, out, nbytes / 16, *k, st);
    else
        e = otc_impl::tt_ecb_decrypt(in, out, nbytes / 16, *k, st);
    if (e != hipSuccess) return hip_fail(e, "aes_ecb launch");
    return OTC_OK;
}

static int ctr_common(const void *in, void *out, size_t nbytes, const otc_aes_key *k, Ctr128 c, bool wrap64,
                      int impl, void *stream)
{
    int r = check_key(k, OTC_DIR_ENCRYPT);
    if (r) return r;
    if ((r = check_bufs(in, out, nbytes, true, "aes_ctr"))) return r;
    if ((r = check_impl(impl))) return r; /* before the empty-call return, as otc_aes_ecb */
    if (nbytes == 0) return OTC_OK;
    hipStream_t st = (hipStream_t)stream;
    const int im = pick_impl(impl, k->bits, nbytes);
    g_last_impl = im;
    hipError_t e;
    if (im == OTC_IMPL_BITSLICE) {
        e = otc_impl::bs_ctr(in, out, nbytes, *k, c, wrap64, st);
    } else if (nbytes >= tt_ctr_persistent_min()) {
        /* the T-table as a persistent claim kernel (first units handed out,
         * the rest claimed): no CU waits on another's static share */
        e = split_claim(
            otc_impl::tt_ctr_claim_units(nbytes, c.lo), 2, false, 0u, st, &g_last_impl,
            [&](SplitClaim cl, hipStream_t ts) { return otc_impl::tt_ctr_claim(in, out, nbytes, *k, c, wrap64, cl, ts); },
            [&](SplitClaim, hipStream_t) { return hipErrorInvalidValue; /* bs_wgs 0: no VALU half */ },
            [&]() { return otc_impl::tt_ctr(in, out, nbytes, *k, c, wrap64, st); });
    } else {
        e = otc_impl::tt_ctr(in, out, nbytes, *k, c, wrap64, st);
    }
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

/* ---- resumable CTR stream (PolarSSL aes_crypt_ctr semantics on device) ----
 * Reference: aes-modes/aes.c:869-900 -- byte-granular nc_off, the keystream
 * block of the current counter kept in stream_block, the counter advanced when
 * a block is generated.  The host edge does the partial blocks: the head
 * (bytes left in stream_block) is one tiny XOR launch with those bytes as
 * kernel arguments, the tail's keystream block is computed on the host (one
 * AES block) and kept in the context; the kernels do every whole block.  A
 * body left misaligned by the head runs the funnel-shift kernel. */
extern "C" int otc_aes_ctr_ctx_init(otc_aes_ctr_ctx *ctx, const uint8_t nonce_counter[16])
{
    if (!ctx || !nonce_counter) return set_err(OTC_ERR_ARG, "null argument");
    memset(ctx, 0, sizeof *ctx);
    memcpy(ctx->nonce_counter, nonce_counter, 16);
    return OTC_OK;
}

extern "C" int otc_aes_ctr_stream(otc_aes_ctr_ctx *ctx, const otc_aes_key *k, size_t length, const void *in,
                                  void *out, int impl, void *stream)
{
    Range rg("otc_aes_ctr_stream");
    if (!ctx) return set_err(OTC_ERR_ARG, "null context");
    if (ctx->nc_off > 15) return set_err(OTC_ERR_ARG, "nc_off must be 0..15");
    int r = check_key(k, OTC_DIR_ENCRYPT);
    if (r) return r;
    if (length == 0) return OTC_OK;
    if (!in || !out) return set_err(OTC_ERR_ARG, "aes_ctr_stream: null buffer");
    const uintptr_t a = (uintptr_t)in, b = (uintptr_t)out;
    if (a != b && a < b + length && b < a + length)
        return set_err(OTC_ERR_ARG, "aes_ctr_stream: input and output overlap partially");
    if ((a & 15u) != (b & 15u))
        return set_err(OTC_ERR_ARG, "aes_ctr_stream: in and out must have the same alignment modulo 16");
    hipStream_t st = (hipStream_t)stream;
    const size_t n0 = ctx->nc_off;
    const size_t head = n0 ? std::min(length, (size_t)16 - n0) : 0;
    if (head) {
        hipError_t e = otc_impl::xor_small(in, out, (uint32_t)head, ctx->stream_block + n0, st);
        if (e != hipSuccess) return hip_fail(e, "ctr_stream head");
    }
    const size_t body = length - head;
    if (body == 0) {
        ctx->nc_off = (n0 + head) & 15u;
        return OTC_OK;
    }
    const uint8_t *bi = (const uint8_t *)in + head;
    uint8_t *bo = (uint8_t *)out + head;
    const Ctr128 c = ctr_from_bytes(ctx->nonce_counter);
    if ((((uintptr_t)bi) & 15u) == 0) {
        if ((r = ctr_common(bi, bo, body, k, c, false, impl, stream))) return r;
    } else {
        hipError_t e = otc_impl::tt_ctr_shift(bi, bo, body, *k, c, st);
        if (e != hipSuccess) return hip_fail(e, "ctr_stream body (misaligned)");
    }
    const uint64_t full = body / 16, tail = body % 16;
    if (tail) { /* keep the keystream block of the partial tail */
        Ctr128 t = ctr_add(c, full, false);
        uint8_t cb[16];
        for (int i = 0; i < 8; ++i) cb[i] = (uint8_t)(t.hi >> (56 - 8 * i));
        for (int i = 0; i < 8; ++i) cb[8 + i] = (uint8_t)(t.lo >> (56 - 8 * i));
        aes_context actx;
        aes_import_rk32(&actx, k->rk, k->nr);
        aes_crypt_ecb(&actx, AES_ENCRYPT, cb, ctx->stream_block);
    }
    const Ctr128 nx = ctr_add(c, full + (tail ? 1 : 0), false);
    for (int i = 0; i < 8; ++i) ctx->nonce_counter[i] = (uint8_t)(nx.hi >> (56 - 8 * i));
    for (int i = 0; i < 8; ++i) ctx->nonce_counter[8 + i] = (uint8_t)(nx.lo >> (56 - 8 * i));
    ctx->nc_off = (size_t)tail;
    return OTC_OK;
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
    hipStream_t st = (hipStream_t)stream;
    auto plain = [&]() { return otc_impl::tt_ctr_batch(msgs, keys, tile_msg, tile_first, ntiles, tile_blocks, nr, st, nullptr); };
    /* large batches: claimed tile runs (first one handed out) instead of the
     * static split over the waves (A/B: OTC_BATCH_CLAIM_MIN_TILES) */
    static const uint64_t min_tiles = [] {
        const char *v = getenv("OTC_BATCH_CLAIM_MIN_TILES");
        return v && *v ? (uint64_t)strtoull(v, nullptr, 10) : (uint64_t)65536;
    }();
    int ran = 0;
    hipError_t e = ntiles >= min_tiles
                       ? split_claim(
                             otc_impl::tt_ctr_batch_units(ntiles), 2, false, 0u, st, &ran,
                             [&](SplitClaim cl, hipStream_t ts) {
                                 return otc_impl::tt_ctr_batch(msgs, keys, tile_msg, tile_first, ntiles, tile_blocks, nr,
                                                               ts, &cl);
                             },
                             [&](SplitClaim, hipStream_t) { return hipErrorInvalidValue; /* no VALU half */ }, plain)
                       : plain();
    if (e != hipSuccess) return hip_fail(e, "ctr_batch launch");
    return OTC_OK;
}

extern "C" int otc_aes_cbc_decrypt_impl(const void *in, void *out, size_t nbytes, const otc_aes_key *k,
                                        const uint8_t iv[16], int impl, void *stream)
{
    Range rg("otc_aes_cbc_decrypt");
    int r = check_key(k, OTC_DIR_DECRYPT);
    if (r) return r;
    if (nbytes % 16) return set_err(OTC_ERR_ARG, "CBC length must be a multiple of 16");
    if (!iv) return set_err(OTC_ERR_ARG, "null iv");
    if ((r = check_bufs(in, out, nbytes, nbytes <= 16, "aes_cbc_decrypt"))) return r;
    if ((r = check_impl(impl))) return r;
    if (nbytes == 0) return OTC_OK;
    hipStream_t st = (hipStream_t)stream;
    hipError_t e;
    g_last_impl = pick_dec_impl(impl, k->bits, nbytes);
    if (const int form = split_form(g_last_impl, nbytes); form >= 0) {
        e = cbc_dec_split(in, out, nbytes / 16, *k, iv, form, st, &g_last_impl);
    } else {
        e = otc_impl::tt_cbc_decrypt(in, out, nbytes / 16, *k, ctr_from_bytes(iv), st);
    }
    if (e != hipSuccess) return hip_fail(e, "cbc_decrypt launch");
    return OTC_OK;
}

extern "C" int otc_aes_cbc_decrypt(const void *in, void *out, size_t nbytes, const otc_aes_key *k,
                                   const uint8_t iv[16], void *stream)
{
    return otc_aes_cbc_decrypt_impl(in, out, nbytes, k, iv, OTC_IMPL_AUTO, stream);
}

extern "C" int otc_aes_cbc_encrypt_segments_impl(const void *in, void *out, size_t seg_bytes, size_t nseg,
                                                 const otc_aes_key *k, const uint8_t iv0[16], int impl, void *stream)
{
    Range rg("otc_aes_cbc_encrypt_segments");
    int r = check_key(k, OTC_DIR_ENCRYPT);
    if (r) return r;
    if (seg_bytes % 16) return set_err(OTC_ERR_ARG, "segment length must be a multiple of 16");
    if (!iv0) return set_err(OTC_ERR_ARG, "null iv");
    if (nseg && seg_bytes > SIZE_MAX / nseg) return set_err(OTC_ERR_ARG, "size overflow");
    if ((r = check_bufs(in, out, seg_bytes * nseg, true, "aes_cbc_encrypt_segments"))) return r;
    if ((r = check_impl(impl))) return r;
    if (nseg == 0 || seg_bytes == 0) return OTC_OK;
    hipStream_t st = (hipStream_t)stream;
    hipError_t e;
    e = seg_enc_run(false, in, out, seg_bytes, nseg, *k, ctr_from_bytes(iv0), st);
    if (e != hipSuccess) return hip_fail(e, "cbc_encrypt_segments launch");
    return OTC_OK;
}

extern "C" int otc_aes_cbc_encrypt_segments(const void *in, void *out, size_t seg_bytes, size_t nseg,
                                            const otc_aes_key *k, const uint8_t iv0[16], void *stream)
{
    return otc_aes_cbc_encrypt_segments_impl(in, out, seg_bytes, nseg, k, iv0, OTC_IMPL_AUTO, stream);
}

extern "C" int otc_aes_cbc_decrypt_segments_impl(const void *in, void *out, size_t seg_bytes, size_t nseg,
                                                 const otc_aes_key *k, const uint8_t iv0[16], int impl, void *stream)
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
    if ((r = check_impl(impl))) return r;
    if (nseg == 0) return OTC_OK;
    hipError_t e;
    g_last_impl = pick_seg_impl(impl, k->bits, seg_bytes * nseg, sb);
    if (const int form = seg_shift_of(sb) < 0 ? -1 : split_form(g_last_impl, seg_bytes * nseg); form >= 0)
        e = seg_dec_split(false, in, out, sb, nseg, *k, ctr_from_bytes(iv0), form, (hipStream_t)stream, &g_last_impl);
    else
        e = otc_impl::tt_cbc_decrypt_seg(in, out, sb, nseg, *k, ctr_from_bytes(iv0), (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "cbc_decrypt_segments launch");
    return OTC_OK;
}

extern "C" int otc_aes_cbc_decrypt_segments(const void *in, void *out, size_t seg_bytes, size_t nseg,
                                            const otc_aes_key *k, const uint8_t iv0[16], void *stream)
{
    return otc_aes_cbc_decrypt_segments_impl(in, out, seg_bytes, nseg, k, iv0, OTC_IMPL_AUTO, stream);
}

/* CFB128 over independent segments (IV_s = iv0 + s, like the CBC sector
 * mode): encryption is one serial chain per segment (one lane each, the
 * sector kernel with the CFB chain step); decryption is fully parallel with
 * IV_s at every segment start.  Both use the ENCRYPTION key schedule. */
static int cfb_seg_common(const void *in, void *out, size_t seg_bytes, size_t nseg, const otc_aes_key *k,
                          const uint8_t iv0[16], void *stream, bool decrypt, const char *what,
                          int impl = OTC_IMPL_AUTO)
{
    int r = check_key(k, OTC_DIR_ENCRYPT);
    if (r) return r;
    if (seg_bytes % 16) return set_err(OTC_ERR_ARG, "segment length must be a multiple of 16");
    if (!iv0) return set_err(OTC_ERR_ARG, "null iv");
    if (nseg && seg_bytes > SIZE_MAX / nseg) return set_err(OTC_ERR_ARG, "size overflow");
    /* decrypt reads block i-1 of the input while another lane writes block
     * i-1 of the output: in place only for encryption (lane-private chains) */
    if ((r = check_bufs(in, out, seg_bytes * nseg, !decrypt, what))) return r;
    if ((r = check_impl(impl))) return r;
    if (nseg == 0 || seg_bytes == 0) return OTC_OK;
    hipError_t e;
    if (decrypt) {
        g_last_impl = pick_seg_impl(impl, k->bits, seg_bytes * nseg, seg_bytes / 16);
        if (const int form = seg_shift_of(seg_bytes / 16) < 0 ? -1 : split_form(g_last_impl, seg_bytes * nseg); form >= 0)
            e = seg_dec_split(true, in, out, seg_bytes / 16, nseg, *k, ctr_from_bytes(iv0), form, (hipStream_t)stream,
                              &g_last_impl);
        else
            e = otc_impl::tt_cfb_decrypt_seg(in, out, seg_bytes / 16, nseg, *k, ctr_from_bytes(iv0),
                                             (hipStream_t)stream);
    } else {
        e = seg_enc_run(true, in, out, seg_bytes, nseg, *k, ctr_from_bytes(iv0), (hipStream_t)stream);
    }
    if (e != hipSuccess) return hip_fail(e, what);
    return OTC_OK;
}

extern "C" int otc_aes_cfb128_encrypt_segments(const void *in, void *out, size_t seg_bytes, size_t nseg,
                                               const otc_aes_key *k, const uint8_t iv0[16], void *stream)
{
    return otc_aes_cfb128_encrypt_segments_impl(in, out, seg_bytes, nseg, k, iv0, OTC_IMPL_AUTO, stream);
}

extern "C" int otc_aes_cfb128_encrypt_segments_impl(const void *in, void *out, size_t seg_bytes, size_t nseg,
                                                    const otc_aes_key *k, const uint8_t iv0[16], int impl,
                                                    void *stream)
{
    Range rg("otc_aes_cfb128_encrypt_segments");
    return cfb_seg_common(in, out, seg_bytes, nseg, k, iv0, stream, false, "cfb128_encrypt_segments", impl);
}

extern "C" int otc_aes_cfb128_decrypt_segments_impl(const void *in, void *out, size_t seg_bytes, size_t nseg,
                                                    const otc_aes_key *k, const uint8_t iv0[16], int impl,
                                                    void *stream)
{
    Range rg("otc_aes_cfb128_decrypt_segments");
    return cfb_seg_common(in, out, seg_bytes, nseg, k, iv0, stream, true, "cfb128_decrypt_segments", impl);
}

extern "C" int otc_aes_cfb128_decrypt_segments(const void *in, void *out, size_t seg_bytes, size_t nseg,
                                               const otc_aes_key *k, const uint8_t iv0[16], void *stream)
{
    return otc_aes_cfb128_decrypt_segments_impl(in, out, seg_bytes, nseg, k, iv0, OTC_IMPL_AUTO, stream);
}

extern "C" int otc_aes_cfb128_decrypt_impl(const void *in, void *out, size_t nbytes, const otc_aes_key *k,
                                           const uint8_t iv[16], int impl, void *stream)
{
    Range rg("otc_aes_cfb128_decrypt");
    int r = check_key(k, OTC_DIR_ENCRYPT);
    if (r) return r;
    if (nbytes % 16) return set_err(OTC_ERR_ARG, "CFB128 device path needs a multiple of 16 bytes");
    if (!iv) return set_err(OTC_ERR_ARG, "null iv");
    if ((r = check_bufs(in, out, nbytes, nbytes <= 16, "aes_cfb128_decrypt"))) return r;
    if ((r = check_impl(impl))) return r;
    if (nbytes == 0) return OTC_OK;
    uint32_t ivw[4];
    memcpy(ivw, iv, 16); /* LE words of the IV bytes, as both kernels load blocks */
    hipStream_t st = (hipStream_t)stream;
    hipError_t e;
    g_last_impl = pick_ecb_impl(impl, k->bits, nbytes);
    if (const int form = split_form(g_last_impl, nbytes); form >= 0)
        e = cfb_dec_split(in, out, nbytes / 16, *k, ivw, form, st, &g_last_impl);
    else
        e = otc_impl::tt_cfb_decrypt(in, out, nbytes / 16, *k, ivw, st);
    if (e != hipSuccess) return hip_fail(e, "cfb_decrypt launch");
    return OTC_OK;
}

extern "C" int otc_aes_cfb128_decrypt(const void *in, void *out, size_t nbytes, const otc_aes_key *k,
                                      const uint8_t iv[16], void *stream)
{
    return otc_aes_cfb128_decrypt_impl(in, out, nbytes, k, iv, OTC_IMPL_AUTO, stream);
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

extern "C" int otc_rc4_crypt_batch(void *states, size_t nstreams, size_t len, const void *in, void *out,
                                   void *stream)
{
    Range rg("otc_rc4_crypt_batch");
    if (nstreams == 0 || len == 0) return OTC_OK;
    if (!states || !in || !out) return set_err(OTC_ERR_ARG, "rc4_crypt_batch: null buffer");
    if ((uintptr_t)states & 3u) return set_err(OTC_ERR_ARG, "rc4_crypt_batch: states must be 4-byte aligned");
    if (len > SIZE_MAX / nstreams) return set_err(OTC_ERR_ARG, "size overflow");
    const uintptr_t a = (uintptr_t)in, b = (uintptr_t)out, n = nstreams * len;
    if (in != out && a < b + n && b < a + n)
        return set_err(OTC_ERR_ARG, "rc4_crypt_batch: input and output overlap partially");
    /* every state is written back in place: it must not alias the data */
    if (nstreams > SIZE_MAX / 264) return set_err(OTC_ERR_ARG, "size overflow");
    const uintptr_t s = (uintptr_t)states, sn = (uintptr_t)nstreams * 264u;
    if ((s < a + n && a < s + sn) || (s < b + n && b < s + sn))
        return set_err(OTC_ERR_ARG, "rc4_crypt_batch: states overlap the input or output");
    hipError_t e = otc_impl::k_rc4_states(states, nstreams, len, in, out, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "rc4_crypt_batch launch");
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

/* Streams for C harnesses (hipStreamCreate: ordered with the legacy default
 * stream, so hipEvents recorded on the default stream bracket work on them) */
extern "C" void *otc_stream_create(void)
{
    hipStream_t s = nullptr;
    hipError_t e = hipStreamCreate(&s);
    if (e != hipSuccess) {
        hip_fail(e, "hipStreamCreate");
        return nullptr;
    }
    return (void *)s;
}
/* a and b each wait for what the other has queued so far: a join point for
 * work split by hand over two streams (otbench's *-split modes) */
extern "C" int otc_stream_join(void *a, void *b)
{
    hipEvent_t ea = nullptr, eb = nullptr;
    hipError_t e = hipEventCreateWithFlags(&ea, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&eb, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventRecord(ea, (hipStream_t)a);
    if (e == hipSuccess) e = hipEventRecord(eb, (hipStream_t)b);
    if (e == hipSuccess) e = hipStreamWaitEvent((hipStream_t)a, eb, 0);
    if (e == hipSuccess) e = hipStreamWaitEvent((hipStream_t)b, ea, 0);
    if (ea) (void)hipEventDestroy(ea); /* released once the waits are satisfied */
    if (eb) (void)hipEventDestroy(eb);
    return e == hipSuccess ? OTC_OK : hip_fail(e, "stream join");
}

extern "C" void otc_stream_destroy(void *s)
{
    if (s) (void)hipStreamDestroy((hipStream_t)s);
}

/* ---- device memory helpers --------------------------------------------- */
extern "C" void *otc_dev_malloc(size_t nbytes)
{
    void *p = nullptr;
    hipError_t e = dev_alloc(&p, nbytes ? nbytes : 16);
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

extern "C" const char *otc_build_info(void)
{
    return "otc: MI355X (gfx950) cipher engine; kernels: aes_tt (LDS T-table), aes_bs (bitsliced VALU), "
           "rc4_multi, xor; runtime: pinned 3-stream pipeline, RCCL multi-GPU";
}

/* Which HIP runtime and RCCL this process actually runs on.  libotc.so links
 * libamdhip64.so.7 / librccl.so.1 by SONAME, and torch ships libraries with
 * the same SONAMEs: inside a torch process the library runs on torch's HIP
 * (7.0) and RCCL, in otbench and the CLIs on /opt/rocm's (7.2).  Every A/B
 * record carries this so the two are never compared unawares. */
extern "C" int otc_runtime_info(char *buf, size_t n)
{
    if (!buf || n == 0) return set_err(OTC_ERR_ARG, "null buffer");
    int rt = 0, drv = 0;
    if (hipRuntimeGetVersion(&rt) != hipSuccess) {
        (void)hipGetLastError();
        rt = -1;
    }
    if (hipDriverGetVersion(&drv) != hipSuccess) {
        (void)hipGetLastError();
        drv = -1;
    }
    int rccl = 0;
    if (ncclGetVersion(&rccl) != ncclSuccess) rccl = -1;
    std::string hip_path, rccl_path;
    if (FILE *f = fopen("/proc/self/maps", "r")) {
        char line[4096];
        while (fgets(line, sizeof line, f)) {
            char *p = strchr(line, '/');
            if (!p) continue;
            p[strcspn(p, "\n")] = 0;
            if (hip_path.empty() && strstr(p, "libamdhip64.so")) hip_path = p;
            if (rccl_path.empty() && strstr(p, "librccl.so")) rccl_path = p;
        }
        fclose(f);
    }
    const int w = snprintf(buf, n,
                           "{\"hip_runtime_version\": %d, \"hip_driver_version\": %d, \"rccl_version\": %d, "
                           "\"libamdhip64\": \"%s\", \"librccl\": \"%s\"}",
                           rt, drv, rccl, hip_path.c_str(), rccl_path.c_str());
    return w < 0 || (size_t)w >= n ? set_err(OTC_ERR_ARG, "buffer too small") : OTC_OK;
}
