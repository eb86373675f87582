/*
 * pipeline.cpp -- host-streamed and multi-GPU jobs of the MI355X cipher engine
 * (C API in otc.h: otc_engine_*, otc_multi_*).
 *
 * The reference's only host path was one synchronous pageable cudaMemcpy in,
 * one launch, one cudaMemcpy out per call (/root/reference/aes-gpu/Source/
 * AES.cu:230-282); it had no multi-device code at all.  Here:
 *
 *  - otc_engine: per GPU a pinned staging ring on the GPU's NUMA node and
 *    three HIP streams, so H2D(k+1) | kernel(k) | D2H(k-1) overlap; copy and
 *    kernel time come from events on those streams (otc_stream_stats).
 *  - otc_multi_run strategy 0 (direct ingest): one host thread per GPU, bound
 *    to the GPU's socket, drives that GPU's engine over its shard.
 *  - otc_multi_run strategy 1 (RCCL root scatter/gather over xGMI): the root
 *    ingests the host stream, ncclScatter deals equal pieces, every GPU runs
 *    the cipher, ncclGather collects.  Scatters and gathers use two separate
 *    communicators (xGMI links are full duplex) and every per-GPU buffer is
 *    double-buffered, so scatter(r+1) | cipher(r) | gather(r-1) overlap.
 *
 * CBC-decrypt halos (the ciphertext block in front of each chunk/shard) are
 * copied out of the input BEFORE any output is written: with host_in ==
 * host_out an in-flight D2H would otherwise overwrite a halo with plaintext.
 */
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "engine_internal.h"
#include "otc.h"
#include "otc_numa.h"

using namespace otc_rt;

namespace {

/* NUMA node of a GPU's PCIe device (sysfs), -1 if unknown or OTC_NUMA=0 */
int gpu_numa_node(int dev)
{
    if (const char *e = getenv("OTC_NUMA"))
        if (!strcmp(e, "0")) return -1;
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, (int)sizeof bus, dev) != hipSuccess) {
        (void)hipGetLastError();
        return -1;
    }
    return otc_numa_node_of_pci(nullptr, bus);
}

/* pinned host window on `node`: NUMA-placed pages, then page-locked */
struct PinnedBuf {
    void *p = nullptr;
    size_t n = 0;
};

hipError_t pinned_alloc(PinnedBuf &b, size_t n, int node)
{
    b.p = otc_dev::alloc_fault() ? nullptr : otc_numa_alloc(n, node);
    if (!b.p) return hipErrorOutOfMemory;
    b.n = n;
    hipError_t e = hipHostRegister(b.p, n, hipHostRegisterDefault);
    if (e != hipSuccess) {
        otc_numa_free(b.p, n);
        b.p = nullptr;
        b.n = 0;
    }
    return e;
}

void pinned_free(PinnedBuf &b)
{
    if (!b.p) return;
    (void)hipHostUnregister(b.p);
    otc_numa_free(b.p, b.n);
    b.p = nullptr;
    b.n = 0;
}

bool is_pinned(const void *p)
{
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

float ev_ms(hipEvent_t a, hipEvent_t b)
{
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, a, b) != hipSuccess) {
        (void)hipGetLastError();
        return 0.f;
    }
    return ms;
}

double since_ms(std::chrono::steady_clock::time_point t0)
{
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

/* CBC-dec halos: for every piece start p (> 0) the 16 input bytes in front of
 * it, captured before any output is written (in-place safety) */
std::vector<uint8_t> capture_halos(const uint8_t *hin, const std::vector<size_t> &starts)
{
    std::vector<uint8_t> h(16 * starts.size(), 0);
    for (size_t i = 0; i < starts.size(); ++i)
        if (starts[i] >= 16) memcpy(&h[16 * i], hin + starts[i] - 16, 16);
    return h;
}

} // namespace

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

/* Launch the cipher on one device chunk.  `blk0` = block offset of the chunk
 * inside the whole stream (CTR); `halo` = for CBC-dec, the 16-byte ciphertext
 * block preceding the chunk (nullptr: the stream IV). */
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

extern "C" int otc_device_numa_node(int dev) { return gpu_numa_node(dev); }

/* ---- L3 streaming engine ------------------------------------------------ */
struct otc_engine {
    int device = 0;
    int numa_node = -1;
    size_t chunk = 0;
    int depth = 0;                   /* ring slots */
    int flags = 0;                   /* OTC_ENGINE_* */
    std::vector<void *> d_in, d_out; /* device ring */
    std::vector<PinnedBuf> h_in, h_out; /* pinned staging ring (pageable callers only) */
    hipStream_t s_h2d = nullptr, s_k = nullptr, s_d2h = nullptr;
    /* timing events per slot: copy start/end and kernel start/end */
    std::vector<hipEvent_t> ev_h2d0, ev_h2d, ev_k0, ev_k, ev_d2h0, ev_d2h;
};

extern "C" otc_engine *otc_engine_create(int device, size_t chunk_bytes, int depth)
{
    return otc_engine_create_ex(device, chunk_bytes, depth, OTC_ENGINE_DEFAULT);
}

extern "C" otc_engine *otc_engine_create_ex(int device, size_t chunk_bytes, int depth, int flags)
{
    if (chunk_bytes == 0) chunk_bytes = 256ull << 20;
    chunk_bytes = (chunk_bytes + 15) & ~(size_t)15;
    if (depth < 2) depth = 3;
    otc_engine *e = new otc_engine();
    e->device = device;
    e->chunk = chunk_bytes;
    e->depth = depth;
    e->flags = flags;
    if (hipSetDevice(device) != hipSuccess) {
        set_err(OTC_ERR_HIP, "hipSetDevice");
        delete e;
        return nullptr;
    }
    e->numa_node = gpu_numa_node(device);
    auto mk = [&](hipStream_t *s) {
        return (flags & OTC_ENGINE_POOLED_QUEUES) ? hipStreamCreateWithFlags(s, hipStreamNonBlocking)
                                                  : dedicated_stream_create(s);
    };
    bool ok = mk(&e->s_h2d) == hipSuccess && mk(&e->s_k) == hipSuccess && mk(&e->s_d2h) == hipSuccess;
    e->d_in.assign(depth, nullptr);
    e->d_out.assign(depth, nullptr);
    e->h_in.assign(depth, PinnedBuf{});
    e->h_out.assign(depth, PinnedBuf{});
    for (auto *v : {&e->ev_h2d0, &e->ev_h2d, &e->ev_k0, &e->ev_k, &e->ev_d2h0, &e->ev_d2h}) v->assign(depth, nullptr);
    for (int i = 0; ok && i < depth; ++i) {
        ok = dev_alloc(&e->d_in[i], chunk_bytes) == hipSuccess && dev_alloc(&e->d_out[i], chunk_bytes) == hipSuccess;
        for (auto *v : {&e->ev_h2d0, &e->ev_h2d, &e->ev_k0, &e->ev_k, &e->ev_d2h0, &e->ev_d2h})
            ok = ok && hipEventCreate(&(*v)[i]) == hipSuccess;
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
    for (hipStream_t s : {e->s_k, e->s_h2d, e->s_d2h})
        if (s) (void)hipStreamSynchronize(s);
    for (int i = 0; i < e->depth; ++i) {
        if (e->d_in[i]) (void)hipFree(e->d_in[i]);
        if (e->d_out[i]) (void)hipFree(e->d_out[i]);
        pinned_free(e->h_in[i]);
        pinned_free(e->h_out[i]);
        for (auto *v : {&e->ev_h2d0, &e->ev_h2d, &e->ev_k0, &e->ev_k, &e->ev_d2h0, &e->ev_d2h})
            if ((*v)[i]) (void)hipEventDestroy((*v)[i]);
    }
    for (hipStream_t s : {e->s_h2d, e->s_k, e->s_d2h})
        if (s) (void)hipStreamDestroy(s);
    delete e;
}

extern "C" int otc_engine_numa_node(const otc_engine *e) { return e ? e->numa_node : -1; }

extern "C" const void *otc_engine_staging(const otc_engine *e, int slot)
{
    if (!e || slot < 0 || slot >= e->depth) return nullptr;
    return e->h_in[slot].p;
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

extern "C" int otc_engine_run(otc_engine *e, int mode, const void *host_in, void *host_out, size_t nbytes,
                              const otc_aes_key *k, const uint8_t ivc[16], uint64_t block_offset, int impl,
                              otc_stream_stats *stats)
{
    Range rg("otc_engine_run");
    if (!e) return set_err(OTC_ERR_ARG, "null engine");
    if (int r = check_stream_args(mode, host_in, host_out, nbytes, k, ivc)) return r;
    if (mode == OTC_MODE_CBC_DEC && block_offset) return set_err(OTC_ERR_ARG, "CBC: pass the halo as iv instead");
    HIPCHK(hipSetDevice(e->device));
    /* Every error return below leaves earlier H2D / kernel / D2H work queued
     * on the engine's streams, and with a pinned host_out those D2H copies
     * would land in caller memory after the error is reported (a caller that
     * frees the buffer on error: use after free).  Drain the streams on any
     * early return; the success path has retired every chunk already. */
    struct DrainOnError {
        otc_engine *e;
        bool armed = true;
        ~DrainOnError()
        {
            if (!armed) return;
            for (hipStream_t s : {e->s_h2d, e->s_k, e->s_d2h})
                if (s) (void)hipStreamSynchronize(s);
            (void)hipGetLastError();
        }
    } drain{e};
    auto t0 = std::chrono::steady_clock::now();
    const bool pin_in = is_pinned(host_in), pin_out = is_pinned(host_out);
    for (int i = 0; i < e->depth; ++i) {
        if (!pin_in && !e->h_in[i].p) HIPCHK(pinned_alloc(e->h_in[i], e->chunk, e->numa_node));
        if (!pin_out && !e->h_out[i].p) HIPCHK(pinned_alloc(e->h_out[i], e->chunk, e->numa_node));
    }
    const size_t C = e->chunk;
    const size_t nchunks = (nbytes + C - 1) / C;
    const uint8_t *hin = (const uint8_t *)host_in;
    uint8_t *hout = (uint8_t *)host_out;
    std::vector<uint8_t> halos;
    if (mode == OTC_MODE_CBC_DEC) {
        std::vector<size_t> starts(nchunks);
        for (size_t c = 0; c < nchunks; ++c) starts[c] = c * C;
        halos = capture_halos(hin, starts);
    }
    double kms = 0.0, h2d_ms = 0.0, d2h_ms = 0.0, stage_ms = 0.0;
    std::vector<int> slot_used(e->depth, 0);

    auto retire = [&](int s, size_t c) -> int { /* chunk c used slot s: wait for its D2H */
        HIPCHK(hipEventSynchronize(e->ev_d2h[s]));
        kms += ev_ms(e->ev_k0[s], e->ev_k[s]);
        h2d_ms += ev_ms(e->ev_h2d0[s], e->ev_h2d[s]);
        d2h_ms += ev_ms(e->ev_d2h0[s], e->ev_d2h[s]);
        if (!pin_out) {
            auto ts = std::chrono::steady_clock::now();
            const size_t poff = c * C;
            memcpy(hout + poff, e->h_out[s].p, std::min(C, nbytes - poff));
            stage_ms += since_ms(ts);
        }
        return OTC_OK;
    };

    for (size_t c = 0; c < nchunks; ++c) {
        const int s = (int)(c % e->depth);
        const size_t off = c * C;
        const size_t n = std::min(C, nbytes - off);
        if (slot_used[s])
            if (int r = retire(s, c - e->depth)) return r;
        const void *src = hin + off;
        if (!pin_in) {
            auto ts = std::chrono::steady_clock::now();
            memcpy(e->h_in[s].p, hin + off, n);
            stage_ms += since_ms(ts);
            src = e->h_in[s].p;
        }
        HIPCHK(hipEventRecord(e->ev_h2d0[s], e->s_h2d));
        HIPCHK(hipMemcpyAsync(e->d_in[s], src, n, hipMemcpyHostToDevice, e->s_h2d));
        HIPCHK(hipEventRecord(e->ev_h2d[s], e->s_h2d));
        HIPCHK(hipStreamWaitEvent(e->s_k, e->ev_h2d[s], 0));
        HIPCHK(hipEventRecord(e->ev_k0[s], e->s_k));
        const uint8_t *hp = (mode == OTC_MODE_CBC_DEC && off > 0) ? &halos[16 * c] : nullptr;
        if (int r = run_chunk(mode, e->d_in[s], e->d_out[s], n, k, ivc, block_offset + off / 16, hp, impl, e->s_k))
            return r;
        HIPCHK(hipEventRecord(e->ev_k[s], e->s_k));
        HIPCHK(hipStreamWaitEvent(e->s_d2h, e->ev_k[s], 0));
        void *dst = pin_out ? (void *)(hout + off) : e->h_out[s].p;
        HIPCHK(hipEventRecord(e->ev_d2h0[s], e->s_d2h));
        HIPCHK(hipMemcpyAsync(dst, e->d_out[s], n, hipMemcpyDeviceToHost, e->s_d2h));
        HIPCHK(hipEventRecord(e->ev_d2h[s], e->s_d2h));
        slot_used[s] = 1;
    }
    for (size_t c = (nchunks > (size_t)e->depth ? nchunks - e->depth : 0); c < nchunks; ++c)
        if (int r = retire((int)(c % e->depth), c)) return r;
    if (stats) {
        stats->total_ms = since_ms(t0);
        stats->kernel_ms = kms;
        stats->h2d_ms = h2d_ms;
        stats->d2h_ms = d2h_ms;
        stats->host_stage_ms = stage_ms;
        stats->bytes = nbytes;
        stats->chunks = (int)nchunks;
        stats->numa_node = e->numa_node;
    }
    drain.armed = false;
    return OTC_OK;
}

/* ---- L4 multi-GPU (single process) -------------------------------------- */
/* ---- RCCL root scatter / gather (otc_multi_run strategy 1) -----------------
 * Round r (buffer set b = r & 1):
 *   root:   H2D(r) -> root_in[b]                      stream sc[0]
 *   all g:  ncclScatter(root_in[b] -> piece_in[b][g])  comm set SC, stream sc[g]
 *   all g:  cipher(piece_in[b][g] -> piece_out[b][g]) stream k[g]
 *   all g:  ncclGather(piece_out[b][g] -> root_out[b]) comm set GA, stream ga[g]
 *   root:   D2H(r) <- root_out[b]                     stream ga[0]
 * Three streams per GPU, the root included: a process gets GPU_MAX_HW_QUEUES
 * (4 here) hardware queues per device, and the root's copies on streams of
 * their own (5 streams with the caller's) made two streams share a queue,
 * which can serialise the phases below without a trace.  The root's H2D
 * precedes its scatter and its D2H follows its gather in stream order anyway;
 * only H2D(r+1) no longer overlaps scatter(r) (xGMI is ~20x PCIe: a few
 * percent).  Buffer reuse two rounds later is ordered by events, so
 * scatter(r+1), cipher(r) and gather(r-1) run at the same time; scatter and
 * gather are on separate communicators because xGMI links are full duplex
 * and one communicator would serialise the two directions.  ncclScatter needs
 * equal counts, so the last round is zero padded.
 *
 * Failure detection: waits poll hipStreamQuery and ncclCommGetAsyncError with a
 * watchdog (OTC_RCCL_TIMEOUT_S, default 600 s); on an async error or timeout
 * every communicator is aborted (ncclCommAbort) instead of destroyed, so a
 * hung peer cannot hang the caller.  All resources are owned by RcclJob and
 * released on every exit path. */
struct RcclJob {
    int n = 0;
    size_t S = 0; /* per-GPU bytes per round */
    std::vector<ncclComm_t> comm_sc, comm_ga;
    std::vector<hipStream_t> sc, kst, ga;         /* per GPU */
    std::vector<void *> pin[2], pout[2];           /* per GPU, double-buffered */
    std::vector<hipEvent_t> ev_sc[2], ev_k[2], ev_ga[2]; /* per GPU */
    void *root_in[2] = {nullptr, nullptr}, *root_out[2] = {nullptr, nullptr};
    bool failed = false;

    ~RcclJob()
    {
        if (!failed)
            for (int g = 0; g < n; ++g) {
                (void)hipSetDevice(g);
                for (hipStream_t s : {sc[g], kst[g], ga[g]})
                    if (s) (void)hipStreamSynchronize(s);
            }
        (void)hipSetDevice(0);
        for (auto *cv : {&comm_sc, &comm_ga})
            for (ncclComm_t c : *cv)
                if (c) {
                    if (failed) ncclCommAbort(c);
                    else ncclCommDestroy(c);
                }
        for (int g = 0; g < n; ++g) {
            (void)hipSetDevice(g);
            for (int b = 0; b < 2; ++b) {
                if (pin[b][g]) (void)hipFree(pin[b][g]);
                if (pout[b][g]) (void)hipFree(pout[b][g]);
                for (hipEvent_t ev : {ev_sc[b][g], ev_k[b][g], ev_ga[b][g]})
                    if (ev) (void)hipEventDestroy(ev);
            }
            for (hipStream_t s : {sc[g], kst[g], ga[g]})
                if (s) (void)hipStreamDestroy(s);
        }
        (void)hipSetDevice(0);
        for (int i = 0; i < 2; ++i) {
            if (root_in[i]) (void)hipFree(root_in[i]);
            if (root_out[i]) (void)hipFree(root_out[i]);
        }
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
            for (auto *cv : {&comm_sc, &comm_ga})
                for (int g = 0; g < n; ++g) {
                    ncclResult_t ae = ncclSuccess;
                    if (ncclCommGetAsyncError((*cv)[g], &ae) == ncclSuccess && ae != ncclSuccess &&
                        ae != ncclInProgress) {
                        failed = true;
                        return set_err(OTC_ERR_RCCL, std::string("RCCL async error on GPU ") + std::to_string(g) +
                                                         ": " + ncclGetErrorString(ae));
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
    J.comm_sc.assign(ngpus, nullptr);
    J.comm_ga.assign(ngpus, nullptr);
    for (auto *v : {&J.sc, &J.kst, &J.ga}) v->assign(ngpus, nullptr);
    for (int b = 0; b < 2; ++b) {
        J.pin[b].assign(ngpus, nullptr);
        J.pout[b].assign(ngpus, nullptr);
        for (auto *v : {&J.ev_sc[b], &J.ev_k[b], &J.ev_ga[b]}) v->assign(ngpus, nullptr);
    }
    std::vector<int> devs(ngpus);
    for (int g = 0; g < ngpus; ++g) devs[g] = g;
    RCCLCHK(ncclCommInitAll(J.comm_sc.data(), ngpus, devs.data()));
    RCCLCHK(ncclCommInitAll(J.comm_ga.data(), ngpus, devs.data()));
    const size_t round = S * (size_t)ngpus;
    for (int g = 0; g < ngpus; ++g) {
        HIPCHK(hipSetDevice(g));
        /* queues of their own: beside a caller's torch / RCCL streams, pooled
         * queues would let scatter, cipher and gather wait behind each other */
        for (hipStream_t *s : {&J.sc[g], &J.kst[g], &J.ga[g]}) HIPCHK(dedicated_stream_create(s));
        for (int b = 0; b < 2; ++b) {
            HIPCHK(dev_alloc(&J.pin[b][g], S));
            HIPCHK(dev_alloc(&J.pout[b][g], S));
            for (hipEvent_t *ev : {&J.ev_sc[b][g], &J.ev_k[b][g], &J.ev_ga[b][g]})
                HIPCHK(hipEventCreateWithFlags(ev, hipEventDisableTiming));
        }
    }
    HIPCHK(hipSetDevice(0));
    for (int i = 0; i < 2; ++i) {
        HIPCHK(dev_alloc(&J.root_in[i], round));
        HIPCHK(dev_alloc(&J.root_out[i], round));
    }
    return OTC_OK;
}

static int rccl_job_run(RcclJob &J, int mode, const uint8_t *hin, uint8_t *hout, size_t nbytes,
                        const otc_aes_key *k, const uint8_t ivc[16], int impl, double timeout_s)
{
    const int ngpus = J.n;
    const size_t S = J.S, round = S * (size_t)ngpus;
    /* the round plan: csrc/cpu/rccl_plan.c (pure, tested on the CPU at N = 2..8) */
    const uint64_t nrounds = otc_rccl_nrounds(nbytes, ngpus, S);
    std::vector<uint8_t> halos;
    if (mode == OTC_MODE_CBC_DEC) {
        std::vector<size_t> starts(nrounds * (size_t)ngpus);
        for (size_t i = 0; i < starts.size(); ++i) starts[i] = otc_rccl_halo_start(nbytes, S, i);
        halos = capture_halos(hin, starts);
    }
    for (size_t r = 0; r < nrounds; ++r) {
        const int b = (int)(r & 1);
        otc_rccl_piece pc;
        if (int e = otc_rccl_plan_piece(nbytes, ngpus, S, r, 0, &pc)) return e;
        const size_t off = pc.round_off, n = pc.round_bytes;
        HIPCHK(hipSetDevice(0));
        /* on sc[0]: after round r-2's scatter (which read root_in[b]), before
         * this round's */
        if (pc.pad_bytes) HIPCHK(hipMemsetAsync(J.root_in[b], 0, round, J.sc[0]));
        HIPCHK(hipMemcpyAsync(J.root_in[b], hin + off, n, hipMemcpyHostToDevice, J.sc[0]));
        /* piece_in[b][g] is free once round r-2's cipher has read it */
        if (r >= 2)
            for (int g = 0; g < ngpus; ++g) {
                HIPCHK(hipSetDevice(g));
                HIPCHK(hipStreamWaitEvent(J.sc[g], J.ev_k[b][g], 0));
            }
        RCCLCHK(ncclGroupStart());
        for (int g = 0; g < ngpus; ++g)
            RCCLCHK(ncclScatter(J.root_in[b], J.pin[b][g], S, ncclUint8, 0, J.comm_sc[g], J.sc[g]));
        RCCLCHK(ncclGroupEnd());
        for (int g = 0; g < ngpus; ++g) {
            HIPCHK(hipSetDevice(g));
            HIPCHK(hipEventRecord(J.ev_sc[b][g], J.sc[g]));
            HIPCHK(hipStreamWaitEvent(J.kst[g], J.ev_sc[b][g], 0));
            /* piece_out[b][g] is free once round r-2's gather has read it */
            if (r >= 2) HIPCHK(hipStreamWaitEvent(J.kst[g], J.ev_ga[b][g], 0));
            if (int e = otc_rccl_plan_piece(nbytes, ngpus, S, r, g, &pc)) return e;
            if (pc.bytes) {
                const uint8_t *hp = (mode == OTC_MODE_CBC_DEC && pc.halo >= 0) ? &halos[16 * (size_t)pc.halo] : nullptr;
                if (int rr = run_chunk(mode, J.pin[b][g], J.pout[b][g], pc.bytes, k, ivc, pc.blk0, hp, impl,
                                       J.kst[g])) {
                    J.failed = true;
                    return rr;
                }
            }
            HIPCHK(hipEventRecord(J.ev_k[b][g], J.kst[g]));
            HIPCHK(hipStreamWaitEvent(J.ga[g], J.ev_k[b][g], 0));
        }
        /* root_out[b] is free once round r-2's D2H has drained it: that D2H
         * precedes this gather on ga[0] */
        HIPCHK(hipSetDevice(0));
        RCCLCHK(ncclGroupStart());
        for (int g = 0; g < ngpus; ++g)
            RCCLCHK(ncclGather(J.pout[b][g], J.root_out[b], S, ncclUint8, 0, J.comm_ga[g], J.ga[g]));
        RCCLCHK(ncclGroupEnd());
        for (int g = 0; g < ngpus; ++g) {
            HIPCHK(hipSetDevice(g));
            HIPCHK(hipEventRecord(J.ev_ga[b][g], J.ga[g]));
        }
        HIPCHK(hipSetDevice(0));
        HIPCHK(hipMemcpyAsync(hout + off, J.root_out[b], n, hipMemcpyDeviceToHost, J.ga[0]));
        /* the host only enqueues; it blocks in the copies when the host
         * buffers are pageable (pin them -- otc_host_register -- to overlap) */
    }
    for (int g = 0; g < ngpus; ++g) {
        HIPCHK(hipSetDevice(g));
        for (hipStream_t s : {J.sc[g], J.kst[g], J.ga[g]})
            if (int w = J.wait(s, timeout_s)) return w;
    }
    HIPCHK(hipSetDevice(0));
    return OTC_OK;
}

/* The communicators, streams and buffers of the last job are cached across
 * calls (2 x ncclCommInitAll + allocation cost more than streaming several
 * GiB); a different GPU count or round size rebuilds them, a failure aborts
 * them, otc_multi_release() frees them.  Never torn down by a static
 * destructor: at process exit the HIP runtime may already be gone. */
static std::mutex g_rccl_mu;
static RcclJob *g_rccl = nullptr;

/* strategy 0 (direct ingest): one cached pipeline engine per logical shard */
static std::mutex g_direct_mu;
static std::vector<otc_engine *> g_direct;

static int rccl_scatter_gather(int ngpus, int mode, const uint8_t *hin, uint8_t *hout, size_t nbytes,
                               const otc_aes_key *k, const uint8_t ivc[16], int impl, size_t chunk_bytes)
{
    const char *to = getenv("OTC_RCCL_TIMEOUT_S");
    const double timeout_s = to ? atof(to) : 600.0;
    /* every H2D / D2H of this job is enqueued from this one thread: with
     * pageable host memory each copy blocks it and the pipeline serialises */
    if (otc_ptr_kind(hin) == OTC_PTR_HOST || otc_ptr_kind(hout) == OTC_PTR_HOST) {
        static std::once_flag once;
        std::call_once(once, [] {
            fprintf(stderr, "otc_multi_run(strategy 1): pageable host buffers -- the root's copies block and the "
                            "pipeline serialises; pin them (otc_host_alloc_pinned / otc_host_register)\n");
        });
    }
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

extern "C" void otc_release_resources(void)
{
    otc_multi_release();
    otc_rt::aux_release_all();
}

/* Logical shards -> devices: shard g runs on device g, or g % ndev when
 * OTC_SHARE_GPUS=1 (rehearses the N-shard path on fewer GPUs). */
static int shard_device(int g, int ndev, bool share) { return share ? g % ndev : g; }

extern "C" int otc_multi_run(int ngpus, int strategy, int mode, const void *host_in, void *host_out, size_t nbytes,
                             const otc_aes_key *k, const uint8_t ivc[16], int impl, size_t chunk_bytes,
                             otc_multi_stats *stats)
{
    Range rg("otc_multi_run");
    if (int r = check_stream_args(mode, host_in, host_out, nbytes, k, ivc)) return r;
    const int ndev = otc_device_count();
    const char *sh = getenv("OTC_SHARE_GPUS");
    const bool share = strategy == 0 && sh && !strcmp(sh, "1");
    if (ngpus < 1 || ndev < 1 || (ngpus > ndev && !share) || ngpus > 64)
        return set_err(OTC_ERR_ARG, "ngpus out of range (" + std::to_string(ndev) + " device(s) visible)");
    const size_t nblk = (nbytes + 15) / 16;
    /* planner: contiguous block-aligned shards, remainder spread over the
     * first shards (nothing dropped, unlike reference test.c:50) */
    std::vector<size_t> boff(ngpus + 1, 0);
    for (int g = 0; g < ngpus; ++g) boff[g + 1] = boff[g] + nblk / ngpus + ((size_t)g < nblk % ngpus ? 1 : 0);
    auto t0 = std::chrono::steady_clock::now();
    int rc = OTC_OK;
    std::vector<int> nodes(ngpus, -1);

    if (strategy == 0) {
        /* one host thread per shard, bound to its GPU's NUMA node, each
         * driving that shard's cached pipeline engine (pinned ring on the same
         * node + 3 streams: created on first use, reused by later calls with
         * the same chunk size, freed by otc_multi_release).  Error messages
         * are thread_local: a worker's is carried back so otc_last_error() on
         * the calling thread reports it. */
        std::lock_guard<std::mutex> lk(g_direct_mu);
        const size_t C = chunk_bytes ? ((chunk_bytes + 15) & ~(size_t)15) : (256ull << 20);
        if (g_direct.size() < (size_t)ngpus) g_direct.resize(ngpus, nullptr);
        /* CBC halos before any thread writes output (in place: a neighbour's
         * D2H would overwrite them) */
        std::vector<size_t> starts(ngpus);
        for (int g = 0; g < ngpus; ++g) starts[g] = std::min(boff[g] * 16, nbytes);
        const std::vector<uint8_t> halos =
            mode == OTC_MODE_CBC_DEC ? capture_halos((const uint8_t *)host_in, starts) : std::vector<uint8_t>();
        std::vector<std::thread> th;
        std::vector<int> res(ngpus, 0);
        std::vector<std::string> msg(ngpus);
        for (int g = 0; g < ngpus; ++g) {
            th.emplace_back([&, g]() {
                const size_t b0 = std::min(boff[g] * 16, nbytes), b1 = std::min(boff[g + 1] * 16, nbytes);
                if (b1 <= b0) return;
                const int dev = shard_device(g, ndev, share);
                nodes[g] = gpu_numa_node(dev);
                (void)otc_numa_bind_thread(nodes[g]); /* staging memcpys on the GPU's socket */
                otc_engine *&e = g_direct[g];
                if (e && (e->chunk != C || e->device != dev)) {
                    otc_engine_destroy(e);
                    e = nullptr;
                }
                if (!e) e = otc_engine_create(dev, C, 3);
                if (!e) {
                    res[g] = OTC_ERR_NOMEM;
                    msg[g] = last_err();
                    return;
                }
                const uint8_t *ivp = ivc;
                uint64_t bo = 0;
                if (mode == OTC_MODE_CBC_DEC) {
                    if (b0 > 0) ivp = &halos[16 * g];
                } else if (mode == OTC_MODE_CTR) {
                    bo = b0 / 16;
                }
                res[g] = otc_engine_run(e, mode, (const uint8_t *)host_in + b0, (uint8_t *)host_out + b0, b1 - b0, k,
                                        ivp, bo, impl, nullptr);
                if (res[g]) {
                    msg[g] = last_err();
                    otc_engine_destroy(e); /* unknown state: rebuild next time */
                    e = nullptr;
                }
            });
        }
        for (auto &t : th) t.join();
        for (int g = 0; g < ngpus; ++g)
            if (res[g]) {
                rc = res[g];
                set_err(rc, "GPU " + std::to_string(shard_device(g, ndev, share)) + " (shard " + std::to_string(g) +
                                "): " + msg[g]);
            }
    } else {
        rc = rccl_scatter_gather(ngpus, mode, (const uint8_t *)host_in, (uint8_t *)host_out, nbytes, k, ivc, impl,
                                 chunk_bytes);
    }
    if (stats) {
        stats->total_ms = since_ms(t0);
        stats->gbps = stats->total_ms > 0 ? (double)nbytes / (stats->total_ms * 1e6) : 0.0;
        stats->ngpus = ngpus;
        stats->strategy = strategy;
        stats->numa_nodes_used = 0;
        unsigned long long seen = 0;
        for (int nd : nodes)
            if (nd >= 0 && nd < 64 && !(seen & (1ull << nd))) {
                seen |= 1ull << nd;
                ++stats->numa_nodes_used;
            }
    }
    return rc;
}

extern "C" int otc_multi_ctr_resident(int ngpus, void *const *dev_bufs, size_t shard_bytes, const otc_aes_key *k,
                                      const uint8_t ctr0[16], int impl, double *elapsed_ms)
{
    Range rg("otc_multi_ctr_resident");
    if (ngpus < 1 || ngpus > otc_device_count()) return set_err(OTC_ERR_ARG, "ngpus out of range");
    if (shard_bytes % 16) return set_err(OTC_ERR_ARG, "shard must be a multiple of 16");
    if (!dev_bufs || !ctr0) return set_err(OTC_ERR_ARG, "null argument");
    struct Streams {
        std::vector<hipStream_t> s;
        ~Streams()
        {
            for (size_t g = 0; g < s.size(); ++g)
                if (s[g]) {
                    (void)hipSetDevice((int)g);
                    (void)hipStreamDestroy(s[g]);
                }
        }
    } st;
    st.s.assign(ngpus, nullptr);
    for (int g = 0; g < ngpus; ++g) {
        HIPCHK(hipSetDevice(g));
        HIPCHK(hipStreamCreateWithFlags(&st.s[g], hipStreamNonBlocking));
        HIPCHK(hipDeviceSynchronize());
    }
    auto t0 = std::chrono::steady_clock::now();
    for (int g = 0; g < ngpus; ++g) {
        HIPCHK(hipSetDevice(g));
        int r = otc_aes_ctr(dev_bufs[g], dev_bufs[g], shard_bytes, k, ctr0, (uint64_t)g * (shard_bytes / 16), impl,
                            st.s[g]);
        if (r) return r;
    }
    for (int g = 0; g < ngpus; ++g) {
        HIPCHK(hipSetDevice(g));
        HIPCHK(hipStreamSynchronize(st.s[g]));
    }
    if (elapsed_ms) *elapsed_ms = since_ms(t0);
    return OTC_OK;
}
