/*
 * engine_internal.h -- helpers shared by the host runtime translation units
 * (engine.cpp: device ops / keys / info; pipeline.cpp: host streaming engine
 * and multi-GPU jobs).  Not part of the public C API (otc.h).
 */
#ifndef OTC_ENGINE_INTERNAL_H
#define OTC_ENGINE_INTERNAL_H

#include <hip/hip_runtime.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <string>
#include <vector>

#include "otc.h"
#include "otc_device.h"

namespace otc_rt {

using otc_dev::Ctr128;

/* error message of the last failing call on this thread (otc_last_error) */
int set_err(int code, const std::string &msg);
std::string last_err();
int hip_fail(hipError_t e, const char *what);

Ctr128 ctr_from_bytes(const uint8_t c[16]);
Ctr128 ctr_add(Ctr128 c, uint64_t n, bool wrap64);
int check_key(const otc_aes_key *k, int dir);
/* destroy the pooled auxiliary streams of the ECB split (engine.cpp) */
void aux_release_all();

/* roctx range for rocprofv3 --marker-trace (a no-op unless a tool is
 * attached): every public entry point is one named range. */
struct Range {
    explicit Range(const char *name) { roctxRangePushA(name); }
    ~Range() { roctxRangePop(); }
    Range(const Range &) = delete;
    Range &operator=(const Range &) = delete;
};

/* A stream with a hardware queue of its own: HIP maps ordinary streams onto
 * GPU_MAX_HW_QUEUES (4) pooled queues per device per process, so in a process
 * that also holds torch's, RCCL's and a profiler's streams a library stream can
 * share a queue with an unrelated one and its work waits behind that stream's
 * (barrier packets are processed in queue order).  A stream created with a CU
 * mask -- here all CUs -- always gets a dedicated queue. */
inline hipError_t dedicated_stream_create(hipStream_t *s)
{
    std::vector<uint32_t> mask((size_t)(otc_dev::device_cus() + 31) / 32, 0xFFFFFFFFu);
    return hipExtStreamCreateWithCUMask(s, (uint32_t)mask.size(), mask.data());
}

/* hipMalloc behind the fault-injection hook */
inline hipError_t dev_alloc(void **p, size_t n)
{
    if (otc_dev::alloc_fault()) return hipErrorOutOfMemory;
    return hipMalloc(p, n);
}

} // namespace otc_rt

#define HIPCHK(expr)                                                  \
    do {                                                              \
        hipError_t _e = (expr);                                       \
        if (_e != hipSuccess) return otc_rt::hip_fail(_e, #expr);     \
    } while (0)

#define RCCLCHK(expr)                                                                               \
    do {                                                                                            \
        ncclResult_t _r = (expr);                                                                   \
        if (_r != ncclSuccess)                                                                      \
            return otc_rt::set_err(OTC_ERR_RCCL, std::string(#expr) + ": " + ncclGetErrorString(_r)); \
    } while (0)

#endif
