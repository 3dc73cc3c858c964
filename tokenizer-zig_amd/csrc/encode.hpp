// Launch interface of the encode kernels (encode.hip) used by the host library.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "tables.hpp"

#ifndef TKZ_MAXB
#define TKZ_MAXB 24  // words of <= TKZ_MAXB bytes keep their symbols in LDS
#endif

namespace tkz {

struct KernelTimers {
    bool enabled = false;
    // k_encode start, k_encode end, k_bpe_deferred end, count + scan end, k_compact end
    hipEvent_t ev[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
};

// Kernel timers for each pass of a call (a call runs one pass per sub-batch); next()
// returns null when profiling is off.
struct TimerSource {
    KernelTimers* (*fn)(void* ctx) = nullptr;
    void* ctx = nullptr;
    KernelTimers* next() const { return fn ? fn(ctx) : nullptr; }
};

enum class EncodeFail { None, WorkspaceTooSmall, DocTooLarge };

// workspace of one pass over the whole batch
size_t workspace_bytes(uint64_t total_bytes, uint64_t n_docs);
// workspace for sub-batches of up to cap_b bytes; the largest cap a workspace supports
size_t workspace_bytes_sub(uint64_t cap_b);
uint64_t sub_batch_cap(size_t ws_bytes);
size_t debug_counters_offset(uint64_t total_bytes, uint64_t n_docs);
size_t stats_offset();  // batch statistics: u64 words at this workspace offset (HDR_* in encode.hip)

// Encodes the batch in one pass when ws_bytes holds it, else in doc-aligned sub-batches
// of the largest size the workspace supports (one host sync per SPLIT_MAX sub-batches).
hipError_t launch_encode(const DevTables& T, const uint8_t* d_bytes, const uint64_t* d_doc_off, uint64_t n_docs,
                         uint64_t total_bytes, uint64_t* d_row_ptr, uint32_t* d_ids, uint64_t* d_offs, void* d_ws,
                         size_t ws_bytes, uint32_t* d_status, hipStream_t st, const TimerSource& timers,
                         EncodeFail* why);

}  // namespace tkz
