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

size_t workspace_bytes(uint64_t total_bytes, uint64_t n_docs);
size_t debug_counters_offset(uint64_t total_bytes, uint64_t n_docs);

hipError_t launch_encode(const DevTables& T, const uint8_t* d_bytes, const uint64_t* d_doc_off, uint64_t n_docs,
                         uint64_t total_bytes, uint64_t* d_row_ptr, uint32_t* d_ids, uint64_t* d_offs, void* d_ws,
                         uint32_t* d_status, hipStream_t st, KernelTimers* tm);

}  // namespace tkz
