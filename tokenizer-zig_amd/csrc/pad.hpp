// Launch interface of the truncation / padding kernels (pad.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace tkz {

// Tokenizer.truncation / Tokenizer.padding (src/lib.zig:41-42, src/types.zig:39-59)
struct PadParams {
    int truncate;          // TruncationParams set
    uint64_t max_length;
    int pad;               // PaddingParams set with a length
    uint64_t length;
    uint32_t pad_id, pad_type_id;
    int left;              // PaddingDirection.left
};

size_t pad_workspace_bytes(uint64_t n_docs);

hipError_t launch_pad(const PadParams& P, const uint64_t* d_row, uint64_t n_docs, const uint32_t* d_ids,
                      const uint64_t* d_offs, uint64_t* d_row2, uint32_t* d_ids2, uint64_t* d_offs2,
                      uint32_t* d_type, uint32_t* d_special, uint32_t* d_attn, void* d_ws, hipStream_t st);

}  // namespace tkz
