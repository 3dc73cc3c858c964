// Launch interface of the batched decode kernels (decode.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace tkz {

// Device view of Tokenizer.decode's tables (lib.zig:163-189, config.zig:459-530)
struct DecTables {
    const uint2* ent;      // per id: {pool offset, byte length | 0x80000000 if a special added token}
    uint32_t n_ent;        // ids >= n_ent decode to nothing
    const uint8_t* pool;   // model-vocab strings
    int decoder;           // 0 none, 1 WordPiece, 2 ByteLevel, 3 BPE
};

// cat_bound: an upper bound of the decoded bytes before the decoder (n_tok x longest string)
size_t decode_workspace_bytes(uint64_t n_docs, uint64_t n_tok, uint64_t cat_bound);

hipError_t launch_decode(const DecTables& D, const uint64_t* d_row_ptr, const uint32_t* d_ids, uint64_t n_docs,
                         uint64_t n_tok, int skip_special, uint64_t cat_bound, uint8_t* d_out, uint64_t* d_out_off,
                         void* d_ws, hipStream_t st);

}  // namespace tkz
