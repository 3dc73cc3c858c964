// Launch interface of the FastTokenizer span-batch kernels (span.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace tkz {

// FastTokenizer.encode's pretoken cap (lib.zig:361-373, arena.zig:192,224-229): only the first
// `max_pretokens` pretokens of a doc are tokenized. In a device copy of the input, every doc
// with more pretokens has the bytes from the start of its (max_pretokens+1)-th pretoken on
// replaced by ' ', which both pretokenizers treat as a delimiter. `pretok` as DevTables.
hipError_t launch_span_clip(int pretok, uint32_t max_pretokens, const uint64_t* d_doc_off, uint64_t n_docs,
                            uint8_t* d_copy, hipStream_t st);

// CSR (row_ptr, ids, offsets) -> dense [n_docs, cap] SpanEncoding rows: len[d] = min(row
// length, keep) with keep <= cap (SpanEncoding.tryAppend, encoding.zig:95-99), ids / offsets of
// the first len[d] tokens, zeros after; attention_mask (optional) 1 / 0.
hipError_t launch_span_fill(const uint64_t* d_row, uint64_t n_docs, const uint32_t* d_ids, const uint64_t* d_offs,
                            uint32_t cap, uint32_t keep, uint32_t* d_len, uint32_t* d_ids2, uint64_t* d_offs2, uint32_t* d_attn,
                            hipStream_t st);

}  // namespace tkz
