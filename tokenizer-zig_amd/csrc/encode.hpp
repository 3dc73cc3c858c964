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

// The segmented path of long BPE pretokens runs (and its workspace arrays exist) for BPE
// tokenizers with compact tables or wide ones with ids < 2^20 - 1 (T.mid: the mid cuckoo
// merge table and the merge rank -> new_id table), no new_id == first merge, whose pre_tokenizer leaves the whole text as one
// pretoken, unless switched off (tkz_set_long_segments). Returns the density of segment
// slots the workspace reserves: 1 = cuts only at dropped chars (a segment and its cut take
// >= 2 bytes), 2 = inert / whitespace cuts too (up to a segment per byte); 0 = off.
inline int seg_mode(const DevTables& T) {
    if (!(T.model == 1 && T.pretok == 0 && (T.compact || (T.mid && T.r2id && T.mtab_m)) && T.seg && !T.chain)) return 0;
    if ((T.inert_lo | T.inert_hi | T.cut_lo | T.cut_hi) != 0ull) return 2;
    return (T.drop_lo | T.drop_hi) != 0ull ? 1 : 0;
}
// workspace of one pass over the whole batch (seg: the segmented path's arrays, seg_mode)
size_t workspace_bytes(uint64_t total_bytes, uint64_t n_docs, int seg = 0);
// workspace for sub-batches of up to cap_b bytes; the largest cap a workspace supports
size_t workspace_bytes_sub(uint64_t cap_b, int seg = 0);
uint64_t sub_batch_cap(size_t ws_bytes, int seg = 0);
size_t debug_counters_offset(uint64_t total_bytes, uint64_t n_docs);
size_t stats_offset();  // batch statistics: u64 words at this workspace offset (HDR_* in encode.hip)
uint32_t seg_bound_errors();  // TKZ_SEG_BOUNDS builds: the segmented path's exceeded bounds (bits), then reset

// The segment memo's entries for n keys (d_keys readable up to limit): see encode.hip
hipError_t launch_seg_memo_build(const DevTables& T, const uint8_t* d_keys, const uint64_t* d_koff, uint32_t n,
                                 uint64_t limit, uint64_t* d_meta, uint32_t* d_toks, uint64_t* d_prof,
                                 hipStream_t st);
// The hot-pair bitmap (DevTables::hot_bits, k x k bits) of the hot keys' pool entries
// d_q[0..k) (1 + offset) and metas d_meta[0..k), with T.smpool set.
hipError_t launch_seg_hot_build(const DevTables& T, const uint32_t* d_q, const uint64_t* d_meta, uint32_t k,
                                uint32_t* d_bits, hipStream_t st);

// Encodes the batch in one pass when ws_bytes holds it, else in doc-aligned sub-batches
// of the largest size the workspace supports (one host sync per SPLIT_MAX sub-batches).
hipError_t launch_encode(const DevTables& T, const uint8_t* d_bytes, const uint64_t* d_doc_off, uint64_t n_docs,
                         uint64_t total_bytes, uint64_t* d_row_ptr, uint32_t* d_ids, uint64_t* d_offs, void* d_ws,
                         size_t ws_bytes, uint32_t* d_status, hipStream_t st, const TimerSource& timers,
                         EncodeFail* why);

}  // namespace tkz
