// MI355X (gfx950) truncation + padding of a batch of encodings (Tokenizer.encode steps 6-7,
// jrc2139/tokenizer-zig src/lib.zig:149-157; Encoding.truncate / Encoding.pad,
// src/encoding.zig:362-437): CSR (row_ptr, ids, offsets) -> CSR with every row truncated to
// max_length and padded to `length`, plus the type_ids / special_token_mask / attention_mask
// rows the reference's Encoding carries. With max_length == length every row has the same
// length and the output is a dense [n_docs, length] tensor (row_ptr[d] = d * length).
//   k_pad_len  — per doc: output length.   k_scan_*  — row offsets (encode.hip).
//   k_pad_fill — one wave per doc: copy / pad each position.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "pad.hpp"

namespace tkz {

__device__ __forceinline__ uint32_t pad_out_len(const PadParams& P, uint64_t l) {
    if (P.truncate && l > P.max_length) l = P.max_length;  // encoding.zig:362-380
    if (P.pad && l < P.length) l = P.length;               // encoding.zig:385-392
    return (uint32_t)l;
}

__global__ __launch_bounds__(256) void k_pad_len(PadParams P, const uint64_t* __restrict__ row_ptr, uint64_t n_docs,
                                                 uint32_t* __restrict__ lens) {
    const uint64_t d = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (d < n_docs) lens[d] = pad_out_len(P, row_ptr[d + 1] - row_ptr[d]);
}

__global__ __launch_bounds__(256) void k_pad_fill(PadParams P, const uint64_t* __restrict__ row_ptr, uint64_t n_docs,
                                                  const uint32_t* __restrict__ ids, const uint64_t* __restrict__ offs,
                                                  const uint64_t* __restrict__ row2, uint32_t* __restrict__ ids2,
                                                  uint64_t* __restrict__ offs2, uint32_t* __restrict__ type_ids,
                                                  uint32_t* __restrict__ special, uint32_t* __restrict__ attention) {
    const int lane = (int)(threadIdx.x & 63);
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t d = wave; d < n_docs; d += nw) {
        const uint64_t src = row_ptr[d], o = row2[d];
        uint64_t l1 = row_ptr[d + 1] - src;
        if (P.truncate && l1 > P.max_length) l1 = P.max_length;
        const uint64_t l2 = row2[d + 1] - o;
        const uint64_t npad = l2 - l1;
        for (uint64_t k = (uint64_t)lane; k < l2; k += 64) {
            // right: tokens then pads; left: pads then tokens (encoding.zig:408-434)
            const bool tok = P.left ? k >= npad : k < l1;
            const uint64_t sk = P.left ? k - npad : k;
            ids2[o + k] = tok ? ids[src + sk] : P.pad_id;
            offs2[o + k] = tok ? offs[src + sk] : 0ull;
            type_ids[o + k] = tok ? 0u : P.pad_type_id;
            special[o + k] = tok ? 0u : 1u;
            attention[o + k] = tok ? 1u : 0u;
        }
    }
}

// from encode.hip
__global__ void k_scan_partials(const uint32_t* counts, uint64_t n, uint64_t* partials);
__global__ void k_scan_top(uint64_t* partials, uint64_t nb, unsigned long long* hdr, int dedup);
__global__ void k_scan_final(const uint32_t* counts, uint64_t n, const uint64_t* partials, uint64_t* row_ptr,
                             const unsigned long long* base_in, unsigned long long* base_out);
uint64_t scan_chunk_elems();

size_t pad_workspace_bytes(uint64_t n_docs) {
    const uint64_t nb = (n_docs + scan_chunk_elems() - 1) / scan_chunk_elems() + 2;
    return (size_t)((n_docs * 4 + 255) / 256 * 256 + nb * 8 + 256);
}

hipError_t launch_pad(const PadParams& P, const uint64_t* d_row, uint64_t n_docs, const uint32_t* d_ids,
                      const uint64_t* d_offs, uint64_t* d_row2, uint32_t* d_ids2, uint64_t* d_offs2,
                      uint32_t* d_type, uint32_t* d_special, uint32_t* d_attn, void* d_ws, hipStream_t st) {
    if (n_docs == 0) return hipMemsetAsync(d_row2, 0, 8, st);
    uint32_t* lens = (uint32_t*)d_ws;
    uint64_t* partials = (uint64_t*)((uint8_t*)d_ws + (n_docs * 4 + 255) / 256 * 256);
    const unsigned b = (unsigned)((n_docs + 255) / 256);
    hipLaunchKernelGGL(k_pad_len, dim3(b), dim3(256), 0, st, P, d_row, n_docs, lens);
    const uint64_t SC = scan_chunk_elems();
    const unsigned nb = (unsigned)((n_docs + SC - 1) / SC);
    hipLaunchKernelGGL(k_scan_partials, dim3(nb), dim3(256), 0, st, (const uint32_t*)lens, n_docs, partials);
    hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(256), 0, st, partials, (uint64_t)nb, (unsigned long long*)nullptr, 0);
    hipLaunchKernelGGL(k_scan_final, dim3(nb), dim3(256), 0, st, (const uint32_t*)lens, n_docs,
                       (const uint64_t*)partials, d_row2, nullptr, nullptr);
    const unsigned fb = (unsigned)(((n_docs + 3) / 4) < 16384 ? (n_docs + 3) / 4 : 16384);
    hipLaunchKernelGGL(k_pad_fill, dim3(fb), dim3(256), 0, st, P, d_row, n_docs, d_ids, d_offs,
                       (const uint64_t*)d_row2, d_ids2, d_offs2, d_type, d_special, d_attn);
    return hipGetLastError();
}

}  // namespace tkz
