// MI355X (gfx950) kernels of the FastTokenizer API over a batch (jrc2139/tokenizer-zig
// src/lib.zig:248-454, SpanEncoding src/encoding.zig:16-224). The tokens come from the
// exact Tokenizer.encode kernels (encode.hip); these kernels apply FastTokenizer's two caps:
//   k_span_clip — pretoken cap (arena.zig:192,224-229): docs with more than max_pretokens
//                 pretokens have their tail blanked in a device copy of the input.
//   k_span_fill — token cap (SpanEncoding.tryAppend, encoding.zig:95-99): CSR -> dense
//                 [n_docs, max_tokens] rows + per-doc length.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "span.hpp"

namespace tkz {

// config.zig:440-450 (Whitespace: " \t\n\r"), config.zig:405-438 (Bert: std.ascii.isWhitespace)
__device__ __forceinline__ bool span_delim(int pretok, uint32_t b) {
    const bool ws = b == ' ' || b == '\t' || b == '\n' || b == '\r';
    return pretok == 2 ? (ws || b == 0x0B || b == 0x0C) : ws;
}

// isPunctuation (config.zig:452-457): the 32 ASCII punctuation bytes
__device__ __forceinline__ bool span_punct(uint32_t b) {
    return (b >= 0x21 && b <= 0x2F) || (b >= 0x3A && b <= 0x40) || (b >= 0x5B && b <= 0x60) ||
           (b >= 0x7B && b <= 0x7E);
}

// One wave per doc. A doc of at most max_pretokens bytes cannot have more pretokens and is
// skipped; longer docs are scanned 64 bytes per step, counting pretoken starts with a ballot.
__global__ __launch_bounds__(256) void k_span_clip(int pretok, uint32_t max_pretokens,
                                                   const uint64_t* __restrict__ doc_off, uint64_t n_docs,
                                                   uint8_t* __restrict__ copy) {
    const int lane = (int)(threadIdx.x & 63);
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t d = wave; d < n_docs; d += nw) {
        const uint64_t s = doc_off[d], len = doc_off[d + 1] - s;
        if (len <= max_pretokens) continue;
        uint64_t seen = 0, cut = len;
        for (uint64_t base = 0; base < len; base += 64) {
            const uint64_t i = base + (uint64_t)lane;
            bool start = false;
            if (i < len) {
                const uint32_t b = copy[s + i];
                const uint32_t p = i ? copy[s + i - 1] : (uint32_t)' ';
                start = !span_delim(pretok, b) &&
                        (span_delim(pretok, p) || (pretok == 2 && (span_punct(b) || span_punct(p))));
            }
            const uint64_t m = __ballot(start);
            const uint64_t c = (uint64_t)__popcll(m);
            if (seen + c > max_pretokens) {  // the (max_pretokens+1)-th start is in this step
                uint64_t mm = m;
                for (uint64_t k = seen; k < max_pretokens; ++k) mm &= mm - 1;  // drop the first ones
                cut = base + (uint64_t)__ffsll((long long)mm) - 1;
                break;
            }
            seen += c;
        }
        for (uint64_t i = cut + (uint64_t)lane; i < len; i += 64) copy[s + i] = (uint8_t)' ';
    }
}

__global__ __launch_bounds__(256) void k_span_fill(const uint64_t* __restrict__ row, uint64_t n_docs,
                                                   const uint32_t* __restrict__ ids, const uint64_t* __restrict__ offs,
                                                   uint32_t cap, uint32_t keep, uint32_t* __restrict__ len_out,
                                                   uint32_t* __restrict__ ids2, uint64_t* __restrict__ offs2,
                                                   uint32_t* __restrict__ attn) {
    const int lane = (int)(threadIdx.x & 63);
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t d = wave; d < n_docs; d += nw) {
        const uint64_t src = row[d], n = row[d + 1] - src;
        const uint32_t l = n < keep ? (uint32_t)n : keep;
        if (lane == 0) len_out[d] = l;
        const uint64_t o = d * (uint64_t)cap;
        for (uint32_t k = (uint32_t)lane; k < cap; k += 64) {
            const bool tok = k < l;
            ids2[o + k] = tok ? ids[src + k] : 0u;
            offs2[o + k] = tok ? offs[src + k] : 0ull;
            if (attn) attn[o + k] = tok ? 1u : 0u;
        }
    }
}

static unsigned span_blocks(uint64_t n_docs) {
    const uint64_t b = (n_docs + 3) / 4;  // 4 waves per block, one doc per wave
    return (unsigned)(b < 16384 ? (b ? b : 1) : 16384);
}

hipError_t launch_span_clip(int pretok, uint32_t max_pretokens, const uint64_t* d_doc_off, uint64_t n_docs,
                            uint8_t* d_copy, hipStream_t st) {
    if (n_docs == 0 || pretok == 0) return hipSuccess;
    hipLaunchKernelGGL(k_span_clip, dim3(span_blocks(n_docs)), dim3(256), 0, st, pretok, max_pretokens, d_doc_off,
                       n_docs, d_copy);
    return hipGetLastError();
}

hipError_t launch_span_fill(const uint64_t* d_row, uint64_t n_docs, const uint32_t* d_ids, const uint64_t* d_offs,
                            uint32_t cap, uint32_t keep, uint32_t* d_len, uint32_t* d_ids2, uint64_t* d_offs2, uint32_t* d_attn,
                            hipStream_t st) {
    if (n_docs == 0) return hipSuccess;
    hipLaunchKernelGGL(k_span_fill, dim3(span_blocks(n_docs)), dim3(256), 0, st, d_row, n_docs, d_ids, d_offs, cap,
                       keep, d_len, d_ids2, d_offs2, d_attn);
    return hipGetLastError();
}

}  // namespace tkz
