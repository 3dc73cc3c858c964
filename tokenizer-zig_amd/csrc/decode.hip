// MI355X (gfx950) batched decode: Tokenizer.decode (jrc2139/tokenizer-zig src/lib.zig:163-189)
// over a CSR batch of token-id sequences, with the config decoders (src/config.zig:488-530).
//
// Per batch (one HIP stream):
//   k_dec_len    — per token: byte length of its model-vocab string (0 when the id is not in
//                  the model vocab, or is a special added token and skip_special is set).
//   k_scan_*     — exclusive scan of the lengths -> token byte positions (encode.hip).
//   k_dec_gather — per token: copy its string from the vocab pool into the concatenation.
//   none / ByteLevel decoder: the concatenation is the output; row offsets = scan at row starts.
//   WordPiece / BPE decoder, which drop or rewrite bytes across token boundaries inside one
//   sequence:
//   k_dec_bounds — bitmap of sequence starts in the concatenation.
//   k_chunk_docs — first sequence boundary of every 4-KiB chunk (encode.hip).
//   k_dec_count  — kept bytes per chunk; k_scan_* -> chunk bases.
//   k_dec_emit   — per chunk: keep flags, wave prefix, write kept bytes, output row offsets.
// Byte work only: no MFMA; the bound is HBM (lengths, strings, output).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "decode.hpp"

namespace tkz {

constexpr int DWAVE = 64;
constexpr int DSTEP = 512;
constexpr uint32_t DCH_LOG2 = 12;  // 4-KiB chunks of the concatenation
constexpr uint32_t SPECIAL_BIT = 0x80000000u;

__device__ __forceinline__ int dlane() { return (int)(threadIdx.x & 63); }

__device__ __forceinline__ int dwave_incl_scan(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);
    return v;
}

// string of id: lib.zig:176-178 (model idToToken), skip test lib.zig:168-174
__device__ __forceinline__ uint32_t dec_len(const DecTables& D, uint32_t id, int skip_special) {
    if (id >= D.n_ent) return 0;
    const uint32_t l = D.ent[id].y;
    if (skip_special && (l & SPECIAL_BIT)) return 0;
    return l & ~SPECIAL_BIT;
}

__global__ __launch_bounds__(256) void k_dec_len(DecTables D, const uint32_t* __restrict__ ids, uint64_t n_tok,
                                                 int skip_special, uint32_t* __restrict__ lens) {
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n_tok; t += (uint64_t)gridDim.x * blockDim.x)
        lens[t] = dec_len(D, ids[t], skip_special);
}

__global__ __launch_bounds__(256) void k_dec_gather(DecTables D, const uint32_t* __restrict__ ids, uint64_t n_tok,
                                                    int skip_special, const uint64_t* __restrict__ tpos,
                                                    uint8_t* __restrict__ cat) {
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n_tok; t += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t id = ids[t];
        const uint32_t l = dec_len(D, id, skip_special);
        if (l == 0) continue;
        const uint8_t* src = D.pool + D.ent[id].x;
        uint8_t* dst = cat + tpos[t];
        for (uint32_t j = 0; j < l; ++j) dst[j] = src[j];
    }
}

// row offsets of the concatenation (= output offsets without a rewriting decoder)
__global__ __launch_bounds__(256) void k_dec_rowoff(const uint64_t* __restrict__ row_ptr, uint64_t n_docs,
                                                    const uint64_t* __restrict__ tpos, uint64_t* __restrict__ cat_off) {
    const uint64_t d = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (d <= n_docs) cat_off[d] = tpos[row_ptr[d]];
}

__global__ __launch_bounds__(256) void k_dec_bounds(const uint64_t* __restrict__ cat_off, uint64_t n_docs,
                                                    uint32_t* __restrict__ bmap) {
    const uint64_t d = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (d > n_docs) return;
    const uint64_t v = cat_off[d];
    atomicOr(&bmap[v >> 5], 1u << (v & 31));
}

struct DecView {
    const uint8_t* cat;
    const uint32_t* bmap;  // bit v: a sequence starts at byte v
    uint64_t total;        // set in-kernel from *total_ptr (the scan's last entry)
    int decoder;
    __device__ __forceinline__ bool starts(uint64_t v) const { return (bmap[v >> 5] >> (v & 31)) & 1u; }
    // keep flag and output value of byte i (config.zig:488-530), one sequence at a time
    __device__ __forceinline__ bool keep(uint64_t i, uint8_t& out) const {
        const uint8_t b = cat[i];
        out = b;
        if (decoder == 1) {  // WordPiece: every "##" (scanning left to right) is dropped
            if (b != '#') return true;
            // a run of k '#' inside one sequence keeps only its last byte, and only if k is odd
            if (i + 1 < total && cat[i + 1] == '#' && !starts(i + 1)) return false;
            uint64_t k = 1;
            for (uint64_t j = i; j > 0 && !starts(j) && cat[j - 1] == '#'; --j) ++k;
            return (k & 1) != 0;
        }
        // BPE: "\xC4\xA0" -> ' '
        if (b == 0xA0 && i > 0 && !starts(i) && cat[i - 1] == 0xC4) return false;
        if (b == 0xC4 && i + 1 < total && !starts(i + 1) && cat[i + 1] == 0xA0) out = ' ';
        return true;
    }
};

__global__ __launch_bounds__(256) void k_dec_count(DecView V, const uint64_t* __restrict__ total_ptr, uint64_t n_chunks,
                                                   uint32_t* __restrict__ counts) {
    V.total = *total_ptr;
    const int lane = dlane();
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t c = wave; c < n_chunks; c += nw) {
        const uint64_t cs = c << DCH_LOG2, ce = min(cs + (1ull << DCH_LOG2), V.total);
        uint32_t n = 0;  // (chunks past the end count 0)
        for (uint64_t i = cs + lane; i < ce; i += DWAVE) {
            uint8_t o;
            n += V.keep(i, o) ? 1u : 0u;
        }
#pragma unroll
        for (int s = 32; s > 0; s >>= 1) n += (uint32_t)__shfl_xor((int)n, s, DWAVE);
        if (lane == 0) counts[c] = n;
    }
}

// per chunk: kept bytes to out[chunk_base ...], out_off of the sequences starting here
__global__ __launch_bounds__(256) void k_dec_emit(DecView V, const uint64_t* __restrict__ total_ptr, uint64_t n_chunks,
                                                  const uint64_t* __restrict__ chunk_base,
                                                  const uint64_t* __restrict__ chunk_doc,
                                                  const uint64_t* __restrict__ cat_off, uint64_t n_docs,
                                                  uint8_t* __restrict__ out, uint64_t* __restrict__ out_off) {
    __shared__ uint32_t pre_all[4][DSTEP];
    V.total = *total_ptr;
    uint32_t* pre = pre_all[threadIdx.x >> 6];
    const int lane = dlane();
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    if (wave == 0) {  // sequences starting at the very end (and trailing empty ones)
        const uint64_t tot = chunk_base[n_chunks];
        for (uint64_t k0 = 0; k0 <= n_docs; k0 += DWAVE) {
            const uint64_t k = n_docs - k0 - (uint64_t)lane;
            const bool at_end = k0 + (uint64_t)lane <= n_docs && cat_off[k] == V.total;
            if (at_end) out_off[k] = tot;
            if (__ballot(at_end) != ~0ull) break;
        }
    }
    for (uint64_t c = wave; c < n_chunks; c += nw) {
        const uint64_t cs = c << DCH_LOG2, ce = min(cs + (1ull << DCH_LOG2), V.total);
        if (cs >= ce) continue;
        uint64_t o = chunk_base[c];
        uint64_t dk = chunk_doc[c];
        for (uint64_t sb = cs; sb < ce; sb += DSTEP) {
            // 8 consecutive bytes per lane
            uint8_t val[8];
            uint32_t km = 0;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const uint64_t i = sb + 8ull * lane + j;
                bool k = false;
                val[j] = 0;
                if (i < ce) k = V.keep(i, val[j]);
                km |= (uint32_t)k << j;
            }
            const uint32_t cnt = (uint32_t)__popc(km);
            const uint32_t inc = (uint32_t)dwave_incl_scan((int)cnt);
            const uint32_t tot = (uint32_t)__shfl((int)inc, DWAVE - 1, DWAVE);
            uint32_t p = inc - cnt;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                pre[8 * lane + j] = p;
                if ((km >> j) & 1u) out[o + p++] = val[j];
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            while (true) {  // sequence starts in this step
                const uint64_t k = dk + (uint64_t)lane;
                const uint64_t kc = k <= n_docs ? k : n_docs;
                const uint64_t v = cat_off[kc];
                const bool in = k <= n_docs && v < min(sb + DSTEP, V.total);
                if (in) out_off[k] = o + pre[v - sb];
                const int n_in = __popcll(__ballot(in));
                dk += (uint64_t)n_in;
                if (n_in < DWAVE) break;
            }
            __builtin_amdgcn_wave_barrier();
            o += tot;
        }
    }
}

// from encode.hip
__global__ void k_scan_partials(const uint32_t* counts, uint64_t n, uint64_t* partials);
__global__ void k_scan_top(uint64_t* partials, uint64_t nb, unsigned long long* hdr, int dedup);
__global__ void k_scan_final(const uint32_t* counts, uint64_t n, const uint64_t* partials, uint64_t* row_ptr,
                             const unsigned long long* base_in, unsigned long long* base_out);
__global__ void k_chunk_docs(const uint64_t* doc_off, uint64_t n_docs, uint32_t ch_log2, uint64_t* chunk_doc,
                             unsigned long long* chunk_ctr, int zero_stats);
uint64_t scan_chunk_elems();

static inline uint64_t dalign(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }

struct DecLayout {
    uint32_t* lens; uint64_t* tpos; uint64_t* partials; uint64_t* cat_off; uint8_t* cat; uint32_t* bmap;
    uint32_t* ccnt; uint64_t* cbase; uint64_t* cdoc; unsigned long long* ctr;
};

static DecLayout dec_layout(void* ws, uint64_t n_docs, uint64_t n_tok, uint64_t cat_bound) {
    DecLayout L;
    const uint64_t nc = (cat_bound >> DCH_LOG2) + 2;
    const uint64_t np = (std::max<uint64_t>(n_tok, nc) + scan_chunk_elems() - 1) / scan_chunk_elems() + 2;
    uint8_t* p = (uint8_t*)ws;
    L.lens = (uint32_t*)p; p += dalign((n_tok + 1) * 4, 256);
    L.tpos = (uint64_t*)p; p += dalign((n_tok + 1) * 8, 256);
    L.partials = (uint64_t*)p; p += dalign(np * 8, 256);
    L.cat_off = (uint64_t*)p; p += dalign((n_docs + 1) * 8, 256);
    L.bmap = (uint32_t*)p; p += dalign((cat_bound / 32 + 2) * 4, 256);
    L.ccnt = (uint32_t*)p; p += dalign(nc * 4, 256);
    L.cbase = (uint64_t*)p; p += dalign((nc + 1) * 8, 256);
    L.cdoc = (uint64_t*)p; p += dalign((nc + 1) * 8, 256);
    L.ctr = (unsigned long long*)p; p += 256;
    L.cat = p;
    return L;
}

size_t decode_workspace_bytes(uint64_t n_docs, uint64_t n_tok, uint64_t cat_bound) {
    const DecLayout L = dec_layout(nullptr, n_docs, n_tok, cat_bound);
    return (size_t)((L.cat - (uint8_t*)nullptr) + dalign(cat_bound + 16, 256));
}

hipError_t launch_decode(const DecTables& D, const uint64_t* d_row_ptr, const uint32_t* d_ids, uint64_t n_docs,
                         uint64_t n_tok, int skip_special, uint64_t cat_bound, uint8_t* d_out, uint64_t* d_out_off,
                         void* d_ws, hipStream_t st) {
    if (n_docs == 0) return hipSuccess;
    const DecLayout L = dec_layout(d_ws, n_docs, n_tok, cat_bound);
    const bool rewrite = D.decoder == 1 || D.decoder == 3;
    uint8_t* cat = rewrite ? L.cat : d_out;
    const unsigned tb = (unsigned)std::min<uint64_t>((n_tok + 255) / 256 + 1, 16384);
    hipLaunchKernelGGL(k_dec_len, dim3(tb), dim3(256), 0, st, D, d_ids, n_tok, skip_special, L.lens);
    const uint64_t SC = scan_chunk_elems();
    const unsigned nb = (unsigned)((n_tok + SC - 1) / SC) + (n_tok == 0 ? 1 : 0);
    hipLaunchKernelGGL(k_scan_partials, dim3(nb), dim3(256), 0, st, (const uint32_t*)L.lens, n_tok, L.partials);
    hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(256), 0, st, L.partials, (uint64_t)nb, (unsigned long long*)nullptr, 0);
    hipLaunchKernelGGL(k_scan_final, dim3(nb), dim3(256), 0, st, (const uint32_t*)L.lens, n_tok,
                       (const uint64_t*)L.partials, L.tpos, nullptr, nullptr);
    if (n_tok == 0) hipMemsetAsync(L.tpos, 0, 8, st);
    hipLaunchKernelGGL(k_dec_gather, dim3(tb), dim3(256), 0, st, D, d_ids, n_tok, skip_special,
                       (const uint64_t*)L.tpos, cat);
    const unsigned db = (unsigned)((n_docs + 1 + 255) / 256);
    uint64_t* cat_off = rewrite ? L.cat_off : d_out_off;
    hipLaunchKernelGGL(k_dec_rowoff, dim3(db), dim3(256), 0, st, d_row_ptr, n_docs, (const uint64_t*)L.tpos, cat_off);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || !rewrite) return e;
    // rewriting decoders: chunked keep/compact over the concatenation (total = tpos[n_tok])
    // chunks cover [0, cat_bound]; the true length is read on the device (no host sync)
    const uint64_t n_chunks = (cat_bound >> DCH_LOG2) + 1;
    if ((e = hipMemsetAsync(L.bmap, 0, (size_t)dalign((cat_bound / 32 + 2) * 4, 256), st)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_dec_bounds, dim3(db), dim3(256), 0, st, (const uint64_t*)cat_off, n_docs, L.bmap);
    hipLaunchKernelGGL(k_chunk_docs, dim3(db), dim3(256), 0, st, (const uint64_t*)cat_off, n_docs, DCH_LOG2, L.cdoc,
                       L.ctr, 0);
    DecView V{cat, L.bmap, 0, D.decoder};
    const uint64_t* total_ptr = L.tpos + n_tok;
    const unsigned cg = (unsigned)std::min<uint64_t>((n_chunks + 3) / 4, 8192);
    hipLaunchKernelGGL(k_dec_count, dim3(cg), dim3(256), 0, st, V, total_ptr, n_chunks, L.ccnt);
    const unsigned nbc = (unsigned)((n_chunks + SC - 1) / SC);
    hipLaunchKernelGGL(k_scan_partials, dim3(nbc), dim3(256), 0, st, (const uint32_t*)L.ccnt, n_chunks, L.partials);
    hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(256), 0, st, L.partials, (uint64_t)nbc, (unsigned long long*)nullptr, 0);
    hipLaunchKernelGGL(k_scan_final, dim3(nbc), dim3(256), 0, st, (const uint32_t*)L.ccnt, n_chunks,
                       (const uint64_t*)L.partials, L.cbase, nullptr, nullptr);
    hipLaunchKernelGGL(k_dec_emit, dim3(cg), dim3(256), 0, st, V, total_ptr, n_chunks, (const uint64_t*)L.cbase,
                       (const uint64_t*)L.cdoc, (const uint64_t*)cat_off, n_docs, d_out, d_out_off);
    return hipGetLastError();
}

}  // namespace tkz
