// MI355X (gfx950) encode kernels: normalizer + pretokenizer scan + BPE / WordPiece
// model + vocab lookup, bit-exact with the reference's Tokenizer.encode
// (jrc2139/tokenizer-zig src/lib.zig:109-160). Integer / indexing work only: no MFMA.
//
// Pipeline for one (sub-)batch, all on one HIP stream:
//   k_chunk_docs   — first document boundary of every chunk (2^k bytes, 512 B..8 KiB);
//                    resets the per-pass counters.
//   k_encode       — persistent grid, one wavefront per block, chunks from a ticket counter.
//                    * scan: 16 B/lane coalesced loads (1 KiB per wave step), ASCII
//                      lowercase (config.zig:364-379), delimiter/punct classes
//                      (config.zig:405-457), document boundaries as forced breaks, word
//                      start/end bit masks, one packed DPP prefix sum -> LDS word ring.
//                    * dispatch, 64 words at a time: BPE words of <= 16 bytes probe the
//                      word memo (the vocab keys' own results); hits are finished on the
//                      spot. Misses of <= 8 bytes go to length-bucket queues that run
//                      register BPE (bpe.zig:173-263) one lane per word when 64 wait;
//                      longer misses are deferred. WordPiece (wordpiece.zig:141-222) runs
//                      in-kernel.
//                    * output: one 32-bit record per word in its chunk's dense word slots
//                      (the token itself for a single narrow token), 2+ tokens in the
//                      chunk's dense token area; per-chunk token counts.
//   k_dedup / k_bpe_deferred / k_dedup_copy — deferred words (> 8 bytes, memo misses):
//                    deduplicated (vocabs with many multi-byte chars), 16-symbol register
//                    BPE one lane per word.
//   k_bpe_long     — pretokens of > 64 bytes, one wavefront per word (the whole-text
//                    pretoken of an unrecognised pre_tokenizer, config.zig:387-402).
//   k_scan_*       — exclusive scan of the chunk token counts -> chunk bases.
//   k_compact      — per chunk: word records -> CSR ids / offsets, row_ptr of the docs that
//                    start in it; k_compact_long — its groups of long words.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <atomic>
#include <vector>

#include "encode.hpp"
#include "tables.hpp"

namespace tkz {

#ifndef TKZ_BPE_BUCKETS
// k_encode's BPE length buckets: 2 = L <= 4 (4-symbol register BPE) and L <= 8 (8 symbols);
// 1 = one 8-symbol queue (1 KB less LDS). With the ASCII byte ids read from the global table
// (TKZ_LDS_BYTE_ID 0) two buckets fit 7,528 B of LDS per one-wave block: 20 resident blocks
// per CU (gfx950 allocates LDS in 1,280-B units, tools/residency.py; 8,088 B gave 18).
// Against one bucket: C1 +0.8 %, C5 even, memo off C1 92.4 vs 70.2 GB/s
// (profiles/r03z_buckets_byteid_ab.txt, r03w_buckets_ab.txt)
#define TKZ_BPE_BUCKETS 2
#endif
constexpr int WAVE = 64;
constexpr int STEP = 1024;  // bytes per wave scan step (16 per lane)
constexpr int HSTEP = 512;  // a half step (the first 32 lanes): ring overflow
constexpr int RBASE = 1024; // ring entries: chunk-relative offset - (step start - RBASE)
constexpr int RCAP = 576;   // word ring slots: <= 63 pending + 1 open + 512 new (a step with
                            // more new words runs as a half step: <= 512)
constexpr int GROUP = 512;  // bytes (long_init) / words (k_compact) per wave pass, 8 per lane
constexpr int QCAP = 127;   // per-bucket queue: <= 63 waiting + 64 dispatched
constexpr int NB = 3;       // WordPiece length buckets: L<=8, L<=16, longer
// BPE keeps only the two short buckets in k_encode; longer memo misses are deferred to
// k_bpe_deferred, so k_encode's register budget is set by the 8-symbol path
template <int MODEL>
struct Buckets { static constexpr int n = MODEL == 1 ? TKZ_BPE_BUCKETS : NB; };
constexpr uint32_t DIRTY = 0xFFFFFFFEu;
constexpr uint32_t LONG_WORD = 64;  // BPE words longer than this (bytes) go to k_bpe_long
// queue entry: byte position (36 bits) | ordinal in its chunk (13 bits) | length (15 bits)
constexpr int POS_BITS = 36;
constexpr uint64_t POS_MASK = (1ull << POS_BITS) - 1;
constexpr uint32_t ORD_MASK = 0x1FFFu;
constexpr int LEN_SHIFT = 49;
constexpr uint32_t LEN_ESC = 0x7FFFu;
#ifndef TKZ_MAXW
#define TKZ_MAXW 16
#endif
#ifndef TKZ_PG
#define TKZ_PG 2  // pairs probed together in the W <= 8 register BPE (3 -> 2: C1 k_encode -1 %, C5 -1.5 %, profiles/r04ab_pg_ab.txt)
#endif
#ifndef TKZ_MINW
#define TKZ_MINW 5
#endif
#ifndef TKZ_ABLATE
#define TKZ_ABLATE 0
#endif
#ifndef TKZ_NT_INPUT
#define TKZ_NT_INPUT 0
#endif
#ifndef TKZ_LDS_BYTE_ID
#define TKZ_LDS_BYTE_ID 0  // k_encode's ASCII byte ids: 1 = an LDS copy (512 B), 0 = the global table
#endif
#ifndef TKZ_VEC_DOCS
#define TKZ_VEC_DOCS 1  // k_encode: a step's doc boundaries by one vector load (0: a scalar walk over doc_off)
#endif
#ifndef TKZ_SEG_FIRST
#define TKZ_SEG_FIRST 1  // the segmented path's iteration 0 through k_seg_first (0: every segment by k_seg_enc)
#endif
#ifndef TKZ_PREFETCH_STEP
#define TKZ_PREFETCH_STEP 0  // k_encode: load the next scan step's input when a step ends (measured: slower, spills)
#endif
#ifndef TKZ_SEG_KP
#define TKZ_SEG_KP 4  // boundary replay: pairs probed together
#endif
#ifndef TKZ_FULL_ABL
#define TKZ_FULL_ABL 0  // k_seg_first timing ablations (wrong results): 1 no boundary walk, 2 no probe loads
#endif
#ifndef TKZ_SEG_ASCII
#define TKZ_SEG_ASCII 1  // seg_encode: all-ASCII groups' symbols from a kept-byte mask
#endif
#ifndef TKZ_SEG_W32
#define TKZ_SEG_W32 1  // k_seg_enc_big: groups of 17..32 symbols lane by lane (0: the wave path for all)
#endif
#ifndef TKZ_LONG_SPEC
#define TKZ_LONG_SPEC 1  // k_bpe_long's LDS path: speculative second rank per round
#endif

// Workspace header: HDR_WORDS u64 words at the start of the workspace. The chunk ticket
// and the deferred-list counts are reset per (sub-)batch; the batch statistics
// (tkz_batch_stats) accumulate over the sub-batches of one call; the two token-base
// slots carry the running token count from one sub-batch to the next.
constexpr int HDR_TICKET = 0;     // chunk ticket counter
constexpr int HDR_DEFER = 1;      // u32 [0] deferred words, [1] dedup owners (this sub-batch)
constexpr int HDR_WORDS = 2;      // pretokens seen by k_encode
constexpr int HDR_HITS = 3;       // pretokens resolved by the word memo / whole-word probe
constexpr int HDR_DBG = 4;        // 12 debug counters (TKZ_PHASES)
constexpr int HDR_DEFERRED = 16;  // deferred words (all sub-batches)
constexpr int HDR_OWNERS = 17;    // deferred words the model ran on after dedup
constexpr int HDR_SUBS = 18;      // sub-batches of the call
constexpr int HDR_BASE = 20;      // [20], [21]: token base of the next sub-batch (ping-pong)
constexpr int HDR_SPLITS = 22;    // k_split: number of sub-batches found, then an error flag
constexpr int HDR_LONG = 24;      // u32 [0] long words (k_bpe_long list, this sub-batch), [1] their ticket
constexpr int HDR_LONGW = 25;     // long words (all sub-batches)
constexpr int HDR_CLONG = 26;     // u32: k_compact's long-word groups (k_compact_long's list)
constexpr int HDR_SEG = 27;       // u32 [0] the segmented path's leftovers (flist), [1] their ticket (+ 28)
constexpr int HDR_SEGW = 29;      // long words encoded by the segmented path (all sub-batches)
constexpr int HDR_LONGB = 30;     // bytes of the long words k_bpe_long ran on (all sub-batches)
constexpr int HDR_N = 32;         // 256 B

__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }

// Barrier for a one-wave block: orders the wave's LDS traffic (lanes exchange state
// through LDS) without the workgroup-scope release of __syncthreads, which waits for
// every outstanding global store of the wave (vmcnt(0)) at each phase change. A wave's
// own global accesses to one address stay in order, so nothing else is needed.
#define WAVE_SYNC()                                          \
    do {                                                     \
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront"); \
        __builtin_amdgcn_wave_barrier();                     \
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront"); \
    } while (0)

// debug build (-DTKZ_PHASES): per-phase s_memtime cycles of k_encode, summed over waves
#ifdef TKZ_PHASES
#define PH_BEGIN() uint64_t ph_t0 = __builtin_amdgcn_s_memtime()
#define PH_END(k) ph[k] += __builtin_amdgcn_s_memtime() - ph_t0
#define PH_LAP(k)                                          \
    do {                                                   \
        const uint64_t ph_t1 = __builtin_amdgcn_s_memtime(); \
        ph[k] += ph_t1 - ph_t0;                            \
        ph_t0 = ph_t1;                                     \
    } while (0)
#elif defined(TKZ_MARKS)  // asm listing markers per phase (static instruction counts)
#define PH_MARK(n) asm volatile("; TKZ_MARK " n)
#define PH_BEGIN() asm volatile("; TKZ_MARK begin")
#define PH_END(k) asm volatile("; TKZ_MARK end " #k)
#define PH_LAP(k) asm volatile("; TKZ_MARK lap " #k)
#else
#define PH_BEGIN()
#define PH_END(k)
#define PH_LAP(k)
#endif
#ifndef PH_MARK
#define PH_MARK(n)
#endif

__device__ __forceinline__ uint32_t seq_len(uint32_t b) {
    // std.unicode.utf8ByteSequenceLength; invalid lead bytes -> 1 (reference: unreachable)
    if (b < 0x80u) return 1;
    if (b >= 0xC0u && b <= 0xDFu) return 2;
    if (b >= 0xE0u && b <= 0xEFu) return 3;
    if (b >= 0xF0u && b <= 0xF7u) return 4;
    return 1;
}
__device__ __forceinline__ uint32_t lower(uint32_t c, int norm) {
    return (norm && c >= 'A' && c <= 'Z') ? (c | 0x20u) : c;
}
// std.ascii.toLower on 8 bytes at once
__device__ __forceinline__ uint64_t lower8(uint64_t x) {
    const uint64_t h = x & 0x7F7F7F7F7F7F7F7Full;
    const uint64_t ge_a = (h + 0x3F3F3F3F3F3F3F3Full) & 0x8080808080808080ull;  // >= 'A'
    const uint64_t gt_z = (h + 0x2525252525252525ull) & 0x8080808080808080ull;  // >  'Z'
    const uint64_t up = ge_a & ~gt_z & ~x & 0x8080808080808080ull;
    return x | (up >> 2);
}
__device__ __forceinline__ bool is_punct(uint32_t c) {
    return (c >= 33 && c <= 47) || (c >= 58 && c <= 64) || (c >= 91 && c <= 96) || (c >= 123 && c <= 126);
}
// inclusive wave prefix sum with DPP row shifts / broadcasts (no LDS round trips)
__device__ __forceinline__ int wave_incl_scan(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);  // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);  // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);  // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false);  // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);  // row_bcast:15
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);  // row_bcast:31
    return v;
}
__device__ __forceinline__ uint32_t rfl(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ uint64_t rfl64(uint64_t x) {
    return ((uint64_t)rfl((uint32_t)(x >> 32)) << 32) | rfl((uint32_t)x);
}
// active lanes of m below this lane
__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
}
__device__ __forceinline__ uint32_t lane63(uint32_t x) { return (uint32_t)__builtin_amdgcn_readlane((int)x, 63); }

// ---------------------------------------------------------------------------
// Byte readers (normalized bytes, word-relative position)
// ---------------------------------------------------------------------------
struct GlbReader {
    const uint8_t* p0;
    int norm;
    __device__ uint32_t operator()(uint32_t p) const { return lower(p0[p], norm); }
    // bytes [start, start+16) of a word of L bytes (zero past L), little-endian
    __device__ void window(uint32_t start, uint32_t L, uint64_t& lo, uint64_t& hi) const {
        lo = hi = 0;
        for (uint32_t j = 0; j < 16 && start + j < L; ++j) {
            const uint64_t b = (*this)(start + j);
            if (j < 8) lo |= b << (8 * j);
            else hi |= b << (8 * (j - 8));
        }
    }
};

// The first 8*NW bytes of a word, aligned to bit 0 of w[0], lowercased if needed.
// Loads NW+1 aligned u64 (the input buffer is readable up to a multiple of 16 bytes).
template <int NW>
struct WordBytes {
    uint64_t w[NW];
    __device__ __forceinline__ void load(const uint8_t* bytes, uint64_t pos, uint64_t limit, int norm) {
        const uint64_t a = pos & ~7ull;
        const uint32_t s = (uint32_t)(pos - a) * 8;
        uint64_t q[NW + 1];
#pragma unroll
        for (int k = 0; k <= NW; ++k)
            q[k] = (a + 8ull * k + 8 <= limit) ? *(const uint64_t*)(bytes + a + 8ull * k) : 0ull;
#pragma unroll
        for (int k = 0; k < NW; ++k) {
            uint64_t v = s ? ((q[k] >> s) | (q[k + 1] << (64 - s))) : q[k];
            w[k] = norm ? lower8(v) : v;
        }
    }
    // byte j for a j that is a compile-time constant after unrolling
    __device__ __forceinline__ uint32_t at(int j) const { return (uint32_t)(w[j >> 3] >> ((j & 7) * 8)) & 0xFFu; }
    // runtime byte index: a bit-tree of selects over scalar copies (an indexed array here
    // is lowered to scratch memory by the compiler)
    __device__ __forceinline__ uint32_t operator()(uint32_t p) const {
        if (NW > 4) return (uint32_t)(sel(p >> 3) >> ((p & 7u) * 8u)) & 0xFFu;  // (W = 32 groups: 64 bytes)
        const uint64_t w0 = w[0], w1 = NW > 1 ? w[1] : 0ull, w2 = NW > 2 ? w[2] : 0ull, w3 = NW > 3 ? w[3] : 0ull;
        const uint32_t i = p >> 3;
        uint64_t v = (NW > 1 && (i & 1u)) ? w1 : w0;
        if (NW > 2) {
            const uint64_t hi = (i & 1u) ? w3 : w2;
            v = (i & 2u) ? hi : v;
        }
        return (uint32_t)(v >> ((p & 7u) * 8u)) & 0xFFu;
    }
    __device__ __forceinline__ uint64_t sel(uint32_t i) const {
        uint64_t r = 0;
#pragma unroll
        for (int k = 0; k < NW; ++k) r = (i == (uint32_t)k) ? w[k] : r;
        return r;
    }
    // bytes [start, start+16) (bytes past the word are garbage; callers mask by length)
    __device__ __forceinline__ void window(uint32_t start, uint32_t L, uint64_t& lo, uint64_t& hi) const {
        (void)L;
        const uint32_t i = start >> 3, sh = (start & 7u) * 8u;
        const uint64_t a = sel(i), b = sel(i + 1), c = sel(i + 2);
        lo = sh ? (a >> sh) | (b << (64 - sh)) : a;
        hi = sh ? (b >> sh) | (c << (64 - sh)) : b;
    }
};

// ---------------------------------------------------------------------------
// Literal BPE.tokenize (bpe.zig:173-263) on a global workspace (long words, and every
// word when a merge has new_id == first). Entry k: ids[k], offs[k] = start | end<<32,
// prs[k] = cached merge value of pair (k, k+1).
// ---------------------------------------------------------------------------
struct GlbSyms {
    uint32_t* ids;
    uint64_t* offs;
    uint32_t* prs;
    __device__ uint32_t id(int k) const { return ids[k]; }
    __device__ uint32_t start(int k) const { return (uint32_t)offs[k]; }
    __device__ uint32_t end(int k) const { return (uint32_t)(offs[k] >> 32); }
    __device__ void set(int k, uint32_t id, uint32_t s, uint32_t e) {
        ids[k] = id;
        offs[k] = (uint64_t)s | ((uint64_t)e << 32);
    }
    __device__ void copy(int w, int r) { ids[w] = ids[r]; offs[w] = offs[r]; }
    __device__ uint32_t pr(int k) const { return prs[k]; }
    __device__ void set_pr(int k, uint32_t v) { prs[k] = v; }
};

template <bool COMPACT>
__device__ __forceinline__ uint32_t pair_value(const DevTables& T, uint32_t a, uint32_t b) {
    if (COMPACT) return merge_probe_compact(T.mtab_c, T.m_bits, a, b);
    uint32_t r, n;
    return merge_probe_wide(T.mtab_w, T.m_bits, a, b, r, n) ? r : NONE;
}

// Bucketized cuckoo merge tables: the compact one (COMPACT) or the mid one (wide ids < 2^20,
// the segmented path). A lookup is two 16-B bucket loads issued together, then a match.
template <bool COMPACT>
__device__ __forceinline__ void cuckoo_buckets(const DevTables& T, uint32_t a, uint32_t b, uint32_t& b1, uint32_t& b2) {
    if (COMPACT) merge_buckets_compact((a << 16) | b, T.m_bits, b1, b2);
    else merge_buckets_mid(a, b, T.mm_bits, b1, b2);
}
template <bool COMPACT>
__device__ __forceinline__ uint4 cuckoo_bucket(const DevTables& T, uint32_t k) {
    return *(const uint4*)((COMPACT ? T.mtab_c : T.mtab_m) + 2 * k);
}
template <bool COMPACT>
__device__ __forceinline__ uint32_t cuckoo_match(const uint4& p, const uint4& q, uint32_t a, uint32_t b) {
    return COMPACT ? merge_match_compact(p, q, (a << 16) | b) : merge_match_mid(p, q, a, b);
}
// a pair's merge value from a cuckoo table (compact: rank << 16 | new_id; mid: the rank)
template <bool COMPACT>
__device__ __forceinline__ uint32_t cuckoo_value(const DevTables& T, uint32_t a, uint32_t b) {
    uint32_t b1, b2;
    cuckoo_buckets<COMPACT>(T, a, b, b1, b2);
    return cuckoo_match<COMPACT>(cuckoo_bucket<COMPACT>(T, b1), cuckoo_bucket<COMPACT>(T, b2), a, b);
}

__device__ __forceinline__ uint32_t char_id(const DevTables& T, const uint32_t* byte_id, uint32_t b0, uint32_t packed,
                                            uint32_t len) {
    // byte_id: an LDS copy of at least the ASCII entries (k_encode holds 128)
    uint32_t id = (len == 1) ? (b0 < 128u ? byte_id[b0] : T.byte_id[b0]) : cp_probe(T.cp_tab, T.cp_bits, packed, len);
    return id == NONE ? T.unk_id : id;  // unk_token if set and in vocab, else NONE = skip the char
}

template <bool COMPACT, class S, class R>
__device__ uint32_t bpe_word(const DevTables& T, const uint32_t* byte_id, S& sy, const R& rd, uint32_t L) {
    // initial symbols: codepoint slices (Utf8Iterator.nextCodepointSlice, bpe.zig:186-211)
    int n = 0;
    for (uint32_t p = 0; p < L;) {
        const uint32_t b0 = rd(p);
        uint32_t len = seq_len(b0);
        if (p + len > L) len = L - p;  // truncated sequence: clamp (reference: out-of-bounds)
        uint32_t packed = b0;
        for (uint32_t j = 1; j < len; ++j) packed |= rd(p + j) << (8 * j);
        const uint32_t id = char_id(T, byte_id, b0, packed, len);
        if (id != NONE) { sy.set(n, id, p, p + len); ++n; }
        p += len;
    }
    for (int k = 0; k + 1 < n; ++k) sy.set_pr(k, pair_value<COMPACT>(T, sy.id(k), sy.id(k + 1)));
    // merge rounds (bpe.zig:214-253)
    while (n > 1) {
        uint32_t best = NONE;
        int bk = 0;
        for (int k = 0; k + 1 < n; ++k) {
            const uint32_t v = sy.pr(k);
            if (v < best) { best = v; bk = k; }
        }
        if (best == NONE) break;
        const uint32_t a = sy.id(bk), b = sy.id(bk + 1);
        uint32_t X;
        if (COMPACT) {
            X = best & 0xFFFFu;
        } else {
            uint32_t r;
            merge_probe_wide(T.mtab_w, T.m_bits, a, b, r, X);
        }
        // left-to-right: replace every (a,b) with X, re-testing at the same position
        int r = 0, w = 0;
        while (r < n) {
            if (r + 1 < n && sy.id(r) == a && sy.id(r + 1) == b) {
                const uint32_t s0 = sy.start(r);
                uint32_t e1 = sy.end(r + 1);
                r += 2;
                while (X == a && r < n && sy.id(r) == b) { e1 = sy.end(r); ++r; }  // new_id == first
                sy.set(w, X, s0, e1);
                sy.set_pr(w, DIRTY);
                if (w > 0) sy.set_pr(w - 1, DIRTY);
                ++w;
            } else {
                if (w != r) { sy.copy(w, r); sy.set_pr(w, sy.pr(r)); }
                ++w;
                ++r;
            }
        }
        n = w;
        for (int k = 0; k + 1 < n; ++k)
            if (sy.pr(k) == DIRTY) sy.set_pr(k, pair_value<COMPACT>(T, sy.id(k), sy.id(k + 1)));
    }
    return (uint32_t)n;
}

// ---------------------------------------------------------------------------
// Register-resident BPE for words of <= W codepoint slices. Same semantics as bpe_word
// for merge tables without a new_id == first merge (T.chain == 0): in a round every
// occurrence of the best pair is a position whose cached pair value equals the round
// minimum (ranks are unique per pair), and left-to-right replacement with re-test ==
// greedy selection inside runs of adjacent candidates. All arrays use compile-time
// indices (unrolled); all pair probes of a round are issued back to back.
// ---------------------------------------------------------------------------
// PACK: the symbol and its offsets in one register -- compact ids: id | start << 16 | end
// << 24 (words <= 255 B); wide ids < 2^20 (the segmented path): id | start << 20 | (end - 1)
// << 26 (words <= 64 B). !PACK (wide): id, and start | end << 16 in sp.
template <int W, bool COMPACT, bool PACK = COMPACT>
struct RegWord {
    uint32_t sy[W];
    uint32_t sp[PACK ? 1 : W];
    uint32_t pr[W];                // cached value of pair (k, k+1); NONE beyond n-2
    int n;
    static constexpr uint32_t SMASK = COMPACT ? 0x00FF0000u : 0x03F00000u;  // (PACK) start, end bits
    static constexpr uint32_t EMASK = COMPACT ? 0xFF000000u : 0xFC000000u;
    __device__ __forceinline__ static uint32_t idv(uint32_t v) {
        return !PACK ? v : COMPACT ? (v & 0xFFFFu) : (v & 0xFFFFFu);
    }
    __device__ __forceinline__ uint32_t start(int k) const {
        return !PACK ? (sp[k] & 0xFFFFu) : COMPACT ? ((sy[k] >> 16) & 0xFFu) : ((sy[k] >> 20) & 63u);
    }
    __device__ __forceinline__ uint32_t end(int k) const {
        return !PACK ? (sp[k] >> 16) : COMPACT ? (sy[k] >> 24) : (sy[k] >> 26) + 1u;
    }
};

// A word-bound token of wide tables with ids < 2^20 (T.mid): id | start << 20 |
// (end - 1) << 26, offsets word-relative (words <= 64 B); bit 31 is clear for end <= 32
__device__ __forceinline__ uint32_t mid_tok(uint32_t id, uint32_t s, uint32_t e) {
    return id | (s << 20) | ((e - 1u) << 26);
}

// Probes the pairs (k, k+1) of `mask`, PG at a time. Every load of a group is issued
// unconditionally (pairs outside the mask read bucket 0), so a group costs one memory
// round trip: loads under per-pair branches were each preceded by a full vmcnt drain.
// Compact table: cuckoo, both candidate buckets of every pair loaded together, so no
// lane ever walks a chain.
template <int W, bool COMPACT, bool PACK>
__device__ __forceinline__ void reg_probe(const DevTables& T, RegWord<W, COMPACT, PACK>& w, uint32_t mask) {
    constexpr int PG = W <= 8 ? TKZ_PG : 4;
    uint32_t retry = 0;  // (wide) pairs whose home slot holds another key
#pragma unroll
    for (int g = 0; g < W - 1; g += PG) {
        if (((mask >> g) & ((1u << PG) - 1)) == 0) continue;
        if (COMPACT || PACK) {  // (PACK && !COMPACT: the mid table)
            uint4 p[PG], q[PG];
#pragma unroll
            for (int k = g; k < g + PG && k < W - 1; ++k) {
                uint32_t b1, b2;
                cuckoo_buckets<COMPACT>(T, w.idv(w.sy[k]), w.idv(w.sy[k + 1]), b1, b2);
                const bool on = (mask >> k) & 1u;
                p[k - g] = cuckoo_bucket<COMPACT>(T, on ? b1 : 0u);
                q[k - g] = cuckoo_bucket<COMPACT>(T, on ? b2 : 0u);
            }
#pragma unroll
            for (int k = g; k < g + PG && k < W - 1; ++k)
                if ((mask >> k) & 1u) w.pr[k] = cuckoo_match<COMPACT>(p[k - g], q[k - g], w.idv(w.sy[k]), w.idv(w.sy[k + 1]));
        } else {
            uint4 s[PG];
#pragma unroll
            for (int k = g; k < g + PG && k < W - 1; ++k) {
                const uint64_t key = ((uint64_t)w.idv(w.sy[k]) << 32) | w.idv(w.sy[k + 1]);
                s[k - g] = T.mtab_w[((mask >> k) & 1u) ? merge_slot_wide(key, T.m_bits) : 0u];
            }
#pragma unroll
            for (int k = g; k < g + PG && k < W - 1; ++k) {
                if ((mask >> k) & 1u) {
                    const uint32_t a = w.idv(w.sy[k]), b = w.idv(w.sy[k + 1]);
                    const bool hit = s[k - g].x == a && s[k - g].y == b;
                    w.pr[k] = hit && s[k - g].z != EMPTY32 ? s[k - g].z : NONE;
                    if (!hit && s[k - g].z != EMPTY32) retry |= 1u << k;
                }
            }
        }
    }
    // (wide) the rare walks past a home slot, after the unrolled groups: a probe loop inside
    // them kept W = 32 words from being fully unrolled (register arrays went to scratch)
    while (!COMPACT && retry) {
        const int k = __builtin_ctz(retry);
        retry &= retry - 1u;
        uint32_t a = 0, b = 0;
#pragma unroll
        for (int j = 0; j < W - 1; ++j)
            if (j == k) { a = w.idv(w.sy[j]); b = w.idv(w.sy[j + 1]); }
        const uint32_t v = pair_value<false>(T, a, b);
#pragma unroll
        for (int j = 0; j < W - 1; ++j)
            if (j == k) w.pr[j] = v;
    }
}

// The pairs (k0, k0+1) and (k0+1, k0+2) where (m & 1) / (m & 2): a round that merged
// one pair dirties at most these two, its neighbours. The three symbols are gathered by
// one compare per position (register arrays take compile-time indices only) and both
// pairs probed together: a fixed cost, where reg_probe's groups run whenever any lane of
// the wave has a dirty pair in them, i.e. nearly all of them every round.
#ifndef TKZ_PROBE3
#define TKZ_PROBE3 1  // bit 0: W = 16 (k_bpe_deferred), bit 1: W <= 8 (k_encode buckets; spills 12 B there)
#endif
template <int W, bool COMPACT, bool PACK>
__device__ __forceinline__ void reg_probe_adj(const DevTables& T, RegWord<W, COMPACT, PACK>& w, int k0, uint32_t m) {
    uint32_t x0 = 0, x1 = 0, x2 = 0;
#pragma unroll
    for (int j = 0; j < W - 1; ++j) {
        const bool c = j == k0;
        x0 = c ? w.sy[j] : x0;
        x1 = c ? w.sy[j + 1] : x1;
        if (j + 2 < W) x2 = c ? w.sy[j + 2] : x2;
    }
    if (COMPACT || PACK) {  // (PACK && !COMPACT: the mid table)
        x0 = w.idv(x0);
        x1 = w.idv(x1);
        x2 = w.idv(x2);
        uint32_t a1, a2, b1, b2;
        cuckoo_buckets<COMPACT>(T, x0, x1, a1, a2);
        cuckoo_buckets<COMPACT>(T, x1, x2, b1, b2);
        const bool ob = (m >> 1) & 1u;
        const uint4 p0 = cuckoo_bucket<COMPACT>(T, a1), q0 = cuckoo_bucket<COMPACT>(T, a2);
        const uint4 p1 = cuckoo_bucket<COMPACT>(T, ob ? b1 : 0u), q1 = cuckoo_bucket<COMPACT>(T, ob ? b2 : 0u);
        const uint32_t va = cuckoo_match<COMPACT>(p0, q0, x0, x1), vb = cuckoo_match<COMPACT>(p1, q1, x1, x2);
        const bool oa = m & 1u;
#pragma unroll
        for (int j = 0; j < W - 1; ++j) {
            if (oa && j == k0) w.pr[j] = va;
            if (ob && j == k0 + 1) w.pr[j] = vb;
        }
    } else {  // wide: both home slots loaded together; a miss there walks on (load <= 1/4)
        x0 = w.idv(x0);
        x1 = w.idv(x1);
        x2 = w.idv(x2);
        const bool oa = m & 1u, ob = (m >> 1) & 1u;
        const uint4 sa = T.mtab_w[oa ? merge_slot_wide(((uint64_t)x0 << 32) | x1, T.m_bits) : 0u];
        const uint4 sb = T.mtab_w[ob ? merge_slot_wide(((uint64_t)x1 << 32) | x2, T.m_bits) : 0u];
        uint32_t va = NONE, vb = NONE;
        if (oa && sa.z != EMPTY32) va = sa.x == x0 && sa.y == x1 ? sa.z : pair_value<false>(T, x0, x1);
        if (ob && sb.z != EMPTY32) vb = sb.x == x1 && sb.y == x2 ? sb.z : pair_value<false>(T, x1, x2);
#pragma unroll
        for (int j = 0; j < W - 1; ++j) {
            if (oa && j == k0) w.pr[j] = va;
            if (ob && j == k0 + 1) w.pr[j] = vb;
        }
    }
}

template <int W, bool COMPACT, bool PACK>
__device__ __forceinline__ void reg_set(RegWord<W, COMPACT, PACK>& w, int j, uint32_t id, uint32_t s, uint32_t e) {
    if (PACK) w.sy[j] = COMPACT ? id | (s << 16) | (e << 24) : id | (s << 20) | ((e - 1u) << 26);
    else { w.sy[j] = id; w.sp[j] = s | (e << 16); }
}

// Initial symbols from a word held in registers. Returns false if > W symbols.
template <int W, bool COMPACT, int NW, class R, bool PACK>
__device__ __forceinline__ bool reg_init(const DevTables& T, const uint32_t* byte_id, RegWord<W, COMPACT, PACK>& w,
                                         const WordBytes<NW>& wb, const R& gr, uint32_t L) {
#pragma unroll
    for (int k = 0; k < W; ++k) w.pr[k] = NONE;
    // fast path: every byte ASCII and in the vocab -> symbol k = byte k
    uint64_t hi = 0;
#pragma unroll
    for (int k = 0; k < NW; ++k) {
        const int lo_b = 8 * k;
        uint64_t m = 0x8080808080808080ull;
        if (lo_b + 8 > (int)L) m = (lo_b >= (int)L) ? 0ull : (m & ((1ull << (8 * (L - lo_b))) - 1));
        hi |= wb.w[k] & m;
    }
    if (hi == 0 && L <= (uint32_t)W) {
        bool ok = true;
#pragma unroll
        for (int j = 0; j < W; ++j)
            if (j < (int)L) w.sy[j] = byte_id[wb.at(j)];
#pragma unroll
        for (int j = 0; j < W; ++j) {
            if (j < (int)L) {
                const uint32_t id = w.sy[j] == NONE ? T.unk_id : w.sy[j];
                ok = ok && id != NONE;
                reg_set(w, j, id, (uint32_t)j, (uint32_t)j + 1);
            }
        }
        if (ok) { w.n = (int)L; return true; }
    }
    // general path: codepoint slices, dropped chars, multi-byte table probes
    int n = 0;
    for (uint32_t p = 0; p < L;) {
        const uint32_t b0 = gr(p);
        uint32_t len = seq_len(b0);
        if (p + len > L) len = L - p;
        uint32_t packed = b0;
        for (uint32_t j = 1; j < len; ++j) packed |= gr(p + j) << (8 * j);
        const uint32_t id = char_id(T, byte_id, b0, packed, len);
        if (id != NONE) {
            if (n == W) return false;
#pragma unroll
            for (int j = 0; j < W; ++j)
                if (j == n) reg_set(w, j, id, p, p + len);
            ++n;
        }
        p += len;
    }
    w.n = n;
    return true;
}

// PROF (the segmented long-pretoken path): the word's edge lists -- the values of the rounds
// that merged its last symbol (RE) and its first symbol (LE), in round order -- go to prof
// as pairs (prof[k] = RE_k | LE_k << 32; SegEdges); returns the number of rounds, and in
// *edges the list lengths (LE bits 0..7, RE bits 8..15).
template <int W, bool COMPACT, bool PROF = false, bool PACK = COMPACT>
__device__ __forceinline__ uint32_t reg_rounds(const DevTables& T, RegWord<W, COMPACT, PACK>& w, uint64_t* prof = nullptr,
                               uint32_t* edges = nullptr) {
    uint32_t n_rounds = 0, lle = 0, lre = 0;
    if (w.n >= 2) reg_probe<W, COMPACT>(T, w, (1u << (w.n - 1)) - 1);
#if TKZ_ABLATE == 2
    return 0;
#endif
    while (w.n >= 2) {
        uint32_t best = NONE;
#pragma unroll
        for (int k = 0; k < W - 1; ++k) best = min(best, w.pr[k]);
        if (best == NONE) break;
        uint32_t X;
        if (COMPACT) {
            X = best & 0xFFFFu;
        } else if (PROF || T.r2id) {  // (the merge rank -> new_id table: one load, no probe walk;
            X = T.r2id[best];             // the segmented path always has it)
        } else {
            uint32_t a = 0, b = 0, r;
#pragma unroll
            for (int k = 0; k < W - 1; ++k)
                if (w.pr[k] == best) { a = w.idv(w.sy[k]); b = w.idv(w.sy[k + 1]); }
            merge_probe_wide(T.mtab_w, T.m_bits, a, b, r, X);
        }
        uint32_t sel = 0, prev = 0;
#pragma unroll
        for (int k = 0; k < W - 1; ++k) {
            const uint32_t c = (w.pr[k] == best) ? (1u - prev) : 0u;
            sel |= c << k;
            prev = c;
        }
        if (PROF) {  // the edge lists (seg_edge_put)
            const uint32_t le = sel & 1u, re = (sel >> (w.n - 2)) & 1u;
            ++n_rounds;
            uint32_t* p32 = (uint32_t*)prof;
            if (re) p32[2 * lre] = best;
            if (le) p32[2 * lle + 1] = best;
            lle += le;
            lre += re;
        }
        uint32_t dirty = 0;
        while (sel) {
            const int k = 31 - __clz(sel);
            sel ^= 1u << k;
#pragma unroll
            for (int j = 0; j < W - 1; ++j) {
                if (j == k) {
                    if (PACK) w.sy[j] = X | (w.sy[j] & w.SMASK) | (w.sy[j + 1] & w.EMASK);
                    else { w.sy[j] = X; w.sp[j] = (w.sp[j] & 0xFFFFu) | (w.sp[j + 1] & 0xFFFF0000u); }
                }
            }
#pragma unroll
            for (int j = 1; j < W - 1; ++j) {
                if (j > k) {
                    w.sy[j] = w.sy[j + 1];
                    w.pr[j] = w.pr[j + 1];
                    if (!PACK) w.sp[j] = w.sp[j + 1];
                }
            }
            --w.n;
            const uint32_t lowk = (2u << k) - 1;  // bits 0..k
            dirty = (dirty & lowk) | ((dirty >> 1) & ~lowk);
            dirty |= (1u << k) | (k > 0 ? (1u << (k - 1)) : 0u);
        }
        // pairs beyond the new end become NONE; recompute the touched ones
        const uint32_t live = (w.n >= 2) ? ((1u << (w.n - 1)) - 1) : 0u;
#pragma unroll
        for (int k = 0; k < W - 1; ++k)
            if (!((live >> k) & 1u)) w.pr[k] = NONE;
        const uint32_t dm = dirty & live;
        if ((W == 16 && (TKZ_PROBE3 & 1)) || (W <= 8 && (TKZ_PROBE3 & 2)) || (PACK && !COMPACT)) {
            const int k0 = dm ? __builtin_ctz(dm) : 0;
            const uint32_t m = dm >> k0;
            if (m <= 3u) {  // one merge: its (at most two) neighbouring pairs
                if (m) reg_probe_adj<W, COMPACT>(T, w, k0, m);
            } else {
                reg_probe<W, COMPACT>(T, w, dm);
            }
        } else {
            reg_probe<W, COMPACT>(T, w, dm);
        }
    }
    if (PROF) *edges = lle | (lre << 8);
    return n_rounds;
}

// ---------------------------------------------------------------------------
// WordPiece.tokenize (wordpiece.zig:141-222)
// ---------------------------------------------------------------------------
// vocab probe for key = [prefix if start>0] ++ word[start:e), hash `h`
template <class R>
__device__ __forceinline__ uint32_t wp_probe(const DevTables& T, const R& rd, uint64_t h, uint32_t klen,
                                             bool with_prefix, uint32_t start) {
    const uint32_t mask = (1u << T.wp_bits) - 1;
    uint32_t idx = (uint32_t)(h >> (64 - T.wp_bits));
    const uint32_t lo = (uint32_t)h, hi = (uint32_t)(h >> 32);
    while (true) {
        const uint4 s = T.wp_tab[idx];
        if (s.w == NONE) return NONE;
        if (s.x == lo && s.y == hi) {
            const uint8_t* ent = T.wp_pool + s.w;
            const uint32_t elen = *(const uint32_t*)ent;
            if (elen == klen) {
                bool ok = true;
                uint32_t q = 0;
                if (with_prefix)
                    for (; q < T.plen && ok; ++q) ok = ent[4 + q] == T.prefix[q];
                const uint32_t pre = with_prefix ? T.plen : 0;
                for (uint32_t j = 0; pre + j < klen && ok; ++j) ok = ent[4 + pre + j] == rd(start + j);
                if (ok) return s.z;
            }
        }
        idx = (idx + 1) & mask;
    }
}

// vocab probe for a key of <= 16 bytes held in registers (k0/k1 zero past klen): the
// short-key table stores the key bytes inline, so the match is exact. TKZ_WPS_WIN 32-B
// slots per round, loaded together (table without wrap-around, load <= 1/4; one slot per
// round measured 3.5 % faster on C3 than two: see memo_probe on the window size)
#ifndef TKZ_WPS_WIN
#define TKZ_WPS_WIN 1
#endif
__device__ __forceinline__ uint32_t wps_probe(const DevTables& T, uint64_t k0, uint64_t k1, uint32_t klen) {
    uint32_t h = memo_slot(k0, k1, klen, T.wps_bits);
    const uint32_t lo = (uint32_t)k0, hi = (uint32_t)(k0 >> 32), k1lo = (uint32_t)k1, k1hi = (uint32_t)(k1 >> 32);
    while (true) {
        const uint4* p = T.wps + 2 * h;
#if TKZ_WPS_WIN == 2
        const uint4 e0 = p[0], e1 = p[1], e2 = p[2], e3 = p[3];
        asm volatile("" ::"v"(e0.x), "v"(e0.y), "v"(e0.z), "v"(e0.w), "v"(e1.x), "v"(e1.y), "v"(e2.x), "v"(e2.y),
                     "v"(e2.z), "v"(e2.w), "v"(e3.x), "v"(e3.y));
#else
        const uint4 e0 = p[0], e1 = p[1];
        const uint4 e2 = make_uint4(~lo, 0u, 0u, 0u), e3 = make_uint4(0u, 0u, 0u, 0u);
        asm volatile("" ::"v"(e0.x), "v"(e0.y), "v"(e0.z), "v"(e0.w), "v"(e1.x), "v"(e1.y));
#endif
        uint32_t found = (((e1.x & 0xFFu) == klen) & (e0.x == lo) & (e0.y == hi) & (e0.z == k1lo) & (e0.w == k1hi)) |
                         ((((e3.x & 0xFFu) == klen) & (e2.x == lo) & (e2.y == hi) & (e2.z == k1lo) & (e2.w == k1hi))
                          << 1);
        const uint32_t empty = (e1.x == 0) | (TKZ_WPS_WIN == 2 ? ((e3.x == 0) << 1) : 0u);
        found &= (empty & (0u - empty)) - 1u;  // hits before the first empty slot
        if (found) return (found & 1u) ? e1.y : e3.y;
        if (empty) return NONE;
        h += TKZ_WPS_WIN;
    }
}

// WordPiece token output: narrow (tok) or wide (ids/offs) word-bound scratch
struct WpSink {
    uint32_t* tok;
    uint32_t* ids;
    uint64_t* offs;
    bool narrow;
    uint32_t first;  // narrow: the first token (a single-token word goes to its word slot)
    __device__ __forceinline__ void put(uint32_t n, uint32_t id, uint32_t s, uint32_t e) {
        if (narrow) {
            const uint32_t x = id | (s << 16) | (e << 24);
            if (n == 0) first = x;
            else tok[n] = x;
        } else {
            ids[n] = id;
            offs[n] = (uint64_t)s | ((uint64_t)e << 32);
        }
    }
};

// For a pretoken of L <= max_chars bytes: tokens to out[0..n). Returns n, or NONE when
// the word is "bad" (caller emits the single UNK).
template <class R>
__device__ uint32_t wordpiece_word(const DevTables& T, const R& rd, uint32_t L, WpSink& out) {
    uint32_t start = 0;
    uint32_t n = 0;
    while (start < L) {
        const bool pre = start > 0;
        uint32_t lim = T.max_key;
        if (pre) {
            lim = T.max_key > T.plen ? T.max_key - T.plen : 0;
            const uint32_t buf_lim = T.plen <= 512 ? 512 - T.plen : 0;  // substr_buf: [512]u8
            if (buf_lim < lim) lim = buf_lim;
        }
        const uint32_t emax = L - start < lim ? L : start + lim;
        const uint32_t pl = pre ? T.plen : 0;
        const bool all_short = pl + (emax - start) <= 16;  // every candidate in the short table
        // G(start, emax) and HP^(emax-start) for candidates of > 16 bytes
        uint64_t g = 0, pw = 1;
        if (!all_short)
            for (uint32_t j = start; j < emax; ++j) { g += (uint64_t)(rd(j) + 1) * pw; pw *= HP; }
        uint64_t w0, w1;
        rd.window(start, L, w0, w1);
        uint32_t found = NONE, e = emax;
        for (; e > start; --e) {
            const uint32_t klen = pl + (e - start);
            uint32_t id;
            if (klen <= 16) {
                const uint32_t nb = e - start;
                uint64_t k0 = nb >= 8 ? w0 : (w0 & ((1ull << (8 * nb)) - 1));
                uint64_t k1 = nb <= 8 ? 0ull : (nb >= 16 ? w1 : (w1 & ((1ull << (8 * (nb - 8))) - 1)));
                if (pl) {  // prepend the continuing-subword prefix (pl < 16 here)
                    const uint32_t sft = 8 * pl;
                    if (sft < 64) {
                        k1 = (k1 << sft) | (k0 >> (64 - sft));
                        k0 = (k0 << sft) | T.pfx0;
                    } else {
                        k1 = (k0 << (sft - 64)) | T.pfx1;
                        k0 = T.pfx0;
                    }
                }
                id = wps_probe(T, k0, k1, klen);
            } else {
                const uint64_t gk = pre ? T.g_prefix + T.p_plen * g : g;
                id = wp_probe(T, rd, wp_final(gk, klen), klen, pre, start);
            }
            if (id != NONE) { found = id; break; }
            if (!all_short) {
                pw *= T.hp_inv;                       // HP^(e-1-start)
                g -= (uint64_t)(rd(e - 1) + 1) * pw;  // drop byte e-1
            }
        }
        if (found == NONE) return NONE;
        out.put(n, found, start, e);
        ++n;
        start = e;
    }
    return n;
}

// ---------------------------------------------------------------------------
// Per-bucket word processing (one lane per word)
//
// Scratch is word-bound: a word's tokens sit at the word's own byte offset (tokens <=
// bytes), so words finish in any order without coordination.
//   tok[p]      narrow token  id | start<<16 | end<<24   (ids < 2^16, word <= 127 B, so
//               bit 31 is always clear)
//   ids/offs[p] wide token    u32 id, start | end<<32    (also the long-word BPE workspace)
// and every word owns a per-chunk slot, indexed by its ordinal among the words that start
// in its chunk (slot = chunk start + ordinal), holding one 32-bit record:
//   bit 31 clear        the word's single narrow token itself (end <= 127: bit 31 clear)
//   bit 31 set          count c in bits 22..28 and an offset in bits 0..21:
//     bits 30,29 = 0,0  narrow tokens word-bound at tok[chunk start + offset]
//     bits 30,29 = 0,1  narrow tokens in the chunk's dense area at element offset
//     bits 30,29 = 1,0  wide tokens at ids/offs[chunk start + offset]; c = 127: the count
//                       is in prs at that position
// Every writer also adds the word's token count to its chunk's count (ccnt, atomics; the
// dispatch batches of k_encode add theirs once per chunk), which the scan of chunk bases
// reads directly: no counting pass over the words.
// ---------------------------------------------------------------------------
constexpr uint32_t NARROW_MAX = 127;
constexpr uint32_t REC_MULTI = 0x80000000u, REC_WIDE = 0x40000000u, REC_DENSE = 0x20000000u;
constexpr uint32_t REC_OFF = 0x3FFFFFu;  // offset bits (chunks are <= 8 KiB)
constexpr int REC_CNT = 22;             // count bits 22..28
__host__ __device__ __forceinline__ uint32_t rec_count(uint32_t r) { return (r >> 31) ? (r >> REC_CNT) & 127u : 1u; }

// All arrays live in one workspace block (layout()); they are addressed from its base
// (k_encode runs out of SGPRs: every separately held pointer was another SGPR pair
// spilled to a VGPR lane and read back by a VALU v_readlane).
struct Scratch {
    uint8_t* base;
    uint64_t tb;
    uint64_t chmask;  // chunk bytes - 1
    uint32_t clog2;   // log2(chunk bytes)
    __device__ __forceinline__ uint64_t* offs() const { return (uint64_t*)base; }
    __device__ __forceinline__ uint32_t* ids() const { return (uint32_t*)(base + tb * 8); }
    __device__ __forceinline__ uint32_t* prs() const { return (uint32_t*)(base + tb * 12); }
    __device__ __forceinline__ uint32_t* tok() const { return (uint32_t*)(base + tb * 16); }
    __device__ __forceinline__ uint32_t* wslot() const { return (uint32_t*)(base + tb * 20); }
    // dense narrow tokens of multi-token BPE words of <= 16 bytes: chunk c's area starts
    // at element c * (chunk bytes + 128) (its words hold at most its bytes + 16 tokens).
    // The dispatch of k_encode fills it from the front (the wave owns the chunk: an LDS
    // counter), the model runs from the back (cfill[c], chunk_commit): the two ends never
    // meet
    __device__ __forceinline__ uint32_t* dtok() const { return (uint32_t*)(base + tb * 24); }
    __host__ __device__ static uint64_t dtok_elems(uint64_t tb) { return tb + tb / 4 + 16640; }
    __host__ __device__ static uint64_t chunk_cap(uint64_t tb) { return tb / 512 + 4; }
    __device__ __forceinline__ uint32_t* cfill() const { return (uint32_t*)(base + tb * 24 + dtok_elems(tb) * 4); }
    // per-chunk token counts
    __device__ __forceinline__ uint32_t* ccnt() const { return cfill() + chunk_cap(tb); }
    __device__ __forceinline__ uint64_t dbase(uint64_t pos) const {
        return (pos >> clog2) * ((1ull << clog2) + 128);
    }
    __device__ __forceinline__ uint64_t slot(uint64_t pos, uint32_t ord) const { return (pos & ~chmask) + ord; }
    // a word's token count -> its chunk's count (the slot index s is in the word's chunk)
    __device__ __forceinline__ void count(uint64_t s, uint32_t c) const {
        if (c) atomicAdd(ccnt() + (s >> clog2), c);
    }
    // writers of the word record; the _nc forms leave the count to the caller
    __device__ __forceinline__ void single_nc(uint64_t s, uint32_t t) const { wslot()[s] = t; }
    __device__ __forceinline__ void single(uint64_t s, uint32_t t) const { single_nc(s, t); count(s, 1); }
    // narrow tokens already at tok[pos..]; c != 1 (c <= 127)
    __device__ __forceinline__ void narrow_nc(uint64_t s, uint64_t pos, uint32_t c) const {
        wslot()[s] = REC_MULTI | (c << REC_CNT) | (uint32_t)(pos & chmask);
    }
    __device__ __forceinline__ void narrow(uint64_t s, uint64_t pos, uint32_t c) const { narrow_nc(s, pos, c); count(s, c); }
    // narrow tokens in the chunk's dense area at element off (c != 1)
    __device__ __forceinline__ void dense_nc(uint64_t s, uint32_t off, uint32_t c) const {
        wslot()[s] = REC_MULTI | REC_DENSE | (c << REC_CNT) | off;
    }
    // wide tokens already at ids/offs[pos..]
    __device__ __forceinline__ void wide_nc(uint64_t s, uint64_t pos, uint32_t c) const {
        wslot()[s] = REC_MULTI | REC_WIDE | (min(c, NARROW_MAX) << REC_CNT) | (uint32_t)(pos & chmask);
        if (c >= NARROW_MAX) prs()[pos] = c;
    }
    __device__ __forceinline__ void wide(uint64_t s, uint64_t pos, uint32_t c) const { wide_nc(s, pos, c); count(s, c); }
    // a segmented long pretoken (REC_SEG): its c tokens are written to the output by
    // k_seg_emit after the compaction, at the position k_compact_long leaves in offs[pos]; a
    // count of >= NARROW_MAX goes to ids[pos] (prs[pos] holds the first group's token offsets)
    __device__ __forceinline__ void seg(uint64_t s, uint64_t pos, uint32_t c) const {
        wslot()[s] = REC_MULTI | REC_WIDE | REC_DENSE | (min(c, NARROW_MAX) << REC_CNT) | (uint32_t)(pos & chmask);
        if (c >= NARROW_MAX) ids()[pos] = c;
        count(s, c);
    }
};
constexpr uint32_t REC_SEG = REC_MULTI | REC_WIDE | REC_DENSE;

// Chunk counters from a converged wave: adds every active lane's token count `cnt` to its
// chunk's ccnt and (ALLOC) allocates `need` dense slots from the back of the chunk's dense
// area, with one atomic per run of adjacent lanes in the same chunk -- a wave's words come
// in queue order, i.e. from one or two chunks (per-lane atomics on the same few counters
// serialised in L2: memo-off C1 2.4x slower). Returns the lane's dense element offset
// (ALLOC, need > 0). ALLOC packs need | cnt << 16: per lane both <= 1023.
template <bool ALLOC>
__device__ __forceinline__ uint32_t chunk_commit(const Scratch& S, bool act, uint64_t pos, uint32_t cnt,
                                                 uint32_t need) {
    const int lane = lane_id();
    const uint32_t v = act ? (ALLOC ? need | (cnt << 16) : cnt) : 0u;
    if (__ballot(v != 0u) == 0ull) return 0u;
    const uint32_t key = act ? (uint32_t)(pos >> S.clog2) : 0xFFFFFFFFu;
    const uint32_t pk = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)key, 0x138, 0xF, 0xF, false);  // wave_shr:1
    const bool head = lane == 0 || pk != key;
    const uint64_t H = __ballot(head);
    const uint32_t inc = (uint32_t)wave_incl_scan((int)v);
    const uint64_t le = (2ull << lane) - 1ull;  // lanes <= this one (lane 63: all)
    const int h = 63 - __clzll((long long)(H & le));
    const uint64_t after = H & ~le;
    const int t = after ? __ffsll((long long)after) - 2 : 63;
    const uint32_t b4 = (uint32_t)__shfl((int)inc, h > 0 ? h - 1 : 0, 64);
    const uint32_t before = h > 0 ? b4 : 0u;
    const uint32_t run = (uint32_t)__shfl((int)inc, t, 64) - before;
    uint32_t base = 0;
    if (head && act) {
        if (ALLOC) {
            if (run & 0xFFFFu) base = atomicAdd(S.cfill() + key, run & 0xFFFFu);
            if (run >> 16) atomicAdd(S.ccnt() + key, run >> 16);
        } else if (run) {
            atomicAdd(S.ccnt() + key, run);
        }
    }
    if (!ALLOC) return 0u;
    base = (uint32_t)__shfl((int)base, h, 64);
    return (1u << S.clog2) + 128u - base - (run & 0xFFFFu) + ((inc - v - before) & 0xFFFFu);
}

template <bool COMPACT>
__device__ __forceinline__ void bpe_long_word(const DevTables& T, const uint32_t* byte_id, const uint8_t* bytes,
                                              uint64_t pos, uint64_t ws, uint32_t L, const Scratch& S) {
    GlbSyms sy{S.ids() + pos, S.offs() + pos, S.prs() + pos};
    const uint32_t c = bpe_word<COMPACT>(T, byte_id, sy, GlbReader{bytes + pos, T.norm}, L);
    S.wide(ws, pos, c);
}

// Register BPE with W symbols on a word whose first 8*NW bytes are in wb, one word per
// lane of a converged wave (act: the lane has a word; the token counts and dense slots are
// committed for the wave together). Returns false (nothing written) when the lane's word
// has more than W symbols.
template <int W, int NW, bool COMPACT>
__device__ __forceinline__ bool bpe_reg_word(const DevTables& T, const uint32_t* byte_id, const uint8_t* bytes,
                                             const WordBytes<NW>& wb, uint64_t pos, uint64_t ws, uint32_t L,
                                             const Scratch& S, bool act) {
    RegWord<W, COMPACT> rw;
    // every caller has L <= 8 * NW: the general (multi-byte) path reads its bytes from wb
    // too (a GlbReader here cost one dependent global load per byte); no word: 0 symbols
    const bool fits = reg_init<W, COMPACT, NW>(T, byte_id, rw, wb, wb, act ? L : 0u);
#if TKZ_ABLATE != 3
    if (fits) reg_rounds<W, COMPACT>(T, rw);
#endif
    const bool emit = act && fits;
    const uint32_t c = emit ? (uint32_t)rw.n : 0u;
#ifndef TKZ_FORCE_WIDE
    if (COMPACT || T.mid) {  // the compact register symbol is the narrow token (T.mid: packed)
#else
    if (false) {
#endif
        // k_encode's bucket runs (W <= 8: a wave's words from one or two chunks) put
        // multi-token results in the chunk's dense area; k_bpe_deferred's length-sorted
        // words (W = 16, from many chunks: one allocation each) at their word-bound position
        // (the word-bound case commits its counts after the writes: rw is dead by then).
        // A T.mid single token ending past byte 32 has bit 31 set: a one-token multi record.
        auto tk = [&](int k) {
            return COMPACT ? rw.sy[k] : mid_tok(rw.idv(rw.sy[k]), rw.start(k), rw.end(k));
        };
        const bool single = c == 1u && (COMPACT || rw.end(0) <= 32u);
        constexpr bool DENSE = W <= 8;
        const uint32_t off = DENSE ? chunk_commit<true>(S, emit, pos, c, c >= 1u && !single ? c : 0u) : 0u;
        if (emit) {
            if (single) {
                S.single_nc(ws, tk(0));
            } else if (c == 0) {
                S.narrow_nc(ws, pos, 0);
            } else {
                uint32_t* dst = DENSE ? S.dtok() + S.dbase(pos) + off : S.tok() + pos;
#pragma unroll
                for (int k = 0; k < W; ++k)
                    if (k < rw.n) dst[k] = tk(k);
                if (DENSE) S.dense_nc(ws, off, c);
                else S.narrow_nc(ws, pos, c);
            }
        }
        if (!DENSE) chunk_commit<false>(S, emit, pos, c, 0u);
    } else {
        if (emit) {
#pragma unroll
            for (int k = 0; k < W; ++k) {
                if (k < rw.n) {
                    S.ids()[pos + k] = rw.idv(rw.sy[k]);
                    S.offs()[pos + k] = (uint64_t)rw.start(k) | ((uint64_t)rw.end(k) << 32);
                }
            }
            S.wide_nc(ws, pos, c);
        }
        chunk_commit<false>(S, emit, pos, c, 0u);
    }
    return fits;
}

// Word memo probe at dispatch for L <= 16 (compact ids; k0/k1 = the word's first 16
// normalized bytes, zero past L). Keys of <= 8 bytes live in the 16-B table, longer ones
// in the 32-B table; both are linear probing without wrap-around at load <= 1/4, one
// 32-bit hash for both (short_key_hash). Every lane loads a window of TKZ_MEMO_WIN 16-B
// blocks at its home slot per round: 2 slots of the 16-B table or 1 of the 32-B table
// with the default 2. The lookups are bound by their load instructions more than by
// their round trips: a 64-B window (4 loads, almost always one round) measured 3-4 %
// slower in k_encode than this 32-B one, an aligned window (no line straddling) and a
// 2-choice cuckoo table (two random lines) slower still. Keys are unique and never
// deleted, so any matching head of the window is the hit; an empty head (and no hit) is
// a miss; else the next window. The asm pins the loads so the compiler cannot sink the
// token words into the hit branch as a second, dependent load. On a hit the word is
// finished (slot ws): a single token goes to the word slot, 2-3 tokens to the word-bound
// scratch.
#ifndef TKZ_MEMO_WIN
#define TKZ_MEMO_WIN 1
#endif
// A memo hit's tokens: one token to the word slot, none as a count of 0, 2-3 to the
// chunk's dense area at element off (dst), allocated for the whole dispatch batch at once.
// The token counts are added by the batch (_nc writers).
__device__ __forceinline__ void memo_emit(const Scratch& S, bool s8, uint32_t meta, uint32_t w, uint32_t t1,
                                          uint32_t t2, uint32_t L, uint64_t ws, uint32_t* dst, uint32_t off) {
    const uint32_t nt = (meta >> 5) & 3u;
    if (nt == 1u) {
        S.single_nc(ws, w);
    } else if (nt == 0u) {
        S.dense_nc(ws, 0, 0);
    } else if (s8) {  // packed: w = id0 | id1 << 16, meta: e0, e1, id2
        const uint32_t b0 = (meta >> 7) & 0xFu, b1 = nt == 3u ? (meta >> 11) & 0xFu : L;
        dst[0] = (w & 0xFFFFu) | (b0 << 24);
        dst[1] = (w >> 16) | (b0 << 16) | (b1 << 24);
        if (nt > 2) dst[2] = (meta >> 15) | (b1 << 16) | (L << 24);
        S.dense_nc(ws, off, nt);
    } else {
        dst[0] = w;
        dst[1] = t1;
        if (nt > 2) dst[2] = t2;
        S.dense_nc(ws, off, nt);
    }
}

// A wide table's memo hit (nt <= 3 tokens id | start << 22 | end << 27) as wide tokens at
// the word's byte offset (a word of <= 16 bytes has room for 3); the count is added by the
// dispatch batch.
__device__ __forceinline__ void memo_emit_wide(const Scratch& S, uint32_t nt, uint32_t t0, uint32_t t1, uint32_t t2,
                                               uint64_t pos, uint64_t ws) {
    const uint32_t t[3] = {t0, t1, t2};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        if ((uint32_t)k < nt) {
            S.ids()[pos + k] = t[k] & 0x3FFFFFu;
            S.offs()[pos + k] = (uint64_t)((t[k] >> 22) & 0x1Fu) | ((uint64_t)(t[k] >> 27) << 32);
        }
    }
    S.wide_nc(ws, pos, nt);
}

// Returns true on a hit, with the slot's meta / token words (t1, t2: tokens 1, 2 of a 32-B slot)
template <bool COMPACT>
__device__ __forceinline__ bool memo_lookup(const DevTables& T, uint64_t k0, uint64_t k1, uint32_t L, uint32_t& hmeta,
                                            uint32_t& hw, uint32_t& ht1, uint32_t& ht2) {
    const bool s8 = COMPACT && L <= 8;  // wide tables: every key in the 32-B table
    uint32_t h = short_key_hash(k0, k1, L) >> (32 - (s8 ? T.memo8_bits : T.memo_bits));  // k1 = 0 when s8
    while (true) {
        const uint4* p = s8 ? T.memo8 + h : T.memo + 2 * h;
#if TKZ_ABLATE == 5  // no memory access: every probe hits a 1-token entry
        const uint4 e0 = make_uint4((uint32_t)k0, (uint32_t)(k0 >> 32), L | (1u << 5), h),
                    e1 = make_uint4((uint32_t)k1, (uint32_t)(k1 >> 32), 0u, (uint32_t)(uintptr_t)p);
        const uint4 e2 = e1, e3 = e1;
#elif TKZ_MEMO_WIN == 1
        // one 16-B slot per round for keys of <= 8 B (their table), the 32-B slot for longer
        // ones: a wave's probe is a gather of 64 distinct lines, bound by the lines the
        // vector memory pipeline looks up per cycle, so the second 16-B block of every
        // short-key window cost as much as the first (round 6)
        const uint4 e0 = p[0];
        uint4 e1 = make_uint4(0u, 0u, 1u, 0u);
        if (!s8) e1 = p[1];
        const uint4 e2 = make_uint4(0u, 0u, 1u, 0u), e3 = e2;
        asm volatile("" ::"v"(e0.x), "v"(e0.y), "v"(e0.z), "v"(e0.w), "v"(e1.x), "v"(e1.y), "v"(e1.z), "v"(e1.w));
#elif TKZ_MEMO_WIN == 4
        const uint4 e0 = p[0], e1 = p[1], e2 = p[2], e3 = p[3];
        asm volatile("" ::"v"(e0.x), "v"(e0.y), "v"(e0.z), "v"(e0.w), "v"(e1.x), "v"(e1.y), "v"(e1.z), "v"(e1.w),
                     "v"(e2.x), "v"(e2.y), "v"(e2.z), "v"(e2.w), "v"(e3.x), "v"(e3.y), "v"(e3.z), "v"(e3.w));
#else
        const uint4 e0 = p[0], e1 = p[1];
        const uint4 e2 = make_uint4(0u, 0u, 1u, 0u), e3 = e2;  // unused (TKZ_MEMO_WIN == 2)
        asm volatile("" ::"v"(e0.x), "v"(e0.y), "v"(e0.z), "v"(e0.w), "v"(e1.x), "v"(e1.y), "v"(e1.z), "v"(e1.w));
#endif
        // heads: every block of the 16-B table; blocks 0 (and 2) of the 32-B table, whose
        // blocks 1 (and 3) hold k1 (64-bit key compares combined in lane masks)
        constexpr bool W4 = TKZ_MEMO_WIN == 4, W1 = TKZ_MEMO_WIN == 1;
        const bool h0 = (((uint64_t)e0.y << 32) | e0.x) == k0 && (e0.z & 0x1Fu) == L;
        const bool h1 = !W1 && (((uint64_t)e1.y << 32) | e1.x) == k0 && (e1.z & 0x1Fu) == L;
        const bool h2 = W4 && (((uint64_t)e2.y << 32) | e2.x) == k0 && (e2.z & 0x1Fu) == L;
        const bool h3 = W4 && (((uint64_t)e3.y << 32) | e3.x) == k0 && (e3.z & 0x1Fu) == L;
        const bool c0 = (((uint64_t)e1.y << 32) | e1.x) == k1;
        const bool c2 = W4 && (((uint64_t)e3.y << 32) | e3.x) == k1;
        const bool found = s8 ? (h0 || h1 || h2 || h3) : ((h0 && c0) || (h2 && c2));
        if (found) {
            const bool u1 = s8 && h1, u2 = h2 && (s8 || c2), u3 = s8 && h3;
            uint32_t meta = u1 ? e1.z : e0.z, w = u1 ? e1.w : e0.w;
            if (W4) {
                meta = u2 ? e2.z : meta;
                w = u2 ? e2.w : w;
                meta = u3 ? e3.z : meta;
                w = u3 ? e3.w : w;
            }
            const uint4 f = u2 ? e3 : e1;  // tokens 1, 2 of a 32-B slot
            hmeta = meta;
            hw = w;
            ht1 = f.z;
            ht2 = f.w;
            return true;
        }
        const bool empty = (e0.z == 0) || (s8 && e1.z == 0) || (W4 && ((e2.z == 0) || (s8 && e3.z == 0)));
        if (empty) return false;
        h += W1 ? 1u : (s8 ? TKZ_MEMO_WIN : TKZ_MEMO_WIN / 2);
    }
}

// Two memo lookups at once (k_encode_blk, TKZ_BLK_W2): each round loads both words' windows
// before comparing either (one memory round trip for both); r = {meta, token 0, tokens 1, 2}.
template <bool COMPACT>
__device__ __forceinline__ void memo_lookup2(const DevTables& T, bool pa, uint64_t a0, uint64_t a1, uint32_t La, bool pb,
                                             uint64_t b0, uint64_t b1, uint32_t Lb, bool& ha, uint4& ra, bool& hb,
                                             uint4& rb) {
    const bool sa = COMPACT && La <= 8, sb = COMPACT && Lb <= 8;
    uint32_t hA = short_key_hash(a0, a1, La) >> (32 - (sa ? T.memo8_bits : T.memo_bits));
    uint32_t hB = short_key_hash(b0, b1, Lb) >> (32 - (sb ? T.memo8_bits : T.memo_bits));
    ha = hb = false;
    auto check = [&](const uint4& e0, const uint4& e1, uint64_t k0, uint64_t k1, uint32_t L, bool s8, bool& pend,
                     bool& h, uint4& r, uint32_t& slot) {
        const bool h0 = (((uint64_t)e0.y << 32) | e0.x) == k0 && (e0.z & 0x1Fu) == L;
        const bool h1 = (((uint64_t)e1.y << 32) | e1.x) == k0 && (e1.z & 0x1Fu) == L;
        const bool c0 = (((uint64_t)e1.y << 32) | e1.x) == k1;
        const bool found = s8 ? (h0 || h1) : (h0 && c0);
        if (found) {
            const bool u1 = s8 && h1;
            r = make_uint4(u1 ? e1.z : e0.z, u1 ? e1.w : e0.w, e1.z, e1.w);
            h = true;
            pend = false;
        } else if ((e0.z == 0) || (s8 && e1.z == 0)) {
            pend = false;
        } else {
            slot += s8 ? 2u : 1u;
        }
    };
    while (pa || pb) {
        const uint4* qa = sa ? T.memo8 + hA : T.memo + 2 * hA;
        const uint4* qb = sb ? T.memo8 + hB : T.memo + 2 * hB;
        const uint4 ea0 = qa[0], ea1 = qa[1], eb0 = qb[0], eb1 = qb[1];
        asm volatile("" ::"v"(ea0.x), "v"(ea0.y), "v"(ea0.z), "v"(ea0.w), "v"(ea1.x), "v"(ea1.y), "v"(ea1.z),
                     "v"(ea1.w), "v"(eb0.x), "v"(eb0.y), "v"(eb0.z), "v"(eb0.w), "v"(eb1.x), "v"(eb1.y), "v"(eb1.z),
                     "v"(eb1.w));
        if (pa) check(ea0, ea1, a0, a1, La, sa, pa, ha, ra, hA);
        if (pb) check(eb0, eb1, b0, b1, Lb, sb, pb, hb, rb, hB);
    }
}

template <int W, int NW, bool COMPACT>
__device__ __forceinline__ void bpe_bucket_word(const DevTables& T, const uint32_t* byte_id, const uint8_t* bytes,
                                                uint64_t limit, uint64_t pos, uint64_t ws, uint32_t L,
                                                const Scratch& S, bool act) {
    WordBytes<NW> wb;
    wb.load(bytes, pos, limit, T.norm);
    if (!bpe_reg_word<W, NW, COMPACT>(T, byte_id, bytes, wb, pos, ws, L, S, act) && act)
        bpe_long_word<COMPACT>(T, byte_id, bytes, pos, ws, L, S);  // > W symbols (rare): its own count
}

// WordPiece.tokenize of one word into its record; returns its token count (the caller
// commits the counts of the wave)
template <class R>
__device__ __forceinline__ uint32_t wp_word_out(const DevTables& T, const R& rd, uint64_t pos, uint64_t ws, uint32_t L,
                                                const Scratch& S, uint32_t* status) {
    uint32_t c = NONE;
    const bool nar = T.narrow && L <= NARROW_MAX;  // count <= L <= 127, offsets <= 127
    WpSink sink{S.tok() + pos, S.ids() + pos, S.offs() + pos, nar, 0u};
    if (L <= T.max_chars) c = wordpiece_word(T, rd, L, sink);
    if (c == NONE) {  // too long or bad -> one UNK (0, L)
        if (T.wp_unk == NONE && T.unk_drop) {  // WordPiece.tokenizeFast: no UNK -> no token
            if (nar) S.narrow_nc(ws, pos, 0); else S.wide_nc(ws, pos, 0);
            return 0u;
        }
        if (T.wp_unk == NONE) *status = 9u;  // TKZ_ERR_MISSING_UNK_TOKEN
        if (T.narrow && L <= NARROW_MAX) {
            // (no UNK: the batch fails with MissingUnkToken; keep the slot a valid token)
            S.single_nc(ws, (T.wp_unk == NONE ? 0u : T.wp_unk) | (L << 24));
        } else {
            S.ids()[pos] = T.wp_unk;
            S.offs()[pos] = (uint64_t)L << 32;
            S.wide_nc(ws, pos, 1);
        }
        return 1u;
    }
    if (nar && c == 1) {
        S.single_nc(ws, sink.first);
    } else if (nar) {
        if (c > 0) S.tok()[pos] = sink.first;
        S.narrow_nc(ws, pos, c);
    } else {
        S.wide_nc(ws, pos, c);
    }
    return c;
}

// Processes `cnt` (<= 64) queued words of bucket `b` (q points at the first), one lane
// per word; the whole wave enters (the token counts are committed per wave).
template <int MODEL, bool COMPACT>
__device__ __forceinline__ void run_bucket(const DevTables& T, const uint32_t* byte_id, const uint64_t* q, int b,
                                           uint32_t cnt, const uint8_t* bytes, uint64_t limit, const Scratch& S,
                                           uint32_t* status) {
    const int lane = lane_id();
    const bool act = (uint32_t)lane < cnt;
    const uint64_t e = act ? q[lane] : 0ull;
    const uint64_t pos = e & POS_MASK;
    const uint64_t ws = S.slot(pos, (uint32_t)(e >> POS_BITS) & ORD_MASK);
    uint32_t L = (uint32_t)(e >> LEN_SHIFT);
    if (L == LEN_ESC) L = S.prs()[pos];  // long pretokens keep their length in the pr slot
#if TKZ_ABLATE == 1
    if (act) S.narrow(ws, pos, 0);
    return;
#endif
    if (MODEL == 1) {
        if (T.chain) {
            if (act) bpe_long_word<COMPACT>(T, byte_id, bytes, pos, ws, L, S);
            return;
        }
        if (b == 0 && TKZ_BPE_BUCKETS == 2) bpe_bucket_word<4, 1, COMPACT>(T, byte_id, bytes, limit, pos, ws, L, S, act);
        else bpe_bucket_word<8, 1, COMPACT>(T, byte_id, bytes, limit, pos, ws, L, S, act);
        return;
    } else {
        uint32_t c = 0;
        if (act) {
            if (b == 0) {
                WordBytes<1> wb;
                wb.load(bytes, pos, limit, T.norm);
                c = wp_word_out(T, wb, pos, ws, L, S, status);
            } else if (L <= 32) {
                WordBytes<4> wb;
                wb.load(bytes, pos, limit, T.norm);
                c = wp_word_out(T, wb, pos, ws, L, S, status);
            } else {
                c = wp_word_out(T, GlbReader{bytes + pos, T.norm}, pos, ws, L, S, status);
            }
        }
        chunk_commit<false>(S, act, pos, c, 0u);
    }
}

// BPE (L <= 8 here): L <= 4, L <= 8; WordPiece: L <= 8, L <= 16, longer
template <int MODEL>
__device__ __forceinline__ int bucket_of(uint32_t L) {
    return MODEL == 1 ? (TKZ_BPE_BUCKETS == 1 ? 0 : (L <= 4 ? 0 : 1)) : (L <= 8 ? 0 : (L <= 16 ? 1 : 2));
}

// Pretokenizer byte classes (config.zig:405-457): split = delimiter, punct = BertPreTokenizer
// punctuation (its own one-byte pretoken).
__device__ __forceinline__ void classify(uint32_t c, int pretok, bool& split, bool& punct) {
    punct = false;
    split = false;
    if (pretok == 1) {
        split = (c == ' ' || c == '\t' || c == '\n' || c == '\r');
    } else if (pretok == 2) {
        punct = is_punct(c);
        split = punct || c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == 0x0B || c == 0x0C;
    }
}

// first doc boundary (index into doc_off) at or after byte position c * chunk, per chunk
__global__ __launch_bounds__(256) void k_chunk_docs(const uint64_t* __restrict__ doc_off, uint64_t n_docs,
                                                    uint32_t ch_log2, uint64_t* __restrict__ chunk_doc,
                                                    unsigned long long* __restrict__ chunk_ctr, int zero_stats) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k == 0) {  // ticket counter + the two deferred-list counts that follow it
        chunk_ctr[HDR_TICKET] = 0;
        chunk_ctr[HDR_DEFER] = 0;
        chunk_ctr[HDR_LONG] = 0;
        chunk_ctr[HDR_CLONG] = 0;
        chunk_ctr[HDR_SEG] = 0;
        chunk_ctr[HDR_SEG + 1] = 0;
        if (zero_stats) {
            chunk_ctr[HDR_SEGW] = 0;  // batch statistics accumulate over the sub-batches of one call
            chunk_ctr[HDR_WORDS] = 0;
            chunk_ctr[HDR_HITS] = 0;
            chunk_ctr[HDR_DEFERRED] = 0;
            chunk_ctr[HDR_OWNERS] = 0;
            chunk_ctr[HDR_SUBS] = 0;
            chunk_ctr[HDR_LONGW] = 0;
            chunk_ctr[HDR_LONGB] = 0;
        }
#if defined(TKZ_PHASES) || defined(TKZ_LONG_STATS) || defined(TKZ_SEG_STATS)
        for (int i = HDR_DBG; i < HDR_DBG + 12; ++i) chunk_ctr[i] = 0;
#endif
    }
    if (k > n_docs) return;
    const uint64_t lo = k == 0 ? 0 : doc_off[k - 1] + 1;
    const uint64_t hi = doc_off[k];
    if (lo > hi) return;  // empty doc: its boundary equals the previous one
    for (uint64_t c = (lo + (1ull << ch_log2) - 1) >> ch_log2; (c << ch_log2) <= hi; ++c) chunk_doc[c] = k;
}

// ---------------------------------------------------------------------------
// k_encode: the batch is a byte stream cut into chunks of 2^ch_log2 bytes. A chunk owns
// the words that START in it (it scans past its end to close the last one); document
// boundaries (doc_off) are forced word breaks. Persistent grid, one wave per block,
// chunks handed out by an atomic ticket counter.
//
// Per 512-B step: classify bytes (8 per lane), word start/end bit masks, one packed DPP
// prefix sum -> word ring (chunk-relative start/end, rebased every step). Complete
// words are dispatched 64 at a time: BPE words of <= 16 bytes probe the word memo right
// away (their bytes are in the LDS copy of the last two steps); the rest, and memo
// misses, go to length-bucket queues that run the model when 64 words are waiting.
// ---------------------------------------------------------------------------
// BPE words of > 8 bytes that the memo did not resolve. Each wave stages them in LDS and
// appends 64 at a time (one atomic per 64 words: a per-word atomic on one counter
// serialised the whole grid).
//
// A batch repeats its rare words (Zipf), so the list is deduplicated before the model
// runs: k_dedup keys every word of <= 32 bytes by its normalized bytes in a hash table
// (first to claim a slot owns the key; a later equal word records its owner), owners go
// to `olist` for k_bpe_deferred, and k_dedup_copy gives every duplicate its owner's
// tokens (offsets are word-relative, so they are the same). Same result as encoding each
// occurrence; words of > 32 bytes and tables with a new_id == first merge are never
// deduplicated. The table is bounded (dd_mask + 1 slots, 16 probes): a word that finds
// no slot is its own owner.
struct Deferred {
    uint64_t* list;
    uint32_t* cnt;              // [0] deferred words, [1] owners in olist
    unsigned long long* dbg;    // debug counters (TKZ_PHASES)
    uint64_t* olist;            // entries of the words the model runs on
    uint64_t* own;              // per list entry: its owner's entry, 0 for owners
    unsigned long long* dd;     // dedup table: the key owner's list entry, 0 = empty (entries
                                // of deferred words are never 0: L >= 9)
    uint32_t dd_mask;
    uint64_t* llist;            // words of > LONG_WORD bytes for k_bpe_long (one wave per word)
    uint32_t* lcnt;             // [0] entries in llist, [1] k_bpe_long's ticket
    uint64_t* flist;            // the long words the segmented path leaves to k_bpe_long
    uint32_t* fcnt;             // [0] entries in flist, [1] (k_bpe_long's ticket over it)
    unsigned long long* seg_words;  // long words the segmented path encoded (all sub-batches)
    unsigned long long* long_bytes; // bytes of the long words k_bpe_long ran on (all sub-batches)
    uint64_t* slist;            // k_encode_blk's memo misses of <= 8 B (k_bpe_short): chunk c's at [c << ch_log2..)
    uint32_t* scnt;             // per chunk: its entries in slist
};

// normalized bytes of a word of L <= 32 bytes, zero past L
__device__ __forceinline__ void dedup_key(const uint8_t* bytes, uint64_t pos, uint64_t limit, int norm, uint32_t L,
                                          WordBytes<4>& wb) {
    wb.load(bytes, pos, limit, norm);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int lo_b = 8 * k;
        if (lo_b >= (int)L) wb.w[k] = 0ull;
        else if (lo_b + 8 > (int)L) wb.w[k] &= (1ull << (8 * (L - lo_b))) - 1;
    }
}

// Two launches: entries [0, first) and then [first, n). A popular word's repeats that
// are in flight together all find its slot empty and all try to claim it, serialising on
// one address; the first launch takes a short prefix of the list, so most keys are
// claimed under little contention and the second launch mostly just reads.
__global__ __launch_bounds__(256) void k_dedup(DevTables T, const uint8_t* __restrict__ bytes, uint64_t limit,
                                               Deferred D, uint64_t first, int second) {
    __shared__ uint32_t wcount[5];  // owners per wave, then the block's base
    const int lane = lane_id();
    const uint64_t n = second ? *D.cnt : min(first, (uint64_t)*D.cnt);
    const uint64_t i0 = second ? first : 0;
    const uint64_t npad = i0 + ((n > i0 ? n - i0 : 0) + 255) / 256 * 256;  // whole blocks iterate together
    for (uint64_t i = i0 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < npad; i += (uint64_t)gridDim.x * blockDim.x) {
        bool owner = false;
        uint64_t e = 0;
        if (i < n) {
            e = D.list[i];
            const uint32_t L = (uint32_t)(e >> LEN_SHIFT);  // LEN_ESC (long) > 32
            uint64_t oe = 0;  // the owner's entry when this word is a repeat
            if (!T.chain && L <= 32) {
                WordBytes<4> wb;
                dedup_key(bytes, e & POS_MASK, limit, T.norm, L, wb);
                uint32_t h = (uint32_t)fmix64(wb.w[0] ^ (wb.w[1] * 0x9E3779B97F4A7C15ull) ^
                                              (wb.w[2] * 0xC2B2AE3D27D4EB4Full) ^ (wb.w[3] * 0x165667B19E3779F9ull) ^
                                              L) & D.dd_mask;
                for (int probe = 0; probe < 16; ++probe, h = (h + 1) & D.dd_mask) {
                    unsigned long long v = D.dd[h];
                    if (v == 0ull) {
                        v = atomicCAS(&D.dd[h], 0ull, (unsigned long long)e);
                        if (v == 0ull) break;  // claimed: owner
                    }
                    if ((uint32_t)(v >> LEN_SHIFT) != L) continue;
                    WordBytes<4> wj;
                    dedup_key(bytes, v & POS_MASK, limit, T.norm, L, wj);
                    if (((wj.w[0] ^ wb.w[0]) | (wj.w[1] ^ wb.w[1]) | (wj.w[2] ^ wb.w[2]) | (wj.w[3] ^ wb.w[3])) == 0ull) {
                        oe = v;
                        break;
                    }
                }
            }
            D.own[i] = oe;
            owner = oe == 0ull;
        }
        // owners to olist: one atomic per block and iteration (one per wave serialised the
        // whole grid on the counter: 1.6M C2 words = 25k atomics on one address)
        const uint64_t m = __ballot(owner);
        const int w = threadIdx.x >> 6;
        if (lane == 0) wcount[w] = (uint32_t)__popcll(m);
        __syncthreads();
        if (threadIdx.x == 0) {
            const uint32_t tot = wcount[0] + wcount[1] + wcount[2] + wcount[3];
            wcount[4] = tot ? atomicAdd(D.cnt + 1, tot) : 0u;
        }
        __syncthreads();
        uint32_t base = wcount[4];
        for (int k = 0; k < w; ++k) base += wcount[k];
        __syncthreads();  // wcount is rewritten by the next iteration
        if (owner)
            D.olist[base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0))] = e;
    }
}

// every duplicate takes its owner's tokens (word-bound scratch, word slot and count).
// Latency bound: one dependent chain per duplicate (entry -> owner's slot -> owner's
// tokens), so every load of a link is issued unconditionally and together: the owner's
// count and slot word, then up to 8 narrow tokens (a duplicate is <= 32 bytes, so a
// narrow count above 8 is rare and copied in a loop).
__global__ __launch_bounds__(256) void k_dedup_copy(Scratch S, Deferred D) {
    const uint64_t n = *D.cnt;
    const uint64_t npad = (n + 63) & ~63ull;  // the lanes of a wave iterate together (chunk_commit)
    uint32_t* __restrict__ tok = S.tok();
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < npad; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t eo = i < n ? D.own[i] : 0ull;
        const bool act = eo != 0ull;
        const uint64_t e = act ? D.list[i] : 0ull;
        const uint64_t pos = e & POS_MASK;
        uint32_t c = 0;
        if (act) {
            const uint64_t po = eo & POS_MASK;
            const uint64_t ws = S.slot(pos, (uint32_t)(e >> POS_BITS) & ORD_MASK);
            const uint64_t wso = S.slot(po, (uint32_t)(eo >> POS_BITS) & ORD_MASK);
            const uint32_t sw = S.wslot()[wso];  // the owner's record
            // the owner's narrow tokens: its dense area slots, or its word-bound scratch
            const uint32_t* src = (sw & REC_DENSE) ? S.dtok() + S.dbase(po) + (sw & REC_OFF) : tok + po;
            uint32_t t[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) t[k] = src[k];  // within the owner's area + 8: in the scratch block
            c = rec_count(sw);
            if (!(sw & REC_MULTI)) {
                S.single_nc(ws, sw);
            } else if (!(sw & REC_WIDE)) {
#pragma unroll
                for (int k = 0; k < 8; ++k)
                    if ((uint32_t)k < c) tok[pos + k] = t[k];
                for (uint32_t k = 8; k < c; ++k) tok[pos + k] = src[k];
                S.narrow_nc(ws, pos, c);
            } else {
                if (c == NARROW_MAX) c = S.prs()[po];
                for (uint32_t k = 0; k < c; ++k) {
                    S.ids()[pos + k] = S.ids()[po + k];
                    S.offs()[pos + k] = S.offs()[po + k];
                }
                S.wide_nc(ws, pos, c);
            }
        }
        chunk_commit<false>(S, act, pos, c, 0u);
    }
}

// One lane per deferred word (owners only): register BPE with 16 symbols, or the
// long-word path.
#ifndef TKZ_DEF_MINB
#define TKZ_DEF_MINB 4
#endif
template <bool COMPACT>
__global__ __launch_bounds__(256, TKZ_DEF_MINB) void k_bpe_deferred(DevTables T, const uint8_t* __restrict__ bytes, uint64_t limit,
                                                      Scratch S, Deferred D) {
    __shared__ uint32_t byte_id[256];
    byte_id[threadIdx.x] = T.byte_id[threadIdx.x];
    __syncthreads();
    const uint64_t* list = T.dedup ? D.olist : D.list;
    const uint64_t n = D.cnt[T.dedup ? 1 : 0];
    // Each block takes 256 entries at a time and counting-sorts them by byte length, so
    // each wave gets words of similar length: a wave runs as many merge rounds as its
    // longest word needs, and lengths across 16 / 32 bytes take different code paths.
    __shared__ uint64_t se[256];
    __shared__ uint32_t hist[36];
    constexpr uint32_t KEYS = 35;  // L 0..32, longer (33), padding (34)
    for (uint64_t base = (uint64_t)blockIdx.x * 256; base < n; base += (uint64_t)gridDim.x * 256) {
        const uint64_t i = base + threadIdx.x;
        const uint64_t e0 = i < n ? list[i] : 0ull;
        const uint32_t L0 = (uint32_t)(e0 >> LEN_SHIFT);
        const uint32_t key = i < n ? min(L0, 33u) : 34u;
        if (threadIdx.x < KEYS) hist[threadIdx.x] = 0;
        __syncthreads();
        const uint32_t r = atomicAdd(&hist[key], 1u);
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t o = 0;
            for (uint32_t k = 0; k < KEYS; ++k) { const uint32_t c = hist[k]; hist[k] = o; o += c; }
        }
        __syncthreads();
        se[hist[key] + r] = e0;
        __syncthreads();
        const bool valid = base + threadIdx.x < n;  // the padding sorts last
        const uint64_t e = valid ? se[threadIdx.x] : 0ull;
        __syncthreads();  // se / hist are rewritten by the next round
        const uint64_t pos = e & POS_MASK;
        const uint64_t ws = S.slot(pos, (uint32_t)(e >> POS_BITS) & ORD_MASK);
        uint32_t L = (uint32_t)(e >> LEN_SHIFT);
        if (L == LEN_ESC) L = S.prs()[pos];
#if TKZ_ABLATE == 1
        if (valid) S.narrow(ws, pos, 0);
        continue;
#endif
        // words of > LONG_WORD bytes: one wavefront each in k_bpe_long (appended 64 at a time)
        const bool lg = L > LONG_WORD;
        const uint64_t lm = __ballot(lg);
        if (lm) {
            const int leader = __ffsll((unsigned long long)lm) - 1;
            uint32_t lb = 0;
            if ((int)(threadIdx.x & 63) == leader) lb = atomicAdd(D.lcnt, (uint32_t)__popcll(lm));
            lb = (uint32_t)__shfl((int)lb, leader, 64);
            if (lg) D.llist[lb + __builtin_amdgcn_mbcnt_hi((uint32_t)(lm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)lm, 0))] = e;
        }
        const bool lit = valid && !lg && (T.chain || L > 32);
        if (lit) bpe_long_word<COMPACT>(T, byte_id, bytes, pos, ws, L, S);
        // register BPE: each width with the wave converged (chunk_commit)
        const bool r2 = valid && !lg && !lit && L <= 16, r4 = valid && !lg && !lit && L > 16;
        if (__ballot(r2)) bpe_bucket_word<16, 2, COMPACT>(T, byte_id, bytes, limit, pos, ws, L, S, r2);
        if (__ballot(r4)) bpe_bucket_word<16, 4, COMPACT>(T, byte_id, bytes, limit, pos, ws, L, S, r4);
    }
}

// k_bpe_short: the memo misses of <= 8 B that k_encode_blk leaves (round 6), listed per
// chunk (chunk c's at slist[c << ch_log2 ..], D.scnt[c] of them). Persistent waves take
// chunks c_first + wave + k * waves, sort the entries into two length-bucket LDS queues
// (<= 4 B: 4-symbol register BPE, 5..8 B: 8 symbols: bpe.zig:213-253 rounds) and run a
// bucket when 64 wait, one lane per word; results go to the chunks' dense areas
// (chunk_commit). The old k_encode ran these queues inside the scan kernel, whose register
// budget they set; here the scan kernel keeps its registers for resident waves.
template <bool COMPACT>
__global__ __launch_bounds__(256) void k_bpe_short(DevTables T, const uint8_t* __restrict__ bytes, uint64_t limit,
                                                   Scratch S, Deferred D, uint64_t c_first, uint64_t c_end,
                                                   uint32_t ch_log2) {
    __shared__ uint64_t q[256 / WAVE][2][QCAP];
    const int lane = lane_id(), wv = (int)(threadIdx.x >> 6);
    const uint64_t nwv = (uint64_t)gridDim.x * (256 / WAVE);
    uint32_t qn0 = 0, qn1 = 0;
    auto run = [&](int b, uint32_t qb, uint32_t take) {
        const bool act = (uint32_t)lane < take;
        const uint64_t e = act ? q[wv][b][qb + lane] : 0ull;
        const uint64_t pos = e & POS_MASK;
        const uint64_t ws = S.slot(pos, (uint32_t)(e >> POS_BITS) & ORD_MASK);
        const uint32_t L = (uint32_t)(e >> LEN_SHIFT);
        if (b == 0) bpe_bucket_word<4, 1, COMPACT>(T, T.byte_id, bytes, limit, pos, ws, L, S, act);
        else bpe_bucket_word<8, 1, COMPACT>(T, T.byte_id, bytes, limit, pos, ws, L, S, act);
    };
    for (uint64_t c = c_first + (uint64_t)blockIdx.x * (256 / WAVE) + (uint64_t)wv; c < c_end; c += nwv) {
        const uint32_t n = D.scnt[c];
        const uint64_t* src = D.slist + (c << ch_log2);
        for (uint32_t j = 0; j < n; j += WAVE) {
            const bool act = j + (uint32_t)lane < n;
            const uint64_t e = act ? src[j + lane] : 0ull;
            const uint32_t L = (uint32_t)(e >> LEN_SHIFT);
            if (T.chain) {  // a new_id == first merge: the literal loop
                if (act) bpe_long_word<COMPACT>(T, T.byte_id, bytes, e & POS_MASK,
                                                S.slot(e & POS_MASK, (uint32_t)(e >> POS_BITS) & ORD_MASK), L, S);
                continue;
            }
            const uint64_t m0 = __ballot(act && L <= 4u), m1 = __ballot(act && L > 4u);
            if (act && L <= 4u) q[wv][0][qn0 + lanes_below(m0)] = e;
            if (act && L > 4u) q[wv][1][qn1 + lanes_below(m1)] = e;
            qn0 += (uint32_t)__popcll(m0);
            qn1 += (uint32_t)__popcll(m1);
            WAVE_SYNC();
            if (qn0 >= (uint32_t)WAVE) { qn0 -= WAVE; run(0, qn0, WAVE); }
            if (qn1 >= (uint32_t)WAVE) { qn1 -= WAVE; run(1, qn1, WAVE); }
            WAVE_SYNC();
        }
    }
    if (qn0) run(0, 0, qn0);
    if (qn1) run(1, 0, qn1);
}

// ---------------------------------------------------------------------------
// k_bpe_long: wave-cooperative BPE.tokenize (bpe.zig:173-263) for pretokens of more than
// LONG_WORD bytes -- one wavefront per word. Such words are what a BPE tokenizer.json with
// an unrecognised pre_tokenizer (ByteLevel, Metaspace, Sequence, ...) produces: the whole
// normalized text is ONE pretoken (config.zig:387-402, lib.zig:121), and the reference's
// merge loop is O(rounds x n) over it.
//
// Exact restatement of the reference's rounds. Symbols keep their initial index q (the
// codepoint slices that have an id, bpe.zig:186-211); a merge rewrites sym[q] and unlinks
// its right partner j from a doubly linked list (nxt / prv; prv[j] = TOMB marks it dead),
// so no array is compacted per round. pr[q] caches the merge value of the pair (q, nxt[q])
// (NONE: no merge / no right partner). Lane l owns a contiguous range of positions, split
// in sub-blocks of SB positions whose minima (smin) are kept, and holds the minimum of
// its own sub-blocks in a register. A round:
//   1. best = wave minimum (DPP) of the lane minima; NONE ends the word (bpe.zig:232);
//   2. candidates = positions with pr == best (ranks are unique per pair: bpe.zig:265-270
//      accepts each (a,b) once, a later duplicate overwrites it), found in the sub-blocks
//      whose minimum is best;
//   3. merges: a != b: every candidate merges (occurrences cannot overlap) -- in parallel;
//      a == b: greedily left to right, a candidate merges unless its left live neighbour
//      just did (bpe.zig:240-252's replace-and-retest); new_id == a (a chain): after each
//      merge the following b's are absorbed too (the retest at the same i). Both walk the
//      candidates in position order, lane by lane;
//   4. the merged positions and their left neighbours are re-probed (one memory round trip
//      for the whole round), and the touched sub-blocks / lane minima recomputed.
// Words of <= LW bytes live in LDS (7.5 KB per wave); longer words use their own scratch
// at the word's byte offset (sym: ids, pr: prs, nxt / prv: offs, st: tok; 20 B per byte)
// with sub-block minima in LDS. Output: wide tokens at ids/offs[pos..] (S.wide).
// ---------------------------------------------------------------------------
constexpr int LW = 512;            // LDS-resident words: <= LW bytes (so <= LW symbols)
constexpr int NSBMAX = 512;        // sub-blocks of a scratch-resident word (minima in LDS)

struct LongSmem {
    union {
        struct {  // LDS-resident word
            uint32_t sym[LW];
            uint32_t pr[LW];
            uint16_t nxt[LW];
            uint16_t prv[LW];
            uint8_t pf[LW];        // the pair of pr[q] is (a, a) or a chain merge: serial round
        } w;
        uint32_t smin[NSBMAX];     // scratch-resident word: sub-block minima
    } u;
    uint8_t dsb[NSBMAX];           // sub-block (LDS word: lane) touched this round
};

struct LdsWord {
    // st_: the initial symbols' byte offsets, in the word's own tok scratch (global: read
    // only at the output; 1 KB less LDS per word = 20 resident words per CU instead of 18)
    uint32_t* sym; uint32_t* pr; uint16_t* nx; uint16_t* pv; uint32_t* st_;
    static constexpr uint32_t NIL = 0xFFFFu, TOMB = 0xFFFEu;
    __device__ __forceinline__ uint32_t nxt(uint32_t q) const { return nx[q]; }
    __device__ __forceinline__ uint32_t prv(uint32_t q) const { return pv[q]; }
    __device__ __forceinline__ uint32_t st(uint32_t q) const { return st_[q]; }
    __device__ __forceinline__ void set_nxt(uint32_t q, uint32_t v) const { nx[q] = (uint16_t)v; }
    __device__ __forceinline__ void set_prv(uint32_t q, uint32_t v) const { pv[q] = (uint16_t)v; }
    __device__ __forceinline__ void set_st(uint32_t q, uint32_t v) const { st_[q] = v; }
};
struct GlbWord {
    uint32_t* sym; uint32_t* pr; uint32_t* nx; uint32_t* pv; uint32_t* st_;
    static constexpr uint32_t NIL = 0xFFFFFFFFu, TOMB = 0xFFFFFFFEu;
    __device__ __forceinline__ uint32_t nxt(uint32_t q) const { return nx[q]; }
    __device__ __forceinline__ uint32_t prv(uint32_t q) const { return pv[q]; }
    __device__ __forceinline__ uint32_t st(uint32_t q) const { return st_[q]; }
    __device__ __forceinline__ void set_nxt(uint32_t q, uint32_t v) const { nx[q] = v; }
    __device__ __forceinline__ void set_prv(uint32_t q, uint32_t v) const { pv[q] = v; }
    __device__ __forceinline__ void set_st(uint32_t q, uint32_t v) const { st_[q] = v; }
};

// wave minimum of a u32, the same DPP ladder as wave_incl_scan (lane 63 holds it)
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)NONE, (int)v, 0x111, 0xF, 0xF, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)NONE, (int)v, 0x112, 0xF, 0xF, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)NONE, (int)v, 0x114, 0xF, 0xF, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)NONE, (int)v, 0x118, 0xF, 0xF, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)NONE, (int)v, 0x142, 0xA, 0xF, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)NONE, (int)v, 0x143, 0xC, 0xF, false));
    return lane63(v);
}
__device__ __forceinline__ uint32_t lane_mbcnt(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
}

// byte length of the symbol starting at word offset s (Utf8Iterator slice, clamped at L)
__device__ __forceinline__ uint32_t sym_len(const uint8_t* wb, uint32_t s, uint32_t L) {
    const uint32_t k = seq_len(wb[s]);  // lowercasing never changes a byte's class
    return s + k > L ? L - s : k;
}

// Initial symbols: the codepoint slices of the word that have an id (bpe.zig:186-211),
// sym[] / st[] in slice order. Returns n. Parallel when the word is well-formed UTF-8
// (every slice starts at a non-continuation byte and ends where the next one starts);
// otherwise lane 0 slices it sequentially (the reference's Utf8Iterator order).
template <class WS>
__device__ uint32_t long_init(const DevTables& T, const uint32_t* byte_id, const uint8_t* bytes, uint64_t pos,
                              uint64_t limit, uint32_t L, const WS& w) {
    const int lane = lane_id();
    const uint8_t* wb = bytes + pos;
    bool ok = true;
    uint32_t n = 0;
    for (uint32_t b0 = 0; b0 < L && ok; b0 += GROUP) {
        WordBytes<2> v;  // this lane's 8 bytes + 8 of lookahead
        const uint32_t o = b0 + 8u * (uint32_t)lane;
        v.load(bytes, pos + o, limit, T.norm);
        const uint32_t nv = o < L ? min(L - o, 8u) : 0u;  // valid bytes of this lane
        uint32_t start = 0, bad = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if ((uint32_t)j >= nv) break;
            const uint32_t c = v.at(j);
            if ((c & 0xC0u) == 0x80u) {
                if (o + (uint32_t)j == 0) bad = 1;  // a word starting with a continuation byte
                continue;
            }
            start |= 1u << j;
            const uint32_t k = seq_len(c);
            if (k > 1) {
                if (o + (uint32_t)j + k > L) bad = 1;  // truncated at the word end
#pragma unroll
                for (int t = 1; t < 4; ++t)
                    if ((uint32_t)t < k && (v.at(j + t) & 0xC0u) != 0x80u) bad = 1;
            } else if (c >= 0x80u) {
                bad = 1;  // invalid lead byte (F8..FF): 1-byte slice, sequential path
            }
            // the byte after the slice must not be a continuation byte (the reference's
            // iterator would slice it on its own there: a stray continuation byte)
            if (o + (uint32_t)j + k < L && (v((uint32_t)j + k) & 0xC0u) == 0x80u) bad = 1;
        }
        if (__ballot(bad) != 0ull) { ok = false; break; }
        // ids of this lane's slices; dropped chars (no id, no unk) are not symbols
        uint32_t ids[8];
        uint32_t keep = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            ids[j] = NONE;
            if ((start >> j) & 1u) {
                const uint32_t c = v.at(j);
                const uint32_t k = seq_len(c);
                uint32_t packed = c;
#pragma unroll
                for (int t = 1; t < 4; ++t)
                    if ((uint32_t)t < k) packed |= v.at(j + t) << (8 * t);
                ids[j] = char_id(T, byte_id, c, packed, k);
                if (ids[j] != NONE) keep |= 1u << j;
            }
        }
        const uint32_t cnt = (uint32_t)__popc(keep);
        const uint32_t inc = (uint32_t)wave_incl_scan((int)cnt);
        uint32_t q = n + inc - cnt;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if ((keep >> j) & 1u) {
                w.sym[q] = ids[j];
                w.set_st(q, o + (uint32_t)j);
                ++q;
            }
        }
        n += lane63(inc);
    }
    if (!ok) {  // sequential slicing (lane 0)
        n = 0;
        if (lane == 0) {
            for (uint32_t p = 0; p < L;) {
                const uint32_t b0 = lower(wb[p], T.norm);
                uint32_t len = seq_len(b0);
                if (p + len > L) len = L - p;
                uint32_t packed = b0;
                for (uint32_t j = 1; j < len; ++j) packed |= lower(wb[p + j], T.norm) << (8 * j);
                const uint32_t id = char_id(T, byte_id, b0, packed, len);
                if (id != NONE) { w.sym[n] = id; w.set_st(n, p); ++n; }
                p += len;
            }
        }
        n = rfl(n);
    }
    return n;
}

// merge value of the pair (x, y): COMPACT rank<<16|new_id, else the rank
template <bool COMPACT>
__device__ __forceinline__ uint32_t long_pair(const DevTables& T, uint32_t x, uint32_t y) {
    return pair_value<COMPACT>(T, x, y);
}

// One word: rounds until no pair merges, then the tokens to ids/offs[pos..] (wide).
template <bool COMPACT, class WS>
__device__ void long_word(const DevTables& T, const uint32_t* byte_id, const uint8_t* bytes, uint64_t pos,
                          uint64_t ws, uint64_t limit, uint32_t L, const WS& w, uint32_t* smin, uint8_t* dsb,
                          const Scratch& S) {
    constexpr uint32_t NIL = WS::NIL, TOMB = WS::TOMB;
    const int lane = lane_id();
    const uint32_t n = long_init(T, byte_id, bytes, pos, limit, L, w);
    WAVE_SYNC();
    // links and the initial pair values (4 probes per lane in flight)
    for (uint32_t q = lane; q < n; q += WAVE) {
        w.set_nxt(q, q + 1 < n ? q + 1 : NIL);
        w.set_prv(q, q > 0 ? q - 1 : NIL);
    }
    for (uint32_t q0 = 0; q0 < n; q0 += 4 * WAVE) {
        uint32_t v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t q = q0 + (uint32_t)(k * WAVE + lane);
            v[k] = q + 1 < n ? long_pair<COMPACT>(T, w.sym[q], w.sym[q + 1]) : NONE;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t q = q0 + (uint32_t)(k * WAVE + lane);
            if (q < n) w.pr[q] = v[k];
        }
    }
    // sub-blocks: SB positions each, NSB of them, B per lane (lane l: [l*B, l*B + B))
    const bool lds = smin == w.pr;  // LDS word: one position per sub-block, smin aliases pr
    const uint32_t SB = lds ? 1u : max(1u, (n + NSBMAX - 1) / NSBMAX);
    const uint32_t NSB = (n + SB - 1) / SB;
    const uint32_t B = (NSB + WAVE - 1) / WAVE;
    const uint32_t s_lo = min((uint32_t)lane * B, NSB), s_hi = min(s_lo + B, NSB);
    WAVE_SYNC();
    for (uint32_t s = lane; s < NSB; s += WAVE) {
        if (!lds) {
            uint32_t m = NONE;
            for (uint32_t q = s * SB; q < min(n, s * SB + SB); ++q) m = min(m, w.pr[q]);
            smin[s] = m;
        }
        dsb[s] = 0;
    }
    WAVE_SYNC();
    uint32_t lm = NONE;
    for (uint32_t s = s_lo; s < s_hi; ++s) lm = min(lm, smin[s]);

    // ---- merge rounds (bpe.zig:214-253) ----
    while (n > 1) {
        const uint32_t best = wave_min_u32(lm);
        if (best == NONE) break;
        const uint64_t mb = __ballot(lm == best);
        const int fl = __ffsll((unsigned long long)mb) - 1;
        // the pair (a, b) of best: from the first candidate
        uint32_t a = 0, b = 0;
        if (lane == fl) {
            for (uint32_t s = s_lo; s < s_hi; ++s) {
                if (smin[s] != best) continue;
                uint32_t q = s * SB;
                while (w.pr[q] != best) ++q;
                a = w.sym[q];
                b = w.sym[w.nxt(q)];
                break;
            }
        }
        a = (uint32_t)__builtin_amdgcn_readlane((int)a, fl);
        b = (uint32_t)__builtin_amdgcn_readlane((int)b, fl);
        uint32_t X;
        if (COMPACT) {
            X = best & 0xFFFFu;
        } else {
            uint32_t r;
            merge_probe_wide(T.mtab_w, T.m_bits, a, b, r, X);
        }
        const bool chain = X == a;  // new_id == first: the retest at i absorbs the following b's
        const bool serial = chain || a == b;
        const bool mine = lm == best;
        // unlinks j = nxt(q) from the list (q keeps the merged symbol)
        auto unlink_next = [&](uint32_t q) {
            const uint32_t j = w.nxt(q), nj = w.nxt(j);
            w.set_nxt(q, nj);
            if (nj != NIL) w.set_prv(nj, q);
            w.set_prv(j, TOMB);
            w.pr[j] = NONE;
            dsb[j / SB] = 1;
        };
        if (!serial) {
            if (mine) {
                for (uint32_t s = s_lo; s < s_hi; ++s) {
                    if (smin[s] != best) continue;
                    for (uint32_t q = s * SB; q < min(n, s * SB + SB); ++q) {
                        if (w.pr[q] != best) continue;
                        w.sym[q] = X;
                        unlink_next(q);
                        w.pr[q] = DIRTY;
                        dsb[s] = 1;
                    }
                }
            }
        } else {
            // in position order, lane by lane, each lane its candidates ascending: a
            // candidate consumed by an earlier merge of the round is dead (TOMB, pr NONE);
            // any other still holds (a, b) and merges (for a == b that is r, r+2, ... of a
            // run); with a chain the merged symbol absorbs the b's that follow it
            for (uint64_t m = mb; m; m &= m - 1) {
                const int ll = __ffsll((unsigned long long)m) - 1;
                if (lane == ll) {
                    for (uint32_t s = s_lo; s < s_hi; ++s) {
                        if (smin[s] != best) continue;
                        for (uint32_t q = s * SB; q < min(n, s * SB + SB); ++q) {
                            if (w.pr[q] != best || w.prv(q) == TOMB) continue;
                            dsb[s] = 1;
                            w.pr[q] = DIRTY;
                            if (w.sym[q] != a || w.nxt(q) == NIL || w.sym[w.nxt(q)] != b) continue;  // (re-probed)
                            w.sym[q] = X;
                            unlink_next(q);
                            if (chain)
                                while (w.nxt(q) != NIL && w.sym[w.nxt(q)] == b) unlink_next(q);
                        }
                    }
                }
                WAVE_SYNC();
            }
        }
        WAVE_SYNC();
        // re-probe every merged position (DIRTY; in the sub-blocks flagged this round) and
        // its live left neighbour
        if (mine) {
            for (uint32_t s = s_lo; s < s_hi; ++s) {
                if (!dsb[s]) continue;
                for (uint32_t q = s * SB; q < min(n, s * SB + SB); ++q) {
                    if (w.pr[q] != DIRTY) continue;
                    const uint32_t nq = w.nxt(q), pq = w.prv(q);
                    const uint32_t vq = nq != NIL ? long_pair<COMPACT>(T, w.sym[q], w.sym[nq]) : NONE;
                    const uint32_t vp = pq != NIL ? long_pair<COMPACT>(T, w.sym[pq], w.sym[q]) : NONE;
                    w.pr[q] = vq;
                    // a left neighbour that merged too (DIRTY) is its owner's to re-probe, with
                    // ITS left neighbour: overwriting it here would hide that second pair
                    if (pq != NIL && w.pr[pq] != DIRTY) {
                        w.pr[pq] = vp;
                        dsb[pq / SB] = 1;
                    }
                }
            }
        }
        WAVE_SYNC();
        // touched sub-blocks -> minima; lane minima
        bool ch = false;
        for (uint32_t s = s_lo; s < s_hi; ++s) {
            if (!dsb[s]) continue;
            dsb[s] = 0;
            ch = true;
            if (!lds) {
                uint32_t m = NONE;
                for (uint32_t q = s * SB; q < min(n, s * SB + SB); ++q) m = min(m, w.pr[q]);
                smin[s] = m;
            }
        }
        if (ch) {
            lm = NONE;
            for (uint32_t s = s_lo; s < s_hi; ++s) lm = min(lm, smin[s]);
        }
        WAVE_SYNC();
    }

    // ---- output (bpe.zig:255-262): live positions in order, wide tokens at pos ----
    const uint32_t q_lo = min(s_lo * SB, n), q_hi = min(s_hi * SB, n);
    uint32_t live = 0;
    for (uint32_t q = q_lo; q < q_hi; ++q) live += (n == 1 || w.prv(q) != TOMB) ? 1u : 0u;
    const uint32_t inc = (uint32_t)wave_incl_scan((int)live);
    const uint32_t c = lane63(inc);
    const uint32_t k0 = inc - live;
    uint32_t* const ids = S.ids() + pos;
    uint64_t* const offs = S.offs() + pos;
    const uint8_t* wb = bytes + pos;
    auto tok_end = [&](uint32_t q) {
        const uint32_t nq = w.nxt(q);
        const uint32_t last = nq == NIL ? n - 1 : nq - 1;
        const uint32_t s0 = w.st(last);
        return s0 + sym_len(wb, s0, L);
    };
    if (lds) {
        uint32_t k = k0;
        for (uint32_t q = q_lo; q < q_hi; ++q) {
            if (n != 1 && w.prv(q) == TOMB) continue;
            ids[k] = w.sym[q];
            offs[k] = (uint64_t)w.st(q) | ((uint64_t)tok_end(q) << 32);
            ++k;
        }
    } else {
        // the word's own scratch is both the work arrays and the output: four passes,
        // each writing a region the pass does not read (sym = ids, pr = prs, nxt / prv =
        // offs, st = tok)
        // pass A: pr = the token end of a live position, NONE for a dead one (the live
        // flag of the later passes: offs, which holds prv, is overwritten by pass B)
        for (uint32_t q = q_lo; q < q_hi; ++q) w.pr[q] = (n == 1 || w.prv(q) != TOMB) ? tok_end(q) : NONE;
        WAVE_SYNC();
        uint32_t k = k0;
        for (uint32_t q = q_lo; q < q_hi; ++q)
            if (w.pr[q] != NONE) { offs[k] = (uint64_t)w.st(q) | ((uint64_t)w.pr[q] << 32); ++k; }
        WAVE_SYNC();
        uint32_t* tmp = S.tok() + pos;  // = st, free now
        k = k0;
        for (uint32_t q = q_lo; q < q_hi; ++q)
            if (w.pr[q] != NONE) tmp[k++] = w.sym[q];
        WAVE_SYNC();
        for (uint32_t k2 = lane; k2 < c; k2 += WAVE) ids[k2] = tmp[k2];
    }
    WAVE_SYNC();
    if (lane == 0) S.wide(ws, pos, c);
}

// Flag of a pair for the serial rounds: (a, a), or a merge whose new id is a (a chain).
// Wide tables carry no new id in the cached value: with a chain merge anywhere, every
// round of a wide table is serial.
template <bool COMPACT>
__device__ __forceinline__ uint32_t long_flag(const DevTables& T, uint32_t x, uint32_t y, uint32_t v) {
    if (v == NONE) return 0;
    return (x == y || (T.chain && (COMPACT ? (v & 0xFFFFu) == x : true))) ? 1u : 0u;
}

// LDS-resident words (<= LW bytes, so n <= 512): lane l owns positions [l*B, l*B + B),
// B = ceil(n / 64) <= 8, and caches their merge values in registers, so the minimum and
// the candidates of a round cost no LDS round trip. The LDS copy pr[] is what the other
// lanes read and write; a lane whose positions another lane touched (a partner unlinked,
// a left neighbour re-probed) reloads its cache (8 independent reads).
template <bool COMPACT>
__device__ void long_word_lds(const DevTables& T, const uint8_t* bytes, uint64_t pos, uint64_t ws, uint64_t limit,
                              uint32_t L, LongSmem& sm, const Scratch& S, unsigned long long* dbg) {
#ifdef TKZ_LONG_STATS  // debug: s_memtime per section, rounds, accepted speculative ranks
    uint64_t lt0 = __builtin_amdgcn_s_memtime(), lt_init = 0, lt_rounds = 0, lt_probe = 0, n_rounds = 0, n_spec = 0;
#else
    (void)dbg;
#endif
    constexpr uint32_t NIL = LdsWord::NIL, TOMB = LdsWord::TOMB;
    constexpr int KB = LW / WAVE;
    const int lane = lane_id();
    LdsWord w{sm.u.w.sym, sm.u.w.pr, sm.u.w.nxt, sm.u.w.prv, S.tok() + pos};
    uint8_t* pf = sm.u.w.pf;
    uint8_t* ldirty = sm.dsb;
    const uint32_t n = long_init(T, T.byte_id, bytes, pos, limit, L, w);
    WAVE_SYNC();
    for (uint32_t q = lane; q < n; q += WAVE) {
        w.set_nxt(q, q + 1 < n ? q + 1 : NIL);
        w.set_prv(q, q > 0 ? q - 1 : NIL);
    }
    for (uint32_t q0 = 0; q0 < n; q0 += 4 * WAVE) {
        uint32_t v[4], x[4], y[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t q = q0 + (uint32_t)(k * WAVE + lane);
            x[k] = q + 1 < n ? w.sym[q] : 0u;
            y[k] = q + 1 < n ? w.sym[q + 1] : 0u;
            v[k] = q + 1 < n ? long_pair<COMPACT>(T, x[k], y[k]) : NONE;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t q = q0 + (uint32_t)(k * WAVE + lane);
            if (q < n) {
                w.pr[q] = v[k];
                pf[q] = (uint8_t)long_flag<COMPACT>(T, x[k], y[k], v[k]);
            }
        }
    }
    const uint32_t B = (n + WAVE - 1) / WAVE;
    const uint32_t q_lo = min((uint32_t)lane * B, n), q_hi = min(q_lo + B, n);
    ldirty[lane] = 0;
    WAVE_SYNC();
    uint32_t prc[KB];
    auto reload = [&]() {
#pragma unroll
        for (int k = 0; k < KB; ++k) {
            const uint32_t q = q_lo + (uint32_t)k;
            const bool in = q < q_hi;
            prc[k] = in ? w.pr[q] : NONE;
        }
    };
    reload();
    auto lane_min = [&]() {
        uint32_t m = NONE;
#pragma unroll
        for (int k = 0; k < KB; ++k) m = min(m, prc[k]);
        return m;
    };
    uint32_t lm = lane_min();
#ifdef TKZ_LONG_STATS
    { const uint64_t t = __builtin_amdgcn_s_memtime(); lt_init = t - lt0; lt0 = t; }
#endif

    // ---- merge rounds (bpe.zig:214-253) ----
    // Speculative second rank (TKZ_LONG_SPEC): with r1 the round's minimum and r2 the next
    // smaller value among the live pairs, the reference's next round merges every
    // occurrence of r2 exactly when (a) no r2 occurrence shares a symbol with, or neighbours,
    // an r1 merge (its pair and its neighbours' symbols are then what they were), and (b)
    // every pair the r1 merges create ranks above r2. Both pairs an r2 merge would create
    // are probed in the same memory round trip as r1's; (a) is checked before, (b) after,
    // and the r2 merges are applied only when both hold -- so a round that passes does two
    // of the reference's rounds (C6 docs: 184 -> 102 rounds). Simple pairs only (a != b, no
    // chain), at most one r2 occurrence per lane, compact tables.
    while (n > 1) {
        const uint32_t best = wave_min_u32(lm);
        if (best == NONE) break;
        uint32_t cm = 0;
#pragma unroll
        for (int k = 0; k < KB; ++k) cm |= (prc[k] == best) ? (1u << k) : 0u;
        const uint64_t mb = __ballot(cm != 0);
        const int fl = __ffsll((unsigned long long)mb) - 1;
        // (a, a) or chain pair: every candidate has the same pair, its flag from one of them
        uint32_t fl_own = 0;
        if (lane == fl) fl_own = pf[q_lo + (uint32_t)__builtin_ctz(cm)];
        const bool serial = __builtin_amdgcn_readlane((int)fl_own, fl) != 0;
        uint32_t r2 = NONE, c2m = 0;
        bool spec = false;
#if TKZ_LONG_SPEC
        if (COMPACT && !serial) {
            uint32_t m2 = NONE;
#pragma unroll
            for (int k = 0; k < KB; ++k) m2 = min(m2, prc[k] != best ? prc[k] : NONE);
            r2 = wave_min_u32(m2);
            if (r2 != NONE) {
#pragma unroll
                for (int k = 0; k < KB; ++k) c2m |= (prc[k] == r2) ? (1u << k) : 0u;
                const bool f2 = c2m != 0u && pf[q_lo + (uint32_t)__builtin_ctz(c2m)] != 0;
                spec = __ballot(f2 || __popc(c2m) > 1) == 0ull;
            }
        }
#endif
        uint32_t X = best & 0xFFFFu, a = 0, b = 0;
        if (serial || !COMPACT) {  // the pair (a, b): from the first candidate
            if (lane == fl) {
                const uint32_t q0 = q_lo + (uint32_t)__builtin_ctz(cm);
                a = w.sym[q0];
                b = w.sym[w.nxt(q0)];
            }
            a = (uint32_t)__builtin_amdgcn_readlane((int)a, fl);
            b = (uint32_t)__builtin_amdgcn_readlane((int)b, fl);
            if (!COMPACT) {
                uint32_t r;
                merge_probe_wide(T.mtab_w, T.m_bits, a, b, r, X);
            }
        }
        const bool chain = serial && X == a;
        auto unlink_next = [&](uint32_t q) {
            const uint32_t j = w.nxt(q), nj = w.nxt(j);
            w.set_nxt(q, nj);
            if (nj != NIL) w.set_prv(nj, q);
            w.set_prv(j, TOMB);
            w.pr[j] = NONE;
            ldirty[j / B] = 1;
        };
        uint32_t mm = 0;  // this lane's positions merged (or re-probed) this round
        if (!serial) {
            for (uint32_t m = cm; m; m &= m - 1) {
                const uint32_t k = (uint32_t)__builtin_ctz(m), q = q_lo + k;
                w.sym[q] = X;
                unlink_next(q);
                w.pr[q] = DIRTY;
                mm |= 1u << k;
            }
        } else {
            for (uint64_t m = mb; m; m &= m - 1) {
                const int ll = __ffsll((unsigned long long)m) - 1;
                if (lane == ll) {
                    for (uint32_t mc = cm; mc; mc &= mc - 1) {
                        const uint32_t k = (uint32_t)__builtin_ctz(mc), q = q_lo + k;
                        if (w.prv(q) == TOMB) continue;  // consumed by an earlier merge of the round
                        w.pr[q] = DIRTY;
                        mm |= 1u << k;
                        if (w.sym[q] != a || w.nxt(q) == NIL || w.sym[w.nxt(q)] != b) continue;
                        w.sym[q] = X;
                        unlink_next(q);
                        if (chain)
                            while (w.nxt(q) != NIL && w.sym[w.nxt(q)] == b) unlink_next(q);
                    }
                }
                WAVE_SYNC();
            }
        }
        WAVE_SYNC();
        // the speculative r2, (a): its occurrence (at most one per lane) isolated from this
        // round's merges -- the merged positions are DIRTY and their consumed partners TOMB
        // until the re-probes below; its neighbours' symbols read now as well
        const uint32_t X2 = r2 & 0xFFFFu;
        uint32_t c2 = 0, pc2 = NIL, sR2 = 0, sL2 = 0;
        bool hasR2 = false, hasL2 = false;
        if (spec) {
            bool bad = false;
            if (c2m) {
                c2 = q_lo + (uint32_t)__builtin_ctz(c2m);
                const uint32_t j2 = w.nxt(c2);
                pc2 = w.prv(c2);
                const uint32_t nj2 = j2 != NIL && j2 != TOMB ? w.nxt(j2) : NIL;
                bad = pc2 == TOMB || j2 == NIL || w.pr[j2] == DIRTY || (pc2 != NIL && w.pr[pc2] == DIRTY) ||
                      (nj2 != NIL && w.pr[nj2] == DIRTY);
                hasR2 = nj2 != NIL;
                sR2 = hasR2 ? (w.pr[nj2] == r2 ? X2 : w.sym[nj2]) : 0u;
                // the left pair belongs to the r2 occurrence before, if pc2 is its partner
                const uint32_t ppc = pc2 != NIL && pc2 != TOMB ? w.prv(pc2) : NIL;
                hasL2 = pc2 != NIL && !(ppc != NIL && ppc != TOMB && w.pr[ppc] == r2);
                sL2 = hasL2 ? w.sym[pc2] : 0u;
            }
            spec = __ballot(bad) == 0ull;
        }
        WAVE_SYNC();  // the (a) reads before the re-probes' writes
        // re-probe each merged position and its live left neighbour (unless that one
        // merged too: its owner re-probes it, with ITS left neighbour)
        uint32_t nmin = NONE;  // the smallest value among the pairs this lane's merges created
#ifdef TKZ_LONG_STATS
        const uint64_t tp0 = __builtin_amdgcn_s_memtime();
        ++n_rounds;
#endif
        for (uint32_t m = mm; m; m &= m - 1) {
            const uint32_t q = q_lo + (uint32_t)__builtin_ctz(m);
            const uint32_t nq = w.nxt(q), pq = w.prv(q), sq = w.sym[q];
            const uint32_t sn = nq != NIL ? w.sym[nq] : 0u, sp = pq != NIL ? w.sym[pq] : 0u;
            const uint32_t vq = nq != NIL ? long_pair<COMPACT>(T, sq, sn) : NONE;
            const uint32_t vp = pq != NIL ? long_pair<COMPACT>(T, sp, sq) : NONE;
            w.pr[q] = vq;
            pf[q] = (uint8_t)long_flag<COMPACT>(T, sq, sn, vq);
            nmin = min(nmin, vq);
            if (pq != NIL && w.pr[pq] != DIRTY) {
                w.pr[pq] = vp;
                pf[pq] = (uint8_t)long_flag<COMPACT>(T, sp, sq, vp);
                ldirty[pq / B] = 1;
                nmin = min(nmin, vp);
            }
        }
        // (b): every pair the r1 merges created ranks above r2; then the r2 merges (the
        // kernel is VALU-issue bound, not latency bound: their probes take a round trip of
        // their own, only in rounds that pass (a))
        if (spec) spec = wave_min_u32(nmin) > r2;
        if (spec && c2m) {
            const uint32_t vr = hasR2 ? long_pair<COMPACT>(T, X2, sR2) : NONE;
            const uint32_t vl = hasL2 ? long_pair<COMPACT>(T, sL2, X2) : NONE;
            w.sym[c2] = X2;
            unlink_next(c2);
            w.pr[c2] = vr;
            pf[c2] = (uint8_t)long_flag<COMPACT>(T, X2, sR2, vr);
            if (hasL2) {
                w.pr[pc2] = vl;
                pf[pc2] = (uint8_t)long_flag<COMPACT>(T, sL2, X2, vl);
                ldirty[pc2 / B] = 1;
            }
        }
#ifdef TKZ_LONG_STATS
        lt_probe += __builtin_amdgcn_s_memtime() - tp0;
        n_spec += spec ? 1 : 0;
#endif
        if (mm || (spec && c2m)) ldirty[lane] = 1;
        WAVE_SYNC();
        if (ldirty[lane]) {
            ldirty[lane] = 0;
            reload();
            lm = lane_min();
        }
        WAVE_SYNC();
    }

#ifdef TKZ_LONG_STATS
    lt_rounds = __builtin_amdgcn_s_memtime() - lt0;
    if (lane == 0) {
        atomicAdd(&dbg[0], (unsigned long long)lt_init);
        atomicAdd(&dbg[1], (unsigned long long)lt_rounds);
        atomicAdd(&dbg[2], (unsigned long long)lt_probe);
        atomicAdd(&dbg[3], (unsigned long long)n_rounds);
        atomicAdd(&dbg[4], (unsigned long long)n_spec);
        atomicAdd(&dbg[5], 1ull);
    }
#endif
    // ---- output (bpe.zig:255-262): live positions in order, wide tokens at pos ----
    uint32_t live = 0;
    for (uint32_t q = q_lo; q < q_hi; ++q) live += (w.prv(q) != TOMB) ? 1u : 0u;
    const uint32_t inc = (uint32_t)wave_incl_scan((int)live);
    const uint32_t c = lane63(inc);
    uint32_t* const ids = S.ids() + pos;
    uint64_t* const offs = S.offs() + pos;
    const uint8_t* wb = bytes + pos;
    uint32_t k = inc - live;
    for (uint32_t q = q_lo; q < q_hi; ++q) {
        if (w.prv(q) == TOMB) continue;
        const uint32_t nq = w.nxt(q);
        const uint32_t last = nq == NIL ? n - 1 : nq - 1;
        const uint32_t s0 = w.st(last);
        ids[k] = w.sym[q];
        offs[k] = (uint64_t)w.st(q) | ((uint64_t)(s0 + sym_len(wb, s0, L)) << 32);
        ++k;
    }
    WAVE_SYNC();
    if (lane == 0) S.wide(ws, pos, c);
}

// ---------------------------------------------------------------------------
// Segmented long pretokens (BPE tables with compact ids, or wide ids < 2^20; no new_id ==
// first merge; tokenizers whose pre_tokenizer leaves the whole text as one pretoken).
//
// Under a ByteLevel / Metaspace / unknown pre_tokenizer the whole text is one pretoken
// (config.zig:387-402, lib.zig:121). It is cut into segments at three kinds of ASCII chars:
//   * dropped: no id and no unk token, BPE.tokenize skips them (bpe.zig:192-208) -- the
//     spaces and newlines of a vocab without such tokens vanish, leaving the words'
//     symbols adjacent;
//   * inert: the char's symbol (its id, or the unk id, bpe.zig:198-205) is in no merge on
//     either side, so no pair ever forms across it (the raw spaces of a SentencePiece vocab
//     with an unk token). An inert char is a segment of its own whose boundaries are never
//     crossed: no check;
//   * whitespace with a mergeable symbol: a cut before it, checked like the others.
// The reference's rounds (bpe.zig:214-253) over the whole symbol sequence are the rounds of
// the segments interleaved -- a round takes the global minimum, which is the minimum of
// every segment holding that pair -- until the first merge of a pair that straddles a cut.
//   * every group of segments (at first each segment alone) is encoded on its own,
//     recording per round its value and whether it changed the group's first / last
//     symbol (its profile);
//   * each boundary between adjacent groups G | H is checked by replaying the two profiles
//     in the reference's order (the smaller next round value first) against the pair
//     (last symbol of G, first symbol of H), re-probed whenever either changes: the
//     boundary is crossed iff at some point that pair's value is below both next round
//     values (a tie counts as crossed, which is always safe);
//   * crossed boundaries join their groups, which are encoded again and their boundaries
//     re-checked, until no boundary is crossed.
// Exactness: joining is always safe (a group is encoded exactly). When no boundary of the
// final groups is crossed in its two-group process, none is crossed in the whole: restrict
// the whole process to G and H up to its first straddling merge -- the other groups'
// rounds only interleave -- and that merge occurs in the G | H process too. So the result
// is the groups' results in order, with pretoken-relative offsets (tests/segment_model.py
// states the algorithm; tests/test_segments.py checks it against the reference loop).
//
// Flat kernels over all long pretokens of the pass -- one lane per group or boundary, as
// many waves as fit, so the short chains of dependent probes of each item overlap (one
// wave per pretoken iterating on its own was bound by those chains: ~86 round trips per
// 512-B doc at 3 waves per SIMD):
//   k_seg_init    wave per pretoken: UTF-8 check, segments, their records; a pretoken that
//                 does not qualify goes to D.flist (k_bpe_long)
//   k_seg_first   (with the segment memo) iteration 0: lane per segment, memo lookups, the
//                 boundaries between two hits checked from registers, misses listed
//   k_seg_enc     lane per listed group (iteration 0 without the memo: every segment),
//                 counting-sorted by length per block: register BPE with the round
//                 profile, W = 4 / 8 / 16 by the wave's longest group; larger groups listed
//   k_seg_enc_big lane per group of 17..32 symbols (W = 32); then the wave's groups of up
//                 to 64 symbols one at a time with the whole wave (more: the pretoken falls
//                 back)
//   k_seg_check   lane per encoded group: its right and left boundaries replayed
//                 (iteration 0 without the memo: each segment's right boundary)
//   k_seg_join    lane per crossed boundary's left head: the joined group's new end, listed
//                 for the next iteration
//   k_seg_count   wave per pretoken: its groups' token count to its word record (REC_SEG);
//                 a pretoken that failed goes to D.flist
//   k_seg_emit    (after the compaction) wave per pretoken: the groups' tokens in order
//                 straight to the output, at the position k_compact_long recorded (they
//                 were written to the scratch and copied from there: 1.3 GB each way on C6)
// List appends go through block-staged LDS lists (BlockList: one global atomic per flush).
// Up to SEG_ITERS iterations of enc / check / join (C6: 2.8 on average, 4 for 99 % of its
// 512-B docs; a 64-KB pretoken needs 3-5, so a 1-MB one would almost surely have failed at 4);
// the later ones run on a smaller grid and cost a launch each when nothing is left. A
// pretoken still joining after them falls back. k_bpe_long then runs on D.flist.
// In-pretoken offsets are 32-bit (segment records; a group's tokens hold offsets relative to
// the group's first byte, 16 bits each), so a pretoken of any length is segmented (round 5:
// <= 32,766 B, the 16-bit pretoken-relative token offsets).
// ---------------------------------------------------------------------------
#ifndef TKZ_SEG_ITERS
#define TKZ_SEG_ITERS 16
#endif
constexpr int SEG_ITERS = TKZ_SEG_ITERS;
constexpr int SEG_ITERS_FULL = 4;  // iterations on the full grid (the rest: a quarter, then 1/16)
constexpr uint32_t SEG_MAX_L = 0x7FFFFFFFu;
constexpr uint32_t SEG_MAX_GROUP = 0xFFFFu;
constexpr uint32_t SEG_BIGP = 4096;  // segments of a pretoken past which its count / emission take a block  // a group's bytes: its tokens' offsets are 16-bit group-relative
// SF_JOINED: joined by k_seg_first; SF_JNEW: joined by the k_seg_check of the current
// iteration, SF_JOLD: of an earlier one (k_seg_join adds it to every group it joins, so the
// next iteration's check sees it). The left-head walks of k_seg_check read only SF_JOINED |
// SF_JOLD (sf_jbefore), so no lane reads a flag another lane of the same launch sets: the
// outcome is the same on every run (round 5 had a bit per iteration, which bounded the
// iterations by the flag bits)
constexpr uint32_t SF_HEAD = 1u, SF_JOINED = 2u, SF_PEND = 4u, SF_INERT = 8u, SF_JOLD = 16u, SF_JNEW = 32u;
constexpr uint32_t SF_HOT_SHIFT = 12;  // bits 12..31: a hot memo hit's index + 1 (k_seg_init -> k_seg_first)
constexpr uint32_t SF_JANY = SF_JOINED | SF_JOLD | SF_JNEW;
__device__ __forceinline__ uint32_t sf_jit(int) { return SF_JNEW; }
__device__ __forceinline__ uint32_t sf_jbefore(int) { return SF_JOINED | SF_JOLD; }
constexpr uint32_t SEG_ALLOC = 2048;  // segment slots a k_seg_init block takes at a time
// Debug builds (-DTKZ_SEG_BOUNDS=1, verdict r5 item 5): every staged list append and flush,
// every segment-record, token and edge-list write of the k_seg_* kernels checks its index
// against its array's bound; a write past it is skipped and recorded (bit `code` of
// g_seg_err, one printf per code) instead of performed, and tkz_batch_stats reports the bits
// (seg_bound_errors). Release builds compile the checks away.
#ifndef TKZ_SEG_BOUNDS
#define TKZ_SEG_BOUNDS 0
#endif
#if TKZ_SEG_BOUNDS
__device__ unsigned int g_seg_err;
__device__ __noinline__ void seg_bound_fail(uint32_t code, uint64_t idx, uint64_t cap) {
    if (!(atomicOr(&g_seg_err, 1u << code) & (1u << code)))
        printf("tkz: segmented path bound %u: index %llu >= %llu\n", code, (unsigned long long)idx,
               (unsigned long long)cap);
}
#define SEG_BOUND(code, idx, cap) \
    ((uint64_t)(idx) < (uint64_t)(cap) || (seg_bound_fail((code), (uint64_t)(idx), (uint64_t)(cap)), false))
#else
#define SEG_BOUND(code, idx, cap) true
#endif
enum { SB_WAVELIST = 1, SB_BLOCKLIST, SB_SO, SB_SE, SB_STAGE, SB_TOK, SB_WTOK, SB_EDGE, SB_JOIN, SB_EMIT, SB_QUEUE,
       SB_FLAG, SB_LIST };
enum { SC_SEGS = 0, SC_PEND = 1, SC_JOIN = SC_PEND + SEG_ITERS + 1, SC_BIG = SC_JOIN + SEG_ITERS, SC_WAV = SC_BIG + SEG_ITERS,
       SC_BIGP = SC_WAV + SEG_ITERS, SC_BIGI = SC_BIGP + 1, SC_N = SC_BIGI + 1 };

struct SegWs {
    uint32_t* ctr;      // SC_* counters, zeroed before k_seg_init
    uint32_t* so;       // segment: pretoken-relative start
    uint32_t* se;       // segment: pretoken-relative end
    uint32_t* spt;      // segment: its pretoken's long-list slot
    uint32_t* sg;       // head: end segment of its group (exclusive, global index)
    uint64_t* smeta;    // head: its last encode (sm_make)
    uint32_t* spool;    // head: 1 + its segment-memo pool entry (tokens and profile there), 0: in the scratch
    uint32_t* sf;       // SF_* flags (HEAD stays set; JOINED = inside a group)
    uint32_t* pbase;    // long-list slot: first segment
    uint32_t* pn;       // long-list slot: segment count
    uint32_t* pst;      // long-list slot: 0 segmented, 1 failed (listed by k_seg_count), 2 not segmented
    uint32_t* plen;     // long-list slot: its length (restored to its pr slot when it fails: k_bpe_long reads it there)
    uint32_t* list[2];  // heads to encode in iteration it >= 1: list[it & 1]
    uint32_t* join;     // left heads of crossed boundaries (this iteration)
    uint64_t cap_seg, cap_list;
};

__device__ __forceinline__ bool ascii_bit(uint64_t lo, uint64_t hi, uint32_t c) {
    return c < 128u && (((c < 64u ? lo : hi) >> (c & 63u)) & 1ull);
}
__device__ __forceinline__ bool seg_drop(const DevTables& T, uint32_t c) { return ascii_bit(T.drop_lo, T.drop_hi, c); }

// A group's meta (smeta, the segment memo): first symbol | last symbol << 20 | tokens << 40
// | edges << 48 (the initial symbols; edges = the lengths of its edge lists: the rounds
// that changed the first symbol, bits 48..55, and the last symbol, bits 56..63); symbols
// < 2^20 (compact, or T.mid)
__device__ __forceinline__ uint64_t sm_make(uint32_t f0, uint32_t l0, uint32_t n, uint32_t edges) {
    return (uint64_t)f0 | ((uint64_t)l0 << 20) | ((uint64_t)n << 40) | ((uint64_t)edges << 48);
}
__device__ __forceinline__ uint32_t sm_first(uint64_t m) { return (uint32_t)m & 0xFFFFFu; }
__device__ __forceinline__ uint32_t sm_last(uint64_t m) { return (uint32_t)(m >> 20) & 0xFFFFFu; }
__device__ __forceinline__ uint32_t sm_ntok(uint64_t m) { return (uint32_t)(m >> 40) & 0xFFu; }
__device__ __forceinline__ uint32_t sm_le(uint64_t m) { return (uint32_t)(m >> 48) & 0xFFu; }
__device__ __forceinline__ uint32_t sm_re(uint64_t m) { return (uint32_t)(m >> 56); }
// the new id of a merge value (compact: rank << 16 | new_id; wide: the rank)
template <bool COMPACT>
__device__ __forceinline__ uint32_t seg_nid(const DevTables& T, uint32_t v) {
    return COMPACT ? v & 0xFFFFu : T.r2id[v];
}
// a segment-memo pool token: id | start << 20 | end << 26 (key-relative, keys <= 16 B)
__device__ __forceinline__ uint32_t pool_tok(uint32_t id, uint32_t s, uint32_t e) { return id | (s << 20) | (e << 26); }

__device__ __forceinline__ uint64_t seg_pos(const Deferred& D, const SegWs& G, uint32_t g) {
    return D.llist[G.spt[g]] & POS_MASK;
}

// Initial symbols of an all-ASCII group of L <= 8 NW bytes: its kept bytes (the dropped
// ones are the cuts' chars), found from a bit mask with their id loads issued together
// (reg_init's general path walks the bytes with one dependent id load each). Returns 0
// when not applicable (a byte >= 0x80 or L > 8 NW), 2 when more than W symbols, else 1.
template <int W, int NW, bool COMPACT, bool PACK>
__device__ __forceinline__ int seg_init_ascii(const DevTables& T, RegWord<W, COMPACT, PACK>& w, const WordBytes<NW>& wb,
                                              uint32_t L) {
    static_assert(NW <= 8, "64-bit kept mask");
    if (L > 8u * NW) return 0;
    uint64_t hi = 0;
#pragma unroll
    for (int k = 0; k < NW; ++k) {
        const int lo_b = 8 * k;
        uint64_t m = 0x8080808080808080ull;
        if (lo_b + 8 > (int)L) m = (lo_b >= (int)L) ? 0ull : (m & ((1ull << (8 * (L - lo_b))) - 1));
        hi |= wb.w[k] & m;
    }
    if (hi) return 0;
    uint64_t kept = 0;
#pragma unroll
    for (int j = 0; j < 8 * NW; ++j)
        if ((uint32_t)j < L && !seg_drop(T, wb.at(j))) kept |= 1ull << j;
    const uint32_t n = (uint32_t)__popcll(kept);
    if (n > (uint32_t)W) return 2;
    uint32_t pk[W], id[W];
    uint64_t m = kept;
#pragma unroll
    for (int k = 0; k < W; ++k) {
        pk[k] = m ? (uint32_t)__builtin_ctzll(m) : 0u;
        m &= m - 1ull;
        id[k] = T.byte_id[wb(pk[k])];
    }
#pragma unroll
    for (int k = 0; k < W; ++k) id[k] = id[k] == NONE ? T.unk_id : id[k];  // (a kept char: unk is set)
#pragma unroll
    for (int k = 0; k < W; ++k) {
        w.pr[k] = NONE;
        if ((uint32_t)k < n) reg_set(w, k, id[k], pk[k], pk[k] + 1u);
    }
    w.n = (int)n;
    return 1;
}

// Encodes group [g, e) of the pretoken at pos (one lane; act = the lane has a group): its
// tokens to tok / prs at the group's first byte (id, start | end << 16; group-relative),
// its edge lists to offs there (pairs RE_k | LE_k << 32: SegEdges), its meta to smeta[g]. Returns
// false if the group holds more than W symbols or spans more than 255 bytes.
template <int W, int NW, bool COMPACT>
__device__ __forceinline__ bool seg_encode(const DevTables& T, const uint8_t* bytes, uint64_t limit, const SegWs& G,
                                           const Scratch& S, uint64_t pos, uint32_t g, uint32_t b0, uint32_t b1,
                                           bool act) {
    if (!act) b0 = b1 = 0u;
    const uint32_t len = b1 - b0;
    const bool ok_len = len <= (COMPACT ? 255u : 64u);  // (packed offsets; a longer group: the wave path)
    RegWord<W, COMPACT, true> rw;
    WordBytes<NW> wb;
    wb.load(bytes, pos + b0, limit, T.norm);
    const uint32_t Lr = act && ok_len ? len : 0u;
    // (W = 32: its arrays would spill)
    const int asc = TKZ_SEG_ASCII && W <= 16 && Lr ? seg_init_ascii<W, NW, COMPACT>(T, rw, wb, Lr) : 0;
    bool fits = asc == 1;
    if (asc == 0)
        fits = len <= 8u * NW ? reg_init<W, COMPACT, NW>(T, T.byte_id, rw, wb, wb, Lr)
                              : reg_init<W, COMPACT, NW>(T, T.byte_id, rw, wb, GlbReader{bytes + pos + b0, T.norm}, Lr);
    const bool ok = act && ok_len && fits;  // (a group whose chars are all dropped: no symbol)
    uint32_t f0 = 0, l0 = 0;
#pragma unroll
    for (int k = 0; k < W; ++k) {
        f0 = k == 0 ? rw.idv(rw.sy[k]) : f0;
        l0 = k == rw.n - 1 ? rw.idv(rw.sy[k]) : l0;
    }
    if (!ok) rw.n = 0;  // no rounds for this lane
    uint32_t edges = 0;
    reg_rounds<W, COMPACT, true>(T, rw, S.offs() + pos + b0, &edges);
    if (ok) {
        uint32_t* tk = S.tok() + pos + b0;
        uint32_t* te = S.prs() + pos + b0;
#pragma unroll
        for (int k = 0; k < W; ++k) {
            if (k < rw.n && SEG_BOUND(SB_TOK, (uint64_t)k, len) && SEG_BOUND(SB_TOK, pos + b0 + k, S.tb)) {
                tk[k] = rw.idv(rw.sy[k]);
                te[k] = rw.start(k) | (rw.end(k) << 16);  // (group-relative)
            }
        }
        G.smeta[g] = sm_make(f0, l0, (uint32_t)rw.n, edges);
        G.spool[g] = 0;
    }
    return ok;
}

// Encodes group [g, e) with the whole wave (groups of more than 32 symbols, or longer than
// 255 B), up to SEGW_K * 64 symbols: position q lives in slot q / 64 of lane q % 64, the
// symbols (and their byte ranges) in registers, staged through LDS (stg: 3 x SEGW_MAX words)
// only to compact them after a round. A round is a wave minimum over the lanes' pair values,
// one ballot of the candidates per slot, the greedy left-to-right choice inside runs of equal
// pairs on the scalar unit (bpe.zig:240-252: after a merge at i the scan goes on at i + 1 of
// the shortened word; a run carries from one slot's 64 positions into the next), the merges,
// the compaction and a probe per pair (issued together). Same outputs as seg_encode.
// Returns false (uniform) if the group has more than SEGW_MAX symbols, spans more than
// SEG_MAX_GROUP bytes, or ends with more than 255 tokens or edge entries (the meta's fields).
constexpr int SEGW_K = 8;
constexpr uint32_t SEGW_MAX = 64u * SEGW_K;
// (K = 1 for groups of <= 64 symbols, the common case: 8 slots cost a 64-symbol group 8 probes
// and an LDS compaction per lane per round, +0.2 ms per C6 iteration)
template <bool COMPACT, int SEGW_K>
__device__ __forceinline__ bool seg_encode_wave_k(const DevTables& T, const uint8_t* bytes, uint64_t limit, const SegWs& G,
                                const Scratch& S, uint64_t pos, uint32_t g, uint32_t e, uint32_t* stg) {
    const int lane = lane_id();
    const uint32_t b0 = G.so[g], len = G.se[e - 1] - b0;
    if (len > SEG_MAX_GROUP) return false;
    uint32_t* const s_sym = stg;
    uint32_t* const s_st = stg + SEGW_MAX;
    uint32_t* const s_en = stg + 2 * SEGW_MAX;
    uint32_t n = 0;
    for (uint32_t r0 = 0; r0 < len; r0 += GROUP) {  // (the pretoken is well-formed UTF-8)
        const uint32_t o = r0 + 8u * (uint32_t)lane;
        WordBytes<2> v;
        v.load(bytes, pos + b0 + o, limit, T.norm);
        const uint32_t nv = o < len ? min(len - o, 8u) : 0u;
        uint32_t ids[8], ends[8], keep = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            ids[j] = NONE;
            ends[j] = 0;
            if ((uint32_t)j < nv) {
                const uint32_t c = v.at(j);
                if ((c & 0xC0u) != 0x80u) {
                    uint32_t k = seq_len(c);
                    if (o + (uint32_t)j + k > len) k = len - o - (uint32_t)j;
                    uint32_t packed = c;
#pragma unroll
                    for (int t = 1; t < 4; ++t)
                        if ((uint32_t)t < k) packed |= v.at(j + t) << (8 * t);
                    ids[j] = char_id(T, T.byte_id, c, packed, k);
                    ends[j] = o + (uint32_t)j + k;
                    if (ids[j] != NONE) keep |= 1u << j;
                }
            }
        }
        const uint32_t cnt = (uint32_t)__popc(keep);
        const uint32_t inc = (uint32_t)wave_incl_scan((int)cnt);
        if (n + lane63(inc) > 64u * SEGW_K) return false;
        uint32_t q = n + inc - cnt;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if ((keep >> j) & 1u) {
                s_sym[q] = ids[j];
                s_st[q] = o + (uint32_t)j;  // (group-relative)
                s_en[q] = ends[j];
                ++q;
            }
        }
        n += lane63(inc);
    }
    if (n == 0) {  // every char dropped: an empty group
        if (lane == 0) { G.smeta[g] = 0; G.spool[g] = 0; }
        return true;
    }
    WAVE_SYNC();
    uint32_t sym[SEGW_K], st[SEGW_K], en[SEGW_K], pv[SEGW_K];
    auto load = [&]() {
#pragma unroll
        for (int k = 0; k < SEGW_K; ++k) {
            const uint32_t q = 64u * (uint32_t)k + (uint32_t)lane;
            const bool in = q < n;
            sym[k] = in ? s_sym[q] : 0u;
            st[k] = in ? s_st[q] : 0u;
            en[k] = in ? s_en[q] : 0u;
        }
    };
    load();
    WAVE_SYNC();
    const uint32_t f0 = s_sym[0];
    const uint32_t l0 = s_sym[n - 1];
    // the symbol after each position: the next lane's of the same slot, lane 0's of the next
    // slot for lane 63 (every lane runs the shuffles: a lane outside a divergent branch
    // does not provide its value)
    auto next_of = [&](const uint32_t* x, int k) {
        const uint32_t sh = (uint32_t)__shfl((int)x[k], (lane + 1) & (WAVE - 1), WAVE);
        const uint32_t nx = k + 1 < SEGW_K ? (uint32_t)__builtin_amdgcn_readlane((int)x[k + 1 < SEGW_K ? k + 1 : k], 0) : 0u;
        return lane == WAVE - 1 ? nx : sh;
    };
    auto probe_all = [&]() {
#pragma unroll
        for (int k = 0; k < SEGW_K; ++k) {
            const uint32_t q = 64u * (uint32_t)k + (uint32_t)lane;
            const uint32_t sn = next_of(sym, k);
            pv[k] = q + 1u < n ? cuckoo_value<COMPACT>(T, sym[k], sn) : NONE;
        }
    };
    probe_all();
    uint64_t* prof = S.offs() + pos + b0;
    uint32_t lle = 0, lre = 0;  // edge list lengths
    while (n >= 2) {
        uint32_t lm = NONE;
#pragma unroll
        for (int k = 0; k < SEGW_K; ++k) lm = min(lm, pv[k]);
        const uint32_t best = wave_min_u32(lm);
        if (best == NONE) break;
        const uint32_t nk = (n + 63u) >> 6;  // slots in use (uniform)
        // the merged positions, slot by slot; a run of candidates carries into the next slot
        uint64_t sel[SEGW_K];
        uint64_t carry = 0;  // the previous slot's last position merged
        uint32_t nsel = 0;
#pragma unroll
        for (int k = 0; k < SEGW_K; ++k) {
            const uint64_t C = __ballot(pv[k] == best);
            uint64_t rem = (uint32_t)k < nk ? C & ~carry : 0ull, sk = 0;
            while (rem) {  // run starts, then every second position of each run
                const uint64_t st0 = rem & ~(rem << 1);
                sk |= st0;
                rem &= ~(st0 | (st0 << 1));
            }
            sel[k] = sk;
            carry = sk >> 63;
            nsel += (uint32_t)__popcll(sk);
        }
        uint32_t le = (uint32_t)(sel[0] & 1ull), re = 0;
#pragma unroll
        for (int k = 0; k < SEGW_K; ++k)
            if ((uint32_t)k == (n - 2u) >> 6) re = (uint32_t)((sel[k] >> ((n - 2u) & 63u)) & 1ull);
        if (lane == 0) {  // the edge lists (reg_rounds)
            uint32_t* p32 = (uint32_t*)prof;
            if (re && SEG_BOUND(SB_EDGE, lre, len)) p32[2 * lre] = best;
            if (le && SEG_BOUND(SB_EDGE, lle, len)) p32[2 * lle + 1] = best;
        }
        lle += le;
        lre += re;
        const uint32_t X = seg_nid<COMPACT>(T, best);
        // merges: q takes X and the end of q + 1, which dies
#pragma unroll
        for (int k = 0; k < SEGW_K; ++k) {
            const uint32_t en_next = next_of(en, k);
            if ((sel[k] >> lane) & 1ull) {
                sym[k] = X;
                en[k] = en_next;
            }
        }
        // compaction through LDS: the live positions in order
        uint32_t nbase = 0;
        uint64_t prev_hi = 0;
#pragma unroll
        for (int k = 0; k < SEGW_K; ++k) {
            const uint64_t dead = (sel[k] << 1) | prev_hi;
            prev_hi = sel[k] >> 63;
            const uint32_t rest = n > 64u * (uint32_t)k ? n - 64u * (uint32_t)k : 0u;
            const uint64_t valid = rest >= 64u ? ~0ull : ((1ull << rest) - 1ull);
            const uint64_t live = valid & ~dead;
            if ((live >> lane) & 1ull) {
                const uint32_t d = nbase + lane_mbcnt(live);
                s_sym[d] = sym[k];
                s_st[d] = st[k];
                s_en[d] = en[k];
            }
            nbase += (uint32_t)__popcll(live);
        }
        n -= nsel;
        WAVE_SYNC();
        load();
        WAVE_SYNC();
        probe_all();
    }
    if (n > 255u || lle > 255u || lre > 255u) return false;  // (meta fields)
#pragma unroll
    for (int k = 0; k < SEGW_K; ++k) {
        const uint32_t q = 64u * (uint32_t)k + (uint32_t)lane;
        if (q < n && SEG_BOUND(SB_WTOK, q, len) && SEG_BOUND(SB_WTOK, pos + b0 + q, S.tb)) {
            S.tok()[pos + b0 + q] = sym[k];
            S.prs()[pos + b0 + q] = st[k] | (en[k] << 16);
        }
    }
    if (lane == 0) {
        G.smeta[g] = sm_make(f0, l0, n, lle | (lre << 8));
        G.spool[g] = 0;
    }
    return true;
}

// a group by the wave: one symbol per lane when it has <= 64, else up to SEGW_MAX
template <bool COMPACT>
__device__ __forceinline__ bool seg_encode_wave(const DevTables& T, const uint8_t* bytes, uint64_t limit, const SegWs& G,
                                                const Scratch& S, uint64_t pos, uint32_t g, uint32_t e, uint32_t* stg) {
    if (seg_encode_wave_k<COMPACT, 1>(T, bytes, limit, G, S, pos, g, e, stg)) return true;
    // (a 64-symbol version's failure: more than 64 symbols, or the meta's fields; rerun wide)
    return seg_encode_wave_k<COMPACT, SEGW_K>(T, bytes, limit, G, S, pos, g, e, stg);
}

// A group's edge lists: RE, the values of the rounds that changed its last symbol, and LE,
// those that changed its first symbol, in round order (a boundary check needs no other
// round: the straddling pair changes only with an edge symbol, and the round that ends a
// pair bounds its merge). Stored as pairs RE_k | LE_k << 32 -- in the scratch at the group's
// first byte (its own encode), or at the start of its segment-memo pool entry (a memo hit:
// [pairs][tokens], 16-B aligned; max(|RE|, |LE|) pairs). Entries 0..3 of each list are held
// in registers (NONE past its length), the rest read from p as the walk reaches them.
struct SegEdges {
    const uint32_t* p;  // the pairs (u32 view: RE_k at p[2k], LE_k at p[2k + 1])
    uint32_t r[4], l[4];
    // pool entry q (1 + offset): the first 4 pairs in two loads
    __device__ __forceinline__ void load_pool(const DevTables& T, uint32_t q, uint32_t nre, uint32_t nle) {
        p = T.smpool + (q - 1u);
        const uint4* e = (const uint4*)p;
        const uint4 a = e[0], b = e[1];
        r[0] = a.x; l[0] = a.y; r[1] = a.z; l[1] = a.w; r[2] = b.x; l[2] = b.y; r[3] = b.z; l[3] = b.w;
        clip(nre, nle);
    }
    // scratch pairs at pr: the first min(4, max(nre, nle)) loaded
    __device__ __forceinline__ void load_scratch(const uint64_t* pr, uint32_t nre, uint32_t nle) {
        const uint32_t n = max(nre, nle);
        uint64_t w[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) w[k] = (uint32_t)k < n ? pr[k] : ~0ull;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            r[k] = (uint32_t)w[k];
            l[k] = (uint32_t)(w[k] >> 32);
        }
        p = (const uint32_t*)pr;
        clip(nre, nle);
    }
    __device__ __forceinline__ void clip(uint32_t nre, uint32_t nle) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            r[k] = (uint32_t)k < nre ? r[k] : NONE;
            l[k] = (uint32_t)k < nle ? l[k] : NONE;
        }
    }
};

// Is the boundary between groups g | h crossed? (one lane) m*: their metas, Eg / Eh: their
// edge lists (g's RE and h's LE are used). A group without symbols (its chars all dropped)
// joins its neighbours: their symbols are adjacent.
//
// The walk takes g's RE and h's LE in rank order; the straddling pair (x, y) starts as
// (g's last initial symbol, h's first) and changes at each entry (x or y becomes that
// round's new id; both on equal values), and the boundary is crossed iff some pair's merge
// value b satisfies b <= the value of the round that ends the pair (both lists exhausted:
// any merge) -- the two groups' processes then disagree with the joint one at b (a tie
// counts as crossed: joining is always exact). The walk does not depend on b, so it is taken
// first, KP pairs at a time, and their probes are issued together (probing at each change
// made the check a chain of dependent loads, and a wave waited for its longest lane's chain).
template <bool COMPACT>
__device__ bool seg_crossed_core(const DevTables& T, uint64_t mg, uint64_t mh, const SegEdges& Eg, const SegEdges& Eh,
                                 const uint32_t* ov) {
    if (sm_ntok(mg) == 0u || sm_ntok(mh) == 0u) return true;
    const uint32_t ng = sm_re(mg), nh = sm_le(mh);
    constexpr int KP = TKZ_SEG_KP;
    uint32_t kx[KP], ky[KP], lim[KP];
    uint32_t r0 = Eg.r[0], r1 = Eg.r[1], r2 = Eg.r[2], r3 = Eg.r[3];
    uint32_t l0 = Eh.l[0], l1 = Eh.l[1], l2 = Eh.l[2], l3 = Eh.l[3];
    uint32_t x = sm_last(mg), y = sm_first(mh), i = 0, j = 0;
    bool done = false;
    while (!done) {
        int np = 0;
        while (np < KP) {  // pairs until KP are recorded or the walk ends
            const uint32_t hc = r0, hd = l0;
#pragma unroll
            for (int k = 0; k < KP; ++k)
                if (k == np) { kx[k] = x; ky[k] = y; lim[k] = min(hc, hd); }
            ++np;
            done = hc == NONE && hd == NONE;
            if (done) break;
            if (hc <= hd) {
                x = seg_nid<COMPACT>(T, hc);
                ++i;
                r0 = r1; r1 = r2; r2 = r3;
                r3 = i + 3u < ng ? Eg.p[2u * (i + 3u)] : NONE;
            }
            if (hd <= hc) {
                y = seg_nid<COMPACT>(T, hd);
                ++j;
                l0 = l1; l1 = l2; l2 = l3;
                l3 = j + 3u < nh ? Eh.p[2u * (j + 3u) + 1u] : NONE;
            }
        }
        // the recorded pairs' probes, loads first
        bool cr = false;
        uint4 pa[KP], pb[KP];
#pragma unroll
        for (int k = 0; k < KP; ++k) {
            uint32_t b1 = 0, b2 = 0;
            if (k < np) cuckoo_buckets<COMPACT>(T, kx[k], ky[k], b1, b2);
#if TKZ_FULL_ABL == 2  // timing only: no probe loads (wrong results)
            pa[k] = make_uint4(b1, b2, kx[k], ky[k]);
            pb[k] = make_uint4(b2, b1, ky[k], kx[k]);
#else
            // the second bucket only where the overflow bitmap says a key may sit there
            const bool two = ov == nullptr || ((ov[b1 >> 5] >> (b1 & 31u)) & 1u);
            pa[k] = cuckoo_bucket<COMPACT>(T, b1);
            pb[k] = two ? cuckoo_bucket<COMPACT>(T, b2) : make_uint4(EMPTY32, EMPTY32, EMPTY32, EMPTY32);
#endif
        }
#pragma unroll
        for (int k = 0; k < KP; ++k) {
            const uint32_t b = cuckoo_match<COMPACT>(pa[k], pb[k], kx[k], ky[k]);
            cr = cr || (k < np && b != NONE && b <= lim[k]);
        }
        if (cr) return true;
    }
    return false;
}

// group g's edge lists, of which RE's first nre and LE's first nle entries are used
template <bool COMPACT>
__device__ __forceinline__ SegEdges seg_edges(const DevTables& T, const SegWs& G, const Scratch& S, uint64_t pos,
                                              uint32_t g, uint32_t nre, uint32_t nle) {
    SegEdges E;
    const uint32_t q = G.spool[g];
    if (q) E.load_pool(T, q, nre, nle);
    else E.load_scratch(S.offs() + pos + G.so[g], nre, nle);
    return E;
}

// The boundary between groups g | h of the pretoken at pos, from their records
template <bool COMPACT>
__device__ bool seg_crossed(const DevTables& T, const SegWs& G, const Scratch& S, uint64_t pos, uint32_t g, uint32_t h,
                            const uint32_t* ov) {
    const uint64_t mg = G.smeta[g], mh = G.smeta[h];
    return seg_crossed_core<COMPACT>(T, mg, mh, seg_edges<COMPACT>(T, G, S, pos, g, sm_re(mg), 0u),
                                     seg_edges<COMPACT>(T, G, S, pos, h, 0u, sm_le(mh)), ov);
}

// The overflow bitmap (DevTables::seg_over) staged in LDS by the whole block (dynamic LDS
// of seg_over_lds(T) bytes; null when the table has none or it is too large)
#ifndef TKZ_SEG_OVER
#define TKZ_SEG_OVER 1  // 0: boundary probes always load both buckets
#endif
constexpr uint32_t SEG_OVER_MAX_BITS = TKZ_SEG_OVER ? 17 : 0;  // (16 KiB of LDS)
inline size_t seg_over_lds(const DevTables& T) {
    return T.seg_over && T.seg_over_bits <= SEG_OVER_MAX_BITS ? ((size_t)1 << T.seg_over_bits) / 8 : 0;
}
__device__ __forceinline__ const uint32_t* seg_over_stage(const DevTables& T, uint32_t* lds) {
    if (!T.seg_over || T.seg_over_bits > SEG_OVER_MAX_BITS) return nullptr;
    const uint32_t nw = max((1u << T.seg_over_bits) / 32u, 1u);
    for (uint32_t i = threadIdx.x; i < nw; i += blockDim.x) lds[i] = T.seg_over[i];
    __syncthreads();
    return lds;
}

// A block's staging of list entries (segment indices) in LDS: lanes append with one LDS
// atomic per wave, and the block moves them to the global list with ONE global atomic per
// flush (coalesced stores). One atomic per wave on a single global counter cost ~10 ns
// each, serialised in L2: 1.6M of them made the first-iteration kernels 36 ms.
template <int CAP>
struct BlockList {
    uint32_t buf[CAP];
    uint32_t n, base;
    __device__ __forceinline__ void init() {
        if (threadIdx.x == 0) n = 0;
        __syncthreads();
    }
    // every lane of the wave calls it (converged)
    __device__ __forceinline__ void push(bool on, uint32_t v) {
        const uint64_t m = __ballot(on);
        if (m == 0ull) return;
        uint32_t b = 0;
        if (lane_id() == 0) b = atomicAdd(&n, (uint32_t)__popcll(m));
        b = rfl(b);
        if (on && SEG_BOUND(SB_BLOCKLIST, b + lane_mbcnt(m), CAP)) buf[b + lane_mbcnt(m)] = v;
    }
    // every thread of the block calls it; flushes when fewer than `room` slots are left
    // (or always, `room` = CAP). An entry past the list's capacity fails its pretoken.
    __device__ __forceinline__ void flush(uint32_t* ctr, uint32_t* list, uint64_t cap, const SegWs& G, uint32_t room) {
        __syncthreads();
        const uint32_t c = n;
        if (c == 0u || c + room <= (uint32_t)CAP) return;  // (uniform: every thread read n after the barrier)
        if (threadIdx.x == 0) base = atomicAdd(ctr, c);
        __syncthreads();
        const uint32_t b = base;
        for (uint32_t i = threadIdx.x; i < c; i += blockDim.x) {
            const uint32_t v = buf[i];
            if ((uint64_t)b + i < cap) list[b + i] = v;
            else if (SEG_BOUND(SB_LIST, v, G.cap_seg)) G.pst[G.spt[v]] = 1;
        }
        __syncthreads();
        if (threadIdx.x == 0) n = 0;
        __syncthreads();
    }
};
constexpr int SEG_BL = 2048;

// A wave's staging of list entries in LDS (buf: CAP entries of its own): lanes append by a
// ballot into a wave-uniform count (no atomic), and the wave moves the entries to the
// global list with ONE global atomic per flush (coalesced stores). No block barrier: with
// BlockList every flush made the block's waves wait for each other.
template <int CAP>
struct WaveList {
    uint32_t* buf;
    uint32_t n;  // (wave-uniform)
    __device__ __forceinline__ void push(bool on, uint32_t v) {
        const uint64_t m = __ballot(on);
        if (on && SEG_BOUND(SB_WAVELIST, n + lane_mbcnt(m), CAP)) buf[n + lane_mbcnt(m)] = v;
        n += (uint32_t)__popcll(m);
    }
    // flushes when fewer than `room` slots are left (room = CAP: always, if any). An entry
    // past the list's capacity fails its pretoken.
    __device__ __forceinline__ void flush(uint32_t* ctr, uint32_t* list, uint64_t cap, const SegWs& G, uint32_t room) {
        if (n == 0u || n + room <= (uint32_t)CAP) return;
        WAVE_SYNC();
        uint32_t b = 0;
        if (lane_id() == 0) b = atomicAdd(ctr, n);
        b = rfl(b);
        for (uint32_t i = (uint32_t)lane_id(); i < n; i += WAVE) {
            const uint32_t v = buf[i];
            if ((uint64_t)b + i < cap) list[b + i] = v;
            else if (SEG_BOUND(SB_LIST, v, G.cap_seg)) G.pst[G.spt[v]] = 1;
        }
        WAVE_SYNC();
        n = 0;
    }
};
constexpr int SEG_WL = 512;  // entries per wave list

// The segment memo lookup of a single segment (L <= 16 bytes at pos + b0): on a hit its
// meta, 1 + the offset of its pool entry (its edge lists and tokens) and its hot index + 1.
__device__ __forceinline__ bool seg_memo_find(const DevTables& T, const uint8_t* bytes, uint64_t limit, uint64_t at,
                                              uint32_t L, uint64_t& meta, uint32_t& q, uint32_t& hot) {
    WordBytes<2> kb;
    kb.load(bytes, at, limit, T.norm);
    const uint64_t k0 = kb.w[0] & ((2ull << (8u * min(L, 8u) - 1u)) - 1u);  // (L >= 1)
    const uint64_t k1 = L > 8u ? kb.w[1] & ((2ull << (8u * (L - 8u) - 1u)) - 1u) : 0ull;
    uint32_t h = short_key_hash(k0, k1, L) >> (32 - T.smemo_bits);
    uint4 a, b;
    while (true) {
        a = T.smemo[2 * h];
        b = T.smemo[2 * h + 1];
        if (b.x == 0u) return false;
        if ((b.x & 31u) == L && a.x == (uint32_t)k0 && a.y == (uint32_t)(k0 >> 32) && a.z == (uint32_t)k1 &&
            a.w == (uint32_t)(k1 >> 32))
            break;
        ++h;
    }
    // slot {len | tokens << 5 | rounds << 10, meta bits 0..31, edges | meta bits 32..39 << 16, pool}
    meta = (uint64_t)b.y | ((uint64_t)((b.z >> 16) & 0xFFu) << 32) | ((uint64_t)((b.x >> 5) & 31u) << 40) |
           ((uint64_t)(b.z & 0xFFFFu) << 48);
    q = b.w + 1u;
    hot = b.x >> 14;  // (hot index + 1; 0: not hot)
    return true;
}

// byte classes of one lane's 8 bytes of a pretoken (o: their offset): kept bytes (not a
// dropped ASCII char; the return value), inert chars, whitespace cuts, and whether the
// UTF-8 is well-formed there (as long_init)
__device__ __forceinline__ uint32_t seg_classify(const DevTables& T, const WordBytes<2>& v, uint32_t o, uint32_t L,
                                                 uint32_t& bad, uint32_t& inert, uint32_t& cut) {
    const uint32_t nv = o < L ? min(L - o, 8u) : 0u;
    uint32_t kept = 0;
    inert = cut = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        if ((uint32_t)j >= nv) break;
        const uint32_t c = v.at(j);
        if (!seg_drop(T, c)) kept |= 1u << j;
        if (ascii_bit(T.inert_lo, T.inert_hi, c)) inert |= 1u << j;
        if (ascii_bit(T.cut_lo, T.cut_hi, c)) cut |= 1u << j;
        if ((c & 0xC0u) == 0x80u) {
            if (o + (uint32_t)j == 0) bad = 1;
            continue;
        }
        const uint32_t k = seq_len(c);
        if (k > 1) {
            if (o + (uint32_t)j + k > L) bad = 1;
#pragma unroll
            for (int t = 1; t < 4; ++t)
                if ((uint32_t)t < k && (v.at(j + t) & 0xC0u) != 0x80u) bad = 1;
        } else if (c >= 0x80u) {
            bad = 1;
        }
        if (o + (uint32_t)j + k < L && (v((uint32_t)j + k) & 0xC0u) == 0x80u) bad = 1;
    }
    return kept;
}

// The segment starts among one lane's 8 bytes: a kept byte after a dropped one, at or after
// an inert char, or at a whitespace cut. pk / pi: the previous byte's kept / inert bit.
__device__ __forceinline__ uint32_t seg_starts(uint32_t kept, uint32_t inert, uint32_t cut, uint32_t pk, uint32_t pi) {
    const uint32_t prev_k = (kept << 1) | pk, prev_i = (inert << 1) | pi;
    return kept & (~prev_k | inert | prev_i | cut) & 0xFFu;
}

// Long pretokens' block-wide kernels (k_seg_init_big, k_seg_count_big, k_seg_emit_big): SEGB_W
// waves per block, a block per listed pretoken while they last (the hardware starts the next block
// where one ends, so a 1-MB document and a 20-KB one balance; blocks past the list exit at once)
constexpr int SEGB_W = 8;
constexpr unsigned SEGB_GRID = 4096;
constexpr uint32_t SEGI_BIG = 16384;  // bytes: longer pretokens take k_seg_init_big
#ifndef TKZ_SEGI_W
#define TKZ_SEGI_W 16  // waves per k_seg_init_big block (8: C10 5.4 ms, the largest pretoken's two passes on 8 waves)
#endif
#ifndef TKZ_SEGI_PR
#define TKZ_SEGI_PR 8
#endif
constexpr int SEGI_W = TKZ_SEGI_W;
constexpr uint32_t SEGI_PR = TKZ_SEGI_PR;  // rounds per piece (at least)
constexpr uint32_t SEGI_MAXP = 512;   // pieces per pretoken (at most: longer ones take longer pieces; 4,096: 82 KB of LDS, one block per CU)

// k_seg_init's per-round steps (also k_seg_init_big's, which runs them on pieces of a long
// pretoken in parallel: ck / ci, the kept / inert bit of the byte before the round, are then
// taken from that byte). SegStage: a wave's LDS staging of one 512-B round.
struct SegStage {
    uint32_t st[GROUP];  // a round's segment starts: offset | inert << 16 | byte << 17
    uint32_t en[GROUP];  // ... and ends (offset + 1)
};
// The kept / inert bits of byte p of the pretoken at pos (the carry into a round at p + 1)
__device__ __forceinline__ void seg_carry(const DevTables& T, const uint8_t* bytes, uint64_t pos, uint32_t p, uint32_t& ck,
                                          uint32_t& ci) {
    const uint32_t c = lower(bytes[pos + p], T.norm);
    ck = seg_drop(T, c) ? 0u : 1u;
    ci = ascii_bit(T.inert_lo, T.inert_hi, c) ? 1u : 0u;
}
// One round [r0, r0 + 512) classified, its segment starts and ends staged in LDS by their
// round-relative index (start: its offset in the round | inert << 16 | byte << 17; end: its
// pretoken offset + 1; the i-th end of the pretoken is segment i's); returns nst | nen << 16,
// and whether the UTF-8 is bad there in `bad_any`
__device__ __forceinline__ uint32_t seg_stage(const DevTables& T, const uint8_t* bytes, uint64_t limit, uint64_t pos,
                                              uint32_t L, uint32_t r0, uint32_t& ck, uint32_t& ci, bool& bad_any,
                                              SegStage& seg_stg) {
    const int lane = lane_id();
    const uint32_t o = r0 + 8u * (uint32_t)lane;
    WordBytes<2> v;
    v.load(bytes, pos + o, limit, T.norm);
    uint32_t bad = 0, inert, cut;
    const uint32_t kept = seg_classify(T, v, o, L, bad, inert, cut);
    bad_any = __ballot(bad) != 0ull;
    const int pl = lane > 0 ? lane - 1 : 0, nl = lane < WAVE - 1 ? lane + 1 : 0;
    const uint32_t pk = (uint32_t)__shfl((int)kept, pl, WAVE), pi = (uint32_t)__shfl((int)inert, pl, WAVE);
    const uint32_t nk = (uint32_t)__shfl((int)kept, nl, WAVE), ni = (uint32_t)__shfl((int)inert, nl, WAVE);
    const uint32_t nc = (uint32_t)__shfl((int)cut, nl, WAVE);
    // the byte after the lane's last: the next lane's first, or the next round's first byte
    // for lane 63 (re-read: its classes as a byte of this pretoken)
    uint32_t nxk = lane < WAVE - 1 ? nk & 1u : 0u, nxi = lane < WAVE - 1 ? ni & 1u : 0u, nxc = lane < WAVE - 1 ? nc & 1u : 0u;
    if (lane == WAVE - 1 && o + 8u < L) {
        const uint32_t c = lower(bytes[pos + o + 8], T.norm);
        nxk = seg_drop(T, c) ? 0u : 1u;
        nxi = ascii_bit(T.inert_lo, T.inert_hi, c) ? 1u : 0u;
        nxc = ascii_bit(T.cut_lo, T.cut_hi, c) ? 1u : 0u;
    }
    const uint32_t starts = seg_starts(kept, inert, cut, lane > 0 ? (pk >> 7) & 1u : ck, lane > 0 ? (pi >> 7) & 1u : ci);
    const uint32_t next_k = (kept >> 1) | (nxk << 7), next_i = (inert >> 1) | (nxi << 7), next_c = (cut >> 1) | (nxc << 7);
    const uint32_t ends = kept & (~next_k | inert | next_i | next_c) & 0xFFu;
    const uint32_t cs = (uint32_t)__popc(starts), ce = (uint32_t)__popc(ends);
    const uint32_t inc = (uint32_t)wave_incl_scan((int)(cs | (ce << 16)));
    uint32_t is = (inc & 0xFFFFu) - cs, ie = (inc >> 16) - ce;
    WAVE_SYNC();
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        if (((starts >> j) & 1u) && SEG_BOUND(SB_STAGE, is, GROUP))
            seg_stg.st[is++] = (8u * (uint32_t)lane + (uint32_t)j) | (((inert >> j) & 1u) << 16) | (v.at(j) << 17);
        if (((ends >> j) & 1u) && SEG_BOUND(SB_STAGE, ie, GROUP)) seg_stg.en[ie++] = o + (uint32_t)j + 1u;
    }
    ck = lane63((kept >> 7) & 1u);
    ci = lane63((inert >> 7) & 1u);
    WAVE_SYNC();
    return lane63(inc);
}
// seg_stage's counts alone (k_seg_init_big's first pass): nst | nen << 16, ck / ci updated
__device__ __forceinline__ uint32_t seg_count_round(const DevTables& T, const uint8_t* bytes, uint64_t limit, uint64_t pos,
                                                    uint32_t L, uint32_t r0, uint32_t& ck, uint32_t& ci, bool& bad_any) {
    const int lane = lane_id();
    const uint32_t o = r0 + 8u * (uint32_t)lane;
    WordBytes<2> v;
    v.load(bytes, pos + o, limit, T.norm);
    uint32_t bad = 0, inert, cut;
    const uint32_t kept = seg_classify(T, v, o, L, bad, inert, cut);
    bad_any = __ballot(bad) != 0ull;
    const int pl = lane > 0 ? lane - 1 : 0, nl = lane < WAVE - 1 ? lane + 1 : 0;
    const uint32_t pk = (uint32_t)__shfl((int)kept, pl, WAVE), pi = (uint32_t)__shfl((int)inert, pl, WAVE);
    const uint32_t nk = (uint32_t)__shfl((int)kept, nl, WAVE), ni = (uint32_t)__shfl((int)inert, nl, WAVE);
    const uint32_t nc = (uint32_t)__shfl((int)cut, nl, WAVE);
    uint32_t nxk = lane < WAVE - 1 ? nk & 1u : 0u, nxi = lane < WAVE - 1 ? ni & 1u : 0u, nxc = lane < WAVE - 1 ? nc & 1u : 0u;
    if (lane == WAVE - 1 && o + 8u < L) {
        const uint32_t c = lower(bytes[pos + o + 8], T.norm);
        nxk = seg_drop(T, c) ? 0u : 1u;
        nxi = ascii_bit(T.inert_lo, T.inert_hi, c) ? 1u : 0u;
        nxc = ascii_bit(T.cut_lo, T.cut_hi, c) ? 1u : 0u;
    }
    const uint32_t starts = seg_starts(kept, inert, cut, lane > 0 ? (pk >> 7) & 1u : ck, lane > 0 ? (pi >> 7) & 1u : ci);
    const uint32_t next_k = (kept >> 1) | (nxk << 7), next_i = (inert >> 1) | (nxi << 7), next_c = (cut >> 1) | (nxc << 7);
    const uint32_t ends = kept & (~next_k | inert | next_i | next_c) & 0xFFu;
    const uint32_t inc = (uint32_t)wave_incl_scan((int)((uint32_t)__popc(starts) | ((uint32_t)__popc(ends) << 16)));
    ck = lane63((kept >> 7) & 1u);
    ci = lane63((inert >> 7) & 1u);
    return lane63(inc);
}
// the staged round's records: starts are segments [ns, ns + nst), ends [ne, ne + nen) (every
// record array written by consecutive lanes: each lane's own 0-8 segments were scattered
// partial-line stores to seven arrays, 5.5 ms on C8)
__device__ __forceinline__ void seg_write(const DevTables& T, const SegWs& G, uint32_t t, uint32_t base, uint32_t r0,
                                          uint32_t ns, uint32_t ne, uint32_t tot, bool defer_sf, const SegStage& seg_stg) {
    const int lane = lane_id();
    const uint32_t nst = tot & 0xFFFFu, nen = tot >> 16;
    for (uint32_t k = (uint32_t)lane; k < nst; k += WAVE) {
        const uint32_t x = seg_stg.st[k];
        const uint32_t s = base + ns + k;
        if (!SEG_BOUND(SB_SO, s, G.cap_seg)) continue;
        G.so[s] = r0 + (x & 0xFFFFu);
        uint32_t f = SF_HEAD;
        if ((x >> 16) & 1u) {  // an inert char's segment is final here: one token, no rounds
            // (its flags, start and meta are all any later kernel reads of it)
            const uint32_t b = T.byte_id[x >> 17];
            const uint32_t id = b == NONE ? T.unk_id : b;
            G.smeta[s] = sm_make(id, id, 1u, 0u);
            f |= SF_INERT;
        } else {
            G.spt[s] = t;
            G.sg[s] = s + 1;
        }
        if (!defer_sf || (f & SF_INERT)) G.sf[s] = f;  // (deferred: the lookups write it)
    }
    for (uint32_t k = (uint32_t)lane; k < nen; k += WAVE)
        if (SEG_BOUND(SB_SE, base + ne + k, G.cap_seg)) G.se[base + ne + k] = seg_stg.en[k];
}
// The segment memo lookup of every non-inert segment k in [k_lo, k_hi) (its bytes were just
// read: L2): a hit's meta and pool entry to its record, a miss (or > 16 B) to the list that
// iteration 0 encodes; from LDS for a one-round pretoken (k_lo = 0)
__device__ __forceinline__ void seg_lookups(const DevTables& T, const uint8_t* bytes, uint64_t limit, const SegWs& G,
                                            uint64_t pos, uint32_t base, uint32_t k_lo, uint32_t k_hi, bool lds,
                                            const SegStage& seg_stg, WaveList<SEG_WL>& miss) {
    const int lane = lane_id();
    for (uint32_t k0 = k_lo; k0 < k_hi; k0 += WAVE) {  // (wave-uniform: the list appends)
        const uint32_t k = k0 + (uint32_t)lane, sl = base + k;
        bool act = k < k_hi, hit = false;
        uint32_t b0 = 0, L = 0, f = 0;
        if (act) {
            if (lds) {
                const uint32_t x = seg_stg.st[k];
                act = !((x >> 16) & 1u);
                b0 = x & 0xFFFFu;
                L = seg_stg.en[k] - b0;
            } else {
                f = G.sf[sl];
                act = !(f & SF_INERT);
                b0 = G.so[sl];
                L = G.se[sl] - b0;
            }
        }
        uint64_t m = 0;
        uint32_t q = 0, hot = 0;
        if (act && L <= 16u) {
            hit = seg_memo_find(T, bytes, limit, pos + b0, L, m, q, hot);
            if (hit) G.smeta[sl] = m;
        }
        // (a miss's pool entry 0: k_seg_first tells hits by it before k_seg_enc writes the
        // misses' records)
        if (act) G.spool[sl] = hit ? q : 0u;
        // a one-round pretoken's flags are written here, with a hot hit's index; a longer
        // one's were written by seg_write: a hot hit's index is added (without it every
        // boundary of a pretoken of > 512 B took k_seg_first's full check: C10 3.8 ms)
        if (act && lds) G.sf[sl] = SF_HEAD | ((hit ? hot : 0u) << SF_HOT_SHIFT);
        if (act && !lds && hit && hot) G.sf[sl] = f | (hot << SF_HOT_SHIFT);
        miss.push(act && !hit, sl);
        miss.flush(G.ctr + SC_PEND, G.list[0], G.cap_list, G, WAVE);
    }
}

__global__ __launch_bounds__(64, 7) void k_seg_init(DevTables T, const uint8_t* __restrict__ bytes, uint64_t limit,
                                                 Scratch S, Deferred D, SegWs G) {
    __shared__ SegStage seg_stg;
    __shared__ uint32_t mbuf[SEG_WL];
    WaveList<SEG_WL> miss{mbuf, 0u};
    const bool look = T.smemo != nullptr && TKZ_SEG_FIRST;  // the segment memo lookups here (not in k_seg_first)
    const int lane = lane_id();
    const uint32_t n_long = *(volatile uint32_t*)D.lcnt;
    uint32_t a_next = 0, a_end = 0;  // the block's unused segment slots [a_next, a_end)
    for (uint32_t t = blockIdx.x; t < n_long; t += gridDim.x) {
        const uint64_t e = D.llist[t];
        const uint64_t pos = e & POS_MASK;
        uint32_t L = (uint32_t)(e >> LEN_SHIFT);
        if (L == LEN_ESC) L = S.prs()[pos];  // (k_encode: a long pretoken's length in its pr slot)
        bool ok = L <= SEG_MAX_L;
        if (lane == 0) G.plen[t] = L;  // (the pr slot is a group's token slot from here on)
        if (ok && L > SEGI_BIG) {  // a long one: k_seg_init_big, a block of waves on its pieces
            if (lane == 0) {  // (listed pretokens <= bytes / SEGI_BIG < cap_list)
                const uint32_t b = atomicAdd(G.ctr + SC_BIGI, 1u);
                if (SEG_BOUND(SB_LIST, b, G.cap_list)) G.join[b] = t;
            }
            continue;
        }
        uint32_t ck = 0, ci = 0;  // the kept / inert bit of the byte before the 512-B round
        auto stage = [&](uint32_t r0, bool& bad_any) -> uint32_t {
            return seg_stage(T, bytes, limit, pos, L, r0, ck, ci, bad_any, seg_stg);
        };
        auto write = [&](uint32_t base, uint32_t r0, uint32_t ns, uint32_t ne, uint32_t tot, bool defer_sf) {
            seg_write(T, G, t, base, r0, ns, ne, tot, defer_sf, seg_stg);
        };
        // a pretoken of one round (<= 512 B: the usual whole doc) is classified once and
        // written from LDS after its slots are known; a longer one counts its segments in
        // a first pass and classifies every round again to write it
        const bool one = L <= (uint32_t)GROUP;
        uint32_t n_seg = 0, tot1 = 0;
        if (ok && one) {
            bool bad;
            tot1 = stage(0, bad);
            ok = !bad;
            n_seg = tot1 & 0xFFFFu;
        }
        for (uint32_t r0 = 0; !one && ok && r0 < L; r0 += GROUP) {  // (pass 1: count only)
            const uint32_t o = r0 + 8u * (uint32_t)lane;
            WordBytes<2> v;
            v.load(bytes, pos + o, limit, T.norm);
            uint32_t bad = 0, inert, cut;
            const uint32_t kept = seg_classify(T, v, o, L, bad, inert, cut);
            ok = __ballot(bad) == 0ull;
            const uint32_t pk = (uint32_t)__shfl((int)kept, lane > 0 ? lane - 1 : 0, WAVE);
            const uint32_t pi = (uint32_t)__shfl((int)inert, lane > 0 ? lane - 1 : 0, WAVE);
            const uint32_t starts =
                seg_starts(kept, inert, cut, lane > 0 ? (pk >> 7) & 1u : ck, lane > 0 ? (pi >> 7) & 1u : ci);
            n_seg += lane63((uint32_t)wave_incl_scan(__popc(starts)));
            ck = lane63((kept >> 7) & 1u);
            ci = lane63((inert >> 7) & 1u);
        }
        ok = ok && n_seg >= 2;
        uint32_t base = 0;
        if (ok) {
            // segment slots from the block's current range (one atomic per SEG_ALLOC slots:
            // one per pretoken on a single counter serialised 1M pretokens in L2)
            if (n_seg > a_end - a_next) {
                // the rest of the old range is never used: unused slots hold sf 0 (iteration
                // 0 walks every slot handed out)
                for (uint32_t s = a_next + lane; s < a_end; s += WAVE) G.sf[s] = 0;
                // (ranges of at most a quarter of the capacity over all blocks: the unused
                // tails stay bounded on small batches)
                const uint32_t want = max(n_seg, (uint32_t)min((uint64_t)SEG_ALLOC, G.cap_seg / (4ull * gridDim.x)));
                uint32_t b = 0;
                if (lane == 0) b = atomicAdd(G.ctr + SC_SEGS, want);
                a_next = rfl(b);
                a_end = (uint64_t)a_next + want <= G.cap_seg ? a_next + want : a_next;
                if (a_end == a_next)  // past the capacity: the slots below it unused (sf 0)
                    for (uint64_t s = (uint64_t)a_next + lane; s < min((uint64_t)a_next + want, G.cap_seg); s += WAVE)
                        G.sf[s] = 0;
            }
            base = a_next;
            ok = n_seg <= a_end - a_next;
            if (ok) a_next += n_seg;
        }
        if (!ok) {
            if (lane == 0) {
                G.pst[t] = 2;
                D.flist[atomicAdd(D.fcnt, 1u)] = e;
            }
            continue;
        }
        if (lane == 0) {
            G.pst[t] = 0;
            G.pbase[t] = base;
            G.pn[t] = n_seg;
        }
        auto lookups = [&](uint32_t n, bool lds) { seg_lookups(T, bytes, limit, G, pos, base, 0u, n, lds, seg_stg, miss); };
        if (one) {
            write(base, 0, 0, 0, tot1, look);
            if (look) lookups(n_seg, true);
            continue;
        }
        // pass 2: the segments' records (each segment: iteration 0's group, a head)
        uint32_t ns = 0, ne = 0;
        ck = ci = 0;
        for (uint32_t r0 = 0; r0 < L; r0 += GROUP) {
            bool bad;
            const uint32_t tot = stage(r0, bad);
            write(base, r0, ns, ne, tot, false);
            ns += tot & 0xFFFFu;
            ne += tot >> 16;
        }
        if (look) {  // (the records just written by this wave's other lanes: stores complete first)
            __threadfence_block();
            lookups(n_seg, false);
        }
    }
    miss.flush(G.ctr + SC_PEND, G.list[0], G.cap_list, G, SEG_WL);
    for (uint32_t s = a_next + lane; s < a_end; s += WAVE) G.sf[s] = 0;
}

// Pretokens longer than SEGI_BIG (k_seg_init lists them in G.join), a block of SEGI_W waves
// each: k_seg_init's two passes over the pretoken's 512-B rounds run on pieces of >= SEGI_PR
// rounds in parallel (a 1-MB document was one wave's 4,096 serial rounds: C10 k_seg_init 19 ms
// per step). Pass 1 counts each piece's segment starts and ends (the carry into a piece is
// its previous byte's classes), wave 0 turns them into prefixes and allocates the pretoken's
// slots, pass 2 writes each piece's records at its prefix and looks its segments up.
__global__ __launch_bounds__(64 * SEGI_W) void k_seg_init_big(DevTables T, const uint8_t* __restrict__ bytes, uint64_t limit,
                                                              Scratch S, Deferred D, SegWs G) {
    __shared__ SegStage stg[SEGI_W];
    __shared__ uint32_t mbuf[SEGI_W][SEG_WL];
    __shared__ uint32_t cnt_s[SEGI_MAXP], cnt_e[SEGI_MAXP];
    __shared__ uint32_t res[4];  // bad / ok, base, n_seg
    const int lane = lane_id(), wv = (int)(threadIdx.x >> 6);
    WaveList<SEG_WL> miss{mbuf[wv], 0u};
    const bool look = T.smemo != nullptr && TKZ_SEG_FIRST;
    const uint32_t nb = min(*(volatile uint32_t*)(G.ctr + SC_BIGI), (uint32_t)G.cap_list);
    for (uint32_t b = blockIdx.x; b < nb; b += gridDim.x) {
        const uint32_t t = G.join[b];
        const uint64_t e = D.llist[t];
        const uint64_t pos = e & POS_MASK;
        const uint32_t L = G.plen[t];
        const uint32_t nr = (L + GROUP - 1u) / GROUP;
        const uint32_t pr = max(SEGI_PR, (nr + SEGI_MAXP - 1u) / SEGI_MAXP), np = (nr + pr - 1u) / pr;
        if (threadIdx.x == 0) res[0] = 0u;
        __syncthreads();
        for (uint32_t p = (uint32_t)wv; p < np; p += SEGI_W) {  // pass 1: counts
            const uint32_t r_lo = p * pr, r_hi = min(nr, r_lo + pr);
            uint32_t ck = 0, ci = 0;
            if (r_lo) seg_carry(T, bytes, pos, r_lo * GROUP - 1u, ck, ci);
            uint32_t cs = 0, ce = 0;
            bool bad_any = false;
            for (uint32_t r = r_lo; r < r_hi; ++r) {
                bool bad;
                const uint32_t tot = seg_count_round(T, bytes, limit, pos, L, r * GROUP, ck, ci, bad);
                cs += tot & 0xFFFFu;
                ce += tot >> 16;
                bad_any = bad_any || bad;
            }
            if (lane == 0) {
                cnt_s[p] = cs;
                cnt_e[p] = ce;
                if (bad_any) res[0] = 1u;
            }
        }
        __syncthreads();
        if (wv == 0) {
            uint32_t run_s = 0, run_e = 0;
            for (uint32_t p0 = 0; p0 < np; p0 += WAVE) {
                const uint32_t p = p0 + (uint32_t)lane;
                const uint32_t cs = p < np ? cnt_s[p] : 0u, ce = p < np ? cnt_e[p] : 0u;
                const uint32_t is = (uint32_t)wave_incl_scan((int)cs), ie = (uint32_t)wave_incl_scan((int)ce);
                if (p < np) {
                    cnt_s[p] = run_s + is - cs;
                    cnt_e[p] = run_e + ie - ce;
                }
                run_s += lane63(is);
                run_e += lane63(ie);
            }
            if (lane == 0) {
                bool ok = res[0] == 0u && run_s >= 2u;
                uint32_t base = 0;
                if (ok) {
                    base = atomicAdd(G.ctr + SC_SEGS, run_s);
                    if ((uint64_t)base + run_s > G.cap_seg) {
                        ok = false;
                        res[3] = 1u;  // (slots handed out past the capacity: sf 0 below it)
                    } else {
                        res[3] = 0u;
                    }
                } else {
                    res[3] = 0u;
                }
                res[0] = ok ? 1u : 0u;
                res[1] = base;
                res[2] = run_s;
            }
        }
        __syncthreads();
        const bool ok = res[0] != 0u;
        const uint32_t base = res[1], n_seg = res[2];
        if (!ok) {
            if (res[3])  // (iteration 0 walks every slot handed out: unused ones hold sf 0)
                for (uint64_t sl = (uint64_t)base + threadIdx.x; sl < G.cap_seg; sl += blockDim.x) G.sf[sl] = 0;
            if (threadIdx.x == 0) {
                G.pst[t] = 2;
                D.flist[atomicAdd(D.fcnt, 1u)] = e;
            }
            __syncthreads();
            continue;
        }
        for (uint32_t p = (uint32_t)wv; p < np; p += SEGI_W) {  // pass 2: records, lookups
            const uint32_t r_lo = p * pr, r_hi = min(nr, r_lo + pr);
            uint32_t ck = 0, ci = 0;
            if (r_lo) seg_carry(T, bytes, pos, r_lo * GROUP - 1u, ck, ci);
            uint32_t ns = cnt_s[p], ne = cnt_e[p];
            const uint32_t ns0 = ns;
            for (uint32_t r = r_lo; r < r_hi; ++r) {
                bool bad;
                const uint32_t tot = seg_stage(T, bytes, limit, pos, L, r * GROUP, ck, ci, bad, stg[wv]);
                seg_write(T, G, t, base, r * GROUP, ns, ne, tot, false, stg[wv]);
                ns += tot & 0xFFFFu;
                ne += tot >> 16;
            }
            if (look) {  // (the records just written by this wave's other lanes: stores complete first)
                __threadfence_block();
                seg_lookups(T, bytes, limit, G, pos, base, ns0, ns, false, stg[wv], miss);
            }
        }
        if (threadIdx.x == 0) {
            G.pst[t] = 0;
            G.pbase[t] = base;
            G.pn[t] = n_seg;
        }
        __syncthreads();
    }
    miss.flush(G.ctr + SC_PEND, G.list[0], G.cap_list, G, SEG_WL);
}

// Iteration 0 with the segment memo: lane per segment, a wave over 63 consecutive segments
// (lane 63 reads the next one as the right neighbour of lane 62). k_seg_init looked every
// segment up in the memo (a hit's meta and pool entry are in its record; the misses are
// listed for k_seg_enc / k_seg_check, which check both their boundaries); here the
// boundary between two hits is checked. Between two hot hits it is one bit of the hot-pair
// bitmap; the other boundaries are queued per wave and checked 64 at a time (a lane's
// walk and probes ran while the hot lanes of its wave idled). Inert segments are final (no
// boundary of theirs is ever crossed); a tokenizer whose cuts are all inert skips this.
template <bool COMPACT>
__global__ __launch_bounds__(256, 6) void k_seg_first(DevTables T, const uint8_t* __restrict__ bytes, uint64_t limit,
                                                   Deferred D, SegWs G) {
    __shared__ uint32_t lbuf[4][SEG_WL];
    __shared__ uint32_t cbuf[4][2 * WAVE];  // a wave's boundaries (left segment) for the full check
    const int lane = lane_id();
    WaveList<SEG_WL> join{lbuf[threadIdx.x >> 6], 0u};
    uint32_t* cq = cbuf[threadIdx.x >> 6];
    uint32_t nq = 0;  // (wave-uniform)
    const uint32_t hk = T.hot_bits ? T.hot_k : 0u;
    extern __shared__ uint32_t over_lds[];
    const uint32_t* ov = seg_over_stage(T, over_lds);
    // the full check of the last cnt queued boundaries (s, s + 1), a lane each
    auto full = [&](uint32_t cnt) {
        WAVE_SYNC();
        const bool act = (uint32_t)lane < cnt;
        const uint32_t s = act ? cq[nq - cnt + (uint32_t)lane] : 0u;
        WAVE_SYNC();
        nq -= cnt;
        bool cr = false;
        if (act) {
            const uint64_t m = G.smeta[s], mn = G.smeta[s + 1];
            const uint32_t q = G.spool[s], qn = G.spool[s + 1];
            SegEdges E, En;
            E.load_pool(T, q, sm_re(m), 0u);
            En.load_pool(T, qn, 0u, sm_le(mn));
#if TKZ_FULL_ABL == 1  // timing only: the loads, no walk (wrong results)
            cr = (E.r[0] ^ En.l[0] ^ (uint32_t)m ^ (uint32_t)mn) == 0x12345678u;
#else
            cr = seg_crossed_core<COMPACT>(T, m, mn, E, En, ov);
#endif
        }
        // (an atomic OR: segment s + 1 may be the next wave's lane 0, which reads its hot
        // index from the same word -- a plain store erased it)
        if (cr) atomicOr(G.sf + s + 1, SF_JOINED);
        join.push(cr, s);
        join.flush(G.ctr + SC_JOIN, G.join, G.cap_list, G, WAVE);
    };
    const uint32_t n = (uint32_t)min((uint64_t)*(volatile uint32_t*)(G.ctr + SC_SEGS), G.cap_seg);
    const uint32_t nw = (n + (WAVE - 2)) / (WAVE - 1);
    const uint32_t wpb = blockDim.x >> 6;
    for (uint32_t w0 = blockIdx.x * wpb; w0 < nw; w0 += gridDim.x * wpb) {
        const uint32_t w = w0 + (threadIdx.x >> 6);
        const uint32_t s = (WAVE - 1) * w + (uint32_t)lane;
        const bool in = w < nw && s < n;
        const uint32_t sf = in ? G.sf[s] : 0u, t0 = in ? G.spt[s] : 0u, q0 = in ? G.spool[s] : 0u;
        const bool v = sf != 0u;  // (unused slots: sf 0)
        const bool inert = (sf & SF_INERT) != 0u;
        const uint32_t t = v ? t0 : ~0u;
        const bool hit = v && !inert && q0 != 0u;
        const uint32_t hot = hit ? sf >> SF_HOT_SHIFT : 0u;  // (hot index + 1)
        const bool own = v && lane < WAVE - 1;  // (lane 63: the next wave's segment)
        // the boundary (s, s + 1) between two hits of one pretoken (an inert one has no pool entry)
        const int nx = lane + 1 < WAVE ? lane + 1 : lane;
        const uint32_t tn = (uint32_t)__shfl((int)t, nx, WAVE);
        const uint32_t hn = (uint32_t)__shfl((int)(hit ? 1u : 0u), nx, WAVE);
        const uint32_t hotn = (uint32_t)__shfl((int)hot, nx, WAVE);
        const bool both = own && hit && hn != 0u && tn == t;
        // (hot indices past the bitmap's k: the memo ranks more keys than a smaller bitmap,
        // tkz_set_hot_pairs / the memory budget, holds)
        const bool hh = both && hot != 0u && hotn != 0u && hot <= hk && hotn <= hk;
        bool cr = false;
        if (hh) {
            const uint32_t x = (hot - 1u) * hk + (hotn - 1u);
            cr = ((T.hot_bits[x >> 5] >> (x & 31u)) & 1u) != 0u;
        }
        const bool rest = both && !hh;
        const uint64_t mq = __ballot(rest);
        if (rest && SEG_BOUND(SB_QUEUE, nq + lane_mbcnt(mq), 2 * WAVE)) cq[nq + lane_mbcnt(mq)] = s;
        nq += (uint32_t)__popcll(mq);
        if (cr && SEG_BOUND(SB_FLAG, s + 1, n)) atomicOr(G.sf + s + 1, SF_JOINED);  // (as in full())
        join.push(cr, s);
        join.flush(G.ctr + SC_JOIN, G.join, G.cap_list, G, WAVE);  // (<= 63 entries per push)
        if (nq >= (uint32_t)WAVE) full(WAVE);
    }
    if (nq) full(nq);
    join.flush(G.ctr + SC_JOIN, G.join, G.cap_list, G, SEG_WL);
}

// Iteration `it`: encodes the listed heads' groups (iteration 0: every segment but the
// inert ones, in index order), 256 per block counting-sorted by byte length so a wave's
// lanes share W.
#ifndef TKZ_SEG_ENC_MINW
#define TKZ_SEG_ENC_MINW 4  // waves per SIMD k_seg_enc is fitted to (4: 128 VGPRs, 6 spilled; vs 3: C6 -1.5 %, C9 -1.8 %, r05j)
#endif
template <bool COMPACT>
__global__ __launch_bounds__(256, TKZ_SEG_ENC_MINW) void k_seg_enc(DevTables T, const uint8_t* __restrict__ bytes, uint64_t limit,
                                                 Scratch S, Deferred D, SegWs G, int it) {
    // a round's groups counting-sorted by length class with their records (group, its end
    // segment, byte range, pretoken position): each record read once, its loads issued in
    // two rounds (the encode re-read them behind a chain of dependent loads)
    __shared__ struct {
        uint32_t g[256], e[256], b0[256], b1[256], plo[256], phi[256];
    } srt;
    __shared__ uint32_t hist[4];
    __shared__ BlockList<1024> big;
    const int tid = threadIdx.x;
    big.init();
    const bool all = it == 0 && (T.smemo == nullptr || !TKZ_SEG_FIRST);  // every segment slot in index order (else the list)
    const uint32_t n = all ? (uint32_t)min((uint64_t)*(volatile uint32_t*)(G.ctr + SC_SEGS), G.cap_seg)
                           : min(*(volatile uint32_t*)(G.ctr + SC_PEND + it), (uint32_t)G.cap_list);
    const uint32_t* lst = G.list[it & 1];
    for (uint32_t k0 = (uint32_t)blockIdx.x * 256u; k0 < n; k0 += gridDim.x * 256u) {
        const uint32_t k = k0 + (uint32_t)tid;
        uint32_t g = 0, cls = 4, e = 0, b0 = 0, b1 = 0;
        uint64_t pos = 0;
        if (k < n) {
            g = all ? k : lst[k];
            const uint32_t f = all ? G.sf[g] : SF_HEAD;
            const uint32_t t = G.spt[g];
            e = G.sg[g];
            b0 = G.so[g];
            if (f != 0u && !(f & SF_INERT)) {  // (unused slots have sf 0)
                const uint32_t st = G.pst[t];
                pos = D.llist[t] & POS_MASK;
                b1 = G.se[e - 1];
                if (st == 0) {
                    const uint32_t len = b1 - b0;
                    cls = len <= 4u ? 0u : len <= 8u ? 1u : len <= 255u ? 2u : 3u;
                }
            }
        }
        if (tid < 4) hist[tid] = 0;
        __syncthreads();
        uint32_t slot = 0;
        if (cls < 4) slot = atomicAdd(&hist[cls], 1u);
        __syncthreads();
        if (cls < 4) {
            uint32_t off = 0;
            for (uint32_t c = 0; c < cls; ++c) off += hist[c];
            const uint32_t o = off + slot;
            srt.g[o] = g;
            srt.e[o] = e;
            srt.b0[o] = b0;
            srt.b1[o] = b1;
            srt.plo[o] = (uint32_t)pos;
            srt.phi[o] = (uint32_t)(pos >> 32);
        }
        const uint32_t m = hist[0] + hist[1] + hist[2] + hist[3];
        __syncthreads();
        const uint32_t q = (uint32_t)tid;
        const bool act = q < m;
        const uint32_t gq = act ? srt.g[q] : 0u, eq = act ? srt.e[q] : 0u;
        const uint32_t b0q = act ? srt.b0[q] : 0u, b1q = act ? srt.b1[q] : 0u;
        const uint64_t posq = act ? ((uint64_t)srt.phi[q] << 32) | srt.plo[q] : 0ull;
        const uint32_t len = b1q - b0q;
        __syncthreads();  // (the next round's sort overwrites srt)
        // the wave's longest group picks W (uniform)
        uint32_t lm = act ? len : 0u;
        lm = max(lm, (uint32_t)__shfl_xor((int)lm, 1, WAVE));
        lm = max(lm, (uint32_t)__shfl_xor((int)lm, 2, WAVE));
        lm = max(lm, (uint32_t)__shfl_xor((int)lm, 4, WAVE));
        lm = max(lm, (uint32_t)__shfl_xor((int)lm, 8, WAVE));
        lm = max(lm, (uint32_t)__shfl_xor((int)lm, 16, WAVE));
        lm = max(lm, (uint32_t)__shfl_xor((int)lm, 32, WAVE));
        lm = rfl(lm);
        bool done = false;
        if (lm <= 4u) done = seg_encode<4, 1, COMPACT>(T, bytes, limit, G, S, posq, gq, b0q, b1q, act);
        else if (lm <= 8u) done = seg_encode<8, 1, COMPACT>(T, bytes, limit, G, S, posq, gq, b0q, b1q, act);
        else done = seg_encode<16, 4, COMPACT>(T, bytes, limit, G, S, posq, gq, b0q, b1q, act && len <= 255u);
        (void)eq;
        // groups of more than 16 symbols (or 255 bytes): listed for k_seg_enc_big, in the
        // next iteration's list (free until k_seg_join refills it; the join list holds
        // k_seg_first's entries in iteration 0)
        big.push(act && !done, gq);
        if (act && it > 0) G.sf[gq] = SF_HEAD;  // (PEND cleared; only this lane touches sf[gq] in this kernel)
        big.flush(G.ctr + SC_BIG + it, G.list[(it + 1) & 1], G.cap_list, G, blockDim.x);
    }
    big.flush(G.ctr + SC_BIG + it, G.list[(it + 1) & 1], G.cap_list, G, 1024);
}

// Iteration `it`: the listed groups of more than 16 symbols, lane per group with W = 32
// (a group of 17..32 symbols costs its lane what a wave-wide encode costs the whole wave:
// the rounds are probe-latency bound, so 64 groups at a time, not one); the wave's groups
// of more than 32 symbols then one at a time with the whole wave (<= 64; more: fallback).
#ifndef TKZ_SEG_WAVE_LIST
#define TKZ_SEG_WAVE_LIST 1  // k_seg_enc_big lists its wave-path groups for k_seg_enc_wave (0: encodes them itself)
#endif
#ifndef TKZ_SEG_BIG_MINW
#define TKZ_SEG_BIG_MINW 3  // waves per SIMD k_seg_enc_big is fitted to (3: 168 VGPRs, some spilled; vs 2 at 235 VGPRs: C6 +2.5 %, C9 +1.4 %; 4: slower)
#endif
template <bool COMPACT>
__global__ __launch_bounds__(256, TKZ_SEG_BIG_MINW) void k_seg_enc_big(DevTables T, const uint8_t* __restrict__ bytes, uint64_t limit,
                                                     Scratch S, Deferred D, SegWs G, int it) {
    __shared__ uint32_t stg[4][3 * SEGW_MAX];
    const int lane = lane_id(), wv = threadIdx.x >> 6;
    const uint32_t n = min(*(volatile uint32_t*)(G.ctr + SC_BIG + it), (uint32_t)G.cap_list);
    const uint32_t n_pad = (n + 255u) & ~255u;
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n_pad; k += gridDim.x * blockDim.x) {
        const bool act = k < n;
        const uint32_t g = act ? G.list[(it + 1) & 1][k] : 0u;
        const uint32_t len = act ? G.se[G.sg[g] - 1] - G.so[g] : 0u;
        const uint64_t pos = act ? seg_pos(D, G, g) : 0ull;
        const uint32_t e = act ? G.sg[g] : 0u;
        const bool done =
            TKZ_SEG_W32 && seg_encode<32, 8, COMPACT>(T, bytes, limit, G, S, pos, g, act ? G.so[g] : 0u,
                                                      act ? G.so[g] + len : 0u, act && len <= 255u);
        if (TKZ_SEG_WAVE_LIST) {
            // groups of > 32 symbols (or > 255 B) to k_seg_enc_wave, one wave each, listed after
            // this iteration's big list in the same array (a wave here encoded its own ones one
            // after another: a latency chain per group, and this kernel's 168 VGPRs for it)
            const uint64_t mb = __ballot(act && !done);
            if (mb) {
                uint32_t b = 0;
                if (lane == 0) b = atomicAdd(G.ctr + SC_WAV + it, (uint32_t)__popcll(mb));
                b = rfl(b);
                if (act && !done) {
                    const uint64_t i = (uint64_t)n + b + lanes_below(mb);
                    if (SEG_BOUND(SB_LIST, i, G.cap_list) && i < G.cap_list) G.list[(it + 1) & 1][i] = g;
                    else G.pst[G.spt[g]] = 1;  // (past the list's capacity: the pretoken falls back)
                }
            }
            continue;
        }
        for (uint64_t mb = __ballot(act && !done); mb; mb &= mb - 1ull) {
            const int ln = __ffsll((long long)mb) - 1;
            const uint32_t gb = (uint32_t)__shfl((int)g, ln, WAVE);
            const uint64_t pb = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(pos >> 32), ln, WAVE) << 32) |
                                (uint32_t)__shfl((int)(uint32_t)pos, ln, WAVE);
            const uint32_t eb = (uint32_t)__shfl((int)e, ln, WAVE);
            if (!seg_encode_wave<COMPACT>(T, bytes, limit, G, S, pb, gb, eb, stg[wv]) && lane == 0)
                G.pst[G.spt[gb]] = 1;
        }
    }
}

// Iteration `it`: the groups k_seg_enc_big listed for the wave path (> 32 symbols or > 255 B),
// one wave each (seg_encode_wave: 64 symbols per slot, up to 512)
template <bool COMPACT>
__global__ __launch_bounds__(64) void k_seg_enc_wave(DevTables T, const uint8_t* __restrict__ bytes, uint64_t limit,
                                                     Scratch S, Deferred D, SegWs G, int it) {
    __shared__ uint32_t stg[3 * SEGW_MAX];
    const uint32_t nb = min(*(volatile uint32_t*)(G.ctr + SC_BIG + it), (uint32_t)G.cap_list);
    const uint32_t n = min(*(volatile uint32_t*)(G.ctr + SC_WAV + it), (uint32_t)(G.cap_list - nb));
    for (uint32_t w = blockIdx.x; w < n; w += gridDim.x) {
        const uint32_t g = G.list[(it + 1) & 1][nb + w];
        const uint64_t pos = seg_pos(D, G, g);
        const uint32_t e = G.sg[g];
        if (!seg_encode_wave<COMPACT>(T, bytes, limit, G, S, pos, g, e, stg) && lane_id() == 0) G.pst[G.spt[g]] = 1;
        WAVE_SYNC();
    }
}

// Iteration `it`: the boundaries of the groups encoded in it (iteration 0: every segment's
// right boundary; later: the listed heads' right and left boundaries). A crossed boundary
// marks its right group sf_jit(it); the left-head walks read the earlier iterations' bits
// only (the groups as this iteration found them), so no lane reads a flag another lane of
// this launch sets and the outcome is the same on every run.
#ifndef TKZ_SEG_CHECK_MINW
#define TKZ_SEG_CHECK_MINW 5
#endif
template <bool COMPACT>
__global__ __launch_bounds__(256, TKZ_SEG_CHECK_MINW) void k_seg_check(DevTables T, Scratch S, Deferred D, SegWs G, int it) {
    const bool all = it == 0 && (T.smemo == nullptr || !TKZ_SEG_FIRST);  // as k_seg_enc
    const uint32_t n = all ? (uint32_t)min((uint64_t)*(volatile uint32_t*)(G.ctr + SC_SEGS), G.cap_seg)
                           : min(*(volatile uint32_t*)(G.ctr + SC_PEND + it), (uint32_t)G.cap_list);
    __shared__ uint32_t lbuf[4][SEG_WL];
    WaveList<SEG_WL> join{lbuf[threadIdx.x >> 6], 0u};
    extern __shared__ uint32_t over_lds[];
    const uint32_t* ov = seg_over_stage(T, over_lds);
    const uint32_t* lst = G.list[it & 1];
    const uint32_t n_pad = (n + 63u) & ~63u;  // whole waves in the loop (wave-aggregated appends)
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n_pad; k += gridDim.x * blockDim.x) {
        uint32_t g = 0, t = 0;
        bool act = k < n;
        if (act) {
            g = all ? k : lst[k];
            if (all) {
                const uint32_t f = G.sf[g];
                act = f != 0u && !(f & SF_INERT);
            }
        }
        if (act) {
            t = G.spt[g];
            act = G.pst[t] == 0;
        }
        uint32_t ja = 0, jb = 0;  // the left heads of this lane's crossed boundaries (+1; 0 = none)
        if (act) {
            // every record both checks read, in two rounds of loads issued together (the
            // checks' loads behind their conditions made a chain of ~6 round trips per lane)
            const uint32_t e = G.sg[g], qg = G.spool[g], sog = G.so[g];
            const uint64_t mg = G.smeta[g];
            const uint32_t cap = (uint32_t)min(G.cap_seg, (uint64_t)0xFFFFFFFFu);
            const uint32_t ec = e < cap ? e : g, pc = g > 0u ? g - 1u : g;
            const uint64_t pos = D.llist[t] & POS_MASK;
            const uint32_t first = G.pbase[t], end = first + G.pn[t];
            const uint32_t sfe = G.sf[ec], qe = G.spool[ec], soe = G.so[ec];
            const uint64_t me = G.smeta[ec];
            uint32_t p = pc, sfp = G.sf[pc], qp = G.spool[pc], sop = G.so[pc];
            uint64_t mp = G.smeta[pc];
            auto edges = [&](uint32_t q, uint32_t so, uint32_t nre, uint32_t nle) {
                SegEdges E;
                if (q) E.load_pool(T, q, nre, nle);
                else E.load_scratch(S.offs() + pos + so, nre, nle);
                return E;
            };
            const SegEdges Eg = edges(qg, sog, sm_re(mg), sm_le(mg));
            if (e < end && !(sfe & SF_INERT) &&
                seg_crossed_core<COMPACT>(T, mg, me, Eg, edges(qe, soe, 0u, sm_le(me)), ov)) {
                atomicOr(G.sf + e, sf_jit(it));
                ja = g + 1;
            }
            // the left boundary (iteration 0 with the memo: the previous segment if it is a
            // hit; a miss checks it as its right one)
            if (it > 0 && g > first && (sfp & sf_jbefore(it))) {  // the previous head (the first segment is never joined)
                do --p;
                while (G.sf[p] & sf_jbefore(it));
                sfp = G.sf[p];
                qp = G.spool[p];
                sop = G.so[p];
                mp = G.smeta[p];
            }
            if (!all && g > first && (it > 0 || qp != 0u) && !(sfp & SF_INERT)) {
                if (seg_crossed_core<COMPACT>(T, mp, mg, edges(qp, sop, sm_re(mp), 0u), Eg, ov)) {
                    atomicOr(G.sf + g, sf_jit(it));
                    jb = p + 1;
                }
            }
        }
        join.push(ja != 0u, ja - 1u);
        join.push(jb != 0u, jb - 1u);
        join.flush(G.ctr + SC_JOIN + it, G.join, G.cap_list, G, 2 * WAVE);
    }
    join.flush(G.ctr + SC_JOIN + it, G.join, G.cap_list, G, SEG_WL);
}

// Iteration `it`: each crossed boundary's left head (not itself joined) takes the groups
// joined to its right and is listed for iteration it + 1 (in the last iteration its
// pretoken falls back instead)
__global__ __launch_bounds__(256) void k_seg_join(Deferred D, SegWs G, int it) {
    (void)D;  // (one list entry per lane; appends to the next pending list per block)
    __shared__ uint32_t lbuf[4][SEG_WL];
    WaveList<SEG_WL> pend{lbuf[threadIdx.x >> 6], 0u};
    const uint32_t n = min(*(volatile uint32_t*)(G.ctr + SC_JOIN + it), (uint32_t)G.cap_list);
    const uint32_t n_pad = (n + 63u) & ~63u;
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n_pad; k += gridDim.x * blockDim.x) {
        bool lst = false;
        uint32_t p = 0, t = 0;
        if (k < n) {
            p = G.join[k];
            t = G.spt[p];
            if (!(G.sf[p] & SF_JANY) && G.pst[t] == 0) {
                const uint32_t end = G.pbase[t] + G.pn[t];
                uint32_t e = G.sg[p];
                while (e < end) {
                    const uint32_t f = G.sf[e];
                    if (!(f & SF_JANY)) break;
                    // (joined in this iteration: an earlier one's for the next check; every
                    // group joined in it lies on the walk of some listed left head)
                    if ((f & (SF_JNEW | SF_JOLD)) == SF_JNEW) atomicOr(G.sf + e, SF_JOLD);
                    e = G.sg[e];
                }
                // (a head listed twice: by its own crossed boundary and a joined neighbour's
                // -- from iteration 1 on; iteration 0 checks every boundary once and lists its
                // left segment, so no head is listed twice and no atomic is needed)
                if (e != G.sg[p] && (it == 0 || !(atomicOr(G.sf + p, SF_PEND) & SF_PEND)) &&
                    SEG_BOUND(SB_JOIN, p, G.cap_seg)) {
                    G.sg[p] = e;
                    lst = true;
                }
            }
        }
        if (it + 1 >= SEG_ITERS) {  // still joining after the last iteration: falls back
            if (lst) G.pst[t] = 1;
            continue;
        }
        pend.push(lst, p);
        pend.flush(G.ctr + SC_PEND + it + 1, G.list[(it + 1) & 1], G.cap_list, G, WAVE);
    }
    if (it + 1 < SEG_ITERS) pend.flush(G.ctr + SC_PEND + it + 1, G.list[(it + 1) & 1], G.cap_list, G, SEG_WL);
}

#ifdef TKZ_SEG_STATS
// debug: the segmented path's list sizes to the header's debug words (segments, the pending
// lists of iterations 0-3, the join lists of 0-2, the big lists of 0-2, the wave list of 1;
// tools/seg_stats.py)
__global__ void k_seg_stats(Deferred D, SegWs G) {
    const int i = threadIdx.x;
    if (i >= 12) return;
    const int src[12] = {SC_SEGS, SC_PEND, SC_PEND + 1, SC_PEND + 2, SC_PEND + 3, SC_JOIN, SC_JOIN + 1,
                         SC_JOIN + 2, SC_BIG, SC_BIG + 1, SC_BIG + 2, SC_WAV + 1};
    D.dbg[i] += G.ctr[src[i]];
}
#endif

// One wave per long pretoken (tokenizers whose pretokenizer splits: a long pretoken is rare
// there, and the compaction copies it): the groups' tokens in order (wide, at ids /
// offs[pos..]) and the word record; failed pretokens to D.flist
__global__ __launch_bounds__(64) void k_seg_out(DevTables T, Scratch S, Deferred D, SegWs G) {
    // Rounds of 128 segments, two per lane, their record loads issued together; a round's
    // tokens staged in LDS, then stored by consecutive lanes (the lanes' own runs of 1-3
    // tokens were scattered partial-line stores)
    constexpr uint32_t STG = 512;
    __shared__ uint32_t sid[STG], ssa[STG];  // id | length << 20, start (32-bit pretoken offset): 4 KiB, 8 waves per SIMD
    const int lane = lane_id();
    const uint32_t n_long = *(volatile uint32_t*)D.lcnt;
    uint32_t taken = 0;
    for (uint32_t t = blockIdx.x; t < n_long; t += gridDim.x) {
        const uint32_t st = G.pst[t];
        const uint64_t e = D.llist[t];
        const uint32_t first = G.pbase[t], ns = G.pn[t];
        if (st == 2) continue;
        if (st == 1) {
            if (lane == 0) {
                // (its first group's tokens may have taken the pr slot of its length)
                if ((uint32_t)(e >> LEN_SHIFT) == LEN_ESC) S.prs()[e & POS_MASK] = G.plen[t];
                D.flist[atomicAdd(D.fcnt, 1u)] = e;
            }
            continue;
        }
        const uint64_t pos = e & POS_MASK;
        const uint64_t ws = S.slot(pos, (uint32_t)(e >> POS_BITS) & ORD_MASK);
        uint32_t base = 0;
        for (uint32_t s0 = 0; s0 < ns; s0 += 2 * WAVE) {
            uint32_t c[2], b0[2], q[2], f0[2], np[2];
            bool hd[2], in[2];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const uint32_t i = s0 + (uint32_t)lane + (uint32_t)j * WAVE;
                const uint32_t s = first + (i < ns ? i : 0u);
                const uint32_t f = G.sf[s];
                const uint64_t m = G.smeta[s];
                b0[j] = G.so[s];
                q[j] = G.spool[s];
                hd[j] = i < ns && !(f & SF_JANY);
                in[j] = (f & SF_INERT) != 0u;
                f0[j] = sm_first(m);
                np[j] = max(sm_le(m), sm_re(m));  // (a pool entry: its edge pairs, then the tokens)
                c[j] = hd[j] ? sm_ntok(m) : 0u;
            }
            const uint32_t i0 = (uint32_t)wave_incl_scan((int)c[0]);
            const uint32_t t0 = lane63(i0);
            const uint32_t i1 = (uint32_t)wave_incl_scan((int)c[1]) + t0;
            const uint32_t tot = lane63(i1);
            const bool stage = tot <= STG && T.max_key < 4096u;  // (uniform; a token spans <= max_key bytes)
            uint32_t* ids = S.ids() + pos + base;
            uint64_t* offs = S.offs() + pos + base;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                if (hd[j] && c[j]) {
                    const uint32_t o = (j ? i1 : i0) - c[j];
                    // (memo hits: key-relative tokens in the pool; inert: the char's one
                    // token; else tok / prs)
                    const uint32_t* pl = q[j] ? T.smpool + (q[j] - 1u) + 2u * np[j] : S.tok() + pos + b0[j];
                    const uint32_t* pe = S.prs() + pos + b0[j];
                    for (uint32_t k = 0; k < c[j]; ++k) {
                        uint32_t id = f0[j], a = b0[j], z = b0[j] + 1u;
                        if (!in[j]) {
                            const uint32_t x = pl[k];
                            const uint32_t y = q[j] ? 0u : pe[k];
                            id = q[j] ? x & 0xFFFFFu : x;
                            a = b0[j] + (q[j] ? (x >> 20) & 63u : y & 0xFFFFu);
                            z = b0[j] + (q[j] ? x >> 26 : y >> 16);
                        }
                        if (stage && SEG_BOUND(SB_EMIT, o + k, STG)) {
                            sid[o + k] = id | ((z - a) << 20);  // (ids < 2^20; a token < 4096 B: checked below)
                            ssa[o + k] = a;
                        } else {
                            ids[o + k] = id;
                            offs[o + k] = (uint64_t)a | ((uint64_t)z << 32);
                        }
                    }
                }
            }
            if (stage) {
                WAVE_SYNC();
                for (uint32_t j = (uint32_t)lane; j < tot; j += WAVE) {
                    ids[j] = sid[j] & 0xFFFFFu;
                    offs[j] = (uint64_t)ssa[j] | ((uint64_t)(ssa[j] + (sid[j] >> 20)) << 32);
                }
                WAVE_SYNC();
            }
            base += tot;
        }
        WAVE_SYNC();
        if (lane == 0) S.wide(ws, pos, base);
        ++taken;
    }
    if (lane == 0 && taken) atomicAdd(D.seg_words, (unsigned long long)taken);
}

// Whole-text pretokenizers (T.pretok == 0: every doc is a long pretoken): one wave per
// pretoken, before the scan: the token count of its groups to its word record (REC_SEG);
// failed pretokens to D.flist (k_bpe_long)
__global__ __launch_bounds__(64) void k_seg_count(Scratch S, Deferred D, SegWs G) {
    const int lane = lane_id();
    const uint32_t n_long = *(volatile uint32_t*)D.lcnt;
    uint32_t taken = 0;
    for (uint32_t t = blockIdx.x; t < n_long; t += gridDim.x) {
        const uint32_t st = G.pst[t];
        const uint64_t e = D.llist[t];
        const uint32_t first = G.pbase[t], ns = G.pn[t];
        if (st == 2) continue;
        if (st == 1) {
            if (lane == 0) {
                // (its first group's tokens may have taken the pr slot of its length)
                if ((uint32_t)(e >> LEN_SHIFT) == LEN_ESC) S.prs()[e & POS_MASK] = G.plen[t];
                D.flist[atomicAdd(D.fcnt, 1u)] = e;
            }
            continue;
        }
        const uint64_t pos = e & POS_MASK;
        const uint64_t ws = S.slot(pos, (uint32_t)(e >> POS_BITS) & ORD_MASK);
        if (ns > SEG_BIGP) {  // many segments: k_seg_count_big / k_seg_emit_big, a block each
            if (lane == 0) {  // (listed pretokens <= bytes / (2 SEG_BIGP) < cap_list)
                const uint32_t b = atomicAdd(G.ctr + SC_BIGP, 1u);
                if (SEG_BOUND(SB_LIST, b, G.cap_list)) G.join[b] = t;
            }
            ++taken;
            continue;
        }
        uint32_t c = 0;
        for (uint32_t i = (uint32_t)lane; i < ns; i += WAVE) {
            const uint32_t f = G.sf[first + i];
            const uint64_t m = G.smeta[first + i];
            c += (f & SF_JANY) ? 0u : sm_ntok(m);
        }
        c = lane63((uint32_t)wave_incl_scan((int)c));
        if (lane == 0) S.seg(ws, pos, c);
        ++taken;
    }
    if (lane == 0 && taken) atomicAdd(D.seg_words, (unsigned long long)taken);
}

// One round of a segmented pretoken's emission (k_seg_emit / k_seg_emit_big): segments
// [s0, s0 + 128) of the ns from `first`, two per lane with their record loads issued
// together, their tokens staged in LDS (sid / ssa, SEG_STG entries) and stored by consecutive
// lanes at ids / offs (the round's first output token); returns the round's token count.
constexpr uint32_t SEG_STG = 512;
__device__ __forceinline__ uint32_t seg_emit_round(const DevTables& T, const Scratch& S, const SegWs& G, uint64_t pos,
                                                   uint32_t first, uint32_t ns, uint32_t s0, uint32_t* ids,
                                                   uint64_t* offs, uint32_t* sid, uint32_t* ssa) {
    const int lane = lane_id();
    uint32_t c[2], b0[2], q[2], f0[2], np[2];
    bool hd[2], in[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const uint32_t i = s0 + (uint32_t)lane + (uint32_t)j * WAVE;
        const uint32_t sg = first + (i < ns ? i : 0u);
        const uint32_t f = G.sf[sg];
        const uint64_t m = G.smeta[sg];
        b0[j] = G.so[sg];
        q[j] = G.spool[sg];
        hd[j] = i < ns && !(f & SF_JANY);
        in[j] = (f & SF_INERT) != 0u;
        f0[j] = sm_first(m);
        np[j] = max(sm_le(m), sm_re(m));  // (a pool entry: its edge pairs, then the tokens)
        c[j] = hd[j] ? sm_ntok(m) : 0u;
    }
    const uint32_t i0 = (uint32_t)wave_incl_scan((int)c[0]);
    const uint32_t t0 = lane63(i0);
    const uint32_t i1 = (uint32_t)wave_incl_scan((int)c[1]) + t0;
    const uint32_t tot = lane63(i1);
    const bool stage = tot <= SEG_STG && T.max_key < 4096u;  // (uniform; a token spans <= max_key bytes)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        if (hd[j] && c[j]) {
            const uint32_t o = (j ? i1 : i0) - c[j];
            // (memo hits: key-relative tokens in the pool; inert: the char's one token; else
            // tok / prs)
            const uint32_t* pl = q[j] ? T.smpool + (q[j] - 1u) + 2u * np[j] : S.tok() + pos + b0[j];
            const uint32_t* pe = S.prs() + pos + b0[j];
            for (uint32_t k = 0; k < c[j]; ++k) {
                uint32_t id = f0[j], a = b0[j], z = b0[j] + 1u;
                if (!in[j]) {
                    const uint32_t x = pl[k];
                    const uint32_t y = q[j] ? 0u : pe[k];
                    id = q[j] ? x & 0xFFFFFu : x;
                    a = b0[j] + (q[j] ? (x >> 20) & 63u : y & 0xFFFFu);
                    z = b0[j] + (q[j] ? x >> 26 : y >> 16);
                }
                if (stage && SEG_BOUND(SB_EMIT, o + k, SEG_STG)) {
                    sid[o + k] = id | ((z - a) << 20);  // (ids < 2^20; a token < 4096 B: checked above)
                    ssa[o + k] = a;
                } else {
                    ids[o + k] = id;
                    offs[o + k] = (uint64_t)a | ((uint64_t)z << 32);
                }
            }
        }
    }
    if (stage) {
        WAVE_SYNC();
        for (uint32_t j = (uint32_t)lane; j < tot; j += WAVE) {
            ids[j] = sid[j] & 0xFFFFFu;
            offs[j] = (uint64_t)ssa[j] | ((uint64_t)(ssa[j] + (sid[j] >> 20)) << 32);
        }
        WAVE_SYNC();
    }
    return tot;
}

// One wave per segmented pretoken, after the compaction: the groups' tokens in order to the
// output at the position k_compact_long left in offs[pos] (the token count is k_seg_count's:
// the same heads, the same counts). Pretokens of more than SEG_BIGP segments: k_seg_emit_big.
__global__ __launch_bounds__(64) void k_seg_emit(DevTables T, Scratch S, Deferred D, SegWs G, uint32_t* __restrict__ ids_out,
                                                uint64_t* __restrict__ offs_out) {
    // Rounds of 128 segments, two per lane, their record loads issued together; a round's
    // tokens staged in LDS, then stored by consecutive lanes (the lanes' own runs of 1-3
    // tokens were scattered partial-line stores)
    __shared__ uint32_t sid[SEG_STG], ssa[SEG_STG];  // id | length << 20, start (32-bit pretoken offset): 4 KiB, 8 waves per SIMD
    const uint32_t n_long = *(volatile uint32_t*)D.lcnt;
    for (uint32_t t = blockIdx.x; t < n_long; t += gridDim.x) {
        const uint32_t st = G.pst[t];
        const uint64_t e = D.llist[t];
        const uint32_t first = G.pbase[t], ns = G.pn[t];
        if (st != 0 || ns > SEG_BIGP) continue;
        const uint64_t pos = e & POS_MASK;
        const uint64_t oo = S.offs()[pos];  // (k_compact_long; read before any token is written)
        uint32_t base = 0;
        for (uint32_t s0 = 0; s0 < ns; s0 += 2 * WAVE)
            base += seg_emit_round(T, S, G, pos, first, ns, s0, ids_out + oo + base, offs_out + oo + base, sid, ssa);
        WAVE_SYNC();
    }
}

// Segmented pretokens of more than SEG_BIGP segments (k_seg_count lists them in G.join), a
// block of 8 waves each: a 1-MB document was one wave's serial work in k_seg_count /
// k_seg_emit (C10: 13.5 ms per step). k_seg_count_big: the waves count the tokens of 128-segment
// rounds in stripes, wave 0 turns the counts into exclusive prefixes (kept at
// G.sg[first + 128 r]: group ends are not read after the iterations) and writes the record;
// k_seg_emit_big: the waves emit the rounds in stripes at their prefixes.
__global__ __launch_bounds__(64 * SEGB_W) void k_seg_count_big(Scratch S, Deferred D, SegWs G) {
    const int lane = lane_id(), wv = (int)(threadIdx.x >> 6);
    const uint32_t nb = min(*(volatile uint32_t*)(G.ctr + SC_BIGP), (uint32_t)G.cap_list);
    for (uint32_t b = blockIdx.x; b < nb; b += gridDim.x) {
        const uint32_t t = G.join[b];
        const uint64_t e = D.llist[t];
        const uint32_t first = G.pbase[t], ns = G.pn[t];
        const uint32_t nr = (ns + 2u * WAVE - 1u) / (2u * WAVE);
        for (uint32_t r = (uint32_t)wv; r < nr; r += SEGB_W) {
            uint32_t c = 0;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const uint32_t i = r * 2u * WAVE + (uint32_t)lane + (uint32_t)j * WAVE;
                if (i < ns) {
                    const uint32_t f = G.sf[first + i];
                    c += (f & SF_JANY) ? 0u : sm_ntok(G.smeta[first + i]);
                }
            }
            c = lane63((uint32_t)wave_incl_scan((int)c));
            if (lane == 0) G.sg[first + r * 2u * WAVE] = c;
        }
        __syncthreads();
        if (wv == 0) {
            uint32_t run = 0;
            for (uint32_t r0 = 0; r0 < nr; r0 += WAVE) {
                const uint32_t r = r0 + (uint32_t)lane;
                const uint32_t c = r < nr ? G.sg[first + r * 2u * WAVE] : 0u;
                const uint32_t inc = (uint32_t)wave_incl_scan((int)c);
                if (r < nr) G.sg[first + r * 2u * WAVE] = run + inc - c;
                run += lane63(inc);
            }
            if (lane == 0) {
                const uint64_t pos = e & POS_MASK;
                S.seg(S.slot(pos, (uint32_t)(e >> POS_BITS) & ORD_MASK), pos, run);
            }
        }
        __syncthreads();
    }
}

constexpr int SEGE_W = 16;  // k_seg_emit_big's waves per block
__global__ __launch_bounds__(64 * SEGE_W) void k_seg_emit_big(DevTables T, Scratch S, Deferred D, SegWs G,
                                                              uint32_t* __restrict__ ids_out,
                                                              uint64_t* __restrict__ offs_out) {
    __shared__ uint32_t sid[SEGE_W][SEG_STG], ssa[SEGE_W][SEG_STG];
    const int wv = (int)(threadIdx.x >> 6);
    const uint32_t nb = min(*(volatile uint32_t*)(G.ctr + SC_BIGP), (uint32_t)G.cap_list);
    for (uint32_t b = blockIdx.x; b < nb; b += gridDim.x) {
        const uint32_t t = G.join[b];
        const uint64_t e = D.llist[t];
        const uint32_t first = G.pbase[t], ns = G.pn[t];
        const uint64_t pos = e & POS_MASK;
        const uint64_t oo = S.offs()[pos];  // (k_compact_long; no token of this pretoken lands there before all read it)
        __syncthreads();
        const uint32_t nr = (ns + 2u * WAVE - 1u) / (2u * WAVE);
        for (uint32_t r = (uint32_t)wv; r < nr; r += SEGE_W) {
            const uint32_t base = G.sg[first + r * 2u * WAVE];
            seg_emit_round(T, S, G, pos, first, ns, r * 2u * WAVE, ids_out + oo + base, offs_out + oo + base, sid[wv],
                           ssa[wv]);
        }
        __syncthreads();
    }
}

// The segment memo's entries: seg_encode (W = 16) of each key (lane per key, no
// normalizer: the keys are the normalized bytes a segment is looked up by). meta[i] =
// sm_make(...) (~0: more than 16 symbols or none), toks[16 i + k] the tokens (pool_tok),
// prof[16 i + k] the edge-list pairs (SegEdges), prof[16 i + 15] the round count.
template <bool COMPACT>
__global__ __launch_bounds__(256) void k_seg_memo_build(DevTables T, const uint8_t* __restrict__ keys,
                                                        const uint64_t* __restrict__ koff, uint32_t n, uint64_t limit,
                                                        uint64_t* __restrict__ meta, uint32_t* __restrict__ toks,
                                                        uint64_t* __restrict__ prof) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const bool act = i < n;
    const uint64_t o = act ? koff[i] : 0ull;
    const uint32_t L = act ? (uint32_t)(koff[i + 1] - o) : 0u;
    T.norm = 0;
    RegWord<16, COMPACT, true> rw;
    WordBytes<2> wb;
    wb.load(keys, o, limit, 0);
    const bool fits = reg_init<16, COMPACT, 2>(T, T.byte_id, rw, wb, wb, act && L <= 16u ? L : 0u);
    const bool ok = act && L <= 16u && fits && rw.n > 0;
    uint32_t f0 = 0, l0 = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        f0 = k == 0 ? rw.idv(rw.sy[k]) : f0;
        l0 = k == rw.n - 1 ? rw.idv(rw.sy[k]) : l0;
    }
    if (!ok) rw.n = 0;
    uint32_t edges = 0;
    const uint32_t nr = reg_rounds<16, COMPACT, true>(T, rw, prof + 16ull * (act ? i : 0u), &edges);
    if (!act) return;
    prof[16ull * i + 15] = nr;  // (at most 15 rounds: slot 15 holds the count)
#pragma unroll
    for (int k = 0; k < 16; ++k)
        if (k < rw.n) toks[16ull * i + k] = pool_tok(rw.idv(rw.sy[k]), rw.start(k), rw.end(k));
    meta[i] = ok ? sm_make(f0, l0, (uint32_t)rw.n, edges) : ~0ull;
}

hipError_t launch_seg_memo_build(const DevTables& T, const uint8_t* d_keys, const uint64_t* d_koff, uint32_t n,
                                 uint64_t limit, uint64_t* d_meta, uint32_t* d_toks, uint64_t* d_prof,
                                 hipStream_t st) {
    if (n == 0) return hipSuccess;
    if (T.compact)
        hipLaunchKernelGGL(k_seg_memo_build<true>, dim3((n + 255) / 256), dim3(256), 0, st, T, d_keys, d_koff, n,
                           limit, d_meta, d_toks, d_prof);
    else
        hipLaunchKernelGGL(k_seg_memo_build<false>, dim3((n + 255) / 256), dim3(256), 0, st, T, d_keys, d_koff, n,
                           limit, d_meta, d_toks, d_prof);
    return hipGetLastError();
}

// The hot-pair bitmap: bit a * k + b = is the boundary between hot keys a | b crossed, by
// the check k_seg_first runs (seg_crossed_core on their pool entries); a thread per 32 bits
template <bool COMPACT>
__global__ __launch_bounds__(256) void k_seg_hot_build(DevTables T, const uint32_t* __restrict__ hq,
                                                       const uint64_t* __restrict__ hm, uint32_t k,
                                                       uint32_t* __restrict__ bits) {
    const uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t kk = (uint64_t)k * k;
    if (w >= (kk + 31) / 32) return;
    uint32_t out = 0;
    for (uint32_t i = 0; i < 32u; ++i) {
        const uint64_t x = w * 32u + i;
        if (x >= kk) break;
        const uint32_t a = (uint32_t)(x / k), b = (uint32_t)(x % k);
        const uint64_t ma = hm[a], mb = hm[b];
        SegEdges Ea, Eb;
        Ea.load_pool(T, hq[a], sm_re(ma), 0u);
        Eb.load_pool(T, hq[b], 0u, sm_le(mb));
        if (seg_crossed_core<COMPACT>(T, ma, mb, Ea, Eb, nullptr)) out |= 1u << i;
    }
    bits[w] = out;
}

hipError_t launch_seg_hot_build(const DevTables& T, const uint32_t* d_q, const uint64_t* d_meta, uint32_t k,
                                uint32_t* d_bits, hipStream_t st) {
    const uint64_t nw = ((uint64_t)k * k + 31) / 32;
    if (nw == 0) return hipSuccess;
    const unsigned grid = (unsigned)((nw + 255) / 256);
    if (T.compact) hipLaunchKernelGGL(k_seg_hot_build<true>, dim3(grid), dim3(256), 0, st, T, d_q, d_meta, k, d_bits);
    else hipLaunchKernelGGL(k_seg_hot_build<false>, dim3(grid), dim3(256), 0, st, T, d_q, d_meta, k, d_bits);
    return hipGetLastError();
}

// one wavefront per long word, words taken from the list by a ticket
#ifndef TKZ_LONG_WORDB
#define TKZ_LONG_WORDB 5
#endif
template <bool COMPACT>
__global__ __launch_bounds__(64, TKZ_LONG_WORDB) void k_bpe_long(DevTables T, const uint8_t* __restrict__ bytes,
                                                                uint64_t limit, Scratch S, Deferred D) {
    __shared__ LongSmem sm;
    const int lane = lane_id();
    const uint32_t n = *(volatile uint32_t*)D.lcnt;
    WAVE_SYNC();
    while (true) {
        // a drained list ends the block without an atomic: the grid's one ticket atomic
        // per block on the same counter cost 0.09 ms with no long words at all
        if (rfl(*(volatile uint32_t*)(D.lcnt + 1)) >= n) break;
        uint32_t t = 0;
        if (lane == 0) t = atomicAdd(D.lcnt + 1, 1u);
        t = rfl(t);
        if (t >= n) break;
        const uint64_t e = D.llist[t];
        const uint64_t pos = e & POS_MASK;
        const uint64_t ws = S.slot(pos, (uint32_t)(e >> POS_BITS) & ORD_MASK);
        uint32_t L = (uint32_t)(e >> LEN_SHIFT);
        if (L == LEN_ESC) L = S.prs()[pos];
        L = rfl(L);
        if (lane == 0) atomicAdd(D.long_bytes, (unsigned long long)L);
        if (L <= (uint32_t)LW) {
            long_word_lds<COMPACT>(T, bytes, pos, ws, limit, L, sm, S, D.dbg);
        } else {
            uint32_t* o32 = (uint32_t*)(S.offs() + pos);
            GlbWord w{S.ids() + pos, S.prs() + pos, o32, o32 + L, S.tok() + pos};
            long_word<COMPACT>(T, T.byte_id, bytes, pos, ws, limit, L, w, sm.u.smin, sm.dsb, S);
        }
        WAVE_SYNC();
    }
}

// Scan state of the wave's current chunk. It lives in LDS, not registers: the word
// phases (BPE rounds) need every register, the scan touches this once per step.
struct ScanState {
    uint64_t c, cs, sb, dk, nbd;
    uint32_t n_st, n_en, head, d0, carry, in_chunk;
    uint32_t n_words;  // words of this chunk started so far (their ordinals 0..n_words-1)
    int32_t obase;     // ordinal of ring slot 0 in the current step
    uint32_t srel;     // chunk-relative start of the last scanned step; ring entries are
                       // u16 offsets from srel - RBASE: the words still pending from the
                       // step before it (>= srel - RBASE) keep valid entries
    uint32_t cstart;   // chunk-relative start of the open word carried over a step
    uint32_t carried;  // ring slot cidx holds that word (its start entry is stale)
    uint32_t cidx;
    uint32_t old_end;  // ring slots < old_end hold words from before the last scanned step:
                       // they must be dispatched before the next scan overwrites their bytes
                       // in stepbuf
    uint32_t flush_all;  // the chunk is scanned: dispatch partial batches too
};

template <int NQB, int NBID>
struct Smem {
    uint64_t q[NQB][QCAP];       // length buckets (+ BPE: the deferred-word staging queue)
    uint16_t wst[RCAP];          // word ring: start / end relative to (step start - RBASE)
    uint16_t wen[RCAP];
    // normalized bytes of the current and previous step; entries 256, 257 mirror 0, 1 (a
    // word's 24-byte window never wraps)
    uint64_t stepbuf[2 * STEP / 8 + 2];
    uint32_t byte_id[NBID];      // BPE only, ASCII bytes (the rest from T.byte_id): 5 waves/SIMD
    ScanState ss;
    uint32_t n_words, n_hits;    // batch statistics of this wave (HDR_WORDS, HDR_HITS)
    // doc boundaries of the step (TKZ_VEC_DOCS): a 1024-bit map, lane i's 16 bytes in bits
    // 16 i.. (128 B: with 256 B Smem was 7,784 B, past the 7,680 B of six 1,280-B LDS units,
    // and the CU held 18 k_encode blocks instead of 20)
    uint32_t bd[WAVE / 2];
};

// dynamic chunk queue: robust to however many blocks are actually co-resident
__device__ __forceinline__ uint64_t next_ticket(unsigned long long* ctr) {
    unsigned long long t = 0;
    if (lane_id() == 0) t = atomicAdd(ctr, 1ull);
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(t >> 32)) << 32) |
           (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)t);
}

// 8-bit masks of delimiter / punct bytes among the 8 bytes of v (config.zig:405-457)
__device__ __forceinline__ uint32_t zero_bytes32(uint32_t y) {
    return ~(((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y) & 0x80808080u;  // 0x80 where the byte is 0
}
__device__ __forceinline__ uint32_t gather4(uint32_t t) { return (((t >> 7) * 0x01020408u) >> 24) & 0xFu; }
__device__ __forceinline__ uint32_t eq_any32(uint32_t x, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3) {
    return zero_bytes32(x ^ (c0 * 0x01010101u)) | zero_bytes32(x ^ (c1 * 0x01010101u)) |
           zero_bytes32(x ^ (c2 * 0x01010101u)) | zero_bytes32(x ^ (c3 * 0x01010101u));
}
// 0x80 in every byte lo <= b <= hi of y (bytes of y have bit 7 clear, so no carries
// cross bytes)
__device__ __forceinline__ uint32_t in_range32(uint32_t y, uint32_t lo, uint32_t hi) {
    return (y + (128u - lo) * 0x01010101u) & ~(y + (127u - hi) * 0x01010101u);
}
// 0x80 in every byte of x that is one of is_punct's 32 ASCII punctuation bytes
// (config.zig:452-457): SWAR range tests (a per-byte test compiled to branches)
__device__ __forceinline__ uint32_t punct32(uint32_t x) {
    const uint32_t y = x & 0x7F7F7F7Fu;
    return (in_range32(y, 33, 47) | in_range32(y, 58, 64) | in_range32(y, 91, 96) | in_range32(y, 123, 126)) & ~x &
           0x80808080u;
}
__device__ __forceinline__ void class_masks(uint64_t v, int pretok, uint32_t& split, uint32_t& punct) {
    split = 0;
    punct = 0;
    if (pretok == 0) return;
    const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    uint32_t tl = eq_any32(lo, ' ', '\t', '\n', '\r'), th = eq_any32(hi, ' ', '\t', '\n', '\r');
    if (pretok == 2) {
        tl |= zero_bytes32(lo ^ 0x0B0B0B0Bu) | zero_bytes32(lo ^ 0x0C0C0C0Cu);
        th |= zero_bytes32(hi ^ 0x0B0B0B0Bu) | zero_bytes32(hi ^ 0x0C0C0C0Cu);
        punct = gather4(punct32(lo)) | (gather4(punct32(hi)) << 4);
    }
    split = gather4(tl) | (gather4(th) << 4) | punct;
}

__device__ __forceinline__ void begin_chunk(const DevTables& T, const uint8_t* bytes, const uint64_t* doc_off,
                                            uint64_t n_docs, uint32_t ch_log2, const uint64_t* chunk_doc,
                                            uint64_t R0, ScanState& s) {
    s.cs = s.c << ch_log2;
    s.sb = s.cs;
    s.dk = chunk_doc[s.c];
    s.nbd = s.dk <= n_docs ? doc_off[s.dk] : ~0ull;
    s.n_st = s.n_en = s.head = s.d0 = 0;
    s.n_words = 0;
    s.obase = 0;
    s.srel = s.cstart = s.carried = s.cidx = s.old_end = s.flush_all = 0;
    s.carry = 1;  // bit 0: previous byte is a delimiter, bit 1: previous byte is punct
    if (s.cs > R0) {
        bool sp, pu;
        classify(lower(bytes[s.cs - 1], T.norm), T.pretok, sp, pu);
        s.carry = (uint32_t)sp | ((uint32_t)pu << 1);
        // a word running into this chunk belongs to the previous one: its end is the
        // first end recorded here -> ring slot 0, never dispatched
        if (!sp || pu) { s.n_st = 1; s.head = 1; s.d0 = 1; }
    }
    s.in_chunk = 1;
}

__device__ __forceinline__ ScanState load_state(const ScanState& m) {
    ScanState s;
    s.c = rfl64(m.c); s.cs = rfl64(m.cs); s.sb = rfl64(m.sb); s.dk = rfl64(m.dk); s.nbd = rfl64(m.nbd);
    s.n_st = rfl(m.n_st); s.n_en = rfl(m.n_en); s.head = rfl(m.head); s.d0 = rfl(m.d0); s.carry = rfl(m.carry);
    s.in_chunk = rfl(m.in_chunk);
    s.n_words = rfl(m.n_words);
    s.obase = (int32_t)rfl((uint32_t)m.obase);
    s.srel = rfl(m.srel); s.cstart = rfl(m.cstart); s.carried = rfl(m.carried); s.cidx = rfl(m.cidx);
    s.old_end = rfl(m.old_end); s.flush_all = rfl(m.flush_all);
    return s;
}

template <int MODEL, bool COMPACT>
__global__ __launch_bounds__(64, TKZ_MINW) void k_encode(DevTables T, const uint8_t* __restrict__ bytes,
                                               const uint64_t* __restrict__ doc_off, uint64_t n_docs, uint64_t limit,
                                               uint32_t ch_log2, const uint64_t* __restrict__ chunk_doc,
                                               unsigned long long* __restrict__ chunk_ctr, Scratch S,
                                               uint32_t* __restrict__ chunk_words, uint32_t* __restrict__ doc_word,
                                               Deferred D, uint32_t* __restrict__ status) {
    constexpr int NBK = Buckets<MODEL>::n;
    constexpr int DQ = NBK;  // BPE: staging queue index of deferred words
    __shared__ Smem<MODEL == 1 ? NBK + 1 : NBK, MODEL == 1 && TKZ_LDS_BYTE_ID ? 128 : 1> sm;
    const int lane = lane_id();
    if (MODEL == 1)
        for (int i = lane; i < 128 && TKZ_LDS_BYTE_ID; i += WAVE) sm.byte_id[i] = T.byte_id[i];
    uint32_t qn[NBK];
#pragma unroll
    for (int k = 0; k < NBK; ++k) qn[k] = 0;
    uint32_t dqn = 0;
    // the current chunk's tokens resolved at dispatch, and the front fill of its dense area
    uint32_t ctok = 0, dfill = 0;
#if TKZ_PREFETCH_STEP
    // the next scan step's 16 B per lane, loaded when a step ends (the dispatch phases in
    // between hide its latency; a scan-only run waited on every step's load: 81 % wait)
    uint4 pfq = make_uint4(0u, 0u, 0u, 0u);
    uint64_t pf_sb = ~0ull;
#endif
    // word-level shortcut at dispatch: the BPE word memo, or for WordPiece the whole-word
    // vocab probe (a word that is itself a key of <= 16 bytes is one token (0, L): the
    // first candidate of WordPiece.tokenize, wordpiece.zig:160-190)
    const bool memo = (MODEL == 1 && T.memo != nullptr) || (MODEL == 0 && T.wps != nullptr);
    {
        ScanState s;
        const uint64_t R0 = doc_off[0], R1 = doc_off[n_docs];
        s.c = (R0 >> ch_log2) + next_ticket(chunk_ctr);
        s.in_chunk = 0;
        s.n_st = s.n_en = s.head = s.d0 = 0;
        s.carried = s.cidx = s.old_end = s.flush_all = 0;
        if (s.c < ((R1 + (1ull << ch_log2) - 1) >> ch_log2))
            begin_chunk(T, bytes, doc_off, n_docs, ch_log2, chunk_doc, R0, s);
        if (lane == 0) { sm.ss = s; sm.n_words = 0; sm.n_hits = 0; }
    }
    WAVE_SYNC();
    const uint32_t* byte_id = TKZ_LDS_BYTE_ID ? sm.byte_id : T.byte_id;
    bool flush = false;
#ifdef TKZ_RESIDENCY
    if (lane == 0) atomicMax(&status[2], atomicAdd(&status[1], 1u) + 1u);
#endif

#ifdef TKZ_PHASES
    uint64_t ph[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#endif
    // state machine with one site for each phase (keeps one inlined copy per bucket)
    while (true) {
        PH_BEGIN();
        // (1) a full bucket (or, when flushing, any non-empty one) -> run the model
        int b = -1;
        uint32_t take = 0;
#pragma unroll
        for (int k = 0; k < NBK; ++k)
            if (qn[k] >= WAVE) { b = k; take = WAVE; }
        if (b < 0 && flush) {
#pragma unroll
            for (int k = NBK - 1; k >= 0; --k)
                if (qn[k] > 0) { b = k; take = qn[k]; }
        }
        if (MODEL == 1 && (dqn >= WAVE || (b < 0 && flush && dqn > 0))) {
            const uint32_t take_d = min(dqn, (uint32_t)WAVE);
            dqn -= take_d;
            uint32_t base = 0;
            if (lane == 0) base = atomicAdd(D.cnt, take_d);
            base = rfl(base);
            if ((uint32_t)lane < take_d) D.list[base + lane] = sm.q[DQ][dqn + lane];
            WAVE_SYNC();
            PH_END(0);
            continue;
        }
        if (b >= 0) {
            uint32_t qb = 0;
#pragma unroll
            for (int k = 0; k < NBK; ++k)
                if (k == b) { qn[k] -= take; qb = qn[k]; }
            run_bucket<MODEL, COMPACT>(T, byte_id, &sm.q[b][qb], b, take, bytes, limit, S, status);
            WAVE_SYNC();
            PH_END(1);
            continue;
        }
        // (2) complete words in the ring -> word memo / buckets, in full batches of 64; a
        // partial batch only for words the next scan would evict from stepbuf, or when the
        // chunk is scanned (a step holds ~85 words in C1: one batch and a third per step,
        // not two)
        const uint32_t head = rfl(sm.ss.head), n_en = rfl(sm.ss.n_en);
        const uint32_t old_end = rfl(sm.ss.old_end), flush_all = rfl(sm.ss.flush_all);
#if TKZ_ABLATE >= 6  // timing only: the scan alone (words are never dispatched)
        if (head < n_en) {
            if (lane == 0) sm.ss.head = n_en;
            WAVE_SYNC();
            continue;
        }
#endif
        if (head < n_en && (n_en - head >= (uint32_t)WAVE || head < old_end || flush_all)) {
            const uint64_t cs = rfl64(sm.ss.cs);
            const int32_t obase = (int32_t)rfl((uint32_t)sm.ss.obase);
            const uint32_t fsrel = rfl(sm.ss.srel) - (uint32_t)RBASE;  // ring entry base (wraps; entries >= RBASE then)
            const uint32_t cstart = rfl(sm.ss.cstart), carried = rfl(sm.ss.carried), cidx = rfl(sm.ss.cidx);
            const uint32_t chunk = min(n_en - head, (uint32_t)WAVE);
            int bk = -1, dl = -1;
            uint64_t ent = 0;
            PH_LAP(6);
            const bool act = (uint32_t)lane < chunk;
            uint32_t L = 0, ord = 0;
            uint64_t pos = 0, ws = 0, k0 = 0, k1 = 0;
            if (act) {
                const uint32_t r = head + lane;
                const uint32_t rs = (carried && r == cidx) ? cstart : fsrel + sm.wst[r];
                L = fsrel + sm.wen[r] - rs;
                pos = cs + rs;
                ord = (uint32_t)(obase + (int32_t)(head + lane));
                ws = cs + ord;
                if (memo && L <= 16) {
                    // bytes [pos, pos + 16) by 32-bit byte-aligns of the 24-byte window
                    const uint32_t a = (uint32_t)(pos >> 3) & (2u * STEP / 8u - 1u), b = (uint32_t)pos & 7u;
                    const uint64_t q0 = sm.stepbuf[a], q1 = sm.stepbuf[a + 1], q2 = sm.stepbuf[a + 2];
                    const bool h4 = b >= 4u;
                    const uint32_t u0 = h4 ? (uint32_t)(q0 >> 32) : (uint32_t)q0;
                    const uint32_t u1 = h4 ? (uint32_t)q1 : (uint32_t)(q0 >> 32);
                    const uint32_t u2 = h4 ? (uint32_t)(q1 >> 32) : (uint32_t)q1;
                    const uint32_t u3 = h4 ? (uint32_t)q2 : (uint32_t)(q1 >> 32);
                    const uint32_t u4 = h4 ? (uint32_t)(q2 >> 32) : (uint32_t)q2;
                    k0 = (uint64_t)__builtin_amdgcn_alignbyte(u1, u0, b) |
                         ((uint64_t)__builtin_amdgcn_alignbyte(u2, u1, b) << 32);
                    k1 = (uint64_t)__builtin_amdgcn_alignbyte(u3, u2, b) |
                         ((uint64_t)__builtin_amdgcn_alignbyte(u4, u3, b) << 32);
                    // zero past L (L >= 1): 2 << (8n - 1) wraps to 0 at n = 8
                    k0 &= (2ull << (8u * min(L, 8u) - 1u)) - 1u;
                    k1 = L > 8u ? k1 & ((2ull << (8u * min(L - 8u, 8u) - 1u)) - 1u) : 0ull;
                }
            }
            uint32_t hmeta = 0, hw = 0, ht1 = 0, ht2 = 0;  // a BPE memo hit
            bool hit = false;
            if (act) {
                bool done = false;
#if TKZ_ABLATE != 1
                if (memo && L <= 16) {
                    if (MODEL == 1) {
                        done = hit = memo_lookup<COMPACT>(T, k0, k1, L, hmeta, hw, ht1, ht2);
                    } else if (L <= T.max_chars && L <= T.max_key) {
                        const uint32_t id = wps_probe(T, k0, k1, L);
                        if (id != NONE) {
                            if (T.narrow) {
                                S.single_nc(ws, id | (L << 24));
                            } else {
                                S.ids()[pos] = id;
                                S.offs()[pos] = (uint64_t)L << 32;
                                S.wide_nc(ws, pos, 1);
                            }
                            done = hit = true;
                        }
                    }
#if TKZ_ABLATE == 4
                    if (!done) { S.narrow(ws, pos, 0); done = true; }  // misses dropped
#endif
                }
#endif
                if (!done) {
                    if (MODEL == 1 && L > 8) dl = 0;  // deferred to k_bpe_deferred
                    else bk = bucket_of<MODEL>(L);
                    ent = pos | ((uint64_t)ord << POS_BITS) | ((uint64_t)min(L, LEN_ESC) << LEN_SHIFT);
                    if (L >= LEN_ESC) S.prs()[pos] = L;  // full length for the long path
                }
            }
            if (MODEL == 1 && memo && !COMPACT && !T.mid) {
                // wide tables: a hit's tokens (id | start << 22 | end << 27) as wide tokens at
                // the word's byte offset (the word record holds no 32-bit id)
                const uint32_t nt = hit ? (hmeta >> 5) & 3u : 0u;
                if (hit) memo_emit_wide(S, nt, hw, ht1, ht2, pos, ws);
                ctok += lane63((uint32_t)wave_incl_scan((int)nt));
            } else if (MODEL == 1 && memo) {
                // memo hits: 2-3 tokens go to the front of the chunk's dense area (the wave
                // owns the chunk: a fill counter in a register, no atomic; offsets from
                // ballots), coalesced, and k_compact streams them; the batch's token count
                // joins the chunk's
                const uint32_t nt = hit ? (hmeta >> 5) & 3u : 0u;
                const uint64_t m1 = __ballot(nt == 1u), m2 = __ballot(nt == 2u), m3 = __ballot(nt == 3u);
                const uint32_t need = 2u * (uint32_t)__popcll(m2) + 3u * (uint32_t)__popcll(m3);
                if (hit) {
                    const uint32_t off = dfill + 2u * lanes_below(m2) + 3u * lanes_below(m3);
                    if (!COMPACT) {  // T.mid: the wide memo's tokens (id | start << 22 | end << 27) packed
                        hw = mid_tok(hw & 0x3FFFFFu, (hw >> 22) & 31u, hw >> 27);
                        ht1 = mid_tok(ht1 & 0x3FFFFFu, (ht1 >> 22) & 31u, ht1 >> 27);
                        ht2 = mid_tok(ht2 & 0x3FFFFFu, (ht2 >> 22) & 31u, ht2 >> 27);
                    }
                    memo_emit(S, COMPACT && L <= 8u, hmeta, hw, ht1, ht2, L, ws, S.dtok() + S.dbase(cs) + off, off);
                }
                dfill += need;
                ctok += (uint32_t)__popcll(m1) + need;
            } else if (MODEL == 0 && memo) {
                ctok += (uint32_t)__popcll(__ballot(hit));
            }
            PH_LAP(7);
            uint32_t missed = 0;  // words of this batch queued for the model
            if (MODEL == 1) {
                const uint64_t m = __ballot(dl == 0);
                if (dl == 0) {
                    const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
                    sm.q[DQ][dqn + r] = ent;
                }
                dqn += (uint32_t)__popcll(m);
                missed += (uint32_t)__popcll(m);
            }
#pragma unroll
            for (int bb = 0; bb < NBK; ++bb) {
                const uint64_t m = __ballot(bk == bb);
                if (bk == bb) {
                    const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
                    sm.q[bb][qn[bb] + r] = ent;
                }
                qn[bb] += (uint32_t)__popcll(m);
                missed += (uint32_t)__popcll(m);
            }
#ifndef TKZ_NO_STATS
            if (lane == 0) { sm.n_words += chunk; sm.n_hits += chunk - missed; }
#endif
#ifdef TKZ_COUNT_WORDS
            if (lane == 0) { atomicAdd(&status[1], chunk); atomicAdd(&status[2], 1u); }  // words, batches
#endif
            WAVE_SYNC();
            if (lane == 0) sm.ss.head = head + chunk;
            WAVE_SYNC();
            PH_END(2);
            continue;
        }
        ScanState s = load_state(sm.ss);
        const uint64_t R0 = doc_off[0], R1 = doc_off[n_docs];
        const uint64_t ce = s.cs + (1ull << ch_log2);
        // (3) scan the next 1-KiB step (past the chunk end only to close its last word)
        const bool open = s.n_en < s.n_st && s.n_en >= s.d0;  // this chunk's last word is unclosed
        if (s.in_chunk && (s.sb < ce || open) && s.sb < R1) {
            const uint64_t sb = s.sb;
            // rebase the ring to this step: the pending words [head, n_en) (all from the
            // last scanned step: older ones were flushed) and the open word move to the
            // front; the open word's chunk-relative start is kept in cstart
            const uint32_t srel = (uint32_t)(sb - s.cs);
            if (s.head <= s.n_en) {
                const uint32_t dz = srel - s.srel;  // the last step's size
                if (s.n_st > s.n_en) {
                    if (!(s.carried && s.cidx == s.n_en)) s.cstart = (s.srel - (uint32_t)RBASE) + sm.wst[s.n_en];
                    s.carried = 1;
                } else {
                    s.carried = 0;
                }
                const uint32_t nsurv = s.n_st - s.head;
                if ((uint32_t)lane < nsurv) {  // reads before writes (in-order LDS per wave)
                    const uint32_t a = sm.wst[s.head + lane], e = sm.wen[s.head + lane];
                    sm.wst[lane] = (uint16_t)(a - dz);
                    sm.wen[lane] = (uint16_t)(e - dz);
                }
                s.cidx = s.n_en - s.head;
                s.old_end = nsurv;
                s.n_st = nsurv;
                s.n_en -= s.head;
                s.head = s.d0 = 0;
            } else {  // an unclosed dummy (the previous chunk's word runs on): nothing pending
                s.old_end = 0;
            }
            s.srel = srel;
            // ring slot r of this step holds the word with ordinal obase + r
            s.obase = (int32_t)s.n_words - (int32_t)s.n_st;
            // valid bytes of this lane: [R0, R1)
            const int r0 = R0 > sb ? (int)min(R0 - sb, (uint64_t)STEP) : 0;
            const int r1 = (int)min(R1 - sb, (uint64_t)STEP);
            const int lo = min(max(r0 - 16 * lane, 0), 16), hi = min(max(r1 - 16 * lane, 0), 16);
            const uint32_t vm = ((1u << hi) - 1) & ~((1u << lo) - 1);
            // lane byte offsets rematerialised per step (the register allocator would keep
            // them live across the word phases and spill them to scratch)
            uint32_t l16 = (uint32_t)lane * 16u;
            asm volatile("" : "+v"(l16));
            uint64_t v0 = 0, v1 = 0;
#if TKZ_PREFETCH_STEP
            const bool pf_hit = pf_sb == sb;  // (uniform)
#else
            constexpr bool pf_hit = false;
#endif
            if (vm) {
#if TKZ_PREFETCH_STEP
                const uint4 q = pf_hit ? pfq : *(const uint4*)(bytes + sb + l16);
#elif TKZ_NT_INPUT  // streamed input read once: keep it from displacing the tables in L2
                const uint4 q = __builtin_nontemporal_load((const uint4*)(bytes + sb + l16));
#else
                const uint4 q = *(const uint4*)(bytes + sb + l16);
#endif
                v0 = ((uint64_t)q.y << 32) | q.x;
                v1 = ((uint64_t)q.w << 32) | q.z;
            }
            (void)pf_hit;
            // document boundaries in this step, before v is used (their loads overlap the
            // step's vector load). Lane i holds boundary dk + i (one vector load; a scalar
            // walk over doc_off waited on one dependent load per boundary), set in the
            // byte lanes' masks by LDS ORs; a step with 64 or more boundaries walks them
            // on the scalar unit. (dkh, nbdh): the state at the half-step point, where a
            // half step resumes.
            const uint64_t dk0 = s.dk;
            uint64_t dkh = s.dk, nbdh = s.nbd;
            uint32_t BD = 0;
#ifdef TKZ_NO_DOCWALK  // timing only: no doc boundaries (wrong results)
            s.nbd = ~0ull;
#endif
            // (the first VDL lanes only: loading 64 entries per step cost 1.9M more L2 misses
            // per C1 step than the walk; a step with VDL or more boundaries walks them)
            constexpr int VDL = 16;
            const uint64_t kl = dk0 + (uint64_t)lane;
            const uint64_t bl =
                TKZ_VEC_DOCS && s.nbd < sb + STEP && lane < VDL && kl <= n_docs ? doc_off[kl] : ~0ull;
            const uint64_t mbl = __ballot(bl < sb + STEP);
            const bool vec_docs = TKZ_VEC_DOCS && s.nbd < sb + STEP && (mbl >> (VDL - 1)) == 0ull;
            if (vec_docs) {
                // (the syncs order the lanes' LDS accesses for the compiler too: without them
                // a lane that ORs nothing reads back the 0 it stored)
                if (lane < WAVE / 2) sm.bd[lane] = 0;
                WAVE_SYNC();
                if (bl < sb + STEP) atomicOr(&sm.bd[(uint32_t)(bl - sb) >> 5], 1u << ((uint32_t)(bl - sb) & 31u));
                WAVE_SYNC();
                BD = (sm.bd[lane >> 1] >> ((lane & 1) * 16)) & 0xFFFFu;
                const uint32_t nb = (uint32_t)__popcll(mbl), nh = (uint32_t)__popcll(__ballot(bl < sb + HSTEP));
                s.dk = dk0 + nb;
                s.nbd = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(bl >> 32), (int)nb) << 32) |
                        (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)bl, (int)nb);
                dkh = dk0 + nh;
                nbdh = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(bl >> 32), (int)nh) << 32) |
                       (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)bl, (int)nh);
            }
            while (!vec_docs && s.nbd < sb + STEP) {
                const uint32_t o = (uint32_t)(s.nbd - sb);
                if ((int)(o >> 4) == lane) BD |= 1u << (o & 15u);
                ++s.dk;
                s.nbd = s.dk <= n_docs ? doc_off[s.dk] : ~0ull;
                if (o < (uint32_t)HSTEP) { dkh = s.dk; nbdh = s.nbd; }
            }
            if (T.norm) { v0 = lower8(v0); v1 = lower8(v1); }
            {
                // (a step starts 512-B aligned, after a half step not 1-KiB aligned: wraps)
                const uint32_t si = ((uint32_t)(sb >> 3) + 2u * (uint32_t)lane) & (2u * STEP / 8u - 1u);
                sm.stepbuf[si] = v0;
                sm.stepbuf[si + 1] = v1;
                if (si == 0u) { sm.stepbuf[2 * STEP / 8] = v0; sm.stepbuf[2 * STEP / 8 + 1] = v1; }  // mirror of 0, 1
            }
            PH_LAP(8);
            uint32_t split, punct, split1, punct1;
            class_masks(v0, T.pretok, split, punct);
            class_masks(v1, T.pretok, split1, punct1);
            const uint32_t Sm = split | (split1 << 8) | (~vm & 0xFFFFu);  // invalid bytes split
            const uint32_t P = (punct | (punct1 << 8)) & vm;
            const uint32_t x = Sm | (P << 16);
            const uint32_t up = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x138, 0xF, 0xF, false);  // wave_shr:1
            const uint32_t prev = lane == 0 ? s.carry : ((up >> 15) & 1u) | (((up >> 31) & 1u) << 1);
            const uint32_t Sprev = ((Sm << 1) | (prev & 1u)) & 0xFFFFu;
            const uint32_t Pprev = ((P << 1) | (prev >> 1)) & 0xFFFFu;
            // start: word byte after a delimiter or a doc boundary, or a punct byte;
            // end (exclusive): delimiter or boundary after a word byte, or byte after punct
            // (chunks are multiples of 512 B = 32 lanes: bytes past the chunk end start none)
            uint32_t starts = ((~Sm & (Sprev | BD)) | P) & 0xFFFFu;
            uint32_t ends = ((~Sprev & (Sm | BD)) | Pprev) & 0xFFFFu;
            if (sb + l16 >= ce) starts = 0;
            // one packed prefix sum: starts in bits 0..15, ends in bits 16..31 (<= 1024 each)
            uint32_t cnt = (uint32_t)__popc(starts) | ((uint32_t)__popc(ends) << 16);
            uint32_t inc = (uint32_t)wave_incl_scan((int)cnt);
            uint32_t tot = lane63(inc);
            uint32_t zstep = STEP;
            int lastl = WAVE - 1;
            if (s.n_st + (tot & 0xFFFFu) > (uint32_t)RCAP) {
                // more new words than the ring holds (< 2 bytes per word): a half step, the
                // first 32 lanes (<= 512 new words); the doc walk resumes at its half point
                zstep = HSTEP;
                lastl = WAVE / 2 - 1;
                if (lane >= WAVE / 2) { starts = 0; ends = 0; }
                cnt = (uint32_t)__popc(starts) | ((uint32_t)__popc(ends) << 16);
                inc = (uint32_t)wave_incl_scan((int)cnt);
                tot = lane63(inc);
                s.dk = dkh;
                s.nbd = nbdh;
            }
            const uint32_t last = (uint32_t)__builtin_amdgcn_readlane((int)x, lastl);
            s.carry = ((last >> 15) & 1u) | (((last >> 31) & 1u) << 1);
            uint32_t ks = s.n_st + (inc & 0xFFFFu) - (cnt & 0xFFFFu);
            uint32_t ke = s.n_en + (inc >> 16) - (cnt >> 16);
            const uint32_t kmax = s.n_st + (tot & 0xFFFFu);  // ends past the last start close nothing
            const uint32_t rel = l16 + (uint32_t)RBASE;  // entries: from srel - RBASE
            // one write per set bit (a lane holds 0-8 starts / ends, mostly 2-3): the VALU
            // issue slots are the kernel's bound, the loop control runs on the SALU
            for (uint32_t m = starts; m; m &= m - 1u) sm.wst[ks++] = (uint16_t)(rel + (uint32_t)__builtin_ctz(m));
            for (uint32_t m = ends; m && ke < kmax; m &= m - 1u) sm.wen[ke++] = (uint16_t)(rel + (uint32_t)__builtin_ctz(m));
            PH_LAP(9);
            // ordinal of the first word at or after each doc boundary of this step that
            // this chunk owns (row_ptr is resolved from it in k_compact)
            if (vec_docs) {  // lane i: boundary dk0 + i
                const uint32_t excl = (inc & 0xFFFFu) - (cnt & 0xFFFFu);
                const uint64_t vend = min(min(ce, R1), sb + zstep);
                const bool wr = bl < vend;
                const uint32_t o = wr ? (uint32_t)(bl - sb) : 0u;
                const int l4 = (int)(o >> 4) * 4;
                const uint32_t before = (uint32_t)__builtin_amdgcn_ds_bpermute(l4, (int)excl) +
                                        (uint32_t)__popc((uint32_t)__builtin_amdgcn_ds_bpermute(l4, (int)starts) &
                                                         ((1u << (o & 15u)) - 1u));
                if (wr) doc_word[kl] = s.n_words + before;
            } else {
                const uint32_t excl = (inc & 0xFFFFu) - (cnt & 0xFFFFu);
                const uint64_t vend = min(min(ce, R1), sb + zstep);
                for (uint64_t k = dk0; k < s.dk; ++k) {
                    const uint64_t bv = doc_off[k];
                    if (bv >= vend) break;
                    const uint32_t o = (uint32_t)(bv - sb);
                    const uint32_t l = o >> 4;
                    const uint32_t before = (uint32_t)__builtin_amdgcn_readlane((int)excl, (int)l) +
                                            (uint32_t)__popc((uint32_t)__builtin_amdgcn_readlane((int)starts, (int)l) &
                                                             ((1u << (o & 15u)) - 1u));
                    if (lane == 0) doc_word[k] = s.n_words + before;
                }
            }
            s.n_words += tot & 0xFFFFu;
            s.n_st += tot & 0xFFFFu;
            s.n_en += tot >> 16;
            if (s.n_en > s.n_st) s.n_en = s.n_st;  // ends past the chunk's last word
            s.sb = sb + zstep;
            {
                const bool open2 = s.n_en < s.n_st && s.n_en >= s.d0;
                s.flush_all = ((s.sb < ce || open2) && s.sb < R1) ? 0u : 1u;  // no further scan step
            }
#if TKZ_PREFETCH_STEP
            pf_sb = ~0ull;
            if (!s.flush_all && s.sb + (uint64_t)STEP <= limit) {  // (the whole next step is readable)
                pfq = *(const uint4*)(bytes + s.sb + l16);
                pf_sb = s.sb;
            }
#endif
            WAVE_SYNC();
            if (lane == 0) sm.ss = s;
            WAVE_SYNC();
            PH_END(3);
            continue;
        }
        if (s.in_chunk && open) {  // the batch ends at a step boundary inside a word
            if (lane == 0) {
                sm.wen[s.n_en] = (uint16_t)(R1 - s.cs - s.srel + (uint64_t)RBASE);
                sm.ss.n_en = s.n_en + 1;
                sm.ss.flush_all = 1;
            }
            WAVE_SYNC();
            PH_END(4);
            continue;
        }
        // (4) next chunk
        if (s.in_chunk) {
#if TKZ_ABLATE >= 6  // no word was dispatched: the chunk has none for k_compact
            if (lane == 0) chunk_words[s.c] = 0;
#else
            if (lane == 0) chunk_words[s.c] = s.n_words;
#endif
            if (lane == 0) {  // the chunk's dispatch-resolved tokens (the model adds the rest)
                if (ctok) atomicAdd(S.ccnt() + s.c, ctok);
            }
            ctok = 0;
            dfill = 0;
            s.c = (R0 >> ch_log2) + next_ticket(chunk_ctr);
            if (s.c < ((R1 + (1ull << ch_log2) - 1) >> ch_log2)) {
                begin_chunk(T, bytes, doc_off, n_docs, ch_log2, chunk_doc, R0, s);
            } else {
                s.in_chunk = 0;
            }
            WAVE_SYNC();
            if (lane == 0) sm.ss = s;
            WAVE_SYNC();
            PH_END(5);
            continue;
        }
        if (!flush) { flush = true; continue; }
        break;
    }
    if (lane == 0) {
        atomicAdd(chunk_ctr + HDR_WORDS, (unsigned long long)sm.n_words);
        atomicAdd(chunk_ctr + HDR_HITS, (unsigned long long)sm.n_hits);
    }
#ifdef TKZ_PHASES
    if (lane == 0)
        for (int k = 0; k < 10; ++k) atomicAdd(&D.dbg[k], (unsigned long long)ph[k]);
#endif
#ifdef TKZ_RESIDENCY
    if (lane == 0) atomicSub(&status[1], 1u);
#endif
}

// ---------------------------------------------------------------------------
// k_encode_docs: k_encode for a pretokenizer that never splits (T.pretok == 0: ByteLevel,
// Metaspace, none -- config.zig:387-402, lib.zig:121), one thread per doc. Every doc is
// one pretoken, so the scan has nothing to find: doc k's word starts at doc_off[k] and ends
// at doc_off[k + 1]. A chunk's words are the docs starting in it, with ordinal k -
// chunk_doc[c]; an empty doc is a word of no tokens (an empty record), so the ordinals are
// dense without a scan and doc_word[k] is the doc's own ordinal. A doc of <= 16 B probes the
// word memo (hit: the record, 2-3 tokens from the back of the chunk's dense area), any
// other goes to the deferred list (k_bpe_deferred; > 64 B on to the long list and the
// segmented path). k_encode's byte scan of such docs cost 1.17 ms per 512-MB step (C6; its
// per-step state machine), for words it then only measured.
// ---------------------------------------------------------------------------
template <bool COMPACT>
__global__ __launch_bounds__(256) void k_encode_docs(DevTables T, const uint8_t* __restrict__ bytes,
                                                     const uint64_t* __restrict__ doc_off, uint64_t n_docs,
                                                     uint64_t limit, uint32_t ch_log2,
                                                     const uint64_t* __restrict__ chunk_doc,
                                                     unsigned long long* __restrict__ chunk_ctr, Scratch S,
                                                     uint32_t* __restrict__ chunk_words,
                                                     uint32_t* __restrict__ doc_word, Deferred D) {
    __shared__ uint32_t red[3][256 / WAVE];
    __shared__ uint32_t dbase;
    const int lane = lane_id(), wv = threadIdx.x >> 6;
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t R0 = doc_off[0], R1 = doc_off[n_docs];
    // chunk c's word count: the docs starting in it (chunk_doc of the next chunk, or n_docs
    // past R1: k_chunk_docs fills only chunks starting at or before R1)
    {
        const uint64_t c = (R0 >> ch_log2) + i, c_end = (R1 + (1ull << ch_log2) - 1) >> ch_log2;
        if (c < c_end) {
            const uint64_t a = min(chunk_doc[c], n_docs);
            const uint64_t b = ((c + 1) << ch_log2) <= R1 ? min(chunk_doc[c + 1], n_docs) : n_docs;
            chunk_words[c] = (uint32_t)(b - a);
        }
    }
    const bool act = i < n_docs;
    uint64_t pos = 0, ws = 0;
    uint32_t L = 0;
    if (act) {
        pos = doc_off[i];
        L = (uint32_t)min(doc_off[i + 1] - pos, (uint64_t)0xFFFFFFFFu);
        const uint64_t c = pos >> ch_log2;
        const uint32_t ord = (uint32_t)(i - chunk_doc[c]);
        ws = (c << ch_log2) + ord;
        doc_word[i] = ord;
    }
    const bool memo = T.memo != nullptr;
    uint32_t hmeta = 0, hw = 0, ht1 = 0, ht2 = 0;
    bool hit = false;
    if (act && memo && L >= 1u && L <= 16u) {
        WordBytes<2> kb;
        kb.load(bytes, pos, limit, T.norm);
        const uint64_t k0 = kb.w[0] & ((2ull << (8u * min(L, 8u) - 1u)) - 1u);
        const uint64_t k1 = L > 8u ? kb.w[1] & ((2ull << (8u * (L - 8u) - 1u)) - 1u) : 0ull;
        hit = memo_lookup<COMPACT>(T, k0, k1, L, hmeta, hw, ht1, ht2);
    }
    // memo hits: the record, and 2-3 tokens from the back of the chunk's dense area
    // (chunk_commit: one atomic per run of same-chunk lanes, with the chunk's token count)
    const uint32_t nt = hit ? (hmeta >> 5) & 3u : 0u;
    const uint32_t need = nt >= 2u ? nt : 0u;
    const uint32_t off = chunk_commit<true>(S, hit, pos, nt, need);
    if (hit) {
        if (!COMPACT) {  // T.mid: the wide memo's tokens (id | start << 22 | end << 27) packed
            hw = mid_tok(hw & 0x3FFFFFu, (hw >> 22) & 31u, hw >> 27);
            ht1 = mid_tok(ht1 & 0x3FFFFFu, (ht1 >> 22) & 31u, ht1 >> 27);
            ht2 = mid_tok(ht2 & 0x3FFFFFu, (ht2 >> 22) & 31u, ht2 >> 27);
        }
        memo_emit(S, COMPACT && L <= 8u, hmeta, hw, ht1, ht2, L, ws, S.dtok() + S.dbase(pos) + off, off);
    } else if (act && L == 0u) {
        S.dense_nc(ws, 0, 0);  // an empty doc: a word of no tokens
    }
    // the rest to the deferred list; statistics (pretokens = non-empty docs, memo hits):
    // one atomic each per block (per wave, the list's counter cost 0.2 ms per 1M docs)
    const bool dl = act && !hit && L > 0u;
    const uint64_t m = __ballot(dl);
    const uint64_t mw = __ballot(act && L > 0u), mh = __ballot(hit);  // (ballots of the whole wave)
    if (lane == 0) {
        red[0][wv] = (uint32_t)__popcll(mw);
        red[1][wv] = (uint32_t)__popcll(mh);
        red[2][wv] = (uint32_t)__popcll(m);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t a = 0, b = 0, d = 0;
        for (int w = 0; w < 256 / WAVE; ++w) { a += red[0][w]; b += red[1][w]; d += red[2][w]; }
        if (a) atomicAdd(chunk_ctr + HDR_WORDS, (unsigned long long)a);
        if (b) atomicAdd(chunk_ctr + HDR_HITS, (unsigned long long)b);
        dbase = d ? atomicAdd(D.cnt, d) : 0u;
    }
    __syncthreads();
    if (dl) {
        uint32_t before = 0;
        for (int w = 0; w < wv; ++w) before += red[2][w];
        const uint32_t ord = (uint32_t)(ws - ((pos >> ch_log2) << ch_log2));
        D.list[dbase + before + lanes_below(m)] = pos | ((uint64_t)ord << POS_BITS) | ((uint64_t)min(L, LEN_ESC) << LEN_SHIFT);
        if (L >= LEN_ESC) S.prs()[pos] = L;  // full length for the long path
    }
}

// ---------------------------------------------------------------------------
// k_encode_blk: k_encode for the splitting pretokenizers (T.pretok 1 Whitespace /
// WhitespaceSplit, 2 BertPreTokenizer: config.zig:405-457), rebuilt without the per-step
// state machine (round 6, verdict r5 item 2). A 256-thread block takes chunks c0 + blockIdx.x
// + k * gridDim.x; per chunk, in four barrier-separated phases:
//   (1) its bytes (32 per thread, two 16-B loads) staged normalized in LDS, and its doc
//       boundaries (one doc_off load per thread per round) as a bitmap;
//   (2) byte classes -> start / end masks (the previous byte's classes from the thread
//       before), ONE block prefix sum of the packed start / end counts: a word's ordinal is
//       its start's rank, its end the (rank + d0)-th end (d0: a word of the previous chunk
//       runs in). Starts and ends go to the two u16 halves of the word's record slot
//       (chunk start + ordinal, the slot its record replaces); doc_word from the start ranks;
//       the chunk's last word, when it runs past the chunk, closed from the staged 64-B tail
//       (a global scan past it only for longer words);
//   (3) one lane per word: the record slot's start / end, the key from the LDS stage, the
//       word memo probe (hits: the record, 2-3 tokens to the front of the chunk's dense area
//       by an LDS fill counter), misses to per-wave length-bucket queues (register BPE when
//       64 wait) or the deferred list (BPE > 8 B), as k_encode's dispatch did.
// The scan state lives in no LDS struct and no wave walks a ring: k_encode spent its time in
// the save / reload of that state per phase and in the wave-serial 1-KiB steps.
// Outputs are k_encode's exactly (records, dense areas, ccnt, chunk_words, doc_word, the
// deferred list), so every later kernel is unchanged.
// ---------------------------------------------------------------------------
constexpr int EB_T = 256, EB_NW = EB_T / WAVE;
constexpr uint32_t EB_CH = 8192;  // largest chunk (CH_MAX_LOG2)
constexpr uint32_t EB_TAIL = 64;  // bytes of the next chunk staged (keys of the last word)
#ifndef TKZ_EB_WCAP
#define TKZ_EB_WCAP 1536
#endif
constexpr uint32_t EB_WCAP = TKZ_EB_WCAP;  // words of a chunk whose start / end stay in LDS
template <int NQ>
struct EbSmem {
    uint64_t q[EB_NW][NQ][QCAP];            // per wave: length buckets (+ BPE: deferred staging)
    uint64_t stage[(EB_CH + EB_TAIL) / 8 + 2];  // the chunk's normalized bytes (+ tail)
    uint32_t bd[EB_CH / 32];                // doc boundaries: bit j of word i = byte 32 i + j
    uint32_t st[EB_T];                      // per thread: its start mask
    uint16_t lex[EB_T];                     // per thread: starts before it in its wave
    uint8_t xl[EB_T];                       // per thread: classes of its last byte
    uint32_t wsum[EB_NW];                   // per wave: packed start | end << 16 counts
    uint32_t nb_rel;                        // first doc boundary at or past the chunk end (rel)
    uint32_t open_end;                      // the open last word's end (rel)
    uint32_t more;                          // a further round of doc boundaries
    uint32_t dfill;                         // the chunk's dense area: front fill
    uint32_t sfill;                         // the chunk's short-miss list (BPE)
    uint32_t d0c;                           // d0 | classes of byte cs - 1 << 1 (thread 0)
    uint32_t went[EB_WCAP];                 // words < EB_WCAP: start | end << 16 (the rest: record slots)
};
#ifndef TKZ_BLK_MINW
#define TKZ_BLK_MINW 7  // (72 VGPRs, 21,600 B of LDS: 7 blocks per CU; 6: C1 +3 %, C5 +3.5 %)
#endif
#ifndef TKZ_BLK_ABL
#define TKZ_BLK_ABL 0
#endif
// k_encode_blk's barrier: orders the block's LDS traffic only. __syncthreads() is also a
// workgroup release of global memory (s_waitcnt vmcnt(0)): every barrier waited for the
// wave's outstanding record / token stores of the previous phase
#define EB_SYNC()                                                         \
    do {                                                                  \
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");   \
        __builtin_amdgcn_s_barrier();                                     \
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");   \
    } while (0)
#ifndef TKZ_BLK_DOCPF
#define TKZ_BLK_DOCPF 1  // k_encode_blk: the next chunk's chunk_doc / doc_off loaded during this chunk's words
#endif
#ifndef TKZ_BLK_PF
#define TKZ_BLK_PF 0  // k_encode_blk: the next chunk's bytes / boundaries into L2 during the words phase
#endif
#ifndef TKZ_BLK_W2
#define TKZ_BLK_W2 0  // k_encode_blk: two words per lane per round (measured slower: C1 1.21 vs 1.12 ms)
#endif

template <int MODEL, bool COMPACT>
__global__ __launch_bounds__(EB_T, TKZ_BLK_MINW) void k_encode_blk(DevTables T, const uint8_t* __restrict__ bytes,
                                                       const uint64_t* __restrict__ doc_off, uint64_t n_docs,
                                                       uint64_t limit, uint32_t ch_log2,
                                                       const uint64_t* __restrict__ chunk_doc,
                                                       unsigned long long* __restrict__ hdr, Scratch S,
                                                       uint32_t* __restrict__ chunk_words,
                                                       uint32_t* __restrict__ doc_word, Deferred D,
                                                       uint32_t* __restrict__ status) {
    // WordPiece: its three length buckets run in the kernel; BPE: misses of <= 8 B go to
    // the chunk's short list for k_bpe_short (no staging: an LDS fill counter per chunk),
    // longer ones are staged (queue 0) for k_bpe_deferred's list
    constexpr int NBK = MODEL == 1 ? 0 : Buckets<MODEL>::n;
    constexpr int SQ = 1, DQ = 0;
    constexpr int NQ = MODEL == 1 ? 1 : NBK;
    __shared__ EbSmem<NQ> sm;
    uint16_t* const lw16 = (uint16_t*)sm.went;
    const int t = (int)threadIdx.x, lane = lane_id(), wv = t >> 6;
    const uint64_t R0 = doc_off[0], R1 = doc_off[n_docs];
    const uint32_t CB = 1u << ch_log2;  // chunk bytes
    const uint64_t c_first = R0 >> ch_log2, c_end = (R1 + CB - 1) >> ch_log2;
    const bool memo = (MODEL == 1 && T.memo != nullptr) || (MODEL == 0 && T.wps != nullptr);
    const uint32_t* byte_id = T.byte_id;
    uint16_t* const h16 = (uint16_t*)S.wslot();
    uint32_t qn[NQ];
#pragma unroll
    for (int k = 0; k < NQ; ++k) qn[k] = 0;
    uint32_t n_words = 0, n_hits = 0;  // (per wave)
    if (t < (int)(EB_CH / 32)) sm.bd[t] = 0u;
    if (t == 0) sm.nb_rel = 0xFFFFFFFFu;
    uint64_t c_prev = ~0ull;
#ifdef TKZ_PHASES
    uint64_t ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t pt = __builtin_amdgcn_s_memtime();
#define EBP(k)                                           \
    do {                                                 \
        const uint64_t pt1 = __builtin_amdgcn_s_memtime(); \
        ph[k] += pt1 - pt;                               \
        pt = pt1;                                        \
    } while (0)
#else
#define EBP(k)
#endif
    EB_SYNC();
    // the chunk's first doc_off entries are loaded one chunk ahead (during the previous
    // chunk's words phase): chunk_doc -> doc_off was two dependent round trips per chunk
    uint64_t dk_nx = 0, b_nx = ~0ull;
    if (TKZ_BLK_DOCPF && c_first + blockIdx.x < c_end) {
        dk_nx = chunk_doc[c_first + blockIdx.x];
        b_nx = dk_nx + (uint64_t)t <= n_docs ? doc_off[dk_nx + (uint64_t)t] : ~0ull;
    }
    for (uint64_t c = c_first + blockIdx.x; c < c_end; c += gridDim.x) {
        const uint64_t cs = c << ch_log2, ce = cs + CB;
        const uint64_t dk_next = TKZ_BLK_DOCPF && c + gridDim.x < c_end ? chunk_doc[c + gridDim.x] : 0ull;
        // ---- (1) the bytes (registers, staged in LDS below); doc boundaries -> bitmap
        const uint64_t b0 = cs + 32u * (uint32_t)t;
        const bool cls = 32u * (uint32_t)t < CB;  // the thread classifies bytes of the chunk
        uint64_t v[4] = {0ull, 0ull, 0ull, 0ull};
        if (32u * (uint32_t)t < CB + EB_TAIL) {
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const uint64_t a = b0 + 16u * u;
                // chunk bytes: units with a byte in [R0, R1); tail (chunks < 8 KiB): readable units
                if (cls ? (a < R1 && a + 16u > R0) : (a + 16u <= limit)) {
                    const uint4 q = *(const uint4*)(bytes + a);
                    v[2 * u] = ((uint64_t)q.y << 32) | q.x;
                    v[2 * u + 1] = ((uint64_t)q.w << 32) | q.z;
                }
            }
        }
        // the tail of an 8-KiB chunk: threads 0..3, a 16-B unit each
        const bool tail_thr = CB == EB_CH && t < (int)(EB_TAIL / 16);
        uint64_t tv0 = 0ull, tv1 = 0ull;
        if (tail_thr && ce + 16u * (uint32_t)t + 16u <= limit) {
            const uint4 q = *(const uint4*)(bytes + ce + 16u * (uint32_t)t);
            tv0 = ((uint64_t)q.y << 32) | q.x;
            tv1 = ((uint64_t)q.w << 32) | q.z;
        }
        if (t == 0) {  // classes of byte cs - 1: a word running in belongs to the previous chunk
            uint32_t carry0 = 1u, d0 = 0u;
            if (cs > R0) {
                bool sp, pu;
                classify(lower(bytes[cs - 1], T.norm), T.pretok, sp, pu);
                carry0 = (uint32_t)sp | ((uint32_t)pu << 1);
                d0 = (!sp || pu) ? 1u : 0u;
            }
            sm.d0c = d0 | (carry0 << 1);
        }
        const uint64_t dk = TKZ_BLK_DOCPF ? dk_nx : chunk_doc[c];
        const uint64_t blim = min(ce, R1);  // boundaries this chunk owns: [cs, min(ce, R1))
        const uint64_t bfirst = TKZ_BLK_DOCPF ? b_nx : (dk + (uint64_t)t <= n_docs ? doc_off[dk + (uint64_t)t] : ~0ull);
        if (bfirst < blim) atomicOr(&sm.bd[(uint32_t)(bfirst - cs) >> 5], 1u << ((uint32_t)(bfirst - cs) & 31u));
        else if (bfirst != ~0ull) atomicMin(&sm.nb_rel, (uint32_t)min(bfirst - cs, (uint64_t)0xFFFFFFFFu));
        if (t == EB_T - 1) sm.more = bfirst < blim ? 1u : 0u;
        EBP(0);  // chunk loads (the wave waits for its doc_off load: the LDS OR)
        EB_SYNC();  // (A)
        EBP(1);
        const uint32_t d0c = sm.d0c, d0 = d0c & 1u;
        uint32_t rounds = 1;
        if (sm.more) {  // > 256 boundaries in the chunk (docs of < 32 B)
            bool more = true;
            while (more) {
                const uint64_t k = dk + (uint64_t)rounds * EB_T + (uint64_t)t;
                const uint64_t b = k <= n_docs ? doc_off[k] : ~0ull;
                if (b < blim) atomicOr(&sm.bd[(uint32_t)(b - cs) >> 5], 1u << ((uint32_t)(b - cs) & 31u));
                else if (b != ~0ull) atomicMin(&sm.nb_rel, (uint32_t)min(b - cs, (uint64_t)0xFFFFFFFFu));
                ++rounds;
                more = __syncthreads_or(t == EB_T - 1 && b < blim) != 0;
            }
        }
        if (t == 0) {
            sm.dfill = 0u;
            if (MODEL == 1) {
                if (c_prev != ~0ull) D.scnt[c_prev] = sm.sfill;
                sm.sfill = 0u;
            }
        }
        // ---- (2) classes, starts / ends, the block prefix sum
        uint32_t Sm = 0u, P = 0u;
        if (cls) {
            uint32_t vm = 0u;
            if (b0 < R1 && b0 + 32u > R0) {
                const uint32_t lo = R0 > b0 ? (uint32_t)(R0 - b0) : 0u;
                const uint32_t hi = (uint32_t)min(R1 - b0, (uint64_t)32u);
                vm = (hi == 32u ? 0xFFFFFFFFu : (1u << hi) - 1u) & ~((1u << lo) - 1u);
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                uint32_t sp, pu;
                class_masks(v[k], T.pretok, sp, pu);
                Sm |= sp << (8 * k);
                P |= pu << (8 * k);
            }
            Sm |= ~vm;  // invalid bytes split
            P &= vm;
        }
        if (32u * (uint32_t)t < CB + EB_TAIL) {
#pragma unroll
            for (int k = 0; k < 4; ++k) sm.stage[4 * t + k] = T.norm ? lower8(v[k]) : v[k];
        }
        if (tail_thr) {
            sm.stage[EB_CH / 8 + 2 * t] = T.norm ? lower8(tv0) : tv0;
            sm.stage[EB_CH / 8 + 2 * t + 1] = T.norm ? lower8(tv1) : tv1;
        }
        const uint32_t BD = cls ? sm.bd[t] : 0u;
        sm.xl[t] = (uint8_t)(((Sm >> 31) & 1u) | (((P >> 31) & 1u) << 1));
        EBP(2);  // classes + stage
        EB_SYNC();  // (B)
        EBP(1);
        if (t < (int)(EB_CH / 32)) sm.bd[t] = 0u;  // (read above; the next chunk's ORs follow barrier D)
        uint32_t starts = 0u, ends = 0u;
        if (cls) {
            const uint32_t prev = t == 0 ? d0c >> 1 : (uint32_t)sm.xl[t - 1];
            const uint32_t Sprev = (Sm << 1) | (prev & 1u), Pprev = (P << 1) | (prev >> 1);
            // start: word byte after a delimiter or at a doc boundary, or a punct byte; end
            // (exclusive): delimiter or boundary after a word byte, or the byte after a punct
            starts = (~Sm & (Sprev | BD)) | P;
            ends = (~Sprev & (Sm | BD)) | Pprev;
        }
        const uint32_t cnt = (uint32_t)__popc(starts) | ((uint32_t)__popc(ends) << 16);
        const uint32_t inc = (uint32_t)wave_incl_scan((int)cnt);
        if (lane == WAVE - 1) sm.wsum[wv] = inc;
        sm.st[t] = starts;
        sm.lex[t] = (uint16_t)((inc - cnt) & 0xFFFFu);
        EBP(3);  // starts / ends, wave scan
        EB_SYNC();  // (C)
        EBP(1);
        uint32_t woff = 0u, tot = 0u;
#pragma unroll
        for (int w = 0; w < EB_NW; ++w) {
            const uint32_t s = sm.wsum[w];
            woff += w < wv ? s : 0u;
            tot += s;
        }
        const uint32_t n_st = tot & 0xFFFFu, n_en = tot >> 16;
        {
            // word k: start in the low half of its record slot, end in the high half (offsets
            // from cs); the (k + d0)-th end closes word k
            const uint32_t ex = woff + inc - cnt;
            uint32_t k = ex & 0xFFFFu;
            for (uint32_t m = starts; m; m &= m - 1u, ++k) {
                const uint16_t o = (uint16_t)(32u * (uint32_t)t + (uint32_t)__builtin_ctz(m));
                if (k < EB_WCAP) lw16[2 * k] = o;
                else h16[2 * (cs + k)] = o;
            }
            int e = (int)(ex >> 16) - (int)d0;
            for (uint32_t m = ends; m; m &= m - 1u, ++e) {
                const uint16_t o = (uint16_t)(32u * (uint32_t)t + (uint32_t)__builtin_ctz(m));
                if (e >= 0 && (uint32_t)e < n_st) {
                    if ((uint32_t)e < EB_WCAP) lw16[2 * e + 1] = o;
                    else h16[2 * (cs + (uint32_t)e) + 1] = o;
                }
            }
        }
        // doc boundaries: the ordinal of the first word at or after each (k_compact's row_ptr)
        for (uint32_t r = 0; r < rounds; ++r) {
            const uint64_t k = dk + (uint64_t)r * EB_T + (uint64_t)t;
            const uint64_t b = r == 0 ? bfirst : (k <= n_docs ? doc_off[k] : ~0ull);
            if (b < blim) {
                const uint32_t o = (uint32_t)(b - cs), T5 = o >> 5, wT = T5 >> 6;
                uint32_t before = 0u;
#pragma unroll
                for (int w = 0; w < EB_NW; ++w) before += w < (int)wT ? sm.wsum[w] & 0xFFFFu : 0u;
                before += (uint32_t)sm.lex[T5] + (uint32_t)__popc(sm.st[T5] & ((1u << (o & 31u)) - 1u));
                doc_word[k] = before;
            }
        }
        if (t == 0) chunk_words[c] = n_st;
        EBP(4);  // scatter, doc_word
        // the chunk's last word runs past its end: close it (the first split byte at or past
        // ce, the next doc boundary, R1; the byte after a punct)
        const bool open = n_st > 0u && n_en < n_st + d0;
        if (wv == 0) {
            if (open) {
                const uint64_t nb = sm.nb_rel == 0xFFFFFFFFu ? ~0ull : cs + sm.nb_rel;
                const uint64_t lim = min(R1, nb);
                uint64_t q_end;
                if (sm.xl[CB / 32 - 1] & 2u) {
                    q_end = ce;  // the open word is the punct byte ce - 1
                } else {
                    const uint32_t j = CB + (uint32_t)lane;
                    const uint32_t by = (uint32_t)(sm.stage[j >> 3] >> ((j & 7u) * 8u)) & 0xFFu;
                    bool sp, pu;
                    classify(by, T.pretok, sp, pu);
                    const uint64_t m = __ballot(sp || ce + (uint64_t)lane >= lim);
                    if (m) {
                        q_end = ce + (uint64_t)(__ffsll((long long)m) - 1);
                    } else {  // a word of > 64 B past the chunk: 1-KiB steps over global memory
                        q_end = lim;
                        for (uint64_t q = ce + EB_TAIL; q < lim; q += (uint64_t)STEP) {
                            const uint64_t a = q + 16u * (uint32_t)lane;
                            uint64_t x0 = 0ull, x1 = 0ull;
                            if (a < lim) {
                                const uint4 qq = *(const uint4*)(bytes + a);
                                x0 = ((uint64_t)qq.y << 32) | qq.x;
                                x1 = ((uint64_t)qq.w << 32) | qq.z;
                            }
                            uint32_t s0, p0, s1, p1;
                            class_masks(x0, T.pretok, s0, p0);
                            class_masks(x1, T.pretok, s1, p1);
                            uint32_t sm16 = s0 | (s1 << 8);
                            if (a + 16u > lim) sm16 |= a >= lim ? 0xFFFFu : ~((1u << (uint32_t)(lim - a)) - 1u) & 0xFFFFu;
                            const uint64_t mm = __ballot(sm16 != 0u);
                            if (mm) {
                                const int l = __ffsll((long long)mm) - 1;
                                const uint32_t sl = (uint32_t)__shfl((int)sm16, l, 64);
                                q_end = min(lim, q + 16u * (uint64_t)l + (uint64_t)__builtin_ctz(sl));
                                break;
                            }
                        }
                    }
                }
                if (lane == 0) sm.open_end = (uint32_t)min(q_end - cs, (uint64_t)0xFFFFFFFFu);
            }
            if (lane == 0) sm.nb_rel = 0xFFFFFFFFu;
        }
        if (n_st > EB_WCAP) __threadfence_block();  // (words past EB_WCAP: their entries in global memory)
        EBP(5);  // the open word
        EB_SYNC();  // (D)
        EBP(1);
        // ---- (3) one lane per word (TKZ_BLK_W2: two words per lane, their memo probes issued
        // together): memo probe, records; misses to the queues
        const uint32_t open_end = sm.open_end;
        if (TKZ_BLK_DOCPF && c + gridDim.x < c_end) {
            dk_nx = dk_next;
            b_nx = dk_nx + (uint64_t)t <= n_docs ? doc_off[dk_nx + (uint64_t)t] : ~0ull;
        }
        uint32_t ctok = 0;
        // the next chunk's bytes and its chunk_doc entry into L2 while this chunk's words run
        // (loads whose values only feed a register kept live to the chunk's end)
        const uint64_t c_nx = c + gridDim.x;
        uint32_t pf = 0;
        if (TKZ_BLK_PF && c_nx < c_end) {
            const uint64_t a = (c_nx << ch_log2) + 128u * (uint32_t)t;
            if (t < (int)(CB / 128u) && a + 4u <= limit) pf = *(const uint32_t*)(bytes + a);
            else if (t == EB_T - 1) pf = (uint32_t)chunk_doc[c_nx];
        }
        // word `ord` of the chunk: its length, position and (<= 16 B, memo) normalized key
        auto prep = [&](uint32_t ord, bool& act, uint32_t& L, uint64_t& pos, uint64_t& k0, uint64_t& k1) {
            act = ord < n_st;
            L = 0;
            pos = 0;
            k0 = k1 = 0;
            if (act) {
                // (two loads and a select: a pointer select compiled to a FLAT load, whose wait
                // is also a wait for every outstanding global store of the wave)
                uint32_t e32 = sm.went[min(ord, EB_WCAP - 1u)];
                asm volatile("" : "+v"(e32));
                if (ord >= EB_WCAP) e32 = S.wslot()[cs + ord];
                const uint32_t s = e32 & 0xFFFFu;
                const uint32_t en = (open && ord == n_st - 1u) ? open_end : (e32 >> 16);
                L = en - s;
                pos = cs + s;
                if (memo && L <= 16u) {
                    const uint32_t a = s >> 3, sh = (s & 7u) * 8u;
                    const uint64_t q0 = sm.stage[a], q1 = sm.stage[a + 1], q2 = sm.stage[a + 2];
                    k0 = sh ? (q0 >> sh) | (q1 << (64u - sh)) : q0;
                    k1 = sh ? (q1 >> sh) | (q2 << (64u - sh)) : q1;
                    k0 &= (2ull << (8u * min(L, 8u) - 1u)) - 1u;
                    k1 = L > 8u ? k1 & ((2ull << (8u * (L - 8u) - 1u)) - 1u) : 0ull;
                }
            }
        };
        // the word's record (a memo hit; WordPiece: the whole-word probe here) or its queue
        // entry; wave-collective (converged)
        auto finish = [&](bool act, uint32_t ord, uint32_t L, uint64_t pos, uint64_t k0, uint64_t k1, bool hit,
                          uint4 r) {
            const uint64_t ws = cs + ord;
            int bk = -1, dl = -1;
            uint64_t ent = 0;
#if TKZ_BLK_ABL  // timing only (wrong results): 1 no word work, 2 keys but no memo probe
            if (act) S.single_nc(ws, TKZ_BLK_ABL == 2 ? short_key_hash(k0, k1, L) & 0xFFFFu : L);
            ctok += (uint32_t)__popcll(__ballot(act));
            return;
#endif
            uint32_t hmeta = r.x, hw = r.y, ht1 = r.z, ht2 = r.w;
            if (act) {
                bool done = hit;
                if (MODEL == 0 && memo && L <= 16u && L <= T.max_chars && L <= T.max_key) {
                    const uint32_t id = wps_probe(T, k0, k1, L);
                    if (id != NONE) {
                        if (T.narrow) {
                            S.single_nc(ws, id | (L << 24));
                        } else {
                            S.ids()[pos] = id;
                            S.offs()[pos] = (uint64_t)L << 32;
                            S.wide_nc(ws, pos, 1);
                        }
                        done = hit = true;
                    }
                }
                if (!done) {
                    if (MODEL == 1) dl = L > 8u ? DQ : SQ;  // k_bpe_deferred / k_bpe_short
                    else bk = bucket_of<MODEL>(L);
                    ent = pos | ((uint64_t)ord << POS_BITS) | ((uint64_t)min(L, LEN_ESC) << LEN_SHIFT);
                    if (L >= LEN_ESC) S.prs()[pos] = L;  // full length for the long path
                }
            }
            if (MODEL == 1 && memo && !COMPACT && !T.mid) {
                const uint32_t nt = hit ? (hmeta >> 5) & 3u : 0u;
                if (hit) memo_emit_wide(S, nt, hw, ht1, ht2, pos, ws);
                ctok += lane63((uint32_t)wave_incl_scan((int)nt));
            } else if (MODEL == 1 && memo) {
                // 2-3 tokens to the front of the chunk's dense area (an LDS fill counter per
                // chunk, one atomic per wave batch)
                const uint32_t nt = hit ? (hmeta >> 5) & 3u : 0u;
                const uint64_t m1 = __ballot(nt == 1u), m2 = __ballot(nt == 2u), m3 = __ballot(nt == 3u);
                const uint32_t need = 2u * (uint32_t)__popcll(m2) + 3u * (uint32_t)__popcll(m3);
                uint32_t fb = 0;
                if (need && lane == 0) fb = atomicAdd(&sm.dfill, need);
                fb = rfl(fb);
                if (hit) {
                    const uint32_t off = fb + 2u * lanes_below(m2) + 3u * lanes_below(m3);
                    if (!COMPACT) {  // T.mid: the wide memo's tokens (id | start << 22 | end << 27) packed
                        hw = mid_tok(hw & 0x3FFFFFu, (hw >> 22) & 31u, hw >> 27);
                        ht1 = mid_tok(ht1 & 0x3FFFFFu, (ht1 >> 22) & 31u, ht1 >> 27);
                        ht2 = mid_tok(ht2 & 0x3FFFFFu, (ht2 >> 22) & 31u, ht2 >> 27);
                    }
                    memo_emit(S, COMPACT && L <= 8u, hmeta, hw, ht1, ht2, L, ws, S.dtok() + S.dbase(cs) + off, off);
                }
                ctok += (uint32_t)__popcll(m1) + need;
            } else if (MODEL == 0 && memo) {
                ctok += (uint32_t)__popcll(__ballot(hit));
            }
            n_words += (uint32_t)__popcll(__ballot(act));
            n_hits += (uint32_t)__popcll(__ballot(hit));
            // misses to the wave's queues; a queue of >= 64 runs (each held <= 63 before)
            if (MODEL == 1) {
                const uint64_t ms = __ballot(dl == SQ);
                if (ms) {  // to the chunk's short list: contiguous, one LDS atomic per wave batch
                    uint32_t b = 0;
                    if (lane == 0) b = atomicAdd(&sm.sfill, (uint32_t)__popcll(ms));
                    b = rfl(b);
                    if (dl == SQ) D.slist[cs + b + lanes_below(ms)] = ent;
                }
                const uint64_t m = __ballot(dl == DQ);
                if (dl == DQ) sm.q[wv][DQ][qn[DQ] + lanes_below(m)] = ent;
                qn[DQ] += (uint32_t)__popcll(m);
            }
#pragma unroll
            for (int bb = 0; bb < NBK; ++bb) {
                const uint64_t m = __ballot(bk == bb);
                if (bk == bb) sm.q[wv][bb][qn[bb] + lanes_below(m)] = ent;
                qn[bb] += (uint32_t)__popcll(m);
            }
            WAVE_SYNC();
            if (MODEL == 1) {
                if (qn[DQ] >= (uint32_t)WAVE) {
                    qn[DQ] -= WAVE;
                    uint32_t b = 0;
                    if (lane == 0) b = atomicAdd(D.cnt, (uint32_t)WAVE);
                    b = rfl(b);
                    D.list[b + lane] = sm.q[wv][DQ][qn[DQ] + lane];
                }
            }
#pragma unroll
            for (int bb = 0; bb < NBK; ++bb) {
                if (qn[bb] >= (uint32_t)WAVE) {
                    qn[bb] -= WAVE;
                    run_bucket<MODEL, COMPACT>(T, byte_id, &sm.q[wv][bb][qn[bb]], bb, WAVE, bytes, limit, S, status);
                }
            }
            WAVE_SYNC();
        };
        if (MODEL == 1 && !TKZ_BLK_ABL) {
            // BPE: the same work with few divergent branches (each one is 3-4 scalar
            // instructions of exec-mask bookkeeping, and the CU's one scalar unit issues them
            // for all its waves: round 6's first k_encode_blk issued 335M SALU per C1 launch,
            // about half the kernel's time at one per cycle per CU). Inactive lanes read the
            // chunk's last word; one memo probe round for every lane, further rounds only for
            // the lanes that need them; records and tokens computed with selects.
            const uint32_t* ms8 = (const uint32_t*)T.memo8;
            (void)ms8;
            for (uint32_t base = 64u * (uint32_t)wv; base < n_st; base += EB_T) {
                const uint32_t ord = base + (uint32_t)lane;
                const bool act = ord < n_st;
                const uint32_t oc = act ? ord : n_st - 1u;
                uint32_t e32 = sm.went[min(oc, EB_WCAP - 1u)];
                asm volatile("" : "+v"(e32));  // (not merged with the global load into a FLAT load)
                if (base + (uint32_t)WAVE > EB_WCAP && oc >= EB_WCAP) e32 = S.wslot()[cs + oc];
                const uint32_t s0 = e32 & 0xFFFFu;
                const uint32_t en = (open && oc == n_st - 1u) ? open_end : (e32 >> 16);
                const uint32_t L = en - s0;
                const uint64_t pos = cs + s0, ws = cs + ord;
                const uint32_t Lk = min(max(L, 1u), 16u);
                bool hit = false;
                uint32_t hmeta = 0, hw = 0, ht1 = 0, ht2 = 0;
                if (memo) {
                    const uint32_t a = s0 >> 3, sh = (s0 & 7u) * 8u;
                    const uint64_t q0 = sm.stage[a], q1 = sm.stage[a + 1], q2 = sm.stage[a + 2];
                    uint64_t k0 = sh ? (q0 >> sh) | (q1 << (64u - sh)) : q0;
                    uint64_t k1 = sh ? (q1 >> sh) | (q2 << (64u - sh)) : q1;
                    k0 &= (2ull << (8u * min(Lk, 8u) - 1u)) - 1u;
                    k1 = Lk > 8u ? k1 & ((2ull << (8u * (Lk - 8u) - 1u)) - 1u) : 0ull;
                    const bool s8 = COMPACT && Lk <= 8u;
                    uint32_t h = short_key_hash(k0, k1, Lk) >> (32 - (s8 ? T.memo8_bits : T.memo_bits));
                    bool pend = act && L <= 16u;
                    while (true) {  // (one round for nearly every lane: load <= 1/8)
                        const uint4* pp = s8 ? T.memo8 + h : T.memo + 2 * h;
                        const uint4 e0 = pp[0];
                        uint4 e1 = make_uint4(0u, 0u, 1u, 0u);
                        if (!s8) e1 = pp[1];
                        const bool h0 = (((uint64_t)e0.y << 32) | e0.x) == k0 && (e0.z & 0x1Fu) == Lk;
                        const bool c0 = s8 || (((uint64_t)e1.y << 32) | e1.x) == k1;
                        const bool found = pend && h0 && c0;
                        hmeta = found ? e0.z : hmeta;
                        hw = found ? e0.w : hw;
                        ht1 = found ? e1.z : ht1;
                        ht2 = found ? e1.w : ht2;
                        hit = hit || found;
                        pend = pend && !found && e0.z != 0u;
                        if (!__ballot(pend)) break;
                        h += pend ? 1u : 0u;
                    }
                }
                const uint32_t nt = hit ? (hmeta >> 5) & 3u : 0u;
                const uint64_t m1 = __ballot(nt == 1u), m2 = __ballot(nt == 2u), m3 = __ballot(nt == 3u);
                const uint32_t need = 2u * (uint32_t)__popcll(m2) + 3u * (uint32_t)__popcll(m3);
                uint32_t fb = 0;
                if (need && lane == 0) fb = atomicAdd(&sm.dfill, need);
                fb = rfl(fb);
                const uint32_t off = fb + 2u * lanes_below(m2) + 3u * lanes_below(m3);
                // tokens: packed 16-B slot (L <= 8) or the 32-B slot's three; T.mid: re-packed
                const bool pk = COMPACT && L <= 8u;
                const uint32_t b0 = (hmeta >> 7) & 0xFu, b1 = nt == 3u ? (hmeta >> 11) & 0xFu : L;
                uint32_t t0 = hw, t1 = ht1, t2 = ht2;
                if (!COMPACT) {  // T.mid: the wide memo's tokens (id | start << 22 | end << 27) packed
                    t0 = mid_tok(t0 & 0x3FFFFFu, (t0 >> 22) & 31u, t0 >> 27);
                    t1 = mid_tok(t1 & 0x3FFFFFu, (t1 >> 22) & 31u, t1 >> 27);
                    t2 = mid_tok(t2 & 0x3FFFFFu, (t2 >> 22) & 31u, t2 >> 27);
                }
                const uint32_t rec = nt == 1u ? t0 : (REC_MULTI | REC_DENSE | (nt << REC_CNT) | (nt >= 2u ? off : 0u));
                if (pk) {  // the 16-B slot's packed form: ids in w, split points and id 2 in the meta
                    t0 = (hw & 0xFFFFu) | (b0 << 24);
                    t1 = (hw >> 16) | (b0 << 16) | (b1 << 24);
                    t2 = (hmeta >> 15) | (b1 << 16) | (L << 24);
                }
                if (hit) S.wslot()[ws] = rec;
                if (nt >= 2u) {
                    uint32_t* dst = S.dtok() + S.dbase(cs) + off;
                    dst[0] = t0;
                    dst[1] = t1;
                    if (nt == 3u) dst[2] = t2;
                }
                ctok += (uint32_t)__popcll(m1) + need;
                n_hits += (uint32_t)__popcll(__ballot(hit));
                // misses: <= 8 B to the chunk's short list, longer ones staged for the deferred list
                const bool miss = act && !hit;
                const uint64_t ent = pos | ((uint64_t)ord << POS_BITS) | ((uint64_t)min(L, LEN_ESC) << LEN_SHIFT);
                if (miss && L >= LEN_ESC) S.prs()[pos] = L;  // full length for the long path
                const uint64_t mss = __ballot(miss && L <= 8u), msd = __ballot(miss && L > 8u);
                if (mss) {
                    uint32_t b = 0;
                    if (lane == 0) b = atomicAdd(&sm.sfill, (uint32_t)__popcll(mss));
                    b = rfl(b);
                    if (miss && L <= 8u) D.slist[cs + b + lanes_below(mss)] = ent;
                }
                if (msd) {
                    if (miss && L > 8u) sm.q[wv][DQ][qn[DQ] + lanes_below(msd)] = ent;
                    qn[DQ] += (uint32_t)__popcll(msd);
                    if (qn[DQ] >= (uint32_t)WAVE) {
                        WAVE_SYNC();
                        qn[DQ] -= WAVE;
                        uint32_t b = 0;
                        if (lane == 0) b = atomicAdd(D.cnt, (uint32_t)WAVE);
                        b = rfl(b);
                        D.list[b + lane] = sm.q[wv][DQ][qn[DQ] + lane];
                        WAVE_SYNC();
                    }
                }
            }
            if (wv == 0 && lane == 0) n_words += n_st;
        } else {
            for (uint32_t base = 64u * (uint32_t)wv; base < n_st; base += EB_T) {
                bool aA;
                uint32_t LA;
                uint64_t pA, kA0, kA1;
                prep(base + (uint32_t)lane, aA, LA, pA, kA0, kA1);
                finish(aA, base + (uint32_t)lane, LA, pA, kA0, kA1, false, make_uint4(0u, 0u, 0u, 0u));
            }
        }
        if (lane == 0 && ctok) atomicAdd(S.ccnt() + c, ctok);
        if (TKZ_BLK_PF && t == EB_T - 1 && c_nx < c_end) {  // and the first doc_off line of the next chunk
            const uint64_t dn = pf;  // (the low half of chunk_doc[c_nx]; only an address hint)
            if (dn <= n_docs) pf += (uint32_t)doc_off[dn];
        }
        asm volatile("" ::"v"(pf));
        EBP(6);  // words
        c_prev = c;
    }
    if (MODEL == 1) {
        EB_SYNC();
        if (t == 0 && c_prev != ~0ull) D.scnt[c_prev] = sm.sfill;
    }
    // the waves' partial queues
    if (MODEL == 1 && qn[DQ] > 0u) {
        uint32_t b = 0;
        if (lane == 0) b = atomicAdd(D.cnt, qn[DQ]);
        b = rfl(b);
        if ((uint32_t)lane < qn[DQ]) D.list[b + lane] = sm.q[wv][DQ][lane];
    }
#pragma unroll
    for (int bb = 0; bb < NBK; ++bb) {
        if (qn[bb] > 0u) run_bucket<MODEL, COMPACT>(T, byte_id, &sm.q[wv][bb][0], bb, qn[bb], bytes, limit, S, status);
    }
    if (lane == 0) {
        if (n_words) atomicAdd(hdr + HDR_WORDS, (unsigned long long)n_words);
        if (n_hits) atomicAdd(hdr + HDR_HITS, (unsigned long long)n_hits);
    }
#ifdef TKZ_PHASES
    EBP(7);  // tail: the last flushes
    if (lane == 0)
        for (int k = 0; k < 8; ++k) atomicAdd(&D.dbg[k], (unsigned long long)ph[k]);
#endif
#undef EBP
}

// ---------------------------------------------------------------------------
// token counts of 8 word records r[0..8) (words w0..w0+7 of a chunk; w >= W: none);
// bits of `kind`: 2 per word (0 single narrow token = the record, 1 narrow multi, 2 wide)
// ---------------------------------------------------------------------------
template <bool SEGW>  // (SEGW: REC_SEG records may occur)
__device__ __forceinline__ uint32_t rec_counts(const Scratch& S, uint64_t cs, uint32_t w0, uint32_t W,
                                               const uint32_t (&r)[8], uint32_t (&c)[8], uint32_t& kind) {
    uint32_t s = 0;
    kind = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const uint32_t x = r[j];
        uint32_t n = w0 + j < W ? rec_count(x) : 0u;
        uint32_t k = 0;
        if (x & REC_MULTI) {
            k = (x & REC_WIDE) ? 2u : 1u;
            if (k == 2u && n == NARROW_MAX)
                n = ((SEGW && (x & REC_SEG) == REC_SEG) ? S.ids() : S.prs())[cs + (x & REC_OFF)];
        }
        c[j] = n;
        kind |= k << (2 * j);
        s += n;
    }
    return s;
}

// ---------------------------------------------------------------------------
// scan of per-doc counts -> row_ptr (u64, n+1)
// ---------------------------------------------------------------------------
constexpr int SCAN_T = 256;
constexpr int SCAN_IT = 16;
constexpr int SCAN_CHUNK = SCAN_T * SCAN_IT;
uint64_t scan_chunk_elems() { return SCAN_CHUNK; }  // elements per k_scan_partials block

__device__ __forceinline__ uint64_t block_excl_scan(uint64_t v, uint64_t* tmp, uint64_t& total) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    uint64_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint64_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) tmp[w] = x;
    __syncthreads();
    uint64_t off = 0;
    for (int i = 0; i < w; ++i) off += tmp[i];
    total = 0;
    for (int i = 0; i < SCAN_T / 64; ++i) total += tmp[i];
    __syncthreads();
    return off + x - v;
}

__global__ __launch_bounds__(SCAN_T) void k_scan_partials(const uint32_t* __restrict__ counts, uint64_t n,
                                                          uint64_t* __restrict__ partials) {
    __shared__ uint64_t tmp[SCAN_T / 64];
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_CHUNK;
    uint64_t s = 0;
    for (int i = 0; i < SCAN_IT; ++i) {
        const uint64_t k = base + (uint64_t)i * SCAN_T + threadIdx.x;
        if (k < n) s += counts[k];
    }
    uint64_t total;
    block_excl_scan(s, tmp, total);
    if (threadIdx.x == 0) partials[blockIdx.x] = total;
}

__global__ __launch_bounds__(SCAN_T) void k_scan_top(uint64_t* __restrict__ partials, uint64_t nb,
                                                     unsigned long long* __restrict__ hdr, int dedup) {
    __shared__ uint64_t tmp[SCAN_T / 64];
    if (hdr && threadIdx.x == 0) {  // encode: this sub-batch's deferred / long-word counts -> statistics
        const uint32_t* dc = (const uint32_t*)(hdr + HDR_DEFER);
        hdr[HDR_DEFERRED] += dc[0];
        hdr[HDR_OWNERS] += dedup ? dc[1] : dc[0];  // the words k_bpe_deferred ran on
        hdr[HDR_LONGW] += ((const uint32_t*)(hdr + HDR_LONG))[0];
        hdr[HDR_SUBS] += 1;
    }
    uint64_t carry = 0;
    for (uint64_t b0 = 0; b0 < nb; b0 += SCAN_T) {
        const uint64_t k = b0 + threadIdx.x;
        const uint64_t v = k < nb ? partials[k] : 0;
        uint64_t total;
        const uint64_t e = block_excl_scan(v, tmp, total);
        if (k < nb) partials[k] = carry + e;
        carry += total;
    }
}

// row_ptr[k] = base + exclusive prefix of counts; *base_out = the total (the token base
// of the next sub-batch). base_in / base_out may be null (base 0, not recorded).
__global__ __launch_bounds__(SCAN_T) void k_scan_final(const uint32_t* __restrict__ counts, uint64_t n,
                                                       const uint64_t* __restrict__ partials,
                                                       uint64_t* __restrict__ row_ptr,
                                                       const unsigned long long* __restrict__ base_in,
                                                       unsigned long long* __restrict__ base_out) {
    __shared__ uint64_t tmp[SCAN_T / 64];
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_CHUNK + (uint64_t)threadIdx.x * SCAN_IT;
    uint32_t c[SCAN_IT];
    uint64_t s = 0;
#pragma unroll
    for (int i = 0; i < SCAN_IT; ++i) {
        const uint64_t k = base + i;
        c[i] = k < n ? counts[k] : 0;
        s += c[i];
    }
    uint64_t total;
    uint64_t off = partials[blockIdx.x] + block_excl_scan(s, tmp, total) + (base_in ? *base_in : 0ull);
#pragma unroll
    for (int i = 0; i < SCAN_IT; ++i) {
        const uint64_t k = base + i;
        if (k < n) row_ptr[k] = off;
        off += c[i];
        if (k + 1 == n) {
            row_ptr[n] = off;
            if (base_out) *base_out = off;
        }
    }
}


// ---------------------------------------------------------------------------
// compaction: dense word slots -> CSR (batch order), one wave per chunk; also writes
// row_ptr[k] for the doc boundaries inside the chunk (from the boundary's word ordinal)
// ---------------------------------------------------------------------------
#ifndef TKZ_CABL
#define TKZ_CABL 0  // k_compact traffic ablations (wrong results): 1 no scratch token loads, 2 no offsets, 3 no CSR
#endif
constexpr int CTMP = 1024;  // LDS source table per wave (tokens of 512 words)

// LDS source table entry of one output token: bit 31 clear = the narrow token itself
// (word-slot singles); set = scratch source: bit 30 = wide (bits 0..29 = chunk-relative
// offset into ids / offs), else narrow at bits 0..28 of the chunk's dense area (bit 29)
// or of the word-bound tok array. Emits the token of entry e, with the narrow scratch
// word x = tok[src] already loaded (ignored unless the entry is a narrow scratch source)
__device__ __forceinline__ void emit_token_x(const Scratch& S, uint64_t cs, uint32_t e, uint32_t x, uint32_t* ids,
                                             uint64_t* offs, uint64_t o, bool mid) {
    if ((e >> 30) == 3u) {  // wide (rare): dependent loads
        const uint64_t src = cs + (e & 0x3FFFFFFFu);
        ids[o] = S.ids()[src];
        offs[o] = S.offs()[src];
        return;
    }
    const uint32_t v = (e >> 31) ? x : e;
#if TKZ_CABL == 2  // traffic only: ids stored, offsets not (wrong results)
    ids[o] = v;
    return;
#elif TKZ_CABL == 3  // traffic only: no CSR stores (wrong results)
    if (v == 0xFFFFFFFFu) ids[o] = v;
    return;
#endif
    if (mid) {  // id | start << 20 | (end - 1) << 26
        ids[o] = v & 0xFFFFFu;
        offs[o] = (uint64_t)((v >> 20) & 63u) | ((uint64_t)((v >> 26) + 1u) << 32);
    } else {
        ids[o] = v & 0xFFFFu;
        offs[o] = (uint64_t)((v >> 16) & 0xFFu) | ((uint64_t)(v >> 24) << 32);
    }
}
#ifndef TKZ_CU
#define TKZ_CU 10  // output tokens per lane per k_compact emission round
#endif
#ifndef TKZ_ALIGN_OUT
#define TKZ_ALIGN_OUT 0  // k_compact's stores aligned to 64 output tokens (A/B knob)
#endif
// the LDS source entry of token k of a word with record sl
__device__ __forceinline__ uint32_t token_src(uint32_t kind, uint32_t sl, uint32_t k) {
    if (kind == 0) return sl;
    if (kind == 2) return 0xC0000000u | ((sl & REC_OFF) + k);
    return 0x80000000u | (sl & REC_DENSE) | ((sl & REC_OFF) + k);
}

#ifndef TKZ_COMPACT_MINB
#define TKZ_COMPACT_MINB 7  // waves per SIMD (7 vs 6: k_compact -1...-3 %, profiles/r03e_ab.txt)
#endif
// SEGW: the call's segmented pretokens carry REC_SEG records (k_seg_count): their groups go
// to k_compact_long, which records their output positions for k_seg_emit
template <bool SEGW>
__global__ __launch_bounds__(256, TKZ_COMPACT_MINB) void k_compact(const uint64_t* __restrict__ doc_off, uint64_t n_docs,
                                                 uint32_t ch_log2, uint64_t n_chunks,
                                                 const uint64_t* __restrict__ chunk_doc,
                                                 const uint64_t* __restrict__ chunk_base, Scratch S,
                                                 const uint32_t* __restrict__ chunk_words,
                                                 const uint32_t* __restrict__ doc_word,
                                                 uint64_t* __restrict__ row_ptr, uint32_t* __restrict__ ids,
                                                 uint64_t* __restrict__ offs, uint64_t* __restrict__ lg_list,
                                                 uint32_t* __restrict__ lg_cnt, int mid) {
    __shared__ uint32_t tmp_all[4][CTMP];  // per wave: boundary prefixes, then the source table
    const int lane = lane_id();
    uint32_t* tmp = tmp_all[threadIdx.x >> 6];
    uint32_t* pre = tmp;
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    const uint64_t R0 = doc_off[0], R1 = doc_off[n_docs];
    const uint64_t c_lo = R0 >> ch_log2, c_end = (R1 + (1ull << ch_log2) - 1) >> ch_log2;
    if (wave == 0) {
        // boundaries at R1 (the end of the last doc and trailing empty docs) follow every token
        const uint64_t tot = chunk_base[n_chunks];
        for (uint64_t k0 = 0; k0 <= n_docs; k0 += WAVE) {
            const uint64_t k = n_docs - k0 - (uint64_t)lane;
            const bool at_end = k0 + (uint64_t)lane <= n_docs && doc_off[k] == R1;
            if (at_end) row_ptr[k] = tot;
            if (__ballot(at_end) != ~0ull) break;
        }
    }
    for (uint64_t c = c_lo + wave; c < c_end; c += nw) {
        const uint64_t cs = c << ch_log2;
        const uint64_t bend = min(cs + (1ull << ch_log2), R1);  // boundaries this chunk resolves
        const uint32_t W = chunk_words[c];
        uint64_t out = chunk_base[c];
        uint64_t dk = chunk_doc[c];
        const uint32_t* tsrc = S.tok() + cs;                // word-bound narrow tokens
        const uint32_t* dsrc = S.dtok() + S.dbase(cs);      // the chunk's dense area
        for (uint32_t g0 = 0; g0 < W; g0 += GROUP) {
            const uint32_t w0 = g0 + 8u * (uint32_t)lane;
            // the next 64 doc boundaries, loaded together with this group's word data
            uint64_t bk = dk + (uint64_t)lane;
            uint64_t bv = doc_off[bk <= n_docs ? bk : n_docs];
            uint32_t bow = doc_word[bk <= n_docs ? bk : n_docs];
            // word counts and slots (tokens of singles) of this lane's 8 words: unconditional
            // loads (lanes past W read the chunk's first words and discard them), issued
            // with the boundary loads: one memory round trip (loads under a branch were
            // each followed by a wait)
            const uint32_t wi = w0 < W ? w0 : 0u;
            const uint4 sa = *(const uint4*)(S.wslot() + cs + wi);
            const uint4 sb = *(const uint4*)(S.wslot() + cs + wi + 4);
            uint32_t cc[8], kd;
            const uint32_t sl[8] = {sa.x, sa.y, sa.z, sa.w, sb.x, sb.y, sb.z, sb.w};
            const uint32_t s = rec_counts<SEGW>(S, cs, w0, W, sl, cc, kd);
            PH_MARK("c_counts");
            const int inc = wave_incl_scan((int)s);
            const uint32_t tot = (uint32_t)__shfl(inc, WAVE - 1, WAVE);
            const uint32_t o0 = (uint32_t)(inc - (int)s);
            // (a segmented pretoken's tokens are written after the compaction: k_compact_long
            // records its output position)
            bool segw = false;
            if (SEGW) {
#pragma unroll
                for (int j = 0; j < 8; ++j) segw = segw || (w0 + (uint32_t)j < W && (sl[j] & REC_SEG) == REC_SEG);
            }
            const bool long_grp = tot > (uint32_t)CTMP || __ballot(s > 64u || segw) != 0ull;
            // doc boundaries whose first word is in this group: tokens before it (64 at a time)
            {
                uint32_t o = o0;
#pragma unroll
                for (int j = 0; j < 8; ++j) { pre[8 * lane + j] = o; o += cc[j]; }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                while (true) {
                    const bool in = bk <= n_docs && bv < bend && bow < g0 + GROUP;
                    if (in) row_ptr[bk] = out + pre[bow - g0];
                    const int n_in = __popcll(__ballot(in));
                    dk += (uint64_t)n_in;
                    if (n_in < WAVE) break;
                    bk = dk + (uint64_t)lane;  // 64 boundaries in one group: load the next 64
                    bv = doc_off[bk <= n_docs ? bk : n_docs];
                    bow = doc_word[bk <= n_docs ? bk : n_docs];
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
            PH_MARK("c_bounds");
            if (tot == 0) continue;
            // (a lane whose words hold many tokens would fill the table alone: word by word)
            if (!long_grp) {
                uint32_t o = o0;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const uint32_t kind = (kd >> (2 * j)) & 3u;
                    for (uint32_t k = 0; k < cc[j]; ++k) tmp[o + k] = token_src(kind, sl[j], k);
                    o += cc[j];
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                PH_MARK("c_fill");
                // TKZ_CU tokens per lane per round: every scratch load of the round is issued
                // before any store (one memory round trip per round, not one per 64 tokens)
                // TKZ_ALIGN_OUT: lanes map to output positions aligned to 64 tokens (mis = out
                // mod 64), so every 64-lane store covers whole 128-B lines but at the ends
#if TKZ_ALIGN_OUT
                const uint32_t mis = (uint32_t)out & 63u;
#else
                const uint32_t mis = 0;
#endif
                for (uint32_t u0 = 0; u0 < tot + mis; u0 += TKZ_CU * WAVE) {
                    uint32_t e[TKZ_CU], x[TKZ_CU];
#pragma unroll
                    for (int k = 0; k < TKZ_CU; ++k) {
                        const uint32_t t = u0 + (uint32_t)(k * WAVE + lane) - mis;  // wraps below 0
                        e[k] = t < tot ? tmp[t] : 0u;
                    }
#pragma unroll
                    for (int k = 0; k < TKZ_CU; ++k)
#if TKZ_CABL == 1  // timing / traffic only: no scratch token loads (wrong results)
                        x[k] = e[k];
#else
                        x[k] = (((e[k] >> 29) & 1u) ? dsrc : tsrc)[(e[k] >> 31) ? (e[k] & 0x1FFFFFFFu) : 0u];
#endif
#pragma unroll
                    for (int k = 0; k < TKZ_CU; ++k) {
                        const uint32_t t = u0 + (uint32_t)(k * WAVE + lane) - mis;
                        if (t < tot) emit_token_x(S, cs, e[k], x[k], ids, offs, out + t, mid != 0);
                    }
                }
                __builtin_amdgcn_wave_barrier();
            } else {
                // more tokens than the source table, or long words (a one-pretoken doc of
                // 512 B holds ~120 tokens): listed for k_compact_long (its code here cost
                // the common path an occupancy step)
                if (lane == 0) {
                    const uint32_t i = atomicAdd(lg_cnt, 1u);
                    lg_list[2 * i] = c | ((uint64_t)g0 << 40);
                    lg_list[2 * i + 1] = out;
                }
                __builtin_amdgcn_wave_barrier();
            }
            PH_MARK("c_emit");
            out += tot;
        }
        // boundaries after the chunk's last word
        while (true) {
            const uint64_t k = dk + (uint64_t)lane;
            const bool in = k <= n_docs && doc_off[k] < bend;
            if (in) row_ptr[k] = out;
            const int n_in = __popcll(__ballot(in));
            dk += (uint64_t)n_in;
            if (n_in < WAVE) break;
        }
    }
}

// k_compact's groups of long words (listed by k_compact: {chunk | first word << 40, output
// position}), one wave per group: the lanes' word counts and records staged in LDS, then
// word by word (lanes in order, 8 words each), the wave copying each word's tokens
// (coalesced, 2 x 64 loads in flight). Capacity: a listed group holds > 1024 tokens or a
// lane's 8 words > 64, so there are fewer than tokens / 64 + 1 <= bytes / 64 + 1 of them
// (2 u64 each in the dead deferred list, bytes / 9 + 64 u64).
__global__ __launch_bounds__(256) void k_compact_long(uint32_t ch_log2, Scratch S,
                                                      const uint32_t* __restrict__ chunk_words,
                                                      const uint64_t* __restrict__ lg_list,
                                                      const uint32_t* __restrict__ lg_cnt, uint32_t* __restrict__ ids,
                                                      uint64_t* __restrict__ offs, int mid) {
    __shared__ uint32_t tmp_all[4][16 * WAVE];
    const int lane = lane_id();
    uint32_t* tmp = tmp_all[threadIdx.x >> 6];
    const uint32_t n = *lg_cnt;
    for (uint32_t i = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; i < n; i += (gridDim.x * blockDim.x) >> 6) {
        const uint64_t e = lg_list[2 * i];
        const uint64_t out = lg_list[2 * i + 1];
        const uint64_t c = e & ((1ull << 40) - 1);
        const uint32_t g0 = (uint32_t)(e >> 40);
        const uint64_t cs = c << ch_log2;
        const uint32_t W = chunk_words[c];
        const uint32_t* tsrc = S.tok() + cs;
        const uint32_t* dsrc = S.dtok() + S.dbase(cs);
        const uint32_t w0 = g0 + 8u * (uint32_t)lane;
        const uint32_t wi = w0 < W ? w0 : 0u;
        const uint4 sa = *(const uint4*)(S.wslot() + cs + wi);
        const uint4 sb = *(const uint4*)(S.wslot() + cs + wi + 4);
        uint32_t cc[8], kd;
        const uint32_t sl[8] = {sa.x, sa.y, sa.z, sa.w, sb.x, sb.y, sb.z, sb.w};
        const uint32_t s = rec_counts<true>(S, cs, w0, W, sl, cc, kd);
        uint64_t lanes = __ballot(s != 0u);
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            tmp[16 * lane + 2 * j] = cc[j];
            tmp[16 * lane + 2 * j + 1] = sl[j];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        uint64_t oo = out;  // words in order: lane by lane, 8 per lane
        while (lanes) {
            const int ln = __ffsll((long long)lanes) - 1;
            lanes &= lanes - 1ull;
            for (int j = 0; j < 8; ++j) {
                const uint32_t n = rfl(tmp[16 * ln + 2 * j]);
                const uint32_t r = rfl(tmp[16 * ln + 2 * j + 1]);
                if (n == 0u) continue;
                if (!(r & REC_MULTI)) {
                    if (lane == 0) emit_token_x(S, cs, r, 0u, ids, offs, oo, mid != 0);
                } else if ((r & REC_SEG) == REC_SEG) {  // k_seg_emit writes its tokens at oo
                    if (lane == 0) S.offs()[cs + (r & REC_OFF)] = oo;
                } else if (r & REC_WIDE) {
                    const uint64_t src = cs + (r & REC_OFF);
                    for (uint32_t k0 = 0; k0 < n; k0 += 2 * WAVE) {
                        uint32_t iv[2];
                        uint64_t ov[2];
#pragma unroll
                        for (int u = 0; u < 2; ++u) {
                            const uint32_t k = min(k0 + (uint32_t)(u * WAVE + lane), n - 1u);
                            iv[u] = S.ids()[src + k];
                            ov[u] = S.offs()[src + k];
                        }
#pragma unroll
                        for (int u = 0; u < 2; ++u) {
                            const uint32_t k = k0 + (uint32_t)(u * WAVE + lane);
                            if (k < n) { ids[oo + k] = iv[u]; offs[oo + k] = ov[u]; }
                        }
                    }
                } else {
                    const uint32_t* src = ((r & REC_DENSE) ? dsrc : tsrc) + (r & REC_OFF);
                    for (uint32_t k0 = 0; k0 < n; k0 += 2 * WAVE) {
                        uint32_t xv[2];
#pragma unroll
                        for (int u = 0; u < 2; ++u) xv[u] = src[min(k0 + (uint32_t)(u * WAVE + lane), n - 1u)];
#pragma unroll
                        for (int u = 0; u < 2; ++u) {
                            const uint32_t k = k0 + (uint32_t)(u * WAVE + lane);
                            if (k < n) emit_token_x(S, cs, 0x80000000u, xv[u], ids, offs, oo + k, mid != 0);
                        }
                    }
                }
                oo += n;
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// ---------------------------------------------------------------------------
// sub-batches: when the workspace cannot hold one pass over the whole batch, the docs are
// cut into doc-aligned sub-batches that each fit it. Every sub-batch is encoded as a batch
// of its own on rebased offsets (bytes from a 512-B aligned base P, so chunks and scan
// steps keep their alignment); its outputs go straight to their final place: row_ptr at
// its first doc, ids / offsets at the token base left by the previous sub-batch (a device
// value: no host round trip between sub-batches).
// ---------------------------------------------------------------------------
constexpr uint32_t SPLIT_MAX = 4096;  // sub-batches found per k_split launch

// Greedy doc-aligned cuts from doc d_start: each sub-batch holds at most cap_d docs and
// cap_b bytes counted from its aligned base. Entry j = {first doc, base P, end byte};
// entry k (k = the count) = {next first doc}. One thread (a handful of binary searches).
__global__ void k_split(const uint64_t* __restrict__ doc_off, uint64_t n_docs, uint64_t d_start, uint64_t cap_b,
                        uint64_t cap_d, uint64_t* __restrict__ splits, unsigned long long* __restrict__ hdr) {
    if (threadIdx.x != 0) return;
    uint64_t d0 = d_start;
    uint32_t k = 0, bad = 0;
    while (d0 < n_docs && k < SPLIT_MAX) {
        const uint64_t P = doc_off[d0] & ~511ull;
        uint64_t lo = d0, hi = min(n_docs, d0 + cap_d);  // doc_off[lo] - P <= cap_b holds for lo = d0
        while (lo < hi) {
            const uint64_t mid = lo + (hi - lo + 1) / 2;
            if (doc_off[mid] - P <= cap_b) lo = mid;
            else hi = mid - 1;
        }
        if (lo == d0) { bad = 1; break; }  // doc d0 alone is larger than a sub-batch
        splits[3 * k] = d0;
        splits[3 * k + 1] = P;
        splits[3 * k + 2] = doc_off[lo];
        ++k;
        d0 = lo;
    }
    splits[3 * k] = d0;
    hdr[HDR_SPLITS] = k;
    hdr[HDR_SPLITS + 1] = bad;
}

__global__ __launch_bounds__(256) void k_rebase(const uint64_t* __restrict__ doc_off, uint64_t n, uint64_t P,
                                                uint64_t* __restrict__ out) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        out[i] = doc_off[i] - P;
}

// ---------------------------------------------------------------------------
// host-side launch
// ---------------------------------------------------------------------------
static inline uint64_t align_up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }

constexpr uint32_t CH_MIN_LOG2 = 9;   // 512 B (half a scan step: the rest of the step starts no word)
#ifndef TKZ_CH_MAX_LOG2
#define TKZ_CH_MAX_LOG2 13
#endif
constexpr uint32_t CH_MAX_LOG2 = TKZ_CH_MAX_LOG2;  // 8 KiB
constexpr uint64_t POS_LIMIT = 1ull << POS_BITS;   // byte positions of one pass (queue entries)

struct WsLayout {
    unsigned long long* hdr;  // HDR_* (chunk ticket first)
    Scratch S;
    uint32_t* cfill;          // per-chunk dense-area fill counters (S.cfill())
    uint32_t* ccnt;           // per-chunk token counts (S.ccnt())
    uint64_t* chunk_doc; uint32_t* chunk_words; uint64_t* chunk_base;
    uint32_t* doc_word; uint64_t* partials;
    Deferred D;
    SegWs G;                  // the segmented path's arrays (seg layouts only)
    uint64_t tb, n_chunks;
    uint8_t* end;  // first byte past the layout
};

// deferred-list capacity: words of >= 9 bytes (each followed by a delimiter or a doc
// boundary, hence the +1 per doc)
static uint64_t defer_cap(uint64_t total_bytes, uint64_t n_docs) { return total_bytes / 9 + n_docs + 64; }

// dedup table slots: a power of two >= 2x the list capacity, at most 4M (32 MB)
static uint64_t dedup_slots(uint64_t total_bytes, uint64_t n_docs) {
    uint64_t s = 64;
    while (s < 2 * defer_cap(total_bytes, n_docs) && s < (1ull << 22)) s <<= 1;
    return s;
}

static uint64_t max_chunks(uint64_t total_bytes) { return (total_bytes >> CH_MIN_LOG2) + 2; }

// workspace of one pass over total_bytes / n_docs: the header, scratch 29 B per input byte
// (offs 8, ids 4, prs 4, tok 4, wslot 4, dense token areas 5), per-chunk arrays, 4 B per
// doc boundary, the deferred and long-word lists (about 2.8 B per input byte), the dedup
// table (<= 32 MB), scan partials
static WsLayout layout(void* ws, uint64_t total_bytes, uint64_t n_docs, int seg = 0) {
    WsLayout L;
    L.tb = align_up(total_bytes + 16, 64);
    const uint64_t nc = max_chunks(total_bytes) + 1;
    uint8_t* p = (uint8_t*)ws;
    L.hdr = (unsigned long long*)p;
    p += HDR_N * 8;
    L.S.base = p;  // offs 8, ids 4, prs 4, tok 4, wslot 4 bytes per element, then the dense
                   // token areas (5 B per byte) and the per-chunk fill counters and counts
    L.S.tb = L.tb;
    p += L.tb * 24 + Scratch::dtok_elems(L.tb) * 4 + align_up(2 * Scratch::chunk_cap(L.tb) * 4, 256);
    L.S.chmask = 0;
    L.S.clog2 = 0;
    L.cfill = (uint32_t*)(L.S.base + L.tb * 24 + Scratch::dtok_elems(L.tb) * 4);
    L.ccnt = L.cfill + Scratch::chunk_cap(L.tb);
    L.chunk_doc = (uint64_t*)p; p += align_up(nc * 8, 256);
    L.chunk_words = (uint32_t*)p; p += align_up(nc * 4, 256);
    L.chunk_base = (uint64_t*)p; p += align_up(nc * 8, 256);
    L.doc_word = (uint32_t*)p; p += align_up((n_docs + 1) * 4, 256);
    L.D.cnt = (uint32_t*)(L.hdr + HDR_DEFER);
    L.D.dbg = L.hdr + HDR_DBG;
    L.D.list = (uint64_t*)p;
    p += align_up(defer_cap(total_bytes, n_docs) * 8, 256);
    L.D.olist = (uint64_t*)p;
    p += align_up(defer_cap(total_bytes, n_docs) * 8, 256);
    L.D.own = (uint64_t*)p;
    p += align_up(defer_cap(total_bytes, n_docs) * 8, 256);
    L.D.dd = (unsigned long long*)p;
    L.D.dd_mask = (uint32_t)(dedup_slots(total_bytes, n_docs) - 1);
    p += align_up(dedup_slots(total_bytes, n_docs) * 8, 256);
    L.D.lcnt = (uint32_t*)(L.hdr + HDR_LONG);
    L.D.llist = (uint64_t*)p;  // words of > LONG_WORD bytes: disjoint, so < bytes / (LONG_WORD + 1)
    p += align_up((total_bytes / (LONG_WORD + 1) + 64) * 8, 256);
    L.D.flist = (uint64_t*)p;
    p += align_up((total_bytes / (LONG_WORD + 1) + 64) * 8, 256);
    L.D.fcnt = (uint32_t*)(L.hdr + HDR_SEG);
    L.D.seg_words = L.hdr + HDR_SEGW;
    L.D.long_bytes = L.hdr + HDR_LONGB;
    L.D.scnt = (uint32_t*)p;
    p += align_up(nc * 4, 256);
    // the short-miss lists live in the scratch's offs array (8 B per input byte: chunk c's at
    // offs[c << ch_log2 ..], at most one word per byte): k_encode_blk runs only where nothing
    // writes offs before k_bpe_short has read them (compact or T.mid tokens, no chain merge)
    L.D.slist = (uint64_t*)L.S.base;
    L.partials = (uint64_t*)p;
    const uint64_t nb = (nc + SCAN_CHUNK - 1) / SCAN_CHUNK + 1;
    p += align_up(nb * 8, 256) + 1024;
    L.G = SegWs{};
    if (seg) {  // segments (seg 1): >= 1 kept byte then >= 1 dropped byte; (seg 2) >= 1 byte
        const uint64_t cap_long = total_bytes / (LONG_WORD + 1) + 64;
        SegWs& G = L.G;
        G.cap_seg = (seg >= 2 ? total_bytes : total_bytes / 2) + cap_long + 64;
        // (a list entry per miss or join: up to one per segment, and seg 2 has up to one
        // segment per byte -- a list past its capacity fails its pretoken)
        G.cap_list = (seg >= 2 ? G.cap_seg : G.cap_seg / 2) + 64;
        auto take = [&](uint64_t bytes) { uint8_t* q = p; p += align_up(bytes, 256); return q; };
        G.ctr = (uint32_t*)take(SC_N * 4);
        G.so = (uint32_t*)take(G.cap_seg * 4);
        G.se = (uint32_t*)take(G.cap_seg * 4);
        G.spt = (uint32_t*)take(G.cap_seg * 4);
        G.sg = (uint32_t*)take(G.cap_seg * 4);
        G.sf = (uint32_t*)take(G.cap_seg * 4);
        G.smeta = (uint64_t*)take(G.cap_seg * 8);
        G.spool = (uint32_t*)take(G.cap_seg * 4);
        G.pbase = (uint32_t*)take(cap_long * 4);
        G.pn = (uint32_t*)take(cap_long * 4);
        G.pst = (uint32_t*)take(cap_long * 4);
        G.plen = (uint32_t*)take(cap_long * 4);
        G.list[0] = (uint32_t*)take(G.cap_list * 4);
        G.list[1] = (uint32_t*)take(G.cap_list * 4);
        G.join = (uint32_t*)take(G.cap_list * 4);
    }
    L.end = p;
    L.n_chunks = 0;
    return L;
}

// the bounds a TKZ_SEG_BOUNDS build found exceeded (bits SB_*; 0 in release builds); reset
uint32_t seg_bound_errors() {
#if TKZ_SEG_BOUNDS
    unsigned int v = 0, z = 0;
    if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_seg_err), sizeof v) != hipSuccess) return 0xFFFFFFFFu;
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_seg_err), &z, sizeof z);
    return v;
#else
    return 0;
#endif
}

// byte offset of the debug counters (the workspace header's HDR_DBG words)
size_t debug_counters_offset(uint64_t, uint64_t) { return (size_t)HDR_DBG * 8; }
size_t stats_offset() { return 0; }

size_t workspace_bytes(uint64_t total_bytes, uint64_t n_docs, int seg) {
    const WsLayout L = layout(nullptr, total_bytes, n_docs, seg);
    return (size_t)(L.end - (uint8_t*)nullptr);
}

// sub-batch geometry for a cap of cap_b bytes: docs per sub-batch (cut earlier when docs
// average < 8 B), and the workspace of one such pass plus the rebased offsets and splits
static uint64_t sub_docs(uint64_t cap_b) { return cap_b / 8 + 1024; }
size_t workspace_bytes_sub(uint64_t cap_b, int seg) {
    return workspace_bytes(cap_b, sub_docs(cap_b), seg) + align_up((sub_docs(cap_b) + 1) * 8, 256) +
           align_up((3ull * SPLIT_MAX + 1) * 8, 256);
}
// the largest sub-batch a workspace of ws_bytes supports (0: too small for any)
uint64_t sub_batch_cap(size_t ws_bytes, int seg) {
    uint64_t lo = 0, hi = POS_LIMIT - 1024;
    while (lo < hi) {
        const uint64_t mid = lo + (hi - lo + 1) / 2;
        if (workspace_bytes_sub(mid, seg) <= ws_bytes) lo = mid;
        else hi = mid - 1;
    }
    return lo < 4096 ? 0 : lo;
}

// Launch geometry caches, one slot per device of the calling thread (tkz_encode_batch_gpus
// encodes from one host thread per device): relaxed atomics, so concurrent first calls
// at worst compute the same value twice.
constexpr int MAX_DEVICES = 64;
static int current_device() {
    int dev = 0;
    (void)hipGetDevice(&dev);
    return dev >= 0 && dev < MAX_DEVICES ? dev : 0;
}
static int device_cus(int dev) {
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    return cus > 0 ? cus : 256;
}

template <int MODEL, bool COMPACT>
static int encode_grid() {
    static std::atomic<int> cache[MAX_DEVICES];
    const int dev = current_device();
    int g = cache[dev].load(std::memory_order_relaxed);
    if (g == 0) {
        const int cus = device_cus(dev);
        int per = 8;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_encode<MODEL, COMPACT>, 64, 0) != hipSuccess || per < 1)
            per = 4;
        g = cus * per;
        cache[dev].store(g, std::memory_order_relaxed);
        if (getenv("TKZ_DEBUG"))
            fprintf(stderr, "tkz: k_encode<%d,%d> dev %d: %d CUs x %d blocks/CU, LDS %zu B/block\n", MODEL, (int)COMPACT,
                    dev, cus, per, sizeof(Smem<MODEL == 1 ? Buckets<MODEL>::n + 1 : Buckets<MODEL>::n, MODEL == 1 ? 128 : 1>));
    }
    return g;
}
// grid of k_bpe_long: one-wave blocks, as many as fit (LDS: ~9 KB each)
static int long_grid() {
    static std::atomic<int> cache[MAX_DEVICES];
    const int dev = current_device();
    int g = cache[dev].load(std::memory_order_relaxed);
    if (g == 0) {
        int per = 16;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_bpe_long<true>, 64, 0) != hipSuccess || per < 1)
            per = 8;
        g = device_cus(dev) * per;
        cache[dev].store(g, std::memory_order_relaxed);
        if (getenv("TKZ_DEBUG"))
            fprintf(stderr, "tkz: k_bpe_long dev %d: %d blocks/CU, LDS %zu B/block\n", dev, per, sizeof(LongSmem));
    }
    return g;
}
// grid of the deferred-word kernels: 8 blocks of 256 per CU
static int deferred_grid() {
    static std::atomic<int> cache[MAX_DEVICES];
    const int dev = current_device();
    int g = cache[dev].load(std::memory_order_relaxed);
    if (g == 0) {
        g = device_cus(dev) * 8;
        cache[dev].store(g, std::memory_order_relaxed);
    }
    return g;
}

#ifndef TKZ_DOCS
#define TKZ_DOCS 1  // whole-text BPE pretokenizers: k_encode_docs (0: k_encode's scan)
#endif
// grid of k_bpe_short: its resident blocks (persistent waves over the chunks: a second
// round of blocks would start its chunks late)
template <bool COMPACT>
static int short_grid() {
    static std::atomic<int> cache[MAX_DEVICES];
    const int dev = current_device();
    int g = cache[dev].load(std::memory_order_relaxed);
    if (g == 0) {
        int per = 4;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_bpe_short<COMPACT>, 256, 0) != hipSuccess || per < 1)
            per = 4;
        g = device_cus(dev) * per;
        cache[dev].store(g, std::memory_order_relaxed);
    }
    return g;
}
#ifndef TKZ_BLK
#define TKZ_BLK 1  // splitting pretokenizers: k_encode_blk (0: k_encode's persistent waves)
#endif
// grid of k_encode_blk: its resident blocks (chunks are strided over them)
template <int MODEL, bool COMPACT>
static int blk_grid() {
    static std::atomic<int> cache[MAX_DEVICES];
    const int dev = current_device();
    int g = cache[dev].load(std::memory_order_relaxed);
    if (g == 0) {
        int per = 4;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_encode_blk<MODEL, COMPACT>, EB_T, 0) != hipSuccess ||
            per < 1)
            per = 2;
        g = device_cus(dev) * per;
        cache[dev].store(g, std::memory_order_relaxed);
        if (getenv("TKZ_DEBUG"))
            fprintf(stderr, "tkz: k_encode_blk<%d,%d> dev %d: %d blocks/CU, LDS %zu B/block\n", MODEL, (int)COMPACT, dev,
                    per, sizeof(EbSmem<MODEL == 1 ? Buckets<MODEL>::n + 1 : Buckets<MODEL>::n>));
    }
    return g;
}
template <int MODEL, bool COMPACT>
static hipError_t launch_main(const DevTables& T, const uint8_t* bytes, const uint64_t* doc_off, uint64_t n_docs,
                              uint64_t limit, uint32_t ch_log2, const WsLayout& W, uint32_t* status, hipStream_t st) {
    if (MODEL == 1 && TKZ_DOCS && T.pretok == 0 && (COMPACT || T.mid || !T.memo)) {
        // (a wide table's memo tokens past 2^20: k_encode writes them as wide tokens)
        const uint64_t nthr = max(n_docs, W.n_chunks);
        hipLaunchKernelGGL((k_encode_docs<COMPACT>), dim3((unsigned)((nthr + 255) / 256)), dim3(256), 0, st, T, bytes,
                           doc_off, n_docs, limit, ch_log2, (const uint64_t*)W.chunk_doc, W.hdr, W.S, W.chunk_words,
                           W.doc_word, W.D);
        return hipGetLastError();
    }
    if (TKZ_BLK && T.pretok != 0 && MODEL == 1 && (COMPACT || T.mid) && !T.chain) {
        const uint64_t g = (uint64_t)blk_grid<MODEL, COMPACT>();
        const uint64_t grid = W.n_chunks < g ? W.n_chunks : g;
        if (grid == 0) return hipSuccess;
        hipLaunchKernelGGL((k_encode_blk<MODEL, COMPACT>), dim3((unsigned)grid), dim3(EB_T), 0, st, T, bytes, doc_off,
                           n_docs, limit, ch_log2, (const uint64_t*)W.chunk_doc, W.hdr, W.S, W.chunk_words,
                           W.doc_word, W.D, status);
        if (MODEL == 1) {
            hipLaunchKernelGGL((k_bpe_short<COMPACT>), dim3((unsigned)short_grid<COMPACT>()), dim3(256), 0, st, T, bytes, limit,
                               W.S, W.D, (uint64_t)0, (uint64_t)W.n_chunks, ch_log2);
        }
        return hipGetLastError();
    }
    const uint64_t g = (uint64_t)encode_grid<MODEL, COMPACT>();
    const uint64_t grid = W.n_chunks < g ? W.n_chunks : g;
    if (grid == 0) return hipSuccess;
    hipLaunchKernelGGL((k_encode<MODEL, COMPACT>), dim3((unsigned)grid), dim3(64), 0, st, T, bytes, doc_off, n_docs,
                       limit, ch_log2, (const uint64_t*)W.chunk_doc, W.hdr, W.S, W.chunk_words, W.doc_word,
                       W.D, status);
    return hipGetLastError();
}

// The segmented path on the long-word list, then k_bpe_long on the pretokens it leaves
template <bool COMPACT>
static void launch_segmented(const DevTables& T, const uint8_t* d_bytes, uint64_t limit, const WsLayout& W,
                             hipStream_t st) {
    const int dgrid = deferred_grid();
    const unsigned wg = (unsigned)dgrid * 4;  // one-wave blocks
    hipLaunchKernelGGL(k_seg_init, dim3(wg), dim3(64), 0, st, T, d_bytes, limit, W.S, W.D, W.G);
    hipLaunchKernelGGL(k_seg_init_big, dim3(SEGB_GRID), dim3(64 * SEGI_W), 0, st, T, d_bytes, limit, W.S, W.D, W.G);
    const bool checked = (T.drop_lo | T.drop_hi | T.cut_lo | T.cut_hi) != 0ull;  // cuts that need checks
    if (T.smemo && TKZ_SEG_FIRST && checked)
        hipLaunchKernelGGL(k_seg_first<COMPACT>, dim3(dgrid), dim3(256), seg_over_lds(T), st, T, d_bytes, limit, W.D, W.G);
    for (int it = 0; it < SEG_ITERS; ++it) {
        // (the work left shrinks geometrically: a later iteration is a launch of few blocks,
        // whose waves find an empty list and exit when the pass has converged)
        const unsigned gi = (unsigned)std::max(1, it < SEG_ITERS_FULL ? dgrid : it < 2 * SEG_ITERS_FULL ? dgrid / 4 : dgrid / 16);
        hipLaunchKernelGGL(k_seg_enc<COMPACT>, dim3(gi), dim3(256), 0, st, T, d_bytes, limit, W.S, W.D, W.G, it);
        hipLaunchKernelGGL(k_seg_enc_big<COMPACT>, dim3(gi), dim3(256), 0, st, T, d_bytes, limit, W.S, W.D, W.G,
                           it);
        if (TKZ_SEG_WAVE_LIST)
            hipLaunchKernelGGL(k_seg_enc_wave<COMPACT>, dim3(gi * 4), dim3(64), 0, st, T, d_bytes, limit, W.S, W.D, W.G,
                               it);
        hipLaunchKernelGGL(k_seg_check<COMPACT>, dim3(gi), dim3(256), seg_over_lds(T), st, T, W.S, W.D, W.G, it);
        hipLaunchKernelGGL(k_seg_join, dim3(gi), dim3(256), 0, st, W.D, W.G, it);
    }
#ifdef TKZ_SEG_STATS
    hipLaunchKernelGGL(k_seg_stats, dim3(1), dim3(64), 0, st, W.D, W.G);
#endif
    if (T.pretok == 0)  // (whole-text pretokenizers: the tokens go to the output after the compaction)
    {
        hipLaunchKernelGGL(k_seg_count, dim3(wg), dim3(64), 0, st, W.S, W.D, W.G);
        hipLaunchKernelGGL(k_seg_count_big, dim3(SEGB_GRID), dim3(64 * SEGB_W), 0, st, W.S, W.D, W.G);
    }
    else
        hipLaunchKernelGGL(k_seg_out, dim3(wg), dim3(64), 0, st, T, W.S, W.D, W.G);
    Deferred D2 = W.D;
    D2.llist = W.D.flist;
    D2.lcnt = W.D.fcnt;
    hipLaunchKernelGGL(k_bpe_long<COMPACT>, dim3(long_grid()), dim3(64), 0, st, T, d_bytes, limit, W.S, D2);
}

// One pass: docs doc_off[0..n_docs] (positions into d_bytes, < total_bytes), outputs at
// the token base *base_in (0 when null); the total goes to *base_out when non-null.
static hipError_t encode_pass(const DevTables& T, const uint8_t* d_bytes, const uint64_t* d_doc_off, uint64_t n_docs,
                              uint64_t total_bytes, uint64_t* d_row_ptr, uint32_t* d_ids, uint64_t* d_offs,
                              const WsLayout& W0, uint32_t* d_status, hipStream_t st, KernelTimers* tm,
                              const unsigned long long* base_in, unsigned long long* base_out, int zero_stats) {
    WsLayout W = W0;
    const uint64_t limit = align_up(total_bytes, 16);  // readable end of the input buffer
    // chunk size: >= 4 chunks per resident wave, 512 B .. 8 KiB
    const uint64_t g = (uint64_t)(T.model == 1 ? (T.compact ? encode_grid<1, true>() : encode_grid<1, false>())
                                               : encode_grid<0, false>());
    uint32_t ch_log2 = CH_MIN_LOG2;
    while (ch_log2 < CH_MAX_LOG2 && (total_bytes >> (ch_log2 + 1)) >= 4 * g) ++ch_log2;
    W.n_chunks = (total_bytes >> ch_log2) + 1;  // covers [0, total]
    W.S.chmask = (1ull << ch_log2) - 1;
    W.S.clog2 = ch_log2;
    hipError_t e;
    const uint64_t kb = (n_docs + 1 + 255) / 256;
    if ((e = hipMemsetAsync(W.cfill, 0, (size_t)W.n_chunks * 4, st)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(W.ccnt, 0, (size_t)W.n_chunks * 4, st)) != hipSuccess) return e;
    // (k_bpe_short reads every chunk's short-list count; k_encode_blk writes those of the chunks in [R0, R1))
    if (T.model == 1 && TKZ_BLK && T.pretok != 0 && (T.compact || T.mid) && !T.chain &&
        (e = hipMemsetAsync(W.D.scnt, 0, (size_t)W.n_chunks * 4, st)) != hipSuccess)
        return e;
    hipLaunchKernelGGL(k_chunk_docs, dim3((unsigned)kb), dim3(256), 0, st, d_doc_off, n_docs, ch_log2, W.chunk_doc,
                       W.hdr, zero_stats);
    if (tm && tm->enabled) hipEventRecord(tm->ev[0], st);
    if (T.model == 1) {
        e = T.compact ? launch_main<1, true>(T, d_bytes, d_doc_off, n_docs, limit, ch_log2, W, d_status, st)
                      : launch_main<1, false>(T, d_bytes, d_doc_off, n_docs, limit, ch_log2, W, d_status, st);
    } else {
        e = launch_main<0, false>(T, d_bytes, d_doc_off, n_docs, limit, ch_log2, W, d_status, st);
    }
    if (e != hipSuccess) return e;
    if (tm && tm->enabled) hipEventRecord(tm->ev[1], st);
    if (T.model == 1) {
        const int dgrid = deferred_grid();
        if (T.dedup) {
            if ((e = hipMemsetAsync(W.D.dd, 0, (size_t)(W.D.dd_mask + 1) * 8, st)) != hipSuccess) return e;
#ifndef TKZ_DEDUP_FIRST
#define TKZ_DEDUP_FIRST 16384
#endif
            hipLaunchKernelGGL(k_dedup, dim3(dgrid), dim3(256), 0, st, T, d_bytes, limit, W.D,
                               (uint64_t)TKZ_DEDUP_FIRST, 0);
            hipLaunchKernelGGL(k_dedup, dim3(dgrid), dim3(256), 0, st, T, d_bytes, limit, W.D,
                               (uint64_t)TKZ_DEDUP_FIRST, 1);
        }
        if (T.compact)
            hipLaunchKernelGGL(k_bpe_deferred<true>, dim3(dgrid), dim3(256), 0, st, T, d_bytes, limit, W.S, W.D);
        else
            hipLaunchKernelGGL(k_bpe_deferred<false>, dim3(dgrid), dim3(256), 0, st, T, d_bytes, limit, W.S, W.D);
        // long words: one wavefront each (the grid drains the list; idle blocks exit at once);
        // the segmented path first, k_bpe_long on what it leaves
        if (W.G.ctr) {  // the segmented path, then k_bpe_long on the pretokens it leaves
            if ((e = hipMemsetAsync(W.G.ctr, 0, SC_N * 4, st)) != hipSuccess) return e;
            if (T.compact) launch_segmented<true>(T, d_bytes, limit, W, st);
            else launch_segmented<false>(T, d_bytes, limit, W, st);
        } else if (T.compact)
            hipLaunchKernelGGL(k_bpe_long<true>, dim3(long_grid()), dim3(64), 0, st, T, d_bytes, limit, W.S, W.D);
        else
            hipLaunchKernelGGL(k_bpe_long<false>, dim3(long_grid()), dim3(64), 0, st, T, d_bytes, limit, W.S, W.D);
        if (T.dedup) hipLaunchKernelGGL(k_dedup_copy, dim3(dgrid), dim3(256), 0, st, W.S, W.D);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    if (tm && tm->enabled) hipEventRecord(tm->ev[2], st);
    const unsigned nblk = (unsigned)((W.n_chunks + SCAN_CHUNK - 1) / SCAN_CHUNK);
    hipLaunchKernelGGL(k_scan_partials, dim3(nblk), dim3(SCAN_T), 0, st, (const uint32_t*)W.ccnt, W.n_chunks,
                       W.partials);
    hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(SCAN_T), 0, st, W.partials, (uint64_t)nblk, W.hdr,
                       (int)(T.model == 1 && T.dedup));
    hipLaunchKernelGGL(k_scan_final, dim3(nblk), dim3(SCAN_T), 0, st, (const uint32_t*)W.ccnt, W.n_chunks,
                       (const uint64_t*)W.partials, W.chunk_base, base_in, base_out);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (tm && tm->enabled) hipEventRecord(tm->ev[3], st);
#ifndef TKZ_CGRID
#define TKZ_CGRID 65536  // k_compact blocks cap: one chunk per wave up to 256k chunks (2 GiB)
#endif
    uint64_t kgrid = (W.n_chunks + 3) / 4;
    if (kgrid > TKZ_CGRID) kgrid = TKZ_CGRID;
    const bool segw = T.model == 1 && W.G.ctr && T.pretok == 0;  // (REC_SEG records: launch_segmented)
    if (segw)
        hipLaunchKernelGGL(k_compact<true>, dim3((unsigned)kgrid), dim3(256), 0, st, d_doc_off, n_docs, ch_log2,
                           W.n_chunks, (const uint64_t*)W.chunk_doc, (const uint64_t*)W.chunk_base, W.S,
                           (const uint32_t*)W.chunk_words, (const uint32_t*)W.doc_word, d_row_ptr, d_ids, d_offs,
                           W.D.list, (uint32_t*)(W.hdr + HDR_CLONG), T.mid);
    else
        hipLaunchKernelGGL(k_compact<false>, dim3((unsigned)kgrid), dim3(256), 0, st, d_doc_off, n_docs, ch_log2,
                           W.n_chunks, (const uint64_t*)W.chunk_doc, (const uint64_t*)W.chunk_base, W.S,
                           (const uint32_t*)W.chunk_words, (const uint32_t*)W.doc_word, d_row_ptr, d_ids, d_offs,
                           W.D.list, (uint32_t*)(W.hdr + HDR_CLONG), T.mid);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(k_compact_long, dim3(1024), dim3(256), 0, st, ch_log2, W.S, (const uint32_t*)W.chunk_words,
                       (const uint64_t*)W.D.list, (const uint32_t*)(W.hdr + HDR_CLONG), d_ids, d_offs, T.mid);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (segw)  // the segmented pretokens' tokens, at the positions k_compact_long left
    {
        hipLaunchKernelGGL(k_seg_emit, dim3((unsigned)deferred_grid() * 4), dim3(64), 0, st, T, W.S, W.D, W.G, d_ids,
                           d_offs);
        hipLaunchKernelGGL(k_seg_emit_big, dim3(SEGB_GRID), dim3(64 * SEGE_W), 0, st, T, W.S, W.D, W.G, d_ids, d_offs);
    }
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (tm && tm->enabled) hipEventRecord(tm->ev[4], st);
    return hipSuccess;
}

hipError_t launch_encode(const DevTables& T, const uint8_t* d_bytes, const uint64_t* d_doc_off, uint64_t n_docs,
                         uint64_t total_bytes, uint64_t* d_row_ptr, uint32_t* d_ids, uint64_t* d_offs, void* d_ws,
                         size_t ws_bytes, uint32_t* d_status, hipStream_t st, const TimerSource& timers,
                         EncodeFail* why) {
    if (why) *why = EncodeFail::None;
    if (n_docs == 0) return hipMemsetAsync(d_row_ptr, 0, 8, st);
    // the segmented path when the workspace holds its arrays (sized by tkz_device_workspace_size)
    const int segm = seg_mode(T);
    const int seg1 = segm && workspace_bytes(total_bytes, n_docs, segm) <= ws_bytes ? segm : 0;
    if (total_bytes < POS_LIMIT && workspace_bytes(total_bytes, n_docs, seg1) <= ws_bytes) {  // one pass
        const WsLayout W = layout(d_ws, total_bytes, n_docs, seg1);
        return encode_pass(T, d_bytes, d_doc_off, n_docs, total_bytes, d_row_ptr, d_ids, d_offs, W, d_status, st,
                           timers.next(), nullptr, nullptr, 1);
    }
    int segs = segm;
    uint64_t cap_b = segs ? sub_batch_cap(ws_bytes, segs) : 0;
    if (cap_b == 0) {
        segs = 0;
        cap_b = sub_batch_cap(ws_bytes);
    }
    if (cap_b == 0) {
        if (why) *why = EncodeFail::WorkspaceTooSmall;
        return hipErrorInvalidValue;
    }
    const uint64_t cap_d = sub_docs(cap_b);
    const WsLayout W = layout(d_ws, cap_b, cap_d, segs);
    uint64_t* d_off_sub = (uint64_t*)W.end;
    uint64_t* d_splits = (uint64_t*)(W.end + align_up((cap_d + 1) * 8, 256));
    hipError_t e;
    if ((e = hipMemsetAsync(W.hdr + HDR_BASE, 0, 16, st)) != hipSuccess) return e;
    std::vector<uint64_t> hs(3 * SPLIT_MAX + 1);
    unsigned long long hh[2];
    uint64_t d_start = 0, sub = 0;
    while (d_start < n_docs) {
        hipLaunchKernelGGL(k_split, dim3(1), dim3(64), 0, st, d_doc_off, (uint64_t)n_docs, d_start, cap_b, cap_d,
                           d_splits, W.hdr);
        if ((e = hipMemcpyAsync(hh, W.hdr + HDR_SPLITS, 16, hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
        if ((e = hipMemcpyAsync(hs.data(), d_splits, hs.size() * 8, hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
        if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
        const uint64_t K = hh[0];
        if (hh[1] && K == 0) {
            if (why) *why = EncodeFail::DocTooLarge;
            return hipErrorInvalidValue;
        }
        for (uint64_t j = 0; j < K; ++j, ++sub) {
            const uint64_t d0 = hs[3 * j], P = hs[3 * j + 1], end = hs[3 * j + 2], d1 = hs[3 * (j + 1)];
            const uint64_t n = d1 - d0;
            hipLaunchKernelGGL(k_rebase, dim3((unsigned)std::min<uint64_t>((n + 256) / 256, 4096)), dim3(256), 0, st,
                               d_doc_off + d0, n + 1, P, d_off_sub);
            e = encode_pass(T, d_bytes + P, d_off_sub, n, end - P, d_row_ptr + d0, d_ids, d_offs, W, d_status, st,
                            timers.next(), W.hdr + HDR_BASE + (sub & 1), W.hdr + HDR_BASE + ((sub + 1) & 1),
                            sub == 0);
            if (e != hipSuccess) return e;
        }
        d_start = hs[3 * K];
        if (hh[1]) {  // the cuts stopped at a doc that no sub-batch holds
            if (why) *why = EncodeFail::DocTooLarge;
            return hipErrorInvalidValue;
        }
    }
    return hipSuccess;
}

}  // namespace tkz
