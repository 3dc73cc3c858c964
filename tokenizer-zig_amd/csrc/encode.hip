// MI355X (gfx950) encode kernels: normalizer + pretokenizer scan + BPE / WordPiece
// model + vocab lookup, bit-exact with the reference's Tokenizer.encode
// (jrc2139/tokenizer-zig src/lib.zig:109-160). Integer / indexing work only: no MFMA.
//
// Pipeline for one batch (all on one HIP stream):
//   k_encode  — one wavefront per document (persistent grid, doc-strided):
//               * scan: 8 B/lane coalesced loads (512 B per wave step), ASCII lowercase
//                 (config.zig:364-379), delimiter/punct classification
//                 (config.zig:405-457), word start/end events from lane bit masks +
//                 neighbour-lane shuffles, wave prefix sums -> LDS word ring;
//                 normalized bytes staged in a 1 KiB LDS window.
//               * model: one LANE per word (words are ~6 symbols, far below 64).
//                 Words of <= MAXB bytes keep their symbols in lane-private LDS
//                 columns (conflict-free [k][lane] layout); longer words run the same
//                 algorithm on a global workspace. BPE follows BPE.tokenize
//                 (bpe.zig:173-263) literally, with a per-pair rank cache so each round
//                 re-probes only the pairs a merge touched; WordPiece follows
//                 WordPiece.tokenize (wordpiece.zig:141-222) with incremental
//                 polynomial hashes.
//               * output: wave prefix sum of per-word token counts -> tokens written
//                 to the doc's bound-layout slot of the scratch (tokens <= bytes), count
//                 per doc.
//   k_scan_*  — exclusive scan of per-doc counts -> CSR row_ptr (u64).
//   k_compact — copy each doc's tokens from its scratch slot to the CSR arrays.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "tables.hpp"
#include "encode.hpp"

namespace tkz {

constexpr int WAVE = 64;
constexpr int STEP = 512;   // bytes per wave scan step (8 per lane)
constexpr int WIN = 1024;   // LDS byte window (two steps)
constexpr int WCAP = 640;   // word ring capacity: >= 63 leftover + 1 open + 512 new
constexpr uint32_t DIRTY = 0xFFFFFFFEu;
constexpr int RW = 16;      // register-resident BPE: max symbols per word
#ifndef TKZ_ABLATE
#define TKZ_ABLATE 0
#endif

__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }

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
__device__ __forceinline__ bool is_punct(uint32_t c) {
    return (c >= 33 && c <= 47) || (c >= 58 && c <= 64) || (c >= 91 && c <= 96) || (c >= 123 && c <= 126);
}
__device__ __forceinline__ int wave_incl_scan(int v) {
    const int lane = lane_id();
#pragma unroll
    for (int o = 1; o < WAVE; o <<= 1) {
        int t = __shfl_up(v, o, WAVE);
        if (lane >= o) v += t;
    }
    return v;
}

// ---------------------------------------------------------------------------
// Symbol storage for one word: LDS columns (short words) or global (long words).
// Entry k: id, start, end (word-relative byte offsets), pair cache pr[k] =
// merge value of (sym k, sym k+1) [compact: rank<<16|new_id; wide: rank].
// ---------------------------------------------------------------------------
template <bool COMPACT>
struct LdsSyms {
    uint32_t* a;  // COMPACT: id | start<<16 | end<<24 ; else id
    uint32_t* b;  // pair cache
    uint32_t* c;  // !COMPACT: start | end<<16
    __device__ uint32_t id(int k) const { return COMPACT ? (a[k * WAVE] & 0xFFFFu) : a[k * WAVE]; }
    __device__ uint32_t start(int k) const { return COMPACT ? ((a[k * WAVE] >> 16) & 0xFFu) : (c[k * WAVE] & 0xFFFFu); }
    __device__ uint32_t end(int k) const { return COMPACT ? (a[k * WAVE] >> 24) : (c[k * WAVE] >> 16); }
    __device__ void set(int k, uint32_t id, uint32_t s, uint32_t e) {
        if (COMPACT) a[k * WAVE] = id | (s << 16) | (e << 24);
        else { a[k * WAVE] = id; c[k * WAVE] = s | (e << 16); }
    }
    __device__ void copy(int w, int r) {
        a[w * WAVE] = a[r * WAVE];
        if (!COMPACT) c[w * WAVE] = c[r * WAVE];
    }
    __device__ uint32_t pr(int k) const { return b[k * WAVE]; }
    __device__ void set_pr(int k, uint32_t v) { b[k * WAVE] = v; }
};

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

// Byte readers (normalized bytes, word-relative position)
struct WinReader {
    const uint8_t* win;
    uint32_t base;  // window index of word byte 0
    __device__ uint32_t operator()(uint32_t p) const { return win[(base + p) & (WIN - 1)]; }
};
struct GlbReader {
    const uint8_t* p0;
    int norm;
    __device__ uint32_t operator()(uint32_t p) const { return lower(p0[p], norm); }
};

template <bool COMPACT>
__device__ __forceinline__ uint32_t pair_value(const DevTables& T, uint32_t a, uint32_t b) {
    if (COMPACT) return merge_probe_compact(T.mtab_c, T.m_bits, a, b);
    uint32_t r, n;
    return merge_probe_wide(T.mtab_w, T.m_bits, a, b, r, n) ? r : NONE;
}

// BPE.tokenize (bpe.zig:173-263) for one pretoken of L bytes. Returns #tokens.
template <bool COMPACT, class S, class R>
__device__ uint32_t bpe_word(const DevTables& T, S& sy, const R& rd, uint32_t L) {
    // initial symbols: codepoint slices (Utf8Iterator.nextCodepointSlice, bpe.zig:186-211)
    int n = 0;
    for (uint32_t p = 0; p < L;) {
        const uint32_t b0 = rd(p);
        uint32_t len = seq_len(b0);
        if (p + len > L) len = L - p;  // truncated sequence: clamp (reference: out-of-bounds)
        uint32_t id;
        if (len == 1) {
            id = T.byte_id[b0];
        } else {
            uint32_t packed = b0;
            for (uint32_t j = 1; j < len; ++j) packed |= rd(p + j) << (8 * j);
            id = cp_probe(T.cp_tab, T.cp_bits, packed, len);
        }
        if (id == NONE) id = T.unk_id;  // unk_token if set and in vocab, else skip the char
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
// Register-resident BPE for words of <= W codepoint slices (the common case).
// Same semantics as bpe_word (bpe.zig:173-263) for merge tables without a
// new_id == first merge (T.chain == 0): in a round every occurrence of the best pair
// is a position whose cached pair value equals the round minimum (ranks are unique per
// pair), and left-to-right replacement with re-test == greedy selection inside runs
// of adjacent candidates. All arrays are indexed with compile-time indices (unrolled),
// and all pair probes of a round are issued back to back.
// ---------------------------------------------------------------------------
template <int W, bool COMPACT>
struct RegWord {
    uint32_t sy[W];                   // COMPACT: id | start<<16 | end<<24 ; else id
    uint32_t sp[COMPACT ? 1 : W];     // !COMPACT: start | end<<16
    uint32_t pr[W];                   // cached value of pair (k, k+1)
    int n;

    template <int K> __device__ __forceinline__ uint32_t id() const { return COMPACT ? (sy[K] & 0xFFFFu) : sy[K]; }
    __device__ __forceinline__ uint32_t idv(uint32_t v) const { return COMPACT ? (v & 0xFFFFu) : v; }
};

template <int W, bool COMPACT>
__device__ __forceinline__ void reg_probe(const DevTables& T, RegWord<W, COMPACT>& w, uint32_t mask) {
    if (COMPACT) {
        uint2 s[W - 1];
#pragma unroll
        for (int k = 0; k < W - 1; ++k) {
            if ((mask >> k) & 1u) {
                const uint32_t key = (w.idv(w.sy[k]) << 16) | w.idv(w.sy[k + 1]);
                s[k] = T.mtab_c[merge_slot_compact(key, T.m_bits)];
            }
        }
#pragma unroll
        for (int k = 0; k < W - 1; ++k) {
            if ((mask >> k) & 1u) {
                const uint32_t key = (w.idv(w.sy[k]) << 16) | w.idv(w.sy[k + 1]);
                uint32_t v;
                if (s[k].x == key) v = s[k].y;
                else if (s[k].x == EMPTY32) v = NONE;
                else v = merge_probe_compact(T.mtab_c, T.m_bits, w.idv(w.sy[k]), w.idv(w.sy[k + 1]));
                w.pr[k] = v;
            }
        }
    } else {
        uint4 s[W - 1];
#pragma unroll
        for (int k = 0; k < W - 1; ++k) {
            if ((mask >> k) & 1u) {
                const uint64_t key = ((uint64_t)w.sy[k] << 32) | w.sy[k + 1];
                s[k] = T.mtab_w[merge_slot_wide(key, T.m_bits)];
            }
        }
#pragma unroll
        for (int k = 0; k < W - 1; ++k) {
            if ((mask >> k) & 1u) {
                uint32_t v;
                if (s[k].z == EMPTY32) v = NONE;
                else if (s[k].x == w.sy[k] && s[k].y == w.sy[k + 1]) v = s[k].z;
                else v = pair_value<false>(T, w.sy[k], w.sy[k + 1]);
                w.pr[k] = v;
            }
        }
    }
}

// Returns false if the word has more than W symbols (caller uses the global path).
template <int W, bool COMPACT, class R>
__device__ bool bpe_word_reg(const DevTables& T, RegWord<W, COMPACT>& w, const R& rd, uint32_t L) {
    int n = 0;
    for (uint32_t p = 0; p < L;) {
        const uint32_t b0 = rd(p);
        uint32_t len = seq_len(b0);
        if (p + len > L) len = L - p;
        uint32_t id;
        if (len == 1) {
            id = T.byte_id[b0];
        } else {
            uint32_t packed = b0;
            for (uint32_t j = 1; j < len; ++j) packed |= rd(p + j) << (8 * j);
            id = cp_probe(T.cp_tab, T.cp_bits, packed, len);
        }
        if (id == NONE) id = T.unk_id;
        if (id != NONE) {
            if (n == W) return false;
            const uint32_t v = COMPACT ? (id | (p << 16) | ((p + len) << 24)) : id;
#pragma unroll
            for (int j = 0; j < W; ++j) {
                if (j == n) {
                    w.sy[j] = v;
                    if (!COMPACT) w.sp[j] = p | ((p + len) << 16);
                }
            }
            ++n;
        }
        p += len;
    }
    w.n = n;
#if TKZ_ABLATE == 3
    return true;
#endif
    if (n >= 2) reg_probe<W, COMPACT>(T, w, (1u << (n - 1)) - 1);
#if TKZ_ABLATE == 2
    return true;
#endif
    while (w.n >= 2) {
        const int nn = w.n;
        uint32_t best = NONE;
#pragma unroll
        for (int k = 0; k < W - 1; ++k)
            if (k < nn - 1) best = min(best, w.pr[k]);
        if (best == NONE) break;
        uint32_t X;
        if (COMPACT) {
            X = best & 0xFFFFu;
        } else {
            uint32_t a = 0, b = 0, r;
#pragma unroll
            for (int k = 0; k < W - 1; ++k)
                if (k < nn - 1 && w.pr[k] == best) { a = w.sy[k]; b = w.sy[k + 1]; }
            merge_probe_wide(T.mtab_w, T.m_bits, a, b, r, X);
        }
        uint32_t sel = 0, prev = 0;
#pragma unroll
        for (int k = 0; k < W - 1; ++k) {
            const uint32_t c = (k < nn - 1 && w.pr[k] == best) ? (1u - prev) : 0u;
            sel |= c << k;
            prev = c;
        }
        uint32_t dirty = 0;
        while (sel) {
            const int k = 31 - __clz(sel);
            sel ^= 1u << k;
#pragma unroll
            for (int j = 0; j < W - 1; ++j) {
                if (j == k) {
                    if (COMPACT) w.sy[j] = X | (w.sy[j] & 0x00FF0000u) | (w.sy[j + 1] & 0xFF000000u);
                    else { w.sy[j] = X; w.sp[j] = (w.sp[j] & 0xFFFFu) | (w.sp[j + 1] & 0xFFFF0000u); }
                }
            }
#pragma unroll
            for (int j = 1; j < W - 1; ++j) {
                if (j > k) {
                    w.sy[j] = w.sy[j + 1];
                    w.pr[j] = w.pr[j + 1];
                    if (!COMPACT) w.sp[j] = w.sp[j + 1];
                }
            }
            --w.n;
            const uint32_t lowk = (2u << k) - 1;  // bits 0..k
            dirty = (dirty & lowk) | ((dirty >> 1) & ~lowk);
            dirty |= (1u << k) | (k > 0 ? (1u << (k - 1)) : 0u);
        }
        dirty &= (w.n >= 2) ? ((1u << (w.n - 1)) - 1) : 0u;
        reg_probe<W, COMPACT>(T, w, dirty);
    }
    return true;
}

// WordPiece vocab probe for key = [prefix if start>0] ++ word[start:e), hash `h`.
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

// WordPiece.tokenize (wordpiece.zig:141-222) for a pretoken of L <= max_chars bytes.
// Returns #tokens, or NONE when the word is "bad" (caller emits the single UNK).
template <class S, class R>
__device__ uint32_t wordpiece_word(const DevTables& T, S& sy, const R& rd, uint32_t L) {
    uint32_t start = 0;
    int n = 0;
    while (start < L) {
        const bool pre = start > 0;
        uint32_t lim = T.max_key;
        if (pre) {
            lim = T.max_key > T.plen ? T.max_key - T.plen : 0;
            const uint32_t buf_lim = T.plen <= 512 ? 512 - T.plen : 0;  // substr_buf: [512]u8
            if (buf_lim < lim) lim = buf_lim;
        }
        uint32_t emax = L - start < lim ? L : start + lim;
        // G(start, emax) and HP^(emax-start)
        uint64_t g = 0, pw = 1;
        for (uint32_t j = start; j < emax; ++j) { g += (uint64_t)(rd(j) + 1) * pw; pw *= HP; }
        uint32_t found = NONE, e = emax;
        for (; e > start; --e) {
            const uint64_t gk = pre ? T.g_prefix + T.p_plen * g : g;
            const uint32_t klen = (pre ? T.plen : 0) + (e - start);
            const uint32_t id = wp_probe(T, rd, wp_final(gk, klen), klen, pre, start);
            if (id != NONE) { found = id; break; }
            pw *= T.hp_inv;                              // HP^(e-1-start)
            g -= (uint64_t)(rd(e - 1) + 1) * pw;         // drop byte e-1
        }
        if (found == NONE) return NONE;
        sy.set(n++, found, start, e);
        start = e;
    }
    return (uint32_t)n;
}

// ---------------------------------------------------------------------------
// k_encode
// ---------------------------------------------------------------------------
template <int MODEL, bool COMPACT, int MAXB>
struct Smem {
    static constexpr int NARR = (MODEL == 1) ? 0 : 2;
    uint64_t win[WIN / 8];
    uint32_t wst[WCAP];
    uint32_t wen[WCAP];
    uint32_t byte_id[256];
    uint32_t slot[NARR > 0 ? NARR : 1][NARR > 0 ? MAXB : 1][WAVE];
};

template <int MODEL, bool COMPACT, int MAXB>
__global__ __launch_bounds__(64) void k_encode(DevTables T, const uint8_t* __restrict__ bytes,
                                               const uint64_t* __restrict__ doc_off, uint64_t n_docs,
                                               uint32_t* __restrict__ s_ids, uint64_t* __restrict__ s_offs,
                                               uint32_t* __restrict__ s_prs, uint32_t* __restrict__ counts,
                                               uint32_t* __restrict__ status) {
    __shared__ Smem<MODEL, COMPACT, MAXB> sm;
    const int lane = lane_id();
    if (MODEL == 1) {
        for (int i = lane; i < 256; i += WAVE) sm.byte_id[i] = T.byte_id[i];
        T.byte_id = sm.byte_id;
    }
    __syncthreads();
    const uint8_t* win = (const uint8_t*)sm.win;

    for (uint64_t d = blockIdx.x; d < n_docs; d += gridDim.x) {
        const uint64_t db = doc_off[d], de = doc_off[d + 1];
        const uint64_t a0 = db & ~(uint64_t)7;
        const uint32_t mis = (uint32_t)(db - a0);
        uint32_t n_st = 0, n_en = 0, head = 0, run = 0;
        uint32_t carry_s = 1, carry_p = 0;  // previous byte: split?, punct?

        for (uint64_t sb = a0; sb < de; sb += STEP) {
            const uint64_t base = sb + 8ull * lane;
            uint64_t v = 0;
            if (base < de && base + 8 > db) v = *(const uint64_t*)(bytes + base);
            uint32_t S = 0, P = 0;
            uint64_t nv = 0;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const uint64_t pos = base + j;
                const bool valid = pos >= db && pos < de;
                const uint32_t c = lower((uint32_t)(v >> (8 * j)) & 0xFFu, T.norm);
                nv |= (uint64_t)c << (8 * j);
                bool split = !valid, punct = false;
                if (valid) {
                    if (T.pretok == 1) split = (c == ' ' || c == '\t' || c == '\n' || c == '\r');
                    else if (T.pretok == 2) {
                        punct = is_punct(c);
                        split = punct || c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == 0x0B || c == 0x0C;
                    }
                }
                S |= (uint32_t)split << j;
                P |= (uint32_t)punct << j;
            }
            sm.win[((sb - a0 + 8ull * lane) & (WIN - 1)) >> 3] = nv;
            // previous byte state for bit 0
            const uint32_t up_s = (uint32_t)__shfl_up((int)((S >> 7) & 1), 1, WAVE);
            const uint32_t up_p = (uint32_t)__shfl_up((int)((P >> 7) & 1), 1, WAVE);
            const uint32_t ps = lane == 0 ? carry_s : up_s;
            const uint32_t pp = lane == 0 ? carry_p : up_p;
            const uint32_t Sprev = ((S << 1) | ps) & 0xFFu;
            const uint32_t Pprev = ((P << 1) | pp) & 0xFFu;
            const uint32_t starts = ((~S & Sprev) | P) & 0xFFu;        // run start or punct byte
            const uint32_t ends = ((S & ~Sprev) | Pprev) & 0xFFu;      // run end or byte after punct
            carry_s = (uint32_t)__shfl((int)((S >> 7) & 1), WAVE - 1, WAVE);
            carry_p = (uint32_t)__shfl((int)((P >> 7) & 1), WAVE - 1, WAVE);
            const int cs = __popc(starts), ce = __popc(ends);
            const int is = wave_incl_scan(cs), ie = wave_incl_scan(ce);
            {
                uint32_t m = starts, k = n_st + (uint32_t)(is - cs);
                while (m) { const int j = __ffs(m) - 1; m &= m - 1; sm.wst[k++ % WCAP] = (uint32_t)(base + j - db); }
                m = ends; k = n_en + (uint32_t)(ie - ce);
                while (m) { const int j = __ffs(m) - 1; m &= m - 1; sm.wen[k++ % WCAP] = (uint32_t)(base + j - db); }
            }
            n_st += (uint32_t)__shfl(is, WAVE - 1, WAVE);
            n_en += (uint32_t)__shfl(ie, WAVE - 1, WAVE);
            const bool last_step = sb + STEP >= de;
            if (last_step && (carry_s == 0 || carry_p) && n_en < n_st) {
                // the doc's last byte is inside a word and de is exactly at this step's end
                if (lane == 0) sm.wen[n_en % WCAP] = (uint32_t)(de - db);
                ++n_en;
            }
            __syncthreads();

            // ---- model over every complete word, 64 words per round ----
            while (head < n_en) {
                const uint32_t batch = min(n_en - head, (uint32_t)WAVE);
                const bool active = (uint32_t)lane < batch;
                uint32_t wrel = 0, L = 0, cnt = 0;
                bool lng = false;
                if (active) {
                    wrel = sm.wst[(head + lane) % WCAP];
                    L = sm.wen[(head + lane) % WCAP] - wrel;
                }
                RegWord<RW, COMPACT> rw;
                rw.n = 0;
                if (MODEL == 1) {
                    bool fits = false;
#if TKZ_ABLATE == 1
                    if (false)
#else
                    if (active && !T.chain)
#endif
                        fits = bpe_word_reg<RW, COMPACT>(T, rw, WinReader{win, wrel + mis}, L);
#if TKZ_ABLATE == 1
                    fits = true;
#endif
                    lng = active && !fits;
                    if (lng) {
                        const uint64_t o = db + wrel;
                        GlbSyms sy{s_ids + o, s_offs + o, s_prs + o};
                        cnt = bpe_word<COMPACT>(T, sy, GlbReader{bytes + db + wrel, T.norm}, L);
                    } else if (active) {
                        cnt = (uint32_t)rw.n;
                    }
                } else {
                    lng = active && L > MAXB && L <= T.max_chars;
                    LdsSyms<false> sy{&sm.slot[0][0][lane], nullptr, &sm.slot[1][0][lane]};
                    if (active && !lng) {
                        if (L > T.max_chars) cnt = NONE;
                        else cnt = wordpiece_word(T, sy, WinReader{win, wrel + mis}, L);
                    } else if (lng) {
                        const uint64_t o = db + wrel;
                        GlbSyms gs{s_ids + o, s_offs + o, s_prs + o};
                        cnt = wordpiece_word(T, gs, GlbReader{bytes + db + wrel, T.norm}, L);
                    }
                    if (active && cnt == NONE) {  // too long or bad -> one UNK (0, L)
                        if (T.wp_unk == NONE) *status = 9u;  // TKZ_ERR_MISSING_UNK_TOKEN
                        if (lng) {
                            s_ids[db + wrel] = T.wp_unk;
                            s_offs[db + wrel] = (uint64_t)L << 32;
                        } else {
                            sy.set(0, T.wp_unk, 0, L);
                        }
                        cnt = 1;
                    }
                }
                const int inc = wave_incl_scan((int)cnt);
                const uint32_t exc = (uint32_t)inc - cnt;
                const uint32_t tot = (uint32_t)__shfl(inc, WAVE - 1, WAVE);
                // long words: move their tokens from the word's workspace to the final slot,
                // one word at a time in word order (dst <= src always).
                uint64_t lm = __ballot(lng);
                if (lm) {
                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
                    while (lm) {
                        const int l = __builtin_ctzll(lm);
                        lm &= lm - 1;
                        const uint64_t src = db + __shfl(wrel, l, WAVE);
                        const uint64_t dst = db + run + __shfl(exc, l, WAVE);
                        const uint32_t c = (uint32_t)__shfl((int)cnt, l, WAVE);
                        if (src != dst) {
                            for (uint32_t i0 = 0; i0 < c; i0 += WAVE) {
                                const uint32_t i = i0 + lane;
                                uint32_t id = 0;
                                uint64_t of = 0;
                                if (i < c) { id = s_ids[src + i]; of = s_offs[src + i]; }
                                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
                                if (i < c) { s_ids[dst + i] = id; s_offs[dst + i] = of; }
                                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
                            }
                        }
                    }
                }
                if (active && !lng) {
                    const uint64_t o = db + run + exc;
                    if (MODEL == 1) {
#pragma unroll
                        for (int k = 0; k < RW; ++k) {
                            if (k < (int)cnt) {
                                const uint32_t v = rw.sy[k];
                                uint32_t id, st, en;
                                if (COMPACT) { id = v & 0xFFFFu; st = (v >> 16) & 0xFFu; en = v >> 24; }
                                else { id = v; st = rw.sp[k] & 0xFFFFu; en = rw.sp[k] >> 16; }
                                s_ids[o + k] = id;
                                s_offs[o + k] = (uint64_t)st | ((uint64_t)en << 32);
                            }
                        }
                    } else {
                        LdsSyms<false> sy{&sm.slot[0][0][lane], nullptr, &sm.slot[1][0][lane]};
                        for (uint32_t k = 0; k < cnt; ++k) {
                            s_ids[o + k] = sy.id(k);
                            s_offs[o + k] = (uint64_t)sy.start(k) | ((uint64_t)sy.end(k) << 32);
                        }
                    }
                }
                run += tot;
                head += batch;
            }
            __syncthreads();
        }
        if (lane == 0) counts[d] = run;
    }
}

// ---------------------------------------------------------------------------
// scan of per-doc counts -> row_ptr (u64, n+1)
// ---------------------------------------------------------------------------
constexpr int SCAN_T = 256;
constexpr int SCAN_IT = 16;
constexpr int SCAN_CHUNK = SCAN_T * SCAN_IT;

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

__global__ __launch_bounds__(SCAN_T) void k_scan_top(uint64_t* __restrict__ partials, uint64_t nb) {
    __shared__ uint64_t tmp[SCAN_T / 64];
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

__global__ __launch_bounds__(SCAN_T) void k_scan_final(const uint32_t* __restrict__ counts, uint64_t n,
                                                       const uint64_t* __restrict__ partials,
                                                       uint64_t* __restrict__ row_ptr) {
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
    uint64_t off = partials[blockIdx.x] + block_excl_scan(s, tmp, total);
#pragma unroll
    for (int i = 0; i < SCAN_IT; ++i) {
        const uint64_t k = base + i;
        if (k < n) row_ptr[k] = off;
        off += c[i];
        if (k + 1 == n) row_ptr[n] = off;
    }
}

// ---------------------------------------------------------------------------
// compaction: scratch (bound layout at doc byte offsets) -> CSR
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_compact(const uint64_t* __restrict__ doc_off, uint64_t n_docs,
                                                 const uint32_t* __restrict__ counts,
                                                 const uint64_t* __restrict__ row_ptr,
                                                 const uint32_t* __restrict__ s_ids, const uint64_t* __restrict__ s_offs,
                                                 uint32_t* __restrict__ ids, uint64_t* __restrict__ offs) {
    const int lane = lane_id();
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t d = wave; d < n_docs; d += nw) {
        const uint64_t src = doc_off[d], dst = row_ptr[d];
        const uint32_t c = counts[d];
        for (uint32_t i = lane; i < c; i += WAVE) {
            ids[dst + i] = s_ids[src + i];
            offs[dst + i] = s_offs[src + i];
        }
    }
}

// ---------------------------------------------------------------------------
// host-side launch
// ---------------------------------------------------------------------------
static inline uint64_t align_up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }

size_t workspace_bytes(uint64_t total_bytes, uint64_t n_docs) {
    const uint64_t tb = align_up(total_bytes + 16, 64);
    const uint64_t nb = (n_docs + SCAN_CHUNK - 1) / SCAN_CHUNK + 1;
    return (size_t)(tb * 4 + tb * 8 + tb * 4 + align_up(n_docs * 4 + 4, 256) + align_up(nb * 8, 256) + 1024);
}

template <int MODEL, bool COMPACT, int MAXB>
static hipError_t launch_main(const DevTables& T, const uint8_t* bytes, const uint64_t* doc_off, uint64_t n_docs,
                              uint32_t* s_ids, uint64_t* s_offs, uint32_t* s_prs, uint32_t* counts,
                              uint32_t* status, hipStream_t st) {
    static int grid_cache = 0;
    if (grid_cache == 0) {
        int dev = 0, cus = 256, per = 8;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_encode<MODEL, COMPACT, MAXB>, 64, 0) != hipSuccess ||
            per < 1)
            per = 4;
        grid_cache = cus * per;
    }
    const uint64_t grid = n_docs < (uint64_t)grid_cache ? n_docs : (uint64_t)grid_cache;
    if (grid == 0) return hipSuccess;
    hipLaunchKernelGGL((k_encode<MODEL, COMPACT, MAXB>), dim3((unsigned)grid), dim3(64), 0, st, T, bytes, doc_off,
                       n_docs, s_ids, s_offs, s_prs, counts, status);
    return hipGetLastError();
}

hipError_t launch_encode(const DevTables& T, const uint8_t* d_bytes, const uint64_t* d_doc_off, uint64_t n_docs,
                         uint64_t total_bytes, uint64_t* d_row_ptr, uint32_t* d_ids, uint64_t* d_offs, void* d_ws,
                         uint32_t* d_status, hipStream_t st, KernelTimers* tm) {
    const uint64_t tb = align_up(total_bytes + 16, 64);
    const uint64_t nb = (n_docs + SCAN_CHUNK - 1) / SCAN_CHUNK + 1;
    uint8_t* p = (uint8_t*)d_ws;
    uint32_t* s_ids = (uint32_t*)p; p += tb * 4;
    uint64_t* s_offs = (uint64_t*)p; p += tb * 8;
    uint32_t* s_prs = (uint32_t*)p; p += tb * 4;
    uint32_t* counts = (uint32_t*)p; p += align_up(n_docs * 4 + 4, 256);
    uint64_t* partials = (uint64_t*)p;

    if (n_docs == 0) {
        return hipMemsetAsync(d_row_ptr, 0, 8, st);
    }
    if (tm && tm->enabled) hipEventRecord(tm->ev[0], st);
    hipError_t e;
    if (T.model == 1) {
        e = T.compact ? launch_main<1, true, TKZ_MAXB>(T, d_bytes, d_doc_off, n_docs, s_ids, s_offs, s_prs, counts, d_status, st)
                      : launch_main<1, false, TKZ_MAXB>(T, d_bytes, d_doc_off, n_docs, s_ids, s_offs, s_prs, counts, d_status, st);
    } else {
        e = launch_main<0, false, TKZ_MAXB>(T, d_bytes, d_doc_off, n_docs, s_ids, s_offs, s_prs, counts, d_status, st);
    }
    if (e != hipSuccess) return e;
    if (tm && tm->enabled) hipEventRecord(tm->ev[1], st);
    const unsigned nblk = (unsigned)((n_docs + SCAN_CHUNK - 1) / SCAN_CHUNK);
    hipLaunchKernelGGL(k_scan_partials, dim3(nblk), dim3(SCAN_T), 0, st, counts, n_docs, partials);
    hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(SCAN_T), 0, st, partials, (uint64_t)nblk);
    hipLaunchKernelGGL(k_scan_final, dim3(nblk), dim3(SCAN_T), 0, st, counts, n_docs, partials, d_row_ptr);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (tm && tm->enabled) hipEventRecord(tm->ev[2], st);
    uint64_t cgrid = (n_docs + 3) / 4;
    if (cgrid > 8192) cgrid = 8192;
    hipLaunchKernelGGL(k_compact, dim3((unsigned)cgrid), dim3(256), 0, st, d_doc_off, n_docs, counts, d_row_ptr,
                       s_ids, s_offs, d_ids, d_offs);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (tm && tm->enabled) hipEventRecord(tm->ev[3], st);
    return hipSuccess;
}

}  // namespace tkz
