// GPU-resident lookup tables shared by the host builder (tokenizer.cpp) and the HIP
// kernels (encode.hip). Every table is an open-addressed, linear-probed power-of-two
// array built once on the host (Tokenizer.fromJson time) and uploaded once; they are
// a few MB at most and stay L2 / Infinity-Cache resident while the batch streams.
//
//   merge table (BPE, bpe.zig:40 merges: u64 pair -> PairVal{rank,new_id})
//     compact: 8-B slot {key = a<<16|b, val = rank<<16|new_id}  (ids, ranks < 0xFFFF),
//              two-slot buckets, cuckoo (two candidate buckets per key)
//     wide:   16-B slot {key lo, key hi, rank, new_id}
//   char table (BPE initial symbols, bpe.zig:186-205 vocab.get(codepoint bytes))
//     1-byte slices: direct 256-entry id array; 2..4-byte slices: 16-B slot
//     {packed bytes, len, id, 0}
//   string table (WordPiece, wordpiece.zig:187 vocab.get(prefix ++ bytes))
//     16-B slot {h64 lo, h64 hi, id, pool offset}; pool entry = u32 len + bytes,
//     every hit is verified byte-for-byte against the pool.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#if defined(__HIPCC__)
#define TKZ_HD __host__ __device__ __forceinline__
#else
#define TKZ_HD inline
#endif

namespace tkz {

constexpr uint32_t NONE = 0xFFFFFFFFu;
constexpr uint32_t EMPTY32 = 0xFFFFFFFFu;

// polynomial string hash over (byte + 1), mod 2^64 (WordPiece keys)
constexpr uint64_t HP = 0x100000001B3ull;

TKZ_HD uint64_t fmix64(uint64_t k) {
    k ^= k >> 33; k *= 0xff51afd7ed558ccdull; k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ull; k ^= k >> 33;
    return k;
}
TKZ_HD uint32_t fmix32(uint32_t h) {
    h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
    return h;
}
TKZ_HD uint64_t wp_final(uint64_t g, uint32_t klen) { return fmix64(g ^ ((uint64_t)klen * 0x9E3779B97F4A7C15ull)); }

// -------- merge table ---------------------------------------------------------
TKZ_HD uint32_t merge_slot_compact(uint32_t key, uint32_t bits) { return (key * 0x9E3779B1u) >> (32 - bits); }
TKZ_HD uint32_t merge_slot_wide(uint64_t key, uint32_t bits) { return (uint32_t)(fmix64(key) >> (64 - bits)); }

// Compact merge table: bucketized cuckoo hash. Bucket = 16 B = two 8-B slots
// {a<<16|b, rank<<16|new_id}; every key sits in one of its two buckets (2^bits buckets,
// load <= 1/2), so a lookup is exactly two 16-B loads issued together, never a chain.
TKZ_HD void merge_buckets_compact(uint32_t key, uint32_t bits, uint32_t& b1, uint32_t& b2) {
    b1 = (key * 0x9E3779B1u) >> (32 - bits);
    b2 = fmix32(key ^ 0x5bd1e995u) >> (32 - bits);
    if (b2 == b1) b2 = b1 ^ 1u;
}
TKZ_HD uint32_t merge_match_compact(const uint4& p, const uint4& q, uint32_t key) {
    uint32_t v = NONE;
    v = q.z == key ? q.w : v;
    v = q.x == key ? q.y : v;
    v = p.z == key ? p.w : v;
    v = p.x == key ? p.y : v;
    return v;
}
// Returns rank<<16|new_id, or NONE.
TKZ_HD uint32_t merge_probe_compact(const uint2* tab, uint32_t bits, uint32_t a, uint32_t b) {
    const uint32_t key = (a << 16) | b;
    uint32_t b1, b2;
    merge_buckets_compact(key, bits, b1, b2);
    const uint4 p = *(const uint4*)(tab + 2 * b1), q = *(const uint4*)(tab + 2 * b2);
    return merge_match_compact(p, q, key);
}

// Mid merge table (wide tables with ids < 2^20 - 1 and ranks < 2^24 - 1: the segmented
// path of 100k+-id vocabs): a bucketized cuckoo table like the compact one -- 16-B buckets
// of two 8-B slots, two candidate buckets, a lookup = two 16-B loads issued together -- with
// slot {a | b << 20 (low 32 bits), b >> 12 | rank << 8}; the new id comes from the rank ->
// new_id table. 8 B per slot instead of the wide table's 16 B at load 1/4: 106k merges in
// 2 MB (L2-resident) instead of 8 MB. An empty slot is all ones (a < 2^20 - 1: no key is).
TKZ_HD void merge_buckets_mid(uint32_t a, uint32_t b, uint32_t bits, uint32_t& b1, uint32_t& b2) {
    const uint32_t h = a * 0x85EBCA77u + b * 0x9E3779B1u;
    b1 = h >> (32 - bits);
    b2 = fmix32(h ^ 0x5bd1e995u) >> (32 - bits);
    if (b2 == b1) b2 = b1 ^ 1u;
}
TKZ_HD uint2 mid_slot(uint32_t a, uint32_t b, uint32_t rank) { return uint2{a | (b << 20), (b >> 12) | (rank << 8)}; }
// rank, or NONE
TKZ_HD uint32_t merge_match_mid(const uint4& p, const uint4& q, uint32_t a, uint32_t b) {
    const uint32_t lo = a | (b << 20), hb = b >> 12;
    uint32_t v = NONE;
    v = q.z == lo && (q.w & 0xFFu) == hb ? q.w >> 8 : v;
    v = q.x == lo && (q.y & 0xFFu) == hb ? q.y >> 8 : v;
    v = p.z == lo && (p.w & 0xFFu) == hb ? p.w >> 8 : v;
    v = p.x == lo && (p.y & 0xFFu) == hb ? p.y >> 8 : v;
    return v;
}
TKZ_HD uint32_t merge_probe_mid(const uint2* tab, uint32_t bits, uint32_t a, uint32_t b) {
    uint32_t b1, b2;
    merge_buckets_mid(a, b, bits, b1, b2);
    const uint4 p = *(const uint4*)(tab + 2 * b1), q = *(const uint4*)(tab + 2 * b2);
    return merge_match_mid(p, q, a, b);
}

// Returns true + (rank, new_id) if present.
TKZ_HD bool merge_probe_wide(const uint4* tab, uint32_t bits, uint32_t a, uint32_t b, uint32_t& rank, uint32_t& nid) {
    const uint64_t key = ((uint64_t)a << 32) | b;
    const uint32_t mask = (1u << bits) - 1;
    uint32_t h = merge_slot_wide(key, bits);
    while (true) {
        uint4 s = tab[h];
        if (s.z == EMPTY32) return false;  // empty slot: rank field EMPTY
        if (s.x == a && s.y == b) { rank = s.z; nid = s.w; return true; }
        h = (h + 1) & mask;
    }
}

// -------- char table (multi-byte codepoint slices) ----------------------------
TKZ_HD uint32_t cp_slot(uint32_t packed, uint32_t len, uint32_t bits) {
    return fmix32(packed ^ (len * 0x9E3779B9u)) >> (32 - bits);
}
TKZ_HD uint32_t cp_probe(const uint4* tab, uint32_t bits, uint32_t packed, uint32_t len) {
    const uint32_t mask = (1u << bits) - 1;
    uint32_t h = cp_slot(packed, len, bits);
    while (true) {
        uint4 s = tab[h];
        if (s.y == len && s.x == packed) return s.z;
        if (s.y == 0) return NONE;  // len 0 = empty
        h = (h + 1) & mask;
    }
}

// -------- word memo (BPE): vocab key (<= 16 B) -> its BPE tokens ----------------
// 32-B slot = 2 x uint4: {key bytes 0-7, key bytes 8-15} and {len | ntok<<8, tok0, tok1,
// tok2} with tok = id | start<<16 | end<<24 (compact ids). Filled at upload time from
// the GPU encode of every short vocab key; info == 0 marks an empty slot.
// One 32-bit hash for every short key (<= 16 bytes, zero past len): both memo tables
// and the WordPiece short-key table take its top bits, so a wave probing keys of mixed
// lengths computes it once (two hash functions ran as two divergent paths).
TKZ_HD uint32_t short_key_hash(uint64_t k0, uint64_t k1, uint32_t len) {
    uint32_t h = ((uint32_t)(k0 >> 32) ^ (len << 27)) * 0x9E3779B1u ^ (uint32_t)k0;
    h = ((h ^ (uint32_t)k1) * 0x85EBCA77u) ^ (uint32_t)(k1 >> 32);
    return h * 0xC2B2AE3Du;
}
TKZ_HD uint32_t memo8_slot(uint64_t k0, uint32_t len, uint32_t bits) { return short_key_hash(k0, 0, len) >> (32 - bits); }
TKZ_HD uint32_t memo_slot(uint64_t k0, uint64_t k1, uint32_t len, uint32_t bits) {
    return short_key_hash(k0, k1, len) >> (32 - bits);
}

// -------- word memo slots ---------------------------------------------------------
// Both memo tables start every slot with the same 16-byte head {k0 lo, k0 hi, meta, w},
// meta = len | nt << 5 (len <= 16, nt <= 3 tokens; 0 = empty slot). A 32-B slot goes on
// with {k1 lo, k1 hi, token 1, token 2} and w = token 0; tokens are narrow (id | start << 16
// | end << 24). A 16-B slot (words of <= 8 bytes) holds w = the token when nt == 1; for
// nt = 2, 3 contiguous tokens covering [0, len) it packs the ids and split points:
// w = id0 | id1 << 16, meta |= e0 << 7 | e1 << 11 | id2 << 15.
constexpr uint32_t MEMO_RESERVED = 0x1Fu;  // meta of a slot being written (no len matches)

TKZ_HD bool memo8_pack(uint32_t len, uint32_t nt, const uint32_t* t, uint32_t& meta, uint32_t& w) {
    if (nt > 3u || len > 8u || len == 0u) return false;
    if (nt <= 1u) {
        meta = len | (nt << 5);
        w = nt ? t[0] : 0u;
        return true;
    }
    uint32_t prev = 0;
    for (uint32_t i = 0; i < nt; ++i) {
        if (((t[i] >> 16) & 0xFFu) != prev) return false;  // a dropped char: not contiguous
        prev = t[i] >> 24;
    }
    if (prev != len) return false;
    const uint32_t e0 = t[0] >> 24, e1 = nt == 3u ? t[1] >> 24 : 0u, id2 = nt == 3u ? t[2] & 0xFFFFu : 0u;
    meta = len | (nt << 5) | (e0 << 7) | (e1 << 11) | (id2 << 15);
    w = (t[0] & 0xFFFFu) | (t[1] << 16);
    return true;
}

// -------- everything a kernel needs, passed by value ---------------------------
struct DevTables {
    int model;            // 0 WordPiece, 1 BPE
    int norm;             // 0 none, 1 ASCII lowercase
    int pretok;           // 0 none, 1 whitespace, 2 bert
    int compact;          // BPE: 16-bit ids/ranks
    int chain;            // BPE: some merge has new_id == first (literal sequential path only)
    int mid;              // BPE, wide tables with ids < 2^20: word-bound tokens packed as
                          // id | start << 20 | (end - 1) << 26 (words <= 64 B), not wide
    int narrow;           // every vocab id < 2^16 (4-byte packed scratch tokens)
    // BPE
    const uint32_t* byte_id;  // [256]
    const uint4* cp_tab;
    uint32_t cp_bits;
    uint32_t unk_id;          // BPE: id for unknown chars, NONE = drop the char
    const uint2* mtab_c;
    const uint4* mtab_w;
    uint32_t m_bits;
    // WordPiece
    const uint4* wp_tab;
    uint32_t wp_bits;
    const uint8_t* wp_pool;
    const uint8_t* prefix;    // continuing_subword_prefix bytes (device)
    uint32_t plen;
    uint32_t wp_unk;          // NONE -> MissingUnkToken when needed
    int dedup;                // BPE: deduplicate the deferred words before the model (k_dedup)
    int unk_drop;             // FastTokenizer: a word needing a missing UNK yields no token
                              // (wordpiece.zig:241,297) instead of MissingUnkToken
    uint32_t max_chars;       // max_input_chars_per_word (clamped to 2^32-1)
    uint32_t max_key;         // longest vocab key in bytes
    uint64_t g_prefix;        // polynomial hash of the prefix
    uint64_t p_plen;          // HP^plen
    uint64_t hp_inv;          // HP^-1 mod 2^64
    const uint4* wps;         // keys of <= 16 bytes, bytes inline: {k0, k1}, {len | 0x100, id}
    uint32_t wps_bits;
    uint64_t pfx0, pfx1;      // prefix bytes packed little-endian (when plen <= 16)
    // BPE word memo (nullptr = off)
    const uint4* memo;        // 32-B slots {k0, k1}, {len | nt<<8, t0, t1, t2}
    uint32_t memo_bits;
    const uint4* memo8;       // keys <= 8 B: 16-B slots {k0, len | nt<<8 | 1<<16, t0}; nt = 0xFF: see memo
    uint32_t memo8_bits;
    // BPE long pretokens: ASCII bytes that are never a symbol (no vocab id and no unk, so
    // BPE.tokenize skips them, bpe.zig:192-208), bit c of drop_lo / drop_hi (c - 64), and
    // the switch of the segmented path that cuts long pretokens at them (k_bpe_long)
    uint64_t drop_lo, drop_hi;
    // ASCII chars whose symbol (own id, or unk) is in no merge, as first or second: no pair
    // ever forms across them, so they cut a pretoken exactly (inert_*); ASCII whitespace
    // with a mergeable symbol: the segmented path cuts before it and checks the cut (cut_*)
    uint64_t inert_lo, inert_hi, cut_lo, cut_hi;
    int seg;
    const uint32_t* r2id;     // wide tables (T.mid): merge rank -> new_id (the segmented path)
    const uint2* mtab_m;      // wide tables (T.mid): the mid cuckoo merge table, or null
    uint32_t mm_bits;
    // the segmented path's cuckoo table (compact, or mid): bit b set iff some merge whose
    // first bucket is b sits in its second one -- clear: a pair is in bucket b or nowhere (one
    // load); null = always both buckets
    const uint32_t* seg_over;
    uint32_t seg_over_bits;
    // segment memo (the segmented path's first encode of single segments; nullptr = off):
    // 32-B slots {key bytes 0-15}, {len | tokens << 5 | rounds << 10 | (hot index + 1) << 14,
    // meta bits 0..31, edges | meta bits 32..39 << 16, pool offset}; pool entry (16-B aligned)
    // = the edge-list pairs (SegEdges), then the tokens (id | start << 20 | end << 26) --
    // seg_encode's outputs for the key
    const uint4* smemo;
    uint32_t smemo_bits;
    const uint32_t* smpool;
    // hot pairs: hot_k memo keys (the lowest token ids) and, for each ordered pair (a, b) of
    // them, whether the boundary between a and b as adjacent segments is crossed (bit
    // a * hot_k + b; computed at build by the same check, k_seg_hot_build); null = none
    const uint32_t* hot_bits;
    uint32_t hot_k;
};

}  // namespace tkz
