// Host side of the MI355X tokenizer: tokenizer.json loader (restating
// jrc2139/tokenizer-zig src/config.zig:59-457), GPU table construction, the C ABI of
// include/tkz.h, and the host-only API pieces (decode, vocab queries, added tokens).
// Encode always runs on the GPU (encode.hip); there is no CPU fallback.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/tkz.h"
#include "decode.hpp"
#include "encode.hpp"
#include "json.hpp"
#include "pad.hpp"
#include "span.hpp"
#include "tables.hpp"

// smallest sub-batch a device workspace must hold (tkz_device_workspace_min)
constexpr uint64_t TKZ_SUB_MIN = 1ull << 20;

using tkz::DevTables;
using tkz::NONE;
namespace json = tkz::json;

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

uint32_t seq_len_host(uint8_t b) {
    if (b < 0x80) return 1;
    if (b >= 0xC0 && b <= 0xDF) return 2;
    if (b >= 0xE0 && b <= 0xEF) return 3;
    if (b >= 0xF0 && b <= 0xF7) return 4;
    return 1;
}

uint32_t pow2_bits(size_t n_slots_min) {
    uint32_t bits = 4;
    while (((size_t)1 << bits) < n_slots_min) ++bits;
    return bits;
}

// Cuckoo insertion of every merge into 2^bits two-slot buckets (random-walk eviction,
// deterministic). False if some insertion walks too long (the caller grows the table).
template <class M>
static bool build_cuckoo(const M& merges, uint32_t bits, std::vector<uint2>& tab) {
    tab.assign((size_t)2 << bits, uint2{tkz::EMPTY32, tkz::EMPTY32});
    uint64_t rng = 0x9E3779B97F4A7C15ull;
    for (auto& kv : merges) {
        uint2 cur{((uint32_t)(kv.first >> 32) << 16) | (uint32_t)kv.first, (kv.second.first << 16) | kv.second.second};
        uint32_t b1, b2;
        tkz::merge_buckets_compact(cur.x, bits, b1, b2);
        bool placed = false;
        for (uint32_t bk : {b1, b2})
            for (int s = 0; s < 2 && !placed; ++s)
                if (tab[2 * bk + s].x == tkz::EMPTY32) { tab[2 * bk + s] = cur; placed = true; }
        uint32_t bk = b1;
        for (int it = 0; it < 4096 && !placed; ++it) {
            rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17;
            std::swap(cur, tab[2 * bk + (rng & 1)]);
            uint32_t c1, c2;
            tkz::merge_buckets_compact(cur.x, bits, c1, c2);
            bk = bk == c1 ? c2 : c1;
            for (int s = 0; s < 2 && !placed; ++s)
                if (tab[2 * bk + s].x == tkz::EMPTY32) { tab[2 * bk + s] = cur; placed = true; }
        }
        if (!placed) return false;
    }
    return true;
}

// The mid cuckoo table (tables.hpp): same insertion as build_cuckoo, 8-B slots keyed by
// (a, b) with the rank
template <class M>
static bool build_cuckoo_mid(const M& merges, uint32_t bits, std::vector<uint2>& tab) {
    tab.assign((size_t)2 << bits, uint2{tkz::EMPTY32, tkz::EMPTY32});
    uint64_t rng = 0x9E3779B97F4A7C15ull;
    auto ab = [](const uint2& s, uint32_t& a, uint32_t& b) { a = s.x & 0xFFFFFu; b = (s.x >> 20) | ((s.y & 0xFFu) << 12); };
    for (auto& kv : merges) {
        uint2 cur = tkz::mid_slot((uint32_t)(kv.first >> 32), (uint32_t)kv.first, kv.second.first);
        uint32_t a, b, b1, b2;
        ab(cur, a, b);
        tkz::merge_buckets_mid(a, b, bits, b1, b2);
        bool placed = false;
        for (uint32_t bk : {b1, b2})
            for (int s = 0; s < 2 && !placed; ++s)
                if (tab[2 * bk + s].x == tkz::EMPTY32) { tab[2 * bk + s] = cur; placed = true; }
        uint32_t bk = b1;
        for (int it = 0; it < 4096 && !placed; ++it) {
            rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17;
            std::swap(cur, tab[2 * bk + (rng & 1)]);
            uint32_t c1, c2;
            ab(cur, a, b);
            tkz::merge_buckets_mid(a, b, bits, c1, c2);
            bk = bk == c1 ? c2 : c1;
            for (int s = 0; s < 2 && !placed; ++s)
                if (tab[2 * bk + s].x == tkz::EMPTY32) { tab[2 * bk + s] = cur; placed = true; }
        }
        if (!placed) return false;
    }
    return true;
}

// The overflow bitmap of a two-bucket cuckoo table (DevTables::seg_over): bit b1 for every
// key that sits in its second bucket. key_buckets(slot, b1, b2) gives a stored slot's buckets.
template <class F>
static std::vector<uint32_t> cuckoo_over(const std::vector<uint2>& tab, uint32_t bits, F key_buckets) {
    std::vector<uint32_t> over(std::max<size_t>(((size_t)1 << bits) / 32, 1), 0u);
    for (size_t i = 0; i < tab.size(); ++i) {
        if (tab[i].x == tkz::EMPTY32) continue;
        uint32_t b1, b2;
        key_buckets(tab[i], b1, b2);
        if (i / 2 != b1) over[b1 >> 5] |= 1u << (b1 & 31u);
    }
    return over;
}

uint64_t inv_mod_2_64(uint64_t a) {  // a odd; Newton iteration
    uint64_t x = a;
    for (int i = 0; i < 6; ++i) x *= 2 - a * x;
    return x;
}

// tkz_host_profile_read fields (ms unless noted)
enum {
    HP_CALLS, HP_CHUNKS, HP_BYTES_IN, HP_BYTES_OUT, HP_WALL, HP_ALLOC, HP_WAIT, HP_FIXUP,
    HP_H2D, HP_ENC, HP_D2H, HP_H2D_SPAN, HP_ENC_SPAN, HP_D2H_SPAN, HP_FIRST_ENC, HP_LAST_D2H,
    HP_OUT_PAGEABLE,  // output arrays (ids, offsets) the pinned pool could not serve (malloc'd)
    HP_N
};

struct DeviceState {
    bool ready = false;
    int device = -1;
    hipStream_t stream = nullptr;
    DevTables T{};
    std::vector<void*> allocs;
    // staging for the host-buffer API (grow-only)
    uint8_t* d_bytes = nullptr; size_t cap_bytes = 0;
    uint64_t* d_off = nullptr; size_t cap_off = 0;
    uint64_t* d_row = nullptr; size_t cap_row = 0;
    uint32_t* d_ids = nullptr; size_t cap_tok = 0;
    uint64_t* d_offs = nullptr; size_t cap_offs = 0;
    void* d_ws = nullptr; size_t cap_ws = 0;
    uint32_t* d_status = nullptr;
    // pipelined host batches: device-to-host stream, per-chunk events, page-locked counts
    hipStream_t d2h = nullptr;
    std::vector<hipEvent_t> chunk_ev;
    uint64_t* h_cnt = nullptr; size_t cap_h_cnt = 0;
    std::vector<uint64_t> h_off;  // rebased doc offsets of every chunk
    // BPE word memo (vocab key -> tokens), built on the GPU at first device use
    bool memo_built = false;
    const uint4* memo = nullptr;
    uint32_t memo_bits = 0;
    const uint4* memo8 = nullptr;
    uint32_t memo8_bits = 0;
    size_t memo_entries = 0;
    size_t memo_bytes = 0;  // both device tables
    const uint4* smemo = nullptr;  // segment memo (seg_mode tokenizers)
    uint32_t smemo_bits = 0;
    const uint32_t* smpool = nullptr;
    const uint32_t* hot_bits = nullptr;  // hot-pair bitmap (DevTables::hot_bits)
    uint32_t hot_k = 0;
    size_t smemo_entries = 0;
    size_t smemo_bytes = 0;  // segment memo table + pool
    // hot-pair candidates in rank order (pool entry + 1, meta; build_hot takes the first
    // hot_k), the bitmap (owned here, rebuilt by tkz_set_hot_pairs) and its build time
    std::vector<uint32_t> hot_q_host;
    std::vector<uint64_t> hot_m_host;
    uint32_t* hot_alloc = nullptr;
    size_t hot_bytes = 0;
    double hot_build_ms = 0;
    // batched decode tables (model-vocab strings + special flags), rebuilt when the added
    // vocab changes
    tkz::DecTables DT{};
    uint64_t dec_version = ~0ull;
    uint32_t* d_dec_ids = nullptr; size_t cap_dec_ids = 0;
    uint64_t* d_dec_row = nullptr; size_t cap_dec_row = 0;
    uint8_t* d_dec_out = nullptr; size_t cap_dec_out = 0;
    uint64_t* d_dec_off = nullptr; size_t cap_dec_off = 0;
    uint8_t* d_dec_ws = nullptr; size_t cap_dec_ws = 0;
    // truncation / padding outputs of the host-buffer batch API
    uint64_t* d_row2 = nullptr; size_t cap_row2 = 0;
    uint32_t* d_ids2 = nullptr; size_t cap_ids2 = 0;
    uint64_t* d_offs2 = nullptr; size_t cap_offs2 = 0;
    uint32_t* d_masks = nullptr; size_t cap_masks = 0;  // type_ids | special | attention
    uint8_t* d_pad_ws = nullptr; size_t cap_pad_ws = 0;
    // FastTokenizer span batches of the host-buffer API
    uint8_t* d_fast_ws = nullptr; size_t cap_fast_ws = 0;
    uint32_t* d_span = nullptr; size_t cap_span = 0;  // len | ids | attention
    uint64_t* d_span_offs = nullptr; size_t cap_span_offs = 0;
    // profiling: one event set per call since the last read
    bool profile = false;
    std::vector<tkz::KernelTimers> timers;
    size_t n_timed = 0;
    // host-buffer path timeline (profiling on): per chunk, timing events around its input
    // copy, its encode and its output slices; host timers around allocation, waits and the
    // row_ptr fix-up. Accumulated over calls (tkz_host_profile_read)
    std::vector<hipEvent_t> hp_ev;  // 5 per chunk: in0, in1, enc1 (stream) | out0, out1 (d2h)
    double hp[HP_N] = {};
};

}  // namespace

struct tkz_tokenizer {
    // ---- config (what loadConfig installed) ----
    int model = 0, norm = 0, pretok = 0, decoder = 0, has_pp = 0;
    std::vector<std::string> keys;                      // vocab keys, document order
    std::unordered_map<std::string, uint32_t> vocab;    // model vocab
    std::unordered_map<uint32_t, const std::string*> vocab_r;
    std::unordered_map<uint64_t, std::pair<uint32_t, uint32_t>> merges;  // pair -> (rank, new_id)
    size_t n_accepted = 0;
    bool has_unk = false;
    std::string unk, prefix = "##";
    uint64_t max_chars = 100;
    // ---- added vocab (src/vocab.zig) ----
    std::unordered_map<std::string, uint32_t> added_t2i;
    std::unordered_map<uint32_t, std::string> added_i2t;
    std::unordered_set<std::string> special;
    uint64_t added_version = 0;  // bumped by every added token (decode tables follow it)
    // ---- Tokenizer.truncation / Tokenizer.padding (lib.zig:41-42), off by default ----
    tkz::PadParams pp{};
    std::string pad_token = "[PAD]";
    uint32_t next_id = 0;
    // ---- host images of the GPU tables ----
    bool compact = false;
    uint32_t bpe_unk = NONE, wp_unk = NONE, max_key = 0;
    std::vector<uint32_t> byte_id;
    std::vector<uint4> cp_tab; uint32_t cp_bits = 4;
    std::vector<uint2> mtab_c; std::vector<uint4> mtab_w; uint32_t m_bits = 4;
    std::vector<uint4> wp_tab; uint32_t wp_bits = 4;
    std::vector<uint4> wps_tab; uint32_t wps_bits = 4;  // short keys, bytes inline (2 x uint4 per slot)
    std::vector<uint8_t> wp_pool;
    std::vector<uint32_t> r2id;  // wide BPE tables: merge rank -> new_id (the segmented path)
    std::vector<uint2> mtab_m; uint32_t mm_bits = 4;  // wide tables, ids < 2^20 - 1: mid cuckoo merge table
    std::vector<uint32_t> seg_over; uint32_t seg_over_bits = 0;  // the segmented path's table's overflow bits
    // every merge ranks after every merge that creates one of its parts (merges_ordered):
    // the condition under which the segmented path's edge-list boundary check is exact
    bool merges_ordered = true;
    bool seg_want = true;  // tkz_set_long_segments
    int64_t hot_want = -1;  // tkz_set_hot_pairs: keys of the hot-pair bitmap (-1: TKZ_HOT_K or 65,536)
    DevTables hostT{};
    // ---- device ----
    bool memo_on = true;
    int dedup_mode = -1;  // tkz_set_dedup: -1 auto, 0 off, 1 on
    uint64_t host_chunk = 32ull << 20;  // tkz_set_host_pipeline: input bytes per chunk, 0 = off
    double host_ratio = 0;              // tokens per input byte of the last host batch
    size_t n_cp = 0;      // multi-byte codepoints in the vocab
    std::mutex mu;
    DeviceState dev;
    int want_device = -1;  // tkz_opts.device: the device the state binds to (-1: current at first use)
    // tkz_encode_batch_gpus: encode-only copies of the tables, one per gpu_mask bit, made on
    // first use and kept (each binds to its device and uploads its tables once)
    std::vector<std::pair<int, tkz_tokenizer*>> replicas;
    int virtual_devices = 0;  // tkz_set_virtual_devices (tests): gpu_mask bit i -> device i % count
};

namespace {

// Host memory for tkz_encode_batch's CSR output. The device-to-host copy of the output
// is the largest cost of the host-buffer path (1.3 GB for C1 at 25 GB/s into pageable
// memory); into page-locked memory it runs at full PCIe rate. Page-locking is itself
// slow, so blocks are pooled: tkz_batch_free returns them, the next batch reuses them.
// Process-wide (tkz_batch_free has no tokenizer handle); never destroyed (no HIP calls at
// exit). Requests below 1 MiB, and any the pool cannot serve, use malloc.
struct PinnedPool {
    struct Blk { void* p; size_t n; bool used; };
    std::mutex mu;
    std::vector<Blk> blks;
    static constexpr size_t MIN_BYTES = 1u << 20;
    static constexpr size_t MAX_FREE_BYTES = 8ull << 30;  // cached, unused page-locked bytes
    void* get(size_t n) {
        std::lock_guard<std::mutex> g(mu);
        Blk* best = nullptr;
        for (auto& b : blks)  // best fit among free blocks, at most 2x the request
            if (!b.used && b.n >= n && b.n <= 2 * n && (!best || b.n < best->n)) best = &b;
        if (best) { best->used = true; return best->p; }
        void* p = nullptr;
        if (hipHostMalloc(&p, n, hipHostMallocDefault) != hipSuccess) return nullptr;
        blks.push_back(Blk{p, n, true});
        return p;
    }
    bool put(void* p) {
        if (!p) return true;
        std::lock_guard<std::mutex> g(mu);
        bool found = false;
        size_t free_bytes = 0;
        for (auto& b : blks) {
            if (b.p == p) { b.used = false; found = true; }
            if (!b.used) free_bytes += b.n;
        }
        while (found && free_bytes > MAX_FREE_BYTES) {  // release the largest free blocks
            auto it = blks.end();
            for (auto j = blks.begin(); j != blks.end(); ++j)
                if (!j->used && (it == blks.end() || j->n > it->n)) it = j;
            if (it == blks.end()) break;
            (void)hipHostFree(it->p);
            free_bytes -= it->n;
            blks.erase(it);
        }
        return found;
    }
};
PinnedPool& pinned_pool() {
    static PinnedPool* P = new PinnedPool;
    return *P;
}
void* out_alloc(size_t n, bool* pinned = nullptr) {
    void* p = n >= PinnedPool::MIN_BYTES ? pinned_pool().get(n) : nullptr;
    if (pinned) *pinned = p != nullptr;
    return p ? p : malloc(n);
}
void out_free(void* p) {
    if (p && !pinned_pool().put(p)) free(p);
}

const json::Value* get_str(const json::Value* o, const char* k) {
    const json::Value* v = o->get(k);
    return (v && v->is(json::Type::String)) ? v : nullptr;
}

int parse_vocab(tkz_tokenizer* t, const json::Value* m) {
    const json::Value* vv = m->get("vocab");
    if (!vv || !vv->is(json::Type::Object)) return fail(TKZ_ERR_MISSING_VOCAB, "model.vocab missing or not an object");
    t->keys.reserve(vv->obj.size());
    for (auto& kv : vv->obj) {
        const json::Value* v = kv.second.get();
        // config.zig:162-166: integer -> @intCast(u32); 0xFFFFFFFF is reserved here
        if (!v->is(json::Type::Integer) || v->i < 0 || v->i >= 0xFFFFFFFFll)
            return fail(TKZ_ERR_INVALID_VOCAB_ENTRY, "vocab entry '" + kv.first + "' is not a valid u32 id");
        t->keys.push_back(kv.first);
        t->vocab[kv.first] = (uint32_t)v->i;
    }
    for (auto& k : t->keys) t->vocab_r[t->vocab[k]] = &k;  // unique ids assumed; last wins
    return TKZ_OK;
}

// config.zig:124-295
int parse_model(tkz_tokenizer* t, const json::Value* root) {
    const json::Value* m = root->get("model");
    if (!m || !m->is(json::Type::Object)) return fail(TKZ_ERR_MISSING_MODEL, "missing 'model' object");
    const json::Value* ty = get_str(m, "type");
    std::string type = ty ? ty->s : "WordPiece";
    if (type == "WordPiece") {
        t->model = 0;
        int rc = parse_vocab(t, m);
        if (rc) return rc;
        const json::Value* u = get_str(m, "unk_token");
        t->unk = u ? u->s : "[UNK]";
        t->has_unk = true;
        const json::Value* p = get_str(m, "continuing_subword_prefix");
        t->prefix = p ? p->s : "##";
        const json::Value* mc = m->get("max_input_chars_per_word");
        t->max_chars = (mc && mc->is(json::Type::Integer) && mc->i >= 0) ? (uint64_t)mc->i : 100;
        return TKZ_OK;
    }
    if (type == "BPE") {
        t->model = 1;
        int rc = parse_vocab(t, m);
        if (rc) return rc;
        const json::Value* mv = m->get("merges");
        uint32_t rank = 0;
        if (mv && mv->is(json::Type::Array)) {
            for (auto& item : mv->arr) {
                std::string first, second;
                if (item->is(json::Type::String)) {
                    // std.mem.splitScalar(u8, s, ' '): first two segments (config.zig:238-241)
                    const std::string& s = item->s;
                    size_t sp = s.find(' ');
                    if (sp == std::string::npos) continue;
                    first = s.substr(0, sp);
                    size_t sp2 = s.find(' ', sp + 1);
                    second = s.substr(sp + 1, sp2 == std::string::npos ? std::string::npos : sp2 - sp - 1);
                } else if (item->is(json::Type::Array) && item->arr.size() == 2) {
                    if (!item->arr[0]->is(json::Type::String) || !item->arr[1]->is(json::Type::String)) continue;
                    first = item->arr[0]->s;
                    second = item->arr[1]->s;
                } else {
                    continue;
                }
                auto ia = t->vocab.find(first);
                if (ia == t->vocab.end()) continue;
                auto ib = t->vocab.find(second);
                if (ib == t->vocab.end()) continue;
                if (first.size() + second.size() > 512) continue;  // merged_buf: [512]u8
                auto in = t->vocab.find(first + second);
                if (in == t->vocab.end()) continue;
                t->merges[((uint64_t)ia->second << 32) | ib->second] = {rank, in->second};  // put overwrites
                ++rank;
            }
        }
        t->n_accepted = rank;
        const json::Value* u = get_str(m, "unk_token");
        t->has_unk = u != nullptr;
        if (u) t->unk = u->s;
        return TKZ_OK;
    }
    return fail(TKZ_ERR_UNSUPPORTED_MODEL_TYPE, "unsupported model type '" + type + "'");
}

bool add_token(tkz_tokenizer* t, const std::string& content, bool has_id, uint32_t id, bool special) {
    // vocab.zig:39-81 addSpecialToken / addToken
    if (t->added_t2i.count(content)) return false;
    uint32_t i = has_id ? id : t->next_id;
    if (i >= t->next_id) t->next_id = i + 1;
    t->added_t2i[content] = i;
    t->added_i2t[i] = content;
    if (special) t->special.insert(content);
    ++t->added_version;
    return true;
}

// Does every merge rank after every merge that creates one of its parts? (a token created by
// several merges counts with the largest of their ranks.) Then a round of BPE.tokenize only
// creates pairs that rank above it (bpe.zig:214-253: the new pairs all hold the new token), so
// a group's round values strictly increase, and the segmented path's boundary check may bound
// a straddling pair by the next round that changes an edge symbol alone (encode.hip
// seg_crossed_core; the rounds in between rank below it). A trained table (every merge makes a
// new token from existing ones) always qualifies; a hand-made one may not: e.g. merges
// (ab,c), (c,d), (a,b) encode "abcd" as [ab, cd], and its groups abc | d would be judged
// uncrossed. Such tables run without the segmented path (tests/test_segments.py).
static bool merges_ordered(const std::unordered_map<uint64_t, std::pair<uint32_t, uint32_t>>& merges) {
    std::unordered_map<uint32_t, uint32_t> made;  // token -> 1 + the largest rank creating it
    for (auto& kv : merges) {
        uint32_t& r = made[kv.second.second];
        r = std::max(r, kv.second.first + 1u);
    }
    for (auto& kv : merges) {
        const uint32_t rank = kv.second.first;
        for (uint32_t part : {(uint32_t)(kv.first >> 32), (uint32_t)kv.first}) {
            auto it = made.find(part);
            if (it != made.end() && it->second > rank) return false;  // (created at or after `rank`)
        }
    }
    return true;
}

void build_tables(tkz_tokenizer* t) {
    // BPE initial-symbol tables
    t->byte_id.assign(256, NONE);
    size_t n_cp = 0;
    for (auto& k : t->keys) {
        if (k.size() == 1) t->byte_id[(uint8_t)k[0]] = t->vocab[k];
        else if (k.size() <= 4 && seq_len_host((uint8_t)k[0]) >= k.size()) ++n_cp;
    }
    t->n_cp = n_cp;
    t->cp_bits = pow2_bits(n_cp * 2 + 2);
    t->cp_tab.assign((size_t)1 << t->cp_bits, uint4{0, 0, 0, 0});
    for (auto& k : t->keys) {
        if (k.size() < 2 || k.size() > 4 || seq_len_host((uint8_t)k[0]) < k.size()) continue;
        uint32_t packed = 0;
        for (size_t j = 0; j < k.size(); ++j) packed |= (uint32_t)(uint8_t)k[j] << (8 * j);
        uint32_t len = (uint32_t)k.size(), mask = (1u << t->cp_bits) - 1;
        uint32_t h = tkz::cp_slot(packed, len, t->cp_bits);
        while (t->cp_tab[h].y != 0) h = (h + 1) & mask;
        t->cp_tab[h] = uint4{packed, len, t->vocab[k], 0};
    }
    t->bpe_unk = NONE;
    if (t->model == 1 && t->has_unk) {
        auto it = t->vocab.find(t->unk);
        if (it != t->vocab.end()) t->bpe_unk = it->second;
    }
    // merge table
    uint32_t max_id = 0;
    for (auto& kv : t->vocab) max_id = std::max(max_id, kv.second);
    t->compact = (max_id < 0xFFFFu) && (t->n_accepted < 0xFFFFu);
    t->m_bits = pow2_bits(t->merges.size() * 4 + 4);
    const uint32_t mmask = (1u << t->m_bits) - 1;
    if (t->compact) {
        // bucketized cuckoo (tables.hpp): 2^bits two-slot buckets, >= 2 slots per merge
        t->m_bits = pow2_bits(t->merges.size() + 2);
        while (!build_cuckoo(t->merges, t->m_bits, t->mtab_c)) ++t->m_bits;
        t->mtab_w.assign(1, uint4{tkz::EMPTY32, tkz::EMPTY32, tkz::EMPTY32, tkz::EMPTY32});
    } else {
        t->mtab_w.assign((size_t)1 << t->m_bits, uint4{tkz::EMPTY32, tkz::EMPTY32, tkz::EMPTY32, tkz::EMPTY32});
        for (auto& kv : t->merges) {
            uint32_t h = tkz::merge_slot_wide(kv.first, t->m_bits);
            while (t->mtab_w[h].z != tkz::EMPTY32) h = (h + 1) & mmask;
            t->mtab_w[h] = uint4{(uint32_t)(kv.first >> 32), (uint32_t)kv.first, kv.second.first, kv.second.second};
        }
        t->mtab_c.assign(1, uint2{tkz::EMPTY32, tkz::EMPTY32});
    }
    // WordPiece string table
    t->wp_bits = pow2_bits(t->keys.size() * 2 + 2);
    t->wp_tab.assign((size_t)1 << t->wp_bits, uint4{0, 0, NONE, NONE});
    t->wp_pool.clear();
    t->max_key = 0;
    const uint32_t wmask = (1u << t->wp_bits) - 1;
    for (auto& k : t->keys) {
        uint64_t g = 0, pw = 1;
        for (unsigned char ch : k) { g += (uint64_t)(ch + 1) * pw; pw *= tkz::HP; }
        uint64_t h = tkz::wp_final(g, (uint32_t)k.size());
        uint32_t off = (uint32_t)t->wp_pool.size();
        uint32_t len = (uint32_t)k.size();
        t->wp_pool.resize(off + 4 + ((len + 3) & ~3u), 0);
        memcpy(&t->wp_pool[off], &len, 4);
        memcpy(&t->wp_pool[off + 4], k.data(), len);
        uint32_t idx = (uint32_t)(h >> (64 - t->wp_bits));
        while (t->wp_tab[idx].w != NONE) idx = (idx + 1) & wmask;
        t->wp_tab[idx] = uint4{(uint32_t)h, (uint32_t)(h >> 32), t->vocab[k], off};
        t->max_key = std::max<uint32_t>(t->max_key, len);
    }
    if (t->wp_pool.empty()) t->wp_pool.resize(4, 0);
    // short-key table (<= 16 bytes): exact inline compare on the device
    {
        size_t n_short = 0;
        for (auto& k : t->keys) n_short += k.size() <= 16;
        // load <= 1/4, linear probing without wrap-around into a zero tail: wps_probe reads
        // one 32-B slot per round (TKZ_WPS_WIN; two per round measured 3.5 % slower on C3)
        constexpr size_t PAD = 64;
        t->wps_bits = pow2_bits(n_short * 4 + 2);
        for (;;) {
            t->wps_tab.assign((((size_t)1 << t->wps_bits) + PAD) * 2, uint4{0, 0, 0, 0});
            bool overflow = false;
            for (auto& k : t->keys) {
                if (k.size() > 16) continue;
                uint64_t k0 = 0, k1 = 0;
                memcpy(&k0, k.data(), std::min<size_t>(k.size(), 8));
                if (k.size() > 8) memcpy(&k1, k.data() + 8, k.size() - 8);
                size_t h = tkz::memo_slot(k0, k1, (uint32_t)k.size(), t->wps_bits);
                while (t->wps_tab[2 * h + 1].x != 0) ++h;
                if (2 * (h + 2) >= t->wps_tab.size()) { overflow = true; break; }
                t->wps_tab[2 * h] = uint4{(uint32_t)k0, (uint32_t)(k0 >> 32), (uint32_t)k1, (uint32_t)(k1 >> 32)};
                t->wps_tab[2 * h + 1] = uint4{(uint32_t)k.size() | 0x100u, t->vocab[k], 0, 0};
            }
            if (!overflow) break;
            ++t->wps_bits;
        }
    }
    t->wp_unk = NONE;
    if (t->model == 0) {
        auto it = t->vocab.find(t->unk);
        if (it != t->vocab.end()) t->wp_unk = it->second;
    }
    // host view (debug lookups use the same probe code as the kernels)
    DevTables& T = t->hostT;
    T.model = t->model; T.norm = t->norm; T.pretok = t->pretok; T.compact = t->compact ? 1 : 0;
    T.chain = 0;
    T.narrow = max_id <= 0xFFFFu ? 1 : 0;
    T.mid = (t->model == 1 && !t->compact && max_id < (1u << 20)) ? 1 : 0;
    for (auto& kv : t->merges)
        if (kv.second.second == (uint32_t)(kv.first >> 32)) T.chain = 1;
    T.byte_id = t->byte_id.data(); T.cp_tab = t->cp_tab.data(); T.cp_bits = t->cp_bits; T.unk_id = t->bpe_unk;
    // the segmented path's cut chars (ASCII): dropped (no id, no unk: bpe.zig:192-208),
    // inert (its symbol -- own id or unk, bpe.zig:198-205 -- is in no merge on either side:
    // no pair forms across it) and whitespace with a mergeable symbol (a checked cut)
    T.drop_lo = T.drop_hi = T.inert_lo = T.inert_hi = T.cut_lo = T.cut_hi = 0;
    t->r2id.clear();
    if (t->model == 1) {
        std::unordered_set<uint32_t> in_merge;
        uint32_t max_rank = 0;
        for (auto& kv : t->merges) {
            in_merge.insert((uint32_t)(kv.first >> 32));
            in_merge.insert((uint32_t)kv.first);
            max_rank = std::max(max_rank, kv.second.first);
        }
        for (uint32_t c = 0; c < 128; ++c) {
            const uint32_t sym = t->byte_id[c] != NONE ? t->byte_id[c] : t->bpe_unk;
            const uint64_t bit = 1ull << (c & 63);
            const bool ws = c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == 0x0B || c == 0x0C;
            if (sym == NONE) (c < 64 ? T.drop_lo : T.drop_hi) |= bit;
            else if (!in_merge.count(sym)) (c < 64 ? T.inert_lo : T.inert_hi) |= bit;
            else if (ws) (c < 64 ? T.cut_lo : T.cut_hi) |= bit;
        }
        t->mtab_m.clear();
        if (!t->compact && !t->merges.empty() && max_rank < 0xFFFFFEu) {
            t->r2id.assign((size_t)max_rank + 1, NONE);
            for (auto& kv : t->merges) t->r2id[kv.second.first] = kv.second.second;
            uint32_t max_id = 0;
            for (auto& kv : t->vocab) max_id = std::max(max_id, kv.second);
            if (max_id < (1u << 20) - 1) {
                t->mm_bits = pow2_bits(t->merges.size() + 2);
                while (!build_cuckoo_mid(t->merges, t->mm_bits, t->mtab_m)) ++t->mm_bits;
            }
        }
    }
    T.r2id = t->r2id.empty() ? nullptr : t->r2id.data();
    T.mtab_m = t->mtab_m.empty() ? nullptr : t->mtab_m.data();
    T.mm_bits = t->mm_bits;
    t->seg_over.clear();
    t->seg_over_bits = 0;
    if (t->compact && !t->merges.empty()) {
        const uint32_t bits = t->m_bits;
        t->seg_over = cuckoo_over(t->mtab_c, bits, [bits](const uint2& sl, uint32_t& b1, uint32_t& b2) {
            tkz::merge_buckets_compact(sl.x, bits, b1, b2);
        });
        t->seg_over_bits = bits;
    } else if (!t->mtab_m.empty()) {
        const uint32_t bits = t->mm_bits;
        t->seg_over = cuckoo_over(t->mtab_m, bits, [bits](const uint2& sl, uint32_t& b1, uint32_t& b2) {
            tkz::merge_buckets_mid(sl.x & 0xFFFFFu, (sl.x >> 20) | ((sl.y & 0xFFu) << 12), bits, b1, b2);
        });
        t->seg_over_bits = bits;
    }
    T.seg_over = t->seg_over.empty() ? nullptr : t->seg_over.data();
    T.seg_over_bits = t->seg_over_bits;
    t->merges_ordered = merges_ordered(t->merges);
    T.seg = t->seg_want && t->merges_ordered;
    T.mtab_c = t->mtab_c.data(); T.mtab_w = t->mtab_w.data(); T.m_bits = t->m_bits;
    T.wp_tab = t->wp_tab.data(); T.wp_bits = t->wp_bits; T.wp_pool = t->wp_pool.data();
    T.prefix = (const uint8_t*)t->prefix.data(); T.plen = (uint32_t)t->prefix.size();
    T.wp_unk = t->wp_unk;
    T.max_chars = (uint32_t)std::min<uint64_t>(t->max_chars, 0xFFFFFFFFull);
    T.max_key = t->max_key;
    uint64_t gp = 0, pw = 1;
    for (unsigned char ch : t->prefix) { gp += (uint64_t)(ch + 1) * pw; pw *= tkz::HP; }
    T.g_prefix = gp; T.p_plen = pw; T.hp_inv = inv_mod_2_64(tkz::HP);
    T.wps = t->wps_tab.data(); T.wps_bits = t->wps_bits;
    T.pfx0 = T.pfx1 = 0;
    if (t->prefix.size() <= 16) {
        memcpy(&T.pfx0, t->prefix.data(), std::min<size_t>(t->prefix.size(), 8));
        if (t->prefix.size() > 8) memcpy(&T.pfx1, t->prefix.data() + 8, t->prefix.size() - 8);
    }
}

int load(tkz_tokenizer* t, const char* js, size_t n) {
    json::ValuePtr root = json::parse(js, n);
    if (!root || !root->is(json::Type::Object)) return fail(TKZ_ERR_INVALID_JSON, "invalid JSON");
    int rc = parse_model(t, root.get());
    if (rc) return rc;
    // config.zig:82-86 + lib.zig:66-72
    const json::Value* at = root->get("added_tokens");
    if (at && at->is(json::Type::Array)) {
        for (auto& item : at->arr) {
            if (!item->is(json::Type::Object)) continue;
            const json::Value* c = get_str(item.get(), "content");
            if (!c) continue;
            const json::Value* idv = item->get("id");
            bool has_id = idv && idv->is(json::Type::Integer) && idv->i >= 0 && idv->i <= 0xFFFFFFFFll;
            const json::Value* sp = item->get("special");
            bool special = sp && sp->is(json::Type::Bool) && sp->b;
            add_token(t, c->s, has_id, has_id ? (uint32_t)idv->i : 0, special);
        }
    }
    const json::Value* nv = root->get("normalizer");  // config.zig:339-362
    if (nv && nv->is(json::Type::Object)) {
        const json::Value* ty = get_str(nv, "type");
        if (ty && (ty->s == "BertNormalizer" || ty->s == "Lowercase")) t->norm = 1;
    }
    const json::Value* pv = root->get("pre_tokenizer");  // config.zig:381-403
    if (pv && pv->is(json::Type::Object)) {
        const json::Value* ty = get_str(pv, "type");
        if (ty && ty->s == "BertPreTokenizer") t->pretok = 2;
        else if (ty && (ty->s == "Whitespace" || ty->s == "WhitespaceSplit")) t->pretok = 1;
    }
    const json::Value* dv = root->get("decoder");  // config.zig:459-486
    if (dv && dv->is(json::Type::Object)) {
        const json::Value* ty = get_str(dv, "type");
        if (ty && ty->s == "WordPiece") t->decoder = 1;
        else if (ty && ty->s == "ByteLevel") t->decoder = 2;
        else if (ty && ty->s == "BPE") t->decoder = 3;
    }
    const json::Value* pp = root->get("post_processor");  // config.zig:532-549 (no-op)
    if (pp && pp->is(json::Type::Object)) {
        const json::Value* ty = get_str(pp, "type");
        if (ty && (ty->s == "TemplateProcessing" || ty->s == "BertProcessing")) t->has_pp = 1;
    }
    build_tables(t);
    return TKZ_OK;
}

// ------------------------------------------------------------------ device
template <class V>
int upload(DeviceState& d, const std::vector<V>& v, const V** out) {
    void* p = nullptr;
    size_t n = std::max<size_t>(v.size() * sizeof(V), 16);
    if (hipMalloc(&p, n) != hipSuccess) return fail(TKZ_ERR_DEVICE, "hipMalloc failed for table");
    d.allocs.push_back(p);
    if (!v.empty() && hipMemcpy(p, v.data(), v.size() * sizeof(V), hipMemcpyHostToDevice) != hipSuccess)
        return fail(TKZ_ERR_DEVICE, "hipMemcpy failed for table");
    *out = (const V*)p;
    return TKZ_OK;
}

int build_memo(tkz_tokenizer* t);

// auto: deduplicate the deferred BPE words when the vocab has many multi-byte chars.
// Such vocabs leave multi-byte words to the model (the general codepoint path, several
// times the cost of an ASCII word), where dedup pays for its extra passes (C2: deferred
// phase 0.87 -> 0.41 ms); on ASCII vocabs the deferred phase costs the same either way
// and the copied words make k_compact ~4 % slower (C1/C4). Results are identical.
#ifndef TKZ_DEDUP_MIN_CP
#define TKZ_DEDUP_MIN_CP 256
#endif
static void apply_dedup(tkz_tokenizer* t) {
    t->dev.T.dedup = t->model == 1 && (t->dedup_mode < 0 ? t->n_cp >= TKZ_DEDUP_MIN_CP : t->dedup_mode != 0);
}

int ensure_device(tkz_tokenizer* t) {
    DeviceState& d = t->dev;
    if (d.ready) {
        hipSetDevice(d.device);
        return TKZ_OK;
    }
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count < 1)
        return fail(TKZ_ERR_DEVICE, "no HIP device available (the encode path is GPU-only)");
    if (t->want_device >= 0) {
        if (t->want_device >= count) return fail(TKZ_ERR_INVALID_ARGUMENT, "tkz_opts.device: no such device");
        if (hipSetDevice(t->want_device) != hipSuccess) return fail(TKZ_ERR_DEVICE, "hipSetDevice failed");
    }
    if (hipGetDevice(&d.device) != hipSuccess) return fail(TKZ_ERR_DEVICE, "hipGetDevice failed");
    if (hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking) != hipSuccess)
        return fail(TKZ_ERR_DEVICE, "hipStreamCreate failed");
    d.T = t->hostT;
    int rc;
    const uint32_t* bid; const uint4* cpt; const uint2* mc; const uint4* mw; const uint4* wpt; const uint8_t* pool;
    const uint4* wps;
    const uint8_t* pre;
    const uint32_t* r2id;
    const uint2* mtm;
    const uint32_t* sov;
    std::vector<uint8_t> prev(t->prefix.begin(), t->prefix.end());
    if ((rc = upload(d, t->byte_id, &bid)) || (rc = upload(d, t->cp_tab, &cpt)) || (rc = upload(d, t->mtab_c, &mc)) ||
        (rc = upload(d, t->mtab_w, &mw)) || (rc = upload(d, t->wp_tab, &wpt)) || (rc = upload(d, t->wp_pool, &pool)) ||
        (rc = upload(d, prev, &pre)) || (rc = upload(d, t->wps_tab, &wps)) || (rc = upload(d, t->r2id, &r2id)) ||
        (rc = upload(d, t->mtab_m, &mtm)) || (rc = upload(d, t->seg_over, &sov)))
        return rc;
    d.T.seg_over = t->seg_over.empty() ? nullptr : sov;
    d.T.r2id = t->r2id.empty() ? nullptr : r2id;
    d.T.mtab_m = t->mtab_m.empty() ? nullptr : mtm;
    d.T.wps = wps;
    d.T.byte_id = bid; d.T.cp_tab = cpt; d.T.mtab_c = mc; d.T.mtab_w = mw; d.T.wp_tab = wpt; d.T.wp_pool = pool;
    d.T.prefix = pre;
    if (hipMalloc(&d.d_status, 16) != hipSuccess) return fail(TKZ_ERR_DEVICE, "hipMalloc failed");
    d.T.memo = nullptr;
    d.T.memo8 = nullptr;
    d.T.smemo = nullptr;
    d.T.hot_bits = nullptr;
    d.T.hot_k = 0;
    apply_dedup(t);
    d.ready = true;
    if (t->memo_on && (rc = build_memo(t))) return rc;
    return TKZ_OK;
}

// Word memo: BPE of every vocab key of 1..16 bytes, computed by the GPU encode path
// itself (no normalizer, whole key = one pretoken), stored in a verified hash table.
// A pretoken equal to a key then skips the merge rounds; the result is the same by
// construction (same kernel, same input bytes).
// Vocab keys of 1..16 bytes plus the variants a text carries as whole words although they
// are no key themselves: the capitalised form (no normalizer: a lowercasing one never leaves
// it) and, when punctuation stays attached (Whitespace, or no split at all), the key
// followed by one of TKZ_MEMO_PUNCT.
#ifndef TKZ_MEMO_VARIANTS
#define TKZ_MEMO_VARIANTS 3  // bit 0: capitalised first letter, bit 1: + trailing punctuation
#endif
#ifndef TKZ_MEMO_PUNCT
#define TKZ_MEMO_PUNCT ",."
#endif
static std::vector<std::string> memo_keys(const tkz_tokenizer* t, bool punct_whole, size_t* n_base = nullptr) {
    std::vector<std::string> out;
    std::unordered_set<std::string> have;
    for (auto& k : t->keys)
        if (!k.empty() && k.size() <= 16 && have.insert(k).second) out.push_back(k);
    if (n_base) *n_base = out.size();  // (the vocab keys; their variants follow)
    const bool cap = (TKZ_MEMO_VARIANTS & 1) && t->norm == 0;
    const bool punct = (TKZ_MEMO_VARIANTS & 2) && (t->pretok == 1 || (punct_whole && t->pretok == 0));
    auto add = [&](std::string v) {
        if (v.size() <= 16 && have.insert(v).second) out.push_back(std::move(v));
    };
    for (size_t i = 0, n0 = out.size(); i < n0; ++i) {
        const std::string k = out[i];
        const bool up = cap && k[0] >= 'a' && k[0] <= 'z';
        std::string ck = k;
        if (up) { ck[0] = (char)(k[0] - 32); add(ck); }
        if (punct)
            for (const char* p = TKZ_MEMO_PUNCT; *p; ++p) {
                add(k + *p);
                if (up) add(ck + *p);
            }
    }
    return out;
}

// The hot-pair bitmap: k x k bits over the first k ranked hot-key candidates (k_seg_first reads
// one bit for a boundary between two of them instead of walking their edge lists). k is the
// tkz_set_hot_pairs setting (default: the TKZ_HOT_K environment variable, else 65,536: a
// 512-MB bitmap, ~115 ms to build), capped by the candidates and by a budget of 1/64 of the
// device's free memory (it was allocated with no check). Rebuilt on each call;
// the staging buffers are freed once it is built.
#ifndef TKZ_HOT_DEFAULT
#define TKZ_HOT_DEFAULT 65536  // (C6 k_seg_first with 4096 keys 4.11 ms, 16384: 3.31 (r05r), 32768: 2.46, 65536: 1.80 (r05zm))
#endif
int build_hot(tkz_tokenizer* t) {
    DeviceState& d = t->dev;
    if (d.hot_alloc) hipFree(d.hot_alloc);
    d.hot_alloc = nullptr;
    d.hot_bits = nullptr;
    d.hot_k = 0;
    d.hot_bytes = 0;
    d.hot_build_ms = 0;
    d.T.hot_bits = nullptr;
    d.T.hot_k = 0;
    int64_t want = t->hot_want;
    if (want < 0) {
        const char* env = getenv("TKZ_HOT_K");
        want = env ? std::max<int64_t>(0, atoll(env)) : TKZ_HOT_DEFAULT;
    }
    uint64_t k = std::min<uint64_t>((uint64_t)want, d.hot_q_host.size());
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) return fail(TKZ_ERR_DEVICE, "hipMemGetInfo failed");
    const uint64_t budget = free_b / 64;
    while (k && (k * k + 7) / 8 > budget) k = k * 7 / 8;
    if (k == 0) return TKZ_OK;
    const auto t0 = std::chrono::steady_clock::now();
    const size_t nw = (size_t)((k * k + 31) / 32);
    uint32_t *dq = nullptr, *db = nullptr;
    uint64_t* dm = nullptr;
    auto cleanup = [&]() { if (dq) hipFree(dq); if (dm) hipFree(dm); };
    if (hipMalloc((void**)&dq, k * 4) != hipSuccess || hipMalloc((void**)&dm, k * 8) != hipSuccess ||
        hipMalloc((void**)&db, nw * 4) != hipSuccess) {
        (void)hipGetLastError();  // no room: every boundary takes the full check
        cleanup();
        return TKZ_OK;
    }
    hipError_t e = hipMemcpyAsync(dq, d.hot_q_host.data(), k * 4, hipMemcpyHostToDevice, d.stream);
    if (e == hipSuccess) e = hipMemcpyAsync(dm, d.hot_m_host.data(), k * 8, hipMemcpyHostToDevice, d.stream);
    if (e == hipSuccess) e = tkz::launch_seg_hot_build(d.T, dq, dm, (uint32_t)k, db, d.stream);
    if (e == hipSuccess) e = hipStreamSynchronize(d.stream);
    cleanup();
    if (e != hipSuccess) {
        hipFree(db);
        return fail(TKZ_ERR_DEVICE, std::string("hot pair build failed: ") + hipGetErrorString(e));
    }
    d.hot_alloc = db;
    d.hot_bits = db;
    d.hot_k = (uint32_t)k;
    d.hot_bytes = nw * 4;
    d.hot_build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    d.T.hot_bits = db;
    d.T.hot_k = (uint32_t)k;
    return TKZ_OK;
}

// Segment memo (seg_mode tokenizers: the segmented path's first encode of single segments):
// seg_encode's outputs for every memo key, computed by the GPU (k_seg_memo_build), in an
// open-addressed table of 32-B slots + a pool (tables.hpp). A segment equal to a key then
// skips its register BPE; the outputs are the same by construction.
int build_seg_memo(tkz_tokenizer* t) {
    DeviceState& d = t->dev;
    if (!tkz::seg_mode(d.T)) return TKZ_OK;
    size_t n_base = 0;
    std::vector<std::string> keys = memo_keys(t, true, &n_base);
    const size_t n = keys.size();
    if (n == 0) return TKZ_OK;
    std::vector<uint64_t> off(n + 1, 0);
    std::string blob;
    for (size_t i = 0; i < n; ++i) { blob += keys[i]; off[i + 1] = blob.size(); }
    const size_t padded = (blob.size() + 32 + 15) / 16 * 16;
    blob.resize(padded, '\0');
    uint8_t* dk = nullptr; uint64_t* doff = nullptr; uint64_t* dmeta = nullptr; uint32_t* dtok = nullptr;
    uint64_t* dprof = nullptr;
    auto cleanup = [&]() { for (void* p : {(void*)dk, (void*)doff, (void*)dmeta, (void*)dtok, (void*)dprof}) if (p) hipFree(p); };
    if (hipMalloc((void**)&dk, padded) != hipSuccess || hipMalloc((void**)&doff, (n + 1) * 8) != hipSuccess ||
        hipMalloc((void**)&dmeta, n * 8) != hipSuccess || hipMalloc((void**)&dtok, n * 64) != hipSuccess ||
        hipMalloc((void**)&dprof, n * 128) != hipSuccess) {
        cleanup();
        return fail(TKZ_ERR_OUT_OF_MEMORY, "device allocation failed (segment memo)");
    }
    hipMemcpyAsync(dk, blob.data(), padded, hipMemcpyHostToDevice, d.stream);
    hipMemcpyAsync(doff, off.data(), (n + 1) * 8, hipMemcpyHostToDevice, d.stream);
    hipError_t e = tkz::launch_seg_memo_build(d.T, dk, doff, (uint32_t)n, padded, dmeta, dtok, dprof, d.stream);
    std::vector<uint64_t> meta(n), prof(n * 16);
    std::vector<uint32_t> tok(n * 16);
    if (e == hipSuccess) {
        hipMemcpyAsync(meta.data(), dmeta, n * 8, hipMemcpyDeviceToHost, d.stream);
        hipMemcpyAsync(tok.data(), dtok, n * 64, hipMemcpyDeviceToHost, d.stream);
        hipMemcpyAsync(prof.data(), dprof, n * 128, hipMemcpyDeviceToHost, d.stream);
        e = hipStreamSynchronize(d.stream);
    }
    cleanup();
    if (e != hipSuccess) return fail(TKZ_ERR_DEVICE, std::string("segment memo build failed: ") + hipGetErrorString(e));
    size_t cnt = 0;
    for (size_t i = 0; i < n; ++i) cnt += meta[i] != ~0ull;
    if (cnt == 0) return TKZ_OK;
    constexpr size_t PAD = 64;  // linear probing without wrap-around into a zero tail
    uint32_t bits = pow2_bits(cnt * 4 + 2);
    // Hot keys: the TKZ_HOT_K keys whose tokens have the lowest ids (a BPE vocab numbers its
    // tokens in merge order, so these are the most frequent words), a capitalised or
    // punctuated variant ranked as if its ids were TKZ_HOT_VARIANT times larger (text carries
    // them far less often than the vocab key itself: on C6 the hot pairs then cover 97 % of
    // the boundaries between memo hits instead of 84 %); every ordered pair of them gets its
    // boundary check computed here once (k_seg_hot_build), and k_seg_first reads a bit
    // instead of walking and probing when both neighbours are hot.
#ifndef TKZ_HOT_MAX
#define TKZ_HOT_MAX 65536  // hot-key candidates ranked in the memo (the bitmap's k is at most this)
#endif
    std::vector<uint32_t> hot(n, 0);  // hot index + 1
    uint32_t hot_k = 0;  // (candidates: build_hot keeps the first tkz_set_hot_pairs / budget of them)
#ifndef TKZ_HOT_VARIANT
#define TKZ_HOT_VARIANT 8
#endif
    {
        std::vector<std::pair<uint64_t, uint32_t>> by;  // (rank: largest token id, variants scaled; key)
        for (size_t i = 0; i < n; ++i) {
            if (meta[i] == ~0ull) continue;
            const uint32_t nt = (uint32_t)(meta[i] >> 40) & 0xFFu;
            uint32_t mx = 0;
            for (uint32_t j = 0; j < nt; ++j) mx = std::max(mx, tok[16 * i + j] & 0xFFFFFu);
            by.push_back({(uint64_t)mx * (i < n_base ? 1u : TKZ_HOT_VARIANT), (uint32_t)i});
        }
        std::sort(by.begin(), by.end());
        hot_k = (uint32_t)std::min<size_t>(by.size(), TKZ_HOT_MAX);
        for (uint32_t h = 0; h < hot_k; ++h) hot[by[h].second] = h + 1;
    }
    std::vector<uint32_t> hot_q(hot_k);
    std::vector<uint64_t> hot_m(hot_k);
    std::vector<uint4> tab;
    std::vector<uint32_t> pool;
    for (;;) {
        tab.assign((((size_t)1 << bits) + PAD) * 2, uint4{0, 0, 0, 0});
        pool.clear();
        bool overflow = false;
        for (size_t i = 0; i < n && !overflow; ++i) {
            if (meta[i] == ~0ull) continue;
            const std::string& k = keys[i];
            const uint32_t L = (uint32_t)k.size();
            // meta: first | last << 20 | tokens << 40 | edges << 48 (encode.hip sm_make)
            const uint32_t nt = (uint32_t)(meta[i] >> 40) & 0xFFu, ed = (uint32_t)(meta[i] >> 48);
            uint64_t k0 = 0, k1 = 0;
            memcpy(&k0, k.data(), std::min<size_t>(8, k.size()));
            if (k.size() > 8) memcpy(&k1, k.data() + 8, k.size() - 8);
            size_t h = tkz::short_key_hash(k0, k1, L) >> (32 - bits);
            while (tab[2 * h + 1].x != 0) ++h;
            if (2 * (h + 2) >= tab.size()) { overflow = true; break; }
            const uint32_t rounds = (uint32_t)prof[16 * i + 15];  // (k_seg_memo_build: the round count)
            tab[2 * h] = uint4{(uint32_t)k0, (uint32_t)(k0 >> 32), (uint32_t)k1, (uint32_t)(k1 >> 32)};
            tab[2 * h + 1] = uint4{L | (nt << 5) | (rounds << 10) | (hot[i] << 14), (uint32_t)meta[i],
                                   ed | ((uint32_t)(meta[i] >> 32) & 0xFFu) << 16, (uint32_t)pool.size()};
            if (hot[i]) {
                hot_q[hot[i] - 1] = (uint32_t)pool.size() + 1u;
                hot_m[hot[i] - 1] = meta[i];
            }
            // [edge-list pairs RE_k | LE_k << 32, max(|RE|, |LE|) of them][tokens], 16-B
            // aligned (k_seg_first loads the first 4 pairs as two 16-B vectors)
            const uint32_t nle = ed & 0xFFu, nre = ed >> 8;
            for (uint32_t k = 0; k < std::max(nle, nre); ++k) {
                pool.push_back(k < nre ? (uint32_t)prof[16 * i + k] : ~0u);
                pool.push_back(k < nle ? (uint32_t)(prof[16 * i + k] >> 32) : ~0u);
            }
            for (uint32_t j = 0; j < nt; ++j) pool.push_back(tok[16 * i + j]);
            while (pool.size() % 4) pool.push_back(0u);
        }
        if (!overflow) break;
        ++bits;
    }
    pool.resize(pool.size() + 8, 0u);  // (the last entry's 32-B load)
    const uint4* dt = nullptr;
    const uint32_t* dp = nullptr;
    int rc = upload(d, tab, &dt);
    if (rc || (rc = upload(d, pool, &dp))) return rc;
    d.smemo = dt;
    d.smemo_bits = bits;
    d.smpool = dp;
    d.smemo_entries = cnt;
    d.T.smemo = dt;
    d.T.smemo_bits = bits;
    d.T.smpool = dp;
    d.smemo_bytes = tab.size() * sizeof(uint4) + pool.size() * 4;
    d.hot_q_host = std::move(hot_q);
    d.hot_m_host = std::move(hot_m);
    return build_hot(t);
}

int build_memo(tkz_tokenizer* t) {
    DeviceState& d = t->dev;
    d.T.memo = nullptr;
    d.T.memo8 = nullptr;
    d.T.smemo = nullptr;
    d.T.hot_bits = nullptr;
    d.T.hot_k = 0;
    if (d.memo_built) {
        if (d.memo) d.T.memo = d.memo;
        d.T.memo_bits = d.memo_bits;
        d.T.memo8 = d.memo8;
        d.T.memo8_bits = d.memo8_bits;
        d.T.smemo = d.smemo;
        d.T.smemo_bits = d.smemo_bits;
        d.T.smpool = d.smpool;
        d.T.hot_bits = d.hot_bits;
        d.T.hot_k = d.hot_k;
        return TKZ_OK;
    }
    d.memo_built = true;
    if (int rc = build_seg_memo(t)) return rc;
    // compact tables: narrow tokens (id | start << 16 | end << 24), keys <= 8 B in the 16-B
    // table; wide tables (ids <= 2^22): id | start << 22 | end << 27, every key in the 32-B
    // table. A table with a new_id == first merge is built by the same (literal) kernel path.
    const bool wide = !t->compact;
    if (t->model != 1) return TKZ_OK;
    if (wide) {
        uint32_t max_id = 0;
        for (auto& kv : t->vocab) max_id = std::max(max_id, kv.second);
        if (max_id >= (1u << 22)) return TKZ_OK;
    }
    std::vector<const std::string*> keys;
    for (auto& k : t->keys)
        if (!k.empty() && k.size() <= 16) keys.push_back(&k);
    if (keys.empty()) return TKZ_OK;
    // Variants of the vocab keys that text carries as whole pretokens although they are no
    // vocab key themselves: the capitalised form (no normalizer: a lowercasing one never
    // leaves it) and, under Whitespace pretokenization (punctuation stays attached), the
    // key followed by one of TKZ_MEMO_PUNCT. Their BPE is computed like the keys' (same
    // kernel, one pretoken each), so a hit is still the kernel's own result.
#ifndef TKZ_MEMO_VARIANTS
#define TKZ_MEMO_VARIANTS 3  // bit 0: capitalised first letter, bit 1: + trailing punctuation
#endif
#ifndef TKZ_MEMO_PUNCT
#define TKZ_MEMO_PUNCT ",."
#endif
    std::vector<std::string> variants;
    {
        std::unordered_set<std::string> have;
        for (auto* k : keys) have.insert(*k);
        const bool cap = (TKZ_MEMO_VARIANTS & 1) && t->norm == 0;
        const bool punct = (TKZ_MEMO_VARIANTS & 2) && t->pretok == 1;
        auto add = [&](std::string v) {
            if (v.size() <= 16 && have.insert(v).second) variants.push_back(std::move(v));
        };
        for (size_t i = 0, n0 = keys.size(); i < n0; ++i) {
            const std::string& k = *keys[i];
            const bool up = cap && k[0] >= 'a' && k[0] <= 'z';
            std::string ck = k;
            if (up) { ck[0] = (char)(k[0] - 32); add(ck); }
            if (punct)
                for (const char* p = TKZ_MEMO_PUNCT; *p; ++p) {
                    add(k + *p);
                    if (up) add(ck + *p);
                }
        }
        for (auto& v : variants) keys.push_back(&v);
    }
    std::vector<uint64_t> off(keys.size() + 1, 0);
    std::string blob;
    for (size_t i = 0; i < keys.size(); ++i) { blob += *keys[i]; off[i + 1] = blob.size(); }
    const uint64_t total = blob.size();
    const size_t padded = (size_t)((total + 16 + 15) / 16 * 16);
    blob.resize(padded, '\0');
    const size_t n = keys.size();
    const size_t ws = tkz::workspace_bytes(total, n);
    uint8_t* db = nullptr; uint64_t* doff = nullptr; uint64_t* drow = nullptr; uint32_t* dids = nullptr;
    uint64_t* doffs = nullptr; void* dws = nullptr;
    auto cleanup = [&]() {
        for (void* p : {(void*)db, (void*)doff, (void*)drow, (void*)dids, (void*)doffs, dws}) if (p) hipFree(p);
    };
    if (hipMalloc((void**)&db, padded) != hipSuccess || hipMalloc((void**)&doff, (n + 1) * 8) != hipSuccess ||
        hipMalloc((void**)&drow, (n + 1) * 8) != hipSuccess || hipMalloc((void**)&dids, (total + 1) * 4) != hipSuccess ||
        hipMalloc((void**)&doffs, (total + 1) * 8) != hipSuccess || hipMalloc(&dws, ws) != hipSuccess) {
        cleanup();
        return fail(TKZ_ERR_OUT_OF_MEMORY, "device allocation failed (word memo)");
    }
    hipMemcpyAsync(db, blob.data(), padded, hipMemcpyHostToDevice, d.stream);
    hipMemcpyAsync(doff, off.data(), (n + 1) * 8, hipMemcpyHostToDevice, d.stream);
    hipMemsetAsync(d.d_status, 0, 4, d.stream);
    DevTables Tm = d.T;
    Tm.norm = 0;
    Tm.pretok = 0;
    Tm.memo = nullptr;
    Tm.memo8 = nullptr;
    Tm.seg = 0;  // (keys of <= 16 bytes: never long pretokens)
    hipError_t e = tkz::launch_encode(Tm, db, doff, n, total, drow, dids, doffs, dws, ws, d.d_status, d.stream,
                                      tkz::TimerSource{}, nullptr);
    std::vector<uint64_t> row(n + 1);
    std::vector<uint32_t> ids(total + 1);
    std::vector<uint64_t> offs(total + 1);
    if (e == hipSuccess) {
        hipMemcpyAsync(row.data(), drow, (n + 1) * 8, hipMemcpyDeviceToHost, d.stream);
        hipMemcpyAsync(ids.data(), dids, (total + 1) * 4, hipMemcpyDeviceToHost, d.stream);
        hipMemcpyAsync(offs.data(), doffs, (total + 1) * 8, hipMemcpyDeviceToHost, d.stream);
        e = hipStreamSynchronize(d.stream);
    }
    cleanup();
    if (e != hipSuccess) return fail(TKZ_ERR_DEVICE, std::string("word memo build failed: ") + hipGetErrorString(e));
    // keys of <= 8 bytes whose tokens fit a 16-B slot (memo8_pack): the 16-B table; keys of
    // 9..16 bytes with <= 3 tokens: the 32-B table; any other key is left to the model
    size_t cnt = 0, cnt8 = 0;
    for (size_t i = 0; i < n; ++i) {
        const uint64_t nt = row[i + 1] - row[i];
        if (keys[i]->size() <= 8 && !wide) ++cnt8;
        else if (nt <= 3) ++cnt;
    }
    // Load factor <= 1/8 (TKZ_MEMO_SCALE slots per key before the power-of-two round-up)
    // and linear probing WITHOUT wrap-around into a zero tail: the dispatch probe
    // (memo_probe) reads a 32-B window per round (2 slots of the 16-B table, 1 of the
    // 32-B one); at this load a wave of lookups rarely needs a second round. The tail
    // keeps >= 4 empty slots after the last used one. (Scale 8 measured 1-2 % faster in
    // k_encode than 4 with the 32-B window. With the key variants (capitalised, ","/"."
    // suffixed) a 32k vocab has ~100k keys: the two tables are ~16-32 MB, MALL-resident,
    // not L2-sized; tkz_get_memo_info reports the entries and bytes.)
    constexpr size_t PAD = 64;
#ifndef TKZ_MEMO_SCALE
#define TKZ_MEMO_SCALE 8
#endif
    uint32_t bits = pow2_bits(cnt * TKZ_MEMO_SCALE + 2), bits8 = pow2_bits(cnt8 * TKZ_MEMO_SCALE + 2);
    std::vector<uint4> tab, tab8;
    for (;;) {
        tab.assign((((size_t)1 << bits) + PAD) * 2, uint4{0, 0, 0, 0});
        tab8.assign(((size_t)1 << bits8) + PAD, uint4{0, 0, 0, 0});
        bool overflow = false;
        for (size_t i = 0; i < n && !overflow; ++i) {
            const uint64_t nt = row[i + 1] - row[i];
            const std::string& k = *keys[i];
            const uint32_t L = (uint32_t)k.size();
            uint64_t k0 = 0, k1 = 0;
            memcpy(&k0, k.data(), std::min<size_t>(8, k.size()));
            if (k.size() > 8) memcpy(&k1, k.data() + 8, k.size() - 8);
            if (nt > 3) continue;
            uint32_t tok[3] = {0, 0, 0};
            for (uint64_t j = 0; j < nt; ++j) {
                const uint64_t o = offs[row[i] + j];
                tok[j] = wide ? ids[row[i] + j] | ((uint32_t)(o & 0x1F) << 22) | ((uint32_t)((o >> 32) & 0x1F) << 27)
                              : ids[row[i] + j] | ((uint32_t)(o & 0xFF) << 16) | ((uint32_t)((o >> 32) & 0xFF) << 24);
            }
            if (L <= 8 && !wide) {
                uint32_t meta, w;
                if (!tkz::memo8_pack(L, (uint32_t)nt, tok, meta, w)) continue;
                size_t h = tkz::memo8_slot(k0, L, bits8);
                while (tab8[h].z != 0) ++h;
                if (h + 4 >= tab8.size()) { overflow = true; break; }
                tab8[h] = uint4{(uint32_t)k0, (uint32_t)(k0 >> 32), meta, w};
                continue;
            }
            size_t h = tkz::memo_slot(k0, k1, L, bits);
            while (tab[2 * h].z != 0) ++h;
            if (2 * (h + 2) >= tab.size()) { overflow = true; break; }
            tab[2 * h] = uint4{(uint32_t)k0, (uint32_t)(k0 >> 32), L | ((uint32_t)nt << 5), tok[0]};
            tab[2 * h + 1] = uint4{(uint32_t)k1, (uint32_t)(k1 >> 32), tok[1], tok[2]};
        }
        if (!overflow) break;
        ++bits;
        ++bits8;
    }
    const uint4* dm = nullptr;
    const uint4* dm8 = nullptr;
    int rc = upload(d, tab, &dm);
    if (rc || (rc = upload(d, tab8, &dm8))) return rc;
    d.memo = dm;
    d.memo_bits = bits;
    d.memo8 = dm8;
    d.memo8_bits = bits8;
    d.memo_entries = cnt + cnt8;
    d.memo_bytes = (tab.size() + tab8.size()) * sizeof(uint4);
    d.T.memo = dm;
    d.T.memo_bits = bits;
    d.T.memo8 = dm8;
    d.T.memo8_bits = bits8;
    return TKZ_OK;
}

template <class P>
int grow(P*& p, size_t& cap, size_t need_elems) {
    if (need_elems <= cap && p) return TKZ_OK;
    if (p) hipFree((void*)p);
    p = nullptr;
    size_t n = std::max<size_t>(need_elems + need_elems / 4, 64);
    if (hipMalloc((void**)&p, n * sizeof(P)) != hipSuccess) { cap = 0; return fail(TKZ_ERR_OUT_OF_MEMORY, "device allocation failed"); }
    cap = n;
    return TKZ_OK;
}

// kernel timers of the next encode pass (profiling on): one event set per pass
static tkz::KernelTimers* next_timers(void* ctx) {
    DeviceState& d = *(DeviceState*)ctx;
    if (d.n_timed >= d.timers.size()) {
        d.timers.emplace_back();
        for (auto& e : d.timers.back().ev) hipEventCreate(&e);
        d.timers.back().enabled = true;
    }
    return &d.timers[d.n_timed++];
}

int run_device(tkz_tokenizer* t, const uint8_t* d_bytes, const uint64_t* d_off, size_t n_docs, uint64_t total,
               uint64_t* d_row, uint32_t* d_ids, uint64_t* d_offs, void* d_ws, size_t ws_bytes, uint32_t* d_status,
               hipStream_t st, const tkz::DevTables* tables = nullptr) {
    DeviceState& d = t->dev;
    tkz::TimerSource ts;
    if (d.profile) { ts.fn = next_timers; ts.ctx = &d; }
    tkz::EncodeFail why = tkz::EncodeFail::None;
    hipError_t e = tkz::launch_encode(tables ? *tables : d.T, d_bytes, d_off, n_docs, total, d_row, d_ids, d_offs, d_ws,
                                      ws_bytes, d_status, st, ts, &why);
    if (why == tkz::EncodeFail::WorkspaceTooSmall)
        return fail(TKZ_ERR_INVALID_ARGUMENT, "workspace too small (< tkz_device_workspace_min)");
    if (why == tkz::EncodeFail::DocTooLarge)
        return fail(TKZ_ERR_INVALID_ARGUMENT, "a document is larger than the sub-batch this workspace supports");
    if (e != hipSuccess) return fail(TKZ_ERR_DEVICE, std::string("kernel launch failed: ") + hipGetErrorString(e));
    return TKZ_OK;
}

// Host-buffer batch encode into device outputs (staging owned by the tokenizer).
int encode_host_to_device(tkz_tokenizer* t, const uint8_t* bytes, const uint64_t* doc_off, size_t n_docs,
                          uint64_t* n_tokens) {
    int rc = ensure_device(t);
    if (rc) return rc;
    DeviceState& d = t->dev;
    const uint64_t total = n_docs ? doc_off[n_docs] : 0;
    const uint64_t base = n_docs ? doc_off[0] : 0;
    if (base != 0) return fail(TKZ_ERR_INVALID_ARGUMENT, "doc_off[0] must be 0");
    uint64_t max_doc = 0;
    for (size_t i = 0; i < n_docs; ++i) {
        if (doc_off[i + 1] < doc_off[i]) return fail(TKZ_ERR_INVALID_ARGUMENT, "doc_off must be non-decreasing");
        max_doc = std::max<uint64_t>(max_doc, doc_off[i + 1] - doc_off[i]);
    }
    const size_t padded = (size_t)((total + 16 + 15) / 16 * 16);
    if ((rc = grow(d.d_bytes, d.cap_bytes, padded)) || (rc = grow(d.d_off, d.cap_off, n_docs + 1)) ||
        (rc = grow(d.d_row, d.cap_row, n_docs + 1)) || (rc = grow(d.d_ids, d.cap_tok, total + 1)) ||
        (rc = grow(d.d_offs, d.cap_offs, total + 1)))
        return rc;
    // one-pass workspace when the device's free memory holds it (less a 2-GiB margin for
    // the other buffers and other processes on the device); else the largest that does,
    // but never less than a sub-batch holding the largest doc (a sub-batch starts at a
    // 512-B aligned base): launch_encode then runs doc-aligned sub-batches (as DeviceBatch
    // does on the device API). Only a device that cannot hold even that fails, with
    // TKZ_ERR_OUT_OF_MEMORY. d.d_ws follows every grow (null after a failed one: grow has
    // freed the old buffer).
    const int seg = tkz::seg_mode(d.T);
    const size_t ws = tkz::workspace_bytes(total, n_docs, seg);
    if (ws > d.cap_ws || !d.d_ws) {
        size_t fr = 0, tot = 0, lim = SIZE_MAX;
        if (hipMemGetInfo(&fr, &tot) == hipSuccess) {
            const size_t margin = (size_t)2 << 30;
            const size_t avail = fr + (d.d_ws ? d.cap_ws : 0);  // (the old workspace is freed first)
            lim = avail > margin ? avail - margin : 0;
        }
        const size_t need = tkz::workspace_bytes_sub(std::max<uint64_t>(max_doc + 512, TKZ_SUB_MIN), seg);
        uint8_t* wsp = (uint8_t*)d.d_ws;
        rc = TKZ_ERR_OUT_OF_MEMORY;
        if (ws / 4 * 5 <= lim) {  // (grow adds 1/4)
            rc = grow(wsp, d.cap_ws, ws);
            d.d_ws = wsp;
        }
        if (rc) {
            rc = grow(wsp, d.cap_ws, std::max(std::min(lim, ws / 4 * 5) / 5 * 4, need));
            d.d_ws = wsp;
            if (rc) return rc;
            g_last_error.clear();  // (the first attempt's message)
        }
    }
    hipStream_t st = d.stream;
    if (total) hipMemcpyAsync(d.d_bytes, bytes, total, hipMemcpyHostToDevice, st);
    hipMemsetAsync(d.d_bytes + total, 0, padded - total, st);
    hipMemcpyAsync(d.d_off, doc_off, (n_docs + 1) * 8, hipMemcpyHostToDevice, st);
    hipMemsetAsync(d.d_status, 0, 4, st);
    if ((rc = run_device(t, d.d_bytes, d.d_off, n_docs, total, d.d_row, d.d_ids, d.d_offs, d.d_ws, d.cap_ws, d.d_status,
                         st)))
        return rc;
    uint32_t status = 0;
    uint64_t nt = 0;
    hipMemcpyAsync(&status, d.d_status, 4, hipMemcpyDeviceToHost, st);
    hipMemcpyAsync(&nt, d.d_row + n_docs, 8, hipMemcpyDeviceToHost, st);
    hipError_t e = hipStreamSynchronize(st);
    if (e != hipSuccess) return fail(TKZ_ERR_DEVICE, std::string("device error: ") + hipGetErrorString(e));
    if (status == TKZ_ERR_MISSING_UNK_TOKEN) return fail(TKZ_ERR_MISSING_UNK_TOKEN, "MissingUnkToken");
    if (status) return fail((int)status, "device reported an error");
    *n_tokens = nt;
    return TKZ_OK;
}

// FastTokenizer batch (lib.zig:352-413) on the device. Workspace: clipped input copy |
// CSR row_ptr | CSR ids | CSR offsets | encode workspace.
struct FastWs {
    uint8_t* copy;
    uint64_t* row;
    uint32_t* ids;
    uint64_t* offs;
    void* enc;
};
static uint64_t al256(uint64_t x) { return (x + 255) / 256 * 256; }
size_t fast_workspace_bytes(uint64_t total, size_t n_docs, int seg = 0) {
    return (size_t)(al256(total + 32) + al256((n_docs + 1) * 8) + al256((total + 1) * 4) + al256((total + 1) * 8) +
                    tkz::workspace_bytes(total, n_docs, seg) + 256);
}
static FastWs fast_layout(void* ws, uint64_t total, size_t n_docs) {
    uint8_t* p = (uint8_t*)(((uintptr_t)ws + 255) / 256 * 256);
    FastWs f;
    f.copy = p; p += al256(total + 32);
    f.row = (uint64_t*)p; p += al256((n_docs + 1) * 8);
    f.ids = (uint32_t*)p; p += al256((total + 1) * 4);
    f.offs = (uint64_t*)p; p += al256((total + 1) * 8);
    f.enc = p;
    return f;
}

int run_fast_device(tkz_tokenizer* t, const uint8_t* d_bytes, const uint64_t* d_off, size_t n_docs, uint64_t total,
                    uint64_t max_doc, const tkz_fast_options& o, uint32_t* d_len, uint32_t* d_ids, uint64_t* d_offs,
                    uint32_t* d_attn, void* d_ws, size_t ws_bytes, uint32_t* d_status, hipStream_t st) {
    DeviceState& d = t->dev;
    const uint32_t max_pretokens = o.max_sequence_length / 4;  // arena.zig:192
    const uint32_t cap = o.max_tokens;
    const uint32_t keep = d.T.pretok == 0 && max_pretokens == 0 ? 0 : cap;  // the whole-input span is dropped too
    FastWs f = fast_layout(d_ws, total, n_docs);
    const uint8_t* in = d_bytes;
    if (d.T.pretok != 0 && n_docs && (max_doc == 0 || max_doc > max_pretokens)) {
        const uint64_t rd = (total + 15) / 16 * 16;  // readable extent of the caller's buffer
        if (rd) hipMemcpyAsync(f.copy, d_bytes, rd, hipMemcpyDeviceToDevice, st);
        hipMemsetAsync(f.copy + rd, 0, 16, st);
        hipError_t e = tkz::launch_span_clip(d.T.pretok, max_pretokens, d_off, n_docs, f.copy, st);
        if (e != hipSuccess) return fail(TKZ_ERR_DEVICE, std::string("clip launch failed: ") + hipGetErrorString(e));
        in = f.copy;
    }
    tkz::DevTables T = d.T;
    T.unk_drop = 1;  // WordPiece.tokenizeFast (wordpiece.zig:241,297)
    // the encode workspace is what is left of the caller's: launch_encode picks the
    // segmented arrays, the plain layout or sub-batches by its size
    const size_t used = (size_t)((uint8_t*)f.enc - (uint8_t*)d_ws);
    int rc = run_device(t, in, d_off, n_docs, total, f.row, f.ids, f.offs, f.enc, ws_bytes > used ? ws_bytes - used : 0,
                        d_status, st, &T);
    if (rc) return rc;
    hipError_t e = tkz::launch_span_fill(f.row, n_docs, f.ids, f.offs, cap, keep, d_len, d_ids, d_offs, d_attn, st);
    if (e != hipSuccess) return fail(TKZ_ERR_DEVICE, std::string("span launch failed: ") + hipGetErrorString(e));
    return TKZ_OK;
}

// Device tables for the batched decode: per id {pool offset, length | special bit} over
// every model and added id, and the model-vocab string pool (lib.zig:163-189).
int ensure_decode(tkz_tokenizer* t) {
    int rc = ensure_device(t);
    if (rc) return rc;
    DeviceState& d = t->dev;
    if (d.dec_version == t->added_version) return TKZ_OK;
    uint64_t n_ent = 0;
    for (auto& kv : t->vocab_r) n_ent = std::max<uint64_t>(n_ent, (uint64_t)kv.first + 1);
    for (auto& kv : t->added_i2t) n_ent = std::max<uint64_t>(n_ent, (uint64_t)kv.first + 1);
    if (n_ent > (1ull << 28)) return fail(TKZ_ERR_INVALID_ARGUMENT, "token ids too sparse for the device decode table");
    std::vector<uint2> ent((size_t)std::max<uint64_t>(n_ent, 1), uint2{0, 0});
    std::vector<uint8_t> pool;
    for (auto& kv : t->vocab_r) {
        ent[kv.first] = uint2{(uint32_t)pool.size(), (uint32_t)kv.second->size()};
        pool.insert(pool.end(), kv.second->begin(), kv.second->end());
    }
    for (auto& kv : t->added_i2t)
        if (t->special.count(kv.second)) ent[kv.first].y |= 0x80000000u;
    if (pool.empty()) pool.push_back(0);
    const uint2* de; const uint8_t* dp;
    if ((rc = upload(d, ent, &de)) || (rc = upload(d, pool, &dp))) return rc;
    d.DT.ent = de;
    d.DT.n_ent = (uint32_t)n_ent;
    d.DT.pool = dp;
    d.DT.decoder = t->decoder;
    d.dec_version = t->added_version;
    return TKZ_OK;
}

uint64_t decode_bound(const tkz_tokenizer* t, uint64_t n_tokens) {
    size_t mx = 1;
    for (auto& k : t->keys) mx = std::max(mx, k.size());
    return n_tokens * (uint64_t)mx + 16;
}

// An encode-only copy of t bound to `device`: the host images of the device tables and the
// settings that shape a batch (memo, dedup, host pipeline, truncation / padding). Not the
// vocab maps: a replica only runs tkz_encode_batch.
tkz_tokenizer* clone_for_encode(const tkz_tokenizer* t, int device) {
    tkz_tokenizer* r = new (std::nothrow) tkz_tokenizer();
    if (!r) return nullptr;
    r->model = t->model; r->norm = t->norm; r->pretok = t->pretok; r->decoder = t->decoder; r->has_pp = t->has_pp;
    r->keys = t->keys;  // the word memo is built from the vocab keys
    r->prefix = t->prefix;
    r->pp = t->pp; r->pad_token = t->pad_token;
    r->compact = t->compact; r->bpe_unk = t->bpe_unk; r->wp_unk = t->wp_unk; r->max_key = t->max_key;
    r->byte_id = t->byte_id;
    r->cp_tab = t->cp_tab; r->cp_bits = t->cp_bits;
    r->mtab_c = t->mtab_c; r->mtab_w = t->mtab_w; r->m_bits = t->m_bits;
    r->wp_tab = t->wp_tab; r->wp_bits = t->wp_bits;
    r->wps_tab = t->wps_tab; r->wps_bits = t->wps_bits;
    r->wp_pool = t->wp_pool;
    r->r2id = t->r2id;
    r->mtab_m = t->mtab_m; r->mm_bits = t->mm_bits;
    r->seg_over = t->seg_over; r->seg_over_bits = t->seg_over_bits;
    r->hostT = t->hostT;
    r->memo_on = t->memo_on; r->dedup_mode = t->dedup_mode; r->host_chunk = t->host_chunk; r->n_cp = t->n_cp;
    r->merges_ordered = t->merges_ordered; r->seg_want = t->seg_want; r->hot_want = t->hot_want;
    r->want_device = device;
    return r;
}

// first doc of each of k parts of docs [0, n) with about equal bytes (cut[0] = 0, cut[k] = n)
std::vector<size_t> byte_balanced_cuts(const uint64_t* doc_off, size_t n, size_t k) {
    std::vector<size_t> cut(k + 1, 0);
    cut[k] = n;
    const uint64_t base = doc_off[0], total = doc_off[n] - base;
    for (size_t j = 1; j < k; ++j) {
        const uint64_t target = base + (uint64_t)((unsigned __int128)total * j / k);
        size_t c = (size_t)(std::lower_bound(doc_off, doc_off + n + 1, target) - doc_off);
        cut[j] = std::min(std::max(c, cut[j - 1]), n);
    }
    return cut;
}

void fill_stats(const uint64_t* h, tkz_batch_stats* out) {
    out->pretokens = h[2];
    out->memo_hits = h[3];
    out->deferred = h[16];
    out->deferred_model = h[17];
    out->sub_batches = h[18];
    out->long_words = h[25];
    out->long_segmented = h[29];
    out->long_fallback_bytes = h[30];
    out->seg_bound_errors = tkz::seg_bound_errors();
}

}  // namespace

extern "C" {

const char* tkz_last_error(void) { return g_last_error.c_str(); }

int tkz_create_from_json(const char* js, size_t n, tkz_tokenizer** out) {
    if (!js || !out) return fail(TKZ_ERR_INVALID_ARGUMENT, "null argument");
    *out = nullptr;
    tkz_tokenizer* t = new (std::nothrow) tkz_tokenizer();
    if (!t) return fail(TKZ_ERR_OUT_OF_MEMORY, "out of memory");
    int rc;
    try {
        rc = load(t, js, n);
    } catch (const std::bad_alloc&) {
        rc = fail(TKZ_ERR_OUT_OF_MEMORY, "out of memory");
    }
    if (rc) { delete t; return rc; }
    *out = t;
    return TKZ_OK;
}

void tkz_opts_default(tkz_opts* o) {
    if (!o) return;
    o->device = -1;
    o->word_memo = 1;
    o->dedup = -1;
    o->host_chunk = 32ull << 20;
}

int tkz_create_from_json_opts(const char* js, size_t n, const tkz_opts* opts, tkz_tokenizer** out) {
    int rc = tkz_create_from_json(js, n, out);
    if (rc || !opts) return rc;
    tkz_tokenizer* t = *out;
    if (opts->device < -1) { tkz_destroy(t); *out = nullptr; return fail(TKZ_ERR_INVALID_ARGUMENT, "tkz_opts.device < -1"); }
    t->want_device = opts->device;
    t->memo_on = opts->word_memo != 0;
    t->dedup_mode = opts->dedup < 0 ? -1 : (opts->dedup != 0);
    t->host_chunk = opts->host_chunk == 0 ? 0 : std::max<uint64_t>(opts->host_chunk, TKZ_SUB_MIN);
    return TKZ_OK;
}

int tkz_create_from_file(const char* path, tkz_tokenizer** out) {
    if (!path || !out) return fail(TKZ_ERR_INVALID_ARGUMENT, "null argument");
    FILE* f = fopen(path, "rb");
    if (!f) return fail(TKZ_ERR_FILE_NOT_FOUND, std::string("cannot open ") + path);
    std::string buf;
    char tmp[1 << 16];
    size_t r;
    while ((r = fread(tmp, 1, sizeof tmp, f)) > 0) {
        buf.append(tmp, r);
        if (buf.size() > 100ull * 1024 * 1024) { fclose(f); return fail(TKZ_ERR_FILE_TOO_BIG, "file > 100 MiB"); }
    }
    fclose(f);
    return tkz_create_from_json(buf.data(), buf.size(), out);
}

void tkz_destroy(tkz_tokenizer* t) {
    if (!t) return;
    for (auto& r : t->replicas) tkz_destroy(r.second);
    DeviceState& d = t->dev;
    if (d.ready) {
        hipSetDevice(d.device);
        hipStreamSynchronize(d.stream);
        for (void* p : d.allocs) hipFree(p);
        if (d.hot_alloc) hipFree(d.hot_alloc);
        for (void* p : {(void*)d.d_bytes, (void*)d.d_off, (void*)d.d_row, (void*)d.d_ids, (void*)d.d_offs, d.d_ws,
                        (void*)d.d_status, (void*)d.d_dec_ids, (void*)d.d_dec_row, (void*)d.d_dec_out,
                        (void*)d.d_dec_off, (void*)d.d_dec_ws, (void*)d.d_row2, (void*)d.d_ids2, (void*)d.d_offs2,
                        (void*)d.d_masks, (void*)d.d_pad_ws, (void*)d.d_fast_ws, (void*)d.d_span,
                        (void*)d.d_span_offs})
            if (p) hipFree(p);
        for (auto& tm : d.timers) for (auto& e : tm.ev) if (e) hipEventDestroy(e);
        for (hipEvent_t e : d.chunk_ev) hipEventDestroy(e);
        for (hipEvent_t e : d.hp_ev) hipEventDestroy(e);
        if (d.h_cnt) hipHostFree(d.h_cnt);
        if (d.d2h) { hipStreamSynchronize(d.d2h); hipStreamDestroy(d.d2h); }
        hipStreamDestroy(d.stream);
    }
    delete t;
}

int tkz_get_info(const tkz_tokenizer* t, tkz_info* o) {
    if (!t || !o) return fail(TKZ_ERR_INVALID_ARGUMENT, "null argument");
    o->model = t->model; o->normalizer = t->norm; o->pre_tokenizer = t->pretok; o->decoder = t->decoder;
    o->has_post_processor = t->has_pp;
    o->model_vocab_size = t->vocab.size(); o->added_vocab_size = t->added_t2i.size();
    o->n_merges = t->n_accepted;
    o->unk_id = t->model == 1 ? t->bpe_unk : t->wp_unk;
    o->max_input_chars_per_word = t->max_chars;
    o->compact_tables = t->compact ? 1 : 0;
    o->merges_ordered = t->model == 1 && t->merges_ordered ? 1 : 0;
    o->long_segments = tkz::seg_mode(t->hostT) != 0 ? 1 : 0;
    return TKZ_OK;
}

int tkz_get_memo_info(const tkz_tokenizer* t, uint64_t* entries, uint64_t* table_bytes) {
    if (!t || !entries || !table_bytes) return fail(TKZ_ERR_INVALID_ARGUMENT, "null argument");
    tkz_memo_info m;
    tkz_get_memo_info_ext(t, &m);
    *entries = m.word_entries;
    *table_bytes = m.word_bytes + m.seg_bytes + m.hot_bitmap_bytes;
    return TKZ_OK;
}

int tkz_get_memo_info_ext(const tkz_tokenizer* t, tkz_memo_info* m) {
    if (!t || !m) return fail(TKZ_ERR_INVALID_ARGUMENT, "null argument");
    const DeviceState& d = t->dev;
    memset(m, 0, sizeof(*m));
    if (!d.ready) return TKZ_OK;
    if (d.T.memo) { m->word_entries = d.memo_entries; m->word_bytes = d.memo_bytes; }
    if (d.T.smemo) { m->seg_entries = d.smemo_entries; m->seg_bytes = d.smemo_bytes; }
    if (d.T.hot_bits) {
        m->hot_keys = d.hot_k;
        m->hot_bitmap_bytes = d.hot_bytes;
        m->hot_build_ms = d.hot_build_ms;
    }
    return TKZ_OK;
}

int tkz_set_hot_pairs(tkz_tokenizer* t, int64_t max_keys) {
    if (!t) return fail(TKZ_ERR_INVALID_ARGUMENT, "null");
    std::lock_guard<std::mutex> g(t->mu);
    t->hot_want = max_keys < 0 ? -1 : max_keys;
    if (!t->dev.ready || !t->memo_on || !t->dev.smemo) return TKZ_OK;  // (applies when the memo is built)
    hipSetDevice(t->dev.device);
    return build_hot(t);
}

int tkz_device_available(void) {
    int count = 0;
    return (hipGetDeviceCount(&count) == hipSuccess && count > 0) ? 1 : 0;
}

int tkz_set_dedup(tkz_tokenizer* t, int mode) {
    if (!t) return fail(TKZ_ERR_INVALID_ARGUMENT, "null");
    std::lock_guard<std::mutex> g(t->mu);
    t->dedup_mode = mode < 0 ? -1 : (mode != 0);
    apply_dedup(t);
    return TKZ_OK;
}

int tkz_set_host_pipeline(tkz_tokenizer* t, size_t chunk_bytes) {
    if (!t) return fail(TKZ_ERR_INVALID_ARGUMENT, "null");
    std::lock_guard<std::mutex> g(t->mu);
    // every chunk costs a full encode launch sequence: chunks below 1 MiB are clamped up
    t->host_chunk = chunk_bytes == 0 ? 0 : std::max<uint64_t>(chunk_bytes, TKZ_SUB_MIN);
    return TKZ_OK;
}

int tkz_set_word_memo(tkz_tokenizer* t, int on) {
    if (!t) return fail(TKZ_ERR_INVALID_ARGUMENT, "null");
    std::lock_guard<std::mutex> g(t->mu);
    t->memo_on = on != 0;
    if (!t->dev.ready) return TKZ_OK;
    if (!t->memo_on) { t->dev.T.memo = nullptr; t->dev.T.memo8 = nullptr; t->dev.T.smemo = nullptr; t->dev.T.hot_bits = nullptr; t->dev.T.hot_k = 0; return TKZ_OK; }
    return build_memo(t);
}

int tkz_set_long_segments(tkz_tokenizer* t, int on) {
    if (!t) return fail(TKZ_ERR_INVALID_ARGUMENT, "null");
    std::lock_guard<std::mutex> g(t->mu);
    t->seg_want = on != 0;
    t->hostT.seg = t->seg_want && t->merges_ordered;  // (an unordered merge table: never, merges_ordered)
    t->dev.T.seg = t->hostT.seg;
    return TKZ_OK;
}

int tkz_set_device(int device) {
    hipError_t e = hipSetDevice(device);
    return e == hipSuccess ? TKZ_OK : fail(TKZ_ERR_DEVICE, hipGetErrorString(e));
}

size_t tkz_device_workspace_size(const tkz_tokenizer* t, uint64_t total_bytes, size_t n_docs) {
    return tkz::workspace_bytes(total_bytes, n_docs, (t ? tkz::seg_mode(t->hostT) : 0));
}

size_t tkz_device_workspace_min(const tkz_tokenizer*) { return tkz::workspace_bytes_sub(TKZ_SUB_MIN); }

size_t tkz_device_workspace_size_sub(const tkz_tokenizer* t, uint64_t sub_batch_bytes) {
    return tkz::workspace_bytes_sub(std::max<uint64_t>(sub_batch_bytes, TKZ_SUB_MIN), (t ? tkz::seg_mode(t->hostT) : 0));
}

int tkz_device_batch_stats(const tkz_tokenizer* t, const void* d_ws, tkz_batch_stats* out) {
    if (!t || !out) return fail(TKZ_ERR_INVALID_ARGUMENT, "null argument");
    const void* ws = d_ws ? d_ws : t->dev.d_ws;
    if (!ws) return fail(TKZ_ERR_INVALID_ARGUMENT, "no workspace");
    uint64_t h[32];
    // the encode streams are non-blocking (a null-stream copy does not wait for them):
    // wait for all work of the tokenizer's device (which owns the workspace; the calling
    // thread may have another device current), so the statistics are those of the last batch
    int cur = -1;
    hipGetDevice(&cur);
    const int dev = t->dev.ready ? t->dev.device : cur;
    if (dev != cur) hipSetDevice(dev);
    hipError_t e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(h, (const uint8_t*)ws + tkz::stats_offset(), sizeof h, hipMemcpyDeviceToHost);
    if (dev != cur) hipSetDevice(cur);
    if (e != hipSuccess) return fail(TKZ_ERR_DEVICE, hipGetErrorString(e));
    fill_stats(h, out);
    return TKZ_OK;
}

int tkz_device_batch_stats_stream(const tkz_tokenizer* t, const void* d_ws, void* stream, tkz_batch_stats* out) {
    if (!t || !out) return fail(TKZ_ERR_INVALID_ARGUMENT, "null argument");
    const void* ws = d_ws ? d_ws : t->dev.d_ws;
    if (!ws) return fail(TKZ_ERR_INVALID_ARGUMENT, "no workspace");
    if (!stream && !t->dev.ready) return fail(TKZ_ERR_INVALID_ARGUMENT, "no stream");
    hipStream_t st = stream ? (hipStream_t)stream : t->dev.stream;
    uint64_t h[32];
    hipError_t e = hipMemcpyAsync(h, (const uint8_t*)ws + tkz::stats_offset(), sizeof h, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return fail(TKZ_ERR_DEVICE, hipGetErrorString(e));
    fill_stats(h, out);
    return TKZ_OK;
}

int tkz_encode_batch_device(tkz_tokenizer* t, const uint8_t* d_bytes, const uint64_t* d_doc_off, size_t n_docs,
                            uint64_t total_bytes, uint64_t* d_row_ptr, uint32_t* d_ids, tkz_offset* d_offsets,
                            void* d_ws, size_t ws_bytes, uint32_t* d_status, void* stream) {
    if (!t || !d_doc_off || !d_row_ptr || !d_ws || !d_status || (n_docs && (!d_ids || !d_offsets || !d_bytes)))
        return fail(TKZ_ERR_INVALID_ARGUMENT, "null argument");
    if (ws_bytes < tkz::workspace_bytes(total_bytes, n_docs) && ws_bytes < tkz::workspace_bytes_sub(TKZ_SUB_MIN))
        return fail(TKZ_ERR_INVALID_ARGUMENT, "workspace too small");
    std::lock_guard<std::mutex> g(t->mu);
    int rc = ensure_device(t);
    if (rc) return rc;
    hipStream_t st = stream ? (hipStream_t)stream : t->dev.stream;
    return run_device(t, d_bytes, d_doc_off, n_docs, total_bytes, d_row_ptr, d_ids, (uint64_t*)d_offsets, d_ws,
                      ws_bytes, d_status, st);
}

// tkz_encode_batch without truncation / padding, with the PCIe copies overlapped: the docs
// are cut into chunks of about t->host_chunk input bytes; chunk k's input copy and encode
// run while the CSR slice of chunk k-1 goes to the host on a second stream (the copies run
// in opposite directions). On the device each chunk is a batch of its own: its bytes at a
// 256-B aligned offset db[k] of the staging buffer (zero-padded as a whole batch is), its
// doc offsets rebased to 0, its outputs at token offset db[k] (a chunk has no more tokens
// than bytes) and its row_ptr chunk-relative (the host adds the chunk's token base). The host arrays must exist before the
// total is known: they are sized from the previous batch's tokens per byte + 1/8; a
// batch that outgrows them moves to exact-size arrays once every chunk is encoded.
static int encode_batch_pipelined(tkz_tokenizer* t, const uint8_t* bytes, const uint64_t* doc_off, size_t n_docs,
                                  tkz_batch* out) {
    int rc = ensure_device(t);
    if (rc) return rc;
    DeviceState& d = t->dev;
    const uint64_t total = doc_off[n_docs];
    if (doc_off[0] != 0) return fail(TKZ_ERR_INVALID_ARGUMENT, "doc_off[0] must be 0");
    for (size_t i = 0; i < n_docs; ++i)
        if (doc_off[i + 1] < doc_off[i]) return fail(TKZ_ERR_INVALID_ARGUMENT, "doc_off must be non-decreasing");
    std::vector<size_t> cut{0};
    for (size_t i = 1; i <= n_docs; ++i)
        if (i == n_docs || doc_off[i] - doc_off[cut.back()] >= t->host_chunk) cut.push_back(i);
    const size_t K = cut.size() - 1;
    std::vector<uint64_t> db(K + 1, 0);  // device byte (and token) offset of each chunk
    size_t ws_max = 0;
    for (size_t k = 0; k < K; ++k) {
        const uint64_t len = doc_off[cut[k + 1]] - doc_off[cut[k]];
        db[k + 1] = (db[k] + len + 32 + 255) / 256 * 256;
        ws_max = std::max(ws_max, tkz::workspace_bytes(len, cut[k + 1] - cut[k], tkz::seg_mode(d.T)));
    }
    // rebased doc offsets, chunk k's n_k + 1 entries from index cut[k] + k
    d.h_off.resize(n_docs + K);
    for (size_t k = 0; k < K; ++k)
        for (size_t i = cut[k]; i <= cut[k + 1]; ++i) d.h_off[i + k] = doc_off[i] - doc_off[cut[k]];
    if ((rc = grow(d.d_bytes, d.cap_bytes, db[K])) || (rc = grow(d.d_off, d.cap_off, n_docs + K)) ||
        (rc = grow(d.d_row, d.cap_row, n_docs + 1)) || (rc = grow(d.d_ids, d.cap_tok, db[K])) ||
        (rc = grow(d.d_offs, d.cap_offs, db[K])))
        return rc;
    uint8_t* wsp = (uint8_t*)d.d_ws;
    if ((rc = grow(wsp, d.cap_ws, ws_max))) return rc;
    d.d_ws = wsp;
    if (!d.d2h && hipStreamCreateWithFlags(&d.d2h, hipStreamNonBlocking) != hipSuccess)
        return fail(TKZ_ERR_DEVICE, "hipStreamCreate failed");
    while (d.chunk_ev.size() < K) {
        hipEvent_t e;
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return fail(TKZ_ERR_DEVICE, "hipEventCreate failed");
        d.chunk_ev.push_back(e);
    }
    if (d.cap_h_cnt < K) {
        if (d.h_cnt) hipHostFree(d.h_cnt);
        d.h_cnt = nullptr;
        d.cap_h_cnt = 0;
        if (hipHostMalloc((void**)&d.h_cnt, K * 8, hipHostMallocDefault) != hipSuccess)
            return fail(TKZ_ERR_OUT_OF_MEMORY, "hipHostMalloc failed");
        d.cap_h_cnt = K;
    }
    const bool prof = d.profile;
    using clk = std::chrono::steady_clock;
    const auto ms_since = [](clk::time_point a) { return std::chrono::duration<double, std::milli>(clk::now() - a).count(); };
    const auto t_call = clk::now();
    if (prof) {
        while (d.hp_ev.size() < 5 * K) {
            hipEvent_t e;
            if (hipEventCreate(&e) != hipSuccess) return fail(TKZ_ERR_DEVICE, "hipEventCreate failed");
            d.hp_ev.push_back(e);
        }
    }
    auto rec = [&](size_t k, int j, hipStream_t s) { if (prof) hipEventRecord(d.hp_ev[5 * k + j], s); };
    uint64_t cap = std::min<uint64_t>(total + 1, (uint64_t)((double)total * t->host_ratio * 1.125) + 4096);
    out->n_docs = n_docs;
    auto t_alloc = clk::now();
    out->row_ptr = (uint64_t*)out_alloc((n_docs + 1) * 8);
    bool pin_ids = false, pin_offs = false;
    out->ids = (uint32_t*)out_alloc(cap * 4, &pin_ids);
    out->offsets = (tkz_offset*)out_alloc(cap * 8, &pin_offs);
    double alloc_ms = ms_since(t_alloc), wait_ms = 0;
    if (!out->row_ptr || !out->ids || !out->offsets) {
        tkz_batch_free(out);
        return fail(TKZ_ERR_OUT_OF_MEMORY, "out of memory");
    }
    hipStream_t st = d.stream;
    hipMemsetAsync(d.d_status, 0, 4, st);
    hipMemcpyAsync(d.d_off, d.h_off.data(), (n_docs + K) * 8, hipMemcpyHostToDevice, st);
    std::vector<uint64_t> tb(K + 1, 0);  // token base of each chunk
    size_t sent = 0;                     // chunks whose CSR slices are queued on d2h
    bool ok = true;
    auto queue_slice = [&](size_t k) {
        const uint64_t b = db[k], nk = tb[k + 1] - tb[k];
        rec(k, 3, d.d2h);
        hipMemcpyAsync(out->row_ptr + cut[k], d.d_row + cut[k], (cut[k + 1] - cut[k]) * 8, hipMemcpyDeviceToHost, d.d2h);
        if (nk) {
            hipMemcpyAsync(out->ids + tb[k], d.d_ids + b, nk * 4, hipMemcpyDeviceToHost, d.d2h);
            hipMemcpyAsync(out->offsets + tb[k], d.d_offs + b, nk * 8, hipMemcpyDeviceToHost, d.d2h);
        }
        rec(k, 4, d.d2h);
    };
    // The output side runs on a host thread of its own: it waits for chunk k's token count
    // (its event), places the chunk's CSR slice at the running token base and queues it on
    // the d2h stream, while this thread keeps queueing inputs and encodes (a pageable input
    // copy blocks its caller until staged; waiting for counts here as well serialised every
    // chunk's input copy behind the previous chunk's encode).
    std::mutex mu;
    std::condition_variable cv;
    size_t recorded = 0;  // chunks whose event is recorded (mu)
    bool abort_out = false;
    std::thread out_thr([&] {
        hipSetDevice(d.device);
        for (size_t k = 0; k < K; ++k) {
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return recorded > k || abort_out; });
                if (recorded <= k) return;
            }
            const auto t_w = clk::now();
            const bool ok_k = hipEventSynchronize(d.chunk_ev[k]) == hipSuccess;
            wait_ms += ms_since(t_w);
            if (!ok_k) { ok = false; return; }
            tb[k + 1] = tb[k] + d.h_cnt[k];
            if (sent == k && tb[k + 1] <= cap) {
                hipStreamWaitEvent(d.d2h, d.chunk_ev[k], 0);
                queue_slice(k);
                sent = k + 1;
            }
        }
    });
    auto stop_out = [&] {
        { std::lock_guard<std::mutex> lk(mu); abort_out = true; }
        cv.notify_all();
        out_thr.join();
    };
    for (size_t k = 0; k < K; ++k) {
        const uint64_t b = db[k], len = doc_off[cut[k + 1]] - doc_off[cut[k]];
        rec(k, 0, st);
        if (len) hipMemcpyAsync(d.d_bytes + b, bytes + doc_off[cut[k]], len, hipMemcpyHostToDevice, st);
        rec(k, 1, st);
        hipMemsetAsync(d.d_bytes + b + len, 0, (len + 16 + 15) / 16 * 16 - len, st);
        if ((rc = run_device(t, d.d_bytes + b, d.d_off + cut[k] + k, cut[k + 1] - cut[k], len, d.d_row + cut[k],
                             d.d_ids + b, d.d_offs + b, d.d_ws, d.cap_ws, d.d_status, st))) {
            stop_out();
            hipStreamSynchronize(st);
            hipStreamSynchronize(d.d2h);
            tkz_batch_free(out);
            return rc;
        }
        rec(k, 2, st);
        hipMemcpyAsync(&d.h_cnt[k], d.d_row + cut[k + 1], 8, hipMemcpyDeviceToHost, st);
        hipEventRecord(d.chunk_ev[k], st);
        { std::lock_guard<std::mutex> lk(mu); recorded = k + 1; }
        cv.notify_all();
    }
    out_thr.join();
    uint32_t status = 0;
    hipMemcpyAsync(&status, d.d_status, 4, hipMemcpyDeviceToHost, st);
    hipError_t e1 = hipStreamSynchronize(st);
    hipError_t e2 = hipStreamSynchronize(d.d2h);
    if (!ok || e1 != hipSuccess || e2 != hipSuccess) {
        tkz_batch_free(out);
        return fail(TKZ_ERR_DEVICE, std::string("device error: ") + hipGetErrorString(e1 != hipSuccess ? e1 : e2));
    }
    if (status) {
        tkz_batch_free(out);
        if (status == TKZ_ERR_MISSING_UNK_TOKEN) return fail(TKZ_ERR_MISSING_UNK_TOKEN, "MissingUnkToken");
        return fail((int)status, "device reported an error");
    }
    const uint64_t nt = tb[K];
    if (sent < K) {  // outgrew the estimate: exact-size arrays, then the remaining slices
        uint32_t* ids = (uint32_t*)out_alloc(std::max<uint64_t>(nt, 1) * 4, &pin_ids);
        tkz_offset* offs = (tkz_offset*)out_alloc(std::max<uint64_t>(nt, 1) * 8, &pin_offs);
        if (!ids || !offs) {
            out_free(ids);
            out_free(offs);
            tkz_batch_free(out);
            return fail(TKZ_ERR_OUT_OF_MEMORY, "out of memory");
        }
        t_alloc = clk::now();
        memcpy(ids, out->ids, tb[sent] * 4);
        memcpy(offs, out->offsets, tb[sent] * 8);
        alloc_ms += ms_since(t_alloc);
        out_free(out->ids);
        out_free(out->offsets);
        out->ids = ids;
        out->offsets = offs;
        for (size_t k = sent; k < K; ++k) queue_slice(k);
        if ((e2 = hipStreamSynchronize(d.d2h)) != hipSuccess) {
            tkz_batch_free(out);
            return fail(TKZ_ERR_DEVICE, std::string("device error: ") + hipGetErrorString(e2));
        }
    }
    const auto t_fix = clk::now();
    for (size_t k = 1; k < K; ++k)
        for (size_t i = cut[k]; i < cut[k + 1]; ++i) out->row_ptr[i] += tb[k];
    out->row_ptr[n_docs] = nt;
    out->n_tokens = nt;
    if (total) t->host_ratio = (double)nt / (double)total;
    if (prof) {  // every event has completed (both streams synchronized above)
        double* hp = d.hp;
        const double fix_ms = ms_since(t_fix);
        auto el = [&](size_t ka, int ja, size_t kb, int jb) {
            float v = 0;
            return hipEventElapsedTime(&v, d.hp_ev[5 * ka + ja], d.hp_ev[5 * kb + jb]) == hipSuccess ? (double)v : 0.0;
        };
        for (size_t k = 0; k < K; ++k) {
            hp[HP_H2D] += el(k, 0, k, 1);
            hp[HP_ENC] += el(k, 1, k, 2);
            hp[HP_D2H] += el(k, 3, k, 4);
        }
        hp[HP_H2D_SPAN] += el(0, 0, K - 1, 1);
        hp[HP_ENC_SPAN] += el(0, 1, K - 1, 2);
        hp[HP_D2H_SPAN] += el(0, 3, K - 1, 4);
        hp[HP_FIRST_ENC] += el(0, 0, 0, 2);    // first chunk in and encoded: nothing to overlap yet
        hp[HP_LAST_D2H] += el(K - 1, 2, K - 1, 4);  // last chunk's count read, slice out: the tail
        hp[HP_CALLS] += 1;
        hp[HP_CHUNKS] += (double)K;
        hp[HP_BYTES_IN] += (double)total;
        hp[HP_BYTES_OUT] += (double)((n_docs + 1) * 8 + nt * 12);
        hp[HP_ALLOC] += alloc_ms;
        hp[HP_WAIT] += wait_ms;
        hp[HP_FIXUP] += fix_ms;
        hp[HP_OUT_PAGEABLE] += (double)(!pin_ids) + (double)(!pin_offs);
        hp[HP_WALL] += ms_since(t_call);
    }
    return TKZ_OK;
}

int tkz_encode_batch(tkz_tokenizer* t, const uint8_t* bytes, const uint64_t* doc_off, size_t n_docs, tkz_batch* out) {
    if (!t || !doc_off || !out || (n_docs && !bytes && doc_off[n_docs] > 0)) return fail(TKZ_ERR_INVALID_ARGUMENT, "null argument");
    memset(out, 0, sizeof *out);
    std::lock_guard<std::mutex> g(t->mu);
    const bool padded = t->pp.truncate || t->pp.pad;
    if (!padded && n_docs && t->host_chunk && t->host_ratio > 0 && doc_off[n_docs] >= 2 * t->host_chunk)
        return encode_batch_pipelined(t, bytes, doc_off, n_docs, out);
    uint64_t nt = 0;
    int rc = encode_host_to_device(t, bytes, doc_off, n_docs, &nt);
    if (rc) return rc;
    if (!padded && n_docs && doc_off[n_docs]) t->host_ratio = (double)nt / (double)doc_off[n_docs];
    DeviceState& d = t->dev;
    const uint64_t* src_row = d.d_row;
    const uint32_t* src_ids = d.d_ids;
    const uint64_t* src_offs = d.d_offs;
    const uint64_t cap = nt + (t->pp.pad ? (uint64_t)n_docs * t->pp.length : 0) + 1;  // padded tokens bound
    if (padded) {  // Tokenizer.encode steps 6-7 (lib.zig:149-157) on the device
        if ((rc = grow(d.d_row2, d.cap_row2, n_docs + 1)) || (rc = grow(d.d_ids2, d.cap_ids2, cap)) ||
            (rc = grow(d.d_offs2, d.cap_offs2, cap)) || (rc = grow(d.d_masks, d.cap_masks, 3 * cap)) ||
            (rc = grow(d.d_pad_ws, d.cap_pad_ws, tkz::pad_workspace_bytes(n_docs))))
            return rc;
        hipError_t pe = tkz::launch_pad(t->pp, d.d_row, n_docs, d.d_ids, d.d_offs, d.d_row2, d.d_ids2, d.d_offs2,
                                        d.d_masks, d.d_masks + cap, d.d_masks + 2 * cap, d.d_pad_ws, d.stream);
        if (pe != hipSuccess) return fail(TKZ_ERR_DEVICE, std::string("pad launch failed: ") + hipGetErrorString(pe));
        hipMemcpyAsync(&nt, d.d_row2 + n_docs, 8, hipMemcpyDeviceToHost, d.stream);
        if (hipStreamSynchronize(d.stream) != hipSuccess) return fail(TKZ_ERR_DEVICE, "device error");
        src_row = d.d_row2;
        src_ids = d.d_ids2;
        src_offs = d.d_offs2;
    }
    out->n_docs = n_docs;
    out->n_tokens = nt;
    out->row_ptr = (uint64_t*)out_alloc((n_docs + 1) * 8);
    out->ids = (uint32_t*)out_alloc(std::max<uint64_t>(nt, 1) * 4);
    out->offsets = (tkz_offset*)out_alloc(std::max<uint64_t>(nt, 1) * 8);
    if (padded) {
        out->type_ids = (uint32_t*)out_alloc(std::max<uint64_t>(nt, 1) * 4);
        out->special_token_mask = (uint32_t*)out_alloc(std::max<uint64_t>(nt, 1) * 4);
        out->attention_mask = (uint32_t*)out_alloc(std::max<uint64_t>(nt, 1) * 4);
    }
    if (!out->row_ptr || !out->ids || !out->offsets ||
        (padded && (!out->type_ids || !out->special_token_mask || !out->attention_mask))) {
        tkz_batch_free(out);
        return fail(TKZ_ERR_OUT_OF_MEMORY, "out of memory");
    }
    hipMemcpyAsync(out->row_ptr, src_row, (n_docs + 1) * 8, hipMemcpyDeviceToHost, d.stream);
    if (nt) {
        hipMemcpyAsync(out->ids, src_ids, nt * 4, hipMemcpyDeviceToHost, d.stream);
        hipMemcpyAsync(out->offsets, src_offs, nt * 8, hipMemcpyDeviceToHost, d.stream);
    }
    if (padded && nt) {
        hipMemcpyAsync(out->type_ids, d.d_masks, nt * 4, hipMemcpyDeviceToHost, d.stream);
        hipMemcpyAsync(out->special_token_mask, d.d_masks + cap, nt * 4, hipMemcpyDeviceToHost, d.stream);
        hipMemcpyAsync(out->attention_mask, d.d_masks + 2 * cap, nt * 4, hipMemcpyDeviceToHost, d.stream);
    }
    hipError_t e = hipStreamSynchronize(d.stream);
    if (e != hipSuccess) { tkz_batch_free(out); return fail(TKZ_ERR_DEVICE, hipGetErrorString(e)); }
    return TKZ_OK;
}

void tkz_batch_free(tkz_batch* b) {
    if (!b) return;
    out_free(b->row_ptr); out_free(b->ids); out_free(b->offsets);
    out_free(b->type_ids); out_free(b->special_token_mask); out_free(b->attention_mask);
    memset(b, 0, sizeof *b);
}

int tkz_set_virtual_devices(tkz_tokenizer* t, int n) {
    if (!t || n < 0) return fail(TKZ_ERR_INVALID_ARGUMENT, "invalid argument");
    std::lock_guard<std::mutex> g(t->mu);
    t->virtual_devices = n;
    return TKZ_OK;
}

// tkz_encode_batch over the GPUs of gpu_mask: the docs are cut into one doc-aligned part
// per device with about equal bytes; each part runs tkz_encode_batch on its device's
// replica of the tables from its own host thread (the parts are independent: Tokenizer.encode
// only reads the tables, lib.zig:109-160), and the parts' CSR arrays are concatenated with
// row_ptr rebased to each part's token base.
int tkz_encode_batch_gpus(tkz_tokenizer* t, const uint8_t* bytes, const uint64_t* doc_off, size_t n_docs,
                          uint32_t gpu_mask, tkz_batch* out) {
    if (!t || !doc_off || !out || (n_docs && !bytes && doc_off[n_docs] > doc_off[0]))
        return fail(TKZ_ERR_INVALID_ARGUMENT, "null argument");
    memset(out, 0, sizeof *out);
    for (size_t i = 0; i < n_docs; ++i)
        if (doc_off[i + 1] < doc_off[i]) return fail(TKZ_ERR_INVALID_ARGUMENT, "doc_off must be non-decreasing");
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count < 1)
        return fail(TKZ_ERR_DEVICE, "no HIP device available (the encode path is GPU-only)");
    if (gpu_mask == 0) return fail(TKZ_ERR_INVALID_ARGUMENT, "gpu_mask selects no device");
    std::vector<tkz_tokenizer*> rep;
    std::vector<int> dev;
    bool masks = false;
    int caller_dev = 0;
    (void)hipGetDevice(&caller_dev);
    {
        std::lock_guard<std::mutex> g(t->mu);
        masks = t->pp.truncate || t->pp.pad;
        for (int i = 0; i < 32; ++i) {
            if (!((gpu_mask >> i) & 1u)) continue;
            if (!t->virtual_devices && i >= count)
                return fail(TKZ_ERR_INVALID_ARGUMENT, "gpu_mask names device " + std::to_string(i) + " of " +
                                                          std::to_string(count));
            const int d = t->virtual_devices ? i % count : i;
            tkz_tokenizer* r = nullptr;
            for (auto& x : t->replicas)
                if (x.first == i && x.second->want_device == d) r = x.second;
            if (!r) {
                if (!(r = clone_for_encode(t, d))) return fail(TKZ_ERR_OUT_OF_MEMORY, "out of memory");
                t->replicas.emplace_back(i, r);
            }
            // settings changed since the replica was made, under the replica's own lock: a
            // concurrent tkz_encode_batch_gpus call may be encoding on it (tkz_encode_batch
            // holds r->mu and reads these fields; build_memo swaps its tables and status word)
            std::lock_guard<std::mutex> gr(r->mu);
            r->pp = t->pp;
            r->pad_token = t->pad_token;
            r->host_chunk = t->host_chunk;
            if (r->dedup_mode != t->dedup_mode) { r->dedup_mode = t->dedup_mode; apply_dedup(r); }
            if (r->memo_on != t->memo_on) {
                r->memo_on = t->memo_on;
                if (r->dev.ready) {
                    if (!r->memo_on) { r->dev.T.memo = nullptr; r->dev.T.memo8 = nullptr; }
                    else {
                        hipSetDevice(r->dev.device);
                        int rc = build_memo(r);
                        if (rc) return rc;
                    }
                }
            }
            rep.push_back(r);
            dev.push_back(d);
        }
    }
    const size_t K = std::max<size_t>(1, std::min(rep.size(), std::max<size_t>(n_docs, 1)));
    const std::vector<size_t> cut = byte_balanced_cuts(doc_off, n_docs, K);
    std::vector<tkz_batch> part(K);
    std::vector<int> rc(K, TKZ_OK);
    std::vector<std::string> err(K);
    auto run = [&](size_t k) {
        const size_t d0 = cut[k], n = cut[k + 1] - d0;
        if (n == 0 && k > 0) return;  // an empty part (very unequal docs): nothing to encode
        std::vector<uint64_t> off(n + 1);
        for (size_t i = 0; i <= n; ++i) off[i] = doc_off[d0 + i] - doc_off[d0];
        if (hipSetDevice(dev[k]) != hipSuccess) { rc[k] = TKZ_ERR_DEVICE; err[k] = "hipSetDevice failed"; return; }
        rc[k] = tkz_encode_batch(rep[k], bytes ? bytes + doc_off[d0] : bytes, off.data(), n, &part[k]);
        if (rc[k]) err[k] = g_last_error;
    };
    std::vector<std::thread> th;
    for (size_t k = 1; k < K; ++k) th.emplace_back(run, k);
    run(0);
    for (auto& x : th) x.join();
    hipSetDevice(caller_dev);
    auto free_parts = [&]() { for (auto& b : part) tkz_batch_free(&b); };
    for (size_t k = 0; k < K; ++k)
        if (rc[k]) { free_parts(); return fail(rc[k], "device " + std::to_string(dev[k]) + ": " + err[k]); }
    std::vector<uint64_t> tb(K + 1, 0);
    for (size_t k = 0; k < K; ++k) tb[k + 1] = tb[k] + part[k].n_tokens;
    const uint64_t nt = tb[K];
    out->n_docs = n_docs;
    out->n_tokens = nt;
    out->row_ptr = (uint64_t*)out_alloc((n_docs + 1) * 8);
    out->ids = (uint32_t*)out_alloc(std::max<uint64_t>(nt, 1) * 4);
    out->offsets = (tkz_offset*)out_alloc(std::max<uint64_t>(nt, 1) * 8);
    if (masks) {
        out->type_ids = (uint32_t*)out_alloc(std::max<uint64_t>(nt, 1) * 4);
        out->special_token_mask = (uint32_t*)out_alloc(std::max<uint64_t>(nt, 1) * 4);
        out->attention_mask = (uint32_t*)out_alloc(std::max<uint64_t>(nt, 1) * 4);
    }
    if (!out->row_ptr || !out->ids || !out->offsets ||
        (masks && (!out->type_ids || !out->special_token_mask || !out->attention_mask))) {
        free_parts();
        tkz_batch_free(out);
        return fail(TKZ_ERR_OUT_OF_MEMORY, "out of memory");
    }
    auto merge = [&](size_t k) {
        const tkz_batch& b = part[k];
        const size_t d0 = cut[k];
        for (size_t i = 0; i < b.n_docs; ++i) out->row_ptr[d0 + i] = b.row_ptr[i] + tb[k];
        if (b.n_tokens) {
            memcpy(out->ids + tb[k], b.ids, b.n_tokens * 4);
            memcpy(out->offsets + tb[k], b.offsets, b.n_tokens * 8);
            if (masks) {
                memcpy(out->type_ids + tb[k], b.type_ids, b.n_tokens * 4);
                memcpy(out->special_token_mask + tb[k], b.special_token_mask, b.n_tokens * 4);
                memcpy(out->attention_mask + tb[k], b.attention_mask, b.n_tokens * 4);
            }
        }
    };
    th.clear();
    for (size_t k = 1; k < K; ++k) th.emplace_back(merge, k);
    merge(0);
    for (auto& x : th) x.join();
    out->row_ptr[n_docs] = nt;
    free_parts();
    return TKZ_OK;
}

const char* tkz_id_to_token(const tkz_tokenizer* t, uint32_t id, size_t* len);

int tkz_encode(tkz_tokenizer* t, const uint8_t* text, size_t len, int add_special_tokens, tkz_encoding* out) {
    (void)add_special_tokens;  // post-processor is a no-op (config.zig:551-555)
    if (!t || !out || (len && !text)) return fail(TKZ_ERR_INVALID_ARGUMENT, "null argument");
    memset(out, 0, sizeof *out);
    uint64_t off[2] = {0, len};
    tkz_batch b;
    int rc = tkz_encode_batch(t, text, off, 1, &b);
    if (rc) return rc;
    const size_t n = (size_t)b.n_tokens;
    out->len = n;
    const size_t m = std::max<size_t>(n, 1);
    out->ids = (uint32_t*)malloc(m * 4);
    out->type_ids = (uint32_t*)calloc(m, 4);
    out->offsets = (tkz_offset*)malloc(m * 8);
    out->special_token_mask = (uint32_t*)calloc(m, 4);
    out->attention_mask = (uint32_t*)malloc(m * 4);
    out->tokens = (const char**)malloc(m * sizeof(char*));
    out->token_lens = (uint32_t*)malloc(m * 4);
    if (!out->ids || !out->type_ids || !out->offsets || !out->special_token_mask || !out->attention_mask ||
        !out->tokens || !out->token_lens) {
        tkz_batch_free(&b);
        tkz_encoding_free(out);
        return fail(TKZ_ERR_OUT_OF_MEMORY, "out of memory");
    }
    for (size_t i = 0; i < n; ++i) {
        out->ids[i] = b.ids[i];
        out->offsets[i] = b.offsets[i];
        out->attention_mask[i] = b.attention_mask ? b.attention_mask[i] : 1;
        out->type_ids[i] = b.type_ids ? b.type_ids[i] : 0;
        out->special_token_mask[i] = b.special_token_mask ? b.special_token_mask[i] : 0;
        if (b.special_token_mask && b.special_token_mask[i]) {  // a pad position: pad_token (encoding.zig:404)
            out->tokens[i] = t->pad_token.c_str();
            out->token_lens[i] = (uint32_t)t->pad_token.size();
            continue;
        }
        auto it = t->vocab_r.find(b.ids[i]);  // model vocab (Token.value), encoding.zig:272-280
        out->tokens[i] = it != t->vocab_r.end() ? it->second->c_str() : "";
        out->token_lens[i] = it != t->vocab_r.end() ? (uint32_t)it->second->size() : 0;
    }
    tkz_batch_free(&b);
    return TKZ_OK;
}

void tkz_encoding_free(tkz_encoding* e) {
    if (!e) return;
    free(e->ids); free(e->type_ids); free(e->offsets); free(e->special_token_mask); free(e->attention_mask);
    free((void*)e->tokens); free(e->token_lens);
    memset(e, 0, sizeof *e);
}

int tkz_decode(const tkz_tokenizer* t, const uint32_t* ids, size_t n, int skip_special, char** out, size_t* out_len) {
    if (!t || !out || (n && !ids)) return fail(TKZ_ERR_INVALID_ARGUMENT, "null argument");
    std::string r;
    for (size_t i = 0; i < n; ++i) {  // lib.zig:167-179
        if (skip_special) {
            auto a = t->added_i2t.find(ids[i]);
            if (a != t->added_i2t.end() && t->special.count(a->second)) continue;
        }
        auto it = t->vocab_r.find(ids[i]);
        if (it != t->vocab_r.end()) r += *it->second;
    }
    std::string o;
    if (t->decoder == 1) {  // config.zig:488-505: drop every "##"
        for (size_t i = 0; i < r.size();) {
            if (i + 1 < r.size() && r[i] == '#' && r[i + 1] == '#') i += 2;
            else o.push_back(r[i++]);
        }
    } else if (t->decoder == 3) {  // config.zig:512-530: "\xC4\xA0" -> ' '
        for (size_t i = 0; i < r.size();) {
            if (i + 1 < r.size() && (uint8_t)r[i] == 0xC4 && (uint8_t)r[i + 1] == 0xA0) { o.push_back(' '); i += 2; }
            else o.push_back(r[i++]);
        }
    } else {
        o.swap(r);  // none / ByteLevel copy (config.zig:507-510)
    }
    char* s = (char*)malloc(o.size() + 1);
    if (!s) return fail(TKZ_ERR_OUT_OF_MEMORY, "out of memory");
    memcpy(s, o.data(), o.size());
    s[o.size()] = 0;
    *out = s;
    if (out_len) *out_len = o.size();
    return TKZ_OK;
}

void tkz_string_free(char* s) { free(s); }

size_t tkz_get_vocab_size(const tkz_tokenizer* t) { return t ? t->vocab.size() + t->added_t2i.size() : 0; }

int tkz_token_to_id(const tkz_tokenizer* t, const char* tok, size_t len, uint32_t* id) {
    if (!t || (!tok && len)) return 0;
    std::string k(tok ? tok : "", len);
    auto a = t->added_t2i.find(k);
    if (a != t->added_t2i.end()) { if (id) *id = a->second; return 1; }
    auto it = t->vocab.find(k);
    if (it != t->vocab.end()) { if (id) *id = it->second; return 1; }
    return 0;
}

const char* tkz_id_to_token(const tkz_tokenizer* t, uint32_t id, size_t* len) {
    if (!t) return nullptr;
    auto a = t->added_i2t.find(id);
    if (a != t->added_i2t.end()) { if (len) *len = a->second.size(); return a->second.c_str(); }
    auto it = t->vocab_r.find(id);
    if (it != t->vocab_r.end()) { if (len) *len = it->second->size(); return it->second->c_str(); }
    return nullptr;
}

size_t tkz_add_special_tokens(tkz_tokenizer* t, const char* const* toks, const size_t* lens, size_t n) {
    return tkz_add_special_tokens_ids(t, toks, lens, nullptr, n);
}

size_t tkz_add_special_tokens_ids(tkz_tokenizer* t, const char* const* toks, const size_t* lens, const uint32_t* ids,
                                  size_t n) {
    if (!t || (n && (!toks || !lens))) return 0;
    std::lock_guard<std::mutex> g(t->mu);
    size_t added = 0;
    for (size_t i = 0; i < n; ++i) {
        const bool has_id = ids && ids[i] != TKZ_NO_ID;
        added += add_token(t, std::string(toks[i], lens[i]), has_id, has_id ? ids[i] : 0, true) ? 1 : 0;
    }
    return added;
}

int tkz_debug_merge_lookup(const tkz_tokenizer* t, uint32_t a, uint32_t b, uint32_t* rank, uint32_t* new_id) {
    if (!t || t->model != 1) return 0;
    if (t->compact) {
        if (a >= 0xFFFFu || b >= 0xFFFFu) return 0;
        uint32_t v = tkz::merge_probe_compact(t->mtab_c.data(), t->m_bits, a, b);
        if (v == NONE) return 0;
        if (rank) *rank = v >> 16;
        if (new_id) *new_id = v & 0xFFFFu;
        return 1;
    }
    uint32_t r, nid;
    if (!tkz::merge_probe_wide(t->mtab_w.data(), t->m_bits, a, b, r, nid)) return 0;
    if (rank) *rank = r;
    if (new_id) *new_id = nid;
    return 1;
}

size_t tkz_debug_counters_offset(uint64_t total_bytes, size_t n_docs) {
    return tkz::debug_counters_offset(total_bytes, n_docs);
}

int tkz_debug_vocab_lookup(const tkz_tokenizer* t, const char* key, size_t len, uint32_t* id) {
    if (!t || (!key && len)) return 0;
    uint64_t g = 0, pw = 1;
    for (size_t i = 0; i < len; ++i) { g += (uint64_t)((uint8_t)key[i] + 1) * pw; pw *= tkz::HP; }
    const uint64_t h = tkz::wp_final(g, (uint32_t)len);
    const uint32_t mask = (1u << t->wp_bits) - 1;
    uint32_t idx = (uint32_t)(h >> (64 - t->wp_bits));
    while (true) {
        const uint4 s = t->wp_tab[idx];
        if (s.w == NONE) return 0;
        if (s.x == (uint32_t)h && s.y == (uint32_t)(h >> 32)) {
            uint32_t elen;
            memcpy(&elen, &t->wp_pool[s.w], 4);
            if (elen == len && memcmp(&t->wp_pool[s.w + 4], key, len) == 0) {
                // 1-4 byte keys must also be reachable through the BPE char tables
                if (id) *id = s.z;
                return 1;
            }
        }
        idx = (idx + 1) & mask;
    }
}

// ---- plumbing for benches / tests: device memory, sync, kernel timers ----------
void* tkz_dev_alloc(size_t n) {
    void* p = nullptr;
    if (hipMalloc(&p, n ? n : 16) != hipSuccess) return nullptr;
    return p;
}
void tkz_dev_free(void* p) { if (p) hipFree(p); }
int tkz_memcpy_htod(void* dst, const void* src, size_t n) {
    return hipMemcpy(dst, src, n, hipMemcpyHostToDevice) == hipSuccess ? TKZ_OK : fail(TKZ_ERR_DEVICE, "memcpy");
}
int tkz_memcpy_dtoh(void* dst, const void* src, size_t n) {
    return hipMemcpy(dst, src, n, hipMemcpyDeviceToHost) == hipSuccess ? TKZ_OK : fail(TKZ_ERR_DEVICE, "memcpy");
}
int tkz_memset_dev(void* dst, int v, size_t n) {
    return hipMemset(dst, v, n) == hipSuccess ? TKZ_OK : fail(TKZ_ERR_DEVICE, "memset");
}
int tkz_dev_mem_info(size_t* free_bytes, size_t* total_bytes) {
    if (!free_bytes || !total_bytes) return fail(TKZ_ERR_INVALID_ARGUMENT, "null");
    return hipMemGetInfo(free_bytes, total_bytes) == hipSuccess ? TKZ_OK : fail(TKZ_ERR_DEVICE, "hipMemGetInfo");
}
void* tkz_stream_create(void) {
    hipStream_t s = nullptr;
    return hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess ? (void*)s : nullptr;
}
void tkz_stream_destroy(void* s) { if (s) hipStreamDestroy((hipStream_t)s); }
int tkz_device_synchronize(void) {
    hipError_t e = hipDeviceSynchronize();
    return e == hipSuccess ? TKZ_OK : fail(TKZ_ERR_DEVICE, hipGetErrorString(e));
}
int tkz_synchronize(tkz_tokenizer* t) {
    if (!t) return fail(TKZ_ERR_INVALID_ARGUMENT, "null");
    if (!t->dev.ready) return TKZ_OK;
    hipError_t e = hipStreamSynchronize(t->dev.stream);
    return e == hipSuccess ? TKZ_OK : fail(TKZ_ERR_DEVICE, hipGetErrorString(e));
}
int tkz_profile_enable(tkz_tokenizer* t, int on) {
    if (!t) return fail(TKZ_ERR_INVALID_ARGUMENT, "null");
    t->dev.profile = on != 0;
    t->dev.n_timed = 0;
    return TKZ_OK;
}
int tkz_set_truncation(tkz_tokenizer* t, int enabled, size_t max_length, size_t stride) {
    if (!t) return fail(TKZ_ERR_INVALID_ARGUMENT, "null");
    (void)stride;  // the reference ignores it (encoding.zig:368, "TODO: implement stride/overflowing")
    std::lock_guard<std::mutex> g(t->mu);
    t->pp.truncate = enabled ? 1 : 0;
    t->pp.max_length = max_length;
    return TKZ_OK;
}

int tkz_set_padding(tkz_tokenizer* t, int enabled, size_t length, uint32_t pad_id, uint32_t pad_type_id,
                    const char* pad_token, size_t pad_token_len, int direction) {
    if (!t || (pad_token_len && !pad_token)) return fail(TKZ_ERR_INVALID_ARGUMENT, "null");
    std::lock_guard<std::mutex> g(t->mu);
    t->pp.pad = enabled && length > 0 ? 1 : 0;  // length null (0): nothing to pad to (encoding.zig:385)
    t->pp.length = length;
    t->pp.pad_id = pad_id;
    t->pp.pad_type_id = pad_type_id;
    t->pp.left = direction ? 1 : 0;
    t->pad_token = pad_token ? std::string(pad_token, pad_token_len) : std::string("[PAD]");
    return TKZ_OK;
}

uint64_t tkz_pad_capacity(const tkz_tokenizer* t, size_t n_docs, uint64_t n_tokens) {
    if (!t) return 0;
    return n_tokens + (t->pp.pad ? (uint64_t)n_docs * t->pp.length : 0) + 1;
}

size_t tkz_pad_workspace_size(size_t n_docs) { return tkz::pad_workspace_bytes(n_docs); }

int tkz_pad_batch_device(tkz_tokenizer* t, const uint64_t* d_row_ptr, const uint32_t* d_ids,
                         const tkz_offset* d_offsets, size_t n_docs, uint64_t* d_row_ptr2, uint32_t* d_ids2,
                         tkz_offset* d_offsets2, uint32_t* d_type_ids, uint32_t* d_special_mask,
                         uint32_t* d_attention_mask, void* d_workspace, size_t workspace_bytes, void* stream) {
    if (!t || !d_row_ptr || !d_row_ptr2 || (n_docs && (!d_ids || !d_offsets || !d_ids2 || !d_offsets2 ||
                                                         !d_type_ids || !d_special_mask || !d_attention_mask)))
        return fail(TKZ_ERR_INVALID_ARGUMENT, "null argument");
    if (workspace_bytes < tkz::pad_workspace_bytes(n_docs)) return fail(TKZ_ERR_INVALID_ARGUMENT, "workspace too small");
    std::lock_guard<std::mutex> g(t->mu);
    int rc = ensure_device(t);
    if (rc) return rc;
    hipStream_t st = stream ? (hipStream_t)stream : t->dev.stream;
    hipError_t e = tkz::launch_pad(t->pp, d_row_ptr, n_docs, d_ids, (const uint64_t*)d_offsets, d_row_ptr2, d_ids2,
                                   (uint64_t*)d_offsets2, d_type_ids, d_special_mask, d_attention_mask, d_workspace,
                                   st);
    if (e != hipSuccess) return fail(TKZ_ERR_DEVICE, std::string("pad launch failed: ") + hipGetErrorString(e));
    return TKZ_OK;
}

size_t tkz_fast_workspace_size(const tkz_tokenizer* t, uint64_t total_bytes, size_t n_docs) {
    return fast_workspace_bytes(total_bytes, n_docs, (t ? tkz::seg_mode(t->hostT) : 0));
}

int tkz_fast_encode_batch_device(tkz_tokenizer* t, const uint8_t* d_bytes, const uint64_t* d_doc_off, size_t n_docs,
                                 uint64_t total_bytes, uint64_t max_doc_bytes, const tkz_fast_options* opts,
                                 uint32_t* d_len, uint32_t* d_ids, tkz_offset* d_offsets, uint32_t* d_attention_mask,
                                 void* d_ws, size_t ws_bytes, uint32_t* d_status, void* stream) {
    if (!t || !opts || !d_doc_off || !d_ws || !d_status ||
        (n_docs && (!d_len || !d_bytes || (opts->max_tokens && (!d_ids || !d_offsets)))))
        return fail(TKZ_ERR_INVALID_ARGUMENT, "null argument");
    if (ws_bytes < fast_workspace_bytes(total_bytes, n_docs, 0))  // (the segmented arrays are optional)
        return fail(TKZ_ERR_INVALID_ARGUMENT, "workspace too small");
    std::lock_guard<std::mutex> g(t->mu);
    int rc = ensure_device(t);
    if (rc) return rc;
    hipStream_t st = stream ? (hipStream_t)stream : t->dev.stream;
    return run_fast_device(t, d_bytes, d_doc_off, n_docs, total_bytes, max_doc_bytes, *opts, d_len, d_ids,
                           (uint64_t*)d_offsets, d_attention_mask, d_ws, ws_bytes, d_status, st);
}

int tkz_fast_encode_batch(tkz_tokenizer* t, const uint8_t* bytes, const uint64_t* doc_off, size_t n_docs,
                          const tkz_fast_options* opts, tkz_span_batch* out) {
    if (!t || !doc_off || !opts || !out || (n_docs && !bytes && doc_off[n_docs] > 0))
        return fail(TKZ_ERR_INVALID_ARGUMENT, "null argument");
    memset(out, 0, sizeof *out);
    if (n_docs && doc_off[0] != 0) return fail(TKZ_ERR_INVALID_ARGUMENT, "doc_off[0] must be 0");
    uint64_t max_doc = 0;
    for (size_t i = 0; i < n_docs; ++i) {
        if (doc_off[i + 1] < doc_off[i]) return fail(TKZ_ERR_INVALID_ARGUMENT, "doc_off must be non-decreasing");
        max_doc = std::max<uint64_t>(max_doc, doc_off[i + 1] - doc_off[i]);
    }
    std::lock_guard<std::mutex> g(t->mu);
    int rc = ensure_device(t);
    if (rc) return rc;
    DeviceState& d = t->dev;
    const uint64_t total = n_docs ? doc_off[n_docs] : 0;
    const uint64_t cap = opts->max_tokens;
    const uint64_t cells = (uint64_t)n_docs * cap;
    const size_t padded = (size_t)((total + 16 + 15) / 16 * 16);
    if ((rc = grow(d.d_bytes, d.cap_bytes, padded)) || (rc = grow(d.d_off, d.cap_off, n_docs + 1)) ||
        (rc = grow(d.d_fast_ws, d.cap_fast_ws, fast_workspace_bytes(total, n_docs, tkz::seg_mode(d.T)))) ||
        (rc = grow(d.d_span, d.cap_span, n_docs + 2 * cells + 1)) ||
        (rc = grow(d.d_span_offs, d.cap_span_offs, cells + 1)))
        return rc;
    hipStream_t st = d.stream;
    if (total) hipMemcpyAsync(d.d_bytes, bytes, total, hipMemcpyHostToDevice, st);
    hipMemsetAsync(d.d_bytes + total, 0, padded - total, st);
    hipMemcpyAsync(d.d_off, doc_off, (n_docs + 1) * 8, hipMemcpyHostToDevice, st);
    hipMemsetAsync(d.d_status, 0, 4, st);
    uint32_t* d_len = d.d_span;
    uint32_t* d_ids = d.d_span + n_docs;
    uint32_t* d_attn = d_ids + cells;
    if ((rc = run_fast_device(t, d.d_bytes, d.d_off, n_docs, total, max_doc, *opts, d_len, d_ids, d.d_span_offs, d_attn,
                              d.d_fast_ws, d.cap_fast_ws * sizeof *d.d_fast_ws, d.d_status, st)))
        return rc;
    out->n_docs = n_docs;
    out->capacity = (uint32_t)cap;
    out->len = (uint32_t*)out_alloc(std::max<size_t>(n_docs, 1) * 4);
    out->ids = (uint32_t*)out_alloc(std::max<uint64_t>(cells, 1) * 4);
    out->offsets = (tkz_offset*)out_alloc(std::max<uint64_t>(cells, 1) * 8);
    out->attention_mask = (uint32_t*)out_alloc(std::max<uint64_t>(cells, 1) * 4);
    if (!out->len || !out->ids || !out->offsets || !out->attention_mask) {
        hipStreamSynchronize(st);
        tkz_span_batch_free(out);
        return fail(TKZ_ERR_OUT_OF_MEMORY, "out of memory");
    }
    uint32_t status = 0;
    hipMemcpyAsync(&status, d.d_status, 4, hipMemcpyDeviceToHost, st);
    if (n_docs) hipMemcpyAsync(out->len, d_len, n_docs * 4, hipMemcpyDeviceToHost, st);
    if (cells) {
        hipMemcpyAsync(out->ids, d_ids, cells * 4, hipMemcpyDeviceToHost, st);
        hipMemcpyAsync(out->offsets, d.d_span_offs, cells * 8, hipMemcpyDeviceToHost, st);
        hipMemcpyAsync(out->attention_mask, d_attn, cells * 4, hipMemcpyDeviceToHost, st);
    }
    hipError_t e = hipStreamSynchronize(st);
    if (e != hipSuccess) { tkz_span_batch_free(out); return fail(TKZ_ERR_DEVICE, hipGetErrorString(e)); }
    if (status) { tkz_span_batch_free(out); return fail((int)status, "device reported an error"); }
    return TKZ_OK;
}

void tkz_span_batch_free(tkz_span_batch* b) {
    if (!b) return;
    out_free(b->len); out_free(b->ids); out_free(b->offsets); out_free(b->attention_mask);
    memset(b, 0, sizeof *b);
}

uint64_t tkz_decode_bound(const tkz_tokenizer* t, uint64_t n_tokens) { return t ? decode_bound(t, n_tokens) : 0; }

size_t tkz_decode_workspace_size(const tkz_tokenizer* t, size_t n_docs, uint64_t n_tokens) {
    return t ? tkz::decode_workspace_bytes(n_docs, n_tokens, decode_bound(t, n_tokens)) : 0;
}

int tkz_decode_batch_device(tkz_tokenizer* t, const uint64_t* d_row_ptr, const uint32_t* d_ids, size_t n_docs,
                            uint64_t n_tokens, int skip_special, uint8_t* d_out, uint64_t out_capacity,
                            uint64_t* d_out_off, void* d_ws, size_t ws_bytes, void* stream) {
    if (!t || (n_docs && (!d_row_ptr || !d_out_off)) || (n_tokens && (!d_ids || !d_out)))
        return fail(TKZ_ERR_INVALID_ARGUMENT, "null argument");
    std::lock_guard<std::mutex> g(t->mu);
    int rc = ensure_decode(t);
    if (rc) return rc;
    const uint64_t bound = decode_bound(t, n_tokens);
    if (out_capacity < bound) return fail(TKZ_ERR_INVALID_ARGUMENT, "output capacity below tkz_decode_bound");
    if (ws_bytes < tkz::decode_workspace_bytes(n_docs, n_tokens, bound))
        return fail(TKZ_ERR_INVALID_ARGUMENT, "workspace smaller than tkz_decode_workspace_size");
    hipStream_t st = stream ? (hipStream_t)stream : t->dev.stream;
    hipError_t e = tkz::launch_decode(t->dev.DT, d_row_ptr, d_ids, n_docs, n_tokens, skip_special ? 1 : 0, bound, d_out,
                                      d_out_off, d_ws, st);
    if (e != hipSuccess) return fail(TKZ_ERR_DEVICE, std::string("decode launch failed: ") + hipGetErrorString(e));
    return TKZ_OK;
}

int tkz_decode_batch(tkz_tokenizer* t, const uint64_t* row_ptr, const uint32_t* ids, size_t n_docs, int skip_special,
                     tkz_text_batch* out) {
    if (!t || !out || !row_ptr) return fail(TKZ_ERR_INVALID_ARGUMENT, "null argument");
    memset(out, 0, sizeof(*out));
    std::lock_guard<std::mutex> g(t->mu);
    int rc = ensure_decode(t);
    if (rc) return rc;
    if (row_ptr[0] != 0) return fail(TKZ_ERR_INVALID_ARGUMENT, "row_ptr[0] must be 0");
    for (size_t i = 0; i < n_docs; ++i)
        if (row_ptr[i + 1] < row_ptr[i]) return fail(TKZ_ERR_INVALID_ARGUMENT, "row_ptr must be non-decreasing");
    const uint64_t nt = row_ptr[n_docs];
    if (nt && !ids) return fail(TKZ_ERR_INVALID_ARGUMENT, "null ids");
    DeviceState& d = t->dev;
    const uint64_t bound = decode_bound(t, nt);
    const size_t ws = tkz::decode_workspace_bytes(n_docs, nt, bound);
    if ((rc = grow(d.d_dec_ids, d.cap_dec_ids, nt + 1)) || (rc = grow(d.d_dec_row, d.cap_dec_row, n_docs + 1)) ||
        (rc = grow(d.d_dec_out, d.cap_dec_out, bound)) || (rc = grow(d.d_dec_off, d.cap_dec_off, n_docs + 1)) ||
        (rc = grow(d.d_dec_ws, d.cap_dec_ws, ws)))
        return rc;
    hipStream_t st = d.stream;
    if (nt) hipMemcpyAsync(d.d_dec_ids, ids, nt * 4, hipMemcpyHostToDevice, st);
    hipMemcpyAsync(d.d_dec_row, row_ptr, (n_docs + 1) * 8, hipMemcpyHostToDevice, st);
    hipError_t e = tkz::launch_decode(d.DT, d.d_dec_row, d.d_dec_ids, n_docs, nt, skip_special ? 1 : 0, bound,
                                      d.d_dec_out, d.d_dec_off, d.d_dec_ws, st);
    if (e != hipSuccess) return fail(TKZ_ERR_DEVICE, std::string("decode launch failed: ") + hipGetErrorString(e));
    out->n_docs = n_docs;
    out->offsets = (uint64_t*)out_alloc((n_docs + 1) * 8);
    if (!out->offsets) return fail(TKZ_ERR_OUT_OF_MEMORY, "out of memory");
    out->offsets[0] = 0;
    if (n_docs) hipMemcpyAsync(out->offsets, d.d_dec_off, (n_docs + 1) * 8, hipMemcpyDeviceToHost, st);
    if ((e = hipStreamSynchronize(st)) != hipSuccess) {
        out_free(out->offsets);
        out->offsets = nullptr;
        return fail(TKZ_ERR_DEVICE, std::string("device error: ") + hipGetErrorString(e));
    }
    const uint64_t nb = out->offsets[n_docs];
    out->n_bytes = nb;
    out->bytes = (char*)out_alloc(nb + 1);
    if (!out->bytes) { out_free(out->offsets); out->offsets = nullptr; return fail(TKZ_ERR_OUT_OF_MEMORY, "out of memory"); }
    if (nb) hipMemcpy(out->bytes, d.d_dec_out, nb, hipMemcpyDeviceToHost);
    out->bytes[nb] = 0;
    return TKZ_OK;
}

void tkz_text_batch_free(tkz_text_batch* b) {
    if (!b) return;
    out_free(b->offsets);
    out_free(b->bytes);
    memset(b, 0, sizeof(*b));
}

// ms[0] = k_encode, ms[1] = k_bpe_deferred, ms[2] = count + scan kernels, ms[3] =
// k_compact, summed over the calls recorded since the last reset. Call after
// tkz_synchronize.
int tkz_host_profile_read(tkz_tokenizer* t, double* out, size_t n, int reset) {
    if (!t || (!out && n)) return fail(TKZ_ERR_INVALID_ARGUMENT, "null argument");
    std::lock_guard<std::mutex> g(t->mu);
    for (size_t i = 0; i < n && i < HP_N; ++i) out[i] = t->dev.hp[i];
    if (reset) for (double& v : t->dev.hp) v = 0;
    return TKZ_OK;
}

void* tkz_host_alloc(size_t n) {
    void* p = nullptr;
    return hipHostMalloc(&p, std::max<size_t>(n, 1), hipHostMallocDefault) == hipSuccess ? p : nullptr;
}
void tkz_host_free(void* p) { if (p) hipHostFree(p); }

int tkz_profile_read(tkz_tokenizer* t, double* ms, uint64_t* n_calls, int reset) {
    if (!t || !ms) return fail(TKZ_ERR_INVALID_ARGUMENT, "null");
    ms[0] = ms[1] = ms[2] = ms[3] = 0;
    for (size_t i = 0; i < t->dev.n_timed; ++i) {
        auto& tm = t->dev.timers[i];
        for (int k = 0; k < 4; ++k) {
            float x = 0;
            hipEventElapsedTime(&x, tm.ev[k], tm.ev[k + 1]);
            ms[k] += x;
        }
    }
    if (n_calls) *n_calls = t->dev.n_timed;
    if (reset) t->dev.n_timed = 0;
    return TKZ_OK;
}

}  // extern "C"
