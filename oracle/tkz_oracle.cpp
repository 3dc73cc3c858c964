// CPU ORACLE — test infrastructure only (see oracle/oracle.py header).
//
// C++17 restatement of the reference's Tokenizer.encode loop
// (jrc2139/tokenizer-zig, src/lib.zig:109-160) used (a) as the parity checker for
// large batches and (b) as the timed CPU baseline ("port") in bench.py. It keeps the
// reference's data structures and per-call allocation pattern on purpose:
//   * string-keyed hash map for the model vocab   (bpe.zig:38, wordpiece.zig:15)
//   * u64-keyed hash map  pair -> {rank,new_id}    (bpe.zig:40, Pair.hash bpe.zig:24-26)
//   * normalized copy per call                     (config.zig:364-379)
//   * pretoken slice list per call                 (config.zig:405-450)
//   * per-pretoken word / char_offsets vectors, O(rounds*n) merge scan,
//     orderedRemove                                (bpe.zig:173-263)
//   * greedy longest-match WordPiece w/ 512-B buf  (wordpiece.zig:141-222)
//   * Encoding.fromTokens arrays + a string dup per token (encoding.zig:246-294)
// The product (tokenizer-zig_amd/) never links this file.
#include <atomic>
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <functional>
#include <queue>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

namespace {

enum { MODEL_WORDPIECE = 0, MODEL_BPE = 1 };
enum { NORM_NONE = 0, NORM_LOWER = 1 };
enum { PRETOK_NONE = 0, PRETOK_WHITESPACE = 1, PRETOK_BERT = 2 };

struct PairVal { uint32_t rank, new_id; };  // bpe.zig:30-33
struct Tok { uint32_t id; std::string_view value; uint32_t start, end; };  // token.zig:83-97

struct Oracle {
    int model, norm, pretok;
    std::string pool;                                   // owns vocab key bytes
    std::unordered_map<std::string_view, uint32_t> vocab;
    std::unordered_map<uint32_t, std::string_view> vocab_r;
    std::unordered_map<uint64_t, PairVal> merges;
    bool has_unk = false;
    std::string unk;
    std::string prefix;
    uint64_t max_chars = 100;
    bool heap_ok = false;     // merges ordered and chain-free (see bpe_tokenize_heap)
    uint64_t heap_bytes = 0;  // pretokens of >= this many bytes take bpe_tokenize_heap (0: never)
};

// std.unicode.utf8ByteSequenceLength; invalid lead -> 1 (reference: unreachable)
inline uint32_t seq_len(uint8_t b) {
    if (b < 0x80) return 1;
    if (b >= 0xC0 && b <= 0xDF) return 2;
    if (b >= 0xE0 && b <= 0xEF) return 3;
    if (b >= 0xF0 && b <= 0xF7) return 4;
    return 1;
}

// config.zig:452-457
inline bool is_punct(uint8_t c) {
    return (c >= 33 && c <= 47) || (c >= 58 && c <= 64) || (c >= 91 && c <= 96) || (c >= 123 && c <= 126);
}
// std.ascii.isWhitespace (Zig 0.15)
inline bool is_ascii_ws(uint8_t c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == 0x0B || c == 0x0C; }
// tokenizeAny delimiters " \t\n\r" (config.zig:444)
inline bool is_ws_delim(uint8_t c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }

// BPE.tokenize (bpe.zig:173-263)
int bpe_tokenize(const Oracle& o, std::string_view seq, std::vector<Tok>& out_tokens) {
    if (seq.empty()) return 0;
    std::vector<uint32_t> word;
    struct Off { uint32_t start, end; };
    std::vector<Off> char_offsets;
    uint32_t byte_idx = 0;
    size_t i = 0;
    while (i < seq.size()) {  // Utf8Iterator.nextCodepointSlice
        uint32_t len = seq_len((uint8_t)seq[i]);
        if (i + len > seq.size()) len = (uint32_t)(seq.size() - i);
        std::string_view ch = seq.substr(i, len);
        auto it = o.vocab.find(ch);
        if (it != o.vocab.end()) {
            word.push_back(it->second);
            char_offsets.push_back({byte_idx, byte_idx + len});
        } else if (o.has_unk) {
            auto u = o.vocab.find(std::string_view(o.unk));
            if (u != o.vocab.end()) {
                word.push_back(u->second);
                char_offsets.push_back({byte_idx, byte_idx + len});
            }
        }
        byte_idx += len;
        i += len;
    }
    while (word.size() > 1) {
        bool found = false;
        uint64_t best_key = 0;
        uint32_t best_rank = 0xFFFFFFFFu;
        for (size_t k = 0; k + 1 < word.size(); ++k) {
            uint64_t key = ((uint64_t)word[k] << 32) | word[k + 1];
            auto it = o.merges.find(key);
            if (it != o.merges.end() && it->second.rank < best_rank) {
                best_rank = it->second.rank;
                best_key = key;
                found = true;
            }
        }
        if (!found) break;
        const PairVal pv = o.merges.find(best_key)->second;
        const uint32_t a = (uint32_t)(best_key >> 32), b = (uint32_t)best_key;
        size_t k = 0;
        while (k + 1 < word.size()) {
            if (word[k] == a && word[k + 1] == b) {
                word[k] = pv.new_id;
                word.erase(word.begin() + (k + 1));               // orderedRemove
                char_offsets[k].end = char_offsets[k + 1].end;
                char_offsets.erase(char_offsets.begin() + (k + 1));
            } else {
                ++k;
            }
        }
    }
    std::vector<Tok> tokens(word.size());
    for (size_t k = 0; k < word.size(); ++k) {
        auto it = o.vocab_r.find(word[k]);
        tokens[k] = {word[k], it != o.vocab_r.end() ? it->second : std::string_view(), char_offsets[k].start, char_offsets[k].end};
    }
    out_tokens.insert(out_tokens.end(), tokens.begin(), tokens.end());
    return 0;
}

// BPE.tokenize (bpe.zig:173-263) with a min-heap of (rank, position) over a linked list --
// O(n log n) instead of O(rounds * n) -- for the very long whole-text pretokens of the
// 4 KB - 1 MB bench docs (C10), where the literal loop above takes minutes per doc. It
// gives the literal loop's result whenever every merge ranks after the merges creating its
// parts and none creates its own left part (Oracle::heap_ok, checked at orc_create):
// a round of rank r then creates only pairs ranked above r, so the pairs of rank r are
// exactly those present when the round starts, and popping them by position merges them
// left to right with the literal loop's rule for runs of equal pairs (after a merge at k
// the scan goes on past the merged symbol, bpe.zig:240-252: a consumed symbol's pair is
// dead). tests/test_oracle_heap.py checks it against the literal loop.
int bpe_tokenize_heap(const Oracle& o, std::string_view seq, std::vector<Tok>& out_tokens) {
    if (seq.empty()) return 0;
    std::vector<uint32_t> sym, st, en;
    uint32_t byte_idx = 0;
    size_t i = 0;
    const uint32_t* unk_id = nullptr;
    uint32_t unk_v = 0;
    if (o.has_unk) {
        auto u = o.vocab.find(std::string_view(o.unk));
        if (u != o.vocab.end()) { unk_v = u->second; unk_id = &unk_v; }
    }
    while (i < seq.size()) {  // Utf8Iterator.nextCodepointSlice (as bpe_tokenize)
        uint32_t len = seq_len((uint8_t)seq[i]);
        if (i + len > seq.size()) len = (uint32_t)(seq.size() - i);
        auto it = o.vocab.find(seq.substr(i, len));
        if (it != o.vocab.end() || unk_id) {
            sym.push_back(it != o.vocab.end() ? it->second : *unk_id);
            st.push_back(byte_idx);
            en.push_back(byte_idx + len);
        }
        byte_idx += len;
        i += len;
    }
    const uint32_t n = (uint32_t)sym.size(), NIL = 0xFFFFFFFFu;
    std::vector<uint32_t> nxt(n), prv(n);
    std::vector<uint8_t> dead(n, 0);
    for (uint32_t k = 0; k < n; ++k) { nxt[k] = k + 1 < n ? k + 1 : NIL; prv[k] = k ? k - 1 : NIL; }
    typedef std::pair<uint32_t, uint32_t> E;  // (rank, position)
    std::priority_queue<E, std::vector<E>, std::greater<E>> heap;
    auto push = [&](uint32_t p) {
        if (p == NIL || nxt[p] == NIL) return;
        auto it = o.merges.find(((uint64_t)sym[p] << 32) | sym[nxt[p]]);
        if (it != o.merges.end()) heap.push({it->second.rank, p});
    };
    for (uint32_t k = 0; k + 1 < n; ++k) push(k);
    while (!heap.empty()) {
        const E top = heap.top();
        heap.pop();
        const uint32_t p = top.second;
        if (dead[p] || nxt[p] == NIL) continue;
        const uint32_t q = nxt[p];
        auto it = o.merges.find(((uint64_t)sym[p] << 32) | sym[q]);
        if (it == o.merges.end() || it->second.rank != top.first) continue;  // (stale: the pair changed)
        sym[p] = it->second.new_id;
        en[p] = en[q];
        dead[q] = 1;
        nxt[p] = nxt[q];
        if (nxt[q] != NIL) prv[nxt[q]] = p;
        push(prv[p]);
        push(p);
    }
    for (uint32_t k = 0; k < n; ++k) {
        if (dead[k]) continue;
        auto it = o.vocab_r.find(sym[k]);
        out_tokens.push_back({sym[k], it != o.vocab_r.end() ? it->second : std::string_view(), st[k], en[k]});
    }
    return 0;
}

// WordPiece.tokenize (wordpiece.zig:141-222)
int wordpiece_tokenize(const Oracle& o, std::string_view chars, std::vector<Tok>& out_tokens) {
    std::vector<Tok> tokens;
    const size_t n = chars.size();
    auto unk_tok = [&](std::vector<Tok>& t) -> int {
        auto u = o.vocab.find(std::string_view(o.unk));
        if (u == o.vocab.end()) return 1;  // error.MissingUnkToken
        t.clear();
        t.push_back({u->second, o.vocab_r.at(u->second), 0, (uint32_t)n});
        return 0;
    };
    if (n > o.max_chars) {
        if (unk_tok(tokens)) return 1;
        out_tokens.insert(out_tokens.end(), tokens.begin(), tokens.end());
        return 0;
    }
    bool is_bad = false;
    size_t start = 0;
    while (start < n) {
        size_t end = n;
        bool found = false;
        uint32_t cur_id = 0;
        while (start < end) {
            char substr_buf[512];
            std::string_view substr;
            if (start > 0) {
                const size_t plen = o.prefix.size(), wlen = end - start;
                if (plen + wlen > sizeof(substr_buf)) { end -= 1; continue; }
                memcpy(substr_buf, o.prefix.data(), plen);
                memcpy(substr_buf + plen, chars.data() + start, wlen);
                substr = std::string_view(substr_buf, plen + wlen);
            } else {
                substr = chars.substr(start, end - start);
            }
            auto it = o.vocab.find(substr);
            if (it != o.vocab.end()) { cur_id = it->second; found = true; break; }
            end -= 1;
        }
        if (!found) { is_bad = true; break; }
        tokens.push_back({cur_id, o.vocab_r.at(cur_id), (uint32_t)start, (uint32_t)end});
        start = end;
    }
    if (is_bad && unk_tok(tokens)) return 1;
    out_tokens.insert(out_tokens.end(), tokens.begin(), tokens.end());
    return 0;
}

struct Encoding {  // encoding.zig:230-241 (owned arrays + duped token strings)
    std::vector<uint32_t> ids, type_ids, special_token_mask, attention_mask;
    std::vector<std::string> tokens;
    std::vector<uint64_t> offsets;
};

// Tokenizer.encode (lib.zig:109-160); writes the doc's tokens at ids/offs[0..count)
int encode_doc(const Oracle& o, const uint8_t* text, size_t len, uint32_t* ids, uint32_t* offs, uint32_t* count,
               int full_encoding) {
    std::string_view normalized((const char*)text, len);
    std::string norm_buf;
    if (o.norm == NORM_LOWER) {  // config.zig:364-379
        norm_buf.resize(len);
        for (size_t i = 0; i < len; ++i) {
            uint8_t c = text[i];
            norm_buf[i] = (char)((c >= 'A' && c <= 'Z') ? (c | 0x20) : c);
        }
        normalized = norm_buf;
    }
    std::vector<std::string_view> pretokens;
    if (o.pretok == PRETOK_WHITESPACE) {  // config.zig:440-450
        size_t i = 0, n = normalized.size();
        while (i < n) {
            while (i < n && is_ws_delim((uint8_t)normalized[i])) ++i;
            size_t j = i;
            while (j < n && !is_ws_delim((uint8_t)normalized[j])) ++j;
            if (j > i) pretokens.push_back(normalized.substr(i, j - i));
            i = j;
        }
    } else if (o.pretok == PRETOK_BERT) {  // config.zig:405-438
        size_t start = 0;
        for (size_t i = 0; i < normalized.size(); ++i) {
            uint8_t c = (uint8_t)normalized[i];
            bool ws = is_ascii_ws(c), p = is_punct(c);
            if (ws || p) {
                if (i > start) pretokens.push_back(normalized.substr(start, i - start));
                if (p) pretokens.push_back(normalized.substr(i, 1));
                start = i + 1;
            }
        }
        if (start < normalized.size()) pretokens.push_back(normalized.substr(start));
    } else {
        pretokens.push_back(normalized);  // lib.zig:121
    }
    std::vector<Tok> all_tokens;
    for (auto p : pretokens) {
        int rc = o.model != MODEL_BPE ? wordpiece_tokenize(o, p, all_tokens)
                 : o.heap_bytes && o.heap_ok && p.size() >= o.heap_bytes ? bpe_tokenize_heap(o, p, all_tokens)
                                                                          : bpe_tokenize(o, p, all_tokens);
        if (rc) return rc;
    }
    const size_t n = all_tokens.size();
    if (full_encoding) {  // Encoding.fromTokens (encoding.zig:246-294)
        Encoding enc;
        enc.ids.resize(n); enc.type_ids.resize(n); enc.tokens.resize(n);
        enc.offsets.resize(n); enc.special_token_mask.resize(n); enc.attention_mask.resize(n);
        for (size_t k = 0; k < n; ++k) {
            const Tok& t = all_tokens[k];
            enc.ids[k] = t.id;
            enc.type_ids[k] = 0;
            enc.tokens[k] = std::string(t.value);
            enc.offsets[k] = ((uint64_t)t.end << 32) | t.start;
            enc.special_token_mask[k] = 0;
            enc.attention_mask[k] = 1;
        }
        for (size_t k = 0; k < n; ++k) {
            ids[k] = enc.ids[k];
            offs[2 * k] = (uint32_t)enc.offsets[k];
            offs[2 * k + 1] = (uint32_t)(enc.offsets[k] >> 32);
        }
    } else {
        for (size_t k = 0; k < n; ++k) {
            ids[k] = all_tokens[k].id;
            offs[2 * k] = all_tokens[k].start;
            offs[2 * k + 1] = all_tokens[k].end;
        }
    }
    *count = (uint32_t)n;
    return 0;
}

}  // namespace

extern "C" {

void* orc_create(int model, int norm, int pretok, const char* vocab_blob, const uint32_t* vocab_lens,
                 const uint32_t* vocab_ids, size_t n_vocab, const uint32_t* ma, const uint32_t* mb,
                 const uint32_t* mr, const uint32_t* mn, size_t n_merges, const char* unk, int64_t unk_len,
                 const char* prefix, size_t prefix_len, uint64_t max_chars) {
    Oracle* o = new Oracle();
    o->model = model; o->norm = norm; o->pretok = pretok;
    size_t total = 0;
    for (size_t i = 0; i < n_vocab; ++i) total += vocab_lens[i];
    o->pool.assign(vocab_blob, total);
    o->vocab.reserve(n_vocab * 2);
    size_t off = 0;
    for (size_t i = 0; i < n_vocab; ++i) {
        std::string_view k(o->pool.data() + off, vocab_lens[i]);
        off += vocab_lens[i];
        o->vocab[k] = vocab_ids[i];
    }
    for (auto& kv : o->vocab) o->vocab_r[kv.second] = kv.first;
    o->merges.reserve(n_merges * 2);
    for (size_t i = 0; i < n_merges; ++i) o->merges[((uint64_t)ma[i] << 32) | mb[i]] = PairVal{mr[i], mn[i]};
    // heap_ok: every merge ranks after every merge creating one of its parts (a token made
    // by several: the largest rank), so no merge creates its own part either
    std::unordered_map<uint32_t, uint64_t> made;  // token -> 1 + the largest rank creating it
    for (auto& kv : o->merges) { uint64_t& r = made[kv.second.new_id]; r = std::max<uint64_t>(r, kv.second.rank + 1ull); }
    o->heap_ok = true;
    for (auto& kv : o->merges)
        for (uint32_t part : {(uint32_t)(kv.first >> 32), (uint32_t)kv.first}) {
            auto it = made.find(part);
            if (it != made.end() && it->second > kv.second.rank) o->heap_ok = false;
        }
    if (unk_len >= 0) { o->has_unk = true; o->unk.assign(unk, (size_t)unk_len); }
    o->prefix.assign(prefix, prefix_len);
    o->max_chars = max_chars;
    return o;
}

void orc_destroy(void* h) { delete (Oracle*)h; }

// BPE pretokens of >= min_bytes bytes take bpe_tokenize_heap (0: never, the default).
// Returns 1 if the merge table allows it (heap_ok), else 0 (and the literal loop stays).
int orc_set_heap(void* h, uint64_t min_bytes) {
    Oracle* o = (Oracle*)h;
    o->heap_bytes = min_bytes;
    return o->heap_ok ? 1 : 0;
}

// Encodes docs [doc_off[i], doc_off[i+1]) of `bytes`. Doc i's tokens are written in a
// bound layout at ids[doc_off[i] ...] / offs[2*doc_off[i] ...] (tokens <= bytes), and its
// count at counts[i]. Returns 0, or 1 on error.MissingUnkToken.
int orc_encode_batch(void* h, const void* bytes, const uint64_t* doc_off, size_t n_docs, uint32_t* counts,
                     uint32_t* ids, uint32_t* offs, int n_threads, int full_encoding) {
    const Oracle& o = *(const Oracle*)h;
    const uint8_t* b = (const uint8_t*)bytes;
    if (n_threads < 1) n_threads = 1;
    std::vector<int> rcs(n_threads, 0);
    // docs handed out in blocks of 64 from a shared counter (Zipf doc lengths: a static
    // split left one thread with the longest docs)
    std::atomic<size_t> next{0};
    auto work = [&](int t) {
        for (;;) {
            const size_t lo = next.fetch_add(64), hi = std::min(n_docs, lo + 64);
            if (lo >= n_docs) return;
            for (size_t d = lo; d < hi; ++d) {
                uint64_t s = doc_off[d], e = doc_off[d + 1];
                int rc = encode_doc(o, b + s, e - s, ids + s, offs + 2 * s, counts + d, full_encoding);
                if (rc) { rcs[t] = rc; return; }
            }
        }
    };
    if (n_threads == 1) {
        work(0);
    } else {
        std::vector<std::thread> th;
        for (int t = 0; t < n_threads; ++t) th.emplace_back(work, t);
        for (auto& x : th) x.join();
    }
    for (int rc : rcs) if (rc) return rc;
    return 0;
}

}  // extern "C"
