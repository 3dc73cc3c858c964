// Synthetic corpora and tokenizer.json builders for the bench configs C0..C4
// (SURVEY.md §8d). Deterministic: doc i of a config is a pure function of
// (config, seed, i), so any subset can be regenerated on the host for parity.
// Built as libtkzsynth.so; used by bench.py and tests (not by the encode path).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <mutex>
#include <queue>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace {

struct Rng {
    uint64_t s;
    explicit Rng(uint64_t seed) : s(seed) {}
    uint64_t next() {
        uint64_t z = (s += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    double uni() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
    uint32_t below(uint32_t n) { return (uint32_t)(((next() >> 32) * (uint64_t)n) >> 32); }
};

uint64_t mix64(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return x;
}

enum Kind { KIND_ASCII = 0, KIND_UTF8 = 1, KIND_BERT = 2 };

struct ConfigSpec {
    int kind;
    int fixed_len;      // >0: every doc exactly this many bytes
    int zmin, zmax;     // zipf length range when fixed_len == 0
    double zs;
    int model;          // 1 = BPE, 0 = WordPiece
    int vocab_size;
    const char* normalizer;    // JSON or "null"
    const char* pre_tokenizer; // JSON
    int lex;            // lexicon variant: 0 = the one the vocab is trained on, 1 = a disjoint one
    int vocab_cfg;      // config whose tokenizer.json this config uses
};

// C0..C4 = BASELINE.json configs; C5 = C1's text statistics and C1's vocab, but words drawn
// from a lexicon generated with another seed (the vocab never saw them: an honest case
// for the vocab-derived word memo); C6 = C1's docs and vocab under a ByteLevel
// pre_tokenizer, which the reference does not recognise (config.zig:387-402): every doc is
// ONE pretoken (lib.zig:121), as it is for most real BPE tokenizer.json files
// C7 = C1's docs under a BPE vocab of more than 65,535 ids and merges (trained on more of
// the same corpus): the wide id / rank tables (the reference's ids and ranks are u32,
// bpe.zig:30-33, config.zig:219)
// C8 = C1's docs and vocab plus an unk token under a Metaspace pre_tokenizer (a
// SentencePiece-style tokenizer.json): whole-doc pretokens where every space and newline is
// the unk symbol (bpe.zig:198-205) instead of a dropped char
// C9 = C7's docs and 106k-id vocab under ByteLevel: whole-doc pretokens with wide ids
// C10 = C1's text in Zipf(4 KB - 1 MB) docs under C6's ByteLevel tokenizer: whole-doc
// pretokens of up to 1 MB (verdict r5 item 1; mean ~188 KB)
// C11 = C5's docs (a lexicon disjoint from the vocab's) under C6's ByteLevel tokenizer:
// whole-doc pretokens whose words the segment memo and hot pairs rarely hold
constexpr int kNumConfigs = 12;
const ConfigSpec kSpecs[kNumConfigs] = {
    {KIND_ASCII, 256, 0, 0, 0.0, 1, 8000, "null", "{\"type\":\"Whitespace\"}", 0, 0},
    {KIND_ASCII, 512, 0, 0, 0.0, 1, 32000, "null", "{\"type\":\"Whitespace\"}", 0, 1},
    {KIND_UTF8, 512, 0, 0, 0.0, 1, 32000,
     "{\"type\":\"Lowercase\"}", "{\"type\":\"Whitespace\"}", 0, 2},
    {KIND_BERT, 512, 0, 0, 0.0, 0, 30000,
     "{\"type\":\"BertNormalizer\",\"clean_text\":true,\"handle_chinese_chars\":true,\"strip_accents\":null,\"lowercase\":true}",
     "{\"type\":\"BertPreTokenizer\"}", 0, 3},
    {KIND_ASCII, 0, 64, 4096, 1.0, 1, 50000, "null", "{\"type\":\"Whitespace\"}", 0, 4},
    {KIND_ASCII, 512, 0, 0, 0.0, 1, 32000, "null", "{\"type\":\"Whitespace\"}", 1, 1},
    {KIND_ASCII, 512, 0, 0, 0.0, 1, 32000, "null",
     "{\"type\":\"ByteLevel\",\"add_prefix_space\":false,\"trim_offsets\":true,\"use_regex\":true}", 0, 6},
    {KIND_ASCII, 512, 0, 0, 0.0, 1, 131072, "null", "{\"type\":\"Whitespace\"}", 0, 7},
    {KIND_ASCII, 512, 0, 0, 0.0, 1, 32000, "null",
     "{\"type\":\"Metaspace\",\"replacement\":\"\u2581\",\"prepend_scheme\":\"always\",\"split\":true}", 0, 8},
    {KIND_ASCII, 512, 0, 0, 0.0, 1, 131072, "null",
     "{\"type\":\"ByteLevel\",\"add_prefix_space\":false,\"trim_offsets\":true,\"use_regex\":true}", 0, 9},
    {KIND_ASCII, 0, 4096, 1048576, 1.0, 1, 32000, "null",
     "{\"type\":\"ByteLevel\",\"add_prefix_space\":false,\"trim_offsets\":true,\"use_regex\":true}", 0, 6},
    {KIND_ASCII, 512, 0, 0, 0.0, 1, 32000, "null",
     "{\"type\":\"ByteLevel\",\"add_prefix_space\":false,\"trim_offsets\":true,\"use_regex\":true}", 1, 6},
};
// the config whose corpus trains config cfg's vocab (C6 / C8: C1's; C9: C7's)
int train_cfg(int cfg) { return cfg == 6 || cfg == 8 ? 1 : cfg == 9 ? 7 : cfg; }

void put_utf8(std::string& s, uint32_t cp) {
    if (cp < 0x80) s.push_back((char)cp);
    else if (cp < 0x800) { s.push_back((char)(0xC0 | (cp >> 6))); s.push_back((char)(0x80 | (cp & 0x3F))); }
    else if (cp < 0x10000) {
        s.push_back((char)(0xE0 | (cp >> 12))); s.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
        s.push_back((char)(0x80 | (cp & 0x3F)));
    } else {
        s.push_back((char)(0xF0 | (cp >> 18))); s.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
        s.push_back((char)(0x80 | ((cp >> 6) & 0x3F))); s.push_back((char)(0x80 | (cp & 0x3F)));
    }
}

const char kLetters[] = "etaoinshrdlcumwfgypbvkjxqz";
const double kLetterFreq[] = {12.7, 9.1, 8.2, 7.5, 7.0, 6.7, 6.3, 6.1, 6.0, 4.3, 4.0, 2.8, 2.8,
                              2.4,  2.4, 2.2, 2.0, 2.0, 1.9, 1.5, 1.0, 0.8, 0.15, 0.15, 0.1, 0.07};

struct Lexicon {
    std::vector<std::vector<uint32_t>> words;  // codepoints, lowercase forms
    std::vector<double> cdf;                   // Zipf(1.07) over ranks
    double letter_cdf[26];
};

uint32_t pick_letter(const Lexicon& L, Rng& r) {
    double u = r.uni() * L.letter_cdf[25];
    int k = 0;
    while (k < 25 && u >= L.letter_cdf[k]) ++k;
    return (uint32_t)kLetters[k];
}

uint32_t pick_char(const Lexicon& L, int kind, Rng& r) {
    if (kind != KIND_UTF8) return pick_letter(L, r);
    double u = r.uni();
    if (u < 0.75) return pick_letter(L, r);
    if (u < 0.90) {
        uint32_t k = r.below(3);
        if (k == 0) { uint32_t c = 0xE0 + r.below(31); return c == 0xF7 ? 0xE9 : c; }  // Latin-1 lowercase
        if (k == 1) { uint32_t c = 0x3B1 + r.below(25); return c == 0x3C2 ? 0x3C3 : c; }  // Greek lowercase
        return 0x430 + r.below(32);                                                     // Cyrillic lowercase
    }
    if (u < 0.98) return 0x4E00 + r.below(400);  // CJK
    return 0x1F600 + r.below(64);                // emoji (4-byte)
}

const Lexicon& lexicon(int kind, int variant) {
    static std::mutex mu;
    static std::map<int, Lexicon*> cache;
    std::lock_guard<std::mutex> g(mu);
    const int key = kind * 16 + variant;
    auto it = cache.find(key);
    if (it != cache.end()) return *it->second;
    Lexicon* L = new Lexicon();
    double acc = 0;
    for (int i = 0; i < 26; ++i) { acc += kLetterFreq[i]; L->letter_cdf[i] = acc; }
    Rng r(0x6c6578696300ull + (uint64_t)kind + 0x9E3779B97F4A7C15ull * (uint64_t)variant);
    const int N = 50000;
    L->words.resize(N);
    for (int w = 0; w < N; ++w) {
        int len = 2;
        while (len < 12 && r.uni() > 0.3) ++len;  // geometric on [2,12]
        for (int k = 0; k < len; ++k) L->words[w].push_back(pick_char(*L, kind, r));
    }
    L->cdf.resize(N);
    acc = 0;
    for (int w = 0; w < N; ++w) { acc += 1.0 / std::pow((double)(w + 1), 1.07); L->cdf[w] = acc; }
    cache[key] = L;
    return *L;
}

uint32_t upper(uint32_t cp) {
    if (cp >= 'a' && cp <= 'z') return cp - 32;
    if (cp >= 0xE0 && cp <= 0xFE && cp != 0xF7) return cp - 32;
    if (cp >= 0x3B1 && cp <= 0x3C9 && cp != 0x3C2) return cp - 32;
    if (cp >= 0x430 && cp <= 0x44F) return cp - 32;
    return cp;
}

// Appends one word (with optional capitalisation / punctuation / OOV digit) to `w`.
void make_word(const Lexicon& L, int kind, Rng& r, std::string& w) {
    double u = r.uni() * L.cdf.back();
    size_t idx = std::lower_bound(L.cdf.begin(), L.cdf.end(), u) - L.cdf.begin();
    if (idx >= L.words.size()) idx = L.words.size() - 1;
    const auto& cps = L.words[idx];
    bool cap = r.uni() < 0.10;
    bool digit = (kind == KIND_BERT) && r.uni() < 0.01;
    size_t dpos = digit ? r.below((uint32_t)cps.size() + 1) : (size_t)-1;
    for (size_t k = 0; k < cps.size(); ++k) {
        if (k == dpos) w.push_back((char)('0' + r.below(10)));
        put_utf8(w, (k == 0 && cap) ? upper(cps[k]) : cps[k]);
    }
    if (dpos == cps.size()) w.push_back((char)('0' + r.below(10)));
    if (r.uni() < 0.03) {
        static const char kPunct[] = ".,;:!?'\"()-";
        w.push_back(kPunct[r.below(sizeof(kPunct) - 1)]);
    }
}

uint32_t doc_length(const ConfigSpec& c, uint64_t seed, uint64_t d) {
    if (c.fixed_len > 0) return (uint32_t)c.fixed_len;
    static std::mutex mu;
    static std::map<std::pair<int, int>, std::vector<double>*> cache;
    std::vector<double>* cdf;
    {
        std::lock_guard<std::mutex> g(mu);
        auto& slot = cache[{c.zmin, c.zmax}];
        if (!slot) {
            slot = new std::vector<double>();
            double acc = 0;
            for (int l = c.zmin; l <= c.zmax; ++l) { acc += 1.0 / std::pow((double)l, c.zs); slot->push_back(acc); }
        }
        cdf = slot;
    }
    Rng r(mix64(seed ^ 0x4c454e) ^ mix64(d + 1));
    double u = r.uni() * cdf->back();
    size_t k = std::lower_bound(cdf->begin(), cdf->end(), u) - cdf->begin();
    return (uint32_t)(c.zmin + std::min(k, (size_t)(c.zmax - c.zmin)));
}

void make_doc(const ConfigSpec& c, uint64_t seed, uint64_t d, uint32_t len, uint8_t* out) {
    const Lexicon& L = lexicon(c.kind, c.lex);
    Rng r(mix64(seed) ^ mix64(d + 0x1234567ull));
    std::string doc, w;
    doc.reserve(len + 64);
    while (true) {
        w.clear();
        make_word(L, c.kind, r, w);
        char sep;
        double u = r.uni();
        sep = u < 0.93 ? ' ' : (u < 0.98 ? '\n' : '\t');
        if (doc.size() + w.size() > len) break;
        doc += w;
        if (doc.size() < len) doc.push_back(sep);
    }
    while (doc.size() < len) doc.push_back(' ');
    memcpy(out, doc.data(), len);
}

// ------------------------------------------------------------------ trainers

std::string json_escape(const std::string& s) {
    std::string o;
    o.push_back('"');
    for (unsigned char ch : s) {
        if (ch == '"') o += "\\\"";
        else if (ch == '\\') o += "\\\\";
        else if (ch < 0x20) { char buf[8]; snprintf(buf, sizeof buf, "\\u%04x", ch); o += buf; }
        else o.push_back((char)ch);
    }
    o.push_back('"');
    return o;
}

bool ws_delim(uint8_t c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }
bool punct(uint8_t c) { return (c >= 33 && c <= 47) || (c >= 58 && c <= 64) || (c >= 91 && c <= 96) || (c >= 123 && c <= 126); }

// Pretoken counts of a training corpus (seed distinct from every bench seed).
std::unordered_map<std::string, uint64_t> train_words(int cfg, size_t n_docs) {
    const ConfigSpec& c = kSpecs[cfg];
    const uint32_t len = 512;
    std::vector<uint8_t> buf(len);
    std::unordered_map<std::string, uint64_t> counts;
    const bool lower = c.kind != KIND_ASCII;  // C2 Lowercase, C3 BertNormalizer
    for (size_t d = 0; d < n_docs; ++d) {
        make_doc(c, 0x747261696eull + cfg, d, len, buf.data());
        if (lower) for (auto& b : buf) if (b >= 'A' && b <= 'Z') b |= 0x20;
        size_t i = 0;
        while (i < len) {
            if (c.kind == KIND_BERT) {
                if (ws_delim(buf[i])) { ++i; continue; }
                if (punct(buf[i])) { counts[std::string(1, (char)buf[i])]++; ++i; continue; }
                size_t j = i;
                while (j < len && !ws_delim(buf[j]) && !punct(buf[j])) ++j;
                counts[std::string((const char*)&buf[i], j - i)]++;
                i = j;
            } else {
                if (ws_delim(buf[i])) { ++i; continue; }
                size_t j = i;
                while (j < len && !ws_delim(buf[j])) ++j;
                counts[std::string((const char*)&buf[i], j - i)]++;
                i = j;
            }
        }
    }
    return counts;
}

std::vector<std::string> split_chars(const std::string& w) {
    std::vector<std::string> out;
    size_t i = 0;
    while (i < w.size()) {
        uint8_t b = (uint8_t)w[i];
        size_t l = b < 0x80 ? 1 : (b < 0xE0 ? 2 : (b < 0xF0 ? 3 : 4));
        out.push_back(w.substr(i, l));
        i += l;
    }
    return out;
}

// BPE tokenizer.json trained on config `cfg`'s corpus; the pre_tokenizer of config
// `pretok_cfg` (C6: C1's vocab and merges under ByteLevel); `unk`: an unk_token appended to
// the vocab (in no merge) or null
std::string bpe_json(int cfg, int pretok_cfg, const char* unk = nullptr) {
    const ConfigSpec& c = kSpecs[cfg];
    auto counts = train_words(cfg, c.vocab_size > 65536 ? 160000 : c.vocab_size >= 50000 ? 60000 : 12000);
    // deterministic order of word types
    std::vector<std::pair<std::string, uint64_t>> types(counts.begin(), counts.end());
    std::sort(types.begin(), types.end());
    std::unordered_map<std::string, uint32_t> vocab;
    std::vector<std::string> id2tok;
    std::map<std::string, uint64_t> char_freq;
    for (auto& t : types) for (auto& ch : split_chars(t.first)) char_freq[ch] += t.second;
    std::vector<std::pair<uint64_t, std::string>> chars;
    for (auto& kv : char_freq) chars.push_back({kv.second, kv.first});
    std::sort(chars.begin(), chars.end(), [](auto& a, auto& b) { return a.first != b.first ? a.first > b.first : a.second < b.second; });
    for (auto& ch : chars) { vocab[ch.second] = (uint32_t)id2tok.size(); id2tok.push_back(ch.second); }
    // words as symbol-id sequences
    std::vector<std::vector<uint32_t>> words(types.size());
    std::vector<uint64_t> wc(types.size());
    for (size_t i = 0; i < types.size(); ++i) {
        for (auto& ch : split_chars(types[i].first)) words[i].push_back(vocab[ch]);
        wc[i] = types[i].second;
    }
    auto key = [](uint32_t a, uint32_t b) { return ((uint64_t)a << 32) | b; };
    std::unordered_map<uint64_t, int64_t> pc;
    std::unordered_map<uint64_t, std::unordered_set<uint32_t>> where;
    for (uint32_t i = 0; i < words.size(); ++i)
        for (size_t k = 0; k + 1 < words[i].size(); ++k) {
            uint64_t p = key(words[i][k], words[i][k + 1]);
            pc[p] += (int64_t)wc[i];
            where[p].insert(i);
        }
    typedef std::pair<int64_t, uint64_t> HE;  // (count, ~pair) -> max count, then min pair
    std::priority_queue<HE> heap;
    for (auto& kv : pc) heap.push({kv.second, ~kv.first});
    std::vector<std::pair<uint32_t, uint32_t>> merges;
    while (id2tok.size() < (size_t)c.vocab_size && !heap.empty()) {
        HE top = heap.top();
        heap.pop();
        uint64_t p = ~top.second;
        auto it = pc.find(p);
        if (it == pc.end() || it->second != top.first) continue;  // stale
        if (top.first < 2) break;
        uint32_t a = (uint32_t)(p >> 32), b = (uint32_t)p;
        std::string m = id2tok[a] + id2tok[b];
        uint32_t nid;
        auto vit = vocab.find(m);
        if (vit == vocab.end()) { nid = (uint32_t)id2tok.size(); vocab[m] = nid; id2tok.push_back(m); }
        else nid = vit->second;
        merges.push_back({a, b});
        std::vector<uint32_t> ws(where[p].begin(), where[p].end());
        std::sort(ws.begin(), ws.end());
        std::unordered_map<uint64_t, int64_t> delta;
        for (uint32_t wi : ws) {
            auto& w = words[wi];
            int64_t cnt = (int64_t)wc[wi];
            for (size_t k = 0; k + 1 < w.size(); ++k) delta[key(w[k], w[k + 1])] -= cnt;
            std::vector<uint32_t> nw;
            for (size_t k = 0; k < w.size();) {
                if (k + 1 < w.size() && w[k] == a && w[k + 1] == b) { nw.push_back(nid); k += 2; }
                else { nw.push_back(w[k]); ++k; }
            }
            w.swap(nw);
            for (size_t k = 0; k + 1 < w.size(); ++k) {
                uint64_t q = key(w[k], w[k + 1]);
                delta[q] += cnt;
                where[q].insert(wi);
            }
        }
        for (auto& kv : delta) {
            if (kv.second == 0) continue;
            int64_t& v = pc[kv.first];
            v += kv.second;
            if (v > 0) heap.push({v, ~kv.first});
        }
        pc.erase(p);
    }
    if (unk) id2tok.push_back(unk);
    std::string j = "{\"version\":\"1.0\",\"truncation\":null,\"padding\":null,\"added_tokens\":[],\"normalizer\":";
    j += c.normalizer;
    j += ",\"pre_tokenizer\":";
    j += kSpecs[pretok_cfg].pre_tokenizer;
    j += ",\"post_processor\":null,\"decoder\":{\"type\":\"BPE\"},\"model\":{\"type\":\"BPE\",\"dropout\":null,"
         "\"unk_token\":";
    j += unk ? json_escape(unk) : std::string("null");
    j += ",\"continuing_subword_prefix\":null,\"end_of_word_suffix\":null,\"fuse_unk\":false,"
         "\"byte_fallback\":false,\"vocab\":{";
    for (size_t i = 0; i < id2tok.size(); ++i) {
        if (i) j.push_back(',');
        j += json_escape(id2tok[i]);
        j += ":" + std::to_string(i);
    }
    j += "},\"merges\":[";
    for (size_t i = 0; i < merges.size(); ++i) {
        if (i) j.push_back(',');
        j += json_escape(id2tok[merges[i].first] + " " + id2tok[merges[i].second]);
    }
    j += "]}}";
    return j;
}

std::string wordpiece_json(int cfg) {
    const ConfigSpec& c = kSpecs[cfg];
    auto counts = train_words(cfg, 12000);
    std::vector<std::pair<uint64_t, std::string>> types;
    for (auto& kv : counts) types.push_back({kv.second, kv.first});
    std::sort(types.begin(), types.end(), [](auto& a, auto& b) { return a.first != b.first ? a.first > b.first : a.second < b.second; });
    std::vector<std::string> toks = {"[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]"};
    std::unordered_set<std::string> have(toks.begin(), toks.end());
    auto add = [&](const std::string& t) { if (have.insert(t).second) toks.push_back(t); };
    std::map<std::string, uint64_t> charset;
    for (auto& t : types) for (auto& ch : split_chars(t.second)) charset[ch] += t.first;
    for (auto& kv : charset) {
        if (kv.first.size() == 1 && kv.first[0] >= '0' && kv.first[0] <= '9') continue;  // digits: OOV -> [UNK]
        add(kv.first);
        add("##" + kv.first);
    }
    const size_t n_words = (size_t)(c.vocab_size * 2 / 3);
    for (auto& t : types) {
        if (toks.size() >= n_words) break;
        bool has_digit = false;
        for (char ch : t.second) has_digit |= (ch >= '0' && ch <= '9');
        if (!has_digit) add(t.second);
    }
    std::unordered_map<std::string, uint64_t> suf;
    for (auto& t : types) {
        auto cs = split_chars(t.second);
        for (size_t s = 1; s < cs.size(); ++s) {
            std::string piece;
            for (size_t e = s; e < cs.size() && e < s + 6; ++e) {
                piece += cs[e];
                bool ok = true;
                for (char ch : piece) ok &= !(ch >= '0' && ch <= '9');
                if (ok && e > s) suf["##" + piece] += t.first;
            }
        }
    }
    std::vector<std::pair<uint64_t, std::string>> sv;
    for (auto& kv : suf) sv.push_back({kv.second, kv.first});
    std::sort(sv.begin(), sv.end(), [](auto& a, auto& b) { return a.first != b.first ? a.first > b.first : a.second < b.second; });
    for (auto& s : sv) { if (toks.size() >= (size_t)c.vocab_size) break; add(s.second); }
    std::string j = "{\"version\":\"1.0\",\"truncation\":null,\"padding\":null,\"added_tokens\":["
                    "{\"id\":0,\"content\":\"[PAD]\",\"single_word\":false,\"lstrip\":false,\"rstrip\":false,\"normalized\":false,\"special\":true},"
                    "{\"id\":1,\"content\":\"[UNK]\",\"single_word\":false,\"lstrip\":false,\"rstrip\":false,\"normalized\":false,\"special\":true},"
                    "{\"id\":2,\"content\":\"[CLS]\",\"single_word\":false,\"lstrip\":false,\"rstrip\":false,\"normalized\":false,\"special\":true},"
                    "{\"id\":3,\"content\":\"[SEP]\",\"single_word\":false,\"lstrip\":false,\"rstrip\":false,\"normalized\":false,\"special\":true},"
                    "{\"id\":4,\"content\":\"[MASK]\",\"single_word\":false,\"lstrip\":false,\"rstrip\":false,\"normalized\":false,\"special\":true}],"
                    "\"normalizer\":";
    j += c.normalizer;
    j += ",\"pre_tokenizer\":";
    j += c.pre_tokenizer;
    j += ",\"post_processor\":{\"type\":\"BertProcessing\",\"sep\":[\"[SEP]\",3],\"cls\":[\"[CLS]\",2]},"
         "\"decoder\":{\"type\":\"WordPiece\",\"prefix\":\"##\",\"cleanup\":true},"
         "\"model\":{\"type\":\"WordPiece\",\"unk_token\":\"[UNK]\",\"continuing_subword_prefix\":\"##\","
         "\"max_input_chars_per_word\":100,\"vocab\":{";
    for (size_t i = 0; i < toks.size(); ++i) {
        if (i) j.push_back(',');
        j += json_escape(toks[i]);
        j += ":" + std::to_string(i);
    }
    j += "}}}";
    return j;
}

}  // namespace

extern "C" {

// Number of bench configs (C0..C4).
int tkz_synth_num_configs(void) { return kNumConfigs; }

// Fills doc_off[0..n_docs] (relative to 0) for docs [first_doc, first_doc+n_docs) of
// config `cfg`; if `out` is non-null also writes the bytes. Returns total bytes.
uint64_t tkz_synth_docs(int cfg, uint64_t seed, uint64_t first_doc, uint64_t n_docs, uint8_t* out,
                        uint64_t* doc_off, int n_threads) {
    if (cfg < 0 || cfg >= kNumConfigs) return 0;
    const ConfigSpec& c = kSpecs[cfg];
    lexicon(c.kind, c.lex);
    doc_off[0] = 0;
    for (uint64_t i = 0; i < n_docs; ++i) doc_off[i + 1] = doc_off[i] + doc_length(c, seed, first_doc + i);
    if (out) {
        if (n_threads < 1) n_threads = 1;
        auto work = [&](int t) {
            uint64_t lo = n_docs * t / n_threads, hi = n_docs * (t + 1) / n_threads;
            for (uint64_t i = lo; i < hi; ++i)
                make_doc(c, seed, first_doc + i, (uint32_t)(doc_off[i + 1] - doc_off[i]), out + doc_off[i]);
        };
        std::vector<std::thread> th;
        for (int t = 1; t < n_threads; ++t) th.emplace_back(work, t);
        work(0);
        for (auto& x : th) x.join();
    }
    return doc_off[n_docs];
}

// Tables of the doc generator for the device port (gen.hip, tkz_gen_create): the config's
// parameters, its lexicon (codepoints of word w at wcp[woff[w] .. woff[w+1])), the
// Zipf(1.07) word cdf and the doc-length cdf (Zipf configs). Pass null arrays to get the
// sizes: p[0..5] = kind, fixed_len, zmin, n_words, n_cps, n_len. Returns 0 on success.
int tkz_synth_tables(int cfg, int64_t* p, uint32_t* wcp, uint32_t* woff, double* wcdf, double* lcdf) {
    if (cfg < 0 || cfg >= kNumConfigs) return 1;
    const ConfigSpec& c = kSpecs[cfg];
    const Lexicon& L = lexicon(c.kind, c.lex);
    uint64_t ncp = 0;
    for (auto& w : L.words) ncp += w.size();
    const int nl = c.fixed_len > 0 ? 0 : c.zmax - c.zmin + 1;
    p[0] = c.kind; p[1] = c.fixed_len; p[2] = c.zmin; p[3] = (int64_t)L.words.size(); p[4] = (int64_t)ncp; p[5] = nl;
    if (!wcp) return 0;
    uint64_t o = 0;
    for (size_t w = 0; w < L.words.size(); ++w) {
        woff[w] = (uint32_t)o;
        for (uint32_t cp : L.words[w]) wcp[o++] = cp;
        wcdf[w] = L.cdf[w];
    }
    woff[L.words.size()] = (uint32_t)o;
    if (nl) {
        doc_length(c, 0, 0);  // builds the cached cdf
        double acc = 0;  // the same sums as doc_length's cache, in the same order
        for (int l = c.zmin; l <= c.zmax; ++l) { acc += 1.0 / std::pow((double)l, c.zs); lcdf[l - c.zmin] = acc; }
    }
    return 0;
}

// Writes the tokenizer.json of config `cfg` into out (if cap is large enough).
// Returns the JSON length.
uint64_t tkz_synth_tokenizer_json(int cfg, char* out, uint64_t cap) {
    if (cfg < 0 || cfg >= kNumConfigs) return 0;
    cfg = kSpecs[cfg].vocab_cfg;
    static std::mutex mu;
    static std::map<int, std::string> cache;
    std::lock_guard<std::mutex> g(mu);
    auto it = cache.find(cfg);
    if (it == cache.end()) {
        std::string j = kSpecs[cfg].model == 1 ? bpe_json(train_cfg(cfg), cfg, cfg == 8 ? "<unk>" : nullptr)
                                                : wordpiece_json(cfg);
        it = cache.emplace(cfg, std::move(j)).first;
    }
    if (out && cap >= it->second.size()) memcpy(out, it->second.data(), it->second.size());
    return it->second.size();
}

}  // extern "C"
