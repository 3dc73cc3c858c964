// Minimal strict JSON DOM for tokenizer.json (RFC 8259). Objects keep document order
// (like std.json.ObjectMap, an array hash map). Restated from Zig 0.15 std.json, which
// config.zig:60 calls as parseFromSlice(std.json.Value, ..., .{}) and maps every error to
// ConfigError.InvalidJson (no reference test pins these two rules):
//  * a duplicate key in any object is an error: ParseOptions.duplicate_field_behavior
//    defaults to .@"error", and Value.jsonParse honours it (error.DuplicateField);
//  * string contents must be well-formed UTF-8 (std.json.Scanner validates every string
//    byte: no overlong forms, no encoded surrogates, nothing above U+10FFFF).
// Integers are JSON numbers without fraction/exponent that fit int64 (std.json's
// `.integer`); everything else numeric is a float (never a vocab id).
#pragma once
#include <cstdint>
#include <cstring>
#include <memory>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

namespace tkz {
namespace json {

struct Value;
using ValuePtr = std::unique_ptr<Value>;

enum class Type { Null, Bool, Integer, Float, String, Array, Object };

struct Value {
    Type type = Type::Null;
    bool b = false;
    int64_t i = 0;
    double f = 0;
    std::string s;
    std::vector<ValuePtr> arr;
    std::vector<std::pair<std::string, ValuePtr>> obj;   // document order
    std::unordered_map<std::string, size_t> index;       // key -> position in obj

    const Value* get(const char* key) const {
        auto it = index.find(key);
        return it == index.end() ? nullptr : obj[it->second].second.get();
    }
    bool is(Type t) const { return type == t; }
};

class Parser {
  public:
    Parser(const char* p, size_t n) : p_(p), end_(p + n) {}
    ValuePtr parse() {
        ws();
        ValuePtr v = value(0);
        if (!v) return nullptr;
        ws();
        if (p_ != end_) return nullptr;
        return v;
    }

  private:
    const char* p_;
    const char* end_;

    void ws() {
        while (p_ < end_ && (*p_ == ' ' || *p_ == '\t' || *p_ == '\n' || *p_ == '\r')) ++p_;
    }
    bool lit(const char* s) {
        size_t n = strlen(s);
        if ((size_t)(end_ - p_) < n || memcmp(p_, s, n) != 0) return false;
        p_ += n;
        return true;
    }
    // length of the well-formed UTF-8 sequence (lead byte >= 0x80) at q, 0 if ill-formed
    // (Unicode Table 3-7, the byte ranges std.json.Scanner accepts)
    static size_t utf8_len(const unsigned char* q, size_t avail) {
        const unsigned c = q[0];
        size_t n;
        unsigned lo = 0x80, hi = 0xBF;
        if (c >= 0xC2 && c <= 0xDF) n = 2;
        else if (c >= 0xE0 && c <= 0xEF) { n = 3; if (c == 0xE0) lo = 0xA0; if (c == 0xED) hi = 0x9F; }
        else if (c >= 0xF0 && c <= 0xF4) { n = 4; if (c == 0xF0) lo = 0x90; if (c == 0xF4) hi = 0x8F; }
        else return 0;
        if (avail < n || q[1] < lo || q[1] > hi) return 0;
        for (size_t k = 2; k < n; ++k)
            if (q[k] < 0x80 || q[k] > 0xBF) return 0;
        return n;
    }
    static void put_utf8(std::string& o, uint32_t cp) {
        if (cp < 0x80) o.push_back((char)cp);
        else if (cp < 0x800) { o.push_back((char)(0xC0 | (cp >> 6))); o.push_back((char)(0x80 | (cp & 0x3F))); }
        else if (cp < 0x10000) {
            o.push_back((char)(0xE0 | (cp >> 12))); o.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
            o.push_back((char)(0x80 | (cp & 0x3F)));
        } else {
            o.push_back((char)(0xF0 | (cp >> 18))); o.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
            o.push_back((char)(0x80 | ((cp >> 6) & 0x3F))); o.push_back((char)(0x80 | (cp & 0x3F)));
        }
    }
    bool hex4(uint32_t& v) {
        if (end_ - p_ < 4) return false;
        v = 0;
        for (int k = 0; k < 4; ++k) {
            char c = *p_++;
            v <<= 4;
            if (c >= '0' && c <= '9') v |= (uint32_t)(c - '0');
            else if (c >= 'a' && c <= 'f') v |= (uint32_t)(c - 'a' + 10);
            else if (c >= 'A' && c <= 'F') v |= (uint32_t)(c - 'A' + 10);
            else return false;
        }
        return true;
    }
    bool string(std::string& o) {
        if (p_ >= end_ || *p_ != '"') return false;
        ++p_;
        o.clear();
        while (true) {
            const char* q = p_;
            while (q < end_ && *q != '"' && *q != '\\' && (unsigned char)*q >= 0x20) {
                if ((unsigned char)*q < 0x80) { ++q; continue; }
                const size_t n = utf8_len((const unsigned char*)q, (size_t)(end_ - q));
                if (n == 0) return false;  // ill-formed UTF-8 in a string
                q += n;
            }
            o.append(p_, q);
            p_ = q;
            if (p_ >= end_) return false;
            char c = *p_;
            if (c == '"') { ++p_; return true; }
            if ((unsigned char)c < 0x20) return false;
            ++p_;  // backslash
            if (p_ >= end_) return false;
            char e = *p_++;
            switch (e) {
                case '"': o.push_back('"'); break;
                case '\\': o.push_back('\\'); break;
                case '/': o.push_back('/'); break;
                case 'b': o.push_back('\b'); break;
                case 'f': o.push_back('\f'); break;
                case 'n': o.push_back('\n'); break;
                case 'r': o.push_back('\r'); break;
                case 't': o.push_back('\t'); break;
                case 'u': {
                    uint32_t cp;
                    if (!hex4(cp)) return false;
                    if (cp >= 0xD800 && cp <= 0xDBFF) {
                        uint32_t lo;
                        if (end_ - p_ >= 6 && p_[0] == '\\' && p_[1] == 'u') {
                            p_ += 2;
                            if (!hex4(lo)) return false;
                            if (lo >= 0xDC00 && lo <= 0xDFFF) cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
                            else return false;
                        } else {
                            return false;  // lone high surrogate
                        }
                    } else if (cp >= 0xDC00 && cp <= 0xDFFF) {
                        return false;      // lone low surrogate
                    }
                    put_utf8(o, cp);
                    break;
                }
                default: return false;
            }
        }
    }
    ValuePtr number() {
        const char* s = p_;
        bool is_float = false;
        if (p_ < end_ && *p_ == '-') ++p_;
        if (p_ >= end_) return nullptr;
        if (*p_ == '0') ++p_;
        else if (*p_ >= '1' && *p_ <= '9') { while (p_ < end_ && *p_ >= '0' && *p_ <= '9') ++p_; }
        else return nullptr;
        if (p_ < end_ && *p_ == '.') {
            is_float = true; ++p_;
            if (p_ >= end_ || !(*p_ >= '0' && *p_ <= '9')) return nullptr;
            while (p_ < end_ && *p_ >= '0' && *p_ <= '9') ++p_;
        }
        if (p_ < end_ && (*p_ == 'e' || *p_ == 'E')) {
            is_float = true; ++p_;
            if (p_ < end_ && (*p_ == '+' || *p_ == '-')) ++p_;
            if (p_ >= end_ || !(*p_ >= '0' && *p_ <= '9')) return nullptr;
            while (p_ < end_ && *p_ >= '0' && *p_ <= '9') ++p_;
        }
        ValuePtr v(new Value());
        std::string tok(s, p_);
        if (!is_float) {
            // int64 range check
            bool neg = tok[0] == '-';
            const char* d = tok.c_str() + (neg ? 1 : 0);
            unsigned __int128 acc = 0;
            bool overflow = false;
            for (; *d; ++d) { acc = acc * 10 + (unsigned)(*d - '0'); if (acc > ((unsigned __int128)1 << 64)) { overflow = true; break; } }
            unsigned __int128 lim = neg ? ((unsigned __int128)1 << 63) : (((unsigned __int128)1 << 63) - 1);
            if (!overflow && acc <= lim) {
                v->type = Type::Integer;
                v->i = neg ? (int64_t)(0 - (uint64_t)acc) : (int64_t)(uint64_t)acc;
                return v;
            }
        }
        v->type = Type::Float;
        v->f = strtod(tok.c_str(), nullptr);
        return v;
    }
    ValuePtr value(int depth) {
        if (depth > 512 || p_ >= end_) return nullptr;
        char c = *p_;
        if (c == '{') {
            ++p_;
            ValuePtr v(new Value());
            v->type = Type::Object;
            ws();
            if (p_ < end_ && *p_ == '}') { ++p_; return v; }
            while (true) {
                ws();
                std::string k;
                if (!string(k)) return nullptr;
                ws();
                if (p_ >= end_ || *p_ != ':') return nullptr;
                ++p_;
                ws();
                ValuePtr child = value(depth + 1);
                if (!child) return nullptr;
                if (v->index.count(k)) return nullptr;  // error.DuplicateField
                v->index.emplace(k, v->obj.size());
                v->obj.emplace_back(std::move(k), std::move(child));
                ws();
                if (p_ < end_ && *p_ == ',') { ++p_; continue; }
                if (p_ < end_ && *p_ == '}') { ++p_; return v; }
                return nullptr;
            }
        }
        if (c == '[') {
            ++p_;
            ValuePtr v(new Value());
            v->type = Type::Array;
            ws();
            if (p_ < end_ && *p_ == ']') { ++p_; return v; }
            while (true) {
                ws();
                ValuePtr child = value(depth + 1);
                if (!child) return nullptr;
                v->arr.push_back(std::move(child));
                ws();
                if (p_ < end_ && *p_ == ',') { ++p_; continue; }
                if (p_ < end_ && *p_ == ']') { ++p_; return v; }
                return nullptr;
            }
        }
        if (c == '"') {
            ValuePtr v(new Value());
            v->type = Type::String;
            if (!string(v->s)) return nullptr;
            return v;
        }
        if (c == 't') { if (!lit("true")) return nullptr; ValuePtr v(new Value()); v->type = Type::Bool; v->b = true; return v; }
        if (c == 'f') { if (!lit("false")) return nullptr; ValuePtr v(new Value()); v->type = Type::Bool; v->b = false; return v; }
        if (c == 'n') { if (!lit("null")) return nullptr; ValuePtr v(new Value()); v->type = Type::Null; return v; }
        if (c == '-' || (c >= '0' && c <= '9')) return number();
        return nullptr;
    }
};

inline ValuePtr parse(const char* p, size_t n) { return Parser(p, n).parse(); }

}  // namespace json
}  // namespace tkz
