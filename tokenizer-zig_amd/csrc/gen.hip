// Device-side bench / test utilities (libtkzgen.so; not the encode path, not in tkz.h):
//  * the synthetic doc generator of synth.cpp (make_doc / make_word / doc_length) ported
//    to the GPU, byte-identical to the host generator: one thread per doc, each doc a
//    pure function of (config, seed, doc index) through the same SplitMix64 stream and
//    the same double-precision cdf searches (built with -ffp-contract=off, so every
//    product rounds exactly as on the host). A rank of a multi-GPU run generates its own
//    shard of the stream in HBM: no host staging beyond nothing at all (SURVEY §8(d):
//    "generate on device per shard").
//  * 64-bit rolling hashes of a device CSR result (tests/shard_hash.py's definition:
//    h = h * M + x mod 2^64 over the values in batch order), so a full-size result is
//    compared with the oracle's committed hashes without a host copy.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#include "gen.h"

namespace {

struct Rng {
    uint64_t s;
    __device__ explicit Rng(uint64_t seed) : s(seed) {}
    __device__ uint64_t next() {
        uint64_t z = (s += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    __device__ double uni() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
    __device__ uint32_t below(uint32_t n) { return (uint32_t)(((next() >> 32) * (uint64_t)n) >> 32); }
};

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return x;
}

constexpr int KIND_BERT = 2;

struct DevGen {
    const uint32_t* wcp;   // lexicon codepoints
    const uint32_t* woff;  // n_words + 1
    const double* wcdf;    // n_words
    const double* lcdf;    // n_len (Zipf lengths)
    uint32_t n_words;
    uint32_t n_len;
    int kind;
    int fixed_len;
    int zmin;
};

// std::lower_bound(cdf, cdf + n, u): first i with !(cdf[i] < u)
__device__ __forceinline__ uint32_t lower_bound(const double* cdf, uint32_t n, double u) {
    uint32_t lo = 0, len = n;
    while (len > 0) {
        const uint32_t half = len >> 1;
        if (cdf[lo + half] < u) { lo += half + 1; len -= half + 1; }
        else len = half;
    }
    return lo;
}

__device__ __forceinline__ uint32_t upper(uint32_t cp) {
    if (cp >= 'a' && cp <= 'z') return cp - 32;
    if (cp >= 0xE0 && cp <= 0xFE && cp != 0xF7) return cp - 32;
    if (cp >= 0x3B1 && cp <= 0x3C9 && cp != 0x3C2) return cp - 32;
    if (cp >= 0x430 && cp <= 0x44F) return cp - 32;
    return cp;
}

__device__ __forceinline__ uint32_t put_utf8(uint8_t* o, uint32_t cp) {
    if (cp < 0x80) { o[0] = (uint8_t)cp; return 1; }
    if (cp < 0x800) { o[0] = (uint8_t)(0xC0 | (cp >> 6)); o[1] = (uint8_t)(0x80 | (cp & 0x3F)); return 2; }
    if (cp < 0x10000) {
        o[0] = (uint8_t)(0xE0 | (cp >> 12)); o[1] = (uint8_t)(0x80 | ((cp >> 6) & 0x3F));
        o[2] = (uint8_t)(0x80 | (cp & 0x3F));
        return 3;
    }
    o[0] = (uint8_t)(0xF0 | (cp >> 18)); o[1] = (uint8_t)(0x80 | ((cp >> 12) & 0x3F));
    o[2] = (uint8_t)(0x80 | ((cp >> 6) & 0x3F)); o[3] = (uint8_t)(0x80 | (cp & 0x3F));
    return 4;
}

// synth.cpp make_word: one word (capitalisation, BERT digit, punctuation) into w; returns
// its byte length (<= 12 codepoints x 4 + digit + punct = 50)
__device__ uint32_t make_word(const DevGen& G, Rng& r, uint8_t* w) {
    const double u = r.uni() * G.wcdf[G.n_words - 1];
    uint32_t idx = lower_bound(G.wcdf, G.n_words, u);
    if (idx >= G.n_words) idx = G.n_words - 1;
    const uint32_t c0 = G.woff[idx], nc = G.woff[idx + 1] - c0;
    const bool cap = r.uni() < 0.10;
    const bool digit = (G.kind == KIND_BERT) && r.uni() < 0.01;
    const uint32_t dpos = digit ? r.below(nc + 1) : 0xFFFFFFFFu;
    uint32_t n = 0;
    for (uint32_t k = 0; k < nc; ++k) {
        if (k == dpos) w[n++] = (uint8_t)('0' + r.below(10));
        const uint32_t cp = G.wcp[c0 + k];
        n += put_utf8(w + n, (k == 0 && cap) ? upper(cp) : cp);
    }
    if (dpos == nc) w[n++] = (uint8_t)('0' + r.below(10));
    if (r.uni() < 0.03) {
        const char punct[] = ".,;:!?'\"()-";
        w[n++] = (uint8_t)punct[r.below(sizeof(punct) - 1)];
    }
    return n;
}

__global__ __launch_bounds__(256) void k_gen_len(DevGen G, uint64_t seed, uint64_t first_doc, uint64_t n,
                                                 uint64_t* __restrict__ len) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (G.fixed_len > 0) { len[i] = (uint64_t)G.fixed_len; return; }
    Rng r(mix64(seed ^ 0x4c454e) ^ mix64(first_doc + i + 1));  // synth.cpp doc_length
    const double u = r.uni() * G.lcdf[G.n_len - 1];
    uint32_t k = lower_bound(G.lcdf, G.n_len, u);
    if (k > G.n_len - 1) k = G.n_len - 1;
    len[i] = (uint64_t)(G.zmin + (int)k);
}

// exclusive scan of len[0..n) into off[1..n] (off[0] = 0), one block: chunks of 1024
__global__ __launch_bounds__(1024) void k_gen_scan(const uint64_t* __restrict__ len, uint64_t n,
                                                   uint64_t* __restrict__ off) {
    __shared__ uint64_t part[1024];
    const uint64_t per = (n + 1023) / 1024;
    const uint64_t a = min(n, per * threadIdx.x), b = min(n, a + per);
    uint64_t s = 0;
    for (uint64_t i = a; i < b; ++i) s += len[i];
    part[threadIdx.x] = s;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {  // Hillis-Steele inclusive scan of the parts
        const uint64_t v = threadIdx.x >= (unsigned)o ? part[threadIdx.x - o] : 0;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    uint64_t acc = part[threadIdx.x] - s;
    if (threadIdx.x == 0) off[0] = 0;
    for (uint64_t i = a; i < b; ++i) { acc += len[i]; off[i + 1] = acc; }
}

// synth.cpp make_doc: one thread per doc, bytes [off[i], off[i+1]) of out
__global__ __launch_bounds__(256) void k_gen_doc(DevGen G, uint64_t seed, uint64_t first_doc, uint64_t n,
                                                 const uint64_t* __restrict__ off, uint8_t* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t o = off[i];
    const uint32_t len = (uint32_t)(off[i + 1] - o);
    uint8_t* d = out + o;
    Rng r(mix64(seed) ^ mix64(first_doc + i + 0x1234567ull));
    uint32_t size = 0;
    uint8_t w[64];
    while (true) {
        const uint32_t wn = make_word(G, r, w);
        const double u = r.uni();
        const uint8_t sep = u < 0.93 ? ' ' : (u < 0.98 ? '\n' : '\t');
        if (size + wn > len) break;
        for (uint32_t k = 0; k < wn; ++k) d[size + k] = w[k];
        size += wn;
        if (size < len) d[size++] = sep;
    }
    for (; size < len; ++size) d[size] = ' ';
}

// ---------------------------------------------------------------------------- hashes
constexpr uint64_t HM = 0x100000001B3ull;

uint64_t mpow(uint64_t b, uint64_t e) {
    uint64_t r = 1;
    while (e) { if (e & 1) r *= b; b *= b; e >>= 1; }
    return r;
}
__device__ uint64_t dpow(uint64_t b, uint64_t e) {
    uint64_t r = 1;
    while (e) { if (e & 1) r *= b; b *= b; e >>= 1; }
    return r;
}
uint64_t inv64(uint64_t a) {  // a odd: Newton iteration for a^-1 mod 2^64
    uint64_t x = a;
    for (int k = 0; k < 6; ++k) x *= 2 - a * x;
    return x;
}

// acc += sum_i x_i * M^(n-1-i) (mod 2^64); thread t takes i = t, t + G, ... with the
// weight stepped by M^-G
template <class T>
__global__ __launch_bounds__(256) void k_hash(const T* __restrict__ x, uint64_t n, uint64_t minv_g,
                                              unsigned long long* __restrict__ acc) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t G = (uint64_t)gridDim.x * blockDim.x;
    uint64_t s = 0;
    if (t < n) {
        uint64_t w = dpow(HM, n - 1 - t);
        for (uint64_t i = t; i < n; i += G) {
            s += (uint64_t)x[i] * w;
            w *= minv_g;
        }
    }
    for (int o = 32; o > 0; o >>= 1) s += (uint64_t)__shfl_xor((long long)s, o, 64);
    if ((threadIdx.x & 63) == 0 && s) atomicAdd(acc, (unsigned long long)s);
}

template <class T>
hipError_t hash_array(const T* d, uint64_t n, uint64_t h0, unsigned long long* d_acc, hipStream_t st, uint64_t* out) {
    if (n == 0) { *out = h0; return hipSuccess; }
    hipError_t e = hipMemsetAsync(d_acc, 0, 8, st);
    if (e != hipSuccess) return e;
    const uint64_t grid = std::min<uint64_t>((n + 255) / 256, 2048);
    const uint64_t G = grid * 256;
    hipLaunchKernelGGL((k_hash<T>), dim3((unsigned)grid), dim3(256), 0, st, d, n, mpow(inv64(HM), G), d_acc);
    unsigned long long acc = 0;
    if ((e = hipMemcpyAsync(&acc, d_acc, 8, hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
    *out = h0 * mpow(HM, n) + (uint64_t)acc;
    return hipSuccess;
}

}  // namespace

struct tkz_gen {
    DevGen G;
    std::vector<void*> allocs;
};

extern "C" {

int tkz_gen_create(const int64_t* p, const uint32_t* wcp, const uint32_t* woff, const double* wcdf,
                   const double* lcdf, tkz_gen** out) {
    *out = nullptr;
    tkz_gen* g = new tkz_gen();
    g->G.kind = (int)p[0];
    g->G.fixed_len = (int)p[1];
    g->G.zmin = (int)p[2];
    g->G.n_words = (uint32_t)p[3];
    g->G.n_len = (uint32_t)p[5];
    auto up = [&](const void* src, size_t n, const void** dst) -> bool {
        void* d = nullptr;
        if (hipMalloc(&d, n ? n : 8) != hipSuccess) return false;
        g->allocs.push_back(d);
        if (n && hipMemcpy(d, src, n, hipMemcpyHostToDevice) != hipSuccess) return false;
        *dst = d;
        return true;
    };
    const size_t nw = (size_t)p[3], ncp = (size_t)p[4], nl = (size_t)p[5];
    if (!up(wcp, ncp * 4, (const void**)&g->G.wcp) || !up(woff, (nw + 1) * 4, (const void**)&g->G.woff) ||
        !up(wcdf, nw * 8, (const void**)&g->G.wcdf) || !up(lcdf, nl * 8, (const void**)&g->G.lcdf)) {
        tkz_gen_destroy(g);
        return 1;
    }
    *out = g;
    return 0;
}

void tkz_gen_destroy(tkz_gen* g) {
    if (!g) return;
    for (void* p : g->allocs) hipFree(p);
    delete g;
}

int tkz_gen_offsets(tkz_gen* g, uint64_t seed, uint64_t first_doc, uint64_t n_docs, uint64_t* d_doc_off,
                    uint64_t* total, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    uint64_t* d_len = nullptr;
    if (hipMallocAsync((void**)&d_len, (n_docs + 1) * 8, st) != hipSuccess) return 1;
    const uint64_t blocks = (n_docs + 255) / 256;
    if (blocks) hipLaunchKernelGGL(k_gen_len, dim3((unsigned)blocks), dim3(256), 0, st, g->G, seed, first_doc, n_docs, d_len);
    hipLaunchKernelGGL(k_gen_scan, dim3(1), dim3(1024), 0, st, (const uint64_t*)d_len, n_docs, d_doc_off);
    uint64_t t = 0;
    hipMemcpyAsync(&t, d_doc_off + n_docs, 8, hipMemcpyDeviceToHost, st);
    hipFreeAsync(d_len, st);
    if (hipStreamSynchronize(st) != hipSuccess || hipGetLastError() != hipSuccess) return 1;
    *total = t;
    return 0;
}

int tkz_gen_bytes(tkz_gen* g, uint64_t seed, uint64_t first_doc, uint64_t n_docs, const uint64_t* d_doc_off,
                  uint8_t* d_out, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    const uint64_t blocks = (n_docs + 255) / 256;
    if (blocks)
        hipLaunchKernelGGL(k_gen_doc, dim3((unsigned)blocks), dim3(256), 0, st, g->G, seed, first_doc, n_docs, d_doc_off,
                           d_out);
    if (hipStreamSynchronize(st) != hipSuccess || hipGetLastError() != hipSuccess) return 1;
    return 0;
}

int tkz_csr_hash_device(const uint64_t* d_row_ptr, uint64_t n_docs, const uint32_t* d_ids, const uint64_t* d_offsets,
                        uint64_t n_tokens, uint64_t out[3], void* stream) {
    hipStream_t st = (hipStream_t)stream;
    unsigned long long* acc = nullptr;
    if (hipMalloc((void**)&acc, 8) != hipSuccess) return 1;
    const uint64_t H0 = 0xCBF29CE484222325ull;
    hipError_t e = hash_array(d_row_ptr, n_docs + 1, H0, acc, st, &out[0]);
    if (e == hipSuccess) e = hash_array(d_ids, n_tokens, H0, acc, st, &out[1]);
    if (e == hipSuccess) e = hash_array(d_offsets, n_tokens, H0, acc, st, &out[2]);
    hipFree(acc);
    return e == hipSuccess ? 0 : 1;
}

}  // extern "C"
