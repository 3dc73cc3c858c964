// Calibration of the memory-side PMC byte counters (FETCH_SIZE / WRITE_SIZE and the
// TCC_EA0 request-size counters) on the access patterns of the encode kernels, against
// known byte counts (MI355X_MICROARCH.md §HBM: "Other access widths are uncalibrated:
// calibrate on a known byte count in your own access pattern").
//   rd8      coalesced 8 B/lane stream read (k_encode's input scan)
//   rd16     coalesced 16 B/lane stream read (the guide's calibrated case)
//   rand16   random 16-B loads over a 1-GiB table (HBM misses)
//   rand32m  random 32-B windows over a 24-MiB table (L2 misses, MALL-resident: the memo)
//   wr4      coalesced 4 B/lane stores (k_compact's ids)
//   wr8      coalesced 8 B/lane stores (k_compact's offsets)
//   wr1      coalesced 1 B/lane stores (the word-count bytes)
//   wr4s     4-B stores to every 6th u32 (word-bound scratch tokens)
//   wrseg4/8 one contiguous, not line-aligned segment per wave, 64 lanes per store
//            (k_compact: ids / offsets of a chunk at its token base)
// usage: fetch_calib  -> one JSON line per kernel: {kernel, bytes (nominal), ms}
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CHECK(x)                                                                  \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
            return 1;                                                             \
        }                                                                         \
    } while (0)

__global__ void rd8(const uint64_t* __restrict__ p, uint64_t n, uint64_t* __restrict__ sink) {
    uint64_t x = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        x ^= p[i];
    if (x == 0x1234567ull) sink[0] = x;
}
__global__ void rd16(const uint4* __restrict__ p, uint64_t n, uint64_t* __restrict__ sink) {
    uint32_t x = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 v = p[i];
        x ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (x == 0x1234567u) sink[0] = x;
}
__global__ void evict(const uint4* __restrict__ p, uint64_t n, uint64_t* __restrict__ sink) {
    uint32_t x = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        x ^= p[i].y;
    if (x == 0x1234567u) sink[0] = x;
}
__device__ __forceinline__ uint64_t mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
// n_probes random 16-B loads (window = 1) or 32-B windows (2) over slots of table (TAG
// only names the dispatch in the profile: 0 = rand16, 1 = MALL warm-up, 2 = rand32m)
template <int TAG>
__global__ void rand_rd(const uint4* __restrict__ p, uint64_t slots, uint64_t n_probes, int window,
                        uint64_t* __restrict__ sink) {
    uint32_t x = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_probes;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t s = mix(i * 0x9E3779B97F4A7C15ull + 1) % (slots - 1);
        const uint4 v = p[s];
        x ^= v.x ^ v.w;
        if (window == 2) {
            const uint4 w = p[s + 1];
            x ^= w.y ^ w.z;
        }
    }
    if (x == 0x1234567u) sink[0] = x;
}
template <class T>
__global__ void wr(T* __restrict__ p, uint64_t n, uint64_t stride) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        p[i * stride] = (T)(i | 1);
}

// k_compact's output pattern: each wave writes one contiguous segment of `len` elements at
// an element offset that is not line-aligned (segments tile the array), 64 lanes per store
template <class T>
__global__ void wr_seg(T* __restrict__ p, uint64_t n_seg, uint32_t len, uint32_t shift) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t w = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; w < n_seg; w += nw) {
        const uint64_t base = w * len + shift;
        for (uint32_t t = lane; t < len; t += 64u) p[base + t] = (T)(t | 1u);
    }
}

int main() {
    const uint64_t BIG = 1ull << 30;  // 1 GiB: past the 256-MiB MALL
    void *a, *b;
    uint64_t* sink;
    CHECK(hipMalloc(&a, BIG));
    CHECK(hipMalloc(&b, BIG));
    CHECK(hipMalloc(&sink, 64));
    CHECK(hipMemset(a, 1, BIG));
    CHECK(hipMemset(b, 2, BIG));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const dim3 G(256 * 32), B(256);
    const uint64_t small_slots = (24ull << 20) / 16;
    for (int rep = 0; rep < 2; ++rep) {  // rep 0 warms up (code, MALL state); rep 1 is reported
        auto run = [&](const char* name, double bytes, auto&& launch, bool cold = true) {
            // evict: stream over b so the next kernel starts from a cold MALL
            if (cold) hipLaunchKernelGGL(evict, G, B, 0, 0, (const uint4*)b, BIG / 16, sink);
            hipEventRecord(e0);
            launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            if (rep == 1) printf("{\"kernel\": \"%s\", \"bytes\": %.0f, \"ms\": %.4f}\n", name, bytes, ms);
        };
        run("rd8", (double)BIG, [&] { hipLaunchKernelGGL(rd8, G, B, 0, 0, (const uint64_t*)a, BIG / 8, sink); });
        run("rd16", (double)BIG, [&] { hipLaunchKernelGGL(rd16, G, B, 0, 0, (const uint4*)a, BIG / 16, sink); });
        const uint64_t np = 1ull << 24;
        run("rand16", (double)np * 16, [&] {
            hipLaunchKernelGGL(rand_rd<0>, G, B, 0, 0, (const uint4*)a, BIG / 16, np, 1, sink);
        });
        // the 24-MiB table: first touched once after the eviction (MALL-resident), then probed
        hipLaunchKernelGGL(evict, G, B, 0, 0, (const uint4*)b, BIG / 16, sink);
        hipLaunchKernelGGL(rand_rd<1>, G, B, 0, 0, (const uint4*)a, small_slots, np, 2, sink);
        run("rand32m", (double)np * 32, [&] {
            hipLaunchKernelGGL(rand_rd<2>, G, B, 0, 0, (const uint4*)a, small_slots, np, 2, sink);
        }, false);
        run("wr4", (double)BIG, [&] { hipLaunchKernelGGL(wr<uint32_t>, G, B, 0, 0, (uint32_t*)a, BIG / 4, 1); });
        run("wr8", (double)BIG, [&] { hipLaunchKernelGGL(wr<uint64_t>, G, B, 0, 0, (uint64_t*)a, BIG / 8, 1); });
        run("wr1", (double)BIG / 4, [&] { hipLaunchKernelGGL(wr<uint8_t>, G, B, 0, 0, (uint8_t*)a, BIG / 4, 1); });
        run("wr4s", (double)(BIG / 24) * 4, [&] {
            hipLaunchKernelGGL(wr<uint32_t>, G, B, 0, 0, (uint32_t*)a, BIG / 24, 6);
        });
        const uint32_t SEG = 1601;  // tokens of a k_compact chunk (C1: ~1700)
        const uint64_t n4 = (BIG / 4 - 64) / SEG, n8 = (BIG / 8 - 64) / SEG;
        run("wrseg4", (double)n4 * SEG * 4, [&] {
            hipLaunchKernelGGL(wr_seg<uint32_t>, G, B, 0, 0, (uint32_t*)a, n4, SEG, 3u);
        });
        run("wrseg8", (double)n8 * SEG * 8, [&] {
            hipLaunchKernelGGL(wr_seg<uint64_t>, G, B, 0, 0, (uint64_t*)a, n8, SEG, 3u);
        });
    }
    CHECK(hipDeviceSynchronize());
    return 0;
}
