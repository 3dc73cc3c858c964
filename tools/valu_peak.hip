// VALU issue-rate microbenchmark (gfx950): wave-level 32-bit integer VALU instructions per
// second with W waves per SIMD, for the issue-bound roofline of k_encode.
// Each lane runs 8 independent v_xad/v_xor chains (asm volatile keeps every instruction).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ __launch_bounds__(64) void k_valu(uint32_t* out, int iters) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            asm volatile("v_xad_u32 %0, %0, %1, %0" : "+v"(a0) : "v"(a1));
            asm volatile("v_xad_u32 %0, %0, %1, %0" : "+v"(a1) : "v"(a2));
            asm volatile("v_xad_u32 %0, %0, %1, %0" : "+v"(a2) : "v"(a3));
            asm volatile("v_xad_u32 %0, %0, %1, %0" : "+v"(a3) : "v"(a4));
            asm volatile("v_xad_u32 %0, %0, %1, %0" : "+v"(a4) : "v"(a5));
            asm volatile("v_xad_u32 %0, %0, %1, %0" : "+v"(a5) : "v"(a6));
            asm volatile("v_xad_u32 %0, %0, %1, %0" : "+v"(a6) : "v"(a7));
            asm volatile("v_xad_u32 %0, %0, %1, %0" : "+v"(a7) : "v"(a0));
        }
    }
    out[blockIdx.x * 64 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

int main() {
    int dev = 0, cus = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int iters = 4096;
    uint32_t* out;
    hipMalloc(&out, (size_t)cus * 4 * 16 * 64 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int w : {1, 2, 4, 5, 8, 16}) {
        const int blocks = cus * 4 * w;  // one-wave blocks: w waves per SIMD
        hipLaunchKernelGGL(k_valu, dim3(blocks), dim3(64), 0, 0, out, 16);
        hipEventRecord(e0);
        hipLaunchKernelGGL(k_valu, dim3(blocks), dim3(64), 0, 0, out, iters);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        const double inst = (double)blocks * iters * 64.0;  // wave-level VALU instructions
        printf("{\"waves_per_simd\": %d, \"ms\": %.4f, \"valu_wave_instr_per_s\": %.4e, \"per_simd_per_ns\": %.4f}\n", w, ms,
               inst / (ms * 1e-3), inst / (ms * 1e-3) / (cus * 4) / 1e9);
    }
    return 0;
}
