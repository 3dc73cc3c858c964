// VALU issue-rate microbenchmark over k_encode's real op mix (gfx950): wave-level
// instructions per second for each opcode class, 8 independent chains per lane, with W
// waves per SIMD (one-wave blocks). Answers whether k_encode (≈ 800M VALU per C1 launch)
// is bound by VALU issue: VOP2 logic/add/shift, VOP3 3-operand ops, cndmask, compares,
// DPP adds and 32-bit multiplies. Output: one JSON line per (op, waves/SIMD).
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHAIN8(ASM)                                          \
    asm volatile(ASM : "+v"(a0) : "v"(a1)); asm volatile(ASM : "+v"(a1) : "v"(a2)); \
    asm volatile(ASM : "+v"(a2) : "v"(a3)); asm volatile(ASM : "+v"(a3) : "v"(a4)); \
    asm volatile(ASM : "+v"(a4) : "v"(a5)); asm volatile(ASM : "+v"(a5) : "v"(a6)); \
    asm volatile(ASM : "+v"(a6) : "v"(a7)); asm volatile(ASM : "+v"(a7) : "v"(a0));

#define CHAIN8C(ASM, ...)                                                              \
    asm volatile(ASM : "+v"(a0) : "v"(a1) : __VA_ARGS__); asm volatile(ASM : "+v"(a1) : "v"(a2) : __VA_ARGS__); \
    asm volatile(ASM : "+v"(a2) : "v"(a3) : __VA_ARGS__); asm volatile(ASM : "+v"(a3) : "v"(a4) : __VA_ARGS__); \
    asm volatile(ASM : "+v"(a4) : "v"(a5) : __VA_ARGS__); asm volatile(ASM : "+v"(a5) : "v"(a6) : __VA_ARGS__); \
    asm volatile(ASM : "+v"(a6) : "v"(a7) : __VA_ARGS__); asm volatile(ASM : "+v"(a7) : "v"(a0) : __VA_ARGS__);

#define KERNELC(NAME, ASM, ...)                                                               \
    __global__ __launch_bounds__(64) void NAME(uint32_t* out, int iters) {                     \
        uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, \
                 a6 = a0 + 6, a7 = a0 + 7;                                                     \
        for (int i = 0; i < iters; ++i) {                                                      \
            _Pragma("unroll") for (int k = 0; k < 8; ++k) { CHAIN8C(ASM, __VA_ARGS__) }               \
        }                                                                                      \
        out[blockIdx.x * 64 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;            \
    }

// 64-bit operands: v_lshl_add_u64 (address arithmetic)
__global__ __launch_bounds__(64) void k_lshladd64(uint32_t* out, int iters) {
    uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    for (int i = 0; i < iters; ++i) {
        _Pragma("unroll") for (int k = 0; k < 8; ++k) { CHAIN8("v_lshl_add_u64 %0, %0, 0, %1") }
    }
    out[blockIdx.x * 64 + threadIdx.x] = (uint32_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}

#define KERNEL(NAME, ASM)                                                                      \
    __global__ __launch_bounds__(64) void NAME(uint32_t* out, int iters) {                     \
        uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, \
                 a6 = a0 + 6, a7 = a0 + 7;                                                     \
        for (int i = 0; i < iters; ++i) {                                                      \
            _Pragma("unroll") for (int k = 0; k < 8; ++k) { CHAIN8(ASM) }                      \
        }                                                                                      \
        out[blockIdx.x * 64 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;            \
    }

KERNEL(k_and, "v_and_b32 %0, %0, %1")
KERNEL(k_add, "v_add_u32 %0, %0, %1")
KERNEL(k_lshr, "v_lshrrev_b32 %0, %1, %0")
KERNEL(k_xad, "v_xad_u32 %0, %0, %1, %0")
KERNEL(k_bfe, "v_bfe_u32 %0, %0, %1, 5")
KERNEL(k_align, "v_alignbyte_b32 %0, %0, %1, 3")
KERNEL(k_or3, "v_or3_b32 %0, %0, %1, %0")
KERNEL(k_mul, "v_mul_lo_u32 %0, %0, %1")
KERNEL(k_dpp, "v_add_u32_dpp %0, %1, %0 row_shr:1 row_mask:0xf bank_mask:0xf")
KERNEL(k_cnd, "v_cmp_gt_u32 vcc, %0, %1\n\tv_cndmask_b32 %0, %0, %1, vcc")
// encoding vs opcode: the same AND as VOP3 (8 B), with a 32-bit literal (VOP2 + literal,
// 8 B), with an inline constant (VOP2, 4 B); a 64-bit address add; cndmask on an SGPR-pair
// mask (VOP3); a VOP2 op interleaved with a SALU op
KERNEL(k_and64, "v_and_b32_e64 %0, %0, %1")
KERNEL(k_andlit, "v_and_b32 %0, 0x7f3a5c1d, %0")
KERNEL(k_andinl, "v_and_b32 %0, 63, %0")
KERNELC(k_cnd64, "v_cmp_gt_u32_e64 s[40:41], %0, %1\n\tv_cndmask_b32_e64 %0, %0, %1, s[40:41]", "s40", "s41")
KERNELC(k_and_salu, "v_and_b32 %0, %0, %1\n\ts_add_u32 s42, s42, 1", "s42", "scc")

typedef void (*kfn)(uint32_t*, int);

int main() {
    int dev = 0, cus = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int iters = 2048;
    uint32_t* out;
    hipMalloc(&out, (size_t)cus * 4 * 16 * 64 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    struct { const char* name; kfn f; int per; } ks[] = {
        {"v_and_b32", k_and, 1}, {"v_add_u32", k_add, 1}, {"v_lshrrev_b32", k_lshr, 1}, {"v_xad_u32", k_xad, 1},
        {"v_bfe_u32", k_bfe, 1}, {"v_alignbyte_b32", k_align, 1}, {"v_or3_b32", k_or3, 1}, {"v_mul_lo_u32", k_mul, 1},
        {"v_add_u32_dpp", k_dpp, 1}, {"v_cmp+v_cndmask", k_cnd, 2},
        {"v_and_b32_e64", k_and64, 1}, {"v_and_b32+literal", k_andlit, 1}, {"v_and_b32+inline", k_andinl, 1},
        {"v_lshl_add_u64", k_lshladd64, 1}, {"v_cmp_e64+v_cndmask_e64", k_cnd64, 2}, {"v_and+s_add (VALU count)", k_and_salu, 1}};
    for (auto& k : ks) {
        for (int w : {1, 2, 4, 5, 8}) {
            const int blocks = cus * 4 * w;
            hipLaunchKernelGGL(k.f, dim3(blocks), dim3(64), 0, 0, out, 16);
            hipEventRecord(e0);
            hipLaunchKernelGGL(k.f, dim3(blocks), dim3(64), 0, 0, out, iters);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            const double inst = (double)blocks * iters * 64.0 * k.per;  // wave-level VALU instructions
            printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"valu_wave_instr_per_s\": %.4e, "
                   "\"per_simd_per_ns\": %.4f}\n", k.name, w, ms, inst / (ms * 1e-3), inst / (ms * 1e-3) / (cus * 4) / 1e9);
        }
    }
    return 0;
}
