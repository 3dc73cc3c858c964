// Blocks of one wave per CU that the occupancy calculator allows for a given LDS size per
// block (the LDS allocation granularity of gfx950 decides k_encode's occupancy).
// build: hipcc --offload-arch=gfx950 -O2 tools/lds_occupancy.hip -o tools/lds_occupancy
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(64) void k_probe(int* out) {
    extern __shared__ int s[];
    s[threadIdx.x] = threadIdx.x;
    __syncthreads();
    if (out) out[threadIdx.x] = s[63 - threadIdx.x];
}

int main() {
    for (int b = 6144; b <= 10240; b += 128) {
        int per = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_probe, 64, (size_t)b) != hipSuccess) return 1;
        printf("%d B/block: %d blocks/CU\n", b, per);
    }
    return 0;
}
