// Which SIMD does each wave of a 512-thread workgroup run on?  Prints HW_ID (SIMD_ID, WAVE_ID, CU_ID) per wave.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ __launch_bounds__(512) void probe(unsigned* out) {
    const unsigned hw = __builtin_amdgcn_s_getreg(4 | (0 << 6) | (31 << 11));  // HW_REG_HW_ID, all 32 bits
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 8 + (threadIdx.x >> 6)] = hw;
    __builtin_amdgcn_s_sleep(100);
}
int main() {
    unsigned* d;
    const int nb = 4;
    hipMalloc(&d, nb * 8 * 4);
    hipLaunchKernelGGL(probe, dim3(nb), dim3(512), 0, 0, d);
    unsigned h[nb * 8];
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    for (int b = 0; b < nb; ++b)
        for (int w = 0; w < 8; ++w) {
            const unsigned x = h[b * 8 + w];
            printf("block %d wave %d: raw %08x wave_id %u simd %u pipe %u cu %u sh %u se %u\n", b, w, x, x & 15,
                   (x >> 4) & 3, (x >> 6) & 3, (x >> 8) & 15, (x >> 12) & 1, (x >> 13) & 7);
        }
    return 0;
}
