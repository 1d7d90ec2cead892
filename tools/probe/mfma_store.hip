// Probe: f32 MFMA stream (8 accumulators, 2 waves/SIMD) with a 16-B-per-lane store burst every TILE MFMAs.
#include <hip/hip_runtime.h>
#include <stdint.h>
typedef float floatx4 __attribute__((ext_vector_type(4)));
template <int MODE>
__global__ __launch_bounds__(256) void mfma_store(float* out, int tiles, float a0, float b0) {
    floatx4 acc[8];
    float a[8], b[4];
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = a0 + threadIdx.x * (i + 1);
#pragma unroll
    for (int k = 0; k < 4; ++k) b[k] = b0 - threadIdx.x * (k + 3);
    // each wave stores into its own 8 KB slice of a 4 MB buffer (L2 resident)
    float* dst = out + ((blockIdx.x * 4 + (threadIdx.x >> 6)) & 511) * 2048 + (threadIdx.x & 63) * 4;
    floatx4 keep[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) keep[i] = floatx4{a[i], b[0], 0.f, 1.f};
    for (int t = 0; t < tiles; ++t) {
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = floatx4{0.f, 0.f, 0.f, 0.f};
        for (int it = 0; it < 8; ++it) {
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[k], acc[i], 0, 0, 0);
        }
        if (MODE == 1) {  // store the accumulators
#pragma unroll
            for (int i = 0; i < 8; ++i) *reinterpret_cast<floatx4*>(dst + i * 256) = acc[i];
        } else if (MODE == 2) {  // copy then store
            floatx4 c[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                c[i] = acc[i];
                asm volatile("" : "+v"(c[i]));
            }
#pragma unroll
            for (int i = 0; i < 8; ++i) *reinterpret_cast<floatx4*>(dst + i * 256) = c[i];
        } else if (MODE == 3) {  // store unrelated registers, fold acc elsewhere
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                keep[i] += acc[i];
                *reinterpret_cast<floatx4*>(dst + i * 256) = keep[i] * 0.5f;
            }
        } else if (MODE == 5 || MODE == 6) {  // stream: every tile writes fresh memory (HBM write stream)
            const int64_t waves = (int64_t)gridDim.x * 4;
            const int64_t w = blockIdx.x * 4 + (threadIdx.x >> 6);
            // MODE 5: wave-private 8 KB blocks; MODE 6: 16 rows x 64 B pieces of a 2 KB-row matrix (GEMM C^T tile)
            const int64_t id = (int64_t)t * waves + w;
            float* d = MODE == 5 ? out + id * 2048 + (threadIdx.x & 63) * 4
                                 : out + ((id >> 2) * 16 + (threadIdx.x & 15)) * 512 + (id & 3) * 128 +
                                       ((threadIdx.x >> 4) & 3) * 4;
#pragma unroll
            for (int i = 0; i < 8; ++i) *reinterpret_cast<floatx4*>(d + (MODE == 5 ? i * 256 : i * 16)) = acc[i];
        } else if (MODE == 4) {  // no stores: fold
#pragma unroll
            for (int i = 0; i < 8; ++i) keep[i] += acc[i];
        }
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += keep[i][0] + keep[i][1] + acc[i][2] + acc[i][3];
    if (s == 12345.f) out[0] = s;
}
extern "C" int run_ms(int mode, int blocks, int tiles, float* out, void* stream) {
    hipStream_t s = (hipStream_t)stream;
    if (mode == 1) hipLaunchKernelGGL(mfma_store<1>, dim3(blocks), dim3(256), 0, s, out, tiles, 1.f, 2.f);
    if (mode == 2) hipLaunchKernelGGL(mfma_store<2>, dim3(blocks), dim3(256), 0, s, out, tiles, 1.f, 2.f);
    if (mode == 3) hipLaunchKernelGGL(mfma_store<3>, dim3(blocks), dim3(256), 0, s, out, tiles, 1.f, 2.f);
    if (mode == 5) hipLaunchKernelGGL(mfma_store<5>, dim3(blocks), dim3(256), 0, s, out, tiles, 1.f, 2.f);
    if (mode == 6) hipLaunchKernelGGL(mfma_store<6>, dim3(blocks), dim3(256), 0, s, out, tiles, 1.f, 2.f);
    if (mode == 4) hipLaunchKernelGGL(mfma_store<4>, dim3(blocks), dim3(256), 0, s, out, tiles, 1.f, 2.f);
    return (int)hipGetLastError();
}
