// Probe: f32 MFMA issue rate with N independent accumulators per wave, no memory traffic.
#include <hip/hip_runtime.h>
#include <stdint.h>
typedef float floatx4 __attribute__((ext_vector_type(4)));
template <int NACC>
__global__ __launch_bounds__(256) void probe(float* out, int iters, float a0, float b0) {
    floatx4 acc[NACC];
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = floatx4{0.f, 0.f, 0.f, 0.f};
    float a = a0 + threadIdx.x, b = b0 - threadIdx.x;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
extern "C" int run_probe(int nacc, int blocks, int iters, float* out, void* stream) {
    if (nacc == 4) hipLaunchKernelGGL(probe<4>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, out, iters, 1.f, 2.f);
    if (nacc == 8) hipLaunchKernelGGL(probe<8>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, out, iters, 1.f, 2.f);
    if (nacc == 16) hipLaunchKernelGGL(probe<16>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, out, iters, 1.f, 2.f);
    return (int)hipGetLastError();
}
