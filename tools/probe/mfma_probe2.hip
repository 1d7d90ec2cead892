// Probe: f32 MFMA issue rate vs operand pattern (same / distinct A and B registers), no memory traffic.
#include <hip/hip_runtime.h>
#include <stdint.h>
typedef float floatx4 __attribute__((ext_vector_type(4)));
template <int NACC, int MODE>
__global__ __launch_bounds__(256) void probe2(float* out, int iters, float a0, float b0) {
    floatx4 acc[NACC];
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = floatx4{0.f, 0.f, 0.f, 0.f};
    float a[NACC], b[4];
#pragma unroll
    for (int i = 0; i < NACC; ++i) a[i] = a0 + threadIdx.x * (i + 1);
#pragma unroll
    for (int k = 0; k < 4; ++k) b[k] = b0 - threadIdx.x * (k + 3);
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int i = 0; i < NACC; ++i)
                acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32((MODE & 1) ? a[i] : a[0], (MODE & 2) ? b[k] : b[0],
                                                              acc[i], 0, 0, 0);
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
template <int NACC, int MODE>
void go(int blocks, int iters, float* out, hipStream_t s) {
    hipLaunchKernelGGL((probe2<NACC, MODE>), dim3(blocks), dim3(256), 0, s, out, iters, 1.f, 2.f);
}
extern "C" int run_probe2(int nacc, int mode, int blocks, int iters, float* out, void* stream) {
    hipStream_t s = (hipStream_t)stream;
    if (nacc == 8) {
        if (mode == 0) go<8, 0>(blocks, iters, out, s);
        if (mode == 1) go<8, 1>(blocks, iters, out, s);
        if (mode == 2) go<8, 2>(blocks, iters, out, s);
        if (mode == 3) go<8, 3>(blocks, iters, out, s);
    } else {
        if (mode == 0) go<16, 0>(blocks, iters, out, s);
        if (mode == 1) go<16, 1>(blocks, iters, out, s);
        if (mode == 2) go<16, 2>(blocks, iters, out, s);
        if (mode == 3) go<16, 3>(blocks, iters, out, s);
    }
    return (int)hipGetLastError();
}
