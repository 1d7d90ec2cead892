// Probe: the linear kernel's LDS-operand MFMA loop alone (no global traffic, no barriers).
#include <hip/hip_runtime.h>
#include <stdint.h>
typedef float floatx4 __attribute__((ext_vector_type(4)));
constexpr int kLd = 36, kBM = 128;
__device__ __forceinline__ floatx4 mfma16(float a, float b, floatx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
template <int MODE>
__global__ __launch_bounds__(256) void probe(float* out, int iters) {
    __shared__ __attribute__((aligned(16))) float buf[2 * kBM * kLd];
    __shared__ __attribute__((aligned(16))) float buf2[2 * kBM * kLd];
    for (int i = threadIdx.x; i < 2 * kBM * kLd; i += 256) buf[i] = (float)(i % 13) * 0.01f;
    __syncthreads();
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c16 = lane & 15;
    floatx4 acc[2][8];
    for (int rt = 0; rt < 2; ++rt) for (int ct = 0; ct < 8; ++ct) acc[rt][ct] = floatx4{0.f, 0.f, 0.f, 0.f};
    const float* Xs = buf;
    const float* Ws = buf + kBM * kLd;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            float4 xb[2], wa[8];
#pragma unroll
            for (int rt = 0; rt < 2; ++rt)
                xb[rt] = *reinterpret_cast<const float4*>(Xs + (wave * 32 + rt * 16 + c16) * kLd + 16 * h + 4 * g);
#pragma unroll
            for (int ct = 0; ct < 8; ++ct)
                wa[ct] = *reinterpret_cast<const float4*>(Ws + (ct * 16 + c16) * kLd + 16 * h + 4 * g);
#pragma unroll
            for (int ct = 0; ct < 8; ++ct)
#pragma unroll
                for (int rt = 0; rt < 2; ++rt) acc[rt][ct] = mfma16(wa[ct].x, xb[rt].x, acc[rt][ct]);
#pragma unroll
            for (int ct = 0; ct < 8; ++ct)
#pragma unroll
                for (int rt = 0; rt < 2; ++rt) acc[rt][ct] = mfma16(wa[ct].y, xb[rt].y, acc[rt][ct]);
#pragma unroll
            for (int ct = 0; ct < 8; ++ct)
#pragma unroll
                for (int rt = 0; rt < 2; ++rt) acc[rt][ct] = mfma16(wa[ct].z, xb[rt].z, acc[rt][ct]);
#pragma unroll
            for (int ct = 0; ct < 8; ++ct)
#pragma unroll
                for (int rt = 0; rt < 2; ++rt) acc[rt][ct] = mfma16(wa[ct].w, xb[rt].w, acc[rt][ct]);
        }
        if (MODE == 1) __syncthreads();
        if (MODE == 2) {
            float4 r = make_float4(it * 1.f, 2.f, 3.f, 4.f);
            const int c4 = (threadIdx.x & 7) * 4;
#pragma unroll
            for (int q = 0; q < 8; ++q)
                *reinterpret_cast<float4*>(buf2 + (((threadIdx.x >> 3) + 32 * (q & 3)) + 128 * (q >> 2)) * kLd + c4) = r;
            __syncthreads();
        }
    }
    float s = 0.f;
    for (int rt = 0; rt < 2; ++rt) for (int ct = 0; ct < 8; ++ct) s += acc[rt][ct][0] + acc[rt][ct][3];
    out[blockIdx.x * 256 + threadIdx.x] = s + buf2[threadIdx.x];
}
extern "C" int run_lds_probe(int mode, int blocks, int iters, float* out, void* stream) {
    if (mode == 0) hipLaunchKernelGGL(probe<0>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, out, iters);
    else if (mode == 1) hipLaunchKernelGGL(probe<1>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, out, iters);
    else hipLaunchKernelGGL(probe<2>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, out, iters);
    return (int)hipGetLastError();
}
