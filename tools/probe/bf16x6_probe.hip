// Precision / layout probe: fp32 GEMM tiles on bf16 MFMA with operands split into three bf16 terms
// (x = h + m + l exactly, products kept down to 2^-16 relative: hh, hm, mh, hl, lh, mm).
// C (16 x 16) = A (16 x K) . B (16 x K)^T per 64-thread block; modes: 0 fp32 16x16x4 MFMA, 1 bf16x6 one
// accumulator, 2 bf16x6 with the small terms in a second accumulator, 3 bf16x3 (hh, hm, mh).
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void split3(const float* x, bf16x8& h, bf16x8& m, bf16x8& l) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const __bf16 hb = (__bf16)x[j];
        const float r = x[j] - (float)hb;
        const __bf16 mb = (__bf16)r;
        const float r2 = r - (float)mb;
        h[j] = hb;
        m[j] = mb;
        l[j] = (__bf16)r2;
    }
}
#define MF(a, b, c) __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0)

__global__ void probe_kernel(const float* A, const float* B, float* C, int K, int mode) {
    const int lane = threadIdx.x, r = lane & 15, g = lane >> 4;
    const float* a = A + ((int64_t)blockIdx.x * 16 + r) * K;
    const float* b = B + ((int64_t)blockIdx.x * 16 + r) * K;
    floatx4 acc = {0.f, 0.f, 0.f, 0.f}, acs = acc;
    if (mode == 0) {
        for (int k = 0; k < K; k += 4) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[k + g], b[k + g], acc, 0, 0, 0);
    } else {
        for (int k = 0; k < K; k += 32) {
            bf16x8 ah, am, al, bh, bm, bl;
            split3(a + k + 8 * g, ah, am, al);
            split3(b + k + 8 * g, bh, bm, bl);
            if (mode == 1) {
                acc = MF(am, bm, acc);
                acc = MF(ah, bl, acc);
                acc = MF(al, bh, acc);
                acc = MF(ah, bm, acc);
                acc = MF(am, bh, acc);
                acc = MF(ah, bh, acc);
            } else if (mode == 2) {
                acs = MF(am, bm, acs);
                acs = MF(ah, bl, acs);
                acs = MF(al, bh, acs);
                acs = MF(ah, bm, acs);
                acs = MF(am, bh, acs);
                acc = MF(ah, bh, acc);
            } else {
                acc = MF(ah, bm, acc);
                acc = MF(am, bh, acc);
                acc = MF(ah, bh, acc);
            }
        }
    }
    // C/D: col = lane & 15 (B row), row = 4g + i (A row)
    for (int i = 0; i < 4; ++i)
        C[((int64_t)blockIdx.x * 16 + 4 * g + i) * 16 + r] = acc[i] + acs[i];
}

extern "C" int run_probe(const float* A, const float* B, float* C, int tiles, int K, int mode, void* stream) {
    hipLaunchKernelGGL(probe_kernel, dim3(tiles), dim3(64), 0, (hipStream_t)stream, A, B, C, K, mode);
    return (int)hipGetLastError();
}
