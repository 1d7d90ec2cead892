// Probe: achievable HBM rates of the embedding kernels' access patterns on gfx950 (16-B lanes):
//   mode 0: 1 stream read -> 2 streams written (the embedding forward: row in, out + LN(out) written)
//   mode 1: 4 streams read -> 1 written (the embedding backward: row, dout, dln, ... in, d_rows out)
//   mode 2: read only (sum kept in a register, one store per thread)      mode 3: write only
//   nt = 1: non-temporal stores.  One-shot grid of `per` float4 per thread, or grid-stride with `blocks` blocks.
#include <hip/hip_runtime.h>
#include <stdint.h>

template <int MODE, bool NT>
__global__ __launch_bounds__(256) void stream_kernel(const float4* __restrict__ a, const float4* __restrict__ b,
                                                     const float4* __restrict__ c, const float4* __restrict__ d,
                                                     float4* __restrict__ o1, float4* __restrict__ o2, int64_t n,
                                                     int per) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        float4 v = a[i];
        if (MODE == 1) {
            const float4 x = b[i], y = c[i], z = d[i];
            v.x += x.x + y.x + z.x; v.y += x.y + y.y + z.y; v.z += x.z + y.z + z.z; v.w += x.w + y.w + z.w;
        }
        if (MODE == 3) v = make_float4((float)i, 0.f, 1.f, 2.f);
        if (MODE == 2) {
            if (v.x == 12345.f) o1[i] = v;
            continue;
        }
        if (NT) {
            typedef float f4 __attribute__((ext_vector_type(4)));
            __builtin_nontemporal_store(f4{v.x, v.y, v.z, v.w}, (f4*)(o1 + i));
            if (MODE == 0) __builtin_nontemporal_store(f4{v.y, v.x, v.w, v.z}, (f4*)(o2 + i));
        } else {
            o1[i] = v;
            if (MODE == 0) o2[i] = make_float4(v.y, v.x, v.w, v.z);
        }
    }
}

extern "C" int run_stream(int mode, int nt, int blocks, const void* a, const void* b, const void* c, const void* d,
                          void* o1, void* o2, int64_t n, hipStream_t s) {
    const float4 *A = (const float4*)a, *B = (const float4*)b, *C = (const float4*)c, *D = (const float4*)d;
    float4 *O1 = (float4*)o1, *O2 = (float4*)o2;
#define L(M, T) hipLaunchKernelGGL((stream_kernel<M, T>), dim3(blocks), dim3(256), 0, s, A, B, C, D, O1, O2, n, 1)
    switch (mode * 2 + nt) {
        case 0: L(0, false); break;
        case 1: L(0, true); break;
        case 2: L(1, false); break;
        case 3: L(1, true); break;
        case 4: L(2, false); break;
        case 5: L(2, true); break;
        case 6: L(3, false); break;
        default: L(3, true); break;
    }
    return hipGetLastError() == hipSuccess ? 0 : 1;
}
