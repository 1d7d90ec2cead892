// Pointwise/normalisation kernels of the ASME transformer block on gfx950 (fp32).
//
// Reference semantics (paths relative to /root/reference/src/asme):
//   SublayerConnection.forward   core/models/common/layers/transformer_layers.py:120-130
//        x + dropout(sublayer(LN(x)))         (pre-LN)
//   TransformerBlock.forward     transformer_layers.py:251-258  (block-level dropout at the end)
//   PositionwiseFeedForward      transformer_layers.py:217-220  W2(dropout(GELU_erf(W1 x)))
//   FFN modifier                 core/models/common/components/representation_modifier/ffn_modifier.py:24-26
//
// The residual kernel fuses one sublayer's epilogue with the NEXT LayerNorm:
//     s   = dropout_b( res + dropout_a(y) )      (stream value, the residual for the next sublayer)
//     out = LN(s)                                (input of the next sublayer; optional)
// so a transformer block costs two of these plus the GEMMs and the attention kernel.
#include "common.h"

using namespace asme;

namespace {
constexpr int kWaves = 4;

template <int VPL>
__device__ __forceinline__ void row_ln(float (&x)[VPL], int lane, int D, float eps, const float* w, const float* b,
                                       float (&y)[VPL], float& mean, float& rstd) {
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < VPL; ++j) s += (lane + 64 * j < D) ? x[j] : 0.f;
    mean = wave_sum(s) / (float)D;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
        const float c = (lane + 64 * j < D) ? x[j] - mean : 0.f;
        q += c * c;
    }
    rstd = rsqrtf(wave_sum(q) / (float)D + eps);
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
        const int e = lane + 64 * j;
        y[j] = e < D ? (x[j] - mean) * rstd * w[e] + b[e] : 0.f;
    }
}

template <int VPL>
__device__ __forceinline__ void row_ln_bwd(const float (&gy)[VPL], const float (&xhat)[VPL], const float* w,
                                           float rstd, int lane, int D, float (&gx)[VPL]) {
    float a = 0.f, b = 0.f, dxh[VPL];
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
        const int e = lane + 64 * j;
        dxh[j] = e < D ? gy[j] * w[e] : 0.f;
        a += dxh[j];
        b += dxh[j] * xhat[j];
    }
    a = wave_sum(a) / (float)D;
    b = wave_sum(b) / (float)D;
#pragma unroll
    for (int j = 0; j < VPL; ++j) gx[j] = rstd * (dxh[j] - a - xhat[j] * b);
}

template <int VPL>
__device__ __forceinline__ void write_partials(float (&acc)[2][VPL], int lane, int wave, int D, float* partials) {
    extern __shared__ __attribute__((aligned(16))) float red[];  // [kWaves][2][D]
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
        for (int j = 0; j < VPL; ++j) {
            const int e = lane + 64 * j;
            if (e < D) red[(wave * 2 + k) * D + e] = acc[k][j];
        }
    __syncthreads();
    for (int c = threadIdx.x; c < 2 * D; c += blockDim.x) {
        float s = 0.f;
        for (int w = 0; w < kWaves; ++w) s += red[w * 2 * D + c];
        partials[(int64_t)blockIdx.x * 2 * D + c] = s;
    }
}

// ------------------------------------------------------------ plain LayerNorm
template <int VPL>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const float* __restrict__ x, int64_t T, int D,
                                                     const float* __restrict__ w, const float* __restrict__ b,
                                                     float eps, float* __restrict__ y, float* __restrict__ stats) {
    const int lane = threadIdx.x & 63;
    const int64_t t = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
    if (t >= T) return;
    float v[VPL], o[VPL], m, r;
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
        const int e = lane + 64 * j;
        v[j] = e < D ? x[t * D + e] : 0.f;
    }
    row_ln<VPL>(v, lane, D, eps, w, b, o, m, r);
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
        const int e = lane + 64 * j;
        if (e < D) y[t * D + e] = o[j];
    }
    if (lane == 0) {
        stats[t * 2] = m;
        stats[t * 2 + 1] = r;
    }
}

template <int VPL>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const float* __restrict__ x, int64_t T, int D,
                                                     const float* __restrict__ w, const float* __restrict__ stats,
                                                     const float* __restrict__ dy, float* __restrict__ dx,
                                                     int accumulate, float* __restrict__ partials) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    float acc[2][VPL];
#pragma unroll
    for (int j = 0; j < VPL; ++j) acc[0][j] = acc[1][j] = 0.f;
    for (int64_t t = (int64_t)blockIdx.x * kWaves + wave; t < T; t += (int64_t)gridDim.x * kWaves) {
        const float m = stats[t * 2], r = stats[t * 2 + 1];
        float xh[VPL], g[VPL], gx[VPL];
#pragma unroll
        for (int j = 0; j < VPL; ++j) {
            const int e = lane + 64 * j;
            xh[j] = e < D ? (x[t * D + e] - m) * r : 0.f;
            g[j] = e < D ? dy[t * D + e] : 0.f;
            acc[0][j] += g[j] * xh[j];
            acc[1][j] += g[j];
        }
        row_ln_bwd<VPL>(g, xh, w, r, lane, D, gx);
#pragma unroll
        for (int j = 0; j < VPL; ++j) {
            const int e = lane + 64 * j;
            if (e < D) dx[t * D + e] = accumulate ? dx[t * D + e] + gx[j] : gx[j];
        }
    }
    write_partials<VPL>(acc, lane, wave, D, partials);
}

// ------------------------------------------------------------ residual + dropout(s) + LayerNorm
template <int VPL>
__global__ __launch_bounds__(256) void residual_ln_fwd_kernel(
    const float* __restrict__ res, const float* __restrict__ y, int64_t T, int D, float pa, uint64_t sa, float pb,
    uint64_t sb, const float* __restrict__ w, const float* __restrict__ b, float eps, float* __restrict__ s_out,
    float* __restrict__ ln_out, float* __restrict__ stats) {
    const int lane = threadIdx.x & 63;
    const int64_t t = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
    if (t >= T) return;
    float v[VPL];
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
        const int e = lane + 64 * j;
        const uint64_t idx = (uint64_t)t * D + e;
        float a = e < D ? y[t * D + e] : 0.f;
        if (pa > 0.f) a *= dropout_factor(sa, 3u, idx, pa);
        float h = (e < D ? res[t * D + e] : 0.f) + a;
        if (pb > 0.f) h *= dropout_factor(sb, 4u, idx, pb);
        v[j] = h;
        if (e < D) s_out[t * D + e] = h;
    }
    if (w) {
        float o[VPL], m, r;
        row_ln<VPL>(v, lane, D, eps, w, b, o, m, r);
#pragma unroll
        for (int j = 0; j < VPL; ++j) {
            const int e = lane + 64 * j;
            if (e < D) ln_out[t * D + e] = o[j];
        }
        if (lane == 0) {
            stats[t * 2] = m;
            stats[t * 2 + 1] = r;
        }
    }
}

template <int VPL>
__global__ __launch_bounds__(256) void residual_ln_bwd_kernel(
    const float* __restrict__ s, int64_t T, int D, float pa, uint64_t sa, float pb, uint64_t sb,
    const float* __restrict__ w, const float* __restrict__ stats, const float* __restrict__ d_s,
    const float* __restrict__ d_ln, float* __restrict__ d_res, float* __restrict__ d_y,
    float* __restrict__ partials) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    float acc[2][VPL];
#pragma unroll
    for (int j = 0; j < VPL; ++j) acc[0][j] = acc[1][j] = 0.f;
    for (int64_t t = (int64_t)blockIdx.x * kWaves + wave; t < T; t += (int64_t)gridDim.x * kWaves) {
        float g[VPL];
#pragma unroll
        for (int j = 0; j < VPL; ++j) {
            const int e = lane + 64 * j;
            g[j] = (d_s && e < D) ? d_s[t * D + e] : 0.f;
        }
        if (w && d_ln) {
            const float m = stats[t * 2], r = stats[t * 2 + 1];
            float xh[VPL], gl[VPL], gx[VPL];
#pragma unroll
            for (int j = 0; j < VPL; ++j) {
                const int e = lane + 64 * j;
                xh[j] = e < D ? (s[t * D + e] - m) * r : 0.f;
                gl[j] = e < D ? d_ln[t * D + e] : 0.f;
                acc[0][j] += gl[j] * xh[j];
                acc[1][j] += gl[j];
            }
            row_ln_bwd<VPL>(gl, xh, w, r, lane, D, gx);
#pragma unroll
            for (int j = 0; j < VPL; ++j) g[j] += gx[j];
        }
#pragma unroll
        for (int j = 0; j < VPL; ++j) {
            const int e = lane + 64 * j;
            if (e >= D) continue;
            const uint64_t idx = (uint64_t)t * D + e;
            float dh = g[j];
            if (pb > 0.f) dh *= dropout_factor(sb, 4u, idx, pb);
            d_res[t * D + e] = dh;
            if (d_y) d_y[t * D + e] = pa > 0.f ? dh * dropout_factor(sa, 3u, idx, pa) : dh;
        }
    }
    if (partials) write_partials<VPL>(acc, lane, wave, D, partials);
}

// ------------------------------------------------------------ GELU(erf) + dropout, elementwise (float4)
__global__ __launch_bounds__(256) void gelu_dropout_fwd_kernel(const float* __restrict__ x, int64_t n, float p,
                                                               uint64_t seed, float* __restrict__ y) {
    const int64_t i4 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t i = i4 * 4;
    if (i >= n) return;
    if (i + 3 < n) {
        float4 v = *reinterpret_cast<const float4*>(x + i);
        float u[4] = {1.f, 1.f, 1.f, 1.f};
        if (p > 0.f) {
            philox_uniform4(seed, 5u, (uint64_t)i >> 2, u);
#pragma unroll
            for (int k = 0; k < 4; ++k) u[k] = u[k] >= p ? 1.f / (1.f - p) : 0.f;
        }
        float4 o;
        o.x = gelu_erf(v.x) * u[0];
        o.y = gelu_erf(v.y) * u[1];
        o.z = gelu_erf(v.z) * u[2];
        o.w = gelu_erf(v.w) * u[3];
        *reinterpret_cast<float4*>(y + i) = o;
    } else {
        for (int64_t k = i; k < n; ++k) y[k] = gelu_erf(x[k]) * (p > 0.f ? dropout_factor(seed, 5u, k, p) : 1.f);
    }
}

__global__ __launch_bounds__(256) void gelu_dropout_bwd_kernel(const float* __restrict__ x,
                                                               const float* __restrict__ dy, int64_t n, float p,
                                                               uint64_t seed, float* __restrict__ dx) {
    const int64_t i4 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t i = i4 * 4;
    if (i >= n) return;
    if (i + 3 < n) {
        float4 v = *reinterpret_cast<const float4*>(x + i);
        float4 g = *reinterpret_cast<const float4*>(dy + i);
        float u[4] = {1.f, 1.f, 1.f, 1.f};
        if (p > 0.f) {
            philox_uniform4(seed, 5u, (uint64_t)i >> 2, u);
#pragma unroll
            for (int k = 0; k < 4; ++k) u[k] = u[k] >= p ? 1.f / (1.f - p) : 0.f;
        }
        float4 o;
        o.x = g.x * u[0] * gelu_erf_grad(v.x);
        o.y = g.y * u[1] * gelu_erf_grad(v.y);
        o.z = g.z * u[2] * gelu_erf_grad(v.z);
        o.w = g.w * u[3] * gelu_erf_grad(v.w);
        *reinterpret_cast<float4*>(dx + i) = o;
    } else {
        for (int64_t k = i; k < n; ++k)
            dx[k] = dy[k] * (p > 0.f ? dropout_factor(seed, 5u, k, p) : 1.f) * gelu_erf_grad(x[k]);
    }
}

inline int vpl_of(int64_t D) { return (int)((D + 63) / 64); }

#define ASME_VPL_DISPATCH(VPLV, ...)                              \
    switch (VPLV) {                                               \
        case 1: { constexpr int VPL = 1; __VA_ARGS__; } break;    \
        case 2: { constexpr int VPL = 2; __VA_ARGS__; } break;    \
        case 3: { constexpr int VPL = 3; __VA_ARGS__; } break;    \
        case 4: { constexpr int VPL = 4; __VA_ARGS__; } break;    \
        case 5: { constexpr int VPL = 5; __VA_ARGS__; } break;    \
        case 6: { constexpr int VPL = 6; __VA_ARGS__; } break;    \
        case 7: { constexpr int VPL = 7; __VA_ARGS__; } break;    \
        case 8: { constexpr int VPL = 8; __VA_ARGS__; } break;    \
        default: set_error("hidden size must be in [1, 512]"); return -1; \
    }
}  // namespace

ASME_API int asme_layernorm_fwd(const float* x, int64_t n_rows, int64_t dim, const float* w, const float* b,
                                float eps, float* y, float* stats, void* stream) {
    ASME_CHECK_ARG(x && w && b && y && stats, "asme_layernorm_fwd: null pointer");
    if (n_rows == 0) return 0;
    const dim3 grid((unsigned)((n_rows + kWaves - 1) / kWaves));
    ASME_VPL_DISPATCH(vpl_of(dim), hipLaunchKernelGGL(ln_fwd_kernel<VPL>, grid, dim3(256), 0, (hipStream_t)stream, x,
                                                      n_rows, (int)dim, w, b, eps, y, stats));
    ASME_LAUNCH_CHECK("asme_layernorm_fwd");
}

ASME_API int asme_layernorm_bwd(const float* x, int64_t n_rows, int64_t dim, const float* w, const float* stats,
                                const float* dy, float* dx, int accumulate, float* partials, int64_t n_partials,
                                void* stream) {
    ASME_CHECK_ARG(x && w && stats && dy && dx && partials && n_partials >= 1, "asme_layernorm_bwd: bad argument");
    if (n_rows == 0) return 0;
    const size_t lds = (size_t)kWaves * 2 * dim * sizeof(float);
    ASME_VPL_DISPATCH(vpl_of(dim),
                      hipLaunchKernelGGL(ln_bwd_kernel<VPL>, dim3((unsigned)n_partials), dim3(256), lds,
                                         (hipStream_t)stream, x, n_rows, (int)dim, w, stats, dy, dx, accumulate,
                                         partials));
    ASME_LAUNCH_CHECK("asme_layernorm_bwd");
}

ASME_API int asme_residual_ln_fwd(const float* res, const float* y, int64_t n_rows, int64_t dim, float p_a,
                                  uint64_t seed_a, float p_b, uint64_t seed_b, const float* w, const float* b,
                                  float eps, float* s_out, float* ln_out, float* stats, void* stream) {
    ASME_CHECK_ARG(res && y && s_out, "asme_residual_ln_fwd: null pointer");
    ASME_CHECK_ARG(!w || (b && ln_out && stats), "asme_residual_ln_fwd: LayerNorm outputs missing");
    ASME_CHECK_ARG(p_a >= 0.f && p_a < 1.f && p_b >= 0.f && p_b < 1.f, "asme_residual_ln_fwd: bad dropout p");
    if (n_rows == 0) return 0;
    const dim3 grid((unsigned)((n_rows + kWaves - 1) / kWaves));
    ASME_VPL_DISPATCH(vpl_of(dim),
                      hipLaunchKernelGGL(residual_ln_fwd_kernel<VPL>, grid, dim3(256), 0, (hipStream_t)stream, res, y,
                                         n_rows, (int)dim, p_a, seed_a, p_b, seed_b, w, b, eps, s_out, ln_out,
                                         stats));
    ASME_LAUNCH_CHECK("asme_residual_ln_fwd");
}

ASME_API int asme_residual_ln_bwd(const float* s, int64_t n_rows, int64_t dim, float p_a, uint64_t seed_a, float p_b,
                                  uint64_t seed_b, const float* w, const float* stats, const float* d_s,
                                  const float* d_ln, float* d_res, float* d_y, float* partials, int64_t n_partials,
                                  void* stream) {
    ASME_CHECK_ARG(d_res, "asme_residual_ln_bwd: null d_res");
    ASME_CHECK_ARG(!(w && d_ln) || (s && stats && partials && n_partials >= 1),
                   "asme_residual_ln_bwd: LayerNorm inputs missing");
    if (n_rows == 0) return 0;
    const bool ln = w && d_ln;
    const int64_t nb = ln ? n_partials : (n_rows + kWaves - 1) / kWaves;
    const size_t lds = ln ? (size_t)kWaves * 2 * dim * sizeof(float) : 0;
    ASME_VPL_DISPATCH(vpl_of(dim),
                      hipLaunchKernelGGL(residual_ln_bwd_kernel<VPL>, dim3((unsigned)nb), dim3(256), lds,
                                         (hipStream_t)stream, s, n_rows, (int)dim, p_a, seed_a, p_b, seed_b, w, stats,
                                         d_s, ln ? d_ln : nullptr, d_res, d_y, ln ? partials : nullptr));
    ASME_LAUNCH_CHECK("asme_residual_ln_bwd");
}

ASME_API int asme_gelu_dropout_fwd(const float* x, int64_t n, float p, uint64_t seed, float* y, void* stream) {
    ASME_CHECK_ARG(x && y, "asme_gelu_dropout_fwd: null pointer");
    ASME_CHECK_ARG(((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0, "asme_gelu_dropout_fwd: 16-B alignment");
    if (n == 0) return 0;
    const int64_t n4 = (n + 3) / 4;
    hipLaunchKernelGGL(gelu_dropout_fwd_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       x, n, p, seed, y);
    ASME_LAUNCH_CHECK("asme_gelu_dropout_fwd");
}

ASME_API int asme_gelu_dropout_bwd(const float* x, const float* dy, int64_t n, float p, uint64_t seed, float* dx,
                                   void* stream) {
    ASME_CHECK_ARG(x && dy && dx, "asme_gelu_dropout_bwd: null pointer");
    ASME_CHECK_ARG(((uintptr_t)x & 15) == 0 && ((uintptr_t)dy & 15) == 0 && ((uintptr_t)dx & 15) == 0,
                   "asme_gelu_dropout_bwd: 16-B alignment");
    if (n == 0) return 0;
    const int64_t n4 = (n + 3) / 4;
    hipLaunchKernelGGL(gelu_dropout_bwd_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       x, dy, n, p, seed, dx);
    ASME_LAUNCH_CHECK("asme_gelu_dropout_bwd");
}
