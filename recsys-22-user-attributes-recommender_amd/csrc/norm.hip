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
#include "rows.h"

using namespace asme;

namespace {
constexpr int kWaves = 4;

// ------------------------------------------------------------ plain LayerNorm
template <class R>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const float* __restrict__ x, int64_t T, int D,
                                                     const float* __restrict__ w, const float* __restrict__ b,
                                                     float eps, float* __restrict__ y, float* __restrict__ stats) {
    const int lane = threadIdx.x & 63, sub = lane % R::LPR;
    const int64_t t = ((int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6)) * R::RPW + lane / R::LPR;
    if (t >= T) return;  // whole row groups leave together
    RowVals<R> v, xh, o;
    float m, r;
    row_load<R>(x + t * D, sub, D, v);
    row_ln_stats<R>(v, sub, D, eps, m, r);
    row_normalise<R>(v, sub, D, m, r, xh);
    row_affine<R>(xh, sub, D, w, b, o);
    row_store<R>(y + t * D, sub, D, o);
    if (sub == 0) {
        stats[t * 2] = m;
        stats[t * 2 + 1] = r;
    }
}

template <class R>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const float* __restrict__ x, int64_t T, int D,
                                                     const float* __restrict__ w, const float* __restrict__ stats,
                                                     const float* __restrict__ dy, float* __restrict__ dx,
                                                     int accumulate, const float* __restrict__ dadd,
                                                     float* __restrict__ partials) {
    const int lane = threadIdx.x & 63, sub = lane % R::LPR, wave = threadIdx.x >> 6;
    float acc[2][R::NV][R::W];
    row_zero<R>(acc[0]);
    row_zero<R>(acc[1]);
    for (int64_t t0 = ((int64_t)blockIdx.x * kWaves + wave) * R::RPW; t0 < T;
         t0 += (int64_t)gridDim.x * kWaves * R::RPW) {
        const int64_t t = t0 + lane / R::LPR;
        const bool live = t < T;
        RowVals<R> v, xh, g, gx;
        const float m = live ? stats[t * 2] : 0.f, r = live ? stats[t * 2 + 1] : 0.f;
        if (live) {
            row_load<R>(x + t * D, sub, D, v);
            row_load<R>(dy + t * D, sub, D, g);
        } else {
            row_zero<R>(v);
            row_zero<R>(g);
        }
        row_normalise<R>(v, sub, D, m, r, xh);
#pragma unroll
        for (int j = 0; j < R::NV; ++j)
#pragma unroll
            for (int i = 0; i < R::W; ++i) {
                acc[0][j][i] += g[j][i] * xh[j][i];
                acc[1][j][i] += g[j][i];
            }
        row_ln_bwd<R>(g, xh, w, r, sub, D, gx);
        if (!live) continue;
        if (accumulate || dadd) {  // dx = LN'(dy) + dx (accumulate) or + dadd (a second gradient of x)
            RowVals<R> old;
            row_load<R>((dadd ? dadd : dx) + t * D, sub, D, old);
#pragma unroll
            for (int j = 0; j < R::NV; ++j)
#pragma unroll
                for (int i = 0; i < R::W; ++i) gx[j][i] += old[j][i];
        }
        row_store<R>(dx + t * D, sub, D, gx);
    }
    write_row_partials<R, 2, kWaves>(acc, lane, wave, D, partials);
}

// ------------------------------------------------------------ residual + dropout(s) + LayerNorm
#ifndef ASME_RLNB_LOAD_NT
#define ASME_RLNB_LOAD_NT 3  // residual_ln_bwd loads non-temporal (bit 0 the gradients, bit 1 the saved s): -4 % per call
#endif
#ifndef ASME_RLN_NT
#define ASME_RLN_NT 3  // non-temporal stores in residual_ln_fwd (bit 0: s, bit 1: LN(s)) / _bwd (bit 2: d_res, bit 3: d_y)
#endif
template <class R>
__global__ __launch_bounds__(256) void residual_ln_fwd_kernel(
    const float* __restrict__ res, const float* __restrict__ y, int64_t T, int D, float pa, uint64_t sa, float pb,
    uint64_t sb, const float* __restrict__ w, const float* __restrict__ b, float eps, float* __restrict__ s_out,
    float* __restrict__ ln_out, float* __restrict__ stats) {
    const int lane = threadIdx.x & 63, sub = lane % R::LPR;
    const int64_t t = ((int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6)) * R::RPW + lane / R::LPR;
    if (t >= T) return;
    RowVals<R> a, h, f;
    row_load<R>(y + t * D, sub, D, a);
    row_load<R>(res + t * D, sub, D, h);
    if (pa > 0.f) {
        row_keep<R>(sa, 3u, (uint64_t)t * D, sub, pa, f);
        row_mul<R>(a, f);
    }
#pragma unroll
    for (int j = 0; j < R::NV; ++j)
#pragma unroll
        for (int i = 0; i < R::W; ++i) h[j][i] += a[j][i];
    if (pb > 0.f) {
        row_keep<R>(sb, 4u, (uint64_t)t * D, sub, pb, f);
        row_mul<R>(h, f);
    }
    row_store<R, (ASME_RLN_NT & 1) != 0>(s_out + t * D, sub, D, h);
    if (w) {
        float m, r;
        row_ln_stats<R>(h, sub, D, eps, m, r);
        row_normalise<R>(h, sub, D, m, r, a);
        row_affine<R>(a, sub, D, w, b, f);
        row_store<R, (ASME_RLN_NT & 2) != 0>(ln_out + t * D, sub, D, f);
        if (sub == 0) {
            stats[t * 2] = m;
            stats[t * 2 + 1] = r;
        }
    }
}

template <class R>
__global__ __launch_bounds__(256) void residual_ln_bwd_kernel(
    const float* __restrict__ s, int64_t T, int D, float pa, uint64_t sa, float pb, uint64_t sb,
    const float* __restrict__ w, const float* __restrict__ stats, const float* __restrict__ d_s,
    const float* __restrict__ d_ln, float* __restrict__ d_res, float* __restrict__ d_y,
    float* __restrict__ partials) {
    const int lane = threadIdx.x & 63, sub = lane % R::LPR, wave = threadIdx.x >> 6;
    float acc[2][R::NV][R::W];
    row_zero<R>(acc[0]);
    row_zero<R>(acc[1]);
    for (int64_t t0 = ((int64_t)blockIdx.x * kWaves + wave) * R::RPW; t0 < T;
         t0 += (int64_t)gridDim.x * kWaves * R::RPW) {
        const int64_t t = t0 + lane / R::LPR;
        const bool live = t < T;
        RowVals<R> g;
        if (live && d_s)
            row_load_p<R, (ASME_RLNB_LOAD_NT & 1) != 0>(d_s + t * D, sub, D, g);
        else
            row_zero<R>(g);
        if (w && d_ln) {
            const float m = live ? stats[t * 2] : 0.f, r = live ? stats[t * 2 + 1] : 0.f;
            RowVals<R> v, xh, gl, gx;
            if (live) {
                row_load_p<R, (ASME_RLNB_LOAD_NT & 2) != 0>(s + t * D, sub, D, v);
                row_load_p<R, (ASME_RLNB_LOAD_NT & 1) != 0>(d_ln + t * D, sub, D, gl);
            } else {
                row_zero<R>(v);
                row_zero<R>(gl);
            }
            row_normalise<R>(v, sub, D, m, r, xh);
#pragma unroll
            for (int j = 0; j < R::NV; ++j)
#pragma unroll
                for (int i = 0; i < R::W; ++i) {
                    acc[0][j][i] += gl[j][i] * xh[j][i];
                    acc[1][j][i] += gl[j][i];
                }
            row_ln_bwd<R>(gl, xh, w, r, sub, D, gx);
#pragma unroll
            for (int j = 0; j < R::NV; ++j)
#pragma unroll
                for (int i = 0; i < R::W; ++i) g[j][i] += gx[j][i];
        }
        if (!live) continue;
        RowVals<R> f;
        if (pb > 0.f) {
            row_keep<R>(sb, 4u, (uint64_t)t * D, sub, pb, f);
            row_mul<R>(g, f);
        }
        row_store<R, (ASME_RLN_NT & 4) != 0>(d_res + t * D, sub, D, g);
        if (d_y) {
            if (pa > 0.f) {
                row_keep<R>(sa, 3u, (uint64_t)t * D, sub, pa, f);
                row_mul<R>(g, f);
            }
            row_store<R, (ASME_RLN_NT & 8) != 0>(d_y + t * D, sub, D, g);
        }
    }
    if (partials) write_row_partials<R, 2, kWaves>(acc, lane, wave, D, partials);
}

template <class R>
inline unsigned row_blocks(int64_t T) {
    const int64_t rows = (int64_t)kWaves * R::RPW;
    return (unsigned)((T + rows - 1) / rows);
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
            gelu_keep_factors(gelu_keep_bits4(seed, (uint64_t)i >> 2, gelu_thresh(p)), 1.f / (1.f - p), u);
        }
        float4 o;
        o.x = gelu_erf(v.x) * u[0];
        o.y = gelu_erf(v.y) * u[1];
        o.z = gelu_erf(v.z) * u[2];
        o.w = gelu_erf(v.w) * u[3];
        *reinterpret_cast<float4*>(y + i) = o;
    } else {
        for (int64_t k = i; k < n; ++k) y[k] = gelu_erf(x[k]) * (p > 0.f ? gelu_keep_factor(seed, (uint64_t)k, p) : 1.f);
    }
}

// y = dropout_p(x) (nn.Dropout in training mode): keep iff u >= p, kept values scaled by 1/(1-p); 4 consecutive
// elements share one Philox4x32-10 block (salt 6).  The backward regenerates the same decisions from (seed, index).
// Reference: UBERT4RecSequenceElementsRepresentationComponent.dropout_embedding (ubert4rec/components.py:157-160).
__global__ __launch_bounds__(256) void dropout_kernel(const float* __restrict__ x, int64_t n, float p, uint64_t seed,
                                                      float* __restrict__ y) {
    const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
    if (i >= n) return;
    float u[4];
    philox_uniform4(seed, 6u, (uint64_t)i >> 2, u);
    const float k = 1.f / (1.f - p);
    if (i + 3 < n && ((uintptr_t)(x + i) & 15) == 0 && ((uintptr_t)(y + i) & 15) == 0) {
        const float4 v = *reinterpret_cast<const float4*>(x + i);
        *reinterpret_cast<float4*>(y + i) = make_float4(u[0] >= p ? v.x * k : 0.f, u[1] >= p ? v.y * k : 0.f,
                                                        u[2] >= p ? v.z * k : 0.f, u[3] >= p ? v.w * k : 0.f);
    } else {
        for (int64_t j = i; j < n && j < i + 4; ++j) y[j] = u[j - i] >= p ? x[j] * k : 0.f;
    }
}

// Dropout2d on (N, C, L) in training mode (NARM's embedding dropout, core/models/common/layers/sequence_embedding.py:
// 72-73 + :92): whole rows of row_len values are kept (scaled by 1 / (1 - p)) or zeroed, one draw per row.
__global__ __launch_bounds__(256) void dropout_rows_kernel(const float* __restrict__ x, int64_t n, int64_t row_len,
                                                           float p, uint64_t seed, float* __restrict__ y) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t row = i / row_len;
    float u[4];
    philox_uniform4(seed, 7u, (uint64_t)row >> 2, u);
    y[i] = u[row & 3] >= p ? x[i] * (1.f / (1.f - p)) : 0.f;
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
            gelu_keep_factors(gelu_keep_bits4(seed, (uint64_t)i >> 2, gelu_thresh(p)), 1.f / (1.f - p), u);
        }
        float4 o;
        o.x = g.x * u[0] * gelu_erf_grad(v.x);
        o.y = g.y * u[1] * gelu_erf_grad(v.y);
        o.z = g.z * u[2] * gelu_erf_grad(v.z);
        o.w = g.w * u[3] * gelu_erf_grad(v.w);
        *reinterpret_cast<float4*>(dx + i) = o;
    } else {
        for (int64_t k = i; k < n; ++k)
            dx[k] = dy[k] * (p > 0.f ? gelu_keep_factor(seed, (uint64_t)k, p) : 1.f) * gelu_erf_grad(x[k]);
    }
}

}  // namespace

ASME_API int asme_layernorm_fwd(const float* x, int64_t n_rows, int64_t dim, const float* w, const float* b,
                                float eps, float* y, float* stats, void* stream) {
    ASME_CHECK_ARG(x && w && b && y && stats, "asme_layernorm_fwd: null pointer");
    if (n_rows == 0) return 0;
    if (with_row_layout(dim, [&](auto layout) {
            using R = decltype(layout);
            hipLaunchKernelGGL(ln_fwd_kernel<R>, dim3(row_blocks<R>(n_rows)), dim3(256), 0, (hipStream_t)stream, x,
                               n_rows, (int)dim, w, b, eps, y, stats);
        }))
        return -1;
    ASME_LAUNCH_CHECK("asme_layernorm_fwd");
}

ASME_API int asme_layernorm_bwd(const float* x, int64_t n_rows, int64_t dim, const float* w, const float* stats,
                                const float* dy, float* dx, int accumulate, float* partials, int64_t n_partials,
                                void* stream) {
    ASME_CHECK_ARG(x && w && stats && dy && dx && partials && n_partials >= 1, "asme_layernorm_bwd: bad argument");
    if (n_rows == 0) return 0;
    const size_t lds = (size_t)kWaves * 2 * dim * sizeof(float);
    if (with_row_layout(dim, [&](auto layout) {
            using R = decltype(layout);
            hipLaunchKernelGGL(ln_bwd_kernel<R>, dim3((unsigned)n_partials), dim3(256), lds, (hipStream_t)stream, x,
                               n_rows, (int)dim, w, stats, dy, dx, accumulate, (const float*)nullptr, partials);
        }))
        return -1;
    ASME_LAUNCH_CHECK("asme_layernorm_bwd");
}

// dx = LN backward of dy + dadd: a tensor feeding both a LayerNorm and a residual (the first pre-LN block
// input) gets its two gradients summed here instead of by a separate add pass.  dadd nullable.
ASME_API int asme_layernorm_bwd_add(const float* x, int64_t n_rows, int64_t dim, const float* w, const float* stats,
                                    const float* dy, const float* dadd, float* dx, float* partials,
                                    int64_t n_partials, void* stream) {
    ASME_CHECK_ARG(x && w && stats && dy && dx && partials && n_partials >= 1, "asme_layernorm_bwd_add: bad argument");
    if (n_rows == 0) return 0;
    const size_t lds = (size_t)kWaves * 2 * dim * sizeof(float);
    if (with_row_layout(dim, [&](auto layout) {
            using R = decltype(layout);
            hipLaunchKernelGGL(ln_bwd_kernel<R>, dim3((unsigned)n_partials), dim3(256), lds, (hipStream_t)stream, x,
                               n_rows, (int)dim, w, stats, dy, dx, 0, dadd, partials);
        }))
        return -1;
    ASME_LAUNCH_CHECK("asme_layernorm_bwd_add");
}

ASME_API int asme_residual_ln_fwd(const float* res, const float* y, int64_t n_rows, int64_t dim, float p_a,
                                  uint64_t seed_a, float p_b, uint64_t seed_b, const float* w, const float* b,
                                  float eps, float* s_out, float* ln_out, float* stats, void* stream) {
    ASME_CHECK_ARG(res && y && s_out, "asme_residual_ln_fwd: null pointer");
    ASME_CHECK_ARG(!w || (b && ln_out && stats), "asme_residual_ln_fwd: LayerNorm outputs missing");
    ASME_CHECK_ARG(p_a >= 0.f && p_a < 1.f && p_b >= 0.f && p_b < 1.f, "asme_residual_ln_fwd: bad dropout p");
    if (n_rows == 0) return 0;
    if (with_row_layout(dim, [&](auto layout) {
            using R = decltype(layout);
            hipLaunchKernelGGL(residual_ln_fwd_kernel<R>, dim3(row_blocks<R>(n_rows)), dim3(256), 0,
                               (hipStream_t)stream, res, y, n_rows, (int)dim, p_a, seed_a, p_b, seed_b, w, b, eps,
                               s_out, ln_out, stats);
        }))
        return -1;
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
    const size_t lds = ln ? (size_t)kWaves * 2 * dim * sizeof(float) : 0;
    if (with_row_layout(dim, [&](auto layout) {
            using R = decltype(layout);
            const unsigned nb = ln ? (unsigned)n_partials : row_blocks<R>(n_rows);
            hipLaunchKernelGGL(residual_ln_bwd_kernel<R>, dim3(nb), dim3(256), lds, (hipStream_t)stream, s, n_rows,
                               (int)dim, p_a, seed_a, p_b, seed_b, w, stats, d_s, ln ? d_ln : nullptr, d_res, d_y,
                               ln ? partials : nullptr);
        }))
        return -1;
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

// y = dropout_p(x); the backward is the same call on dy (identical decisions from the same seed)
ASME_API int asme_dropout(const float* x, int64_t n, float p, uint64_t seed, float* y, void* stream) {
    ASME_CHECK_ARG(x && y, "asme_dropout: null pointer");
    ASME_CHECK_ARG(p >= 0.f && p < 1.f, "asme_dropout: p in [0, 1)");
    if (n == 0) return 0;
    const int64_t n4 = (n + 3) / 4;
    hipLaunchKernelGGL(dropout_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, (hipStream_t)stream, x, n, p,
                       seed, y);
    ASME_LAUNCH_CHECK("asme_dropout");
}

// Row-wise dropout (Dropout2d semantics on (N, C, L): C rows of row_len); the backward is the same call on dy.
ASME_API int asme_dropout_rows(const float* x, int64_t n, int64_t row_len, float p, uint64_t seed, float* y,
                               void* stream) {
    ASME_CHECK_ARG(x && y, "asme_dropout_rows: null pointer");
    ASME_CHECK_ARG(p >= 0.f && p < 1.f && row_len >= 1 && n % row_len == 0, "asme_dropout_rows: bad argument");
    if (n == 0) return 0;
    hipLaunchKernelGGL(dropout_rows_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, x,
                       n, row_len, p, seed, y);
    ASME_LAUNCH_CHECK("asme_dropout_rows");
}
