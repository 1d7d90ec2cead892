// Embedding hot path for ASME on gfx950: fused item-row gather + position add + LayerNorm +
// dropout (+ side-attribute add + second LayerNorm + dropout), its backward, and the
// row scatter-add / position / LayerNorm-parameter reductions.
//
// Reference semantics (paths relative to /root/reference/src/asme):
//   TransformerEmbedding.forward      core/models/common/layers/transformer_layers.py:55-80
//   PreFusionContext...forward        core/models/kebert4rec/components.py:54-63  (second LN)
//   nn.Embedding backward (dense)     autograd embedding_dense_backward           
//   LinearUpscaler.forward            core/models/kebert4rec/layers.py:15-27      (gather-sum, A7)
//
// Layout: table (V, D) fp32 row-major; tokens t = b*L + s; activations (T, D) fp32.
// One 64-lane wave owns one token row; lane l holds elements l + 64*j (coalesced 256-B segments).
#include "rows.h"

using namespace asme;

namespace {

constexpr int kWavesPerBlock = 4;

// One token row per LPR-lane group (rows.h): x = E[id] + P[pos]; y1 = LN1(x); z = drop1(y1) + extra;
// out = drop2(LN2(z)).  stats[t] = (mean1, rstd1, mean2, rstd2).
template <class R>
__global__ __launch_bounds__(256) void emb_fwd_kernel(
    const int64_t* __restrict__ ids, int64_t T, int64_t L, const float* __restrict__ table, int64_t V, int D,
    const float* __restrict__ pos, const float* __restrict__ w1, const float* __restrict__ b1, float eps1, float p1,
    uint64_t s1, const float* __restrict__ extra, const float* __restrict__ w2, const float* __restrict__ b2,
    float eps2, float p2, uint64_t s2, float* __restrict__ out, float* __restrict__ stats, int* __restrict__ err) {
    const int lane = threadIdx.x & 63, sub = lane % R::LPR;
    const int64_t t = ((int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)) * R::RPW + lane / R::LPR;
    if (t >= T) return;
    int64_t id = ids[t];
    if (id < 0 || id >= V) {
        if (sub == 0 && err) atomicOr(err, 1);
        id = 0;
    }
    RowVals<R> x, tmp;
    row_load<R>(table + id * D, sub, D, x);
    if (pos) {
        row_load<R>(pos + (t % L) * D, sub, D, tmp);
#pragma unroll
        for (int j = 0; j < R::NV; ++j)
#pragma unroll
            for (int i = 0; i < R::W; ++i) x[j][i] += tmp[j][i];
    }
    float m1 = 0.f, r1 = 1.f, m2 = 0.f, r2 = 1.f;
    if (w1) {
        row_ln_stats<R>(x, sub, D, eps1, m1, r1);
        row_normalise<R>(x, sub, D, m1, r1, tmp);
        row_affine<R>(tmp, sub, D, w1, b1, x);
    }
    if (p1 > 0.f) {
        row_keep<R>(s1, 1u, (uint64_t)t * D, sub, p1, tmp);
        row_mul<R>(x, tmp);
    }
    if (extra) {
        row_load<R>(extra + t * D, sub, D, tmp);
#pragma unroll
        for (int j = 0; j < R::NV; ++j)
#pragma unroll
            for (int i = 0; i < R::W; ++i) x[j][i] += tmp[j][i];
    }
    if (w2) {
        row_ln_stats<R>(x, sub, D, eps2, m2, r2);
        row_normalise<R>(x, sub, D, m2, r2, tmp);
        row_affine<R>(tmp, sub, D, w2, b2, x);
    }
    if (p2 > 0.f) {
        row_keep<R>(s2, 2u, (uint64_t)t * D, sub, p2, tmp);
        row_mul<R>(x, tmp);
    }
    row_store<R>(out + t * D, sub, D, x);
    if (sub == 0 && stats)
        *reinterpret_cast<float4*>(stats + t * 4) = make_float4(m1, r1, m2, r2);
}

// Recomputes the forward from the saved row statistics; d_rows[t] = dL/dx (the gradient of the
// gathered row AND of the position row), d_extra[t] = dL/dz; block partials of (dw1, db1, dw2, db2).
template <class R>
__global__ __launch_bounds__(256) void emb_bwd_kernel(
    const int64_t* __restrict__ ids, int64_t T, int64_t L, const float* __restrict__ table, int64_t V, int D,
    const float* __restrict__ pos, const float* __restrict__ w1, const float* __restrict__ b1, float p1, uint64_t s1,
    const float* __restrict__ extra, const float* __restrict__ w2, float p2, uint64_t s2,
    const float* __restrict__ dout, const float* __restrict__ stats, float* __restrict__ d_rows,
    float* __restrict__ d_extra, float* __restrict__ partials) {
    const int lane = threadIdx.x & 63, sub = lane % R::LPR, wave = threadIdx.x >> 6;
    float acc[4][R::NV][R::W];
#pragma unroll
    for (int k = 0; k < 4; ++k) row_zero<R>(acc[k]);

    for (int64_t t0 = ((int64_t)blockIdx.x * kWavesPerBlock + wave) * R::RPW; t0 < T;
         t0 += (int64_t)gridDim.x * kWavesPerBlock * R::RPW) {
        const int64_t t = t0 + lane / R::LPR;
        const bool live = t < T;
        RowVals<R> x, xh1, f1, xh2, g, tmp;
        float4 st = make_float4(0.f, 0.f, 0.f, 0.f);
        if (live) {
            int64_t id = ids[t];
            if (id < 0 || id >= V) id = 0;
            st = *reinterpret_cast<const float4*>(stats + t * 4);
            row_load<R>(table + id * D, sub, D, x);
            if (pos) {
                row_load<R>(pos + (t % L) * D, sub, D, tmp);
#pragma unroll
                for (int j = 0; j < R::NV; ++j)
#pragma unroll
                    for (int i = 0; i < R::W; ++i) x[j][i] += tmp[j][i];
            }
            row_load<R>(dout + t * D, sub, D, g);
        } else {
            row_zero<R>(x);
            row_zero<R>(g);
        }
        // recompute z = drop1(LN1(x)) + extra
        if (w1) {
            row_normalise<R>(x, sub, D, st.x, st.y, xh1);
            row_affine<R>(xh1, sub, D, w1, b1, x);
        } else {
#pragma unroll
            for (int j = 0; j < R::NV; ++j)
#pragma unroll
                for (int i = 0; i < R::W; ++i) xh1[j][i] = x[j][i];
        }
        if (p1 > 0.f) {
            row_keep<R>(s1, 1u, (uint64_t)t * D, sub, p1, f1);
            row_mul<R>(x, f1);
        }
        if (extra && live) {
            row_load<R>(extra + t * D, sub, D, tmp);
#pragma unroll
            for (int j = 0; j < R::NV; ++j)
#pragma unroll
                for (int i = 0; i < R::W; ++i) x[j][i] += tmp[j][i];
        }
        if (w2) row_normalise<R>(x, sub, D, st.z, st.w, xh2);
        if (p2 > 0.f) {
            row_keep<R>(s2, 2u, (uint64_t)t * D, sub, p2, tmp);
            row_mul<R>(g, tmp);
        }
        RowVals<R> gz;
        if (w2) {
#pragma unroll
            for (int j = 0; j < R::NV; ++j)
#pragma unroll
                for (int i = 0; i < R::W; ++i) {
                    acc[2][j][i] += g[j][i] * xh2[j][i];
                    acc[3][j][i] += g[j][i];
                }
            row_ln_bwd<R>(g, xh2, w2, st.w, sub, D, gz);
        } else {
#pragma unroll
            for (int j = 0; j < R::NV; ++j)
#pragma unroll
                for (int i = 0; i < R::W; ++i) gz[j][i] = g[j][i];
        }
        if (d_extra && live) row_store<R>(d_extra + t * D, sub, D, gz);
        if (p1 > 0.f) row_mul<R>(gz, f1);  // gz is now d y1
        if (w1) {
#pragma unroll
            for (int j = 0; j < R::NV; ++j)
#pragma unroll
                for (int i = 0; i < R::W; ++i) {
                    acc[0][j][i] += gz[j][i] * xh1[j][i];
                    acc[1][j][i] += gz[j][i];
                }
            row_ln_bwd<R>(gz, xh1, w1, st.y, sub, D, g);
            if (live) row_store<R>(d_rows + t * D, sub, D, g);
        } else if (live) {
            row_store<R>(d_rows + t * D, sub, D, gz);
        }
    }
    if (partials) write_row_partials<R, 4, kWavesPerBlock>(acc, lane, wave, D, partials);
}

template <int VPL>
__global__ __launch_bounds__(256) void scatter_add_rows_kernel(const float* __restrict__ rows,
                                                               const int64_t* __restrict__ ids, int64_t n, int D,
                                                               float* __restrict__ grad, int64_t V, float scale) {
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    if (r >= n) return;
    const int64_t id = ids[r];
    if (id < 0 || id >= V) return;
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
        const int e = lane + 64 * j;
        if (e < D) unsafeAtomicAdd(&grad[id * D + e], rows[r * D + e] * scale);
    }
}

// sum over the batch of per-token rows -> per-position grad; grid (L, nchunk), partial per chunk
__global__ __launch_bounds__(256) void pos_partial_kernel(const float* __restrict__ rows, int64_t B, int64_t L, int D,
                                                          int64_t chunk, float* __restrict__ part) {
    const int64_t p = blockIdx.x;
    const int64_t c = blockIdx.y;
    const int64_t b0 = c * chunk, b1 = min(B, b0 + chunk);
    for (int e = threadIdx.x; e < D; e += blockDim.x) {
        float s = 0.f;
        for (int64_t b = b0; b < b1; ++b) s += rows[(b * L + p) * D + e];
        part[(c * L + p) * D + e] = s;
    }
}

// column sums of a (nrows, width) matrix: a block owns 64 columns; its 16 row-groups of 64 threads each
// sum every 16th row (coalesced 256-B row segments), then a fixed-order LDS tree adds the 16 partials.
constexpr int kRedCols = 64, kRedGroups = 16;
__global__ __launch_bounds__(1024) void reduce_rows_kernel(const float* __restrict__ part, int64_t nrows,
                                                           int64_t width, float* __restrict__ out, int accumulate) {
    __shared__ float red[kRedGroups][kRedCols];
    const int col = threadIdx.x % kRedCols, grp = threadIdx.x / kRedCols;
    const int64_t c = (int64_t)blockIdx.x * kRedCols + col;
    float s = 0.f;
    if (c < width)
        for (int64_t r = grp; r < nrows; r += kRedGroups) s += part[r * width + c];
    red[grp][col] = s;
    __syncthreads();
    for (int h = kRedGroups / 2; h > 0; h >>= 1) {
        if (grp < h) red[grp][col] += red[grp + h][col];
        __syncthreads();
    }
    if (grp == 0 && c < width) out[c] = accumulate ? out[c] + red[0][col] : red[0][col];
}

template <int VPL>
__global__ __launch_bounds__(256) void gather_sum_fwd_kernel(const int64_t* __restrict__ ids, int64_t n, int K,
                                                             int skip_zero, const float* __restrict__ table,
                                                             int64_t V, int D, const float* __restrict__ bias,
                                                             float* __restrict__ out, int accumulate) {
    const int lane = threadIdx.x & 63;
    const int64_t t = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    if (t >= n) return;
    float x[VPL];
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
        const int e = lane + 64 * j;
        x[j] = (bias && e < D) ? bias[e] : 0.f;
    }
    for (int k = 0; k < K; ++k) {
        const int64_t id = ids[t * K + k];
        if ((skip_zero && id == 0) || id < 0 || id >= V) continue;
#pragma unroll
        for (int j = 0; j < VPL; ++j) {
            const int e = lane + 64 * j;
            if (e < D) x[j] += table[id * D + e];
        }
    }
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
        const int e = lane + 64 * j;
        if (e < D) out[t * D + e] = accumulate ? out[t * D + e] + x[j] : x[j];
    }
}

template <int VPL>
__global__ __launch_bounds__(256) void gather_sum_bwd_kernel(const float* __restrict__ dout,
                                                             const int64_t* __restrict__ ids, int64_t n, int K,
                                                             int skip_zero, float* __restrict__ grad, int64_t V,
                                                             int D) {
    const int lane = threadIdx.x & 63;
    const int64_t t = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    if (t >= n) return;
    for (int k = 0; k < K; ++k) {
        const int64_t id = ids[t * K + k];
        if ((skip_zero && id == 0) || id < 0 || id >= V) continue;
#pragma unroll
        for (int j = 0; j < VPL; ++j) {
            const int e = lane + 64 * j;
            if (e < D) unsafeAtomicAdd(&grad[id * D + e], dout[t * D + e]);
        }
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

ASME_API int asme_embedding_fwd(const int64_t* ids, int64_t n_tokens, int64_t seq_len, const float* table,
                                int64_t vocab, int64_t dim, const float* pos_table, const float* ln1_w,
                                const float* ln1_b, float ln1_eps, float p1, uint64_t seed1, const float* extra,
                                const float* ln2_w, const float* ln2_b, float ln2_eps, float p2, uint64_t seed2,
                                float* out, float* stats, int* err_flag, void* stream) {
    ASME_CHECK_ARG(ids && table && out && stats, "asme_embedding_fwd: null pointer");
    ASME_CHECK_ARG(dim >= 1 && dim <= 512 && seq_len >= 1 && n_tokens >= 0, "asme_embedding_fwd: bad shape");
    ASME_CHECK_ARG(p1 >= 0.f && p1 < 1.f && p2 >= 0.f && p2 < 1.f, "asme_embedding_fwd: dropout p must be in [0,1)");
    if (n_tokens == 0) return 0;
    if (with_row_layout(dim, [&](auto layout) {
            using R = decltype(layout);
            const int64_t rows = (int64_t)kWavesPerBlock * R::RPW;
            hipLaunchKernelGGL(emb_fwd_kernel<R>, dim3((unsigned)((n_tokens + rows - 1) / rows)), dim3(256), 0,
                               (hipStream_t)stream, ids, n_tokens, seq_len, table, vocab, (int)dim, pos_table, ln1_w,
                               ln1_b, ln1_eps, p1, seed1, extra, ln2_w, ln2_b, ln2_eps, p2, seed2, out, stats,
                               err_flag);
        }))
        return -1;
    ASME_LAUNCH_CHECK("asme_embedding_fwd");
}

ASME_API int asme_embedding_bwd_partials_count(void) { return 1024; }

ASME_API int asme_embedding_bwd(const int64_t* ids, int64_t n_tokens, int64_t seq_len, const float* table,
                                int64_t vocab, int64_t dim, const float* pos_table, const float* ln1_w,
                                const float* ln1_b, float p1, uint64_t seed1, const float* extra, const float* ln2_w,
                                float p2, uint64_t seed2, const float* dout, const float* stats, float* d_rows,
                                float* d_extra, float* partials, int64_t n_partials, void* stream) {
    ASME_CHECK_ARG(ids && table && dout && stats && d_rows, "asme_embedding_bwd: null pointer");
    ASME_CHECK_ARG(dim >= 1 && dim <= 512, "asme_embedding_bwd: bad shape");
    ASME_CHECK_ARG(!partials || n_partials >= 1, "asme_embedding_bwd: n_partials must be >= 1");
    if (n_tokens == 0) return 0;
    const size_t lds = partials ? (size_t)kWavesPerBlock * 4 * dim * sizeof(float) : 0;
    if (with_row_layout(dim, [&](auto layout) {
            using R = decltype(layout);
            const int64_t rows = (int64_t)kWavesPerBlock * R::RPW;
            // grid-stride with one partial row per block when the LN parameter grads are wanted
            const int64_t nb = partials ? n_partials : (n_tokens + rows - 1) / rows;
            hipLaunchKernelGGL(emb_bwd_kernel<R>, dim3((unsigned)nb), dim3(256), lds, (hipStream_t)stream, ids,
                               n_tokens, seq_len, table, vocab, (int)dim, pos_table, ln1_w, ln1_b, p1, seed1, extra,
                               ln2_w, p2, seed2, dout, stats, d_rows, d_extra, partials);
        }))
        return -1;
    ASME_LAUNCH_CHECK("asme_embedding_bwd");
}

ASME_API int asme_scatter_add_rows(const float* rows, const int64_t* ids, int64_t n_rows, int64_t dim, float* grad,
                                   int64_t vocab, float scale, void* stream) {
    ASME_CHECK_ARG(rows && ids && grad, "asme_scatter_add_rows: null pointer");
    ASME_CHECK_ARG(dim >= 1 && dim <= 512, "asme_scatter_add_rows: bad shape");
    if (n_rows == 0) return 0;
    const dim3 grid((unsigned)((n_rows + kWavesPerBlock - 1) / kWavesPerBlock));
    ASME_VPL_DISPATCH(vpl_of(dim), hipLaunchKernelGGL(scatter_add_rows_kernel<VPL>, grid, dim3(256), 0,
                                                      (hipStream_t)stream, rows, ids, n_rows, (int)dim, grad, vocab,
                                                      scale));
    ASME_LAUNCH_CHECK("asme_scatter_add_rows");
}

ASME_API int asme_position_grad(const float* rows, int64_t batch, int64_t seq_len, int64_t dim, float* workspace,
                                int64_t n_chunks, float* grad_pos, int accumulate, void* stream) {
    ASME_CHECK_ARG(rows && workspace && grad_pos && n_chunks >= 1, "asme_position_grad: bad argument");
    const int64_t chunk = (batch + n_chunks - 1) / n_chunks;
    hipLaunchKernelGGL(pos_partial_kernel, dim3((unsigned)seq_len, (unsigned)n_chunks), dim3(128), 0,
                       (hipStream_t)stream, rows, batch, seq_len, (int)dim, chunk, workspace);
    const int64_t width = seq_len * dim;
    hipLaunchKernelGGL(reduce_rows_kernel, dim3((unsigned)((width + kRedCols - 1) / kRedCols)), dim3(1024), 0,
                       (hipStream_t)stream, workspace, n_chunks, width, grad_pos, accumulate);
    ASME_LAUNCH_CHECK("asme_position_grad");
}

ASME_API int asme_reduce_rows(const float* part, int64_t n_rows, int64_t width, float* out, int accumulate,
                              void* stream) {
    ASME_CHECK_ARG(part && out, "asme_reduce_rows: null pointer");
    if (width == 0) return 0;
    hipLaunchKernelGGL(reduce_rows_kernel, dim3((unsigned)((width + kRedCols - 1) / kRedCols)), dim3(1024), 0,
                       (hipStream_t)stream, part, n_rows, width, out, accumulate);
    ASME_LAUNCH_CHECK("asme_reduce_rows");
}

ASME_API int asme_gather_sum_fwd(const int64_t* ids, int64_t n, int64_t k, int skip_zero, const float* table,
                                 int64_t vocab, int64_t dim, const float* bias, float* out, int accumulate,
                                 void* stream) {
    ASME_CHECK_ARG(ids && table && out && k >= 1, "asme_gather_sum_fwd: bad argument");
    if (n == 0) return 0;
    const dim3 grid((unsigned)((n + kWavesPerBlock - 1) / kWavesPerBlock));
    ASME_VPL_DISPATCH(vpl_of(dim), hipLaunchKernelGGL(gather_sum_fwd_kernel<VPL>, grid, dim3(256), 0,
                                                      (hipStream_t)stream, ids, n, (int)k, skip_zero, table, vocab,
                                                      (int)dim, bias, out, accumulate));
    ASME_LAUNCH_CHECK("asme_gather_sum_fwd");
}

ASME_API int asme_gather_sum_bwd(const float* dout, const int64_t* ids, int64_t n, int64_t k, int skip_zero,
                                 float* grad, int64_t vocab, int64_t dim, void* stream) {
    ASME_CHECK_ARG(ids && grad && dout && k >= 1, "asme_gather_sum_bwd: bad argument");
    if (n == 0) return 0;
    const dim3 grid((unsigned)((n + kWavesPerBlock - 1) / kWavesPerBlock));
    ASME_VPL_DISPATCH(vpl_of(dim), hipLaunchKernelGGL(gather_sum_bwd_kernel<VPL>, grid, dim3(256), 0,
                                                      (hipStream_t)stream, dout, ids, n, (int)k, skip_zero, grad,
                                                      vocab, (int)dim));
    ASME_LAUNCH_CHECK("asme_gather_sum_bwd");
}
