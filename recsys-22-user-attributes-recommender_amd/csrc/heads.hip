// Logit heads, losses and ranking for ASME on gfx950.
//
// Reference semantics (paths relative to /root/reference/src/asme):
//   SASRecProjectionComponent.forward (train)  core/models/sasrec/components.py:34-44
//       pos = sum_d E[pos_ids] * H ; neg = sum_d E[neg_ids] * H          (sampled head)
//   sas_rec_binary_cross_entropy               core/losses/sasrec/sas_rec_losses.py:47-75
//       sum(-log(sigmoid(p)+1e-24)*m - log(1-sigmoid(n)+1e-24)*m) / sum(m)   
//   nn.CrossEntropyLoss(ignore_index=pad)      core/modules/masked_training_module.py:93-111,
//                                              core/losses/sasrec/sas_rec_losses.py:15-32, losses.py:77-115
//   get_true_positives / calc_ndcg             core/metrics/common.py:4-27,118-175 (rank of the target)
#include "rows.h"
#include <algorithm>
#include <cmath>

using namespace asme;

namespace {
constexpr int kWaves = 4;

// Row-layout forms (rows.h) for 16-B aligned D % 4 == 0 tables: a token row is LPR lanes x NV float4 (16 lanes x 2 at
// D = 128: 4 tokens per wave, K per lane group), the dot products reduce inside the lane group on DPP, every load
// and store is a 16-B vector -- instead of one token per wave with 4-B loads and a 6-step ds_bpermute wave sum.
template <class R, int K>
__global__ __launch_bounds__(256) void sampled_fwd4_kernel(const float* __restrict__ H, const float* __restrict__ E,
                                                           const int64_t* __restrict__ pos,
                                                           const int64_t* __restrict__ neg, int64_t T, int D,
                                                           int64_t V, float* __restrict__ pos_out,
                                                           float* __restrict__ neg_out) {
    const int lane = threadIdx.x & 63, sub = lane % R::LPR;
    const int64_t t0 = ((int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6)) * R::RPW * K + lane / R::LPR;
    int64_t ip[K], in[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int64_t t = t0 + (int64_t)k * R::RPW;
        const int64_t a = t < T ? pos[t] : 0, b = t < T ? neg[t] : 0;
        ip[k] = (a < 0 || a >= V) ? 0 : a;
        in[k] = (b < 0 || b >= V) ? 0 : b;
    }
    RowVals<R> h[K], ep[K], en[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int64_t t = t0 + (int64_t)k * R::RPW;
        row_load<R>(H + (t < T ? t : 0) * D, sub, D, h[k]);
        row_load<R>(E + ip[k] * D, sub, D, ep[k]);
        row_load<R>(E + in[k] * D, sub, D, en[k]);
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
        float sp = 0.f, sn = 0.f;
#pragma unroll
        for (int j = 0; j < R::NV; ++j)
#pragma unroll
            for (int i = 0; i < R::W; ++i) {
                sp += ep[k][j][i] * h[k][j][i];
                sn += en[k][j][i] * h[k][j][i];
            }
        sp = row_sum<R::LPR>(sp);
        sn = row_sum<R::LPR>(sn);
        const int64_t t = t0 + (int64_t)k * R::RPW;
        if (sub == 0 && t < T) {
            pos_out[t] = sp;
            neg_out[t] = sn;
        }
    }
}

template <class R, int K>
__global__ __launch_bounds__(256) void sampled_bwd4_kernel(const float* __restrict__ H, const float* __restrict__ E,
                                                           const int64_t* __restrict__ pos,
                                                           const int64_t* __restrict__ neg, int64_t T, int D,
                                                           int64_t V, const float* __restrict__ gpos,
                                                           const float* __restrict__ gneg, float* __restrict__ dH,
                                                           float* __restrict__ dE) {
    const int lane = threadIdx.x & 63, sub = lane % R::LPR;
    const int64_t t0 = ((int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6)) * R::RPW * K + lane / R::LPR;
    int64_t ip[K], in[K];
    float gp[K], gn[K];
    bool okp[K], okn[K];  // out-of-range ids: dH reads row 0 (like the gather), the table gets nothing
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int64_t t = t0 + (int64_t)k * R::RPW;
        const bool live = t < T;
        const int64_t a = live ? pos[t] : -1, b = live ? neg[t] : -1;
        okp[k] = a >= 0 && a < V;
        okn[k] = b >= 0 && b < V;
        ip[k] = okp[k] ? a : 0;
        in[k] = okn[k] ? b : 0;
        gp[k] = live ? gpos[t] : 0.f;
        gn[k] = live ? gneg[t] : 0.f;
    }
    RowVals<R> ep[K], en[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        row_load<R>(E + ip[k] * D, sub, D, ep[k]);
        row_load<R>(E + in[k] * D, sub, D, en[k]);
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int64_t t = t0 + (int64_t)k * R::RPW;
        if (t >= T) break;
        if (dH) {
            RowVals<R> d;
#pragma unroll
            for (int j = 0; j < R::NV; ++j)
#pragma unroll
                for (int i = 0; i < R::W; ++i) d[j][i] = gp[k] * ep[k][j][i] + gn[k] * en[k][j][i];
            row_store<R>(dH + t * D, sub, D, d);
        }
        if (dE) {
            RowVals<R> h;
            row_load<R>(H + t * D, sub, D, h);
#pragma unroll
            for (int j = 0; j < R::NV; ++j) {
                const int c = R::col(sub, j);
                if (c >= D) continue;
#pragma unroll
                for (int i = 0; i < R::W; ++i) {
                    if (okp[k] && gp[k] != 0.f) unsafeAtomicAdd(&dE[ip[k] * D + c + i], gp[k] * h[j][i]);
                    if (okn[k] && gn[k] != 0.f) unsafeAtomicAdd(&dE[in[k] * D + c + i], gn[k] * h[j][i]);
                }
            }
        }
    }
}

// the row layout of the sampled head (the embedding kernels' at D = 128: 16 lanes x 2 float4)
template <class F>
int with_head_layout(int64_t D, F&& f) {
    if (D == 128) {
        f(RowLayout<4, 16, 2>{});
        return 0;
    }
    return with_row_layout(D, f);
}
constexpr int kHeadK = 2;  // tokens per lane group

template <int VPL>
__global__ __launch_bounds__(256) void sampled_fwd_kernel(const float* __restrict__ H, const float* __restrict__ E,
                                                          const int64_t* __restrict__ pos,
                                                          const int64_t* __restrict__ neg, int64_t T, int D,
                                                          int64_t V, float* __restrict__ pos_out,
                                                          float* __restrict__ neg_out) {
    const int lane = threadIdx.x & 63;
    const int64_t t = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
    if (t >= T) return;
    int64_t ip = pos[t], in = neg[t];
    ip = (ip < 0 || ip >= V) ? 0 : ip;
    in = (in < 0 || in >= V) ? 0 : in;
    float sp = 0.f, sn = 0.f;
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
        const int e = lane + 64 * j;
        if (e < D) {
            const float h = H[t * D + e];
            sp += E[ip * D + e] * h;
            sn += E[in * D + e] * h;
        }
    }
    sp = wave_sum(sp);
    sn = wave_sum(sn);
    if (lane == 0) {
        pos_out[t] = sp;
        neg_out[t] = sn;
    }
}

template <int VPL>
__global__ __launch_bounds__(256) void sampled_bwd_kernel(const float* __restrict__ H, const float* __restrict__ E,
                                                          const int64_t* __restrict__ pos,
                                                          const int64_t* __restrict__ neg, int64_t T, int D,
                                                          int64_t V, const float* __restrict__ gpos,
                                                          const float* __restrict__ gneg, float* __restrict__ dH,
                                                          float* __restrict__ dE) {
    const int lane = threadIdx.x & 63;
    const int64_t t = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
    if (t >= T) return;
    int64_t ip = pos[t], in = neg[t];
    const bool okp = ip >= 0 && ip < V, okn = in >= 0 && in < V;
    ip = okp ? ip : 0;
    in = okn ? in : 0;
    const float gp = gpos[t], gn = gneg[t];
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
        const int e = lane + 64 * j;
        if (e < D) {
            const float h = H[t * D + e];
            if (dH) dH[t * D + e] = gp * E[ip * D + e] + gn * E[in * D + e];
            if (dE) {
                if (okp && gp != 0.f) unsafeAtomicAdd(&dE[ip * D + e], gp * h);
                if (okn && gn != 0.f) unsafeAtomicAdd(&dE[in * D + e], gn * h);
            }
        }
    }
}

__device__ __forceinline__ float sigmoidf_ref(float x) { return 1.f / (1.f + expf(-x)); }

// per-block partial sums of the masked BCE terms and of the mask
__global__ __launch_bounds__(256) void bce_fwd_kernel(const float* __restrict__ p, const float* __restrict__ n,
                                                      const uint8_t* __restrict__ mask, int64_t T,
                                                      float* __restrict__ part) {
    __shared__ float sl[kWaves], sm[kWaves];
    float acc = 0.f, cnt = 0.f;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < T; t += (int64_t)gridDim.x * blockDim.x) {
        const float m = mask[t] ? 1.f : 0.f;
        const float lp = logf(sigmoidf_ref(p[t]) + 1e-24f) * m;
        const float ln = logf((1.f - sigmoidf_ref(n[t])) + 1e-24f) * m;
        acc += -lp - ln;
        cnt += m;
    }
    acc = wave_sum(acc);
    cnt = wave_sum(cnt);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        sl[w] = acc;
        sm[w] = cnt;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float a = 0.f, c = 0.f;
        for (int i = 0; i < kWaves; ++i) {
            a += sl[i];
            c += sm[i];
        }
        part[blockIdx.x * 2] = a;
        part[blockIdx.x * 2 + 1] = c;
    }
}

// loss = sum(part.loss) / sum(part.mask); out[0] = loss, out[1] = mask count
__global__ void bce_finish_kernel(const float* __restrict__ part, int nparts, float* __restrict__ out) {
    __shared__ float sa[256], sc[256];
    float a = 0.f, c = 0.f;
    for (int i = threadIdx.x; i < nparts; i += blockDim.x) {
        a += part[2 * i];
        c += part[2 * i + 1];
    }
    sa[threadIdx.x] = a;
    sc[threadIdx.x] = c;
    __syncthreads();
    for (int s = blockDim.x / 2; s > 0; s >>= 1) {
        if (threadIdx.x < s) {
            sa[threadIdx.x] += sa[threadIdx.x + s];
            sc[threadIdx.x] += sc[threadIdx.x + s];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        out[0] = sa[0] / sc[0];
        out[1] = sc[0];
    }
}

__global__ __launch_bounds__(256) void bce_bwd_kernel(const float* __restrict__ p, const float* __restrict__ n,
                                                      const uint8_t* __restrict__ mask, int64_t T,
                                                      const float* __restrict__ dloss,
                                                      const float* __restrict__ stats, float* __restrict__ gp,
                                                      float* __restrict__ gn) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= T) return;
    const float m = mask[t] ? 1.f : 0.f;
    const float g = -dloss[0] / stats[1] * m;  // d loss / d log-term, for both terms
    const float sp = sigmoidf_ref(p[t]);
    const float sn = sigmoidf_ref(n[t]);
    gp[t] = (g / (sp + 1e-24f)) * (1.f - sp) * sp;
    const float tn = 1.f - sn;
    gn[t] = -(g / (tn + 1e-24f)) * (1.f - sn) * sn;
}

// ---------------------------------------------------------------- cross-entropy over a full catalogue
__device__ __forceinline__ void online_merge(float& m, float& s, float m2, float s2) {
    if (m2 == -INFINITY) return;  // empty partner (fewer classes than threads)
    if (m == -INFINITY) {
        m = m2;
        s = s2;
        return;
    }
    const float mn = fmaxf(m, m2);
    s = s * __expf(m - mn) + s2 * __expf(m2 - mn);
    m = mn;
}

__global__ __launch_bounds__(256) void ce_fwd_kernel(const float* __restrict__ logits, int64_t ld,
                                                     const int64_t* __restrict__ targets, int64_t ignore_index,
                                                     int64_t M, int64_t V, float* __restrict__ lse,
                                                     float* __restrict__ row_loss) {
    const int64_t r = blockIdx.x;
    const float* x = logits + r * ld;
    const int64_t tg = targets[r];
    float m = -INFINITY, s = 0.f;
    auto add1 = [&](float v) {
        if (v > m) {
            s = s * __expf(m - v) + 1.f;
            m = v;
        } else {
            s += __expf(v - m);
        }
    };
    // rows of an odd-length catalogue are not 16-B aligned: a scalar head, float4 body (two in flight), tail
    const int64_t head = min(V, (int64_t)(((16 - ((uintptr_t)x & 15)) & 15) >> 2));
    if (threadIdx.x < head) add1(x[threadIdx.x]);
    const float4* x4 = reinterpret_cast<const float4*>(x + head);
    const int64_t n4 = (V - head) >> 2;
    auto add4 = [&](const float4& v) {
        const float mx = fmaxf(fmaxf(v.x, v.y), fmaxf(v.z, v.w));
        if (mx > m) {
            s *= __expf(m - mx);
            m = mx;
        }
        s += (__expf(v.x - m) + __expf(v.y - m)) + (__expf(v.z - m) + __expf(v.w - m));
    };
    int64_t j = threadIdx.x;
    for (; j + blockDim.x < n4; j += 2 * blockDim.x) {
        const float4 a = x4[j], b = x4[j + blockDim.x];
        add4(a);
        add4(b);
    }
    if (j < n4) add4(x4[j]);
    for (int64_t k = head + 4 * n4 + threadIdx.x; k < V; k += blockDim.x) add1(x[k]);
    // wave-level merge
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
        online_merge(m, s, m2, s2);
    }
    __shared__ float sm[kWaves], ss[kWaves];
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        sm[w] = m;
        ss[w] = s;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float mm = sm[0], s0 = ss[0];
        for (int i = 1; i < kWaves; ++i) online_merge(mm, s0, sm[i], ss[i]);
        const float l = mm + logf(s0);
        lse[r] = l;
        const bool valid = tg != ignore_index && tg >= 0 && tg < V;
        row_loss[r] = valid ? l - x[tg] : 0.f;
    }
}

__global__ void ce_finish_kernel(const float* __restrict__ row_loss, const int64_t* __restrict__ targets,
                                 int64_t ignore_index, int64_t M, int64_t V, float* __restrict__ out) {
    __shared__ float sa[256], sc[256];
    float a = 0.f, c = 0.f;
    for (int64_t i = threadIdx.x; i < M; i += blockDim.x) {
        const int64_t tg = targets[i];
        const bool valid = tg != ignore_index && tg >= 0 && tg < V;
        a += row_loss[i];
        c += valid ? 1.f : 0.f;
    }
    sa[threadIdx.x] = a;
    sc[threadIdx.x] = c;
    __syncthreads();
    for (int s = blockDim.x / 2; s > 0; s >>= 1) {
        if (threadIdx.x < s) {
            sa[threadIdx.x] += sa[threadIdx.x + s];
            sc[threadIdx.x] += sc[threadIdx.x + s];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        out[0] = sa[0] / sc[0];  // mean over non-ignored rows (NaN when none, like torch)
        out[1] = sc[0];
    }
}

__global__ __launch_bounds__(256) void ce_bwd_kernel(const float* __restrict__ logits, int64_t ld,
                                                     const float* __restrict__ lse,
                                                     const int64_t* __restrict__ targets, int64_t ignore_index,
                                                     int64_t V, const float* __restrict__ dloss,
                                                     const float* __restrict__ stats, float* __restrict__ dlogits,
                                                     int64_t ldg) {
    const int64_t r = blockIdx.y;
    const int64_t tg = targets[r];
    const bool valid = tg != ignore_index && tg >= 0 && tg < V;
    const float scale = valid ? dloss[0] / stats[1] : 0.f;
    const float l = lse[r];
    const float* x = logits + r * ld;
    float* y = dlogits + r * ldg;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x, t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if ((((uintptr_t)x ^ (uintptr_t)y) & 15) == 0) {  // same alignment: scalar head, float4 body, scalar tail
        const int64_t head = min(V, (int64_t)(((16 - ((uintptr_t)x & 15)) & 15) >> 2));
        for (int64_t j = t0; j < head; j += stride) y[j] = scale * (__expf(x[j] - l) - (j == tg ? 1.f : 0.f));
        const float4* x4 = reinterpret_cast<const float4*>(x + head);
        float4* y4 = reinterpret_cast<float4*>(y + head);
        const int64_t n4 = (V - head) >> 2;
        for (int64_t j = t0; j < n4; j += stride) {
            const float4 v = x4[j];
            const int64_t c = head + 4 * j;
            y4[j] = make_float4(scale * (__expf(v.x - l) - (c == tg ? 1.f : 0.f)),
                                scale * (__expf(v.y - l) - (c + 1 == tg ? 1.f : 0.f)),
                                scale * (__expf(v.z - l) - (c + 2 == tg ? 1.f : 0.f)),
                                scale * (__expf(v.w - l) - (c + 3 == tg ? 1.f : 0.f)));
        }
        for (int64_t j = head + 4 * n4 + t0; j < V; j += stride)
            y[j] = scale * (__expf(x[j] - l) - (j == tg ? 1.f : 0.f));
        return;
    }
    for (int64_t j = t0; j < V; j += stride) {
        const float pj = __expf(x[j] - l);
        y[j] = scale * (pj - (j == tg ? 1.f : 0.f));
    }
}

// ---------------------------------------------------------------- rank of the target item
// rank = 1 + #{j : s_j > s_t} + #{j < t : s_j == s_t}  (descending sort, ties broken by lower id first)
__global__ __launch_bounds__(256) void target_rank_kernel(const float* __restrict__ scores, int64_t ld,
                                                          const int64_t* __restrict__ targets, int64_t V,
                                                          int64_t* __restrict__ ranks) {
    const int64_t r = blockIdx.x;
    const float* x = scores + r * ld;
    const int64_t tg = targets[r];
    const float st = x[tg];
    unsigned long long cnt = 0;
    for (int64_t j = threadIdx.x; j < V; j += blockDim.x) {
        const float v = x[j];
        cnt += (v > st || (v == st && j < tg)) ? 1ull : 0ull;
    }
    __shared__ unsigned long long sc[256];
    sc[threadIdx.x] = cnt;
    __syncthreads();
    for (int s = blockDim.x / 2; s > 0; s >>= 1) {
        if (threadIdx.x < s) sc[threadIdx.x] += sc[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0) ranks[r] = (int64_t)sc[0] + 1;
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

ASME_API int asme_sampled_logits_fwd(const float* hidden, const float* table, const int64_t* pos_ids,
                                     const int64_t* neg_ids, int64_t n_tokens, int64_t dim, int64_t vocab,
                                     float* pos_out, float* neg_out, void* stream) {
    ASME_CHECK_ARG(hidden && table && pos_ids && neg_ids && pos_out && neg_out, "asme_sampled_logits_fwd: null");
    if (n_tokens == 0) return 0;
    if (dim % 4 == 0 && (((uintptr_t)hidden | (uintptr_t)table) & 15) == 0) {
        if (with_head_layout(dim, [&](auto layout) {
                using R = decltype(layout);
                if constexpr (R::W == 4) {
                    const int64_t per = (int64_t)kWaves * R::RPW * kHeadK;
                    hipLaunchKernelGGL(HIP_KERNEL_NAME(sampled_fwd4_kernel<R, kHeadK>),
                                       dim3((unsigned)((n_tokens + per - 1) / per)), dim3(256), 0, (hipStream_t)stream,
                                       hidden, table, pos_ids, neg_ids, n_tokens, (int)dim, vocab, pos_out, neg_out);
                }
            }))
            return -1;
        ASME_LAUNCH_CHECK("asme_sampled_logits_fwd");
    }
    const dim3 grid((unsigned)((n_tokens + kWaves - 1) / kWaves));
    ASME_VPL_DISPATCH(vpl_of(dim), hipLaunchKernelGGL(sampled_fwd_kernel<VPL>, grid, dim3(256), 0,
                                                      (hipStream_t)stream, hidden, table, pos_ids, neg_ids, n_tokens,
                                                      (int)dim, vocab, pos_out, neg_out));
    ASME_LAUNCH_CHECK("asme_sampled_logits_fwd");
}

ASME_API int asme_sampled_logits_bwd(const float* hidden, const float* table, const int64_t* pos_ids,
                                     const int64_t* neg_ids, int64_t n_tokens, int64_t dim, int64_t vocab,
                                     const float* g_pos, const float* g_neg, float* d_hidden, float* d_table,
                                     void* stream) {
    ASME_CHECK_ARG(hidden && table && pos_ids && neg_ids && g_pos && g_neg, "asme_sampled_logits_bwd: null");
    if (n_tokens == 0) return 0;
    if (dim % 4 == 0 && (((uintptr_t)hidden | (uintptr_t)table | (uintptr_t)d_hidden) & 15) == 0) {
        if (with_head_layout(dim, [&](auto layout) {
                using R = decltype(layout);
                if constexpr (R::W == 4) {
                    const int64_t per = (int64_t)kWaves * R::RPW * kHeadK;
                    hipLaunchKernelGGL(HIP_KERNEL_NAME(sampled_bwd4_kernel<R, kHeadK>),
                                       dim3((unsigned)((n_tokens + per - 1) / per)), dim3(256), 0, (hipStream_t)stream,
                                       hidden, table, pos_ids, neg_ids, n_tokens, (int)dim, vocab, g_pos, g_neg,
                                       d_hidden, d_table);
                }
            }))
            return -1;
        ASME_LAUNCH_CHECK("asme_sampled_logits_bwd");
    }
    const dim3 grid((unsigned)((n_tokens + kWaves - 1) / kWaves));
    ASME_VPL_DISPATCH(vpl_of(dim), hipLaunchKernelGGL(sampled_bwd_kernel<VPL>, grid, dim3(256), 0,
                                                      (hipStream_t)stream, hidden, table, pos_ids, neg_ids, n_tokens,
                                                      (int)dim, vocab, g_pos, g_neg, d_hidden, d_table));
    ASME_LAUNCH_CHECK("asme_sampled_logits_bwd");
}

ASME_API int asme_sasrec_bce_fwd(const float* pos_logits, const float* neg_logits, const uint8_t* mask,
                                 int64_t n_tokens, float* workspace, int64_t n_parts, float* out, void* stream) {
    ASME_CHECK_ARG(pos_logits && neg_logits && mask && workspace && out && n_parts >= 1,
                   "asme_sasrec_bce_fwd: bad argument");
    hipLaunchKernelGGL(bce_fwd_kernel, dim3((unsigned)n_parts), dim3(256), 0, (hipStream_t)stream, pos_logits,
                       neg_logits, mask, n_tokens, workspace);
    hipLaunchKernelGGL(bce_finish_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, workspace, (int)n_parts, out);
    ASME_LAUNCH_CHECK("asme_sasrec_bce_fwd");
}

ASME_API int asme_sasrec_bce_bwd(const float* pos_logits, const float* neg_logits, const uint8_t* mask,
                                 int64_t n_tokens, const float* dloss, const float* stats, float* g_pos, float* g_neg,
                                 void* stream) {
    ASME_CHECK_ARG(pos_logits && neg_logits && mask && dloss && stats && g_pos && g_neg,
                   "asme_sasrec_bce_bwd: null pointer");
    if (n_tokens == 0) return 0;
    hipLaunchKernelGGL(bce_bwd_kernel, dim3((unsigned)((n_tokens + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       pos_logits, neg_logits, mask, n_tokens, dloss, stats, g_pos, g_neg);
    ASME_LAUNCH_CHECK("asme_sasrec_bce_bwd");
}

ASME_API int asme_cross_entropy_fwd(const float* logits, int64_t ld, const int64_t* targets, int64_t ignore_index,
                                    int64_t n_rows, int64_t n_classes, float* lse, float* row_loss, float* out,
                                    void* stream) {
    ASME_CHECK_ARG(logits && targets && lse && row_loss && out, "asme_cross_entropy_fwd: null pointer");
    ASME_CHECK_ARG(n_rows >= 1 && n_classes >= 1 && ld >= n_classes, "asme_cross_entropy_fwd: bad shape");
    hipLaunchKernelGGL(ce_fwd_kernel, dim3((unsigned)n_rows), dim3(256), 0, (hipStream_t)stream, logits, ld, targets,
                       ignore_index, n_rows, n_classes, lse, row_loss);
    hipLaunchKernelGGL(ce_finish_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, row_loss, targets, ignore_index,
                       n_rows, n_classes, out);
    ASME_LAUNCH_CHECK("asme_cross_entropy_fwd");
}

ASME_API int asme_cross_entropy_bwd(const float* logits, int64_t ld, const float* lse, const int64_t* targets,
                                    int64_t ignore_index, int64_t n_rows, int64_t n_classes, const float* dloss,
                                    const float* stats, float* dlogits, int64_t ld_dlogits, void* stream) {
    ASME_CHECK_ARG(logits && lse && targets && dloss && stats && dlogits, "asme_cross_entropy_bwd: null pointer");
    if (n_rows == 0) return 0;
    const int64_t bx = std::min<int64_t>((n_classes + 4095) / 4096, 64);  // ~4 float4 per thread
    hipLaunchKernelGGL(ce_bwd_kernel, dim3((unsigned)bx, (unsigned)n_rows), dim3(256), 0, (hipStream_t)stream,
                       logits, ld, lse, targets, ignore_index, n_classes, dloss, stats, dlogits, ld_dlogits);
    ASME_LAUNCH_CHECK("asme_cross_entropy_bwd");
}

ASME_API int asme_target_rank(const float* scores, int64_t ld, const int64_t* targets, int64_t n_rows,
                              int64_t n_items, int64_t* ranks, void* stream) {
    ASME_CHECK_ARG(scores && targets && ranks, "asme_target_rank: null pointer");
    if (n_rows == 0) return 0;
    hipLaunchKernelGGL(target_rank_kernel, dim3((unsigned)n_rows), dim3(256), 0, (hipStream_t)stream, scores, ld,
                       targets, n_items, ranks);
    ASME_LAUNCH_CHECK("asme_target_rank");
}
