// Full-catalogue evaluation without materialising the (queries x |V|) logits, fp32 MFMA on gfx950.
//
// Reference semantics (paths relative to /root/reference/src/asme):
//   SASRecProjectionComponent inference branch   core/models/sasrec/components.py:46-61  (E[items] . h)
//   ItemEmbeddingProjectionLayer (tied + bias)   core/models/common/layers/layers.py:138-143
//   AllItemsSampler + calc_ndcg / get_true_positives / argsort
//                                                core/metrics/container/metrics_sampler.py:51-72,
//                                                core/metrics/common.py:4-27,118-175
// The reference builds (B, |V|, d) item rows, scores every item, argsorts (B, |V|) and reads the
// positives off the top-k.  Here the scores stream through registers:
//   asme_catalog_rank  rank of each query's target = 1 + #{items scoring higher, ties to the lower id}
//                      (single-target NDCG / recall / MRR need nothing else)
//   asme_catalog_topk  the k best (score, item) per query, ties to the lower id
// score(q, i) = h_q . E_i (+ bias_i).  A workgroup = 4 waves x NQT 16-query tiles streams a contiguous item
// range through LDS in 64-item tiles (register-prefetched); S^T = E_tile H^T on v_mfma_f32_16x16x4f32
// exactly as the attention kernels compute K Q^T.  The target's own score is computed by the same MFMA
// sequence (a 16-row tile of the targets' rows), so it compares bit-identically with itself.
#include "common.h"
#include <algorithm>

using namespace asme;

namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int kIT = 64;       // items per LDS tile
constexpr int kNS = kIT / 16; // 16-item sub-tiles
constexpr int kThreads = 256;

__device__ __forceinline__ floatx4 mfma16(float a, float b, floatx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// acc[sub] += Tile[sub*16 + c16][slice g] . f   (lane group g owns features g*D/4 .. +D/4)
template <int D>
__device__ __forceinline__ void tile_dot(const float* __restrict__ tile, int g, int c16, const float (&f)[D / 4],
                                         floatx4 (&acc)[kNS]) {
    constexpr int S = D + 4, DQ = D / 4;
#pragma unroll
    for (int s4 = 0; s4 < DQ / 4; ++s4) {
        float4 a[kNS];
#pragma unroll
        for (int sub = 0; sub < kNS; ++sub)
            a[sub] = *reinterpret_cast<const float4*>(tile + (sub * 16 + c16) * S + g * DQ + 4 * s4);
#pragma unroll
        for (int sub = 0; sub < kNS; ++sub) acc[sub] = mfma16(a[sub].x, f[4 * s4], acc[sub]);
#pragma unroll
        for (int sub = 0; sub < kNS; ++sub) acc[sub] = mfma16(a[sub].y, f[4 * s4 + 1], acc[sub]);
#pragma unroll
        for (int sub = 0; sub < kNS; ++sub) acc[sub] = mfma16(a[sub].z, f[4 * s4 + 2], acc[sub]);
#pragma unroll
        for (int sub = 0; sub < kNS; ++sub) acc[sub] = mfma16(a[sub].w, f[4 * s4 + 3], acc[sub]);
    }
}

// 64 rows x D staged through registers: thread t holds float4 q of (row, col4) = ((t + 256q) / (D/4), ...)
template <int D>
struct Stage {
    static constexpr int N4 = kIT * D / 4 / kThreads;
    float4 r[N4];
    float b;  // bias of item row0 + threadIdx.x (threads < 64)
    __device__ __forceinline__ void load(const float* __restrict__ E, int64_t ld, int64_t row0, int64_t V,
                                         const float* __restrict__ bias) {
        b = (bias && threadIdx.x < kIT && row0 + threadIdx.x < V) ? bias[row0 + threadIdx.x] : 0.f;
#pragma unroll
        for (int q = 0; q < N4; ++q) {
            const int idx = threadIdx.x + kThreads * q;
            const int row = idx / (D / 4), c4 = (idx % (D / 4)) * 4;
            r[q] = row0 + row < V ? *reinterpret_cast<const float4*>(E + (row0 + row) * ld + c4)
                                  : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }
    __device__ __forceinline__ void store(float* __restrict__ tile, float* __restrict__ bias_s) const {
        if (threadIdx.x < kIT) bias_s[threadIdx.x] = b;
#pragma unroll
        for (int q = 0; q < N4; ++q) {
            const int idx = threadIdx.x + kThreads * q;
            const int row = idx / (D / 4), c4 = (idx % (D / 4)) * 4;
            *reinterpret_cast<float4*>(tile + row * (D + 4) + c4) = r[q];
        }
    }
};

__device__ __forceinline__ bool better(float a, int64_t ia, float b, int64_t ib) {
    return a > b || (a == b && ia < ib);
}

enum Mode { MODE_RANK = 0, MODE_TOPK = 1 };

// grid: (query blocks of 4 * NQT * 16 queries, item chunks)
template <int D, int NQT, int MODE, int K>
__global__ __launch_bounds__(kThreads) void catalog_kernel(const float* __restrict__ H, int64_t ldh, int64_t nq,
                                                           const float* __restrict__ E, int64_t lde, int64_t V,
                                                           const float* __restrict__ bias,
                                                           const int64_t* __restrict__ targets, int64_t chunk,
                                                           int32_t* __restrict__ counts, float* __restrict__ part_val,
                                                           int64_t* __restrict__ part_idx,
                                                           const float* __restrict__ tscore_in,
                                                           float* __restrict__ tscore_out, int64_t id_stride,
                                                           int64_t id_offset) {
    constexpr int DQ = D / 4, S = D + 4;
    __shared__ __attribute__((aligned(16))) float Es[kIT * S];
    __shared__ float Bs[kIT];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c16 = lane & 15;
    const int64_t qbase = (int64_t)blockIdx.x * (4 * NQT * 16) + wave * NQT * 16;
    const int64_t i_begin = (int64_t)blockIdx.y * chunk;
    const int64_t i_end = min(V, i_begin + chunk);

    float hq[NQT][DQ];
#pragma unroll
    for (int t = 0; t < NQT; ++t) {
        const int64_t q = qbase + t * 16 + c16;
#pragma unroll
        for (int s4 = 0; s4 < DQ / 4; ++s4) {
            const float4 v = q < nq ? *reinterpret_cast<const float4*>(H + q * ldh + g * DQ + 4 * s4)
                                    : make_float4(0.f, 0.f, 0.f, 0.f);
            hq[t][4 * s4] = v.x;
            hq[t][4 * s4 + 1] = v.y;
            hq[t][4 * s4 + 2] = v.z;
            hq[t][4 * s4 + 3] = v.w;
        }
    }

    // ---- rank mode: each query's target score through the same MFMA sequence (tile of target rows)
    float tscore[NQT];
    int64_t tid[NQT];
    int cnt[NQT];
    // item ids are global: local row j of this (shard of the) table is item j * id_stride + id_offset
    if constexpr (MODE == MODE_RANK) {
#pragma unroll
        for (int t = 0; t < NQT; ++t) {
            const int64_t qq = qbase + t * 16 + c16;
            cnt[t] = 0;
            if (tscore_in) {  // sharded evaluation: the target's score came from its owner's shard
                tscore[t] = qq < nq ? tscore_in[qq] : 0.f;
                tid[t] = qq < nq ? targets[qq] : -1;
                continue;
            }
            __syncthreads();
            // rows w*16 + j of the 64-row tile = target row of query (wave w, tile t, j)
            for (int idx = threadIdx.x; idx < kIT * (D / 4); idx += kThreads) {
                const int row = idx / (D / 4), c4 = (idx % (D / 4)) * 4;
                const int64_t q = (int64_t)blockIdx.x * (4 * NQT * 16) + (row / 16) * NQT * 16 + t * 16 + row % 16;
                int64_t it = q < nq ? (targets ? targets[q] : q) : 0;
                it = (it < 0 || it >= V) ? 0 : it;
                *reinterpret_cast<float4*>(Es + row * S + c4) = *reinterpret_cast<const float4*>(E + it * lde + c4);
            }
            __syncthreads();
            floatx4 st[kNS];
#pragma unroll
            for (int sub = 0; sub < kNS; ++sub) st[sub] = floatx4{0.f, 0.f, 0.f, 0.f};
            tile_dot<D>(Es, g, c16, hq[t], st);
            // the diagonal (row = c16 of this wave's sub-tile) sits in lane group c16 / 4, register c16 % 4
            float diag = 0.f;
#pragma unroll
            for (int sub = 0; sub < kNS; ++sub)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    if (sub == wave && 4 * g + r == c16) diag = st[sub][r];
            diag = __shfl(diag, (c16 / 4) * 16 + c16, 64);
            const int64_t q = qbase + t * 16 + c16;
            int64_t it = q < nq ? (targets ? targets[q] : q) : 0;
            it = (it < 0 || it >= V) ? 0 : it;
            tid[t] = it * id_stride + id_offset;
            tscore[t] = diag + (bias ? bias[it] : 0.f);
            if (tscore_out && q < nq && g == 0) tscore_out[q] = tscore[t];
        }
        if (tscore_out) return;  // target scores only
    }
    float tv[NQT][MODE == MODE_TOPK ? K : 1];
    int64_t ti[NQT][MODE == MODE_TOPK ? K : 1];
    if constexpr (MODE == MODE_TOPK) {
#pragma unroll
        for (int t = 0; t < NQT; ++t)
#pragma unroll
            for (int j = 0; j < K; ++j) {
                tv[t][j] = -INFINITY;
                ti[t][j] = INT64_MAX;
            }
    }

    Stage<D> stg;
    if (i_begin < i_end) stg.load(E, lde, i_begin, V, bias);
    for (int64_t i0 = i_begin; i0 < i_end; i0 += kIT) {
        __syncthreads();
        stg.store(Es, Bs);
        __syncthreads();
        if (i0 + kIT < i_end) stg.load(E, lde, i0 + kIT, V, bias);
#pragma unroll
        for (int t = 0; t < NQT; ++t) {
            floatx4 st[kNS];
#pragma unroll
            for (int sub = 0; sub < kNS; ++sub) st[sub] = floatx4{0.f, 0.f, 0.f, 0.f};
            tile_dot<D>(Es, g, c16, hq[t], st);
#pragma unroll
            for (int sub = 0; sub < kNS; ++sub)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int64_t row = i0 + sub * 16 + 4 * g + r;
                    if (row >= i_end) continue;
                    const int64_t item = row * id_stride + id_offset;
                    const float s = st[sub][r] + Bs[sub * 16 + 4 * g + r];
                    if constexpr (MODE == MODE_RANK) {
                        cnt[t] += (item != tid[t] && better(s, item, tscore[t], tid[t])) ? 1 : 0;
                    } else {
                        if (better(s, item, tv[t][K - 1], ti[t][K - 1])) {  // bubble into the sorted list
                            float cv = s;
                            int64_t ci = item;
#pragma unroll
                            for (int j = 0; j < K; ++j) {
                                if (better(cv, ci, tv[t][j], ti[t][j])) {
                                    const float fv = tv[t][j];
                                    const int64_t fi = ti[t][j];
                                    tv[t][j] = cv;
                                    ti[t][j] = ci;
                                    cv = fv;
                                    ci = fi;
                                }
                            }
                        }
                    }
                }
        }
    }

#pragma unroll
    for (int t = 0; t < NQT; ++t) {
        const int64_t q = qbase + t * 16 + c16;
        if constexpr (MODE == MODE_RANK) {
            int c = cnt[t];
            c += __shfl_xor(c, 16, 64);
            c += __shfl_xor(c, 32, 64);
            if (g == 0 && q < nq && c) atomicAdd(counts + q, c);
        } else {
            if (q < nq) {
                // partials [chunk][query][g][K]
                const int64_t base = ((int64_t)blockIdx.y * nq + q) * 4 * K + g * K;
#pragma unroll
                for (int j = 0; j < K; ++j) {
                    part_val[base + j] = tv[t][j];
                    part_idx[base + j] = ti[t][j];
                }
            }
        }
    }
}

__global__ void rank_finish_kernel(const int32_t* __restrict__ counts, int64_t n, int64_t* __restrict__ ranks) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) ranks[i] = (int64_t)counts[i] + 1;
}

// one workgroup per query: k rounds of a block-wide argmax over the chunks x 4 x K candidates
__global__ __launch_bounds__(256) void topk_merge_kernel(const float* __restrict__ part_val,
                                                         const int64_t* __restrict__ part_idx, int64_t nq,
                                                         int nchunks, int K, int k, float* __restrict__ out_val,
                                                         int64_t* __restrict__ out_idx) {
    __shared__ float rv[256];
    __shared__ int64_t ri[256];
    __shared__ int rs[256];
    const int64_t q = blockIdx.x;
    const int per_chunk = 4 * K;
    const int ncand = nchunks * per_chunk;
    float last_v = INFINITY;
    int64_t last_i = -1;
    for (int round = 0; round < k; ++round) {
        float bv = -INFINITY;
        int64_t bi = INT64_MAX;
        int bs = -1;
        for (int c = threadIdx.x; c < ncand; c += 256) {
            const int ch = c / per_chunk, j = c % per_chunk;
            const int64_t off = ((int64_t)ch * nq + q) * per_chunk + j;
            const float v = part_val[off];
            const int64_t id = part_idx[off];
            // candidates strictly after the previous winner in the (score desc, id asc) order
            const bool after = better(last_v, last_i, v, id);
            if (after && better(v, id, bv, bi)) {
                bv = v;
                bi = id;
                bs = c;
            }
        }
        rv[threadIdx.x] = bv;
        ri[threadIdx.x] = bi;
        rs[threadIdx.x] = bs;
        __syncthreads();
        for (int h = 128; h > 0; h >>= 1) {
            if (threadIdx.x < h && better(rv[threadIdx.x + h], ri[threadIdx.x + h], rv[threadIdx.x], ri[threadIdx.x])) {
                rv[threadIdx.x] = rv[threadIdx.x + h];
                ri[threadIdx.x] = ri[threadIdx.x + h];
                rs[threadIdx.x] = rs[threadIdx.x + h];
            }
            __syncthreads();
        }
        last_v = rv[0];
        last_i = ri[0];
        if (threadIdx.x == 0) {
            out_val[q * k + round] = rv[0];
            out_idx[q * k + round] = ri[0] == INT64_MAX ? -1 : ri[0];
        }
        __syncthreads();
    }
}

struct Plan {
    int64_t qblocks, chunks, chunk;
};
Plan make_plan(int64_t nq, int64_t V, int queries_per_block) {
    Plan p;
    p.qblocks = (nq + queries_per_block - 1) / queries_per_block;
    const int64_t want = std::max<int64_t>(1, 1024 / std::max<int64_t>(1, p.qblocks));  // ~4 workgroups per CU
    p.chunk = std::max<int64_t>(kIT, ((V + want - 1) / want + kIT - 1) / kIT * kIT);
    p.chunks = (V + p.chunk - 1) / p.chunk;
    return p;
}

constexpr int kTopKSlots = 16;  // per-lane list length (k <= 16)

#define ASME_CAT_DIM(DV, ...)                                    \
    switch (DV) {                                                \
        case 32: { constexpr int D = 32; __VA_ARGS__; } break;   \
        case 64: { constexpr int D = 64; __VA_ARGS__; } break;   \
        case 128: { constexpr int D = 128; __VA_ARGS__; } break; \
        default: set_error("catalog: dim must be 32, 64 or 128"); return -1; \
    }

}  // namespace

// ranks[q] = 1 + #{i : score(q,i) > score(q,t_q), or equal with i < t_q}, score = H[q] . E[i] (+ bias[i]).
// counts_ws: nq int32 scratch.  H: (nq x dim, row stride ld_h); E: (V x dim, row stride ld_e).
ASME_API int asme_catalog_rank(const float* H, int64_t ld_h, int64_t nq, int64_t dim, const float* E, int64_t ld_e,
                               int64_t V, const float* bias, const int64_t* targets, int32_t* counts_ws,
                               int64_t* ranks, void* stream) {
    ASME_CHECK_ARG(H && E && targets && counts_ws && ranks, "asme_catalog_rank: null pointer");
    ASME_CHECK_ARG(ld_h % 4 == 0 && ld_e % 4 == 0 && ((uintptr_t)H & 15) == 0 && ((uintptr_t)E & 15) == 0,
                   "asme_catalog_rank: rows must be 16-B aligned");
    if (nq == 0) return 0;
    hipStream_t s = (hipStream_t)stream;
    if (hipMemsetAsync(counts_ws, 0, nq * sizeof(int32_t), s) != hipSuccess) return hip_status(hipGetLastError(), "memset");
    constexpr int NQT = 2;
    const Plan p = make_plan(nq, V, 4 * NQT * 16);
    ASME_CAT_DIM(dim, hipLaunchKernelGGL((catalog_kernel<D, NQT, MODE_RANK, 1>), dim3((unsigned)p.qblocks, (unsigned)p.chunks),
                                         dim3(kThreads), 0, s, H, ld_h, nq, E, ld_e, V, bias, targets, p.chunk, counts_ws,
                                         nullptr, nullptr, nullptr, nullptr, (int64_t)1, (int64_t)0));
    hipLaunchKernelGGL(rank_finish_kernel, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, s, counts_ws, nq, ranks);
    ASME_LAUNCH_CHECK("asme_catalog_rank");
}

ASME_API int64_t asme_catalog_topk_workspace(int64_t nq, int64_t V, int64_t dim) {
    const Plan p = make_plan(nq, V, 4 * 16);
    (void)dim;
    return p.chunks * nq * 4 * kTopKSlots * (int64_t)(sizeof(float) + sizeof(int64_t)) + 16;
}

// the k (<= 16) best (score, item) per query, scores descending, ties to the lower item id
ASME_API int asme_catalog_topk(const float* H, int64_t ld_h, int64_t nq, int64_t dim, const float* E, int64_t ld_e,
                               int64_t V, const float* bias, int64_t id_stride, int64_t id_offset, int64_t k, void* ws,
                               int64_t ws_bytes, float* out_val, int64_t* out_idx, void* stream) {
    ASME_CHECK_ARG(H && E && ws && out_val && out_idx, "asme_catalog_topk: null pointer");
    ASME_CHECK_ARG(k >= 1 && k <= kTopKSlots, "asme_catalog_topk: k must be in [1, 16]");
    ASME_CHECK_ARG(ld_h % 4 == 0 && ld_e % 4 == 0 && ((uintptr_t)H & 15) == 0 && ((uintptr_t)E & 15) == 0,
                   "asme_catalog_topk: rows must be 16-B aligned");
    ASME_CHECK_ARG(ws_bytes >= asme_catalog_topk_workspace(nq, V, dim), "asme_catalog_topk: workspace too small");
    if (nq == 0) return 0;
    hipStream_t s = (hipStream_t)stream;
    const Plan p = make_plan(nq, V, 4 * 16);
    float* pv = reinterpret_cast<float*>(ws);
    int64_t* pi = reinterpret_cast<int64_t*>(reinterpret_cast<char*>(ws) +
                                             ((p.chunks * nq * 4 * kTopKSlots * sizeof(float) + 15) & ~size_t(15)));
    ASME_CAT_DIM(dim, hipLaunchKernelGGL((catalog_kernel<D, 1, MODE_TOPK, kTopKSlots>),
                                         dim3((unsigned)p.qblocks, (unsigned)p.chunks), dim3(kThreads), 0, s, H, ld_h,
                                         nq, E, ld_e, V, bias, nullptr, p.chunk, nullptr, pv, pi, nullptr, nullptr,
                                         id_stride, id_offset));
    hipLaunchKernelGGL(topk_merge_kernel, dim3((unsigned)nq), dim3(256), 0, s, pv, pi, nq, (int)p.chunks, kTopKSlots,
                       (int)k, out_val, out_idx);
    ASME_LAUNCH_CHECK("asme_catalog_topk");
}

// Sharded evaluation (table rows held cyclically: local row j = item j * id_stride + id_offset).
// (1) target scores from the gathered target rows (rows[q] = E[target_q]) through the same MFMA sequence the
//     owner's shard scan uses, so they compare bit-identically there;
ASME_API int asme_catalog_target_scores(const float* H, int64_t ld_h, int64_t nq, int64_t dim, const float* rows,
                                        int64_t ld_rows, const float* row_bias, float* tscore, void* stream) {
    ASME_CHECK_ARG(H && rows && tscore, "asme_catalog_target_scores: null pointer");
    if (nq == 0) return 0;
    constexpr int NQT = 2;
    const int64_t qblocks = (nq + 4 * NQT * 16 - 1) / (4 * NQT * 16);
    // targets == NULL: query q's target is gathered row q (row_bias likewise per query)
    ASME_CAT_DIM(dim, hipLaunchKernelGGL((catalog_kernel<D, NQT, MODE_RANK, 1>), dim3((unsigned)qblocks, 1u), dim3(kThreads),
                                         0, (hipStream_t)stream, H, ld_h, nq, rows, ld_rows, nq, row_bias, nullptr,
                                         (int64_t)kIT, nullptr, nullptr, nullptr, nullptr, tscore, (int64_t)1, (int64_t)0));
    ASME_LAUNCH_CHECK("asme_catalog_target_scores");
}

// (2) per-shard counts of items above each query's target (global ids, ties to the lower id); the ranks
//     are 1 + the all-reduced sum over shards.  counts (nq int32) is overwritten.
ASME_API int asme_catalog_count_above(const float* H, int64_t ld_h, int64_t nq, int64_t dim, const float* E,
                                      int64_t ld_e, int64_t V_local, const float* bias, const int64_t* targets,
                                      const float* tscore, int64_t id_stride, int64_t id_offset, int32_t* counts,
                                      void* stream) {
    ASME_CHECK_ARG(H && E && targets && tscore && counts, "asme_catalog_count_above: null pointer");
    if (nq == 0) return 0;
    hipStream_t s = (hipStream_t)stream;
    if (hipMemsetAsync(counts, 0, nq * sizeof(int32_t), s) != hipSuccess) return hip_status(hipGetLastError(), "memset");
    constexpr int NQT = 2;
    const Plan p = make_plan(nq, V_local, 4 * NQT * 16);
    ASME_CAT_DIM(dim, hipLaunchKernelGGL((catalog_kernel<D, NQT, MODE_RANK, 1>), dim3((unsigned)p.qblocks, (unsigned)p.chunks),
                                         dim3(kThreads), 0, s, H, ld_h, nq, E, ld_e, V_local, bias, targets, p.chunk,
                                         counts, nullptr, nullptr, tscore, nullptr, id_stride, id_offset));
    ASME_LAUNCH_CHECK("asme_catalog_count_above");
}
