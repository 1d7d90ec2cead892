// Full-catalogue logits head fused with CrossEntropyLoss(ignore_index) on gfx950 fp32 MFMA: the (n x |V|)
// logits of BERT4Rec / KeBERT4Rec / SASRec-cross training are never written to HBM.
//
// Reference semantics (paths relative to /root/reference/src/asme):
//   LinearProjectionLayer.forward / ItemEmbeddingProjectionLayer.forward (tied h E^T + b)
//                                       core/models/common/layers/layers.py:105-109, 138-143   
//   MaskedTrainingModule._calc_loss / SingleTargetCrossEntropyLoss (CrossEntropyLoss(ignore_index=pad),
//   mean over non-ignored rows)         core/modules/masked_training_module.py:93-111, core/losses/losses.py:77-115
// The reference computes (B, L, |V|) logits and a dense log_softmax over them (22 GB at C3).
//
//   s[q][i] = H[q] . W[i] + b[i],   lse[q] = log sum_i exp s[q][i],   loss = mean_{valid q} (lse[q] - s[q][t_q])
//   dS = (softmax(s) - onehot(t)) * dloss / count;   dH = dS W;   dW = dS^T H;   db = colsum(dS)
//
// Three MFMA passes over the (query, item) plane, each recomputing s through registers:
//   stats  (queries in registers, items streamed through LDS in 64-row tiles): online (max, sum exp) per
//          query per item chunk + the target logit; a finish kernel merges the chunks into lse and the loss.
//   dH     same tiling: P = exp(s - lse) - onehot, dH += P W_tile (P feeds the MFMA A operand straight from
//          the S^T accumulator registers: lane (g, c16) holds query c16 x items 4g..4g+3 of a 16-item
//          sub-tile, exactly the (row c16, k = g) element the next 16x16x4 MFMA needs).
//   dW,db  transposed: items in registers, queries streamed through LDS; S = H_tile W^T puts query
//          4g+r x item c16 in lane (g, c16), again the A operand of dW += P^T H_tile.
// Work: 2 + 4 + 4 = 10 n|V|d FLOP (vs 6 for the materialised GEMMs) and O((n + |V|) d) HBM bytes
// (vs 4 n|V| bytes written + read several times).  Item chunks (stats, dH) and query chunks (dW) fill the
// chip; their partial slabs are summed in a fixed order (deterministic).
#include "common.h"
#include <algorithm>

using namespace asme;

namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int kT = 64;        // rows per LDS tile
constexpr int kNS = kT / 16;  // 16-row sub-tiles per tile
constexpr int kThreads = 256;
// 16-query tiles per wave (stats, dH) and 16-item tiles per wave (dW).  Measured at C3 (37k x 27k x 128):
// NQT 1 / 2 -> fwd 3.86 / 3.28 ms, bwd 12.4 / 11.0 ms; NIT 1 and 2 within noise.
constexpr int kNQTsel = 2, kNITsel = 1;

__device__ __forceinline__ floatx4 mfma16(float a, float b, floatx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// kT rows x D of a row-major matrix staged through registers (prefetch of the next tile while the
// current one is used); rows at or beyond `end` are zero.
template <int D>
struct Stage {
    static constexpr int N4 = kT * D / 4 / kThreads;
    float4 r[N4];
    __device__ __forceinline__ void load(const float* __restrict__ X, int64_t ld, int64_t row0, int64_t end) {
#pragma unroll
        for (int q = 0; q < N4; ++q) {
            const int idx = threadIdx.x + kThreads * q;
            const int row = idx / (D / 4), c4 = (idx % (D / 4)) * 4;
            r[q] = row0 + row < end ? *reinterpret_cast<const float4*>(X + (row0 + row) * ld + c4)
                                    : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }
    __device__ __forceinline__ void store(float* __restrict__ tile) const {
#pragma unroll
        for (int q = 0; q < N4; ++q) {
            const int idx = threadIdx.x + kThreads * q;
            const int row = idx / (D / 4), c4 = (idx % (D / 4)) * 4;
            *reinterpret_cast<float4*>(tile + row * (D + 4) + c4) = r[q];
        }
    }
};

// Per-wave registers of NT 16-row tiles of X (rows base + t*16 + c16): lane group g owns features
// g*D/4 .. g*D/4 + D/4 - 1, the k-slice it feeds to the 16x16x4 MFMAs.
template <int D, int NT>
__device__ __forceinline__ void load_rows(const float* __restrict__ X, int64_t ld, int64_t base, int64_t end, int g,
                                          int c16, float (&x)[NT][D / 4]) {
    constexpr int DQ = D / 4;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const int64_t r = base + t * 16 + c16;
#pragma unroll
        for (int s4 = 0; s4 < DQ / 4; ++s4) {
            const float4 v = r < end ? *reinterpret_cast<const float4*>(X + r * ld + g * DQ + 4 * s4)
                                     : make_float4(0.f, 0.f, 0.f, 0.f);
            x[t][4 * s4] = v.x;
            x[t][4 * s4 + 1] = v.y;
            x[t][4 * s4 + 2] = v.z;
            x[t][4 * s4 + 3] = v.w;
        }
    }
}

// acc[t][sub] += Tile[sub*16 + c16][g-slice] . x[t]   -> lane (g, c16): (tile row sub*16 + 4g + r, register row c16)
template <int D, int NT>
__device__ __forceinline__ void tile_times_rows(const float* __restrict__ tile, int g, int c16,
                                                const float (&x)[NT][D / 4], floatx4 (&acc)[NT][kNS]) {
    constexpr int S = D + 4, DQ = D / 4;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int sub = 0; sub < kNS; ++sub) acc[t][sub] = floatx4{0.f, 0.f, 0.f, 0.f};
    // two-stage register ring for the LDS row reads (step s4+1 issued before step s4's MFMAs): bounded
    // register use (the fully unrolled loop otherwise keeps every step's reads live) and the LDS latency
    // off the MFMA stream
    float4 ab[2][kNS];
    const float* base = tile + c16 * S + g * DQ;
#pragma unroll
    for (int sub = 0; sub < kNS; ++sub) ab[0][sub] = *reinterpret_cast<const float4*>(base + sub * 16 * S);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s4 = 0; s4 < DQ / 4; ++s4) {
        if (s4 + 1 < DQ / 4) {
#pragma unroll
            for (int sub = 0; sub < kNS; ++sub)
                ab[(s4 + 1) & 1][sub] = *reinterpret_cast<const float4*>(base + sub * 16 * S + 4 * (s4 + 1));
        }
        __builtin_amdgcn_sched_barrier(0);
        const float4(&a)[kNS] = ab[s4 & 1];
        // consecutive MFMAs write different accumulators (dependent latency 40 > issue 32 cycles)
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int sub = 0; sub < kNS; ++sub) acc[t][sub] = mfma16(a[sub].x, x[t][4 * s4], acc[t][sub]);
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int sub = 0; sub < kNS; ++sub) acc[t][sub] = mfma16(a[sub].y, x[t][4 * s4 + 1], acc[t][sub]);
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int sub = 0; sub < kNS; ++sub) acc[t][sub] = mfma16(a[sub].z, x[t][4 * s4 + 2], acc[t][sub]);
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int sub = 0; sub < kNS; ++sub) acc[t][sub] = mfma16(a[sub].w, x[t][4 * s4 + 3], acc[t][sub]);
    }
}

__device__ __forceinline__ bool valid_target(int64_t t, int64_t ignore, int64_t V) {
    return t != ignore && t >= 0 && t < V;
}

// ---------------------------------------------------------------------------------------------- stats
// grid (query blocks of 4*kNQT*16, item chunks).  part[(chunk * n + q) * 2] = (max, sum exp(s - max)).
template <int D, int kNQT>
__global__ __launch_bounds__(kThreads) void lce_stats_kernel(const float* __restrict__ H, int64_t ldh, int64_t n,
                                                             const float* __restrict__ W, int64_t ldw, int64_t V,
                                                             const float* __restrict__ bias,
                                                             const int64_t* __restrict__ targets, int64_t chunk,
                                                             float* __restrict__ part, float* __restrict__ tlogit) {
    constexpr int DQ = D / 4;
    __shared__ __attribute__((aligned(16))) float Ws[kT * (D + 4)];
    __shared__ float Bs[kT];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c16 = lane & 15;
    const int64_t qbase = (int64_t)blockIdx.x * (4 * kNQT * 16) + wave * kNQT * 16;
    const int64_t i_begin = (int64_t)blockIdx.y * chunk, i_end = min(V, i_begin + chunk);
    float hq[kNQT][DQ];
    load_rows<D, kNQT>(H, ldh, qbase, n, g, c16, hq);
    int64_t tq[kNQT];
    float mx[kNQT], sm[kNQT];
#pragma unroll
    for (int t = 0; t < kNQT; ++t) {
        const int64_t q = qbase + t * 16 + c16;
        tq[t] = q < n ? targets[q] : -1;
        mx[t] = -INFINITY;
        sm[t] = 0.f;
    }
    Stage<D> st;
    st.load(W, ldw, i_begin, i_end);
    float bnext = (threadIdx.x < kT && i_begin + threadIdx.x < i_end && bias) ? bias[i_begin + threadIdx.x] : 0.f;
    for (int64_t i0 = i_begin; i0 < i_end; i0 += kT) {
        __syncthreads();
        st.store(Ws);
        if (threadIdx.x < kT) Bs[threadIdx.x] = bnext;
        __syncthreads();
        if (i0 + kT < i_end) {
            st.load(W, ldw, i0 + kT, i_end);
            bnext = (threadIdx.x < kT && i0 + kT + threadIdx.x < i_end && bias) ? bias[i0 + kT + threadIdx.x] : 0.f;
        }
        floatx4 acc[kNQT][kNS];
        tile_times_rows<D, kNQT>(Ws, g, c16, hq, acc);
#pragma unroll
        for (int t = 0; t < kNQT; ++t) {
            float v[kNS][4];
            float tmax = -INFINITY;
#pragma unroll
            for (int sub = 0; sub < kNS; ++sub)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int j = sub * 16 + 4 * g + r;
                    const int64_t item = i0 + j;
                    const float s = acc[t][sub][r] + Bs[j];
                    v[sub][r] = item < i_end ? s : -INFINITY;
                    tmax = fmaxf(tmax, v[sub][r]);
                    if (item == tq[t]) tlogit[qbase + t * 16 + c16] = s;
                }
            const float nm = fmaxf(mx[t], tmax);
            if (nm == -INFINITY) continue;
            float s = 0.f;
#pragma unroll
            for (int sub = 0; sub < kNS; ++sub)
#pragma unroll
                for (int r = 0; r < 4; ++r) s += __expf(v[sub][r] - nm);
            sm[t] = sm[t] * __expf(mx[t] - nm) + s;
            mx[t] = nm;
        }
    }
    // merge the 4 lane groups of each query (items 4g..4g+3 of every sub-tile)
#pragma unroll
    for (int t = 0; t < kNQT; ++t) {
#pragma unroll
        for (int o = 16; o <= 32; o <<= 1) {
            const float m2 = __shfl_xor(mx[t], o, 64), s2 = __shfl_xor(sm[t], o, 64);
            const float nm = fmaxf(mx[t], m2);
            if (nm != -INFINITY) {
                sm[t] = sm[t] * __expf(mx[t] - nm) + s2 * __expf(m2 - nm);
                mx[t] = nm;
            }
        }
        const int64_t q = qbase + t * 16 + c16;
        if (g == 0 && q < n) {
            part[((int64_t)blockIdx.y * n + q) * 2] = mx[t];
            part[((int64_t)blockIdx.y * n + q) * 2 + 1] = sm[t];
        }
    }
}

// one block: lse[q] = merge of the chunks; out[0] = mean over valid rows of lse - s_t (NaN if none), out[1] = count
__global__ __launch_bounds__(1024) void lce_finish_kernel(const float* __restrict__ part, int64_t n, int nchunks,
                                                          const int64_t* __restrict__ targets, int64_t ignore,
                                                          int64_t V, const float* __restrict__ tlogit,
                                                          float* __restrict__ lse, float* __restrict__ out) {
    __shared__ float sa[1024], sc[1024];
    float a = 0.f, c = 0.f;
    for (int64_t q = threadIdx.x; q < n; q += blockDim.x) {
        float m = -INFINITY, s = 0.f;
        for (int k = 0; k < nchunks; ++k) {
            const float m2 = part[((int64_t)k * n + q) * 2], s2 = part[((int64_t)k * n + q) * 2 + 1];
            const float nm = fmaxf(m, m2);
            if (nm == -INFINITY) continue;
            s = s * __expf(m - nm) + s2 * __expf(m2 - nm);
            m = nm;
        }
        const float l = m + logf(s);
        lse[q] = l;
        if (valid_target(targets[q], ignore, V)) {
            a += l - tlogit[q];
            c += 1.f;
        }
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

// ------------------------------------------------------------------------------------------------- dH
// grid (query blocks, item chunks).  dh_part[chunk] (n x D) = sum over the chunk's items of P W.
template <int D, int kNQT>
__global__ __launch_bounds__(kThreads) void lce_dh_kernel(const float* __restrict__ H, int64_t ldh, int64_t n,
                                                          const float* __restrict__ W, int64_t ldw, int64_t V,
                                                          const float* __restrict__ bias,
                                                          const int64_t* __restrict__ targets, int64_t ignore,
                                                          const float* __restrict__ lse,
                                                          const float* __restrict__ dloss,
                                                          const float* __restrict__ stats, int64_t chunk,
                                                          float* __restrict__ dh_part) {
    constexpr int DQ = D / 4, S = D + 4, NF = D / 16;
    __shared__ __attribute__((aligned(16))) float Ws[kT * S];
    __shared__ float Bs[kT];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c16 = lane & 15;
    const int64_t qbase = (int64_t)blockIdx.x * (4 * kNQT * 16) + wave * kNQT * 16;
    const int64_t i_begin = (int64_t)blockIdx.y * chunk, i_end = min(V, i_begin + chunk);
    const float scale = dloss[0] / stats[1];
    float hq[kNQT][DQ];
    load_rows<D, kNQT>(H, ldh, qbase, n, g, c16, hq);
    int64_t tq[kNQT];
    float lq[kNQT], sq[kNQT];
#pragma unroll
    for (int t = 0; t < kNQT; ++t) {
        const int64_t q = qbase + t * 16 + c16;
        tq[t] = q < n ? targets[q] : -1;
        const bool ok = q < n && valid_target(tq[t], ignore, V);
        lq[t] = ok ? lse[q] : 0.f;
        sq[t] = ok ? scale : 0.f;  // ignored / padding rows contribute nothing
    }
    floatx4 dh[kNQT][NF];
#pragma unroll
    for (int t = 0; t < kNQT; ++t)
#pragma unroll
        for (int f = 0; f < NF; ++f) dh[t][f] = floatx4{0.f, 0.f, 0.f, 0.f};
    Stage<D> st;
    st.load(W, ldw, i_begin, i_end);
    float bnext = (threadIdx.x < kT && i_begin + threadIdx.x < i_end && bias) ? bias[i_begin + threadIdx.x] : 0.f;
    for (int64_t i0 = i_begin; i0 < i_end; i0 += kT) {
        __syncthreads();
        st.store(Ws);
        if (threadIdx.x < kT) Bs[threadIdx.x] = bnext;
        __syncthreads();
        if (i0 + kT < i_end) {
            st.load(W, ldw, i0 + kT, i_end);
            bnext = (threadIdx.x < kT && i0 + kT + threadIdx.x < i_end && bias) ? bias[i0 + kT + threadIdx.x] : 0.f;
        }
        floatx4 acc[kNQT][kNS];
        tile_times_rows<D, kNQT>(Ws, g, c16, hq, acc);
        // P in place: lane (g, c16) = query c16 x items sub*16 + 4g + r
#pragma unroll
        for (int t = 0; t < kNQT; ++t)
#pragma unroll
            for (int sub = 0; sub < kNS; ++sub)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int j = sub * 16 + 4 * g + r;
                    const int64_t item = i0 + j;
                    const float p = __expf(acc[t][sub][r] + Bs[j] - lq[t]) - (item == tq[t] ? 1.f : 0.f);
                    acc[t][sub][r] = item < i_end ? p * sq[t] : 0.f;
                }
        // dH[q][f] += sum_items P[q][item] W[item][f]: A = P (row c16 = query, k = g), B = W tile rows
#pragma unroll
        for (int sub = 0; sub < kNS; ++sub)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float* wrow = Ws + (sub * 16 + 4 * g + r) * S + c16;
#pragma unroll
                for (int f = 0; f < NF; ++f) {
                    const float b = wrow[f * 16];
#pragma unroll
                    for (int t = 0; t < kNQT; ++t) dh[t][f] = mfma16(acc[t][sub][r], b, dh[t][f]);
                }
            }
    }
    // lane (g, c16) holds dH[query qbase + t*16 + 4g + r][feature f*16 + c16]
    float* out = dh_part + (int64_t)blockIdx.y * n * D;
#pragma unroll
    for (int t = 0; t < kNQT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int64_t q = qbase + t * 16 + 4 * g + r;
            if (q < n)
#pragma unroll
                for (int f = 0; f < NF; ++f) out[q * D + f * 16 + c16] = dh[t][f][r];
        }
}

// ------------------------------------------------------------------------------------------- dW, db
// grid (item blocks of 4*kNIT*16, query chunks).  dw_part[chunk] (V x D), db_part[chunk] (V).
template <int D, int kNIT>
__global__ __launch_bounds__(kThreads) void lce_dw_kernel(const float* __restrict__ H, int64_t ldh, int64_t n,
                                                          const float* __restrict__ W, int64_t ldw, int64_t V,
                                                          const float* __restrict__ bias,
                                                          const int64_t* __restrict__ targets, int64_t ignore,
                                                          const float* __restrict__ lse,
                                                          const float* __restrict__ dloss,
                                                          const float* __restrict__ stats, int64_t qchunk,
                                                          float* __restrict__ dw_part, float* __restrict__ db_part) {
    constexpr int DQ = D / 4, S = D + 4, NF = D / 16;
    __shared__ __attribute__((aligned(16))) float Hs[kT * S];
    __shared__ float Ls[kT];
    __shared__ int64_t Ts[kT];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c16 = lane & 15;
    const int64_t ibase = (int64_t)blockIdx.x * (4 * kNIT * 16) + wave * kNIT * 16;
    const int64_t q_begin = (int64_t)blockIdx.y * qchunk, q_end = min(n, q_begin + qchunk);
    const float scale = dloss[0] / stats[1];
    float wi[kNIT][DQ];
    load_rows<D, kNIT>(W, ldw, ibase, V, g, c16, wi);
    float bi[kNIT];
    int64_t item[kNIT];
#pragma unroll
    for (int t = 0; t < kNIT; ++t) {
        item[t] = ibase + t * 16 + c16;
        bi[t] = (bias && item[t] < V) ? bias[item[t]] : 0.f;
    }
    floatx4 dw[kNIT][NF];
    float db[kNIT];
#pragma unroll
    for (int t = 0; t < kNIT; ++t) {
        db[t] = 0.f;
#pragma unroll
        for (int f = 0; f < NF; ++f) dw[t][f] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
    Stage<D> st;
    st.load(H, ldh, q_begin, q_end);
    auto row_meta = [&](int64_t q0, float& l, int64_t& tg) {
        const int64_t q = q0 + threadIdx.x;
        const bool ok = q < q_end && valid_target(targets[q < q_end ? q : 0], ignore, V);
        l = ok ? lse[q] : INFINITY;  // exp(s - inf) = 0: padding / ignored queries add nothing
        tg = ok ? targets[q] : -1;
    };
    float lnext = INFINITY;
    int64_t tnext = -1;
    if (threadIdx.x < kT) row_meta(q_begin, lnext, tnext);
    for (int64_t q0 = q_begin; q0 < q_end; q0 += kT) {
        __syncthreads();
        st.store(Hs);
        if (threadIdx.x < kT) {
            Ls[threadIdx.x] = lnext;
            Ts[threadIdx.x] = tnext;
        }
        __syncthreads();
        if (q0 + kT < q_end) {
            st.load(H, ldh, q0 + kT, q_end);
            if (threadIdx.x < kT) row_meta(q0 + kT, lnext, tnext);
        }
        // S[query sub*16 + 4g + r][item t*16 + c16]
        floatx4 acc[kNIT][kNS];
        tile_times_rows<D, kNIT>(Hs, g, c16, wi, acc);
#pragma unroll
        for (int t = 0; t < kNIT; ++t)
#pragma unroll
            for (int sub = 0; sub < kNS; ++sub)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int j = sub * 16 + 4 * g + r;
                    const float p = __expf(acc[t][sub][r] + bi[t] - Ls[j]) - (Ts[j] == item[t] ? 1.f : 0.f);
                    acc[t][sub][r] = p * scale;
                    db[t] += acc[t][sub][r];
                }
        // dW[item][f] += sum_q P[q][item] H[q][f]: A = P (row c16 = item, k = g), B = H tile rows
#pragma unroll
        for (int sub = 0; sub < kNS; ++sub)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float* hrow = Hs + (sub * 16 + 4 * g + r) * S + c16;
#pragma unroll
                for (int f = 0; f < NF; ++f) {
                    const float b = hrow[f * 16];
#pragma unroll
                    for (int t = 0; t < kNIT; ++t) dw[t][f] = mfma16(acc[t][sub][r], b, dw[t][f]);
                }
            }
    }
    float* out = dw_part + (int64_t)blockIdx.y * V * D;
#pragma unroll
    for (int t = 0; t < kNIT; ++t) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int64_t it = ibase + t * 16 + 4 * g + r;
            if (it < V)
#pragma unroll
                for (int f = 0; f < NF; ++f) out[it * D + f * 16 + c16] = dw[t][f][r];
        }
        float b = db[t];
        b += __shfl_xor(b, 16, 64);
        b += __shfl_xor(b, 32, 64);
        if (g == 0 && db_part && item[t] < V) db_part[(int64_t)blockIdx.y * V + item[t]] = b;
    }
}

// out[i] = sum_{c < nparts} part[c * stride + i] (fixed order), float4 lanes
__global__ __launch_bounds__(256) void lce_sum_parts_kernel(const float* __restrict__ part, int64_t stride,
                                                            int nparts, int64_t count, float* __restrict__ out) {
    const int64_t i4 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
    if (i4 >= count) return;
    if (i4 + 4 <= count) {
        float4 s = *reinterpret_cast<const float4*>(part + i4);
        for (int c = 1; c < nparts; ++c) {
            const float4 v = *reinterpret_cast<const float4*>(part + c * stride + i4);
            s.x += v.x;
            s.y += v.y;
            s.z += v.z;
            s.w += v.w;
        }
        *reinterpret_cast<float4*>(out + i4) = s;
    } else {
        for (int64_t i = i4; i < count; ++i) {
            float s = part[i];
            for (int c = 1; c < nparts; ++c) s += part[c * stride + i];
            out[i] = s;
        }
    }
}

struct XPlan {
    int64_t qblocks, ichunks, ichunk;  // stats / dH
    int64_t iblocks, qchunks, qchunk;  // dW
    int nqt, nit;
};
XPlan make_xplan(int64_t n, int64_t V) {
    XPlan p;
    constexpr int kNQT = kNQTsel, kNIT = kNITsel;
    p.nqt = kNQT;
    p.nit = kNIT;
    constexpr int64_t kWant = 1024;  // ~4 workgroups per CU
    p.qblocks = (n + 4 * kNQT * 16 - 1) / (4 * kNQT * 16);
    const int64_t wi = std::max<int64_t>(1, kWant / std::max<int64_t>(1, p.qblocks));
    p.ichunk = std::max<int64_t>(kT, ((V + wi - 1) / wi + kT - 1) / kT * kT);
    p.ichunks = (V + p.ichunk - 1) / p.ichunk;
    p.iblocks = (V + 4 * kNIT * 16 - 1) / (4 * kNIT * 16);
    const int64_t wq = std::max<int64_t>(1, kWant / std::max<int64_t>(1, p.iblocks));
    p.qchunk = std::max<int64_t>(kT, ((n + wq - 1) / wq + kT - 1) / kT * kT);
    p.qchunks = (n + p.qchunk - 1) / p.qchunk;
    return p;
}

#define ASME_XENT_DIM(DV, ...)                                   \
    switch (DV) {                                                \
        case 32: { constexpr int D = 32; __VA_ARGS__; } break;   \
        case 64: { constexpr int D = 64; __VA_ARGS__; } break;   \
        case 128: { constexpr int D = 128; __VA_ARGS__; } break; \
        default: set_error("linear_xent: dim must be 32, 64 or 128"); return -1; \
    }

bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace

ASME_API int64_t asme_linear_xent_fwd_workspace(int64_t n, int64_t V, int64_t dim) {
    (void)dim;
    const XPlan p = make_xplan(n, V);
    return p.ichunks * n * 2 * (int64_t)sizeof(float) + n * (int64_t)sizeof(float);
}

ASME_API int asme_linear_xent_fwd(const float* H, int64_t ld_h, int64_t n, int64_t dim, const float* W, int64_t ld_w,
                                  int64_t V, const float* bias, const int64_t* targets, int64_t ignore_index,
                                  float* lse, float* workspace, int64_t ws_bytes, float* out, void* stream) {
    ASME_CHECK_ARG(H && W && targets && lse && workspace && out, "asme_linear_xent_fwd: null pointer");
    ASME_CHECK_ARG(ld_h % 4 == 0 && ld_w % 4 == 0 && aligned16(H) && aligned16(W),
                   "asme_linear_xent_fwd: rows must be 16-B aligned");
    ASME_CHECK_ARG(n >= 0 && V >= 1, "asme_linear_xent_fwd: bad shape");
    ASME_CHECK_ARG(ws_bytes >= asme_linear_xent_fwd_workspace(n, V, dim), "asme_linear_xent_fwd: workspace too small");
    hipStream_t s = (hipStream_t)stream;
    const XPlan p = make_xplan(n, V);
    float* part = workspace;
    float* tlogit = workspace + p.ichunks * n * 2;
    if (n > 0) {
        ASME_XENT_DIM(dim, {
            if (p.nqt == 1)
                hipLaunchKernelGGL(HIP_KERNEL_NAME(lce_stats_kernel<D, 1>), dim3((unsigned)p.qblocks, (unsigned)p.ichunks),
                                   dim3(kThreads), 0, s, H, ld_h, n, W, ld_w, V, bias, targets, p.ichunk, part, tlogit);
            else
                hipLaunchKernelGGL(HIP_KERNEL_NAME(lce_stats_kernel<D, 2>), dim3((unsigned)p.qblocks, (unsigned)p.ichunks),
                                   dim3(kThreads), 0, s, H, ld_h, n, W, ld_w, V, bias, targets, p.ichunk, part, tlogit);
        });
    }
    hipLaunchKernelGGL(lce_finish_kernel, dim3(1), dim3(1024), 0, s, part, n, (int)p.ichunks, targets, ignore_index,
                       V, tlogit, lse, out);
    ASME_LAUNCH_CHECK("asme_linear_xent_fwd");
}

ASME_API int64_t asme_linear_xent_bwd_workspace(int64_t n, int64_t V, int64_t dim) {
    const XPlan p = make_xplan(n, V);
    const int64_t dh = p.ichunks > 1 ? p.ichunks * n * dim : 0;
    const int64_t dw = p.qchunks > 1 ? p.qchunks * V * (dim + 1) : 0;
    return (dh + dw) * (int64_t)sizeof(float) + 16;
}

// dH (n x dim), dW (V x dim), db (V, nullable) are overwritten (not accumulated).
ASME_API int asme_linear_xent_bwd(const float* H, int64_t ld_h, int64_t n, int64_t dim, const float* W, int64_t ld_w,
                                  int64_t V, const float* bias, const int64_t* targets, int64_t ignore_index,
                                  const float* lse, const float* stats, const float* dloss, float* dH, float* dW,
                                  float* db, float* workspace, int64_t ws_bytes, void* stream) {
    ASME_CHECK_ARG(H && W && targets && lse && stats && dloss && dH && dW, "asme_linear_xent_bwd: null pointer");
    ASME_CHECK_ARG(ld_h % 4 == 0 && ld_w % 4 == 0 && aligned16(H) && aligned16(W) && aligned16(dH) && aligned16(dW),
                   "asme_linear_xent_bwd: rows must be 16-B aligned");
    ASME_CHECK_ARG(ws_bytes >= asme_linear_xent_bwd_workspace(n, V, dim), "asme_linear_xent_bwd: workspace too small");
    hipStream_t s = (hipStream_t)stream;
    const XPlan p = make_xplan(n, V);
    if (n == 0) {
        if (hipMemsetAsync(dW, 0, V * dim * sizeof(float), s) != hipSuccess ||
            (db && hipMemsetAsync(db, 0, V * sizeof(float), s) != hipSuccess))
            return hip_status(hipGetLastError(), "asme_linear_xent_bwd");
        return 0;
    }
    float* dh_part = p.ichunks > 1 ? workspace : dH;
    float* dw_part = p.qchunks > 1 ? workspace + (p.ichunks > 1 ? p.ichunks * n * dim : 0) : dW;
    float* db_part = p.qchunks > 1 ? dw_part + p.qchunks * V * dim : db;
    ASME_XENT_DIM(dim, {
        if (p.nqt == 1)
            hipLaunchKernelGGL(HIP_KERNEL_NAME(lce_dh_kernel<D, 1>), dim3((unsigned)p.qblocks, (unsigned)p.ichunks), dim3(kThreads), 0, s, H,
                               ld_h, n, W, ld_w, V, bias, targets, ignore_index, lse, dloss, stats, p.ichunk, dh_part);
        else
            hipLaunchKernelGGL(HIP_KERNEL_NAME(lce_dh_kernel<D, 2>), dim3((unsigned)p.qblocks, (unsigned)p.ichunks), dim3(kThreads), 0, s, H,
                               ld_h, n, W, ld_w, V, bias, targets, ignore_index, lse, dloss, stats, p.ichunk, dh_part);
        if (p.nit == 1)
            hipLaunchKernelGGL(HIP_KERNEL_NAME(lce_dw_kernel<D, 1>), dim3((unsigned)p.iblocks, (unsigned)p.qchunks), dim3(kThreads), 0, s, H,
                               ld_h, n, W, ld_w, V, bias, targets, ignore_index, lse, dloss, stats, p.qchunk, dw_part,
                               db_part);
        else
            hipLaunchKernelGGL(HIP_KERNEL_NAME(lce_dw_kernel<D, 2>), dim3((unsigned)p.iblocks, (unsigned)p.qchunks), dim3(kThreads), 0, s, H,
                               ld_h, n, W, ld_w, V, bias, targets, ignore_index, lse, dloss, stats, p.qchunk, dw_part,
                               db_part);
    });
    auto sum = [&](const float* part, int64_t stride, int64_t nparts, int64_t count, float* out) {
        const int64_t thr = (count + 3) / 4;
        hipLaunchKernelGGL(lce_sum_parts_kernel, dim3((unsigned)((thr + 255) / 256)), dim3(256), 0, s, part, stride,
                           (int)nparts, count, out);
    };
    if (p.ichunks > 1) sum(dh_part, n * dim, p.ichunks, n * dim, dH);
    if (p.qchunks > 1) {
        sum(dw_part, V * dim, p.qchunks, V * dim, dW);
        if (db) sum(db_part, V, p.qchunks, V, db);
    }
    ASME_LAUNCH_CHECK("asme_linear_xent_bwd");
}
