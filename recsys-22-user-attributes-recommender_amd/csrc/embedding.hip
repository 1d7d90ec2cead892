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
#include <type_traits>
#include <algorithm>

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

// ---------------------------------------------------------------------------------------------
// D % 4 == 0 (every transformer width): K tokens per LPR-lane group, so each wave has 2*K independent
// 512-B row gathers (+ position rows) in flight before the first use -- the random item-row gather is
// latency-bound, not bandwidth-bound, at one row per group.  Both dropouts of a 4-element chunk come
// from ONE Philox4x32-10 block (8 16-bit uniforms: x,y -> drop1, z,w -> drop2; keep iff u16 >=
// round(p * 65536)), and the forward stores the 8 decisions as one keep byte per chunk (bit i: drop1
// of element i, bit 4+i: drop2), (T, D/4) bytes, so the backward never regenerates them.
__device__ __forceinline__ uint32_t emb_thresh(float p) { return (uint32_t)(p * 65536.f + 0.5f); }

__device__ __forceinline__ uint32_t emb_keep_bits(uint64_t seed, uint64_t chunk, uint32_t th1, uint32_t th2) {
    u32x4 c{(uint32_t)chunk, (uint32_t)(chunk >> 32), 0xE3B0C442u, 0x5851F42Du};
    const u32x4 r = philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    uint32_t m = 0;
    m |= ((r.x & 0xFFFFu) >= th1 ? 1u : 0u) | ((r.x >> 16) >= th1 ? 2u : 0u);
    m |= ((r.y & 0xFFFFu) >= th1 ? 4u : 0u) | ((r.y >> 16) >= th1 ? 8u : 0u);
    m |= ((r.z & 0xFFFFu) >= th2 ? 16u : 0u) | ((r.z >> 16) >= th2 ? 32u : 0u);
    m |= ((r.w & 0xFFFFu) >= th2 ? 64u : 0u) | ((r.w >> 16) >= th2 ? 128u : 0u);
    return m;
}

__host__ __device__ inline uint64_t emb_seed(uint64_t s1, uint64_t s2) { return s1 ^ (s2 * 0x9E3779B97F4A7C15ull); }


// Keep bytes of token t: (T, D/4) bytes.  When the row layout covers the row exactly (LPR * NV * 4 == D: D = 128 on
// 16 lanes x 2 chunks, D = 512 on 64 x 2, and every one-chunk layout) a lane's NV bytes are adjacent -- byte
// sub * NV + j holds chunk sub + LPR * j -- so each lane stores / loads them as ONE 8- or 16-bit access per token
// (16-lane groups move 32 contiguous bytes) instead of NV byte accesses; other layouts keep chunk order (byte = chunk).
// ops.embedding_keep_chunks() converts to chunk order.
template <class R>
__device__ __forceinline__ bool emb_keep_packed(int D) { return R::LPR * R::NV * 4 == D; }
// the 16-lane, two-chunk layout is taken for D = 128 only (with_emb_layout): there the width is a compile-time
// constant, so the column bounds checks and the 1 / D of the statistics fold away
template <class R>
__device__ __forceinline__ int emb_width(int D) {
    return ((R::LPR == 16 && R::NV == 2) || (R::LPR == 8 && R::NV == 4)) ? 128 : D;
}
template <class R>
__device__ __forceinline__ void emb_keep_store(uint8_t* __restrict__ keep, int64_t t, int sub, int D,
                                               const uint32_t (&bits)[R::NV]) {
    uint8_t* row = keep + (uint64_t)t * (D >> 2);
    if constexpr (R::LPR == 8 && R::NV == 4) {
        // D = 128 on 8 lanes x 4 chunks (chunks sub + 8j): the bytes of the 16-lane layout -- 16-bit word w holds
        // chunks w and w + 16 -- so the backward (16 lanes) reads them as it always does
        *reinterpret_cast<uint16_t*>(row + sub * 2) = (uint16_t)(bits[0] | (bits[2] << 8));
        *reinterpret_cast<uint16_t*>(row + (sub + 8) * 2) = (uint16_t)(bits[1] | (bits[3] << 8));
        return;
    }
    if (emb_keep_packed<R>(D)) {
        if constexpr (R::NV == 2) {
            *reinterpret_cast<uint16_t*>(row + sub * 2) = (uint16_t)(bits[0] | (bits[1] << 8));
        } else {
#pragma unroll
            for (int j = 0; j < R::NV; ++j) row[sub * R::NV + j] = (uint8_t)bits[j];
        }
        return;
    }
#pragma unroll
    for (int j = 0; j < R::NV; ++j) {
        const int c = R::col(sub, j);
        if (c < D) row[c >> 2] = (uint8_t)bits[j];
    }
}
template <class R>
__device__ __forceinline__ void emb_keep_load(const uint8_t* __restrict__ keep, int64_t t, int sub, int D,
                                              uint32_t (&bits)[R::NV]) {
    const uint8_t* row = keep + (uint64_t)t * (D >> 2);
    if (emb_keep_packed<R>(D)) {
        if constexpr (R::NV == 2) {
            const uint32_t v = *reinterpret_cast<const uint16_t*>(row + sub * 2);
            bits[0] = v & 0xFFu;
            bits[1] = v >> 8;
        } else {
#pragma unroll
            for (int j = 0; j < R::NV; ++j) bits[j] = row[sub * R::NV + j];
        }
        return;
    }
#pragma unroll
    for (int j = 0; j < R::NV; ++j) {
        const int c = R::col(sub, j);
        bits[j] = row[(c < D ? c : 0) >> 2];
    }
}

// LN3 (the fused next LayerNorm): the first transformer block's input norm applied to the embedding output in the
// same pass (transformer_layers.py:251-258 SublayerConnection: x + dropout(sublayer(norm(x))) of block 0), so the
// block reads `out3` and keeps `out` as its residual stream: no separate LayerNorm launch re-reading the rows.
struct EmbLn3 {
    const float* w;
    const float* b;
    float eps;
    float* out;    // forward: the normalised rows (T, D)
    float* stats;  // (T, 2): mean, rstd
    const float* dln;  // backward: gradient of `out` (the gradient of the embedding output itself is `dout`)
    const float* b2;   // backward: LN2's bias (the embedding output is recomputed through LN2's affine)
};

#ifndef ASME_EMB_FWD_HOIST
#define ASME_EMB_FWD_HOIST 1
#endif
// diagnostic builds only (tools/build_variant.sh): 1 = the forward's LayerNorm statistics skipped (mean 0, rstd 1),
// 2 = its dropout decisions not drawn (every element kept, keep bytes still stored)
#ifndef ASME_EMB_DIAG
#define ASME_EMB_DIAG 0
#endif
#ifndef ASME_EMB_NT
#define ASME_EMB_NT 1
#endif
template <class R, int kEmbK, bool LN3, bool LN2 = true>  // kEmbK: tokens per lane group; LN2: as the backward's
__global__ __launch_bounds__(256) void emb_fwd4_kernel(
    const int64_t* __restrict__ ids, int64_t T, int64_t L, const float* __restrict__ table, int64_t V, int D_,
    const float* __restrict__ pos, const float* __restrict__ w1, const float* __restrict__ b1, float eps1, float p1,
    const float* __restrict__ extra, const float* __restrict__ w2, const float* __restrict__ b2, float eps2,
    float p2, uint64_t seed, float* __restrict__ out, float* __restrict__ stats, uint8_t* __restrict__ keep,
    int* __restrict__ err, EmbLn3 l3) {
    static_assert(R::W == 4, "4-wide layout only");
    const int D = emb_width<R>(D_);
    const int lane = threadIdx.x & 63, sub = lane % R::LPR;
    const int64_t t0 = ((int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)) * R::RPW * kEmbK + lane / R::LPR;
    int64_t id[kEmbK];
#pragma unroll
    for (int k = 0; k < kEmbK; ++k) {  // every id requested before the first is checked (one wait, not kEmbK)
        const int64_t t = t0 + (int64_t)k * R::RPW;
        id[k] = t < T ? ids[t] : 0;
    }
#if ASME_EMB_FWD_HOIST
    // LN3's w / b staged in LDS with the id loads in flight, instead of a global round trip (which also waits for the
    // output row stores: vmcnt counts stores) between the first token's stores and its LN3 affine
    // (the 8-lane layout keeps LN1 / LN2's w / b here too: rows 2-5)
    __shared__ __attribute__((aligned(16))) float prm3[R::NV >= 4 ? 6 : 2][512];
    if constexpr (LN3 || R::NV >= 4) {
        for (int e = threadIdx.x; e < D; e += blockDim.x) {
            if (LN3) {
                prm3[0][e] = l3.w[e];
                prm3[1][e] = l3.b[e];
            }
            if constexpr (R::NV >= 4) {
                prm3[2][e] = w1 ? w1[e] : 0.f;
                prm3[3][e] = w1 ? b1[e] : 0.f;
                prm3[4][e] = (LN2 && w2) ? w2[e] : 0.f;
                prm3[5][e] = (LN2 && w2) ? b2[e] : 0.f;
            }
        }
        __syncthreads();
    }
    const float* w3p = prm3[0];
    const float* b3p = prm3[1];
#else
    const float* w3p = l3.w;
    const float* b3p = l3.b;
#endif
#pragma unroll
    for (int k = 0; k < kEmbK; ++k) {
        const int64_t t = t0 + (int64_t)k * R::RPW;
        if (id[k] < 0 || id[k] >= V) {
            if (sub == 0 && t < T && err) atomicOr(err, 1);
            id[k] = 0;
        }
    }
    RowVals<R> x[kEmbK], q[kEmbK];
#pragma unroll
    for (int k = 0; k < kEmbK; ++k) row_load<R>(table + id[k] * D, sub, D, x[k]);
    if (pos) {
#pragma unroll
        for (int k = 0; k < kEmbK; ++k) {
            const int64_t t = t0 + (int64_t)k * R::RPW;
            row_load<R>(pos + ((t < T ? t : 0) % L) * D, sub, D, q[k]);
        }
#pragma unroll
        for (int k = 0; k < kEmbK; ++k)
#pragma unroll
            for (int j = 0; j < R::NV; ++j)
#pragma unroll
                for (int i = 0; i < 4; ++i) x[k][j][i] += q[k][j][i];
    }
    RowVals<R> w1v, b1v, w2v, b2v;
    constexpr bool kPrmLds = R::NV >= 4;  // 16 values per lane: LN1 / LN2 read from LDS where they are used
    if (!kPrmLds) {
        if (w1) {
            row_load<R>(w1, sub, D, w1v);
            row_load<R>(b1, sub, D, b1v);
        }
        if (LN2 && w2) {
            row_load<R>(w2, sub, D, w2v);
            row_load<R>(b2, sub, D, b2v);
        }
    }
    const bool drop = p1 > 0.f || p2 > 0.f;
    const uint32_t th1 = emb_thresh(p1), th2 = emb_thresh(p2);
    const float k1 = 1.f / (1.f - p1), k2 = 1.f / (1.f - p2);
#pragma unroll
    for (int k = 0; k < kEmbK; ++k) {
        const int64_t t = t0 + (int64_t)k * R::RPW;
        if (t >= T) break;
        if (extra) row_load<R>(extra + t * D, sub, D, q[k]);
        float m1 = 0.f, r1 = 1.f, m2 = 0.f, r2 = 1.f;
        RowVals<R> tmp;
        if (w1) {
            if (ASME_EMB_DIAG != 1) row_ln_stats<R>(x[k], sub, D, eps1, m1, r1);
            row_normalise<R>(x[k], sub, D, m1, r1, tmp);
            if constexpr (kPrmLds) {
                row_affine<R>(tmp, sub, D, prm3[2], prm3[3], x[k]);
            } else {
#pragma unroll
                for (int j = 0; j < R::NV; ++j)
#pragma unroll
                    for (int i = 0; i < 4; ++i) x[k][j][i] = tmp[j][i] * w1v[j][i] + b1v[j][i];
            }
        }
        uint32_t bits[R::NV];
        if (drop) {
#pragma unroll
            for (int j = 0; j < R::NV; ++j) {
                const int c = R::col(sub, j);
                bits[j] = c < D ? (ASME_EMB_DIAG == 2 ? 0xFFu : emb_keep_bits(seed, ((uint64_t)t * D + c) >> 2, th1, th2))
                                : 0u;
                if (p1 > 0.f)
#pragma unroll
                    for (int i = 0; i < 4; ++i) x[k][j][i] *= keep_factor_bit(bits[j], i, k1);
            }
        }
        if (extra)
#pragma unroll
            for (int j = 0; j < R::NV; ++j)
#pragma unroll
                for (int i = 0; i < 4; ++i) x[k][j][i] += q[k][j][i];
        if (LN2 && w2) {
            if (ASME_EMB_DIAG != 1) row_ln_stats<R>(x[k], sub, D, eps2, m2, r2);
            row_normalise<R>(x[k], sub, D, m2, r2, tmp);
            if constexpr (kPrmLds) {
                row_affine<R>(tmp, sub, D, prm3[4], prm3[5], x[k]);
            } else {
#pragma unroll
                for (int j = 0; j < R::NV; ++j)
#pragma unroll
                    for (int i = 0; i < 4; ++i) x[k][j][i] = tmp[j][i] * w2v[j][i] + b2v[j][i];
            }
        }
        if (drop) {
            if (p2 > 0.f)
#pragma unroll
                for (int j = 0; j < R::NV; ++j)
#pragma unroll
                    for (int i = 0; i < 4; ++i) x[k][j][i] *= keep_factor_bit(bits[j], 4 + i, k2);
            if (keep) emb_keep_store<R>(keep, t, sub, D, bits);
        }
        row_store<R, ASME_EMB_NT>(out + t * D, sub, D, x[k]);
        if (sub == 0 && stats) *reinterpret_cast<float4*>(stats + t * 4) = make_float4(m1, r1, m2, r2);
        if constexpr (LN3) {
            float m3 = 0.f, r3 = 1.f;
            if (ASME_EMB_DIAG != 1) row_ln_stats<R>(x[k], sub, D, l3.eps, m3, r3);
            row_normalise<R>(x[k], sub, D, m3, r3, tmp);
            row_affine<R>(tmp, sub, D, w3p, b3p, x[k]);
            row_store<R, ASME_EMB_NT>(l3.out + t * D, sub, D, x[k]);
            if (sub == 0) *reinterpret_cast<float2*>(l3.stats + t * 2) = make_float2(m3, r3);
        }
    }
}

// three waves per SIMD: SASRec's variant (LN2 + LN3) needs 170 VGPRs with its LN parameters in LDS; held to 168 it
// spills one 8-byte loop-invariant (12 B of scratch, one reload per pass) and runs 0.103-0.109 vs 0.110-0.118 ms
#ifndef ASME_EMB_BWD_WPE
#define ASME_EMB_BWD_WPE 3
#endif
#ifndef ASME_EMB_BWD_HOIST
#define ASME_EMB_BWD_HOIST 1
#endif
#if ASME_EMB_BWD_WPE
#define ASME_EMB_BWD_ATTR __attribute__((amdgpu_waves_per_eu(ASME_EMB_BWD_WPE, 8)))
#else
#define ASME_EMB_BWD_ATTR
#endif
// LN3: `dout` is the gradient of the embedding output through the residual stream, l3.dln that of the fused
// LayerNorm's output; the output row is recomputed (LN1 / dropout / LN2 affine / dropout, from the stored statistics
// and keep bits) for the LN3 backward, whose parameter gradients are accumulators 4 and 5 of the partials.
// LN2: the second LayerNorm (pre-fusion attributes) is present -- a template flag, so without it (SASRec, BERT4Rec)
// its accumulators and normalised row cost no registers: 200 -> 155 VGPRs at D = 128 with LN3, a third wave per SIMD
// (in-step 0.150-0.154 -> 0.139-0.140 ms per call, same box; forcing a fourth wave spills: 0.315 ms)
template <class R, int kPass, bool LN3, bool LN2>  // kPass: tokens per lane group per grid-stride pass
__global__ __launch_bounds__(256) ASME_EMB_BWD_ATTR void emb_bwd4_kernel(
    const int64_t* __restrict__ ids, int64_t T, int64_t L, const float* __restrict__ table, int64_t V, int D_,
    const float* __restrict__ pos, const float* __restrict__ w1, const float* __restrict__ b1, float p1,
    const float* __restrict__ extra, const float* __restrict__ w2, float p2, uint64_t seed,
    const uint8_t* __restrict__ keep, const float* __restrict__ dout, const float* __restrict__ stats,
    float* __restrict__ d_rows, float* __restrict__ d_extra, float* __restrict__ partials, EmbLn3 l3) {
    static_assert(R::W == 4, "4-wide layout only");
    const int D = D_;  // (a compile-time width here costs 20 spilled VGPRs at the 168-VGPR cap)
    constexpr int NACC = LN3 ? 6 : 4;
    const int lane = threadIdx.x & 63, sub = lane % R::LPR, wave = threadIdx.x >> 6;
    float acc[NACC][R::NV][R::W];
#pragma unroll
    for (int k = 0; k < NACC; ++k) row_zero<R>(acc[k]);
    const bool drop = p1 > 0.f || p2 > 0.f;
    const uint32_t th1 = emb_thresh(p1), th2 = emb_thresh(p2);
    const float k1 = 1.f / (1.f - p1), k2 = 1.f / (1.f - p2);
#if ASME_EMB_BWD_HOIST
    // LN1's w / b and LN3's w staged once per workgroup: each pass reads them from LDS instead of three dependent
    // global (cache-hit) round trips after its row loads
    __shared__ __attribute__((aligned(16))) float prm[5][512];
    for (int e = threadIdx.x; e < D; e += blockDim.x) {
        if (w1) {
            prm[0][e] = w1[e];
            prm[1][e] = b1[e];
        }
        if constexpr (LN3) prm[2][e] = l3.w[e];
        if constexpr (LN2) {
            prm[3][e] = w2[e];
            if constexpr (LN3) prm[4][e] = l3.b2[e];
        }
    }
    __syncthreads();
    const float* w1p = prm[0];
    const float* b1p = prm[1];
    const float* w3p = prm[2];
    const float* w2p = prm[3];
    const float* b2p = prm[4];
#else
    const float* w1p = w1;
    const float* b1p = b1;
    const float* w3p = l3.w;
    const float* w2p = w2;
    const float* b2p = l3.b2;
#endif
    const bool keep_in = keep && drop;
    for (int64_t tb = ((int64_t)blockIdx.x * kWavesPerBlock + wave) * R::RPW * kPass + lane / R::LPR;
         tb - lane / R::LPR < T; tb += (int64_t)gridDim.x * kWavesPerBlock * R::RPW * kPass) {
        int64_t id[kPass];
        float4 st[kPass];
        float2 st3[kPass];
        uint32_t kb[kPass][R::NV];
        RowVals<R> x[kPass], g[kPass], q[kPass], dl[kPass];
#pragma unroll
        for (int k = 0; k < kPass; ++k) {
            const int64_t t = tb + (int64_t)k * R::RPW;
            int64_t v = t < T ? ids[t] : 0;
            id[k] = (v < 0 || v >= V) ? 0 : v;
        }
#pragma unroll
        for (int k = 0; k < kPass; ++k) {
            const int64_t t = tb + (int64_t)k * R::RPW;
            const int64_t tt = t < T ? t : 0;
            row_load<R>(table + id[k] * D, sub, D, x[k]);
            if (pos) row_load<R>(pos + (tt % L) * D, sub, D, q[k]);
            row_load<R>(dout + tt * D, sub, D, g[k]);
            st[k] = *reinterpret_cast<const float4*>(stats + tt * 4);
            if constexpr (LN3) {
                row_load<R>(l3.dln + tt * D, sub, D, dl[k]);
                st3[k] = *reinterpret_cast<const float2*>(l3.stats + tt * 2);
            }
            // the stored keep bits ride with the row loads (one round trip per pass, one access per lane)
            if (keep_in) {
                emb_keep_load<R>(keep, tt, sub, D, kb[k]);
            } else {
#pragma unroll
                for (int j = 0; j < R::NV; ++j) kb[k][j] = 0xFFu;
            }
        }
#pragma unroll
        for (int k = 0; k < kPass; ++k) {
            const int64_t t = tb + (int64_t)k * R::RPW;
            const bool live = t < T;
            if (!live) {
                row_zero<R>(x[k]);
                row_zero<R>(g[k]);
                if constexpr (LN3) row_zero<R>(dl[k]);
            } else if (pos) {
#pragma unroll
                for (int j = 0; j < R::NV; ++j)
#pragma unroll
                    for (int i = 0; i < 4; ++i) x[k][j][i] += q[k][j][i];
            }
            uint32_t bits[R::NV];
#pragma unroll
            for (int j = 0; j < R::NV; ++j) {
                const int c = R::col(sub, j);
                bits[j] = 0xFFu;
                if (drop && live && c < D)
                    bits[j] = keep ? kb[k][j] : emb_keep_bits(seed, ((uint64_t)t * D + c) >> 2, th1, th2);
            }
            // recompute z = drop1(LN1(x)) + extra
            RowVals<R> xh1, xh2;
            if (w1) {
                row_normalise<R>(x[k], sub, D, st[k].x, st[k].y, xh1);
                row_affine<R>(xh1, sub, D, w1p, b1p, x[k]);
            }
            if (p1 > 0.f)
#pragma unroll
                for (int j = 0; j < R::NV; ++j)
#pragma unroll
                    for (int i = 0; i < 4; ++i) x[k][j][i] *= keep_factor_bit(bits[j], i, k1);
            if (LN2) {
                if (extra && live) {
                    row_load<R>(extra + t * D, sub, D, q[k]);
#pragma unroll
                    for (int j = 0; j < R::NV; ++j)
#pragma unroll
                        for (int i = 0; i < 4; ++i) x[k][j][i] += q[k][j][i];
                }
                row_normalise<R>(x[k], sub, D, st[k].z, st[k].w, xh2);
            }
            if constexpr (LN3) {
                // the embedding output drop2(LN2(z)) (or drop2(z) without LN2), then g += LN3 backward of dln
                RowVals<R> xo, xh3, gl;
                if (LN2) {
                    row_affine<R>(xh2, sub, D, w2p, b2p, xo);
                } else {
                    const bool ex = extra && live;
                    if (ex) row_load<R>(extra + t * D, sub, D, q[k]);
#pragma unroll
                    for (int j = 0; j < R::NV; ++j)
#pragma unroll
                        for (int i = 0; i < 4; ++i) xo[j][i] = x[k][j][i] + (ex ? q[k][j][i] : 0.f);
                }
                if (p2 > 0.f)
#pragma unroll
                    for (int j = 0; j < R::NV; ++j)
#pragma unroll
                        for (int i = 0; i < 4; ++i) xo[j][i] *= keep_factor_bit(bits[j], 4 + i, k2);
                row_normalise<R>(xo, sub, D, st3[k].x, st3[k].y, xh3);
#pragma unroll
                for (int j = 0; j < R::NV; ++j)
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        acc[4][j][i] += dl[k][j][i] * xh3[j][i];
                        acc[5][j][i] += dl[k][j][i];
                    }
                row_ln_bwd<R>(dl[k], xh3, w3p, st3[k].y, sub, D, gl);
#pragma unroll
                for (int j = 0; j < R::NV; ++j)
#pragma unroll
                    for (int i = 0; i < 4; ++i) g[k][j][i] += gl[j][i];
            }
            if (p2 > 0.f)
#pragma unroll
                for (int j = 0; j < R::NV; ++j)
#pragma unroll
                    for (int i = 0; i < 4; ++i) g[k][j][i] *= keep_factor_bit(bits[j], 4 + i, k2);
            RowVals<R> gz;
            if (LN2) {
#pragma unroll
                for (int j = 0; j < R::NV; ++j)
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        acc[2][j][i] += g[k][j][i] * xh2[j][i];
                        acc[3][j][i] += g[k][j][i];
                    }
                row_ln_bwd<R>(g[k], xh2, w2p, st[k].w, sub, D, gz);
            } else {
#pragma unroll
                for (int j = 0; j < R::NV; ++j)
#pragma unroll
                    for (int i = 0; i < 4; ++i) gz[j][i] = g[k][j][i];
            }
            if (d_extra && live) row_store<R>(d_extra + t * D, sub, D, gz);
            if (p1 > 0.f)
#pragma unroll
                for (int j = 0; j < R::NV; ++j)
#pragma unroll
                    for (int i = 0; i < 4; ++i) gz[j][i] *= keep_factor_bit(bits[j], i, k1);
            if (w1) {
#pragma unroll
                for (int j = 0; j < R::NV; ++j)
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        acc[0][j][i] += gz[j][i] * xh1[j][i];
                        acc[1][j][i] += gz[j][i];
                    }
                RowVals<R> gx;
                row_ln_bwd<R>(gz, xh1, w1p, st[k].y, sub, D, gx);
                if (live) row_store<R, ASME_EMB_NT>(d_rows + t * D, sub, D, gx);
            } else if (live) {
                row_store<R, ASME_EMB_NT>(d_rows + t * D, sub, D, gz);
            }
        }
    }
    if (partials) write_row_partials<R, NACC, kWavesPerBlock>(acc, lane, wave, D, partials);
}

// D = 128 on 16 lanes x two float4 with the keep bytes given (or no dropout): the operations of
// emb_bwd4_kernel<RowLayout<4, 16, 2>, 1, LN3, LN2> in the same order, as straight-line code -- the width a compile-time
// constant (no column checks), no Philox regeneration path, and no per-lane live branches: every lane loads a real row
// (the tail pass clamps its token to T - 1 and zeroes its gradient inputs), so each pass is one run of loads and one
// run of arithmetic.  (emb_bwd4_kernel's ISA: ~830 VALU per pass, 170 of them register moves around the live / keep
// branches, and one exec-masked branch per LayerNorm stage.)
#ifndef ASME_EMB_BWD128_WPE
#define ASME_EMB_BWD128_WPE 2  // (3: 168 VGPRs and 11 spilled, 116-120 vs 105-108 us at 2 waves per SIMD)
#endif
#ifndef ASME_EMB_BWD128_PF
#define ASME_EMB_BWD128_PF 1
#endif
#ifndef ASME_EMB_BWD128_NT
#define ASME_EMB_BWD128_NT 0  // (A/B) non-temporal loads: bit 0 the incoming gradients, bit 1 the gathered table rows
#endif
template <bool LN3, bool LN2, bool POS, bool DROP>  // POS: a position table; DROP: keep bytes given (some p > 0)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(ASME_EMB_BWD128_WPE, 8))) void emb_bwd128_kernel(
    const int64_t* __restrict__ ids, int64_t T, int64_t L, const float* __restrict__ table, int64_t V,
    const float* __restrict__ pos, const float* __restrict__ w1, const float* __restrict__ b1, float p1,
    const float* __restrict__ extra, const float* __restrict__ w2, float p2, const uint8_t* __restrict__ keep,
    const float* __restrict__ dout, const float* __restrict__ stats, float* __restrict__ d_rows,
    float* __restrict__ d_extra, float* __restrict__ partials, EmbLn3 l3) {
    using R = RowLayout<4, 16, 2>;
    constexpr int D = 128;
    constexpr int NACC = LN3 ? 6 : 4;
    const int lane = threadIdx.x & 63, sub = lane & 15, wave = threadIdx.x >> 6;
    float acc[NACC][R::NV][R::W];
#pragma unroll
    for (int k = 0; k < NACC; ++k) row_zero<R>(acc[k]);
    const bool small = T < ((int64_t)1 << 31) && L < ((int64_t)1 << 31);
    const float k1 = 1.f / (1.f - p1), k2 = 1.f / (1.f - p2);
    __shared__ __attribute__((aligned(16))) float prm[5][D];
    for (int e = threadIdx.x; e < D; e += blockDim.x) {
        prm[0][e] = w1 ? w1[e] : 0.f;
        prm[1][e] = w1 ? b1[e] : 0.f;
        if constexpr (LN3) prm[2][e] = l3.w[e];
        if constexpr (LN2) {
            prm[3][e] = w2[e];
            if constexpr (LN3) prm[4][e] = l3.b2[e];
        }
    }
    __syncthreads();
    const int64_t stride = (int64_t)gridDim.x * kWavesPerBlock * R::RPW;
    // software pipeline (ASME_EMB_BWD128_PF): the next pass's rows are requested before this pass's arithmetic, and the
    // ids two passes ahead -- a row load depends on its id, so ids run one pass ahead of the rows.  At one pass in
    // flight per wave the CU held ~32 KB of loads on average (8 waves, half of them computing), not enough to cover
    // HBM latency; with the next pass in flight every wave keeps its loads outstanding while it computes.
    struct PassIn {
        RowVals<R> x, q, g, dl;
        float4 st;
        float2 st3;
        uint32_t kv;
    };
    auto tok_of = [&](int64_t b) { const int64_t t = b + lane / R::LPR; return t < T ? t : T - 1; };
    // (raw ids: clamped where a row address is formed -- a clamp right after the load made the wave wait for it, and
    // with it for every load issued before, i.e. for the whole next pass, at the top of every pass)
    auto load_id = [&](int64_t b) -> int64_t { return ids[tok_of(b)]; };
    auto load_pass = [&](int64_t b, int64_t raw_id, PassIn& in) {
        const int64_t tt = tok_of(b);
        const int64_t id = (raw_id < 0 || raw_id >= V) ? 0 : raw_id;
        row_load_p<R, (ASME_EMB_BWD128_NT & 2) != 0>(table + id * D, sub, D, in.x);
        // (position t % L in 32-bit arithmetic where the token count allows: a 64-bit remainder is a ~40-instruction
        // sequence per pass)
        const int64_t pr = small ? (int64_t)((uint32_t)tt % (uint32_t)L) : tt % L;
        if constexpr (POS) row_load<R>(pos + pr * D, sub, D, in.q);
        row_load_p<R, (ASME_EMB_BWD128_NT & 1) != 0>(dout + tt * D, sub, D, in.g);
        in.st = *reinterpret_cast<const float4*>(stats + tt * 4);
        in.st3 = make_float2(0.f, 1.f);
        if constexpr (LN3) {
            row_load_p<R, (ASME_EMB_BWD128_NT & 1) != 0>(l3.dln + tt * D, sub, D, in.dl);
            in.st3 = *reinterpret_cast<const float2*>(l3.stats + tt * 2);
        }
        // (the lane's two keep bytes: one 16-bit load, as emb_keep_load; a p = 0 half is all 1s)
        in.kv = DROP ? (uint32_t)*reinterpret_cast<const uint16_t*>(keep + tt * (D >> 2) + sub * 2) : 0xFFFFu;
    };
    int64_t base = ((int64_t)blockIdx.x * kWavesPerBlock + wave) * R::RPW;
    PassIn nin;
    int64_t nid = 0;
    if (ASME_EMB_BWD128_PF && base < T) {
        load_pass(base, load_id(base), nin);
        if (base + stride < T) nid = load_id(base + stride);
    }
    for (; base < T; base += stride) {
        const int64_t t = base + lane / R::LPR;
        const int64_t tt = t < T ? t : T - 1;
        PassIn in;
        if (ASME_EMB_BWD128_PF) {
            in = nin;
            if (base + stride < T) {  // (wave-uniform) the next pass's rows, and the ids of the one after it
                load_pass(base + stride, nid, nin);
                if (base + 2 * stride < T) nid = load_id(base + 2 * stride);
            }
        } else {
            load_pass(base, load_id(base), in);
        }
        RowVals<R>& x = in.x;
        RowVals<R>& q = in.q;
        RowVals<R>& g = in.g;
        RowVals<R>& dl = in.dl;
        const float4 st = in.st;
        const float2 st3 = in.st3;
        uint32_t bits[R::NV] = {in.kv & 0xFFu, in.kv >> 8};
        if (base + R::RPW > T && t >= T) {  // (tail pass only) a token past T: no gradient flows from it
            row_zero<R>(g);
            if constexpr (LN3) row_zero<R>(dl);
        }
        if constexpr (POS)
#pragma unroll
            for (int j = 0; j < R::NV; ++j)
#pragma unroll
                for (int i = 0; i < 4; ++i) x[j][i] += q[j][i];
        // recompute z = drop1(LN1(x)) + extra
        RowVals<R> xh1, xh2;
        if (w1) {
            row_normalise<R>(x, sub, D, st.x, st.y, xh1);
            row_affine<R>(xh1, sub, D, prm[0], prm[1], x);
        } else {
            row_zero<R>(xh1);
        }
        if constexpr (DROP)
#pragma unroll
            for (int j = 0; j < R::NV; ++j)
#pragma unroll
                for (int i = 0; i < 4; ++i) x[j][i] *= keep_factor_bit(bits[j], i, k1);
        if constexpr (LN2) {
            if (extra) {
                row_load<R>(extra + tt * D, sub, D, q);
#pragma unroll
                for (int j = 0; j < R::NV; ++j)
#pragma unroll
                    for (int i = 0; i < 4; ++i) x[j][i] += q[j][i];
            }
            row_normalise<R>(x, sub, D, st.z, st.w, xh2);
        }
        if constexpr (LN3) {
            // the embedding output drop2(LN2(z)) (or drop2(z) without LN2), then g += LN3 backward of dln
            RowVals<R> xo, xh3, gl;
            if constexpr (LN2) {
                row_affine<R>(xh2, sub, D, prm[3], prm[4], xo);
            } else {
                if (extra) row_load<R>(extra + tt * D, sub, D, q);
#pragma unroll
                for (int j = 0; j < R::NV; ++j)
#pragma unroll
                    for (int i = 0; i < 4; ++i) xo[j][i] = x[j][i] + (extra ? q[j][i] : 0.f);
            }
            if constexpr (DROP)
#pragma unroll
                for (int j = 0; j < R::NV; ++j)
#pragma unroll
                    for (int i = 0; i < 4; ++i) xo[j][i] *= keep_factor_bit(bits[j], 4 + i, k2);
            row_normalise<R>(xo, sub, D, st3.x, st3.y, xh3);
#pragma unroll
            for (int j = 0; j < R::NV; ++j)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    acc[4][j][i] += dl[j][i] * xh3[j][i];
                    acc[5][j][i] += dl[j][i];
                }
            row_ln_bwd<R>(dl, xh3, prm[2], st3.y, sub, D, gl);
#pragma unroll
            for (int j = 0; j < R::NV; ++j)
#pragma unroll
                for (int i = 0; i < 4; ++i) g[j][i] += gl[j][i];
        }
        if constexpr (DROP)
#pragma unroll
            for (int j = 0; j < R::NV; ++j)
#pragma unroll
                for (int i = 0; i < 4; ++i) g[j][i] *= keep_factor_bit(bits[j], 4 + i, k2);
        RowVals<R> gz;
        if constexpr (LN2) {
#pragma unroll
            for (int j = 0; j < R::NV; ++j)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    acc[2][j][i] += g[j][i] * xh2[j][i];
                    acc[3][j][i] += g[j][i];
                }
            row_ln_bwd<R>(g, xh2, prm[3], st.w, sub, D, gz);
        } else {
#pragma unroll
            for (int j = 0; j < R::NV; ++j)
#pragma unroll
                for (int i = 0; i < 4; ++i) gz[j][i] = g[j][i];
        }
        if (d_extra && t < T) row_store<R>(d_extra + t * D, sub, D, gz);
        if constexpr (DROP)
#pragma unroll
            for (int j = 0; j < R::NV; ++j)
#pragma unroll
                for (int i = 0; i < 4; ++i) gz[j][i] *= keep_factor_bit(bits[j], i, k1);
        if (w1) {
#pragma unroll
            for (int j = 0; j < R::NV; ++j)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    acc[0][j][i] += gz[j][i] * xh1[j][i];
                    acc[1][j][i] += gz[j][i];
                }
            RowVals<R> gx;
            row_ln_bwd<R>(gz, xh1, prm[0], st.y, sub, D, gx);
            if (t < T) row_store<R, ASME_EMB_NT>(d_rows + t * D, sub, D, gx);
        } else if (t < T) {
            row_store<R, ASME_EMB_NT>(d_rows + t * D, sub, D, gz);
        }
    }
    if (partials) write_row_partials<R, NACC, kWavesPerBlock>(acc, lane, wave, D, partials);
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

// dest[ids[s]] = rows[s] for the s < *count first rows (distinct ids: the dedup's unique rows): one row per wave
template <int VPL>
__global__ __launch_bounds__(256) void scatter_rows_kernel(const float* __restrict__ rows,
                                                           const int64_t* __restrict__ ids,
                                                           const int32_t* __restrict__ count, int64_t cap, int D,
                                                           float* __restrict__ dest, int64_t V) {
    const int lane = threadIdx.x & 63;
    const int64_t s = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    if (s >= cap || s >= (int64_t)*count) return;
    const int64_t id = ids[s];
    if (id < 0 || id >= V) return;
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
        const int e = lane + 64 * j;
        if (e < D) dest[id * D + e] = rows[s * D + e];
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

// The same partial sums with float4 loads: 256 threads = G groups of D / 4 lanes (one whole row per group, one
// 16-B chunk per lane); group g sums the chunk's rows b0 + g, b0 + g + G, ... in four independent chains (the
// loads of four rows in flight per lane), and the G group sums are added in group order through LDS.  D / 4 must
// divide 256 (D a power of two, 4 <= D <= 1024).
__global__ __launch_bounds__(256) void pos_partial4_kernel(const float* __restrict__ rows, int64_t B, int64_t L,
                                                           int D, int64_t chunk, float* __restrict__ part) {
    __shared__ float4 red[256];
    const int64_t p = blockIdx.x, c = blockIdx.y;
    const int lanes = D >> 2, G = 256 / lanes, g = threadIdx.x / lanes, lane = threadIdx.x % lanes;
    const int64_t b0 = c * chunk, b1 = min(B, b0 + chunk);
    const float4* src = reinterpret_cast<const float4*>(rows) + p * lanes + lane;
    const int64_t rstride = L * lanes;  // float4s between consecutive batch rows of position p
    float4 a[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) a[j] = make_float4(0.f, 0.f, 0.f, 0.f);
    int64_t b = b0 + g;
    for (; b + 3 * G < b1; b += 4 * G) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float4 v = src[(b + j * G) * rstride];
            a[j] = make_float4(a[j].x + v.x, a[j].y + v.y, a[j].z + v.z, a[j].w + v.w);
        }
    }
    // at most three rows of this group are left (constant indices: the accumulators stay in registers)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        if (b + j * G < b1) {
            const float4 v = src[(b + j * G) * rstride];
            a[j] = make_float4(a[j].x + v.x, a[j].y + v.y, a[j].z + v.z, a[j].w + v.w);
        }
    }
    red[threadIdx.x] = make_float4((a[0].x + a[1].x) + (a[2].x + a[3].x), (a[0].y + a[1].y) + (a[2].y + a[3].y),
                                   (a[0].z + a[1].z) + (a[2].z + a[3].z), (a[0].w + a[1].w) + (a[2].w + a[3].w));
    __syncthreads();
    if (g == 0) {
        float4 t = red[lane];
        for (int k = 1; k < G; ++k) {
            const float4 v = red[k * lanes + lane];
            t = make_float4(t.x + v.x, t.y + v.y, t.z + v.z, t.w + v.w);
        }
        reinterpret_cast<float4*>(part)[(c * L + p) * lanes + lane] = t;
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
    // four independent chains per thread (rows grp + 16 (4i + j), chain j), added in a fixed order: 4x the
    // loads in flight of a single chain (a few column blocks of a narrow matrix are otherwise latency-bound)
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    if (c < width) {
        int64_t r = grp;
        for (; r + 3 * kRedGroups < nrows; r += 4 * kRedGroups) {
            s0 += part[r * width + c];
            s1 += part[(r + kRedGroups) * width + c];
            s2 += part[(r + 2 * kRedGroups) * width + c];
            s3 += part[(r + 3 * kRedGroups) * width + c];
        }
        for (; r < nrows; r += kRedGroups) s0 += part[r * width + c];
    }
    red[grp][col] = (s0 + s1) + (s2 + s3);
    __syncthreads();
    for (int h = kRedGroups / 2; h > 0; h >>= 1) {
        if (grp < h) red[grp][col] += red[grp + h][col];
        __syncthreads();
    }
    if (grp == 0 && c < width) out[c] = accumulate ? out[c] + red[0][col] : red[0][col];
}

// narrow matrices (the LayerNorm parameter partials: 1,024-2,048 rows x 2d-6d columns): 16 columns per block and 64
// row-groups, so a 256-column sum runs on 16 workgroups with 16 rows per thread instead of 4 workgroups with 64
constexpr int kNarCols = 16, kNarGroups = 64;
__global__ __launch_bounds__(1024) void reduce_rows_narrow_kernel(const float* __restrict__ part, int64_t nrows,
                                                                  int64_t width, float* __restrict__ out,
                                                                  int accumulate) {
    __shared__ float red[kNarGroups][kNarCols];
    const int col = threadIdx.x % kNarCols, grp = threadIdx.x / kNarCols;
    const int64_t c = (int64_t)blockIdx.x * kNarCols + col;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    if (c < width) {
        int64_t r = grp;
        for (; r + 3 * kNarGroups < nrows; r += 4 * kNarGroups) {
            s0 += part[r * width + c];
            s1 += part[(r + kNarGroups) * width + c];
            s2 += part[(r + 2 * kNarGroups) * width + c];
            s3 += part[(r + 3 * kNarGroups) * width + c];
        }
        for (; r < nrows; r += kNarGroups) s0 += part[r * width + c];
    }
    red[grp][col] = (s0 + s1) + (s2 + s3);
    __syncthreads();
    for (int h = kNarGroups / 2; h > 0; h >>= 1) {
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

// out[r] = table[ids[r]] (zero row for ids outside [0, V)); D % 4 == 0: float4 lanes, K rows in flight per
// lane group (the owner side of the row-sharded lookup)
template <class R, int K>
__global__ __launch_bounds__(256) void gather_rows4_kernel(const int64_t* __restrict__ ids, int64_t n,
                                                           const float* __restrict__ table, int64_t V, int D,
                                                           float* __restrict__ out) {
    const int lane = threadIdx.x & 63, sub = lane % R::LPR;
    const int64_t r0 = ((int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)) * R::RPW * K + lane / R::LPR;
    int64_t id[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int64_t r = r0 + (int64_t)k * R::RPW;
        id[k] = r < n ? ids[r] : -1;
    }
    RowVals<R> x[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        if (id[k] >= 0 && id[k] < V) row_load<R>(table + id[k] * D, sub, D, x[k]);
        else row_zero<R>(x[k]);
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int64_t r = r0 + (int64_t)k * R::RPW;
        if (r < n) row_store<R>(out + r * D, sub, D, x[k]);
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

// Row layout of the embedding kernels: at D = 128 a row is 16 lanes x two float4 (4 rows per wave) rather than the
// shared 32 x one float4, so every LayerNorm statistic reduces inside a 16-lane DPP row (no permlane step) and a
// wave has twice the tokens in flight.
#ifndef ASME_EMB_LPR16
#define ASME_EMB_LPR16 1
#endif
#ifndef ASME_EMB_BWD_LPR16
#define ASME_EMB_BWD_LPR16 1
#endif
#ifndef ASME_EMB_K
#define ASME_EMB_K 1
#endif
#ifndef ASME_EMB_BWD_PASS
#define ASME_EMB_BWD_PASS 1
#endif
#ifndef ASME_EMB_BWD128
#define ASME_EMB_BWD128 1  // 0: the D = 128 backward on the general emb_bwd4_kernel (A/B)
#endif
template <class F>
int with_emb_layout(int64_t D, F&& f, bool lpr16 = ASME_EMB_LPR16) {
    if (lpr16 && D == 128) {
        f(RowLayout<4, 16, 2>{});
        return 0;
    }
    return with_row_layout(D, f);
}

namespace {
// the forward at D = 128 on 8 lanes per row (16 values per lane): the per-row work every lane of a row repeats --
// statistics reductions, rsqrt, addressing, ids, stores of statistics -- runs on half as many lanes
#ifndef ASME_EMB_FWD_LPR8
#define ASME_EMB_FWD_LPR8 1
#endif
int embedding_fwd(const int64_t* ids, int64_t n_tokens, int64_t seq_len, const float* table, int64_t vocab,
                  int64_t dim, const float* pos_table, const float* ln1_w, const float* ln1_b, float ln1_eps, float p1,
                  uint64_t seed1, const float* extra, const float* ln2_w, const float* ln2_b, float ln2_eps, float p2,
                  uint64_t seed2, float* out, float* stats, uint8_t* keep_mask, int* err_flag, const EmbLn3* l3,
                  void* stream) {
    ASME_CHECK_ARG(ids && table && out && stats, "asme_embedding_fwd: null pointer");
    ASME_CHECK_ARG(dim >= 1 && dim <= 512 && seq_len >= 1 && n_tokens >= 0, "asme_embedding_fwd: bad shape");
    ASME_CHECK_ARG(p1 >= 0.f && p1 < 1.f && p2 >= 0.f && p2 < 1.f, "asme_embedding_fwd: dropout p must be in [0,1)");
    if (n_tokens == 0) return 0;
    auto body = [&](auto layout) {
            using R = decltype(layout);
            if constexpr (R::W == 4) {
                constexpr int K = ASME_EMB_K;  // tokens per lane group
                const int64_t rows = (int64_t)kWavesPerBlock * R::RPW * K;
                const dim3 grid((unsigned)((n_tokens + rows - 1) / rows));
                auto launch = [&](auto ln3_tag, auto ln2_tag) {
                    constexpr bool LN3 = decltype(ln3_tag)::value, LN2 = decltype(ln2_tag)::value;
                    hipLaunchKernelGGL(HIP_KERNEL_NAME(emb_fwd4_kernel<R, K, LN3, LN2>), grid, dim3(256), 0,
                                       (hipStream_t)stream, ids, n_tokens, seq_len, table, vocab, (int)dim, pos_table,
                                       ln1_w, ln1_b, ln1_eps, p1, extra, ln2_w, ln2_b, ln2_eps, p2,
                                       emb_seed(seed1, seed2), out, stats, keep_mask, err_flag, l3 ? *l3 : EmbLn3{});
                };
                if (l3) {
                    if (ln2_w) launch(std::true_type{}, std::true_type{});
                    else launch(std::true_type{}, std::false_type{});
                } else {
                    if (ln2_w) launch(std::false_type{}, std::true_type{});
                    else launch(std::false_type{}, std::false_type{});
                }
            } else {
                const int64_t rows = (int64_t)kWavesPerBlock * R::RPW;
                hipLaunchKernelGGL(emb_fwd_kernel<R>, dim3((unsigned)((n_tokens + rows - 1) / rows)), dim3(256), 0,
                                   (hipStream_t)stream, ids, n_tokens, seq_len, table, vocab, (int)dim, pos_table,
                                   ln1_w, ln1_b, ln1_eps, p1, seed1, extra, ln2_w, ln2_b, ln2_eps, p2, seed2, out,
                                   stats, err_flag);
            }
        };
    if (ASME_EMB_FWD_LPR8 && dim == 128)
        body(RowLayout<4, 8, 4>{});
    else if (with_emb_layout(dim, body))
        return -1;
    ASME_LAUNCH_CHECK("asme_embedding_fwd");
}
}  // namespace

ASME_API int asme_embedding_fwd(const int64_t* ids, int64_t n_tokens, int64_t seq_len, const float* table,
                                int64_t vocab, int64_t dim, const float* pos_table, const float* ln1_w,
                                const float* ln1_b, float ln1_eps, float p1, uint64_t seed1, const float* extra,
                                const float* ln2_w, const float* ln2_b, float ln2_eps, float p2, uint64_t seed2,
                                float* out, float* stats, uint8_t* keep_mask, int* err_flag, void* stream) {
    return embedding_fwd(ids, n_tokens, seq_len, table, vocab, dim, pos_table, ln1_w, ln1_b, ln1_eps, p1, seed1, extra,
                         ln2_w, ln2_b, ln2_eps, p2, seed2, out, stats, keep_mask, err_flag, nullptr, stream);
}

// asme_embedding_fwd + the first transformer block's input LayerNorm on the output rows (ln3_out = LN3(out),
// ln3_stats (T, 2) = mean, rstd); dim % 4 == 0
ASME_API int asme_embedding_ln_fwd(const int64_t* ids, int64_t n_tokens, int64_t seq_len, const float* table,
                                   int64_t vocab, int64_t dim, const float* pos_table, const float* ln1_w,
                                   const float* ln1_b, float ln1_eps, float p1, uint64_t seed1, const float* extra,
                                   const float* ln2_w, const float* ln2_b, float ln2_eps, float p2, uint64_t seed2,
                                   const float* ln3_w, const float* ln3_b, float ln3_eps, float* out, float* stats,
                                   float* ln3_out, float* ln3_stats, uint8_t* keep_mask, int* err_flag,
                                   void* stream) {
    ASME_CHECK_ARG(ln3_w && ln3_b && ln3_out && ln3_stats, "asme_embedding_ln_fwd: null pointer");
    ASME_CHECK_ARG(dim % 4 == 0, "asme_embedding_ln_fwd: dim must be a multiple of 4");
    const EmbLn3 l3{ln3_w, ln3_b, ln3_eps, ln3_out, ln3_stats, nullptr, nullptr};
    return embedding_fwd(ids, n_tokens, seq_len, table, vocab, dim, pos_table, ln1_w, ln1_b, ln1_eps, p1, seed1, extra,
                         ln2_w, ln2_b, ln2_eps, p2, seed2, out, stats, keep_mask, err_flag, &l3, stream);
}

ASME_API int asme_embedding_bwd_partials_count(void) { return 1024; }

namespace {
int embedding_bwd(const int64_t* ids, int64_t n_tokens, int64_t seq_len, const float* table, int64_t vocab,
                  int64_t dim, const float* pos_table, const float* ln1_w, const float* ln1_b, float p1,
                  uint64_t seed1, const float* extra, const float* ln2_w, float p2, uint64_t seed2,
                  const uint8_t* keep_mask, const float* dout, const float* stats, float* d_rows, float* d_extra,
                  float* partials, int64_t n_partials, const EmbLn3* l3, void* stream) {
    ASME_CHECK_ARG(ids && table && dout && stats && d_rows, "asme_embedding_bwd: null pointer");
    ASME_CHECK_ARG(dim >= 1 && dim <= 512, "asme_embedding_bwd: bad shape");
    ASME_CHECK_ARG(!partials || n_partials >= 1, "asme_embedding_bwd: n_partials must be >= 1");
    if (n_tokens == 0) return 0;
    const size_t lds = partials ? (size_t)kWavesPerBlock * (l3 ? 6 : 4) * dim * sizeof(float) : 0;
    if (with_emb_layout(dim, [&](auto layout) {
            using R = decltype(layout);
            const int64_t rows = (int64_t)kWavesPerBlock * R::RPW;
            // grid-stride with one partial row per block when the LN parameter grads are wanted
            const int64_t nb = partials ? n_partials : (n_tokens + rows - 1) / rows;
            if constexpr (R::W == 4) {
                constexpr int kPass = ASME_EMB_BWD_PASS;  // 2 tokens per pass at 16 lanes: 160 VGPRs, slower (169 vs 121 us)
                const int64_t nb4 = partials ? n_partials : (n_tokens + rows - 1) / rows;
                // D = 128 (16 lanes x two float4) with the keep bytes given or no dropout: the straight-line kernel
                const bool fast = ASME_EMB_BWD128 && R::LPR == 16 && R::NV == 2 && dim == 128 &&
                                  (keep_mask || (p1 == 0.f && p2 == 0.f));
                auto launch = [&](auto ln3_tag, auto ln2_tag) {
                    constexpr bool LN3 = decltype(ln3_tag)::value, LN2 = decltype(ln2_tag)::value;
                    auto go = [&](auto pos_tag, auto drop_tag) {
                        constexpr bool POS = decltype(pos_tag)::value, DROP = decltype(drop_tag)::value;
                        hipLaunchKernelGGL(HIP_KERNEL_NAME(emb_bwd128_kernel<LN3, LN2, POS, DROP>), dim3((unsigned)nb4),
                                           dim3(256), lds, (hipStream_t)stream, ids, n_tokens, seq_len, table, vocab,
                                           pos_table, ln1_w, ln1_b, p1, extra, ln2_w, p2, keep_mask, dout, stats, d_rows,
                                           d_extra, partials, l3 ? *l3 : EmbLn3{});
                    };
                    const bool drop = keep_mask && (p1 > 0.f || p2 > 0.f);
                    if (fast) {
                        if (pos_table) {
                            if (drop) go(std::true_type{}, std::true_type{});
                            else go(std::true_type{}, std::false_type{});
                        } else {
                            if (drop) go(std::false_type{}, std::true_type{});
                            else go(std::false_type{}, std::false_type{});
                        }
                    } else
                        hipLaunchKernelGGL(HIP_KERNEL_NAME(emb_bwd4_kernel<R, kPass, LN3, LN2>), dim3((unsigned)nb4),
                                           dim3(256), lds, (hipStream_t)stream, ids, n_tokens, seq_len, table, vocab,
                                           (int)dim, pos_table, ln1_w, ln1_b, p1, extra, ln2_w, p2,
                                           emb_seed(seed1, seed2), keep_mask, dout, stats, d_rows, d_extra, partials,
                                           l3 ? *l3 : EmbLn3{});
                };
                if (l3) {
                    if (ln2_w) launch(std::true_type{}, std::true_type{});
                    else launch(std::true_type{}, std::false_type{});
                } else {
                    if (ln2_w) launch(std::false_type{}, std::true_type{});
                    else launch(std::false_type{}, std::false_type{});
                }
            } else {
                hipLaunchKernelGGL(emb_bwd_kernel<R>, dim3((unsigned)nb), dim3(256), lds, (hipStream_t)stream, ids,
                                   n_tokens, seq_len, table, vocab, (int)dim, pos_table, ln1_w, ln1_b, p1, seed1,
                                   extra, ln2_w, p2, seed2, dout, stats, d_rows, d_extra, partials);
            }
        }, ASME_EMB_BWD_LPR16))
        return -1;
    ASME_LAUNCH_CHECK("asme_embedding_bwd");
}
}  // namespace

ASME_API int asme_embedding_bwd(const int64_t* ids, int64_t n_tokens, int64_t seq_len, const float* table,
                                int64_t vocab, int64_t dim, const float* pos_table, const float* ln1_w,
                                const float* ln1_b, float p1, uint64_t seed1, const float* extra, const float* ln2_w,
                                float p2, uint64_t seed2, const uint8_t* keep_mask, const float* dout,
                                const float* stats, float* d_rows, float* d_extra, float* partials,
                                int64_t n_partials, void* stream) {
    return embedding_bwd(ids, n_tokens, seq_len, table, vocab, dim, pos_table, ln1_w, ln1_b, p1, seed1, extra, ln2_w,
                         p2, seed2, keep_mask, dout, stats, d_rows, d_extra, partials, n_partials, nullptr, stream);
}

// backward of asme_embedding_ln_fwd: dout = gradient of `out` (the residual stream), dln = gradient of ln3_out;
// partials (n_partials, 6 * dim): LN1 w / b, LN2 w / b, LN3 w / b column partials (LN1 / LN2 rows zero when
// absent); ln2_b is required with ln2_w (the output is recomputed through LN2's affine)
ASME_API int asme_embedding_ln_bwd(const int64_t* ids, int64_t n_tokens, int64_t seq_len, const float* table,
                                   int64_t vocab, int64_t dim, const float* pos_table, const float* ln1_w,
                                   const float* ln1_b, float p1, uint64_t seed1, const float* extra,
                                   const float* ln2_w, const float* ln2_b, float p2, uint64_t seed2,
                                   const float* ln3_w, const float* ln3_stats, const uint8_t* keep_mask,
                                   const float* dout, const float* dln, const float* stats, float* d_rows,
                                   float* d_extra, float* partials, int64_t n_partials, void* stream) {
    ASME_CHECK_ARG(ln3_w && ln3_stats && dln && partials, "asme_embedding_ln_bwd: null pointer");
    ASME_CHECK_ARG(!ln2_w || ln2_b, "asme_embedding_ln_bwd: ln2_b required with ln2_w");
    ASME_CHECK_ARG(dim % 4 == 0, "asme_embedding_ln_bwd: dim must be a multiple of 4");
    const EmbLn3 l3{ln3_w, nullptr, 0.f, nullptr, const_cast<float*>(ln3_stats), dln, ln2_b};
    return embedding_bwd(ids, n_tokens, seq_len, table, vocab, dim, pos_table, ln1_w, ln1_b, p1, seed1, extra, ln2_w,
                         p2, seed2, keep_mask, dout, stats, d_rows, d_extra, partials, n_partials, &l3, stream);
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

ASME_API int asme_scatter_rows(const float* rows, const int64_t* ids, const int32_t* count, int64_t cap, int64_t dim,
                              float* dest, int64_t vocab, void* stream) {
    ASME_CHECK_ARG(rows && ids && count && dest, "asme_scatter_rows: null pointer");
    ASME_CHECK_ARG(dim >= 1 && dim <= 512 && cap >= 0, "asme_scatter_rows: bad shape");
    if (cap == 0) return 0;
    const dim3 grid((unsigned)((cap + kWavesPerBlock - 1) / kWavesPerBlock));
    ASME_VPL_DISPATCH(vpl_of(dim), hipLaunchKernelGGL(scatter_rows_kernel<VPL>, grid, dim3(256), 0,
                                                      (hipStream_t)stream, rows, ids, count, cap, (int)dim, dest,
                                                      vocab));
    ASME_LAUNCH_CHECK("asme_scatter_rows");
}

ASME_API int asme_position_grad(const float* rows, int64_t batch, int64_t seq_len, int64_t dim, float* workspace,
                                int64_t n_chunks, float* grad_pos, int accumulate, void* stream) {
    ASME_CHECK_ARG(rows && workspace && grad_pos && n_chunks >= 1, "asme_position_grad: bad argument");
    const int64_t chunk = (batch + n_chunks - 1) / n_chunks;
    const bool wide = dim >= 4 && dim <= 1024 && (dim & (dim - 1)) == 0 && ((uintptr_t)rows & 15) == 0 &&
                      ((uintptr_t)workspace & 15) == 0;
    if (wide)
        hipLaunchKernelGGL(pos_partial4_kernel, dim3((unsigned)seq_len, (unsigned)n_chunks), dim3(256), 0,
                           (hipStream_t)stream, rows, batch, seq_len, (int)dim, chunk, workspace);
    else
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
    if (width <= kNarCols * kNarGroups && n_rows >= 4 * kNarGroups)
        hipLaunchKernelGGL(reduce_rows_narrow_kernel, dim3((unsigned)((width + kNarCols - 1) / kNarCols)), dim3(1024),
                           0, (hipStream_t)stream, part, n_rows, width, out, accumulate);
    else
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

ASME_API int asme_gather_rows(const int64_t* ids, int64_t n, const float* table, int64_t vocab, int64_t dim,
                              float* out, void* stream) {
    ASME_CHECK_ARG(ids && table && out, "asme_gather_rows: null pointer");
    ASME_CHECK_ARG(dim >= 1 && dim <= 512, "asme_gather_rows: bad shape");
    if (n == 0) return 0;
    if (dim % 4 != 0 || ((uintptr_t)table & 15) || ((uintptr_t)out & 15))
        return asme_gather_sum_fwd(ids, n, 1, 0, table, vocab, dim, nullptr, out, 0, stream);
    if (with_row_layout(dim, [&](auto layout) {
            using R = decltype(layout);
            if constexpr (R::W == 4) {
                constexpr int K = 4;
                const int64_t rows = (int64_t)kWavesPerBlock * R::RPW * K;
                hipLaunchKernelGGL(HIP_KERNEL_NAME(gather_rows4_kernel<R, K>), dim3((unsigned)((n + rows - 1) / rows)),
                                   dim3(256), 0, (hipStream_t)stream, ids, n, table, vocab, (int)dim, out);
            }
        }))
        return -1;
    ASME_LAUNCH_CHECK("asme_gather_rows");
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
