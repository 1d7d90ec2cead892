// Token-major Linear layers of the ASME transformer block with fused epilogues, fp32 MFMA on gfx950.
//
// Reference semantics (paths relative to /root/reference/src/asme):
//   nn.Linear projections         core/models/common/layers/transformer_layers.py:175-199 (Q,K,V,O)
//   PositionwiseFeedForward       transformer_layers.py:212-220  W2(dropout(GELU_erf(W1 x)))
//   SublayerConnection            transformer_layers.py:120-130  x + dropout(sublayer(LN(x)))   (pre-LN)
//   TransformerBlock              transformer_layers.py:251-258  block dropout at the end
//
// Forward  (C = X W^T + b, X: M x K row-major, W: N x K row-major = nn.Linear.weight):
//   EPI_STORE       y = C
//   EPI_GELU_DROP   pre = C; y = dropout(GELU(C))                       (FFN inner layer)
//   EPI_RESLN       s = drop_b(res + drop_a(C)); ln = LN(s) (N == 128)  (sublayer epilogue + next pre-LN)
// Backward (C = dY W, dY: M x N', W: N' x K row-major; the output width is the layer's in_features):
//   EPI_STORE       dX = C (or += C)
//   EPI_GELU_BWD    dX = C * keep * GELU'(pre)                          (through the FFN activation)
//   EPI_RESLN_BWD   d_s = d_in + LN_bwd(C); d_res = drop_b'(d_s); d_y = drop_a'(d_res)  (N == 128)
// Dropout decisions are exactly those of the standalone kernels (norm.hip): element index m*N + n,
// one Philox block per 4 consecutive elements of a row, salts 3/4 (residual) and 5 (FFN).
//
// Kernel shape: C^T tiles are computed (MFMA rows = output features, columns = tokens) so each lane ends
// with 4 consecutive output features of one token: float4 epilogue I/O and per-row reductions with two
// xor shuffles.  Workgroup = 4 waves = 128 tokens x 128 features; wave w owns tokens 32w..32w+31 (2 x 8
// MFMA 16x16 tiles).  The reduction dimension streams through LDS in 32-wide slabs (register-prefetched
// one slab ahead); within a slab lane group g supplies k = 8g .. 8g+7 (ds_read_b128 operand reads).
// Workgroups are mapped XCD-aware: the feature blocks of one token block run on the same XCD (shared L2).
#include "common.h"
#include "rows.h"
#include <algorithm>

using namespace asme;

namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int kBM = 128;  // tokens per workgroup
constexpr int kBN = 128;  // output features per workgroup
constexpr int kBK = 32;   // reduction slab (double-buffered in LDS)
constexpr int kLd = 36;   // LDS row stride (floats)
constexpr int kThreads = 256;

enum Epi { EPI_STORE = 0, EPI_GELU_DROP = 1, EPI_RESLN = 2, EPI_GELU_BWD = 3, EPI_RESLN_BWD = 4 };

__device__ __forceinline__ floatx4 mfma16(float a, float b, floatx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Row slab: 128 rows x 32 floats of a row-major matrix; thread t holds float4 (row (t>>3) + 32q, col (t&7)*4)
__device__ __forceinline__ void load_rows_slab(const float* __restrict__ base, int64_t ld, int64_t row0,
                                               int64_t nrows, int k0, int K, float4 (&r)[4]) {
    const int c4 = (threadIdx.x & 7) * 4;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int64_t row = row0 + (threadIdx.x >> 3) + 32 * q;
        r[q] = (row < nrows && k0 + c4 < K) ? *reinterpret_cast<const float4*>(base + row * ld + k0 + c4)
                                             : make_float4(0.f, 0.f, 0.f, 0.f);
    }
}
__device__ __forceinline__ void store_rows_slab(float* __restrict__ s, const float4 (&r)[4]) {
    const int c4 = (threadIdx.x & 7) * 4;
#pragma unroll
    for (int q = 0; q < 4; ++q) *reinterpret_cast<float4*>(s + ((threadIdx.x >> 3) + 32 * q) * kLd + c4) = r[q];
}
// Column slab for the backward: W is (K x N) row-major and the slab needs [n][k], k in [k0, k0+32):
// thread t gathers 4 consecutive k of column n = t & 127 (lanes read consecutive n: coalesced).
__device__ __forceinline__ void load_cols_slab(const float* __restrict__ w, int64_t ldw, int k0, int K, int n0,
                                               int N, float4 (&r)[4]) {
    const int n = n0 + (threadIdx.x & 127);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int k = k0 + 4 * ((threadIdx.x >> 7) + 2 * q);
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = (n < N && k + i < K) ? w[(int64_t)(k + i) * ldw + n] : 0.f;
        r[q] = make_float4(v[0], v[1], v[2], v[3]);
    }
}
__device__ __forceinline__ void store_cols_slab(float* __restrict__ s, const float4 (&r)[4]) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
        *reinterpret_cast<float4*>(s + (threadIdx.x & 127) * kLd + 4 * ((threadIdx.x >> 7) + 2 * q)) = r[q];
}

template <bool TRANS_W>
__device__ __forceinline__ void load_slab(const float* __restrict__ X, int64_t ldx, int64_t M, int K,
                                          const float* __restrict__ W, int64_t ldw, int N, int64_t m0, int n0, int k0,
                                          float4 (&rx)[4], float4 (&rw)[4]) {
    load_rows_slab(X, ldx, m0, M, k0, K, rx);
    if (TRANS_W)
        load_cols_slab(W, ldw, k0, K, n0, N, rw);
    else
        load_rows_slab(W, ldw, n0, N, k0, K, rw);
}
template <bool TRANS_W>
__device__ __forceinline__ void store_slab(float* __restrict__ buf, const float4 (&rx)[4], const float4 (&rw)[4]) {
    store_rows_slab(buf, rx);
    if (TRANS_W)
        store_cols_slab(buf + kBM * kLd, rw);
    else
        store_rows_slab(buf + kBM * kLd, rw);
}

// acc[rt][ct] += C^T tile (features ct*16.., tokens rt*16..) of this wave for one 32-wide slab in LDS;
// in half h lane group g supplies k = 16h + 4g .. +3 (one ds_read_b128 per operand and half).
__device__ __forceinline__ void slab_mfma(const float* __restrict__ buf, int wave, int g, int c16,
                                          floatx4 (&acc)[2][8]) {
    const float* Xs = buf;
    const float* Ws = buf + kBM * kLd;
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
}

// Persistent tile schedule: the tile list [m-block][n-block] is split into 8 contiguous ranges, one
// per XCD (hardware workgroup ids go round-robin over the XCDs), so the n-blocks of one m-block -- which
// stream the same X slabs -- run side by side on one XCD and share its L2.
struct TileSched {
    int64_t first, stride, count;
    __device__ explicit TileSched(int64_t nt) {
        const int xcd = blockIdx.x % 8, slot = blockIdx.x / 8;
        const int64_t per_xcd = (nt + 7) / 8;
        first = (int64_t)xcd * per_xcd + slot;
        stride = gridDim.x / 8;  // the launch uses a multiple of 8 workgroups
        const int64_t end = min(nt, (int64_t)(xcd + 1) * per_xcd);
        count = first < end ? (end - first + stride - 1) / stride : 0;
    }
    __device__ int64_t tile(int64_t j) const { return first + j * stride; }
};

struct EpiArgs {
    const float* bias;     // [N] (forward)
    // GELU (forward: pre out; backward: pre in)
    float* pre;
    const float* pre_in;
    float p_gelu;
    uint64_t s_gelu;
    // residual + LN
    const float* res;      // forward residual input
    float p_a, p_b;
    uint64_t s_a, s_b;
    const float* ln_w;
    const float* ln_b;
    float eps;
    float* s_out;
    float* stats;          // [M][2] (mean, rstd)
    // backward residual
    const float* s_in;     // forward s
    const float* stats_in;
    const float* d_in;     // upstream gradient of s (nullable)
    float* d_res;
    float* d_y;            // nullable
    float* partials;       // [gridDim][2][N] LN parameter-gradient partials
    int accumulate;
};

template <bool TRANS_W, int EPI>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(2, 2))) void linear_kernel(const float* __restrict__ X, int64_t ldx, int64_t M, int K,
                                                          const float* __restrict__ W, int64_t ldw, int N,
                                                          float* __restrict__ Y, int64_t ldy, EpiArgs ep) {
    __shared__ __attribute__((aligned(16))) float lds[2][(kBM + kBN) * kLd];
    // EPI_RESLN_BWD: per-wave column sums of (d_ln * xhat, d_ln) over this workgroup's rows
    __shared__ float red[EPI == EPI_RESLN_BWD ? 4 * 2 * kBN : 1];
    if constexpr (EPI == EPI_RESLN_BWD) {
        for (int i = threadIdx.x; i < 4 * 2 * kBN; i += kThreads) red[i] = 0.f;
    }
    const int nblk_n = (N + kBN - 1) / kBN;
    const int nslab = (K + kBK - 1) / kBK;
    const TileSched ts(((M + kBM - 1) / kBM) * nblk_n);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c16 = lane & 15;
    const int64_t steps = ts.count * nslab;
    // flattened (tile, slab) pipeline over a double-buffered LDS slab: slab it+1 is stored while slab it
    // is multiplied, slab it+2 is in flight in registers, and a finished tile's epilogue overlaps both
    auto coords = [&](int64_t it, int64_t& m0, int& n0, int& k0) {
        const int j = (int)it / nslab;  // steps < 2^31
        const int t = (int)ts.tile(j);  // tiles < 2^31
        m0 = (int64_t)(t / nblk_n) * kBM;
        n0 = (t % nblk_n) * kBN;
        k0 = ((int)it - j * nslab) * kBK;
    };
    float4 rx[4], rw[4];
    if (steps > 0) {
        int64_t m0;
        int n0, k0;
        coords(0, m0, n0, k0);
        load_slab<TRANS_W>(X, ldx, M, K, W, ldw, N, m0, n0, k0, rx, rw);
        store_slab<TRANS_W>(lds[0], rx, rw);
        if (steps > 1) {
            coords(1, m0, n0, k0);
            load_slab<TRANS_W>(X, ldx, M, K, W, ldw, N, m0, n0, k0, rx, rw);
        }
        __syncthreads();
    }
    floatx4 acc[2][8];
    for (int64_t it = 0; it < steps; ++it) {
        const int slab = (int)it % nslab;
        int64_t m0;
        int n0, k0;
        coords(it, m0, n0, k0);
        if (slab == 0) {
#pragma unroll
            for (int rt = 0; rt < 2; ++rt)
#pragma unroll
                for (int ct = 0; ct < 8; ++ct) acc[rt][ct] = floatx4{0.f, 0.f, 0.f, 0.f};
        }
        slab_mfma(lds[it & 1], wave, g, c16, acc);
        if (it + 1 < steps) store_slab<TRANS_W>(lds[(it + 1) & 1], rx, rw);
        // the prefetch registers are free from here until the next slab's loads are issued below, which
        // keeps the epilogue's register budget; those loads still have a whole slab of MFMA work to land
        if (slab == nslab - 1) {
        if constexpr (EPI == EPI_STORE || EPI == EPI_GELU_DROP || EPI == EPI_GELU_BWD) {
            const float keep_k = ep.p_gelu > 0.f ? 1.f / (1.f - ep.p_gelu) : 1.f;
#pragma unroll
            for (int rt = 0; rt < 2; ++rt) {
                const int64_t m = m0 + wave * 32 + rt * 16 + c16;
                if (m >= M) continue;
#pragma unroll
                for (int ct = 0; ct < 8; ++ct) {
                    const int n = n0 + ct * 16 + 4 * g;
                    if (n >= N) continue;
                    float4 v = make_float4(acc[rt][ct][0], acc[rt][ct][1], acc[rt][ct][2], acc[rt][ct][3]);
                    if (ep.bias) {
                        const float4 bv = *reinterpret_cast<const float4*>(ep.bias + n);
                        v.x += bv.x;
                        v.y += bv.y;
                        v.z += bv.z;
                        v.w += bv.w;
                    }
                    if constexpr (EPI == EPI_GELU_DROP || EPI == EPI_GELU_BWD) {
                        float u[4] = {1.f, 1.f, 1.f, 1.f};
                        if (ep.p_gelu > 0.f) {
                            gelu_keep_factors(gelu_keep_bits4(ep.s_gelu, ((uint64_t)m * N + n) >> 2,
                                                              gelu_thresh(ep.p_gelu)),
                                              keep_k, u);
                        }
                        if constexpr (EPI == EPI_GELU_DROP) {
                            *reinterpret_cast<float4*>(ep.pre + m * ldy + n) = v;
                            v = make_float4(gelu_erf(v.x) * u[0], gelu_erf(v.y) * u[1], gelu_erf(v.z) * u[2],
                                            gelu_erf(v.w) * u[3]);
                        } else {
                            const float4 x = *reinterpret_cast<const float4*>(ep.pre_in + m * ldy + n);
                            v = make_float4(v.x * u[0] * gelu_erf_grad(x.x), v.y * u[1] * gelu_erf_grad(x.y),
                                            v.z * u[2] * gelu_erf_grad(x.z), v.w * u[3] * gelu_erf_grad(x.w));
                        }
                    }
                    float* dst = Y + m * ldy + n;
                    if (EPI == EPI_STORE && ep.accumulate) {
                        const float4 o = *reinterpret_cast<const float4*>(dst);
                        v.x += o.x;
                        v.y += o.y;
                        v.z += o.z;
                        v.w += o.w;
                    }
                    *reinterpret_cast<float4*>(dst) = v;
                }
            }
        }

        if constexpr (EPI == EPI_RESLN) {
            // N == kBN: the tile holds whole rows.  s = drop_b(res + drop_a(C + bias)); ln = LN(s).
            // s overwrites the accumulators in place (register budget), one 16-row tile at a time.
            const float ka = ep.p_a > 0.f ? 1.f / (1.f - ep.p_a) : 1.f;
            const float kb = ep.p_b > 0.f ? 1.f / (1.f - ep.p_b) : 1.f;
#pragma unroll
            for (int rt = 0; rt < 2; ++rt) {
                __builtin_amdgcn_sched_barrier(0);
                const int64_t m = m0 + wave * 32 + rt * 16 + c16;
                const bool ok = m < M;
                float sum = 0.f;
#pragma unroll
                for (int ct = 0; ct < 8; ++ct) {
                    const int n = ct * 16 + 4 * g;
                    float4 a = make_float4(acc[rt][ct][0], acc[rt][ct][1], acc[rt][ct][2], acc[rt][ct][3]);
                    if (ep.bias) {
                        const float4 bv = *reinterpret_cast<const float4*>(ep.bias + n);
                        a.x += bv.x;
                        a.y += bv.y;
                        a.z += bv.z;
                        a.w += bv.w;
                    }
                    float u[4];
                    if (ep.p_a > 0.f) {
                        philox_uniform4(ep.s_a, 3u, ((uint64_t)m * N + n) >> 2, u);
                        a.x *= u[0] >= ep.p_a ? ka : 0.f;
                        a.y *= u[1] >= ep.p_a ? ka : 0.f;
                        a.z *= u[2] >= ep.p_a ? ka : 0.f;
                        a.w *= u[3] >= ep.p_a ? ka : 0.f;
                    }
                    const float4 r = ok ? *reinterpret_cast<const float4*>(ep.res + m * N + n)
                                        : make_float4(0.f, 0.f, 0.f, 0.f);
                    float4 v = make_float4(r.x + a.x, r.y + a.y, r.z + a.z, r.w + a.w);
                    if (ep.p_b > 0.f) {
                        philox_uniform4(ep.s_b, 4u, ((uint64_t)m * N + n) >> 2, u);
                        v.x *= u[0] >= ep.p_b ? kb : 0.f;
                        v.y *= u[1] >= ep.p_b ? kb : 0.f;
                        v.z *= u[2] >= ep.p_b ? kb : 0.f;
                        v.w *= u[3] >= ep.p_b ? kb : 0.f;
                    }
                    if (ok) *reinterpret_cast<float4*>(ep.s_out + m * N + n) = v;
                    acc[rt][ct] = floatx4{v.x, v.y, v.z, v.w};
                    sum += (v.x + v.y) + (v.z + v.w);
                }
                if (!ep.ln_w) continue;
                const float mean = group4_sum(sum) / (float)N;
                float q = 0.f;
#pragma unroll
                for (int ct = 0; ct < 8; ++ct)
#pragma unroll
                    for (int i = 0; i < 4; ++i) q += (acc[rt][ct][i] - mean) * (acc[rt][ct][i] - mean);
                const float rstd = rsqrtf(group4_sum(q) / (float)N + ep.eps);
                if (!ok) continue;
#pragma unroll
                for (int ct = 0; ct < 8; ++ct) {
                    const int n = ct * 16 + 4 * g;
                    const float4 wv = *reinterpret_cast<const float4*>(ep.ln_w + n);
                    const float4 bv = *reinterpret_cast<const float4*>(ep.ln_b + n);
                    *reinterpret_cast<float4*>(Y + m * ldy + n) = make_float4(
                        (acc[rt][ct][0] - mean) * rstd * wv.x + bv.x, (acc[rt][ct][1] - mean) * rstd * wv.y + bv.y,
                        (acc[rt][ct][2] - mean) * rstd * wv.z + bv.z, (acc[rt][ct][3] - mean) * rstd * wv.w + bv.w);
                }
                if (g == 0) *reinterpret_cast<float2*>(ep.stats + m * 2) = make_float2(mean, rstd);
            }
        }
        if constexpr (EPI == EPI_RESLN_BWD) {
            // N == kBN: C = dL/d ln (whole rows).  d_s = d_in + LN_bwd(C); d_res = d_s*keep_b; d_y = d_res*keep_a.
            // One 16-row tile at a time; C*w overwrites the accumulators in place.
            const float ka = ep.p_a > 0.f ? 1.f / (1.f - ep.p_a) : 1.f;
            const float kb = ep.p_b > 0.f ? 1.f / (1.f - ep.p_b) : 1.f;
#pragma unroll
            for (int rt = 0; rt < 2; ++rt) {
                __builtin_amdgcn_sched_barrier(0);
                const int64_t m = m0 + wave * 32 + rt * 16 + c16;
                const bool ok = m < M;
                const float2 st = ok ? *reinterpret_cast<const float2*>(ep.stats_in + m * 2) : make_float2(0.f, 0.f);
                float4 xh[8];
                float sa = 0.f, sb = 0.f;
#pragma unroll
                for (int ct = 0; ct < 8; ++ct) {
                    const int n = ct * 16 + 4 * g;
                    const float4 sv = ok ? *reinterpret_cast<const float4*>(ep.s_in + m * N + n)
                                         : make_float4(0.f, 0.f, 0.f, 0.f);
                    const float4 wv = *reinterpret_cast<const float4*>(ep.ln_w + n);
                    xh[ct] = make_float4((sv.x - st.x) * st.y, (sv.y - st.x) * st.y, (sv.z - st.x) * st.y,
                                         (sv.w - st.x) * st.y);
                    float v[8];
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const float c = acc[rt][ct][i];
                        const float x = i == 0 ? xh[ct].x : (i == 1 ? xh[ct].y : (i == 2 ? xh[ct].z : xh[ct].w));
                        const float wi = i == 0 ? wv.x : (i == 1 ? wv.y : (i == 2 ? wv.z : wv.w));
                        v[i] = c * x;  // LN weight-gradient term
                        v[4 + i] = c;  // LN bias-gradient term
                        const float d = c * wi;
                        sa += d;
                        sb += d * x;
                        acc[rt][ct][i] = d;
                    }
                    // column sums over the 16 rows of this lane group; the owner lane (c16 == 0) adds them into
                    // this wave's LDS row (each column has exactly one owner: deterministic, no atomics)
#pragma unroll
                    for (int i = 0; i < 8; ++i) v[i] = lane16_sum(v[i]);
                    if (c16 == 0) {
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            red[(wave * 2 + 0) * kBN + n + i] += v[i];
                            red[(wave * 2 + 1) * kBN + n + i] += v[4 + i];
                        }
                    }
                }
                sa = group4_sum(sa) / (float)N;
                sb = group4_sum(sb) / (float)N;
                if (!ok) continue;
#pragma unroll
                for (int ct = 0; ct < 8; ++ct) {
                    const int n = ct * 16 + 4 * g;
                    float4 d = make_float4(st.y * (acc[rt][ct][0] - sa - xh[ct].x * sb),
                                           st.y * (acc[rt][ct][1] - sa - xh[ct].y * sb),
                                           st.y * (acc[rt][ct][2] - sa - xh[ct].z * sb),
                                           st.y * (acc[rt][ct][3] - sa - xh[ct].w * sb));
                    if (ep.d_in) {
                        const float4 di = *reinterpret_cast<const float4*>(ep.d_in + m * N + n);
                        d.x += di.x;
                        d.y += di.y;
                        d.z += di.z;
                        d.w += di.w;
                    }
                    float u[4];
                    if (ep.p_b > 0.f) {
                        philox_uniform4(ep.s_b, 4u, ((uint64_t)m * N + n) >> 2, u);
                        d.x *= u[0] >= ep.p_b ? kb : 0.f;
                        d.y *= u[1] >= ep.p_b ? kb : 0.f;
                        d.z *= u[2] >= ep.p_b ? kb : 0.f;
                        d.w *= u[3] >= ep.p_b ? kb : 0.f;
                    }
                    *reinterpret_cast<float4*>(ep.d_res + m * N + n) = d;
                    if (ep.d_y) {
                        if (ep.p_a > 0.f) {
                            philox_uniform4(ep.s_a, 3u, ((uint64_t)m * N + n) >> 2, u);
                            d.x *= u[0] >= ep.p_a ? ka : 0.f;
                            d.y *= u[1] >= ep.p_a ? ka : 0.f;
                            d.z *= u[2] >= ep.p_a ? ka : 0.f;
                            d.w *= u[3] >= ep.p_a ? ka : 0.f;
                        }
                        *reinterpret_cast<float4*>(ep.d_y + m * N + n) = d;
                    }
                }
            }
        }
        }
        if (it + 2 < steps) {
            int64_t m2;
            int n2, k2;
            coords(it + 2, m2, n2, k2);
            load_slab<TRANS_W>(X, ldx, M, K, W, ldw, N, m2, n2, k2, rx, rw);
        }
        __syncthreads();
    }
    if constexpr (EPI == EPI_RESLN_BWD) {
        for (int c = threadIdx.x; c < 2 * kBN; c += kThreads) {
            const int k = c / kBN, n = c % kBN;
            float v = 0.f;
            for (int w = 0; w < 4; ++w) v += red[(w * 2 + k) * kBN + n];
            ep.partials[(int64_t)blockIdx.x * 2 * kBN + c] = v;
        }
    }
}

// persistent grid: 2 resident workgroups per CU (VGPR-bound), a multiple of 8 for the XCD split
int64_t linear_grid(int64_t M, int64_t N) {
    static int n_cu = 0;
    if (n_cu == 0) {
        int dev = 0;
        hipDeviceProp_t prop;
        n_cu = (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
                   ? prop.multiProcessorCount
                   : 256;
    }
    const int64_t ntiles = ((M + kBM - 1) / kBM) * ((N + kBN - 1) / kBN);
    const int64_t grid = std::min<int64_t>((int64_t)n_cu * 2, (ntiles + 7) / 8 * 8);
    return std::max<int64_t>(8, grid / 8 * 8);
}

template <bool TRANS_W, int EPI>
int launch_linear(const float* X, int64_t ldx, int64_t M, int K, const float* W, int64_t ldw, int N, float* Y,
                  int64_t ldy, const EpiArgs& ep, hipStream_t s) {
    const int64_t grid = linear_grid(M, N);
    hipLaunchKernelGGL((linear_kernel<TRANS_W, EPI>), dim3((unsigned)grid), dim3(kThreads), 0, s, X, ldx, M, K, W,
                       ldw, N, Y, ldy, ep);
    return hip_status(hipGetLastError(), "linear");
}

bool shapes_ok(const void* a, int64_t lda, const void* b, int64_t ldb, int K, int N) {
    return K % 4 == 0 && N % 4 == 0 && lda % 4 == 0 && ldb % 4 == 0 && ((uintptr_t)a & 15) == 0 &&
           ((uintptr_t)b & 15) == 0;
}

}  // namespace

// y (n_rows x out_f, row stride ld_y) = x (n_rows x in_f, stride ld_x) . w^T + b      (w: out_f x in_f)
ASME_API int asme_linear_fwd(const float* x, int64_t ld_x, int64_t n_rows, int64_t in_f, const float* w,
                             const float* b, int64_t out_f, float* y, int64_t ld_y, void* stream) {
    ASME_CHECK_ARG(x && w && y, "asme_linear_fwd: null pointer");
    ASME_CHECK_ARG(shapes_ok(x, ld_x, w, in_f, (int)in_f, (int)out_f) && ld_y % 4 == 0 && ((uintptr_t)y & 15) == 0,
                   "asme_linear_fwd: features / strides must be multiples of 4 floats, 16-B aligned");
    if (n_rows == 0) return 0;
    EpiArgs ep{};
    ep.bias = b;
    return launch_linear<false, EPI_STORE>(x, ld_x, n_rows, (int)in_f, w, in_f, (int)out_f, y, ld_y, ep,
                                           (hipStream_t)stream);
}

// dx (n_rows x in_f) (+)= dy (n_rows x out_f) . w      (w: out_f x in_f)
ASME_API int asme_linear_dx(const float* dy, int64_t ld_dy, int64_t n_rows, int64_t out_f, const float* w,
                            int64_t in_f, float* dx, int64_t ld_dx, int accumulate, void* stream) {
    ASME_CHECK_ARG(dy && w && dx, "asme_linear_dx: null pointer");
    ASME_CHECK_ARG(shapes_ok(dy, ld_dy, w, in_f, (int)out_f, (int)in_f) && ld_dx % 4 == 0 &&
                       ((uintptr_t)dx & 15) == 0,
                   "asme_linear_dx: features / strides must be multiples of 4 floats, 16-B aligned");
    if (n_rows == 0) return 0;
    EpiArgs ep{};
    ep.accumulate = accumulate;
    return launch_linear<true, EPI_STORE>(dy, ld_dy, n_rows, (int)out_f, w, in_f, (int)in_f, dx, ld_dx, ep,
                                          (hipStream_t)stream);
}

// pre = x . w^T + b ; y = dropout_p(GELU(pre))      (FFN inner layer; pre/y share the row stride ld_y)
ASME_API int asme_linear_gelu_dropout_fwd(const float* x, int64_t ld_x, int64_t n_rows, int64_t in_f, const float* w,
                                          const float* b, int64_t out_f, float p, uint64_t seed, float* pre,
                                          float* y, int64_t ld_y, void* stream) {
    ASME_CHECK_ARG(x && w && pre && y, "asme_linear_gelu_dropout_fwd: null pointer");
    ASME_CHECK_ARG(shapes_ok(x, ld_x, w, in_f, (int)in_f, (int)out_f) && ld_y % 4 == 0,
                   "asme_linear_gelu_dropout_fwd: features / strides must be multiples of 4 floats");
    ASME_CHECK_ARG(p >= 0.f && p < 1.f, "asme_linear_gelu_dropout_fwd: bad dropout p");
    if (n_rows == 0) return 0;
    EpiArgs ep{};
    ep.bias = b;
    ep.pre = pre;
    ep.p_gelu = p;
    ep.s_gelu = seed;
    return launch_linear<false, EPI_GELU_DROP>(x, ld_x, n_rows, (int)in_f, w, in_f, (int)out_f, y, ld_y, ep,
                                               (hipStream_t)stream);
}

// dx = (dy . w) * keep_p * GELU'(pre)        (pre: n_rows x in_f with row stride ld_dx)
ASME_API int asme_linear_dx_gelu_bwd(const float* dy, int64_t ld_dy, int64_t n_rows, int64_t out_f, const float* w,
                                     int64_t in_f, const float* pre, float p, uint64_t seed, float* dx, int64_t ld_dx,
                                     void* stream) {
    ASME_CHECK_ARG(dy && w && pre && dx, "asme_linear_dx_gelu_bwd: null pointer");
    ASME_CHECK_ARG(shapes_ok(dy, ld_dy, w, in_f, (int)out_f, (int)in_f) && ld_dx % 4 == 0,
                   "asme_linear_dx_gelu_bwd: features / strides must be multiples of 4 floats");
    if (n_rows == 0) return 0;
    EpiArgs ep{};
    ep.pre_in = pre;
    ep.p_gelu = p;
    ep.s_gelu = seed;
    return launch_linear<true, EPI_GELU_BWD>(dy, ld_dy, n_rows, (int)out_f, w, in_f, (int)in_f, dx, ld_dx, ep,
                                             (hipStream_t)stream);
}

// Sublayer epilogue fused into the projection (out_f == 128):
//   a = x . w^T + b;  s_out = drop_b(res + drop_a(a));  ln_out = LN(s_out) (ln_w nullable: no LN)
// res / s_out / ln_out are (n_rows x 128) contiguous; stats (n_rows x 2) = (mean, rstd).
ASME_API int asme_linear_residual_ln_fwd(const float* x, int64_t ld_x, int64_t n_rows, int64_t in_f, const float* w,
                                         const float* b, int64_t out_f, const float* res, float p_a, uint64_t seed_a,
                                         float p_b, uint64_t seed_b, const float* ln_w, const float* ln_b, float eps,
                                         float* s_out, float* ln_out, float* stats, void* stream) {
    ASME_CHECK_ARG(x && w && res && s_out, "asme_linear_residual_ln_fwd: null pointer");
    ASME_CHECK_ARG(!ln_w || (ln_b && ln_out && stats), "asme_linear_residual_ln_fwd: LayerNorm outputs missing");
    ASME_CHECK_ARG(out_f == kBN, "asme_linear_residual_ln_fwd: out_features must be 128");
    ASME_CHECK_ARG(shapes_ok(x, ld_x, w, in_f, (int)in_f, (int)out_f), "asme_linear_residual_ln_fwd: bad strides");
    ASME_CHECK_ARG(p_a >= 0.f && p_a < 1.f && p_b >= 0.f && p_b < 1.f, "asme_linear_residual_ln_fwd: bad dropout p");
    if (n_rows == 0) return 0;
    EpiArgs ep{};
    ep.bias = b;
    ep.res = res;
    ep.p_a = p_a;
    ep.s_a = seed_a;
    ep.p_b = p_b;
    ep.s_b = seed_b;
    ep.ln_w = ln_w;
    ep.ln_b = ln_b;
    ep.eps = eps;
    ep.s_out = s_out;
    ep.stats = stats;
    return launch_linear<false, EPI_RESLN>(x, ld_x, n_rows, (int)in_f, w, in_f, (int)out_f, ln_out, out_f, ep,
                                           (hipStream_t)stream);
}

// Rows of LN parameter-gradient partials asme_linear_dx_residual_ln_bwd writes (2 x 128 floats each).
ASME_API int64_t asme_linear_partials_rows(int64_t n_rows) { return linear_grid(n_rows, kBN); }

// Backward of the sublayer epilogue fused into the consumer's input-gradient GEMM (in_f == 128):
//   C = dy . w (= dL/d ln);  d_s = d_in + LN_bwd(C);  d_res = d_s * keep_b;  d_y = d_res * keep_a
// s / stats: the forward s and its (mean, rstd); d_in (nullable) the residual-path gradient of s;
// partials: asme_linear_partials_rows(n_rows) x [dw(128), db(128)] of the LayerNorm parameters.
ASME_API int asme_linear_dx_residual_ln_bwd(const float* dy, int64_t ld_dy, int64_t n_rows, int64_t out_f,
                                            const float* w, int64_t in_f, const float* s, const float* stats,
                                            const float* ln_w, const float* d_in, float p_a, uint64_t seed_a,
                                            float p_b, uint64_t seed_b, float* d_res, float* d_y, float* partials,
                                            void* stream) {
    ASME_CHECK_ARG(dy && w && s && stats && ln_w && d_res && partials, "asme_linear_dx_residual_ln_bwd: null pointer");
    ASME_CHECK_ARG(in_f == kBN, "asme_linear_dx_residual_ln_bwd: in_features must be 128");
    ASME_CHECK_ARG(shapes_ok(dy, ld_dy, w, in_f, (int)out_f, (int)in_f), "asme_linear_dx_residual_ln_bwd: bad strides");
    if (n_rows == 0) return 0;
    EpiArgs ep{};
    ep.s_in = s;
    ep.stats_in = stats;
    ep.ln_w = ln_w;
    ep.d_in = d_in;
    ep.p_a = p_a;
    ep.s_a = seed_a;
    ep.p_b = p_b;
    ep.s_b = seed_b;
    ep.d_res = d_res;
    ep.d_y = d_y;
    ep.partials = partials;
    return launch_linear<true, EPI_RESLN_BWD>(dy, ld_dy, n_rows, (int)out_f, w, in_f, (int)in_f, d_res, in_f, ep,
                                              (hipStream_t)stream);
}
