// Masked multi-head self-attention for short sequences (L <= 1024, designed for L <= 200) on gfx950.
//
// Reference semantics (paths relative to /root/reference/src/asme):
//   Attention.forward            core/models/common/layers/transformer_layers.py:138-155
//       scores = QK^T / sqrt(dk); masked_fill(mask == 0, -1e9); softmax; dropout(p_attn); P V
//   MultiHeadedAttention.forward transformer_layers.py:181-199 (heads = column blocks of the projections)
//   mask construction            core/models/transformer/sequence_representation.py:34-48
//       causal:        tril(ones(L,L)) * key_padding_mask   (SASRec)
//       bidirectional: key_padding_mask                      (BERT4Rec / KeBERT4Rec)
// The (B,1,L,L) float mask of the reference is never materialised: the kernels derive it from the
// key-validity bytes and causality.  Masked scores are exactly -1e9 (not -inf), so a row with no
// admissible key reproduces the reference's uniform softmax over all L keys.
//
// Layout: Q/K/V rows are token-major with a row stride (the fused QKV projection output (T, 3*H*dk)
// is consumed in place); head h occupies columns [h*dk, (h+1)*dk).  O is (T, H*dk); the softmax row
// statistics are (B*H, L, 2) = (running max, 1 / sum of exp) per query row.
//
// Compute: fp32 MFMA v_mfma_f32_16x16x4f32 (exact f32 FMA chain).  One workgroup = 4 waves = 64 query
// rows (forward / dQ) or 64 key rows (dK/dV) of one (batch, head), 16 rows per wave; the other operand
// streams through LDS in 64-row tiles, register-prefetched one tile ahead (the global loads of tile
// i+1 are in flight while tile i is multiplied).  The softmax is flash-style (running max / sum) in
// the swapped S^T = K Q^T orientation so P^T is directly the B operand of O^T += V^T P^T.  The MFMA
// contraction index is permuted per lane group (lane group g owns feature columns g*dk/4 ..) so each
// lane's operand slice is contiguous: row chunks come from LDS as ds_read_b128, column operands as
// ds_read_b32 (LDS row stride dk+4: both patterns bank-conflict free for the 32-lane halves).
// Every 16-key sub-tile of a 64-key tile has its own accumulator, so consecutive MFMAs are independent.
#include "common.h"

using namespace asme;

namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int kQB = 64;       // rows per workgroup (4 waves x 16)
constexpr int kKT = 64;       // streamed tile rows
constexpr int kNS = kKT / 16; // 16-row sub-tiles per tile
constexpr int kMaxL = 1024;   // LDS-staged key-validity bytes
constexpr float kMaskedScore = -1e9f;
constexpr float kInitMax = -1e30f;

__device__ __forceinline__ floatx4 mfma16(float a, float b, floatx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// keep factors (0 or 1/(1-p)) for the 4 keys key4 .. key4+3 (key4 % 4 == 0) of query row `row`
__device__ __forceinline__ float4 attn_keep4(uint64_t seed, uint64_t row, int key4, float p) {
    u32x4 c{(uint32_t)(key4 >> 2), (uint32_t)row, (uint32_t)(row >> 32), 0x61747466u};
    u32x4 r = philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    const float s = 5.9604644775390625e-08f, k = 1.f / (1.f - p);
    return make_float4((float)(r.x >> 8) * s >= p ? k : 0.f, (float)(r.y >> 8) * s >= p ? k : 0.f,
                       (float)(r.z >> 8) * s >= p ? k : 0.f, (float)(r.w >> 8) * s >= p ? k : 0.f);
}
__device__ __forceinline__ float pick(const float4& v, int i) {
    return i == 0 ? v.x : (i == 1 ? v.y : (i == 2 ? v.z : v.w));
}
// The forward stores the attention-dropout decisions as one nibble per (query row, 4 keys)
// (drop_mask: (B*H*L) x ceil(L/4) bytes, bit r = key 4j+r kept); the backward passes read them instead
// of re-running Philox.
__device__ __forceinline__ uint8_t keep_bits(const float4& f) {
    return (uint8_t)((f.x != 0.f ? 1 : 0) | (f.y != 0.f ? 2 : 0) | (f.z != 0.f ? 4 : 0) | (f.w != 0.f ? 8 : 0));
}
__device__ __forceinline__ float4 bits_keep(uint8_t m, float p) {
    const float k = 1.f / (1.f - p);
    return make_float4(m & 1 ? k : 0.f, m & 2 ? k : 0.f, m & 4 ? k : 0.f, m & 8 ? k : 0.f);
}

// Stage the key-validity row of batch b in LDS; returns whether any key is valid and the last one.
__device__ __forceinline__ void stage_valid(const uint8_t* __restrict__ key_valid, int b, int L, uint8_t* kv_s,
                                            int* flag_s, bool& any_valid, int& last_valid) {
    if (threadIdx.x == 0) flag_s[0] = -1;
    __syncthreads();
    for (int i = threadIdx.x; i < L; i += blockDim.x) {
        const uint8_t v = key_valid ? key_valid[(int64_t)b * L + i] : (uint8_t)1;
        kv_s[i] = v;
        if (v) atomicMax(flag_s, i);
    }
    __syncthreads();
    last_valid = flag_s[0];
    any_valid = last_valid >= 0;
}

// register staging of a kKT x DK tile: 256 threads x N4 float4
template <int DK>
struct Stage {
    static constexpr int N4 = kKT * DK / 4 / 256;
    float4 r[N4];
    __device__ __forceinline__ void load(const float* __restrict__ base, int64_t ld, int row0, int L) {
#pragma unroll
        for (int q = 0; q < N4; ++q) {
            const int idx = threadIdx.x + 256 * q;
            const int row = idx / (DK / 4), c4 = (idx % (DK / 4)) * 4;
            r[q] = row0 + row < L ? *reinterpret_cast<const float4*>(base + (int64_t)(row0 + row) * ld + c4)
                                  : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }
    __device__ __forceinline__ void store(float* tile) const {
#pragma unroll
        for (int q = 0; q < N4; ++q) {
            const int idx = threadIdx.x + 256 * q;
            const int row = idx / (DK / 4), c4 = (idx % (DK / 4)) * 4;
            *reinterpret_cast<float4*>(tile + row * (DK + 4) + c4) = r[q];
        }
    }
};

// this lane's contiguous DQ = DK/4 features of one row, from global memory
template <int DK>
__device__ __forceinline__ void load_row_slice(const float* __restrict__ rowp, bool ok, int g, float (&f)[DK / 4]) {
#pragma unroll
    for (int s4 = 0; s4 < DK / 16; ++s4) {
        const float4 v = ok ? *reinterpret_cast<const float4*>(rowp + g * (DK / 4) + 4 * s4)
                            : make_float4(0.f, 0.f, 0.f, 0.f);
        f[4 * s4] = v.x;
        f[4 * s4 + 1] = v.y;
        f[4 * s4 + 2] = v.z;
        f[4 * s4 + 3] = v.w;
    }
}

// acc[sub] += Tile[sub*16 + c16][slice g] . f  (16 x 16 result per sub-tile, rows of the tile on C/D rows)
template <int DK>
__device__ __forceinline__ void rows_times_slice(const float* __restrict__ tile, int g, int c16,
                                                 const float (&f)[DK / 4], floatx4 (&acc)[kNS]) {
    constexpr int S = DK + 4, DQ = DK / 4;
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

// out[ct] += Tile^T[ct-th 16 columns][rows] . w  where w[sub][s] is the weight of tile row sub*16 + 4g + s
template <int DK>
__device__ __forceinline__ void cols_times_weights(const float* __restrict__ tile, int g, int c16,
                                                   const float (&w)[kNS][4], floatx4 (&out)[DK / 16]) {
    constexpr int S = DK + 4, NCT = DK / 16;
#pragma unroll
    for (int sub = 0; sub < kNS; ++sub)
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int ct = 0; ct < NCT; ++ct)
                out[ct] = mfma16(tile[(sub * 16 + 4 * g + s) * S + ct * 16 + c16], w[sub][s], out[ct]);
}

template <int DK>
__global__ __launch_bounds__(256) void attn_fwd_kernel(const float* __restrict__ q, const float* __restrict__ k,
                                                       const float* __restrict__ v, int64_t ldq, int64_t ldk,
                                                       int64_t ldv, float* __restrict__ o, int64_t ldo,
                                                       float* __restrict__ stats,
                                                       const uint8_t* __restrict__ key_valid, int H, int L,
                                                       int causal, float scale, float p_drop, uint64_t seed,
                                                       uint8_t* __restrict__ drop_mask) {
    constexpr int DQ = DK / 4, NCT = DK / 16, S = DK + 4;
    __shared__ __attribute__((aligned(16))) float Ks[kKT * S];
    __shared__ __attribute__((aligned(16))) float Vs[kKT * S];
    __shared__ uint8_t kv_s[kMaxL];
    __shared__ int flag_s[1];

    const int bh = blockIdx.y, b = bh / H, h = bh % H;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c16 = lane & 15;
    const int qblk = blockIdx.x * kQB;
    const int qi = qblk + wave * 16 + c16;  // this lane's query row (C/D column)
    const int64_t tok0 = (int64_t)b * L;

    bool any_valid;
    int last_valid;
    stage_valid(key_valid, b, L, kv_s, flag_s, any_valid, last_valid);
    int kmax = L;
    if (any_valid) {
        kmax = last_valid + 1;
        if (causal) kmax = min(kmax, min(L, qblk + kQB));
    }
    const float* qh = q + tok0 * ldq + h * DK;
    const float* kh = k + tok0 * ldk + h * DK;
    const float* vh = v + tok0 * ldv + h * DK;

    float qf[DQ];
    load_row_slice<DK>(qh + (int64_t)qi * ldq, qi < L, g, qf);
    floatx4 acc[NCT];
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) acc[ct] = floatx4{0.f, 0.f, 0.f, 0.f};
    float m = kInitMax, l = 0.f;
    const uint64_t drow = (uint64_t)bh * L + (uint64_t)min(qi, L - 1);
    const int L4 = (L + 3) / 4;
    // wave-uniform work limits: waves whose 16 queries are all past L only help stage tiles; under a
    // causal mask (and some admissible key) a 16-key sub-tile that starts after the wave's last query
    // is fully masked and contributes exactly 0, so it is skipped.
    const int wq0 = qblk + wave * 16;
    const bool wave_live = wq0 < L;
    const int wq_last = min(wq0 + 15, L - 1);
    const bool skip_causal = causal && any_valid;

    Stage<DK> sk, sv;
    const int ntiles = (kmax + kKT - 1) / kKT;
    if (ntiles > 0) {
        sk.load(kh, ldk, 0, L);
        sv.load(vh, ldv, 0, L);
    }
    for (int it = 0; it < ntiles; ++it) {
        const int k0 = it * kKT;
        __syncthreads();
        sk.store(Ks);
        sv.store(Vs);
        __syncthreads();
        if (it + 1 < ntiles) {
            sk.load(kh, ldk, k0 + kKT, L);
            sv.load(vh, ldv, k0 + kKT, L);
        }
        if (!wave_live || (skip_causal && k0 > wq_last)) continue;
        floatx4 st[kNS];
#pragma unroll
        for (int sub = 0; sub < kNS; ++sub) st[sub] = floatx4{0.f, 0.f, 0.f, 0.f};
        rows_times_slice<DK>(Ks, g, c16, qf, st);  // S^T[key][query]
        float p[kNS][4];
        float tmax = kInitMax;
#pragma unroll
        for (int sub = 0; sub < kNS; ++sub)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int key = k0 + sub * 16 + 4 * g + r;
                float sv_;
                if (key >= L) {
                    sv_ = -INFINITY;  // not a key at all
                } else {
                    const bool masked = !kv_s[key] || (causal && key > qi);
                    sv_ = masked ? kMaskedScore : st[sub][r] * scale;
                }
                p[sub][r] = sv_;
                tmax = fmaxf(tmax, sv_);
            }
        tmax = group4_max(tmax);
        const float mnew = fmaxf(m, tmax);
        const float alpha = __expf(m - mnew);
        float rs = 0.f;
#pragma unroll
        for (int sub = 0; sub < kNS; ++sub)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                p[sub][r] = __expf(p[sub][r] - mnew);
                rs += p[sub][r];
            }
        rs = group4_sum(rs);
        l = l * alpha + rs;
        m = mnew;
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct) acc[ct] *= alpha;
        if (p_drop > 0.f) {
#pragma unroll
            for (int sub = 0; sub < kNS; ++sub) {
                const int key4 = k0 + sub * 16 + 4 * g;
                const float4 f = attn_keep4(seed, drow, key4, p_drop);
                if (drop_mask && qi < L && key4 < L) drop_mask[drow * L4 + key4 / 4] = keep_bits(f);
                p[sub][0] *= f.x;
                p[sub][1] *= f.y;
                p[sub][2] *= f.z;
                p[sub][3] *= f.w;
            }
        }
        cols_times_weights<DK>(Vs, g, c16, p, acc);  // O^T += V^T P^T
    }
    if (qi < L) {
        const float inv = 1.f / l;
        float* orow = o + (tok0 + qi) * ldo + h * DK;
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct)
            *reinterpret_cast<float4*>(orow + ct * 16 + 4 * g) =
                make_float4(acc[ct][0] * inv, acc[ct][1] * inv, acc[ct][2] * inv, acc[ct][3] * inv);
        // row statistics (running max, 1/sum) rather than m + log(l): for a row with no admissible key
        // every score is -1e9 and m + log(l) would round to -1e9, losing the 1/L of the uniform softmax
        if (g == 0) {
            stats[((int64_t)bh * L + qi) * 2] = m;
            stats[((int64_t)bh * L + qi) * 2 + 1] = inv;
        }
    }
}

// dQ, plus D_i = rowsum(dO_i * O_i) for the dK/dV pass
template <int DK>
__global__ __launch_bounds__(256) void attn_bwd_dq_kernel(
    const float* __restrict__ q, const float* __restrict__ k, const float* __restrict__ v, int64_t ldq, int64_t ldk,
    int64_t ldv, const float* __restrict__ o, int64_t ldo, const float* __restrict__ dout, int64_t lddo,
    const float* __restrict__ stats, float* __restrict__ dsum, float* __restrict__ dq, int64_t lddq,
    const uint8_t* __restrict__ key_valid, int H, int L, int causal, float scale, float p_drop, uint64_t seed,
    const uint8_t* __restrict__ drop_mask) {
    constexpr int DQ = DK / 4, NCT = DK / 16, S = DK + 4;
    __shared__ __attribute__((aligned(16))) float Ks[kKT * S];
    __shared__ __attribute__((aligned(16))) float Vs[kKT * S];
    __shared__ uint8_t kv_s[kMaxL];
    __shared__ int flag_s[1];

    const int bh = blockIdx.y, b = bh / H, h = bh % H;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c16 = lane & 15;
    const int qblk = blockIdx.x * kQB;
    const int qi = qblk + wave * 16 + c16;
    const int64_t tok0 = (int64_t)b * L;

    bool any_valid;
    int last_valid;
    stage_valid(key_valid, b, L, kv_s, flag_s, any_valid, last_valid);
    int kmax = L;
    if (any_valid) {
        kmax = last_valid + 1;
        if (causal) kmax = min(kmax, min(L, qblk + kQB));
    }
    const float* kh = k + tok0 * ldk + h * DK;
    const float* vh = v + tok0 * ldv + h * DK;

    const bool qok = qi < L;
    float qf[DQ], df[DQ], of[DQ];
    load_row_slice<DK>(q + (tok0 + qi) * ldq + h * DK, qok, g, qf);
    load_row_slice<DK>(dout + (tok0 + qi) * lddo + h * DK, qok, g, df);
    load_row_slice<DK>(o + (tok0 + qi) * ldo + h * DK, qok, g, of);
    float dsv = 0.f;
#pragma unroll
    for (int s = 0; s < DQ; ++s) dsv += df[s] * of[s];
    dsv = group4_sum(dsv);  // D for query qi
    if (qok && g == 0) dsum[(int64_t)bh * L + qi] = dsv;
    const float mq = qok ? stats[((int64_t)bh * L + qi) * 2] : 0.f;
    const float iq = qok ? stats[((int64_t)bh * L + qi) * 2 + 1] : 0.f;
    const uint64_t drow = (uint64_t)bh * L + (uint64_t)min(qi, L - 1);
    const int L4 = (L + 3) / 4;
    const int wq0 = qblk + wave * 16;
    const bool wave_live = wq0 < L;
    const int wq_last = min(wq0 + 15, L - 1);
    const bool skip_causal = causal && any_valid;

    floatx4 acc[NCT];
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) acc[ct] = floatx4{0.f, 0.f, 0.f, 0.f};

    Stage<DK> sk, sv;
    const int ntiles = (kmax + kKT - 1) / kKT;
    if (ntiles > 0) {
        sk.load(kh, ldk, 0, L);
        sv.load(vh, ldv, 0, L);
    }
    for (int it = 0; it < ntiles; ++it) {
        const int k0 = it * kKT;
        __syncthreads();
        sk.store(Ks);
        sv.store(Vs);
        __syncthreads();
        if (it + 1 < ntiles) {
            sk.load(kh, ldk, k0 + kKT, L);
            sv.load(vh, ldv, k0 + kKT, L);
        }
        if (!wave_live || (skip_causal && k0 > wq_last)) continue;
        floatx4 st[kNS], dpt[kNS];
#pragma unroll
        for (int sub = 0; sub < kNS; ++sub) st[sub] = dpt[sub] = floatx4{0.f, 0.f, 0.f, 0.f};
        rows_times_slice<DK>(Ks, g, c16, qf, st);   // S^T
        rows_times_slice<DK>(Vs, g, c16, df, dpt);  // dP'^T
        float ds[kNS][4];
#pragma unroll
        for (int sub = 0; sub < kNS; ++sub) {
            float4 f = make_float4(1.f, 1.f, 1.f, 1.f);
            const int key4 = k0 + sub * 16 + 4 * g;
            if (p_drop > 0.f)
                f = drop_mask ? bits_keep(key4 < L ? drop_mask[drow * L4 + key4 / 4] : (uint8_t)0, p_drop)
                              : attn_keep4(seed, drow, key4, p_drop);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int key = k0 + sub * 16 + 4 * g + r;
                float val = 0.f;
                if (key < L && qok) {
                    const bool masked = !kv_s[key] || (causal && key > qi);
                    const float sv_ = masked ? kMaskedScore : st[sub][r] * scale;
                    const float pr = __expf(sv_ - mq) * iq;
                    val = masked ? 0.f : pr * (dpt[sub][r] * pick(f, r) - dsv);
                }
                ds[sub][r] = val;
            }
        }
        cols_times_weights<DK>(Ks, g, c16, ds, acc);  // dQ^T += K^T dS^T
    }
    if (qok) {
        float* row = dq + (tok0 + qi) * lddq + h * DK;
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct)
            *reinterpret_cast<float4*>(row + ct * 16 + 4 * g) =
                make_float4(acc[ct][0] * scale, acc[ct][1] * scale, acc[ct][2] * scale, acc[ct][3] * scale);
    }
}

template <int DK>
__global__ __launch_bounds__(256) void attn_bwd_dkdv_kernel(
    const float* __restrict__ q, const float* __restrict__ k, const float* __restrict__ v, int64_t ldq, int64_t ldk,
    int64_t ldv, const float* __restrict__ dout, int64_t lddo, const float* __restrict__ stats,
    const float* __restrict__ dsum, float* __restrict__ dk, int64_t lddk, float* __restrict__ dv, int64_t lddv,
    const uint8_t* __restrict__ key_valid, int H, int L, int causal, float scale, float p_drop, uint64_t seed,
    const uint8_t* __restrict__ drop_mask) {
    constexpr int DQ = DK / 4, NCT = DK / 16, S = DK + 4;
    __shared__ __attribute__((aligned(16))) float Qs[kKT * S];
    __shared__ __attribute__((aligned(16))) float Ds[kKT * S];
    __shared__ float mx_s[kKT], il_s[kKT], dsum_s[kKT];
    __shared__ uint8_t kv_s[kMaxL];
    __shared__ int flag_s[1];

    const int bh = blockIdx.y, b = bh / H, h = bh % H;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c16 = lane & 15;
    const int kblk = blockIdx.x * kQB;
    const int kj = kblk + wave * 16 + c16;  // this lane's key row (C/D column)
    const int64_t tok0 = (int64_t)b * L;

    bool any_valid;
    int last_valid;
    stage_valid(key_valid, b, L, kv_s, flag_s, any_valid, last_valid);
    const float* qh = q + tok0 * ldq + h * DK;
    const float* doh = dout + tok0 * lddo + h * DK;

    const bool key_ok = kj < L;
    float kf[DQ], vf[DQ];
    load_row_slice<DK>(k + (tok0 + kj) * ldk + h * DK, key_ok, g, kf);
    load_row_slice<DK>(v + (tok0 + kj) * ldv + h * DK, key_ok, g, vf);
    const bool key_masked_pad = key_ok ? !kv_s[kj] : true;

    floatx4 dvt[NCT], dkt[NCT];
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) dvt[ct] = dkt[ct] = floatx4{0.f, 0.f, 0.f, 0.f};

    const int L4 = (L + 3) / 4;
    const int wk0 = kblk + wave * 16;
    const bool wave_live = wk0 < L;
    // causal: queries before this key block see none of its keys (unless no key is valid at all)
    const int q_start = (causal && any_valid) ? kblk : 0;
    // keys of this block that no query can attend (past the last valid key) contribute nothing either
    const bool block_dead = any_valid && kblk > last_valid;
    const int ntiles = block_dead ? 0 : (L - q_start + kKT - 1) / kKT;
    Stage<DK> sq, sd;
    if (ntiles > 0) {
        sq.load(qh, ldq, q_start, L);
        sd.load(doh, lddo, q_start, L);
    }
    for (int it = 0; it < ntiles; ++it) {
        const int q0 = q_start + it * kKT;
        __syncthreads();
        sq.store(Qs);
        sd.store(Ds);
        if (threadIdx.x < kKT) {
            const int qq = q0 + threadIdx.x;
            mx_s[threadIdx.x] = qq < L ? stats[((int64_t)bh * L + qq) * 2] : 0.f;
            il_s[threadIdx.x] = qq < L ? stats[((int64_t)bh * L + qq) * 2 + 1] : 0.f;
            dsum_s[threadIdx.x] = qq < L ? dsum[(int64_t)bh * L + qq] : 0.f;
        }
        __syncthreads();
        if (it + 1 < ntiles) {
            sq.load(qh, ldq, q0 + kKT, L);
            sd.load(doh, lddo, q0 + kKT, L);
        }
        if (!wave_live) continue;
        floatx4 st[kNS], dpt[kNS];
#pragma unroll
        for (int sub = 0; sub < kNS; ++sub) st[sub] = dpt[sub] = floatx4{0.f, 0.f, 0.f, 0.f};
        rows_times_slice<DK>(Qs, g, c16, kf, st);   // S[query][key]
        rows_times_slice<DK>(Ds, g, c16, vf, dpt);  // dP'[query][key]
        float pd[kNS][4], ds[kNS][4];
#pragma unroll
        for (int sub = 0; sub < kNS; ++sub)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int ql = sub * 16 + 4 * g + r;
                const int qq = q0 + ql;
                float pv = 0.f, dsv = 0.f;
                if (qq < L && key_ok) {
                    const bool masked = key_masked_pad || (causal && kj > qq);
                    const float sv_ = masked ? kMaskedScore : st[sub][r] * scale;
                    const float pr = __expf(sv_ - mx_s[ql]) * il_s[ql];
                    float f = 1.f;
                    if (p_drop > 0.f) {
                        const uint64_t row = (uint64_t)bh * L + qq;
                        f = drop_mask ? ((drop_mask[row * L4 + kj / 4] >> (kj & 3)) & 1 ? 1.f / (1.f - p_drop) : 0.f)
                                      : pick(attn_keep4(seed, row, kj & ~3, p_drop), kj & 3);
                    }
                    pv = pr * f;
                    dsv = masked ? 0.f : pr * (dpt[sub][r] * f - dsum_s[ql]);
                }
                pd[sub][r] = pv;
                ds[sub][r] = dsv;
            }
        cols_times_weights<DK>(Ds, g, c16, pd, dvt);  // dV^T += dO^T P
        cols_times_weights<DK>(Qs, g, c16, ds, dkt);  // dK^T += Q^T dS
    }
    if (key_ok) {
        float* krow = dk + (tok0 + kj) * lddk + h * DK;
        float* vrow = dv + (tok0 + kj) * lddv + h * DK;
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct) {
            *reinterpret_cast<float4*>(krow + ct * 16 + 4 * g) =
                make_float4(dkt[ct][0] * scale, dkt[ct][1] * scale, dkt[ct][2] * scale, dkt[ct][3] * scale);
            *reinterpret_cast<float4*>(vrow + ct * 16 + 4 * g) =
                make_float4(dvt[ct][0], dvt[ct][1], dvt[ct][2], dvt[ct][3]);
        }
    }
}

#define ASME_DK_DISPATCH(DKV, ...)                                  \
    switch (DKV) {                                                  \
        case 16: { constexpr int DK = 16; __VA_ARGS__; } break;     \
        case 32: { constexpr int DK = 32; __VA_ARGS__; } break;     \
        case 64: { constexpr int DK = 64; __VA_ARGS__; } break;     \
        case 128: { constexpr int DK = 128; __VA_ARGS__; } break;   \
        default: set_error("attention head size must be 16, 32, 64 or 128"); return -1; \
    }

bool aligned16(const void* p, int64_t ld) { return ((uintptr_t)p & 15) == 0 && (ld % 4) == 0; }

}  // namespace

ASME_API int asme_attention_fwd(const float* q, const float* k, const float* v, int64_t ld_q, int64_t ld_k,
                                int64_t ld_v, const uint8_t* key_valid, int64_t batch, int64_t heads, int64_t seq_len,
                                int64_t head_dim, int causal, float scale, float p_drop, uint64_t seed, float* out,
                                int64_t ld_out, float* lse, uint8_t* drop_mask, void* stream) {
    ASME_CHECK_ARG(q && k && v && out && lse, "asme_attention_fwd: null pointer");
    ASME_CHECK_ARG(seq_len >= 1 && seq_len <= kMaxL, "asme_attention_fwd: seq_len must be in [1, 1024]");
    ASME_CHECK_ARG(p_drop >= 0.f && p_drop < 1.f, "asme_attention_fwd: dropout p must be in [0,1)");
    ASME_CHECK_ARG(aligned16(out, ld_out) && aligned16(q, ld_q) && aligned16(k, ld_k) && aligned16(v, ld_v),
                   "asme_attention_fwd: operands must be 16-B aligned with ld % 4 == 0");
    if (batch == 0) return 0;
    const dim3 grid((unsigned)((seq_len + kQB - 1) / kQB), (unsigned)(batch * heads));
    ASME_DK_DISPATCH(head_dim, hipLaunchKernelGGL(attn_fwd_kernel<DK>, grid, dim3(256), 0, (hipStream_t)stream, q, k,
                                                  v, ld_q, ld_k, ld_v, out, ld_out, lse, key_valid, (int)heads,
                                                  (int)seq_len, causal, scale, p_drop, seed, drop_mask));
    ASME_LAUNCH_CHECK("asme_attention_fwd");
}

ASME_API int asme_attention_bwd(const float* q, const float* k, const float* v, int64_t ld_q, int64_t ld_k,
                                int64_t ld_v, const float* out, int64_t ld_out, const float* dout, int64_t ld_dout,
                                const float* lse, const uint8_t* key_valid, int64_t batch, int64_t heads,
                                int64_t seq_len, int64_t head_dim, int causal, float scale, float p_drop,
                                uint64_t seed, const uint8_t* drop_mask, float* dsum_ws, float* dq, int64_t ld_dq,
                                float* dk, int64_t ld_dk, float* dv, int64_t ld_dv, void* stream) {
    ASME_CHECK_ARG(q && k && v && out && dout && lse && dsum_ws && dq && dk && dv, "asme_attention_bwd: null pointer");
    ASME_CHECK_ARG(seq_len >= 1 && seq_len <= kMaxL, "asme_attention_bwd: seq_len must be in [1, 1024]");
    ASME_CHECK_ARG(aligned16(dq, ld_dq) && aligned16(dk, ld_dk) && aligned16(dv, ld_dv) && aligned16(q, ld_q) &&
                       aligned16(k, ld_k) && aligned16(v, ld_v) && aligned16(out, ld_out) &&
                       aligned16(dout, ld_dout),
                   "asme_attention_bwd: operands must be 16-B aligned with ld % 4 == 0");
    if (batch == 0) return 0;
    hipStream_t s = (hipStream_t)stream;
    const dim3 grid((unsigned)((seq_len + kQB - 1) / kQB), (unsigned)(batch * heads));
    ASME_DK_DISPATCH(
        head_dim,
        hipLaunchKernelGGL(attn_bwd_dq_kernel<DK>, grid, dim3(256), 0, s, q, k, v, ld_q, ld_k, ld_v, out, ld_out, dout,
                           ld_dout, lse, dsum_ws, dq, ld_dq, key_valid, (int)heads, (int)seq_len, causal, scale,
                           p_drop, seed, drop_mask);
        hipLaunchKernelGGL(attn_bwd_dkdv_kernel<DK>, grid, dim3(256), 0, s, q, k, v, ld_q, ld_k, ld_v, dout,
                           ld_dout, lse, dsum_ws, dk, ld_dk, dv, ld_dv, key_valid, (int)heads, (int)seq_len, causal,
                           scale, p_drop, seed, drop_mask));
    ASME_LAUNCH_CHECK("asme_attention_bwd");
}
