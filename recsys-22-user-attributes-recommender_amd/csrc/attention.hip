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
#include <type_traits>

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

// Attention dropout decisions.  One Philox4x32-10 block serves 8 (query row, key) pairs: the block of
// (row, key/32, (key/4)%4) yields 8 16-bit uniforms, word r / half h deciding key 32*(key/32) + 16*h +
// 4*((key/4)%4) + r, so a lane holding keys 4g..4g+3 of two adjacent 16-key sub-tiles needs one block.
// Key kept iff uniform16 >= round(p * 65536) (keep probability within 2^-16 of 1-p), scaled by 1/(1-p).
__device__ __forceinline__ u32x4 attn_philox(uint64_t seed, uint64_t row, int key) {
    u32x4 c{(uint32_t)(((key >> 5) << 2) | ((key >> 2) & 3)), (uint32_t)row, (uint32_t)(row >> 32), 0x61747466u};
    return philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
}
__device__ __forceinline__ uint32_t drop_threshold(float p) { return (uint32_t)(p * 65536.f + 0.5f); }
__device__ __forceinline__ float4 keep_from(const u32x4& r, int half, uint32_t thr, float k) {
    const int sh = half ? 16 : 0;
    return make_float4(((r.x >> sh) & 0xFFFFu) >= thr ? k : 0.f, ((r.y >> sh) & 0xFFFFu) >= thr ? k : 0.f,
                       ((r.z >> sh) & 0xFFFFu) >= thr ? k : 0.f, ((r.w >> sh) & 0xFFFFu) >= thr ? k : 0.f);
}
// keep factors (0 or 1/(1-p)) for the 4 keys key4 .. key4+3 (key4 % 4 == 0) of query row `row`
__device__ __forceinline__ float4 attn_keep4(uint64_t seed, uint64_t row, int key4, float p) {
    return keep_from(attn_philox(seed, row, key4), (key4 >> 4) & 1, drop_threshold(p), 1.f / (1.f - p));
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
    return make_float4(keep_factor_bit(m, 0, k), keep_factor_bit(m, 1, k), keep_factor_bit(m, 2, k),
                       keep_factor_bit(m, 3, k));
}
// A second copy serves the dK/dV pass, whose lanes own keys: u16 words [B*H][ceil(L/16) query groups]
// [4*ceil(L/4) keys], bit i of word (j, key) = query 16j+i kept.  It follows the nibble image, 256-B aligned.
__host__ __device__ inline int64_t mask_nibble_bytes(int64_t bh, int L) { return bh * L * ((L + 3) / 4); }
__host__ __device__ inline int mask_key_stride(int L) { return 4 * ((L + 3) / 4); }
__host__ __device__ inline int64_t mask_tag_offset(int64_t bh, int L) {
    return (((mask_nibble_bytes(bh, L) + 255) & ~(int64_t)255) + bh * ((L + 15) / 16) * mask_key_stride(L) * 2 + 255) &
           ~(int64_t)255;
}
// + a 16-B tag after the key-major words: the forward records whether it stored the query-major nibbles
// (kMaskTagNib) or skipped them because the family-0 backward reads only the key words and the stored dS
// (kMaskTagNoNib); the nibble-reading dQ passes check it and write NaN instead of a dQ from unwritten bits
__host__ __device__ inline int64_t mask_total_bytes(int64_t bh, int L) { return mask_tag_offset(bh, L) + 16; }
constexpr uint32_t kMaskTagNib = 0x3142494Eu, kMaskTagNoNib = 0x3042494Eu;
__device__ __forceinline__ void mask_tag_write(uint8_t* m, int64_t bh_total, int L, bool with_nib) {
    *reinterpret_cast<uint32_t*>(m + mask_tag_offset(bh_total, L)) = with_nib ? kMaskTagNib : kMaskTagNoNib;
}
// the factor a nibble-reading dQ pass scales its output by: `scale`, or NaN when the forward skipped the nibbles
__device__ __forceinline__ float dq_out_scale(const uint8_t* m, int64_t bh_total, int L, float p_drop, float scale) {
    if (!m || !(p_drop > 0.f)) return scale;
    const uint32_t tag = *reinterpret_cast<const uint32_t*>(m + mask_tag_offset(bh_total, L));
    return tag == kMaskTagNib ? scale : __builtin_nanf("");
}
__device__ __forceinline__ uint16_t* mask_keys(uint8_t* m, int64_t bh_total, int L) {
    return reinterpret_cast<uint16_t*>(m + ((mask_nibble_bytes(bh_total, L) + 255) & ~(int64_t)255));
}
// Forward-side store of one 16-key sub-tile's decisions (lane: query row c16 of group q0/16, keys
// key4..key4+3 with key4 = ks + 4g): the nibble for the dQ pass, and via ballots the key-major words
// (one 8-byte store of 4 keys' words per lane group).
__device__ __forceinline__ void store_drop_bits(uint8_t* __restrict__ nib, uint16_t* __restrict__ keyw, int bh,
                                                int L, int qi, int q0, int ks, int g, int c16, const float4& f,
                                                bool with_nib = true) {
    const int L4 = (L + 3) / 4;
    const int key4 = ks + 4 * g;
    if (with_nib && qi < L && key4 < L) nib[((int64_t)bh * L + qi) * L4 + key4 / 4] = keep_bits(f);
    // bit 16g + c16 of each ballot: (key ks+4g+r, query q0+c16)
    const uint64_t b0 = __ballot(f.x != 0.f), b1 = __ballot(f.y != 0.f), b2 = __ballot(f.z != 0.f),
                   b3 = __ballot(f.w != 0.f);
    if (c16 == 0 && key4 < L) {
        const int sh = 16 * g;
        const uint64_t w = ((b0 >> sh) & 0xFFFFull) | (((b1 >> sh) & 0xFFFFull) << 16) |
                           (((b2 >> sh) & 0xFFFFull) << 32) | (((b3 >> sh) & 0xFFFFull) << 48);
        *reinterpret_cast<uint64_t*>(keyw + ((int64_t)bh * ((L + 15) / 16) + q0 / 16) * mask_key_stride(L) + key4) = w;
    }
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

// the sliced image of a tile (rows_times_slice<..., SL = true>): element (r, c) at (c / DQ) * sl + r * (DQ + 4) + c % DQ,
// sl = the slice stride (a multiple of 64 floats)
__host__ __device__ inline int sliced_stride(int Lp, int DK) { return (Lp * (DK / 4 + 4) + 63) & ~63; }
__device__ __forceinline__ int sliced_off(int r, int c, int DQ, int sl) { return (c / DQ) * sl + r * (DQ + 4) + c % DQ; }

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

struct NoFill {
    __device__ __forceinline__ void operator()(int) const {}
};
// acc[sub] += Tile[sub*16 + c16][slice g] . f  (16 x 16 result per sub-tile, rows of the tile on C/D rows).
// fill(s4) runs after step s4's MFMAs are issued, in the same scheduling region: independent vector work of the
// caller that issues in the shadow of this wave's MFMAs.
template <int DK, int NS = kNS, class F = NoFill, bool SL = false>
__device__ __forceinline__ void rows_times_slice(const float* __restrict__ tile, int g, int c16,
                                                 const float (&f)[DK / 4], floatx4 (&acc)[NS], F&& fill = F{},
                                                 int sl = 0) {
    // SL: the tile in the sliced layout (sliced_off): row stride DQ + 4 within each of the 4 column slices, slices
    // sl floats apart (sl % 64 == 0) -- a lane's b128 read lands at bank chunk 5 r + const (DK = 64), so the 16 lanes
    // of each b128 lane group hit 16 distinct chunks (the padded row-major image, stride DK + 4, puts two lanes on
    // one chunk in half the groups: ~1 extra LDS cycle per read)
    constexpr int S = SL ? DK / 4 + 4 : DK + 4, DQ = DK / 4;
    // the b128 row reads of step s4+1 are issued before step s4's MFMAs (LDS latency off the MFMA stream)
    float4 ab[2][NS];
    const float* base = tile + c16 * S + g * (SL ? sl : DQ);
#pragma unroll
    for (int sub = 0; sub < NS; ++sub) ab[0][sub] = *reinterpret_cast<const float4*>(base + sub * 16 * S);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s4 = 0; s4 < DQ / 4; ++s4) {
        if (s4 + 1 < DQ / 4) {
#pragma unroll
            for (int sub = 0; sub < NS; ++sub)
                ab[(s4 + 1) & 1][sub] = *reinterpret_cast<const float4*>(base + sub * 16 * S + 4 * (s4 + 1));
        }
        __builtin_amdgcn_sched_barrier(0);
        const float4(&a)[NS] = ab[s4 & 1];
#pragma unroll
        for (int sub = 0; sub < NS; ++sub) acc[sub] = mfma16(a[sub].x, f[4 * s4], acc[sub]);
#pragma unroll
        for (int sub = 0; sub < NS; ++sub) acc[sub] = mfma16(a[sub].y, f[4 * s4 + 1], acc[sub]);
#pragma unroll
        for (int sub = 0; sub < NS; ++sub) acc[sub] = mfma16(a[sub].z, f[4 * s4 + 2], acc[sub]);
#pragma unroll
        for (int sub = 0; sub < NS; ++sub) acc[sub] = mfma16(a[sub].w, f[4 * s4 + 3], acc[sub]);
        fill(s4);
    }
}

// out[ct] += Tile^T[ct-th 16 columns][rows] . w  where w[sub][s] is the weight of tile row sub*16 + 4g + s
template <int DK, int NS = kNS>
__device__ __forceinline__ void cols_times_weights(const float* __restrict__ tile, int g, int c16,
                                                   const float (&w)[NS][4], floatx4 (&out)[DK / 16]) {
    constexpr int S = DK + 4, NCT = DK / 16;
    // the operands of sub-tile sub+1 are read while sub's MFMAs run: the b32 column reads would otherwise
    // expose their LDS latency before every pair of MFMAs
    float vb[2][4][NCT];
    const float* base = tile + 4 * g * S + c16;
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct) vb[0][s][ct] = base[s * S + ct * 16];
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int sub = 0; sub < NS; ++sub) {
        if (sub + 1 < NS) {
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int ct = 0; ct < NCT; ++ct) vb[(sub + 1) & 1][s][ct] = base[((sub + 1) * 16 + s) * S + ct * 16];
        }
        __builtin_amdgcn_sched_barrier(0);  // keep the prefetch ahead of this sub-tile's MFMAs
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int ct = 0; ct < NCT; ++ct) out[ct] = mfma16(vb[sub & 1][s][ct], w[sub][s], out[ct]);
    }
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
    if (drop_mask && p_drop > 0.f && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0)
        mask_tag_write(drop_mask, gridDim.y, L, true);

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
            const uint32_t thr = drop_threshold(p_drop);
            const float kf = 1.f / (1.f - p_drop);
            uint16_t* keyw = drop_mask ? mask_keys(drop_mask, (int64_t)gridDim.y, L) : nullptr;
            u32x4 rnd;
#pragma unroll
            for (int sub = 0; sub < kNS; ++sub) {
                const int key4 = k0 + sub * 16 + 4 * g;
                if ((sub & 1) == 0) rnd = attn_philox(seed, drow, key4);  // k0 % 64 == 0: pairs share a block
                const float4 f = keep_from(rnd, sub & 1, thr, kf);
                if (drop_mask) store_drop_bits(drop_mask, keyw, bh, L, qi, wq0, k0 + sub * 16, g, c16, f);
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
        const float os = dq_out_scale(drop_mask, gridDim.y, L, p_drop, scale);
        float* row = dq + (tok0 + qi) * lddq + h * DK;
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct)
            *reinterpret_cast<float4*>(row + ct * 16 + 4 * g) =
                make_float4(acc[ct][0] * os, acc[ct][1] * os, acc[ct][2] * os, acc[ct][3] * os);
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

    const int wk0 = kblk + wave * 16;
    // key-major dropout words of this lane's key: group j at keyw_key[j * mask_key_stride(L)]
    const uint16_t* keyw_key = drop_mask ? mask_keys(const_cast<uint8_t*>(drop_mask), (int64_t)gridDim.y, L) +
                                               (int64_t)bh * ((L + 15) / 16) * mask_key_stride(L) + min(kj, L - 1)
                                         : nullptr;
    const int kstride = mask_key_stride(L);
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
                        f = drop_mask ? ((keyw_key[(qq >> 4) * kstride] >> (qq & 15)) & 1 ? 1.f / (1.f - p_drop) : 0.f)
                                      : pick(attn_keep4(seed, (uint64_t)bh * L + qq, kj & ~3, p_drop), kj & 3);
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

// ==================================================================================================
// Resident variants: one 8-wave workgroup per (batch, head) keeps the whole streamed operand pair of
// that head in LDS (K,V for the forward / dQ pass; Q,dO plus the per-query statistics for dK/dV) and
// the waves claim 16-row groups from an LDS counter, most expensive first under a causal mask.  No
// per-tile barriers, each K/V row is read from HBM once per head (not once per 64-query block), and
// fully-masked 16-key sub-tiles are skipped.  Used when 2 * ceil(L/16)*16 * (dk+4) * 4 B fits the
// 160 KiB LDS (L <= 300 at dk = 64); the streaming kernels above cover the rest.
#ifndef ASME_ATTN_DIAG
#define ASME_ATTN_DIAG 0  // diagnostic builds only: 1 = the resident kernels skip their per-head operand loads,
                          // 2 = the dK/dV pass skips its dS stores (the dQ pass reads stale dS: timing only)
#endif
#ifndef ASME_RES_THREADS
#define ASME_RES_THREADS 768  // 12 waves: 3 per SIMD (512: 245/605 us fwd/bwd, 768: 231/588)
#endif
constexpr int kResThreads = ASME_RES_THREADS;  // forward and dQ passes
constexpr int kResThreadsKV = 512;             // dK/dV pass: 168+ VGPRs, 12 waves would spill

__host__ __device__ inline int res_rows(int L) { return (L + 15) & ~15; }
#ifndef ASME_ATTN_SLICED
#define ASME_ATTN_SLICED 1  // the resident forward keeps K in the sliced image (conflict-free b128 row reads)
#endif
inline size_t res_lds_bytes(int L, int DK, bool with_stats, bool k_sliced = false) {
    const size_t Lp = (size_t)res_rows(L);
    const size_t kimg = k_sliced ? (size_t)4 * sliced_stride((int)Lp, DK) : Lp * (DK + 4);
    return (kimg + Lp * (DK + 4)) * sizeof(float) + (with_stats ? 3 * Lp * sizeof(float) : 0) + (Lp + 31) / 32 * 4 + 16;
}

// rows [0, Lp) of two (L x DK) operands into padded LDS images (rows >= L zeroed); 8 float4 in flight
template <int DK, int NT = kResThreads, bool A_SL = false>
__device__ __forceinline__ void load_pair_resident(const float* __restrict__ a, int64_t lda,
                                                   const float* __restrict__ b, int64_t ldb, int L, int Lp,
                                                   float* __restrict__ As, float* __restrict__ Bs) {
    constexpr int C4 = DK / 4, S = DK + 4;
    const int asl = A_SL ? sliced_stride(Lp, DK) : 0;
    const int n4 = Lp * C4;
    // all loads of a batch are issued before the first store: at L = 200, dk = 64 one batch covers the head
    for (int base = threadIdx.x; base < n4; base += NT * 8) {
        float4 ra[8], rb[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int idx = base + u * NT, row = idx / C4, c = (idx % C4) * 4;
            const bool ok = idx < n4 && row < L;
            ra[u] = ok ? *reinterpret_cast<const float4*>(a + (int64_t)row * lda + c) : make_float4(0.f, 0.f, 0.f, 0.f);
            rb[u] = ok ? *reinterpret_cast<const float4*>(b + (int64_t)row * ldb + c) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int idx = base + u * NT, row = idx / C4, c = (idx % C4) * 4;
            if (idx < n4) {
                *reinterpret_cast<float4*>(As + (A_SL ? sliced_off(row, c, DK / 4, asl) : row * S + c)) = ra[u];
                *reinterpret_cast<float4*>(Bs + row * S + c) = rb[u];
            }
        }
    }
}

// key-validity bits (kvw: bit i of word i/32) + (last valid key, work counter) control words
__device__ __forceinline__ void stage_valid_res(const uint8_t* __restrict__ key_valid, int b, int L, int Lp,
                                                uint32_t* kvw, int* ctl) {
    if (threadIdx.x == 0) {
        ctl[0] = -1;
        ctl[1] = 0;
    }
    for (int w = threadIdx.x; w < (Lp + 31) / 32; w += blockDim.x) kvw[w] = 0u;
    __syncthreads();
    for (int i = threadIdx.x; i < L; i += blockDim.x) {
        const bool v = key_valid ? key_valid[(int64_t)b * L + i] != 0 : true;
        if (v) {
            atomicOr(kvw + (i >> 5), 1u << (i & 31));
            atomicMax(ctl, i);
        }
    }
}
// this lane's 4 validity bits for keys ks + 4g .. +3 (ks % 16 == 0)
__device__ __forceinline__ uint32_t valid_bits4(const uint32_t* kvw, int ks, int g) {
    return (kvw[ks >> 5] >> ((ks & 16) + 4 * g)) & 0xFu;
}

// wave-uniform: every key of [k0, k0+n) exists, is valid and (causal) precedes every query >= q0
__device__ __forceinline__ bool chunk_unmasked(const uint32_t* kvw, int k0, int n, int L, int causal, int q0) {
    if (k0 + n > L || (causal && k0 + n - 1 > q0)) return false;
    bool ok = true;
    for (int ks = k0; ks < k0 + n; ks += 16) {
        const uint32_t w = __builtin_amdgcn_readfirstlane(kvw[ks >> 5]);
        ok = ok && ((w >> (ks & 16)) & 0xFFFFu) == 0xFFFFu;
    }
    return ok;
}

__device__ __forceinline__ int claim_group(int* ctl, int lane) {
    int gi = 0;
    if (lane == 0) gi = atomicAdd(ctl + 1, 1);
    return __builtin_amdgcn_readfirstlane(__shfl(gi, 0, 64));
}

template <int DK>
__global__ __launch_bounds__(kResThreads) void attn_fwd_res_kernel(
    const float* __restrict__ q, const float* __restrict__ k, const float* __restrict__ v, int64_t ldq, int64_t ldk,
    int64_t ldv, float* __restrict__ o, int64_t ldo, float* __restrict__ stats, const uint8_t* __restrict__ key_valid,
    int H, int L, int causal, float scale, float p_drop, uint64_t seed, uint8_t* __restrict__ drop_mask,
    int with_nib) {
    constexpr int DQ = DK / 4, NCT = DK / 16, S = DK + 4;
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int Lp = res_rows(L);
    constexpr bool KSL = ASME_ATTN_SLICED;  // K in the sliced image (rows_times_slice's conflict-free row reads)
    const int ksl = KSL ? sliced_stride(Lp, DK) : 0;
    float* Ks = lds;
    float* Vs = Ks + (KSL ? 4 * ksl : Lp * S);
    uint32_t* kvw = reinterpret_cast<uint32_t*>(Vs + Lp * S);
    int* ctl = reinterpret_cast<int*>(kvw + (Lp + 31) / 32);

    const int bh = blockIdx.x, b = bh / H, h = bh % H;
    const int lane = threadIdx.x & 63, g = lane >> 4, c16 = lane & 15;
    const int64_t tok0 = (int64_t)b * L;
    const float* qh = q + tok0 * ldq + h * DK;
    if (drop_mask && p_drop > 0.f && blockIdx.x == 0 && threadIdx.x == 0)
        mask_tag_write(drop_mask, gridDim.x, L, with_nib != 0);

    stage_valid_res(key_valid, b, L, Lp, kvw, ctl);
    if (ASME_ATTN_DIAG != 1)
        load_pair_resident<DK, kResThreads, KSL>(k + tok0 * ldk + h * DK, ldk, v + tok0 * ldv + h * DK, ldv, L, Lp, Ks,
                                                 Vs);
    __syncthreads();
    const int last_valid = ctl[0];
    const bool any_valid = last_valid >= 0;
    const int kend = any_valid ? last_valid + 1 : L;
    const int ngroups = Lp / 16;
    uint16_t* keyw = drop_mask ? mask_keys(drop_mask, (int64_t)gridDim.x, L) : nullptr;

    for (;;) {
        const int gi = claim_group(ctl, lane);
        if (gi >= ngroups) break;
        const int q0 = (causal ? ngroups - 1 - gi : gi) * 16;
        const int qi = q0 + c16;
        // keys past kmax are masked for all 16 queries (and some key is admissible): exact zeros
        const int kmax = (causal && any_valid) ? min(kend, q0 + 16) : kend;
        const int nsub = (kmax + 15) / 16;
        float qf[DQ];
        load_row_slice<DK>(qh + (int64_t)qi * ldq, qi < L, g, qf);
        floatx4 acc[NCT];
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct) acc[ct] = floatx4{0.f, 0.f, 0.f, 0.f};
        float m = kInitMax, l = 0.f;
        const uint64_t drow = (uint64_t)bh * L + (uint64_t)min(qi, L - 1);
        // a chunk of NS 16-key sub-tiles starting at key k0 (online softmax across chunks)
        auto chunk = [&](auto ns_tag, int k0) {
            constexpr int NS = decltype(ns_tag)::value;
            floatx4 st[NS];
#pragma unroll
            for (int sub = 0; sub < NS; ++sub) st[sub] = floatx4{0.f, 0.f, 0.f, 0.f};
            rows_times_slice<DK, NS, NoFill, KSL>(Ks + k0 * (KSL ? DQ + 4 : S), g, c16, qf, st, NoFill{}, ksl);
            float p[NS][4];
            float tmax = kInitMax;
            if (chunk_unmasked(kvw, k0, NS * 16, L, causal, q0)) {
#pragma unroll
                for (int sub = 0; sub < NS; ++sub)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        p[sub][r] = st[sub][r] * scale;
                        tmax = fmaxf(tmax, p[sub][r]);
                    }
            } else {
#pragma unroll
                for (int sub = 0; sub < NS; ++sub) {
                    const uint32_t vb = valid_bits4(kvw, k0 + sub * 16, g);
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int key = k0 + sub * 16 + 4 * g + r;
                        float sv_ = -INFINITY;  // not a key: contributes nothing
                        if (key < L) {
                            const bool masked = !((vb >> r) & 1u) || (causal && key > qi);
                            sv_ = masked ? kMaskedScore : st[sub][r] * scale;
                        }
                        p[sub][r] = sv_;
                        tmax = fmaxf(tmax, sv_);
                    }
                }
            }
            tmax = group4_max(tmax);
            const float mnew = fmaxf(m, tmax);
            const float alpha = __expf(m - mnew);
            float rs = 0.f;
#pragma unroll
            for (int sub = 0; sub < NS; ++sub)
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
                const uint32_t thr = drop_threshold(p_drop);
                const float kf = 1.f / (1.f - p_drop);
                u32x4 rnd;
#pragma unroll
                for (int sub = 0; sub < NS; ++sub) {
                    const int key4 = k0 + sub * 16 + 4 * g;
                    // NS == 4 chunks start at multiples of 64 keys, so sub-tile pairs share a block
                    if (NS == 1 || (sub & 1) == 0) rnd = attn_philox(seed, drow, key4);
                    const float4 f = keep_from(rnd, (key4 >> 4) & 1, thr, kf);
                    if (drop_mask) store_drop_bits(drop_mask, keyw, bh, L, qi, q0, k0 + sub * 16, g, c16, f, with_nib);
                    p[sub][0] *= f.x;
                    p[sub][1] *= f.y;
                    p[sub][2] *= f.z;
                    p[sub][3] *= f.w;
                }
            }
            cols_times_weights<DK, NS>(Vs + k0 * S, g, c16, p, acc);
        };
        // keys >= nsub*16 are beyond kmax: no sub-tile past it is computed
        int c0 = 0;
        for (; c0 + kNS <= nsub; c0 += kNS) chunk(std::integral_constant<int, kNS>{}, c0 * 16);
        for (; c0 < nsub; ++c0) chunk(std::integral_constant<int, 1>{}, c0 * 16);
        if (qi < L) {
            const float inv = 1.f / l;
            float* orow = o + (tok0 + qi) * ldo + h * DK;
#pragma unroll
            for (int ct = 0; ct < NCT; ++ct)
                *reinterpret_cast<float4*>(orow + ct * 16 + 4 * g) =
                    make_float4(acc[ct][0] * inv, acc[ct][1] * inv, acc[ct][2] * inv, acc[ct][3] * inv);
            if (g == 0) {
                stats[((int64_t)bh * L + qi) * 2] = m;
                stats[((int64_t)bh * L + qi) * 2 + 1] = inv;
            }
        }
    }
}

template <int DK>
__global__ __launch_bounds__(kResThreads) void attn_bwd_dq_res_kernel(
    const float* __restrict__ q, const float* __restrict__ k, const float* __restrict__ v, int64_t ldq, int64_t ldk,
    int64_t ldv, const float* __restrict__ o, int64_t ldo, const float* __restrict__ dout, int64_t lddo,
    const float* __restrict__ stats, float* __restrict__ dsum, float* __restrict__ dq, int64_t lddq,
    const uint8_t* __restrict__ key_valid, int H, int L, int causal, float scale, float p_drop, uint64_t seed,
    const uint8_t* __restrict__ drop_mask) {
    constexpr int DQ = DK / 4, NCT = DK / 16, S = DK + 4;
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int Lp = res_rows(L);
    float* Ks = lds;
    float* Vs = Ks + Lp * S;
    uint32_t* kvw = reinterpret_cast<uint32_t*>(Vs + Lp * S);
    int* ctl = reinterpret_cast<int*>(kvw + (Lp + 31) / 32);

    const int bh = blockIdx.x, b = bh / H, h = bh % H;
    const int lane = threadIdx.x & 63, g = lane >> 4, c16 = lane & 15;
    const int64_t tok0 = (int64_t)b * L;

    stage_valid_res(key_valid, b, L, Lp, kvw, ctl);
    if (ASME_ATTN_DIAG != 1)
        load_pair_resident<DK>(k + tok0 * ldk + h * DK, ldk, v + tok0 * ldv + h * DK, ldv, L, Lp, Ks, Vs);
    __syncthreads();
    const int last_valid = ctl[0];
    const bool any_valid = last_valid >= 0;
    const int kend = any_valid ? last_valid + 1 : L;
    const int ngroups = Lp / 16;
    const int L4 = (L + 3) / 4;

    for (;;) {
        const int gi = claim_group(ctl, lane);
        if (gi >= ngroups) break;
        const int q0 = (causal ? ngroups - 1 - gi : gi) * 16;
        const int qi = q0 + c16;
        const bool qok = qi < L;
        const int kmax = (causal && any_valid) ? min(kend, q0 + 16) : kend;
        const int nsub = (kmax + 15) / 16;
        float qf[DQ], df[DQ], of[DQ];
        load_row_slice<DK>(q + (tok0 + qi) * ldq + h * DK, qok, g, qf);
        load_row_slice<DK>(dout + (tok0 + qi) * lddo + h * DK, qok, g, df);
        load_row_slice<DK>(o + (tok0 + qi) * ldo + h * DK, qok, g, of);
        float dsv = 0.f;
#pragma unroll
        for (int s = 0; s < DQ; ++s) dsv += df[s] * of[s];
        dsv = group4_sum(dsv);
        if (qok && g == 0) dsum[(int64_t)bh * L + qi] = dsv;
        const float mq = qok ? stats[((int64_t)bh * L + qi) * 2] : 0.f;
        const float iq = qok ? stats[((int64_t)bh * L + qi) * 2 + 1] : 0.f;
        const uint64_t drow = (uint64_t)bh * L + (uint64_t)min(qi, L - 1);
        floatx4 acc[NCT];
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct) acc[ct] = floatx4{0.f, 0.f, 0.f, 0.f};
        auto chunk = [&](auto ns_tag, int k0) {
            constexpr int NS = decltype(ns_tag)::value;
            floatx4 st[NS], dpt[NS];
            // the chunk's stored dropout decisions are requested before its MFMAs (their latency hides there)
            uint32_t mb[NS];
#pragma unroll
            for (int sub = 0; sub < NS; ++sub) {
                const int key4 = k0 + sub * 16 + 4 * g;
                mb[sub] = (p_drop > 0.f && drop_mask && key4 < L) ? drop_mask[drow * L4 + key4 / 4] : 0u;
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int sub = 0; sub < NS; ++sub) st[sub] = dpt[sub] = floatx4{0.f, 0.f, 0.f, 0.f};
            rows_times_slice<DK, NS>(Ks + k0 * S, g, c16, qf, st);
            rows_times_slice<DK, NS>(Vs + k0 * S, g, c16, df, dpt);
            float ds[NS][4];
#pragma unroll
            for (int sub = 0; sub < NS; ++sub) {
                float4 f = make_float4(1.f, 1.f, 1.f, 1.f);
                const int key4 = k0 + sub * 16 + 4 * g;
                if (p_drop > 0.f)
                    f = drop_mask ? bits_keep((uint8_t)mb[sub], p_drop) : attn_keep4(seed, drow, key4, p_drop);
                const uint32_t vb = valid_bits4(kvw, k0 + sub * 16, g);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int key = key4 + r;
                    float val = 0.f;
                    if (key < L && qok) {
                        const bool masked = !((vb >> r) & 1u) || (causal && key > qi);
                        const float sv_ = masked ? kMaskedScore : st[sub][r] * scale;
                        const float pr = __expf(sv_ - mq) * iq;
                        val = masked ? 0.f : pr * (dpt[sub][r] * pick(f, r) - dsv);
                    }
                    ds[sub][r] = val;
                }
            }
            cols_times_weights<DK, NS>(Ks + k0 * S, g, c16, ds, acc);
        };
        int c0 = 0;
        for (; c0 + kNS <= nsub; c0 += kNS) chunk(std::integral_constant<int, kNS>{}, c0 * 16);
        for (; c0 < nsub; ++c0) chunk(std::integral_constant<int, 1>{}, c0 * 16);
        if (qok) {
            const float os = dq_out_scale(drop_mask, gridDim.x, L, p_drop, scale);
            float* row = dq + (tok0 + qi) * lddq + h * DK;
#pragma unroll
            for (int ct = 0; ct < NCT; ++ct)
                *reinterpret_cast<float4*>(row + ct * 16 + 4 * g) =
                    make_float4(acc[ct][0] * os, acc[ct][1] * os, acc[ct][2] * os, acc[ct][3] * os);
        }
    }
}

// DS = true (the default path): this pass runs FIRST, computes D_i = rowsum(dO_i * O_i) itself and stores every
// dS value it forms (query-major, (B*H) x Lp x Lp) for the dQ pass (attn_bwd_dq_ds_kernel), which then needs one
// product (dQ = dS K) instead of recomputing S and dP.  DS = false: D_i comes from attn_bwd_dq_res_kernel.
template <int DK, bool DS>
__global__ __launch_bounds__(kResThreadsKV) void attn_bwd_dkdv_res_kernel(
    const float* __restrict__ q, const float* __restrict__ k, const float* __restrict__ v, int64_t ldq, int64_t ldk,
    int64_t ldv, const float* __restrict__ dout, int64_t lddo, const float* __restrict__ stats,
    const float* __restrict__ dsum, float* __restrict__ dk, int64_t lddk, float* __restrict__ dv, int64_t lddv,
    const uint8_t* __restrict__ key_valid, int H, int L, int causal, float scale, float p_drop, uint64_t seed,
    const uint8_t* __restrict__ drop_mask, const float* __restrict__ o, int64_t ldo, float* __restrict__ ds_out) {
    constexpr int DQ = DK / 4, NCT = DK / 16, S = DK + 4;
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int Lp = res_rows(L);
    float* Qs = lds;
    float* Ds = Qs + Lp * S;
    float* mx_s = Ds + Lp * S;
    float* il_s = mx_s + Lp;
    float* dsum_s = il_s + Lp;
    uint32_t* kvw = reinterpret_cast<uint32_t*>(dsum_s + Lp);
    int* ctl = reinterpret_cast<int*>(kvw + (Lp + 31) / 32);

    const int bh = blockIdx.x, b = bh / H, h = bh % H;
    const int lane = threadIdx.x & 63, g = lane >> 4, c16 = lane & 15;
    const int64_t tok0 = (int64_t)b * L;

    stage_valid_res(key_valid, b, L, Lp, kvw, ctl);
    if (ASME_ATTN_DIAG != 1)
        load_pair_resident<DK, kResThreadsKV>(q + tok0 * ldq + h * DK, ldq, dout + tok0 * lddo + h * DK, lddo, L, Lp,
                                              Qs, Ds);
    for (int i = threadIdx.x; i < Lp; i += kResThreadsKV) {
        const bool ok = i < L;
        mx_s[i] = ok ? stats[((int64_t)bh * L + i) * 2] : 0.f;
        il_s[i] = ok ? stats[((int64_t)bh * L + i) * 2 + 1] : 0.f;
        if (!DS) dsum_s[i] = ok ? dsum[(int64_t)bh * L + i] : 0.f;
    }
    __syncthreads();
    if (DS && ASME_ATTN_DIAG != 1) {
        // D_i = dO_i . O_i: 16 lanes per query row (a float4 of features each, dO from the LDS image); a thread's
        // O loads for four rows are all issued before the first is used (one round trip per four rows: a dependent
        // load per row cost ~2 us each in this prologue, which nothing overlaps at one workgroup per CU)
        constexpr int kRowStep = kResThreadsKV / 16, kU = 4, FC = (DK + 63) / 64;
        const int c = 4 * (threadIdx.x & 15);
        for (int i0 = threadIdx.x >> 4; i0 < Lp; i0 += kRowStep * kU) {
            float4 ov[kU][FC];
#pragma unroll
            for (int u = 0; u < kU; ++u)
#pragma unroll
                for (int f = 0; f < FC; ++f) {
                    const int i = i0 + u * kRowStep, cc = c + 64 * f;
                    ov[u][f] = (i < L && cc < DK) ? *reinterpret_cast<const float4*>(o + (tok0 + i) * ldo + h * DK + cc)
                                                  : make_float4(0.f, 0.f, 0.f, 0.f);
                }
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                const int i = i0 + u * kRowStep;
                float acc = 0.f;
#pragma unroll
                for (int f = 0; f < FC; ++f) {
                    const int cc = c + 64 * f;
                    if (i < Lp && cc < DK) {
                        const float4 a = *reinterpret_cast<const float4*>(Ds + i * S + cc);
                        acc += a.x * ov[u][f].x + a.y * ov[u][f].y + a.z * ov[u][f].z + a.w * ov[u][f].w;
                    }
                }
#pragma unroll
                for (int off = 8; off >= 1; off >>= 1) acc += __shfl_xor(acc, off, 16);
                if ((threadIdx.x & 15) == 0 && i < Lp) dsum_s[i] = acc;
            }
        }
        __syncthreads();
    }
    float* ds_head = DS ? ds_out + (int64_t)bh * Lp * Lp : nullptr;
    const int last_valid = ctl[0];
    const bool any_valid = last_valid >= 0;
    const int ngroups = Lp / 16;

    for (;;) {
        const int gi = claim_group(ctl, lane);
        if (gi >= ngroups) break;
        const int kb = gi * 16;  // causal: earlier key groups see more queries -> claimed first
        const int kj = kb + c16;
        const bool key_ok = kj < L;
        floatx4 dvt[NCT], dkt[NCT];
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct) dvt[ct] = dkt[ct] = floatx4{0.f, 0.f, 0.f, 0.f};
        // padding keys past the last valid one receive no probability from any query
        const bool dead = any_valid && kb > last_valid;
        if (!dead) {
            float kf[DQ], vf[DQ];
            load_row_slice<DK>(k + (tok0 + kj) * ldk + h * DK, key_ok, g, kf);
            load_row_slice<DK>(v + (tok0 + kj) * ldv + h * DK, key_ok, g, vf);
            const bool key_masked_pad = key_ok ? !((kvw[kj >> 5] >> (kj & 31)) & 1u) : true;
            const uint16_t* keyw_key = drop_mask ? mask_keys(const_cast<uint8_t*>(drop_mask), (int64_t)gridDim.x, L) +
                                                       (int64_t)bh * ((L + 15) / 16) * mask_key_stride(L) + min(kj, L - 1)
                                                 : nullptr;
            const int kstride = mask_key_stride(L);
            const int q_start = (causal && any_valid) ? kb : 0;  // earlier queries see none of these keys
            const int nsub = (Lp - q_start) / 16;
            // P and dS of 16-query sub-tile `sub` of the chunk at qb (this lane: queries qb + 16 sub + 4g .. +3,
            // key kj) from its scores st / dP' dpt and key-major dropout word mw; dS is stored for the dQ pass
            // (ph_tag: dropout decisions recomputed by Philox -- no stored mask -- a branch; the pipelined chunks read
            // the stored mask through selects only)
            const float keepk = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
            const uint32_t mw_or = (p_drop > 0.f && drop_mask) ? 0u : 0xFFFFFFFFu;  // no dropout: every key kept
            auto soft_sub = [&](auto ph_tag, int qb, int sub, const floatx4& stv, const floatx4& dpv, uint32_t mwv_,
                                float (&pd)[4], float (&ds)[4]) {
                constexpr bool PH = decltype(ph_tag)::value;
                const int q4 = qb + sub * 16 + 4 * g;  // this lane's 4 query rows q4 .. q4+3
                const float4 mx4 = *reinterpret_cast<const float4*>(mx_s + q4);
                const float4 il4 = *reinterpret_cast<const float4*>(il_s + q4);
                const float4 ds4 = *reinterpret_cast<const float4*>(dsum_s + q4);
                const uint32_t mw = mwv_ >> (4 * g);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    // branch-free (selects): the pipelined loop keeps this work in the MFMA steps' scheduling regions
                    // (padding query rows read zero statistics: finite values, then discarded)
                    const int qq = q4 + r;
                    const bool ok = qq < L && key_ok;
                    const bool masked = key_masked_pad || (causal && kj > qq);
                    // explicitly rounded operations: the Philox and the stored-mask forms of this code (different
                    // surroundings) must not contract differently -- their results are compared bit for bit
                    const float sv_ = masked ? kMaskedScore : __fmul_rn(stv[r], scale);
                    const float pr = __fmul_rn(__expf(__fsub_rn(sv_, pick(mx4, r))), pick(il4, r));
                    float f;
                    if (PH) {
                        f = 1.f;
                        if (p_drop > 0.f) {
                            f = drop_mask ? ((mw >> r) & 1u ? keepk : 0.f)
                                          : pick(attn_keep4(seed, (uint64_t)bh * L + qq, kj & ~3, p_drop), kj & 3);
                        }
                    } else {
                        f = ((mw | mw_or) >> r) & 1u ? keepk : 0.f;
                    }
                    pd[r] = ok ? __fmul_rn(pr, f) : 0.f;
                    ds[r] = (ok && !masked) ? __fmul_rn(pr, __fmaf_rn(dpv[r], f, -pick(ds4, r))) : 0.f;
                }
                if (DS && ASME_ATTN_DIAG != 2) {  // dS[query q4 + r][key kj]: 16 lanes of a group store 64 contiguous bytes per row
#pragma unroll
                    for (int r = 0; r < 4; ++r) ds_head[(int64_t)(q4 + r) * Lp + kj] = ds[r];
                }
            };
            // the chunk's key-major dropout words, requested before its MFMAs
            auto load_mw = [&](auto ns_tag, int qb, uint32_t* mwv) {
                constexpr int NS = decltype(ns_tag)::value;
#pragma unroll
                for (int sub = 0; sub < NS; ++sub)
                    mwv[sub] = (p_drop > 0.f && drop_mask) ? keyw_key[((qb >> 4) + sub) * kstride] : 0u;
            };
            auto chunk = [&](auto ns_tag, int qb) {
                constexpr int NS = decltype(ns_tag)::value;
                floatx4 st[NS], dpt[NS];
                uint32_t mwv[NS];
                load_mw(ns_tag, qb, mwv);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int sub = 0; sub < NS; ++sub) st[sub] = dpt[sub] = floatx4{0.f, 0.f, 0.f, 0.f};
                rows_times_slice<DK, NS>(Qs + qb * S, g, c16, kf, st);
                rows_times_slice<DK, NS>(Ds + qb * S, g, c16, vf, dpt);
                float pd[NS][4], ds[NS][4];
#pragma unroll
                for (int sub = 0; sub < NS; ++sub)
                    soft_sub(std::true_type{}, qb, sub, st[sub], dpt[sub], mwv[sub], pd[sub], ds[sub]);
                cols_times_weights<DK, NS>(Ds + qb * S, g, c16, pd, dvt);  // dV^T += dO^T P
                cols_times_weights<DK, NS>(Qs + qb * S, g, c16, ds, dkt);  // dK^T += Q^T dS
            };
            // Full 64-query chunks as a two-stage pipeline within the wave: the score products of chunk c + 1 are
            // issued with chunk c's softmax-gradient vector work spread between their steps (it issues in the
            // MFMAs' shadow instead of between chunk c's two MFMA phases), then chunk c's dV / dK products.
            // (dk = 128: the second chunk's scores do not fit the 256 registers of two waves per SIMD: unpipelined)
            // (also unpipelined: dropout without the forward's stored decisions, Philox recomputed per element)
            const bool pipe = DK <= 64 && !(p_drop > 0.f && !drop_mask);
            const int nfull = pipe ? nsub / kNS : 0;
            constexpr int T = 2 * (DQ / 4);  // score-product steps per chunk (Q, then dO)
            if (!pipe) {
                int c0 = 0;
                for (; c0 + kNS <= nsub; c0 += kNS) chunk(std::integral_constant<int, kNS>{}, q_start + c0 * 16);
                for (; c0 < nsub; ++c0) chunk(std::integral_constant<int, 1>{}, q_start + c0 * 16);
            }
            if (pipe && nfull > 0) {
                floatx4 st[kNS], dpt[kNS];
                uint32_t mwv[kNS];
                load_mw(std::integral_constant<int, kNS>{}, q_start, mwv);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int sub = 0; sub < kNS; ++sub) st[sub] = dpt[sub] = floatx4{0.f, 0.f, 0.f, 0.f};
                rows_times_slice<DK, kNS>(Qs + q_start * S, g, c16, kf, st);
                rows_times_slice<DK, kNS>(Ds + q_start * S, g, c16, vf, dpt);
                for (int c = 0; c < nfull; ++c) {
                    const int qb = q_start + c * kKT;
                    float pd[kNS][4], ds[kNS][4];
                    if (c + 1 < nfull) {
                        floatx4 stn[kNS], dptn[kNS];
                        uint32_t mwn[kNS];
                        load_mw(std::integral_constant<int, kNS>{}, qb + kKT, mwn);
#pragma unroll
                        for (int sub = 0; sub < kNS; ++sub) stn[sub] = dptn[sub] = floatx4{0.f, 0.f, 0.f, 0.f};
                        auto fill = [&](int t) {
#pragma unroll
                            for (int sub = t * kNS / T; sub < (t + 1) * kNS / T; ++sub)
                                soft_sub(std::false_type{}, qb, sub, st[sub], dpt[sub], mwv[sub], pd[sub], ds[sub]);
                        };
                        rows_times_slice<DK, kNS>(Qs + (qb + kKT) * S, g, c16, kf, stn, [&](int s4) { fill(s4); });
                        rows_times_slice<DK, kNS>(Ds + (qb + kKT) * S, g, c16, vf, dptn,
                                                  [&](int s4) { fill(DQ / 4 + s4); });
                        __builtin_amdgcn_sched_barrier(0);
                        cols_times_weights<DK, kNS>(Ds + qb * S, g, c16, pd, dvt);  // dV^T += dO^T P
                        cols_times_weights<DK, kNS>(Qs + qb * S, g, c16, ds, dkt);  // dK^T += Q^T dS
#pragma unroll
                        for (int sub = 0; sub < kNS; ++sub) {
                            st[sub] = stn[sub];
                            dpt[sub] = dptn[sub];
                            mwv[sub] = mwn[sub];
                        }
                    } else {
#pragma unroll
                        for (int sub = 0; sub < kNS; ++sub)
                            soft_sub(std::false_type{}, qb, sub, st[sub], dpt[sub], mwv[sub], pd[sub], ds[sub]);
                        cols_times_weights<DK, kNS>(Ds + qb * S, g, c16, pd, dvt);
                        cols_times_weights<DK, kNS>(Qs + qb * S, g, c16, ds, dkt);
                    }
                }
            }
            if (pipe)
                for (int c0 = nfull * kNS; c0 < nsub; ++c0) chunk(std::integral_constant<int, 1>{}, q_start + c0 * 16);
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
}

// dQ = scale * dS K from the dS image attn_bwd_dkdv_res_kernel<DK, true> stored: one workgroup per (batch, head)
// with K resident in LDS, waves claiming 16-query groups (most keys first under a causal mask).  Lane (g, c16) of
// a group reads its query's dS row as float4s (keys 4g .. 4g+3 of each 16-key sub-tile: the weights
// cols_times_weights takes), the next chunk's while the current chunk's MFMAs run.  Only key sub-tiles the dK/dV
// pass formed are read: keys < min(last valid key + 1, q0 + 16) (causal) or < last valid key + 1.
constexpr int kDsThreads = 512;

template <int DK, int NT>
__device__ __forceinline__ void load_one_resident(const float* __restrict__ a, int64_t lda, int L, int Lp,
                                                  float* __restrict__ As) {
    constexpr int C4 = DK / 4, S = DK + 4;
    const int n4 = Lp * C4;
    for (int base = threadIdx.x; base < n4; base += NT * 8) {
        float4 ra[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int idx = base + u * NT, row = idx / C4, c = (idx % C4) * 4;
            ra[u] = (idx < n4 && row < L) ? *reinterpret_cast<const float4*>(a + (int64_t)row * lda + c)
                                          : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int idx = base + u * NT, row = idx / C4, c = (idx % C4) * 4;
            if (idx < n4) *reinterpret_cast<float4*>(As + row * S + c) = ra[u];
        }
    }
}

template <int DK>
__global__ __launch_bounds__(kDsThreads) void attn_bwd_dq_ds_kernel(const float* __restrict__ k, int64_t ldk,
                                                                    const float* __restrict__ ds,
                                                                    float* __restrict__ dq, int64_t lddq,
                                                                    const uint8_t* __restrict__ key_valid, int H,
                                                                    int L, int causal, float scale) {
    constexpr int NCT = DK / 16, S = DK + 4;
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int Lp = res_rows(L);
    float* Ks = lds;
    uint32_t* kvw = reinterpret_cast<uint32_t*>(Ks + Lp * S);
    int* ctl = reinterpret_cast<int*>(kvw + (Lp + 31) / 32);

    const int bh = blockIdx.x, b = bh / H, h = bh % H;
    const int lane = threadIdx.x & 63, g = lane >> 4, c16 = lane & 15;
    const int64_t tok0 = (int64_t)b * L;

    stage_valid_res(key_valid, b, L, Lp, kvw, ctl);
    load_one_resident<DK, kDsThreads>(k + tok0 * ldk + h * DK, ldk, L, Lp, Ks);
    __syncthreads();
    const int last_valid = ctl[0];
    const bool any_valid = last_valid >= 0;
    const int kend = any_valid ? last_valid + 1 : L;
    const int ngroups = Lp / 16;
    const float* ds_head = ds + (int64_t)bh * Lp * Lp;

    for (;;) {
        const int gi = claim_group(ctl, lane);
        if (gi >= ngroups) break;
        const int q0 = (causal ? ngroups - 1 - gi : gi) * 16;
        const int qi = q0 + c16;
        const int kmax = (causal && any_valid) ? min(kend, q0 + 16) : kend;
        const int nsub = (kmax + 15) / 16;
        const float* wrow = ds_head + (int64_t)qi * Lp + 4 * g;
        floatx4 acc[NCT];
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct) acc[ct] = floatx4{0.f, 0.f, 0.f, 0.f};
        // the dS row slice two chunks ahead: the loads of chunk c + 2 are in flight during chunk c's MFMAs (one
        // chunk ahead left ~half the pass waiting on them)
        float4 b0[kNS], b1[kNS], b2[kNS];
        auto fetch = [&](int c, float4 (&dst)[kNS]) {
#pragma unroll
            for (int sub = 0; sub < kNS; ++sub)
                dst[sub] = c + sub < nsub ? *reinterpret_cast<const float4*>(wrow + (c + sub) * 16)
                                          : make_float4(0.f, 0.f, 0.f, 0.f);
        };
        fetch(0, b0);
        fetch(kNS, b1);
        int c0 = 0;
        for (; c0 + kNS <= nsub; c0 += kNS) {
            fetch(c0 + 2 * kNS, b2);
            float w[kNS][4];
#pragma unroll
            for (int sub = 0; sub < kNS; ++sub) {
                w[sub][0] = b0[sub].x;
                w[sub][1] = b0[sub].y;
                w[sub][2] = b0[sub].z;
                w[sub][3] = b0[sub].w;
            }
            cols_times_weights<DK, kNS>(Ks + c0 * 16 * S, g, c16, w, acc);
#pragma unroll
            for (int sub = 0; sub < kNS; ++sub) {
                b0[sub] = b1[sub];
                b1[sub] = b2[sub];
            }
        }
#pragma unroll
        for (int sub = 0; sub < kNS - 1; ++sub) {
            if (c0 + sub < nsub) {
                float w1[1][4] = {{b0[sub].x, b0[sub].y, b0[sub].z, b0[sub].w}};
                cols_times_weights<DK, 1>(Ks + (c0 + sub) * 16 * S, g, c16, w1, acc);
            }
        }
        if (qi < L) {
            float* row = dq + (tok0 + qi) * lddq + h * DK;
#pragma unroll
            for (int ct = 0; ct < NCT; ++ct)
                *reinterpret_cast<float4*>(row + ct * 16 + 4 * g) =
                    make_float4(acc[ct][0] * scale, acc[ct][1] * scale, acc[ct][2] * scale, acc[ct][3] * scale);
        }
    }
}

inline size_t ds_lds_bytes(int L, int DK) {
    const size_t Lp = (size_t)res_rows(L);
    return Lp * (DK + 4) * sizeof(float) + (Lp + 31) / 32 * 4 + 16;
}

template <class K>
bool res_prepare(K kernel, size_t lds) {
    if (lds > 160 * 1024) return false;
    return hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)lds) == hipSuccess;
}

#ifndef ASME_ATTN_SKIP_NIB
#define ASME_ATTN_SKIP_NIB 1  // 0: the forward always stores the keep nibbles (A/B)
#endif
// the family-0 backward runs the dS-storing resident pair (asme_attention_bwd_kernels' first branch)
template <int DK>
bool bwd_stores_ds(int L) {
    return res_prepare(attn_bwd_dkdv_res_kernel<DK, true>, res_lds_bytes(L, DK, true)) &&
           res_prepare(attn_bwd_dq_ds_kernel<DK>, ds_lds_bytes(L, DK));
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

// kernel families (asme_attention_*_kernels): 0 = automatic (resident kernels whenever the head's operands fit LDS;
// backward: dK/dV storing dS, then dQ = dS K), 1 = streaming kernels only, 2 = resident kernels with the backward's
// dQ pass recomputing S and dP (the round-2 path).  1 and 2 exist for the kernel tests and same-process A/B timing;
// the product entry points asme_attention_fwd / _bwd always take 0.  A per-call argument: no process state.
ASME_API int asme_attention_fwd_kernels(int kernels, const float* q, const float* k, const float* v, int64_t ld_q,
                                        int64_t ld_k, int64_t ld_v, const uint8_t* key_valid, int64_t batch,
                                        int64_t heads, int64_t seq_len, int64_t head_dim, int causal, float scale,
                                        float p_drop, uint64_t seed, float* out, int64_t ld_out, float* lse,
                                        uint8_t* drop_mask, void* stream) {
    ASME_CHECK_ARG(q && k && v && out && lse, "asme_attention_fwd: null pointer");
    ASME_CHECK_ARG(kernels >= 0 && kernels <= 2, "asme_attention_fwd: kernel family must be 0, 1 or 2");
    ASME_CHECK_ARG(seq_len >= 1 && seq_len <= kMaxL, "asme_attention_fwd: seq_len must be in [1, 1024]");
    ASME_CHECK_ARG(p_drop >= 0.f && p_drop < 1.f, "asme_attention_fwd: dropout p must be in [0,1)");
    ASME_CHECK_ARG(aligned16(out, ld_out) && aligned16(q, ld_q) && aligned16(k, ld_k) && aligned16(v, ld_v),
                   "asme_attention_fwd: operands must be 16-B aligned with ld % 4 == 0");
    if (batch == 0) return 0;
    const dim3 grid((unsigned)((seq_len + kQB - 1) / kQB), (unsigned)(batch * heads));
    const size_t lds = res_lds_bytes((int)seq_len, (int)head_dim, false, ASME_ATTN_SLICED);
    ASME_DK_DISPATCH(head_dim,
        // the query-major keep nibbles are read only by the dQ passes that regenerate P (families 1 and 2, and family
        // 0 when its dS-storing backward does not fit); the family-0 backward's dK/dV pass reads the key-major words
        // and its dQ pass the stored dS -- so this forward stores the nibbles only when some backward will read them
        const int with_nib = !(kernels == 0 && ASME_ATTN_SKIP_NIB && bwd_stores_ds<DK>((int)seq_len));
        if (kernels != 1 && res_prepare(attn_fwd_res_kernel<DK>, lds))
            hipLaunchKernelGGL(attn_fwd_res_kernel<DK>, dim3((unsigned)(batch * heads)), dim3(kResThreads), lds,
                               (hipStream_t)stream, q, k, v, ld_q, ld_k, ld_v, out, ld_out, lse, key_valid,
                               (int)heads, (int)seq_len, causal, scale, p_drop, seed, drop_mask, with_nib);
        else
            hipLaunchKernelGGL(attn_fwd_kernel<DK>, grid, dim3(256), 0, (hipStream_t)stream, q, k, v, ld_q, ld_k,
                               ld_v, out, ld_out, lse, key_valid, (int)heads, (int)seq_len, causal, scale, p_drop,
                               seed, drop_mask));
    ASME_LAUNCH_CHECK("asme_attention_fwd");
}

ASME_API int asme_attention_fwd(const float* q, const float* k, const float* v, int64_t ld_q, int64_t ld_k,
                                int64_t ld_v, const uint8_t* key_valid, int64_t batch, int64_t heads, int64_t seq_len,
                                int64_t head_dim, int causal, float scale, float p_drop, uint64_t seed, float* out,
                                int64_t ld_out, float* lse, uint8_t* drop_mask, void* stream) {
    return asme_attention_fwd_kernels(0, q, k, v, ld_q, ld_k, ld_v, key_valid, batch, heads, seq_len, head_dim, causal,
                                      scale, p_drop, seed, out, ld_out, lse, drop_mask, stream);
}

// workspace of asme_attention_bwd: D_i (batch*heads*seq_len floats), then (256-B aligned) the dS image of the
// resident path ((batch*heads) x Lp x Lp floats, Lp = seq_len rounded up to 16)
ASME_API int64_t asme_attention_bwd_workspace(int64_t batch, int64_t heads, int64_t seq_len, int64_t head_dim) {
    (void)head_dim;
    const int64_t Lp = res_rows((int)seq_len);
    return ((batch * heads * seq_len * 4 + 255) & ~(int64_t)255) + batch * heads * Lp * Lp * 4;
}

ASME_API int asme_attention_bwd_kernels(int kernels, const float* q, const float* k, const float* v, int64_t ld_q,
                                        int64_t ld_k, int64_t ld_v, const float* out, int64_t ld_out,
                                        const float* dout, int64_t ld_dout, const float* lse,
                                        const uint8_t* key_valid, int64_t batch, int64_t heads, int64_t seq_len,
                                        int64_t head_dim, int causal, float scale, float p_drop, uint64_t seed,
                                        const uint8_t* drop_mask, float* workspace, float* dq, int64_t ld_dq,
                                        float* dk, int64_t ld_dk, float* dv, int64_t ld_dv, void* stream) {
    ASME_CHECK_ARG(q && k && v && out && dout && lse && workspace && dq && dk && dv, "asme_attention_bwd: null pointer");
    ASME_CHECK_ARG(kernels >= 0 && kernels <= 2, "asme_attention_bwd: kernel family must be 0, 1 or 2");
    float* dsum_ws = workspace;
    float* ds_ws = workspace + ((batch * heads * seq_len * 4 + 255) & ~(int64_t)255) / 4;
    ASME_CHECK_ARG(seq_len >= 1 && seq_len <= kMaxL, "asme_attention_bwd: seq_len must be in [1, 1024]");
    ASME_CHECK_ARG(aligned16(dq, ld_dq) && aligned16(dk, ld_dk) && aligned16(dv, ld_dv) && aligned16(q, ld_q) &&
                       aligned16(k, ld_k) && aligned16(v, ld_v) && aligned16(out, ld_out) &&
                       aligned16(dout, ld_dout),
                   "asme_attention_bwd: operands must be 16-B aligned with ld % 4 == 0");
    if (batch == 0) return 0;
    hipStream_t s = (hipStream_t)stream;
    const dim3 grid((unsigned)((seq_len + kQB - 1) / kQB), (unsigned)(batch * heads));
    const dim3 rgrid((unsigned)(batch * heads));
    const size_t lds_dq = res_lds_bytes((int)seq_len, (int)head_dim, false);
    const size_t lds_kv = res_lds_bytes((int)seq_len, (int)head_dim, true);
    const size_t lds_ds = ds_lds_bytes((int)seq_len, (int)head_dim);
    ASME_DK_DISPATCH(
        head_dim,
        if (kernels == 0 && res_prepare(attn_bwd_dkdv_res_kernel<DK, true>, lds_kv) &&
            res_prepare(attn_bwd_dq_ds_kernel<DK>, lds_ds)) {
            // dK/dV first (it stores dS), then dQ = dS K: five products instead of seven
            hipLaunchKernelGGL((attn_bwd_dkdv_res_kernel<DK, true>), rgrid, dim3(kResThreadsKV), lds_kv, s, q, k, v,
                               ld_q, ld_k, ld_v, dout, ld_dout, lse, dsum_ws, dk, ld_dk, dv, ld_dv, key_valid,
                               (int)heads, (int)seq_len, causal, scale, p_drop, seed, drop_mask, out, ld_out, ds_ws);
            hipLaunchKernelGGL(attn_bwd_dq_ds_kernel<DK>, rgrid, dim3(kDsThreads), lds_ds, s, k, ld_k, ds_ws, dq, ld_dq,
                               key_valid, (int)heads, (int)seq_len, causal, scale);
        } else if (kernels != 1 && res_prepare(attn_bwd_dq_res_kernel<DK>, lds_dq) &&
                   res_prepare(attn_bwd_dkdv_res_kernel<DK, false>, lds_kv)) {
            hipLaunchKernelGGL(attn_bwd_dq_res_kernel<DK>, rgrid, dim3(kResThreads), lds_dq, s, q, k, v, ld_q, ld_k,
                               ld_v, out, ld_out, dout, ld_dout, lse, dsum_ws, dq, ld_dq, key_valid, (int)heads,
                               (int)seq_len, causal, scale, p_drop, seed, drop_mask);
            hipLaunchKernelGGL((attn_bwd_dkdv_res_kernel<DK, false>), rgrid, dim3(kResThreadsKV), lds_kv, s, q, k, v,
                               ld_q, ld_k, ld_v, dout, ld_dout, lse, dsum_ws, dk, ld_dk, dv, ld_dv, key_valid,
                               (int)heads, (int)seq_len, causal, scale, p_drop, seed, drop_mask, out, ld_out,
                               nullptr);
        } else {
        hipLaunchKernelGGL(attn_bwd_dq_kernel<DK>, grid, dim3(256), 0, s, q, k, v, ld_q, ld_k, ld_v, out, ld_out, dout,
                           ld_dout, lse, dsum_ws, dq, ld_dq, key_valid, (int)heads, (int)seq_len, causal, scale,
                           p_drop, seed, drop_mask);
        hipLaunchKernelGGL(attn_bwd_dkdv_kernel<DK>, grid, dim3(256), 0, s, q, k, v, ld_q, ld_k, ld_v, dout,
                           ld_dout, lse, dsum_ws, dk, ld_dk, dv, ld_dv, key_valid, (int)heads, (int)seq_len, causal,
                           scale, p_drop, seed, drop_mask);
        });
    ASME_LAUNCH_CHECK("asme_attention_bwd");
}

ASME_API int asme_attention_bwd(const float* q, const float* k, const float* v, int64_t ld_q, int64_t ld_k,
                                int64_t ld_v, const float* out, int64_t ld_out, const float* dout, int64_t ld_dout,
                                const float* lse, const uint8_t* key_valid, int64_t batch, int64_t heads,
                                int64_t seq_len, int64_t head_dim, int causal, float scale, float p_drop,
                                uint64_t seed, const uint8_t* drop_mask, float* workspace, float* dq, int64_t ld_dq,
                                float* dk, int64_t ld_dk, float* dv, int64_t ld_dv, void* stream) {
    return asme_attention_bwd_kernels(0, q, k, v, ld_q, ld_k, ld_v, out, ld_out, dout, ld_dout, lse, key_valid, batch,
                                      heads, seq_len, head_dim, causal, scale, p_drop, seed, drop_mask, workspace, dq,
                                      ld_dq, dk, ld_dk, dv, ld_dv, stream);
}

// bytes of the drop_mask buffer the forward fills when p_drop > 0 (nibble image + key-major words)
ASME_API int64_t asme_attention_dropout_mask_bytes(int64_t batch, int64_t heads, int64_t seq_len) {
    return mask_total_bytes(batch * heads, (int)seq_len);
}
