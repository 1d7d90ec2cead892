// Masked multi-head self-attention for short sequences (L <= 1024, designed for L <= 200) on gfx950.
//
// Reference semantics (paths relative to /root/reference/src/asme):
//   Attention.forward            core/models/common/layers/transformer_layers.py:138-155
//       scores = QK^T / sqrt(dk); masked_fill(mask == 0, -1e9); softmax; dropout(p_attn); P V
//   MultiHeadedAttention.forward transformer_layers.py:181-199 (heads = column blocks of the projections)
//   mask construction            core/models/transformer/sequence_representation.py:34-48
//       causal:        tril(ones(L,L)) * key_padding_mask   (SASRec)
//       bidirectional: key_padding_mask                      (BERT4Rec / KeBERT4Rec)
// The (B,1,L,L) float mask of the reference is never materialised: the kernel derives it from the
// key-validity bytes and causality.  Masked scores are exactly -1e9 (not -inf), so a row with no
// admissible key reproduces the reference's uniform softmax over all L keys.
//
// Layout: Q/K/V rows are token-major with a row stride (the fused QKV projection output (T, 3*H*dk)
// is consumed in place); head h occupies columns [h*dk, (h+1)*dk).  O is (T, H*dk); the softmax row
// statistics are (B*H, L, 2) = (running max, 1 / sum of exp) per query row.
//
// Compute: fp32 MFMA v_mfma_f32_16x16x4f32 (exact f32 FMA chain).  One workgroup = 4 waves =
// 64 query rows (forward / dQ) or 64 key rows (dK/dV) of one (batch, head); the other operand
// streams through LDS in 16-row tiles.  The softmax runs flash-style (running max / sum) in the
// "swapped" S^T = K Q^T orientation so that P^T is directly the B operand of O^T += V^T P^T.
// The contraction index of each MFMA is permuted per lane group (lane group g handles feature
// columns g*dk/4 .. g*dk/4+dk/4-1) so every lane's operand slice is a contiguous register block.
#include "common.h"

using namespace asme;

namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int kQB = 64;       // rows per workgroup (4 waves x 16)
constexpr int kKT = 16;       // streamed tile rows
constexpr int kMaxL = 1024;   // LDS-staged key-validity bytes
constexpr float kMaskedScore = -1e9f;
constexpr float kInitMax = -1e30f;

__device__ __forceinline__ floatx4 mfma16(float a, float b, floatx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Stage the key-validity row of batch b in LDS and derive the admissible key range.
// Returns (via refs) whether any key is valid and the index of the last valid key.
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

// cooperative load of `rows` rows (starting at r0) of a [L][DK] head slice into LDS [kKT][DK+PAD]
template <int DK, int PAD>
__device__ __forceinline__ void load_tile(const float* __restrict__ base, int64_t ld, int r0, int L, float* tile) {
    constexpr int N = kKT * DK;
    for (int i = threadIdx.x; i < N; i += blockDim.x) {
        const int r = i / DK, c = i % DK;
        const int row = r0 + r;
        tile[r * (DK + PAD) + c] = row < L ? base[(int64_t)row * ld + c] : 0.f;
    }
}

template <int DK>
__global__ __launch_bounds__(256) void attn_fwd_kernel(const float* __restrict__ q, const float* __restrict__ k,
                                                       const float* __restrict__ v, int64_t ldq, int64_t ldk,
                                                       int64_t ldv, float* __restrict__ o, int64_t ldo,
                                                       float* __restrict__ lse, const uint8_t* __restrict__ key_valid,
                                                       int H, int L, int causal, float scale, float p_drop,
                                                       uint64_t seed) {
    constexpr int DQ = DK / 4;    // per-lane contraction slice
    constexpr int NCT = DK / 16;  // 16-column output tiles
    __shared__ float Ks[kKT * (DK + 1)];
    __shared__ float Vs[kKT * (DK + 4)];
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
#pragma unroll
    for (int s = 0; s < DQ; ++s) qf[s] = qi < L ? qh[(int64_t)qi * ldq + g * DQ + s] : 0.f;

    floatx4 acc[NCT];
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) acc[ct] = floatx4{0.f, 0.f, 0.f, 0.f};
    float m = kInitMax, l = 0.f;

    for (int k0 = 0; k0 < kmax; k0 += kKT) {
        __syncthreads();
        load_tile<DK, 1>(kh, ldk, k0, L, Ks);
        load_tile<DK, 4>(vh, ldv, k0, L, Vs);
        __syncthreads();
        floatx4 st = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < DQ; ++s) st = mfma16(Ks[c16 * (DK + 1) + g * DQ + s], qf[s], st);
        float p[4];
        float tmax = kInitMax;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int key = k0 + 4 * g + r;
            float sv;
            if (key >= L) {
                sv = -INFINITY;  // not a key at all
            } else {
                const bool masked = !kv_s[key] || (causal && key > qi);
                sv = masked ? kMaskedScore : st[r] * scale;
            }
            p[r] = sv;
            tmax = fmaxf(tmax, sv);
        }
        tmax = group4_max(tmax);
        const float mnew = fmaxf(m, tmax);
        const float alpha = __expf(m - mnew);
        float rs = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            p[r] = __expf(p[r] - mnew);
            rs += p[r];
        }
        rs = group4_sum(rs);
        l = l * alpha + rs;
        m = mnew;
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct) acc[ct] *= alpha;
        if (p_drop > 0.f) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int key = k0 + 4 * g + r;
                const uint64_t idx = ((uint64_t)bh * L + (uint64_t)min(qi, L - 1)) * L + min(key, L - 1);
                p[r] *= dropout_factor(seed, 6u, idx, p_drop);
            }
        }
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
            for (int s = 0; s < 4; ++s) acc[ct] = mfma16(Vs[(4 * g + s) * (DK + 4) + ct * 16 + c16], p[s], acc[ct]);
    }
    if (qi < L) {
        const float inv = 1.f / l;
        float* orow = o + (tok0 + qi) * ldo + h * DK;
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct) {
            float4 w4 = make_float4(acc[ct][0] * inv, acc[ct][1] * inv, acc[ct][2] * inv, acc[ct][3] * inv);
            *reinterpret_cast<float4*>(orow + ct * 16 + 4 * g) = w4;
        }
        // row statistics (running max, 1/sum) rather than m + log(l): for a row with no admissible key
        // every score is -1e9 and m + log(l) would round to -1e9, losing the 1/L of the uniform softmax
        if (g == 0) {
            lse[((int64_t)bh * L + qi) * 2] = m;
            lse[((int64_t)bh * L + qi) * 2 + 1] = inv;
        }
    }
}

// D_i = rowsum(dO_i * O_i) per (b, h, i)
template <int DK>
__global__ __launch_bounds__(256) void attn_bwd_pre_kernel(const float* __restrict__ o, int64_t ldo,
                                                           const float* __restrict__ dout, int64_t lddo,
                                                           float* __restrict__ dsum, int B, int H, int L) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);  // row = (b*H + h)*L + i
    if (row >= (int64_t)B * H * L) return;
    const int i = row % L;
    const int64_t bh = row / L;
    const int b = bh / H, h = bh % H;
    const int64_t t = (int64_t)b * L + i;
    float s = 0.f;
    for (int c = lane; c < DK; c += 64) s += o[t * ldo + h * DK + c] * dout[t * lddo + h * DK + c];
    s = wave_sum(s);
    if (lane == 0) dsum[row] = s;
}

template <int DK>
__global__ __launch_bounds__(256) void attn_bwd_dq_kernel(
    const float* __restrict__ q, const float* __restrict__ k, const float* __restrict__ v, int64_t ldq, int64_t ldk,
    int64_t ldv, const float* __restrict__ dout, int64_t lddo, const float* __restrict__ lse,
    const float* __restrict__ dsum, float* __restrict__ dq, int64_t lddq, const uint8_t* __restrict__ key_valid,
    int H, int L, int causal, float scale, float p_drop, uint64_t seed) {
    constexpr int DQ = DK / 4;
    constexpr int NCT = DK / 16;
    __shared__ float Ks[kKT * (DK + 1)];
    __shared__ float Vs[kKT * (DK + 1)];
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
    const float* qh = q + tok0 * ldq + h * DK;
    const float* kh = k + tok0 * ldk + h * DK;
    const float* vh = v + tok0 * ldv + h * DK;
    const float* doh = dout + tok0 * lddo + h * DK;

    float qf[DQ], df[DQ];
#pragma unroll
    for (int s = 0; s < DQ; ++s) {
        qf[s] = qi < L ? qh[(int64_t)qi * ldq + g * DQ + s] : 0.f;
        df[s] = qi < L ? doh[(int64_t)qi * lddo + g * DQ + s] : 0.f;
    }
    const float mq = qi < L ? lse[((int64_t)bh * L + qi) * 2] : 0.f;
    const float iq = qi < L ? lse[((int64_t)bh * L + qi) * 2 + 1] : 0.f;
    const float dq_row = qi < L ? dsum[(int64_t)bh * L + qi] : 0.f;

    floatx4 acc[NCT];
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) acc[ct] = floatx4{0.f, 0.f, 0.f, 0.f};

    for (int k0 = 0; k0 < kmax; k0 += kKT) {
        __syncthreads();
        load_tile<DK, 1>(kh, ldk, k0, L, Ks);
        load_tile<DK, 1>(vh, ldv, k0, L, Vs);
        __syncthreads();
        floatx4 st = {0.f, 0.f, 0.f, 0.f}, dpt = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < DQ; ++s) {
            st = mfma16(Ks[c16 * (DK + 1) + g * DQ + s], qf[s], st);
            dpt = mfma16(Vs[c16 * (DK + 1) + g * DQ + s], df[s], dpt);
        }
        float ds[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int key = k0 + 4 * g + r;
            float val = 0.f;
            if (key < L && qi < L) {
                const bool masked = !kv_s[key] || (causal && key > qi);
                const float sv = masked ? kMaskedScore : st[r] * scale;
                const float pr = __expf(sv - mq) * iq;
                float dp = dpt[r];
                if (p_drop > 0.f) dp *= dropout_factor(seed, 6u, ((uint64_t)bh * L + qi) * L + key, p_drop);
                val = masked ? 0.f : pr * (dp - dq_row);
            }
            ds[r] = val;
        }
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
            for (int s = 0; s < 4; ++s) acc[ct] = mfma16(Ks[(4 * g + s) * (DK + 1) + ct * 16 + c16], ds[s], acc[ct]);
    }
    if (qi < L) {
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
    int64_t ldv, const float* __restrict__ dout, int64_t lddo, const float* __restrict__ lse,
    const float* __restrict__ dsum, float* __restrict__ dk, int64_t lddk, float* __restrict__ dv, int64_t lddv,
    const uint8_t* __restrict__ key_valid, int H, int L, int causal, float scale, float p_drop, uint64_t seed) {
    constexpr int DQ = DK / 4;
    constexpr int NCT = DK / 16;
    __shared__ float Qs[kKT * (DK + 1)];
    __shared__ float Ds[kKT * (DK + 1)];
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
    const float* kh = k + tok0 * ldk + h * DK;
    const float* vh = v + tok0 * ldv + h * DK;
    const float* doh = dout + tok0 * lddo + h * DK;

    float kf[DQ], vf[DQ];
#pragma unroll
    for (int s = 0; s < DQ; ++s) {
        kf[s] = kj < L ? kh[(int64_t)kj * ldk + g * DQ + s] : 0.f;
        vf[s] = kj < L ? vh[(int64_t)kj * ldv + g * DQ + s] : 0.f;
    }
    const bool key_ok = kj < L;
    const bool key_masked_pad = key_ok ? !kv_s[kj] : true;

    floatx4 dvt[NCT], dkt[NCT];
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) dvt[ct] = dkt[ct] = floatx4{0.f, 0.f, 0.f, 0.f};

    // causal: queries before this key block see none of its keys (unless no key is valid at all)
    const int q_start = (causal && any_valid) ? (kblk / kKT) * kKT : 0;
    for (int q0 = q_start; q0 < L; q0 += kKT) {
        __syncthreads();
        load_tile<DK, 1>(qh, ldq, q0, L, Qs);
        load_tile<DK, 1>(doh, lddo, q0, L, Ds);
        if (threadIdx.x < kKT) {
            const int qq = q0 + threadIdx.x;
            mx_s[threadIdx.x] = qq < L ? lse[((int64_t)bh * L + qq) * 2] : 0.f;
            il_s[threadIdx.x] = qq < L ? lse[((int64_t)bh * L + qq) * 2 + 1] : 0.f;
            dsum_s[threadIdx.x] = qq < L ? dsum[(int64_t)bh * L + qq] : 0.f;
        }
        __syncthreads();
        floatx4 st = {0.f, 0.f, 0.f, 0.f}, dpt = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < DQ; ++s) {
            st = mfma16(Qs[c16 * (DK + 1) + g * DQ + s], kf[s], st);   // S[q][key]
            dpt = mfma16(Ds[c16 * (DK + 1) + g * DQ + s], vf[s], dpt); // dP'[q][key]
        }
        float pd[4], ds[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int qq = q0 + 4 * g + r;
            float pv = 0.f, dsv = 0.f;
            if (qq < L && key_ok) {
                const bool masked = key_masked_pad || (causal && kj > qq);
                const float sv = masked ? kMaskedScore : st[r] * scale;
                const float pr = __expf(sv - mx_s[4 * g + r]) * il_s[4 * g + r];
                float dp = dpt[r];
                float f = 1.f;
                if (p_drop > 0.f) f = dropout_factor(seed, 6u, ((uint64_t)bh * L + qq) * L + kj, p_drop);
                pv = pr * f;
                dp *= f;
                dsv = masked ? 0.f : pr * (dp - dsum_s[4 * g + r]);
            }
            pd[r] = pv;
            ds[r] = dsv;
        }
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                dvt[ct] = mfma16(Ds[(4 * g + s) * (DK + 1) + ct * 16 + c16], pd[s], dvt[ct]);
                dkt[ct] = mfma16(Qs[(4 * g + s) * (DK + 1) + ct * 16 + c16], ds[s], dkt[ct]);
            }
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
                                int64_t ld_out, float* lse, void* stream) {
    ASME_CHECK_ARG(q && k && v && out && lse, "asme_attention_fwd: null pointer");
    ASME_CHECK_ARG(seq_len >= 1 && seq_len <= kMaxL, "asme_attention_fwd: seq_len must be in [1, 1024]");
    ASME_CHECK_ARG(p_drop >= 0.f && p_drop < 1.f, "asme_attention_fwd: dropout p must be in [0,1)");
    ASME_CHECK_ARG(aligned16(out, ld_out), "asme_attention_fwd: output must be 16-B aligned with ld % 4 == 0");
    if (batch == 0) return 0;
    const dim3 grid((unsigned)((seq_len + kQB - 1) / kQB), (unsigned)(batch * heads));
    ASME_DK_DISPATCH(head_dim, hipLaunchKernelGGL(attn_fwd_kernel<DK>, grid, dim3(256), 0, (hipStream_t)stream, q, k,
                                                  v, ld_q, ld_k, ld_v, out, ld_out, lse, key_valid, (int)heads,
                                                  (int)seq_len, causal, scale, p_drop, seed));
    ASME_LAUNCH_CHECK("asme_attention_fwd");
}

ASME_API int asme_attention_bwd(const float* q, const float* k, const float* v, int64_t ld_q, int64_t ld_k,
                                int64_t ld_v, const float* out, int64_t ld_out, const float* dout, int64_t ld_dout,
                                const float* lse, const uint8_t* key_valid, int64_t batch, int64_t heads,
                                int64_t seq_len, int64_t head_dim, int causal, float scale, float p_drop,
                                uint64_t seed, float* dsum_ws, float* dq, int64_t ld_dq, float* dk, int64_t ld_dk,
                                float* dv, int64_t ld_dv, void* stream) {
    ASME_CHECK_ARG(q && k && v && out && dout && lse && dsum_ws && dq && dk && dv, "asme_attention_bwd: null pointer");
    ASME_CHECK_ARG(seq_len >= 1 && seq_len <= kMaxL, "asme_attention_bwd: seq_len must be in [1, 1024]");
    ASME_CHECK_ARG(aligned16(dq, ld_dq) && aligned16(dk, ld_dk) && aligned16(dv, ld_dv),
                   "asme_attention_bwd: gradients must be 16-B aligned with ld % 4 == 0");
    if (batch == 0) return 0;
    hipStream_t s = (hipStream_t)stream;
    const int64_t rows = batch * heads * seq_len;
    const dim3 grid((unsigned)((seq_len + kQB - 1) / kQB), (unsigned)(batch * heads));
    ASME_DK_DISPATCH(
        head_dim,
        hipLaunchKernelGGL(attn_bwd_pre_kernel<DK>, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s, out, ld_out,
                           dout, ld_dout, dsum_ws, (int)batch, (int)heads, (int)seq_len);
        hipLaunchKernelGGL(attn_bwd_dq_kernel<DK>, grid, dim3(256), 0, s, q, k, v, ld_q, ld_k, ld_v, dout, ld_dout,
                           lse, dsum_ws, dq, ld_dq, key_valid, (int)heads, (int)seq_len, causal, scale, p_drop, seed);
        hipLaunchKernelGGL(attn_bwd_dkdv_kernel<DK>, grid, dim3(256), 0, s, q, k, v, ld_q, ld_k, ld_v, dout,
                           ld_dout, lse, dsum_ws, dk, ld_dk, dv, ld_dv, key_valid, (int)heads, (int)seq_len, causal,
                           scale, p_drop, seed));
    ASME_LAUNCH_CHECK("asme_attention_bwd");
}
