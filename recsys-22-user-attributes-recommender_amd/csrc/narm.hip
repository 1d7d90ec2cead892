// NARM's sequential encoders on gfx950: the GRU recurrence of the global encoder (fp32 MFMA, forward and
// backward-through-time) and the attentive local encoder (forward and backward).
//
// Reference semantics (paths relative to /root/reference/src/asme):
//   NarmModel global encoder: nn.GRU(item_embedding_size, global_encoder_size, num_layers, batch_first=True)
//                                                   core/models/narm/components.py:32-56
//   PyTorch's GRU cell:  r = s(Wir x + bir + Whr h + bhr)   z = s(Wiz x + biz + Whz h + bhz)
//                        n = tanh(Win x + bin + r * (Whn h + bhn))   h' = (1 - z) * n + z * h
// The input half (x W_ih^T + b_ih for every step) is one tall GEMM on the Linear kernels and so is every weight
// gradient (dW_ih = dGx^T X, dW_hh = dGh^T H_prev); these kernels run only the sequential part:
//   forward   per step t: G_h = h_{t-1} W_hh^T (MFMA), gates, h_t; stores h_t and (r, z, n, W_hn h + b_hn)
//   backward  per step t (reverse): dh = dH_out[t] + dh_rec; the gate gradients dGx[t] (input side) and dGh[t]
//             (hidden side); dh_rec = dh * z + dGh W_hh (MFMA)
// Layout: one workgroup per 16 sequences (batch rows), HP/16 waves (HP = hidden size padded to a multiple of 16,
// <= 128): wave w owns hidden units 16w .. 16w+15 of all three gates, so the gate math of a unit never leaves its
// lane.  W_hh stays in registers for the whole sequence (the wave's 48 rows x HP in fp32 as MFMA B fragments;
// backward: its 16 columns x 3HP); the recurrent state (forward h, backward the hidden-side gate gradients) goes
// through a double-buffered LDS image, one barrier per step.  v_mfma_f32_16x16x4_f32: A = 16 batch rows x 4 k
// (lane (row, g) supplies k = 16 (kb / 4) + 4 g + kb % 4 -- one ds_read_b128 feeds four steps), B = 4 k x 16 units,
// C: lane (unit, g) holds rows 4g .. 4g+3.  Padded units have zero weights and stay exactly 0 from h_0 = 0.
#include "common.h"

using namespace asme;

namespace {

constexpr int kRows = 16;  // batch rows per workgroup

__device__ __forceinline__ floatx4 mfma4(float a, float b, floatx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + __expf(-x)); }

// gx: (B, L, 3HP) input-side pre-activations incl. b_ih; whh (3HP, HP); bhh (3HP); h0 (B, HP) nullable
// hout: (B, L, HP); gates: (B, L, 4, HP) = r, z, n, W_hn h + b_hn
template <int HP>
__global__ __launch_bounds__(HP / 16 * 64) void gru_fwd_kernel(const float* __restrict__ gx,
                                                               const float* __restrict__ whh,
                                                               const float* __restrict__ bhh,
                                                               const float* __restrict__ h0, int64_t B, int64_t L,
                                                               float* __restrict__ hout, float* __restrict__ gates) {
    constexpr int KS = HP / 4;  // MFMA k steps
    constexpr int LD = HP + 4;  // LDS row stride (floats)
    __shared__ __attribute__((aligned(16))) float hb[2][kRows * LD];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, n16 = lane & 15, g = lane >> 4;
    const int unit = wave * 16 + n16;
    const int64_t row0 = (int64_t)blockIdx.x * kRows;
    // W_hh fragments: wf[q][kb] = W_hh[q * HP + unit][k(kb, g)]
    float wf[3][KS];
#pragma unroll
    for (int q = 0; q < 3; ++q)
#pragma unroll
        for (int kb = 0; kb < KS; ++kb)
            wf[q][kb] = whh[(int64_t)(q * HP + unit) * HP + 16 * (kb / 4) + 4 * g + (kb % 4)];
    float bh[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) bh[q] = bhh[q * HP + unit];
    for (int i = threadIdx.x; i < kRows * HP; i += blockDim.x) {
        const int r = i / HP, c = i % HP;
        const int64_t b = row0 + r;
        hb[0][r * LD + c] = (h0 && b < B) ? h0[b * HP + c] : 0.f;
    }
    __syncthreads();
    // this lane's rows 4g + r; their input-side pre-activations of step t prefetched one step ahead
    float xg[4][3];
    auto load_x = [&](int64_t t) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int64_t b = row0 + 4 * g + r;
#pragma unroll
            for (int q = 0; q < 3; ++q) xg[r][q] = b < B ? gx[(b * L + t) * 3 * HP + q * HP + unit] : 0.f;
        }
    };
    load_x(0);
    for (int64_t t = 0; t < L; ++t) {
        const float* hc = hb[t & 1];
        float* hn = hb[(t & 1) ^ 1];
        floatx4 acc[3];
#pragma unroll
        for (int q = 0; q < 3; ++q) acc[q] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k4 = 0; k4 < HP / 16; ++k4) {
            const float4 a = *reinterpret_cast<const float4*>(hc + n16 * LD + 16 * k4 + 4 * g);
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                acc[q] = mfma4(a.x, wf[q][4 * k4], acc[q]);
                acc[q] = mfma4(a.y, wf[q][4 * k4 + 1], acc[q]);
                acc[q] = mfma4(a.z, wf[q][4 * k4 + 2], acc[q]);
                acc[q] = mfma4(a.w, wf[q][4 * k4 + 3], acc[q]);
            }
        }
        float cur[4][3];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int q = 0; q < 3; ++q) cur[r][q] = xg[r][q];
        if (t + 1 < L) load_x(t + 1);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = 4 * g + r;
            const int64_t b = row0 + row;
            const float hnv = acc[2][r] + bh[2];
            const float rr = sigm(cur[r][0] + acc[0][r] + bh[0]);
            const float zz = sigm(cur[r][1] + acc[1][r] + bh[1]);
            const float nn = tanhf(cur[r][2] + rr * hnv);
            const float h = (1.f - zz) * nn + zz * hc[row * LD + unit];
            hn[row * LD + unit] = h;
            if (b < B) {
                hout[(b * L + t) * HP + unit] = h;
                float* gp = gates + (b * L + t) * 4 * HP + unit;
                gp[0] = rr;
                gp[HP] = zz;
                gp[2 * HP] = nn;
                gp[3 * HP] = hnv;
            }
        }
        __syncthreads();
    }
}

// dhout (B, L, HP) gradient of every output; dhT (B, HP) nullable gradient of the final hidden state;
// dgx (B, L, 3HP) = gradient of the input-side pre-activations; dgh (B, L, 3HP) = of the hidden-side ones
// (W_h* h + b_h*); dh0 (B, HP) nullable
template <int HP>
__global__ __launch_bounds__(HP / 16 * 64) void gru_bwd_kernel(const float* __restrict__ dhout,
                                                               const float* __restrict__ dhT,
                                                               const float* __restrict__ whh,
                                                               const float* __restrict__ h0,
                                                               const float* __restrict__ hout,
                                                               const float* __restrict__ gates, int64_t B, int64_t L,
                                                               float* __restrict__ dgx, float* __restrict__ dgh,
                                                               float* __restrict__ dh0) {
    constexpr int KS = 3 * HP / 4;  // k steps over the 3HP gate gradients
    constexpr int LD = 3 * HP + 4;
    __shared__ __attribute__((aligned(16))) float gb[2][kRows * LD];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, n16 = lane & 15, g = lane >> 4;
    const int unit = wave * 16 + n16;
    const int64_t row0 = (int64_t)blockIdx.x * kRows;
    // W_hh^T fragments: wt[kb] = W_hh[k(kb, g)][unit], k over the 3HP gate rows
    float wt[KS];
#pragma unroll
    for (int kb = 0; kb < KS; ++kb) wt[kb] = whh[(int64_t)(16 * (kb / 4) + 4 * g + (kb % 4)) * HP + unit];
    float dhr[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int64_t b = row0 + 4 * g + r;
        dhr[r] = (dhT && b < B) ? dhT[b * HP + unit] : 0.f;
    }
    for (int64_t t = L - 1; t >= 0; --t) {
        float* gc = gb[t & 1];
        float dz_keep[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = 4 * g + r;
            const int64_t b = row0 + row;
            float d_r = 0.f, d_z = 0.f, d_n = 0.f, rr = 0.f;
            dz_keep[r] = 0.f;
            if (b < B) {
                const float dh = dhout[(b * L + t) * HP + unit] + dhr[r];
                const float* gp = gates + (b * L + t) * 4 * HP + unit;
                rr = gp[0];
                const float zz = gp[HP], nn = gp[2 * HP], hnv = gp[3 * HP];
                const float hprev = t > 0 ? hout[(b * L + t - 1) * HP + unit] : (h0 ? h0[b * HP + unit] : 0.f);
                d_n = dh * (1.f - zz) * (1.f - nn * nn);      // through n = tanh(.)
                d_z = dh * (hprev - nn) * zz * (1.f - zz);    // through z = s(.)
                d_r = d_n * hnv * rr * (1.f - rr);            // through r = s(.) in n
                dz_keep[r] = dh * zz;
                float* gxp = dgx + (b * L + t) * 3 * HP + unit;
                gxp[0] = d_r;
                gxp[HP] = d_z;
                gxp[2 * HP] = d_n;
                float* ghp = dgh + (b * L + t) * 3 * HP + unit;
                ghp[0] = d_r;
                ghp[HP] = d_z;
                ghp[2 * HP] = d_n * rr;
            }
            gc[row * LD + unit] = d_r;
            gc[row * LD + HP + unit] = d_z;
            gc[row * LD + 2 * HP + unit] = d_n * rr;
        }
        __syncthreads();
        floatx4 acc = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k4 = 0; k4 < KS / 4; ++k4) {
            const float4 a = *reinterpret_cast<const float4*>(gc + n16 * LD + 16 * k4 + 4 * g);
            acc = mfma4(a.x, wt[4 * k4], acc);
            acc = mfma4(a.y, wt[4 * k4 + 1], acc);
            acc = mfma4(a.z, wt[4 * k4 + 2], acc);
            acc = mfma4(a.w, wt[4 * k4 + 3], acc);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) dhr[r] = dz_keep[r] + acc[r];
    }
    if (dh0) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int64_t b = row0 + 4 * g + r;
            if (b < B) dh0[b * HP + unit] = dhr[r];
        }
    }
}

// ---------------------------------------------------------------------------------------------- local encoder
// LocalEncoderLayer (core/models/narm/layers.py:32-66): alpha_s = v . sigmoid(P1 + P2_s) with P1 = A1 c_g (N, H),
// P2 = A2 h_i (N, S, H) (the two projections are Linear kernels); c_l = sum_s mask_s alpha_s h_i[s].  One workgroup
// per sequence: the S alphas (one wave per position, lanes over H, wave reduction) go to LDS, then each thread
// owns hidden units and sums over the positions in order (deterministic, no atomics).
constexpr int kAttThreads = 256;

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

__global__ __launch_bounds__(kAttThreads) void narm_attend_fwd_kernel(const float* __restrict__ p1,
                                                                     const float* __restrict__ p2,
                                                                     const float* __restrict__ v,
                                                                     const float* __restrict__ hs,
                                                                     const uint8_t* __restrict__ mask, int64_t S,
                                                                     int64_t H, float* __restrict__ out,
                                                                     float* __restrict__ alpha) {
    extern __shared__ float al[];  // S weights (already multiplied by the mask)
    const int64_t n = blockIdx.x;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const float* P1 = p1 + n * H;
    for (int64_t s = wave; s < S; s += kAttThreads / 64) {
        const float* P2 = p2 + (n * S + s) * H;
        float acc = 0.f;
        for (int64_t h = lane; h < H; h += 64) acc += v[h] * sigm(P1[h] + P2[h]);
        acc = wave_sum(acc);
        if (lane == 0) {
            alpha[n * S + s] = acc;
            al[s] = mask[n * S + s] ? acc : 0.f;
        }
    }
    __syncthreads();
    for (int64_t h = threadIdx.x; h < H; h += kAttThreads) {
        float acc = 0.f;
        for (int64_t s = 0; s < S; ++s) acc += al[s] * hs[(n * S + s) * H + h];
        out[n * H + h] = acc;
    }
}

// gradients of c_l: dP2 (N, S, H), dP1 (N, H), dHs (N, S, H), dv_part (N, H) (summed over N by the caller)
__global__ __launch_bounds__(kAttThreads) void narm_attend_bwd_kernel(
    const float* __restrict__ dc, const float* __restrict__ p1, const float* __restrict__ p2,
    const float* __restrict__ v, const float* __restrict__ hs, const uint8_t* __restrict__ mask,
    const float* __restrict__ alpha, int64_t S, int64_t H, float* __restrict__ dp1, float* __restrict__ dp2,
    float* __restrict__ dhs, float* __restrict__ dv_part) {
    extern __shared__ float sh[];  // [S] dalpha, [S] mask * alpha
    float* dal = sh;
    float* al = sh + S;
    const int64_t n = blockIdx.x;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const float* dC = dc + n * H;
    for (int64_t s = wave; s < S; s += kAttThreads / 64) {
        const bool keep = mask[n * S + s] != 0;
        float acc = 0.f;
        if (keep) {
            const float* Hs = hs + (n * S + s) * H;
            for (int64_t h = lane; h < H; h += 64) acc += dC[h] * Hs[h];
            acc = wave_sum(acc);
        }
        if (lane == 0) {
            dal[s] = acc;
            al[s] = keep ? alpha[n * S + s] : 0.f;
        }
    }
    __syncthreads();
    const float* P1 = p1 + n * H;
    for (int64_t h = threadIdx.x; h < H; h += kAttThreads) {
        const float p1h = P1[h], vh = v[h], dch = dC[h];
        float g1 = 0.f, gv = 0.f;
        for (int64_t s = 0; s < S; ++s) {
            const int64_t o = (n * S + s) * H + h;
            const float sg = sigm(p1h + p2[o]);
            const float d = dal[s] * vh * sg * (1.f - sg);
            dp2[o] = d;
            dhs[o] = al[s] * dch;
            g1 += d;
            gv += dal[s] * sg;
        }
        dp1[n * H + h] = g1;
        dv_part[n * H + h] = gv;
    }
}

#define ASME_GRU_HP(HPV, ...)                                        \
    switch (HPV) {                                                   \
        case 16: { constexpr int HP = 16; __VA_ARGS__; } break;      \
        case 32: { constexpr int HP = 32; __VA_ARGS__; } break;      \
        case 48: { constexpr int HP = 48; __VA_ARGS__; } break;      \
        case 64: { constexpr int HP = 64; __VA_ARGS__; } break;      \
        case 80: { constexpr int HP = 80; __VA_ARGS__; } break;      \
        case 96: { constexpr int HP = 96; __VA_ARGS__; } break;      \
        case 112: { constexpr int HP = 112; __VA_ARGS__; } break;    \
        case 128: { constexpr int HP = 128; __VA_ARGS__; } break;    \
        default: set_error("gru: padded hidden size must be a multiple of 16 in [16, 128]"); return -1; \
    }

}  // namespace

// Forward recurrence of one GRU layer over (B, L) (batch_first).  gx: (B, L, 3*hp) = x W_ih^T + b_ih with the
// gate blocks (r, z, n) each hp wide; whh (3*hp, hp), bhh (3*hp) zero-padded beyond the real hidden size; h0 (B, hp)
// nullable (zeros).  Outputs hout (B, L, hp) and gates (B, L, 4, hp) for the backward.
ASME_API int asme_gru_fwd(const float* gx, const float* whh, const float* bhh, const float* h0, int64_t batch,
                          int64_t seq_len, int64_t hp, float* hout, float* gates, void* stream) {
    ASME_CHECK_ARG(gx && whh && bhh && hout && gates, "asme_gru_fwd: null pointer");
    ASME_CHECK_ARG(batch >= 0 && seq_len >= 1, "asme_gru_fwd: bad shape");
    if (batch == 0) return 0;
    const dim3 grid((unsigned)((batch + kRows - 1) / kRows));
    ASME_GRU_HP(hp, hipLaunchKernelGGL(gru_fwd_kernel<HP>, grid, dim3(HP / 16 * 64), 0, (hipStream_t)stream, gx, whh,
                                       bhh, h0, batch, seq_len, hout, gates));
    ASME_LAUNCH_CHECK("asme_gru_fwd");
}

// Backward through time of asme_gru_fwd: dhout (B, L, hp), dhT (B, hp) nullable; writes dgx, dgh (B, L, 3*hp)
// and dh0 (B, hp, nullable).  dW_ih / dW_hh / biases / dX are the caller's GEMMs over dgx and dgh.
ASME_API int asme_gru_bwd(const float* dhout, const float* dhT, const float* whh, const float* h0, const float* hout,
                          const float* gates, int64_t batch, int64_t seq_len, int64_t hp, float* dgx, float* dgh,
                          float* dh0, void* stream) {
    ASME_CHECK_ARG(dhout && whh && hout && gates && dgx && dgh, "asme_gru_bwd: null pointer");
    ASME_CHECK_ARG(batch >= 0 && seq_len >= 1, "asme_gru_bwd: bad shape");
    if (batch == 0) return 0;
    const dim3 grid((unsigned)((batch + kRows - 1) / kRows));
    ASME_GRU_HP(hp, hipLaunchKernelGGL(gru_bwd_kernel<HP>, grid, dim3(HP / 16 * 64), 0, (hipStream_t)stream, dhout,
                                       dhT, whh, h0, hout, gates, batch, seq_len, dgx, dgh, dh0));
    ASME_LAUNCH_CHECK("asme_gru_bwd");
}

// NARM local encoder forward: p1 (N, H) = A1 c_g, p2 (N, S, H) = A2 h_i, v (H), hs = h_i (N, S, H), mask (N, S) bytes
// (nonzero = real item); writes out = c_l (N, H) and alpha (N, S) (unmasked weights, for the backward).
ASME_API int asme_narm_attend_fwd(const float* p1, const float* p2, const float* v, const float* hs,
                                  const uint8_t* mask, int64_t n, int64_t s, int64_t h, float* out, float* alpha,
                                  void* stream) {
    ASME_CHECK_ARG(p1 && p2 && v && hs && mask && out && alpha, "asme_narm_attend_fwd: null pointer");
    ASME_CHECK_ARG(n >= 0 && s >= 1 && s <= 8192 && h >= 1, "asme_narm_attend_fwd: bad shape");
    if (n == 0) return 0;
    hipLaunchKernelGGL(narm_attend_fwd_kernel, dim3((unsigned)n), dim3(kAttThreads), (size_t)s * 4,
                       (hipStream_t)stream, p1, p2, v, hs, mask, s, h, out, alpha);
    ASME_LAUNCH_CHECK("asme_narm_attend_fwd");
}

// Backward of asme_narm_attend_fwd given dc = dL/dc_l (N, H): dp1 (N, H), dp2 (N, S, H), dhs (N, S, H) and the
// per-sequence partials dv_part (N, H) of dL/dv.
ASME_API int asme_narm_attend_bwd(const float* dc, const float* p1, const float* p2, const float* v, const float* hs,
                                  const uint8_t* mask, const float* alpha, int64_t n, int64_t s, int64_t h,
                                  float* dp1, float* dp2, float* dhs, float* dv_part, void* stream) {
    ASME_CHECK_ARG(dc && p1 && p2 && v && hs && mask && alpha && dp1 && dp2 && dhs && dv_part,
                   "asme_narm_attend_bwd: null pointer");
    ASME_CHECK_ARG(n >= 0 && s >= 1 && s <= 8192 && h >= 1, "asme_narm_attend_bwd: bad shape");
    if (n == 0) return 0;
    hipLaunchKernelGGL(narm_attend_bwd_kernel, dim3((unsigned)n), dim3(kAttThreads), (size_t)s * 8,
                       (hipStream_t)stream, dc, p1, p2, v, hs, mask, alpha, s, h, dp1, dp2, dhs, dv_part);
    ASME_LAUNCH_CHECK("asme_narm_attend_bwd");
}
