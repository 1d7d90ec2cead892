// Row layouts for the per-token kernels (embedding, LayerNorm, residual epilogues) on gfx950.
//
// A token row of D fp32 values is owned by LPR lanes of a 64-lane wave (64/LPR rows per wave).  Lane
// `sub` of a row holds NV chunks of W consecutive values at columns W*sub + W*LPR*j:
//   W = 4 (D % 4 == 0): global_load/store_dwordx4 and ONE Philox4x32-10 call per chunk (the 4 uniforms
//                       of counter idx/4 are exactly the chunk's 4 dropout decisions);
//   W = 1 (other D):    the scalar fallback, LPR = 64.
// LPR is the smallest power of two >= D/W (capped at 64), so D = 128 puts 2 rows in a wave and no lane
// idles.  Row reductions are xor butterflies inside the LPR-lane group.  The LayerNorm statistics and affine spell
// their fused multiply-adds out: clang's contractible a*b+c (llvm.fmuladd) is fused or not per call site, and kernels
// that must agree bit for bit (asme_residual_ln_fwd and the ws GEMM's residual-LN epilogue) inline these helpers in
// different surroundings.
#pragma once
#include "common.h"

namespace asme {

template <int W_, int LPR_, int NV_>
struct RowLayout {
    static constexpr int W = W_, LPR = LPR_, NV = NV_, RPW = 64 / LPR_;
    static __device__ __forceinline__ int col(int sub, int j) { return W * sub + W * LPR * j; }
};

template <class R>
using RowVals = float[R::NV][R::W];

template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}
// v(row r) + v(row r ^ 1) for 16-lane rows (v_permlane16_swap_b32) / v(half h) + v(half h ^ 1) for the two 32-lane
// halves (v_permlane32_swap_b32): VALU lane swaps of gfx950, same operand order in every lane
__device__ __forceinline__ float swap16_sum(float v) {
    const int i = __builtin_bit_cast(int, v);
    const auto r = __builtin_amdgcn_permlane16_swap(i, i, false, false);
    return __builtin_bit_cast(float, (int)r[0]) + __builtin_bit_cast(float, (int)r[1]);
}
__device__ __forceinline__ float swap32_sum(float v) {
    const int i = __builtin_bit_cast(int, v);
    const auto r = __builtin_amdgcn_permlane32_swap(i, i, false, false);
    return __builtin_bit_cast(float, (int)r[0]) + __builtin_bit_cast(float, (int)r[1]);
}

// Sum over the LPR-lane group, every lane gets the total.  No LDS-pipe shuffles (ds_bpermute: ~100-cycle latency
// each, 5 dependent ones per LayerNorm statistic at LPR = 32): DPP quad permutes for lane distance 1 and 2, then
// row_half_mirror / row_mirror (lanes of a group already agree on the partial sums, so a mirror pairs the same
// values as an xor), then the permlane swaps across 16-lane rows and wave halves.
template <int LPR>
__device__ __forceinline__ float row_sum(float v) {
    if constexpr (LPR >= 2) v += dpp_mov<0xB1>(v);    // quad_perm [1,0,3,2]
    if constexpr (LPR >= 4) v += dpp_mov<0x4E>(v);    // quad_perm [2,3,0,1]
    if constexpr (LPR >= 8) v += dpp_mov<0x141>(v);   // row_half_mirror
    if constexpr (LPR >= 16) v += dpp_mov<0x140>(v);  // row_mirror
    if constexpr (LPR >= 32) v = swap16_sum(v);
    if constexpr (LPR >= 64) v = swap32_sum(v);
    return v;
}
// sum over the rows sharing a wave (lanes with equal lane % LPR)
template <int LPR>
__device__ __forceinline__ float cross_row_sum(float v) {
#pragma unroll
    for (int o = LPR; o < 64; o <<= 1) v += __shfl_xor(v, o, 64);
    return v;
}

template <class R>
__device__ __forceinline__ void row_zero(RowVals<R>& x) {
#pragma unroll
    for (int j = 0; j < R::NV; ++j)
#pragma unroll
        for (int i = 0; i < R::W; ++i) x[j][i] = 0.f;
}

// NT: non-temporal loads (rows read once)
template <class R, bool NT>
__device__ __forceinline__ void row_load_p(const float* __restrict__ p, int sub, int D, RowVals<R>& x) {
#pragma unroll
    for (int j = 0; j < R::NV; ++j) {
        const int c = R::col(sub, j);
        if constexpr (R::W == 4 && NT) {
            typedef float f4v __attribute__((ext_vector_type(4)));
            const f4v v = c < D ? __builtin_nontemporal_load(reinterpret_cast<const f4v*>(p + c)) : f4v{0.f, 0.f, 0.f, 0.f};
            x[j][0] = v.x;
            x[j][1] = v.y;
            x[j][2] = v.z;
            x[j][3] = v.w;
        } else if constexpr (R::W == 4) {
            const float4 v = c < D ? *reinterpret_cast<const float4*>(p + c) : make_float4(0.f, 0.f, 0.f, 0.f);
            x[j][0] = v.x;
            x[j][1] = v.y;
            x[j][2] = v.z;
            x[j][3] = v.w;
        } else {
            x[j][0] = c < D ? p[c] : 0.f;
        }
    }
}
template <class R>
__device__ __forceinline__ void row_load(const float* __restrict__ p, int sub, int D, RowVals<R>& x) {
    row_load_p<R, false>(p, sub, D, x);
}

// NT: non-temporal (streaming) stores -- rows the next kernels read back from HBM anyway; a 1-read / 2-write row
// stream runs at 0.89 of 8 TB/s with them vs 0.79 cached (tools/probe/stream_probe.py)
template <class R, bool NT = false>
__device__ __forceinline__ void row_store(float* __restrict__ p, int sub, int D, const RowVals<R>& x) {
#pragma unroll
    for (int j = 0; j < R::NV; ++j) {
        const int c = R::col(sub, j);
        if (c >= D) continue;
        if constexpr (R::W == 4) {
            if constexpr (NT) {
                typedef float f4 __attribute__((ext_vector_type(4)));
                __builtin_nontemporal_store(f4{x[j][0], x[j][1], x[j][2], x[j][3]}, reinterpret_cast<f4*>(p + c));
            } else {
                *reinterpret_cast<float4*>(p + c) = make_float4(x[j][0], x[j][1], x[j][2], x[j][3]);
            }
        } else {
            p[c] = x[j][0];
        }
    }
}

// dropout keep factors (0 or 1/(1-p)) for the elements base + col of this lane (stream `salt`)
template <class R>
__device__ __forceinline__ void row_keep(uint64_t seed, uint32_t salt, uint64_t base, int sub, float p,
                                         RowVals<R>& f) {
    const float k = 1.f / (1.f - p);
#pragma unroll
    for (int j = 0; j < R::NV; ++j) {
        const uint64_t idx = base + (uint64_t)R::col(sub, j);
        if constexpr (R::W == 4) {
            float u[4];
            philox_uniform4(seed, salt, idx >> 2, u);
#pragma unroll
            for (int i = 0; i < 4; ++i) f[j][i] = u[i] >= p ? k : 0.f;
        } else {
            f[j][0] = dropout_factor(seed, salt, idx, p);
        }
    }
}

template <class R>
__device__ __forceinline__ void row_mul(RowVals<R>& x, const RowVals<R>& f) {
#pragma unroll
    for (int j = 0; j < R::NV; ++j)
#pragma unroll
        for (int i = 0; i < R::W; ++i) x[j][i] *= f[j][i];
}

// v / D: a multiply by the exact reciprocal when D is a power of two (every transformer width here: bit-identical to
// the division, without the ~10-instruction IEEE divide sequence per statistic per lane -- the row kernels are VALU-
// bound at 16 lanes per row), else the division
__device__ __forceinline__ float div_by_width(float v, int D) {
    return (D & (D - 1)) == 0 ? v * __builtin_bit_cast(float, (127 - (31 - __builtin_clz((unsigned)D))) << 23)
                              : v / (float)D;
}

template <class R>
__device__ __forceinline__ void row_ln_stats(const RowVals<R>& x, int sub, int D, float eps, float& mean,
                                             float& rstd) {
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < R::NV; ++j)
#pragma unroll
        for (int i = 0; i < R::W; ++i) s += x[j][i];  // out-of-row values are loaded as 0
    mean = div_by_width(row_sum<R::LPR>(s), D);
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < R::NV; ++j) {
        const bool ok = R::col(sub, j) < D;
#pragma unroll
        for (int i = 0; i < R::W; ++i) {
            const float c = ok ? x[j][i] - mean : 0.f;
            q = __builtin_fmaf(c, c, q);  // (explicit: a contractible a*b+c is fused or not per call site)
        }
    }
    rstd = rsqrtf(div_by_width(row_sum<R::LPR>(q), D) + eps);
}

// xhat = (x - mean) * rstd (0 outside the row)
template <class R>
__device__ __forceinline__ void row_normalise(const RowVals<R>& x, int sub, int D, float mean, float rstd,
                                              RowVals<R>& xh) {
#pragma unroll
    for (int j = 0; j < R::NV; ++j) {
        const bool ok = R::col(sub, j) < D;
#pragma unroll
        for (int i = 0; i < R::W; ++i) xh[j][i] = ok ? (x[j][i] - mean) * rstd : 0.f;
    }
}

// y = xh * w + b
template <class R>
__device__ __forceinline__ void row_affine(const RowVals<R>& xh, int sub, int D, const float* __restrict__ w,
                                           const float* __restrict__ b, RowVals<R>& y) {
    RowVals<R> wv, bv;
    row_load<R>(w, sub, D, wv);
    row_load<R>(b, sub, D, bv);
#pragma unroll
    for (int j = 0; j < R::NV; ++j)
#pragma unroll
        for (int i = 0; i < R::W; ++i) y[j][i] = __builtin_fmaf(xh[j][i], wv[j][i], bv[j][i]);
}

// LayerNorm input gradient: gx = rstd * (gy*w - mean(gy*w) - xhat * mean(gy*w*xhat))
template <class R>
__device__ __forceinline__ void row_ln_bwd(const RowVals<R>& gy, const RowVals<R>& xh, const float* __restrict__ w,
                                           float rstd, int sub, int D, RowVals<R>& gx) {
    RowVals<R> wv, dxh;
    row_load<R>(w, sub, D, wv);
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int j = 0; j < R::NV; ++j)
#pragma unroll
        for (int i = 0; i < R::W; ++i) {
            dxh[j][i] = gy[j][i] * wv[j][i];
            a += dxh[j][i];
            b += dxh[j][i] * xh[j][i];
        }
    a = div_by_width(row_sum<R::LPR>(a), D);
    b = div_by_width(row_sum<R::LPR>(b), D);
#pragma unroll
    for (int j = 0; j < R::NV; ++j)
#pragma unroll
        for (int i = 0; i < R::W; ++i) gx[j][i] = rstd * (dxh[j][i] - a - xh[j][i] * b);
}

// Per-block column partials of NACC accumulators: rows of a wave are summed by butterflies, the
// waves of the block through LDS (fixed order), and partials[blockIdx.x][k][D] is written.
template <class R, int NACC, int NWAVES>
__device__ __forceinline__ void write_row_partials(float (&acc)[NACC][R::NV][R::W], int lane, int wave, int D,
                                                   float* __restrict__ partials) {
    extern __shared__ __attribute__((aligned(16))) float red[];  // [NWAVES][NACC][D]
#pragma unroll
    for (int k = 0; k < NACC; ++k)
#pragma unroll
        for (int j = 0; j < R::NV; ++j)
#pragma unroll
            for (int i = 0; i < R::W; ++i) acc[k][j][i] = cross_row_sum<R::LPR>(acc[k][j][i]);
    if (lane < R::LPR) {
#pragma unroll
        for (int k = 0; k < NACC; ++k)
#pragma unroll
            for (int j = 0; j < R::NV; ++j) {
                const int c = R::col(lane, j);
                if (c >= D) continue;
#pragma unroll
                for (int i = 0; i < R::W; ++i) red[(wave * NACC + k) * D + c + i] = acc[k][j][i];
            }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < NACC * D; c += blockDim.x) {
        float s = 0.f;
        for (int w = 0; w < NWAVES; ++w) s += red[w * NACC * D + c];
        partials[(int64_t)blockIdx.x * NACC * D + c] = s;
    }
}

// Calls f(RowLayout<...>{}) for the layout of hidden size D (1 <= D <= 512).
template <class F>
inline int with_row_layout(int64_t D, F&& f) {
    if (D < 1 || D > 512) {
        set_error("hidden size must be in [1, 512]");
        return -1;
    }
    if (D % 4 == 0) {
        const int64_t n4 = D / 4;
        if (n4 <= 4) f(RowLayout<4, 4, 1>{});
        else if (n4 <= 8) f(RowLayout<4, 8, 1>{});
        else if (n4 <= 16) f(RowLayout<4, 16, 1>{});
        else if (n4 <= 32) f(RowLayout<4, 32, 1>{});
        else if (n4 <= 64) f(RowLayout<4, 64, 1>{});
        else f(RowLayout<4, 64, 2>{});
        return 0;
    }
    switch ((D + 63) / 64) {
        case 1: f(RowLayout<1, 64, 1>{}); break;
        case 2: f(RowLayout<1, 64, 2>{}); break;
        case 3: f(RowLayout<1, 64, 3>{}); break;
        case 4: f(RowLayout<1, 64, 4>{}); break;
        case 5: f(RowLayout<1, 64, 5>{}); break;
        case 6: f(RowLayout<1, 64, 6>{}); break;
        case 7: f(RowLayout<1, 64, 7>{}); break;
        default: f(RowLayout<1, 64, 8>{}); break;
    }
    return 0;
}

}  // namespace asme
