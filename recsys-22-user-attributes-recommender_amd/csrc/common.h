// Shared device helpers for the ASME MI355X (gfx950) kernels.
// Wave = 64 lanes. All reductions below are full-wave (64-lane) butterflies.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#define ASME_API extern "C" __attribute__((visibility("default")))

namespace asme {

// ------------------------------------------------------------------ status
void set_error(const std::string& msg);
int hip_status(hipError_t e, const char* where);

#define ASME_CHECK_ARG(cond, msg)            \
    do {                                     \
        if (!(cond)) {                       \
            ::asme::set_error(msg);          \
            return -1;                       \
        }                                    \
    } while (0)

#define ASME_LAUNCH_CHECK(where) return ::asme::hip_status(hipGetLastError(), where)

// ------------------------------------------------------------------ wave ops
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}
// reduce over the 4 lane-groups {l, l^16, l^32, l^48} (the MFMA 16x16 "row group" dimension).  (The gfx950
// v_permlane16/32_swap form of these two measured 1-3 % slower inside the attention kernels: kept on ds_bpermute.)
__device__ __forceinline__ float group4_sum(float v) {
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    return v;
}
__device__ __forceinline__ float group4_max(float v) {
    v = fmaxf(v, __shfl_xor(v, 16, 64));
    v = fmaxf(v, __shfl_xor(v, 32, 64));
    return v;
}
// reduce over the 16 lanes that share (l >> 4)
__device__ __forceinline__ float lane16_sum(float v) {
#pragma unroll
    for (int o = 8; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// ------------------------------------------------------------------ Philox4x32-10
struct u32x4 {
    uint32_t x, y, z, w;
};
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);  // v_bitop3_b32, truth table a^b^c
}
// Each round's two 32x32->64 products are single v_mad_u64_u32 (instead of a mul_hi + mul_lo pair) and
// the key mix a single v_bitop3_b32 (keys must be wave-uniform: kernel arguments).
__device__ __forceinline__ u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
    const uint64_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
    k0 = __builtin_amdgcn_readfirstlane(k0);
    k1 = __builtin_amdgcn_readfirstlane(k1);
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = M0 * c.x, p1 = M1 * c.z;
        c = u32x4{xor3((uint32_t)(p1 >> 32), c.y, k0), (uint32_t)p1, xor3((uint32_t)(p0 >> 32), c.w, k1),
                  (uint32_t)p0};
        k0 += W0;
        k1 += W1;
    }
    return c;
}
// 4 uniforms in [0,1) for the 4 consecutive elements starting at (idx & ~3) of stream `salt`.
__device__ __forceinline__ void philox_uniform4(uint64_t seed, uint32_t salt, uint64_t idx4, float u[4]) {
    u32x4 c{(uint32_t)idx4, (uint32_t)(idx4 >> 32), salt, 0x5851F42Du};
    u32x4 r = philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    const float s = 5.9604644775390625e-08f;  // 2^-24
    u[0] = (float)(r.x >> 8) * s;
    u[1] = (float)(r.y >> 8) * s;
    u[2] = (float)(r.z >> 8) * s;
    u[3] = (float)(r.w >> 8) * s;
}
// GELU-dropout decisions (salt 5, the FFN activation): one Philox4x32-10 block serves the PAIR of 4-element chunks
// (c & ~4, c | 4) -- 8 16-bit uniforms, x and y for the even chunk, z and w for the odd one; element kept iff
// u16 >= round(p * 65536).  A fused-GEMM lane holds two such chunks (16 features apart), so it runs one block for
// both; the row kernels run it per chunk and take their half.  Returns bit i = keep element i of the even chunk,
// bit 4 + i = of the odd chunk.
__device__ __forceinline__ uint32_t gelu_thresh(float p) { return (uint32_t)(p * 65536.f + 0.5f); }
__device__ __forceinline__ uint32_t gelu_keep_bits8(uint64_t seed, uint64_t chunk, uint32_t thr) {
    const uint64_t key = chunk & ~(uint64_t)4;
    u32x4 c{(uint32_t)key, (uint32_t)(key >> 32), 5u, 0x5851F42Du};
    const u32x4 r = philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    uint32_t m = 0;
    m |= ((r.x & 0xFFFFu) >= thr ? 1u : 0u) | ((r.x >> 16) >= thr ? 2u : 0u);
    m |= ((r.y & 0xFFFFu) >= thr ? 4u : 0u) | ((r.y >> 16) >= thr ? 8u : 0u);
    m |= ((r.z & 0xFFFFu) >= thr ? 16u : 0u) | ((r.z >> 16) >= thr ? 32u : 0u);
    m |= ((r.w & 0xFFFFu) >= thr ? 64u : 0u) | ((r.w >> 16) >= thr ? 128u : 0u);
    return m;
}
// this chunk's 4 decisions
__device__ __forceinline__ uint32_t gelu_keep_bits4(uint64_t seed, uint64_t chunk, uint32_t thr) {
    return (gelu_keep_bits8(seed, chunk, thr) >> (((uint32_t)(chunk >> 2) & 1u) * 4u)) & 0xFu;
}
// keep bit b of `bits` -> the factor k (kept) or +0 (dropped): the sign-extended one-bit field (v_bfe_i32: 0 or -1)
// ANDed with k's bits -- two VALU instead of extract, compare and select; x * factor is the same value either way
__device__ __forceinline__ float keep_factor_bit(uint32_t bits, int b, float k) {
    return __int_as_float(__builtin_amdgcn_sbfe((int)bits, (unsigned)b, 1u) & __float_as_int(k));
}
__device__ __forceinline__ void gelu_keep_factors(uint32_t bits4, float k, float (&u)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) u[i] = keep_factor_bit(bits4, i, k);
}
__device__ __forceinline__ float gelu_keep_factor(uint64_t seed, uint64_t idx, float p) {
    return (gelu_keep_bits4(seed, idx >> 2, gelu_thresh(p)) >> (idx & 3)) & 1u ? 1.0f / (1.0f - p) : 0.0f;
}

// dropout keep-factor for element `idx`: 0 (dropped) or 1/(1-p)
__device__ __forceinline__ float dropout_factor(uint64_t seed, uint32_t salt, uint64_t idx, float p) {
    float u[4];
    philox_uniform4(seed, salt, idx >> 2, u);
    const uint32_t k = (uint32_t)idx & 3u;
    const float v = k == 0 ? u[0] : (k == 1 ? u[1] : (k == 2 ? u[2] : u[3]));
    return v >= p ? 1.0f / (1.0f - p) : 0.0f;
}

// GELU(x) = x * Phi(x), Phi(x) = 0.5 * (1 + erf(x / sqrt 2)) (nn.GELU(), the exact-erf form the reference uses) and
// its derivative Phi(x) + x * phi(x).  Phi from erfc: erfc(a) = t * exp(-a^2) * Q(t), t = 1 / (1 + a / 2), where Q
// is a degree-10 weighted Chebyshev fit of erfcx(a) / t over t in (0, 1] (every a >= 0; relative error 4e-8, so the
// negative tail keeps its RELATIVE accuracy), and 1 + erf(z) = 2 - erfc(z) for z >= 0, erfc(-z) below.  With
// a^2 = x^2 / 2 the exponential is phi's own, so both values cost one reciprocal, ONE exponential and eleven FMAs
// (the FFN epilogues evaluate them for all T x 4d activations and are VALU-bound on them; libm's erff alone is 56
// instructions for the pair).  The coefficients carry Phi's 1/2.
__device__ __forceinline__ void gelu_erf_and_grad(float x, float& gelu, float& grad) {
    const float a = fabsf(x) * 0.70710678118654752f;
    const float t = __builtin_amdgcn_rcpf(1.0f + 0.5f * a);
    float q = 0.022210972383618355f;
    q = fmaf(q, t, -0.12038972973823547f);
    q = fmaf(q, t, 0.2531980574131012f);
    q = fmaf(q, t, -0.23490440845489502f);
    q = fmaf(q, t, 0.07135776430368423f);
    q = fmaf(q, t, -0.03194592893123627f);
    q = fmaf(q, t, 0.04737446457147598f);
    q = fmaf(q, t, 0.08755350857973099f);
    q = fmaf(q, t, 0.12345138192176819f);
    q = fmaf(q, t, 0.14104652404785156f);
    q = fmaf(q, t, 0.141047403216362f);
    const float e = __expf(-0.5f * x * x);  // exp(-a^2) = sqrt(2 pi) phi(x)
    const float h = t * e * q;              // erfc(a) / 2
    const float cdf = x >= 0.f ? 1.0f - h : h;
    gelu = x * cdf;
    grad = fmaf(x * 0.3989422804014327f, e, cdf);
}
__device__ __forceinline__ float gelu_erf(float x) {
    float g, d;
    gelu_erf_and_grad(x, g, d);
    return g;
}
__device__ __forceinline__ float gelu_erf_grad(float x) {
    float g, d;
    gelu_erf_and_grad(x, g, d);
    return d;
}

// ---- fp32 products on the bf16 matrix cores (bf16x6)
// gfx950's fp32-input MFMA runs at 1/16 of the bf16 rate.  An fp32 value splits exactly into three bf16
// terms x = h + m + l (h = bf16(x), m = bf16(x - h), l = bf16(x - h - m): 8 significant bits each, the
// differences exact in fp32), and a product a*b is kept to 2^-16 of its size by the six terms
// mm + hl + lh + hm + mh + hh (dropped: ml, lm ~2^-24, ll ~2^-32 -- below fp32's own rounding).  Each bf16
// MFMA product is exact in fp32, so six 16x16x32 bf16 MFMAs (6 x 16 cycles per 32 k) give an fp32 tile at
// 2.7x the rate of eight 16x16x4 fp32 MFMAs (8 x 32 cycles).  Measured against float64
// (tools/probe/bf16x6_probe.py: K = 128 / 512, normal, uniform and wide-range data) the error is at or below
// the fp32 MFMA's: max 2.8e-7 vs 2.8e-7, mean 1.5e-8 vs 2.0e-8 of sum |a*b| (K = 128, normal).
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

// Stores of item-table rows (the optimizer's p / m / v write-back): a row is not read again until a later step
// touches it, so they carry the non-temporal hint instead of displacing the step's working set from the L2 / MALL.
#ifndef ASME_TABLE_NT
#define ASME_TABLE_NT 1
#endif
__device__ __forceinline__ void table_store4(float* p, const float4& v) {
#if ASME_TABLE_NT
    __builtin_nontemporal_store(floatx4{v.x, v.y, v.z, v.w}, reinterpret_cast<floatx4*>(p));
#else
    *reinterpret_cast<float4*>(p) = v;
#endif
}
__device__ __forceinline__ void table_store2(float* p, float a, float b) {
#if ASME_TABLE_NT
    typedef float floatx2_t __attribute__((ext_vector_type(2)));
    __builtin_nontemporal_store(floatx2_t{a, b}, reinterpret_cast<floatx2_t*>(p));
#else
    *reinterpret_cast<float2*>(p) = make_float2(a, b);
#endif
}

struct Bf3 {
    bf16x8 h, m, l;
};
__device__ __forceinline__ Bf3 split_bf3(const float4& a, const float4& b) {
    const float x[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    Bf3 s;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const __bf16 h = (__bf16)x[j];
        const float r = x[j] - (float)h;
        const __bf16 m = (__bf16)r;
        s.h[j] = h;
        s.m[j] = m;
        s.l[j] = (__bf16)(r - (float)m);
    }
    return s;
}
// acc += a . b over one 32-k block, smallest terms first
__device__ __forceinline__ floatx4 mfma_bf3(const Bf3& a, const Bf3& b, floatx4 acc) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.m, b.m, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.h, b.l, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.l, b.h, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.h, b.m, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.m, b.h, acc, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.h, b.h, acc, 0, 0, 0);
}

typedef float floatx16 __attribute__((ext_vector_type(16)));

// acc += a . b over one 16-k step of v_mfma_f32_32x32x16_bf16, the six bf16x6 terms smallest first
__device__ __forceinline__ floatx16 mfma32_bf3(const Bf3& a, const Bf3& b, floatx16 acc) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.m, b.m, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.h, b.l, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.l, b.h, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.h, b.m, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.m, b.h, acc, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.h, b.h, acc, 0, 0, 0);
}

}  // namespace asme
