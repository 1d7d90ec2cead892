// Adam element update shared by the optimizer kernels (adam.hip) and the fused table-gradient apply
// (sharding.hip): one definition, so every path computes bit-identical results.
#pragma once
#include <hip/hip_runtime.h>

namespace asme {

struct AdamHyper {
    float b1, b2, one_minus_b1, one_minus_b2, eps, wd, neg_step_size, inv_bc2_sqrt;
};

// The update is written with explicit fused multiply-adds and no other contraction, so the per-element result
// does not depend on the kernel the function is inlined into: the lazy catch-up must replay the dense update bit
// for bit.  (FMA: one rounding where torch's sequence has two -- at least as accurate; 9 packed operations + 4
// transcendentals per element pair instead of 13 + 4, and the replay is VALU-bound.)  sqrt and the reciprocal
// are the hardware v_sqrt_f32 / v_rcp_f32 (1 ulp) and 1/sqrt(bc2) is a host-precomputed multiplier: a few ulp
// from torch's correctly rounded sequence (far inside the 1e-3 parity bound).
//   g' = g + wd p;  m' = m + (1-b1)(g' - m);  v' = b2 v + ((1-b2) g') g';  p' = p - s m' / (sqrt(v') / sqrt(bc2) + eps)
__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, const AdamHyper& hp) {
#pragma clang fp contract(off)
    if (hp.wd != 0.f) g = __builtin_fmaf(hp.wd, p, g);
    m = __builtin_fmaf(hp.one_minus_b1, g - m, m);
    v = __builtin_fmaf(hp.b2, v, (hp.one_minus_b2 * g) * g);
    const float denom = __builtin_fmaf(__builtin_amdgcn_sqrtf(v), hp.inv_bc2_sqrt, hp.eps);
    p = __builtin_fmaf(hp.neg_step_size, m * __builtin_amdgcn_rcpf(denom), p);
}

// The same update on 4 consecutive elements as two packed pairs (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32:
// IEEE results identical to adam_elem's scalar ops, same order) -- half the VALU issue of the scalar form.
typedef float float2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float2v fma2(float2v a, float2v b, float2v c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ float2v bc2(float x) { return float2v{x, x}; }
__device__ __forceinline__ void adam_elem2(float2v& p, float2v g, float2v& m, float2v& v, const AdamHyper& hp) {
#pragma clang fp contract(off)
    if (hp.wd != 0.f) g = fma2(bc2(hp.wd), p, g);
    m = fma2(bc2(hp.one_minus_b1), g - m, m);
    v = fma2(bc2(hp.b2), v, (hp.one_minus_b2 * g) * g);
    const float2v s = {__builtin_amdgcn_sqrtf(v.x), __builtin_amdgcn_sqrtf(v.y)};
    const float2v d = fma2(s, bc2(hp.inv_bc2_sqrt), bc2(hp.eps));
    const float2v r = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
    p = fma2(bc2(hp.neg_step_size), m * r, p);
}
__device__ __forceinline__ void adam_elem4(float4& P, const float4& G, float4& M, float4& V, const AdamHyper& hp) {
    float2v p0 = {P.x, P.y}, p1 = {P.z, P.w}, m0 = {M.x, M.y}, m1 = {M.z, M.w}, v0 = {V.x, V.y}, v1 = {V.z, V.w};
    adam_elem2(p0, float2v{G.x, G.y}, m0, v0, hp);
    adam_elem2(p1, float2v{G.z, G.w}, m1, v1, hp);
    P = make_float4(p0.x, p0.y, p1.x, p1.y);
    M = make_float4(m0.x, m0.y, m1.x, m1.y);
    V = make_float4(v0.x, v0.y, v1.x, v1.y);
}

// adam_elem with g == 0 and no weight decay (the lazy replay's step), with the same IEEE result op for op:
// fma(c, 0 - m, m) == fma(-c, m, m) (c * (-m) == -(c * m) exactly); (1 - b2) * 0 * 0 == +0 and b2 * v >= +0
// (v never goes negative), so fma(b2, v, +0) == b2 * v rounded.  2 of the 9 operations disappear.
__device__ __forceinline__ void adam_decay(float& p, float& m, float& v, const AdamHyper& hp) {
#pragma clang fp contract(off)
    m = __builtin_fmaf(-hp.one_minus_b1, m, m);
    v = v * hp.b2;
    const float denom = __builtin_fmaf(__builtin_amdgcn_sqrtf(v), hp.inv_bc2_sqrt, hp.eps);
    p = __builtin_fmaf(hp.neg_step_size, m * __builtin_amdgcn_rcpf(denom), p);
}
__device__ __forceinline__ void adam_decay2(float2v& p, float2v& m, float2v& v, const AdamHyper& hp) {
#pragma clang fp contract(off)
    m = fma2(bc2(-hp.one_minus_b1), m, m);
    v = v * hp.b2;
    const float2v s = {__builtin_amdgcn_sqrtf(v.x), __builtin_amdgcn_sqrtf(v.y)};
    const float2v d = fma2(s, bc2(hp.inv_bc2_sqrt), bc2(hp.eps));
    const float2v r = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
    p = fma2(bc2(hp.neg_step_size), m * r, p);
}

// A row AT REST: its moments are exactly +0 and every step it missed ran without weight decay -- a fresh table's
// rows before their first gradient (the lazy state marks them with last_step = kRestStep while the group's weight
// decay is 0, ops.LazyTableState).  The dense zero-gradient update of such a row is the identity bit for bit
// (adam_elem: m' = fma(c, +0 - +0, +0) = +0, v' = fma(b2, +0, +0) = +0, denom = eps, p' = fma(s, +0 * rcp(eps), p)
// = p), so the row is current at every step: the replay kernels take its last step as `upto` (no replay, nothing
// read for it by the flush, last_step left at rest until a real gradient step writes it).
constexpr int32_t kRestStep = -1;
__device__ __forceinline__ int32_t lazy_from(int32_t last, int32_t upto) { return last < 0 ? upto : last; }

}  // namespace asme
