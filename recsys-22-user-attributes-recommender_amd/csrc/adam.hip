// Fused dense Adam (L2 weight decay coupled into the gradient) over many tensors in one launch.
//
// Reference semantics: torch.optim.Adam as configured by
//   SequenceNextItemPredictionTrainingModule.configure_optimizers
//       core/modules/sequence_next_item_prediction_training_module.py:181-185   (wd 1e-3)
//   BaseNextItemPredictionTrainingModule.configure_optimizers
//       core/modules/next_item_prediction_training_module.py:134-138            (wd 0)
//   MaskedTrainingModule.configure_optimizers + LambdaLR warmup
//       core/modules/masked_training_module.py:165-189                          (no wd)
// Per element (fp32, torch's single-tensor Adam; the products fused with their sums, see adam_elem):
//   g  = grad + wd * p
//   m  = m + (1 - b1) * (g - m)                (lerp)
//   v  = v * b2 + (1 - b2) * g * g
//   p  = p + (-step_size) * (m / (sqrt(v) / sqrt(bc2) + eps)),  step_size = lr / bc1
//   (evaluated as m * rcp(sqrt(v) * (1/sqrt(bc2)) + eps) with the hardware sqrt / rcp, see adam_elem)
// Every row of the item table is updated every step: this is the largest HBM stream of the
// training step (7 x |V| x d x 4 B), so the kernel is a pure float4 streaming pass.
//
// The "sparse-gradient" variant takes the table gradient as a compact list of (row, grad-row) pairs
// (row_slot[r] = index into grad_rows or -1) and applies the exact same dense update (g = 0 + wd*p for
// rows without a gradient), saving the dense-gradient write/zero/read traffic.
#include "adam_math.h"
#include "common.h"
#include <algorithm>
#include <cmath>

using namespace asme;

namespace {

constexpr int kMaxTensors = 40;
constexpr int kChunk = 8192;  // elements per block

struct AdamList {
    float* p[kMaxTensors];
    const float* g[kMaxTensors];
    float* m[kMaxTensors];
    float* v[kMaxTensors];
    int64_t n[kMaxTensors];
    int64_t chunk_start[kMaxTensors + 1];
    int count;
};

// one zero-gradient step (weight decay keeps the general form: its gradient wd * p is not zero)
__device__ __forceinline__ void adam_zero_grad_step(float& p, float& m, float& v, const AdamHyper& hp) {
    if (hp.wd != 0.f)
        adam_elem(p, 0.f, m, v, hp);
    else
        adam_decay(p, m, v, hp);
}
__device__ __forceinline__ void adam_zero_grad_step4(float4& P, float4& M, float4& V, const AdamHyper& hp) {
    if (hp.wd != 0.f) {
        adam_elem4(P, make_float4(0.f, 0.f, 0.f, 0.f), M, V, hp);
        return;
    }
    float2v p0 = {P.x, P.y}, p1 = {P.z, P.w}, m0 = {M.x, M.y}, m1 = {M.z, M.w}, v0 = {V.x, V.y}, v1 = {V.z, V.w};
    adam_decay2(p0, m0, v0, hp);
    adam_decay2(p1, m1, v1, hp);
    P = make_float4(p0.x, p0.y, p1.x, p1.y);
    M = make_float4(m0.x, m0.y, m1.x, m1.y);
    V = make_float4(v0.x, v0.y, v1.x, v1.y);
}

__global__ __launch_bounds__(256) void adam_multi_kernel(AdamList L, AdamHyper hp) {
    const int64_t blk = blockIdx.x;
    int ti = 0;
    while (ti + 1 < L.count && L.chunk_start[ti + 1] <= blk) ++ti;
    const int64_t n = L.n[ti];
    const int64_t base = (blk - L.chunk_start[ti]) * kChunk;
    float* __restrict__ p = L.p[ti];
    const float* __restrict__ g = L.g[ti];
    float* __restrict__ m = L.m[ti];
    float* __restrict__ v = L.v[ti];
    const bool vec = (((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) == 0;
    const int64_t end = min(n, base + kChunk);
    if (vec) {
        for (int64_t i = base + 4 * threadIdx.x; i + 3 < end; i += 4 * blockDim.x) {
            float4 P = *reinterpret_cast<const float4*>(p + i);
            const float4 G = g ? *reinterpret_cast<const float4*>(g + i) : make_float4(0.f, 0.f, 0.f, 0.f);
            float4 M = *reinterpret_cast<const float4*>(m + i);
            float4 Vv = *reinterpret_cast<const float4*>(v + i);
            adam_elem4(P, G, M, Vv, hp);
            *reinterpret_cast<float4*>(p + i) = P;
            *reinterpret_cast<float4*>(m + i) = M;
            *reinterpret_cast<float4*>(v + i) = Vv;
        }
        const int64_t tail = base + ((end - base) / 4) * 4;
        for (int64_t i = tail + threadIdx.x; i < end; i += blockDim.x) adam_elem(p[i], g ? g[i] : 0.f, m[i], v[i], hp);
    } else {
        for (int64_t i = base + threadIdx.x; i < end; i += blockDim.x) adam_elem(p[i], g ? g[i] : 0.f, m[i], v[i], hp);
    }
}

// dense update of a (rows x D) table whose gradient is given sparsely: row r has gradient
// grad_rows[row_slot[r]] if row_slot[r] >= 0, else zero.  One thread = 4 consecutive floats.
__global__ __launch_bounds__(256) void adam_rows_kernel(float* __restrict__ p, float* __restrict__ m,
                                                        float* __restrict__ v, int64_t rows, int D,
                                                        const int32_t* __restrict__ row_slot,
                                                        const float* __restrict__ grad_rows, AdamHyper hp) {
    const int64_t nvec = rows * D / 4;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t e = i * 4;
        const int64_t r = e / D;
        const int c = (int)(e - r * D);
        const int32_t slot = row_slot[r];
        float4 G = make_float4(0.f, 0.f, 0.f, 0.f);
        if (slot >= 0) G = *reinterpret_cast<const float4*>(grad_rows + (int64_t)slot * D + c);
        float4 P = *reinterpret_cast<const float4*>(p + e);
        float4 M = *reinterpret_cast<const float4*>(m + e);
        float4 Vv = *reinterpret_cast<const float4*>(v + e);
        adam_elem4(P, G, M, Vv, hp);
        *reinterpret_cast<float4*>(p + e) = P;
        *reinterpret_cast<float4*>(m + e) = M;
        *reinterpret_cast<float4*>(v + e) = Vv;
    }
}

AdamHyper make_hyper(float lr, float b1, float b2, float eps, float wd, int64_t step) {
    AdamHyper h;
    h.b1 = b1;
    h.b2 = b2;
    h.one_minus_b1 = 1.f - b1;
    h.one_minus_b2 = 1.f - b2;
    h.eps = eps;
    h.wd = wd;
    const double bc1 = 1.0 - std::pow((double)b1, (double)step);
    const double bc2 = 1.0 - std::pow((double)b2, (double)step);
    h.neg_step_size = (float)(-(double)lr / bc1);
    h.inv_bc2_sqrt = (float)(1.0 / std::sqrt(bc2));
    return h;
}

}  // namespace

ASME_API int asme_adam_step(int n_tensors, float* const* params, const float* const* grads, float* const* exp_avg,
                            float* const* exp_avg_sq, const int64_t* numels, float lr, float beta1, float beta2,
                            float eps, float weight_decay, int64_t step, void* stream) {
    ASME_CHECK_ARG(n_tensors >= 0 && params && exp_avg && exp_avg_sq && numels, "asme_adam_step: bad argument");
    ASME_CHECK_ARG(step >= 1, "asme_adam_step: step must be >= 1");
    const AdamHyper hp = make_hyper(lr, beta1, beta2, eps, weight_decay, step);
    int i = 0;
    while (i < n_tensors) {
        AdamList L{};
        int64_t blocks = 0;
        int c = 0;
        for (; i < n_tensors && c < kMaxTensors; ++i) {
            if (numels[i] == 0) continue;
            L.p[c] = params[i];
            L.g[c] = grads ? grads[i] : nullptr;
            L.m[c] = exp_avg[i];
            L.v[c] = exp_avg_sq[i];
            L.n[c] = numels[i];
            L.chunk_start[c] = blocks;
            blocks += (numels[i] + kChunk - 1) / kChunk;
            ++c;
        }
        L.chunk_start[c] = blocks;
        L.count = c;
        if (c == 0) break;
        hipLaunchKernelGGL(adam_multi_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, L, hp);
        const int rc = hip_status(hipGetLastError(), "asme_adam_step");
        if (rc) return rc;
    }
    return 0;
}

ASME_API int asme_adam_rows_step(float* param, float* exp_avg, float* exp_avg_sq, int64_t rows, int64_t dim,
                                 const int32_t* row_slot, const float* grad_rows, float lr, float beta1, float beta2,
                                 float eps, float weight_decay, int64_t step, void* stream) {
    ASME_CHECK_ARG(param && exp_avg && exp_avg_sq && row_slot && grad_rows, "asme_adam_rows_step: null pointer");
    ASME_CHECK_ARG(dim % 4 == 0 && step >= 1, "asme_adam_rows_step: dim must be a multiple of 4");
    const AdamHyper hp = make_hyper(lr, beta1, beta2, eps, weight_decay, step);
    const int64_t nvec = rows * dim / 4;
    const int64_t blocks = std::min<int64_t>((nvec + 255) / 256, 256 * 32);
    if (nvec == 0) return 0;
    hipLaunchKernelGGL(adam_rows_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, param, exp_avg,
                       exp_avg_sq, rows, (int)dim, row_slot, grad_rows, hp);
    ASME_LAUNCH_CHECK("asme_adam_rows_step");
}

// ------------------------------------------------------------------------------------------------
// Lazy dense Adam ("exact catch-up").  Dense Adam (every row, every step) on a row whose gradient is
// zero for a run of steps is a deterministic recurrence in (p, m, v) and the per-step constants.  We
// keep, per table row, the step it is up to date with (last_step) and a device history of the per-step
// hyper-parameters; a row is brought up to date by replaying exactly the fp32 operations the dense
// kernel would have executed (same adam_elem, same constants, same order), only when its value is
// needed: before a forward that gathers it, and in a full flush before anything else reads the table.
// The result is bit-identical to running asme_adam_rows_step every step; the HBM traffic per step
// drops from 6 x |V| x d x 4 B to 6 x U x d x 4 B (U = unique rows of the step).
namespace {

static_assert(sizeof(AdamHyper) == 8 * sizeof(float), "hist row = 8 floats");

// hist row 0 is never a step (steps start at 1); its first word holds, as an int32, the first step of the current
// run of steps with identical (b1, b2, 1-b1, 1-b2, eps, wd): hist[t] for t in [const_from, latest recorded step] differ
// at most in neg_step_size / inv_bc2_sqrt.  A replay that starts at or after it reads those two per step and keeps
// the rest in registers (replay_const).  Each step is compared with the row recorded before it (bitwise); a step whose
// predecessor was never recorded (step 1, a resumed run) opens a new run -- rows never replay a step at or before
// the step the lazy state was started at, so the chain only has to hold over steps recorded in order.
__device__ __forceinline__ bool same_consts(const AdamHyper& a, const AdamHyper& b) {
    return __float_as_uint(a.b1) == __float_as_uint(b.b1) && __float_as_uint(a.b2) == __float_as_uint(b.b2) &&
           __float_as_uint(a.one_minus_b1) == __float_as_uint(b.one_minus_b1) &&
           __float_as_uint(a.one_minus_b2) == __float_as_uint(b.one_minus_b2) &&
           __float_as_uint(a.eps) == __float_as_uint(b.eps) && __float_as_uint(a.wd) == __float_as_uint(b.wd);
}
__global__ void record_step_kernel(float* __restrict__ hist, int64_t step, AdamHyper hp) {
    if (threadIdx.x == 0) {
        AdamHyper* h = reinterpret_cast<AdamHyper*>(hist);
        int32_t* const_from = reinterpret_cast<int32_t*>(hist);
        const bool same = step > 1 && same_consts(h[step - 1], hp);
        const int32_t cf = *const_from;
        *const_from = same ? min(cf, (int32_t)step) : (int32_t)step;
        h[step] = hp;
    }
}

// The zero-gradient replay of steps t0+1..upto on a wave's element pairs.  When the whole range lies in the current
// run of constant (b1, b2, eps, wd) (hist row 0, above), only the two step-dependent constants are read per step, the
// next step's pair one iteration ahead (scalar loads off the recurrence), and the weight-decay branch is taken once;
// otherwise every step's full constants are read as before.  Same adam_elem2 / adam_decay2 operations: same bits.
#ifndef ASME_REPLAY_CONST
#define ASME_REPLAY_CONST 1
#endif
template <int NP>
__device__ __forceinline__ void replay_steps(float2v (&P)[NP], float2v (&M)[NP], float2v (&Vv)[NP],
                                             const AdamHyper* __restrict__ hist, int32_t t0, int32_t upto,
                                             int32_t const_from) {
    if (ASME_REPLAY_CONST && t0 + 1 >= const_from) {
        if (t0 >= upto) return;
        AdamHyper hp = hist[upto];
        const float2* __restrict__ lr = reinterpret_cast<const float2*>(hist) + 3;  // (neg_step_size, inv_bc2_sqrt)
        // two steps per trip, their constants loaded a trip ahead: the scalar loads' wait sits behind two steps of
        // vector work, and the loop and address arithmetic (which had matched the replay's VALU count one for one in
        // the flush's PMC pass: SALU 482M vs VALU 455M) is paid once per two steps
        float2 n0 = lr[4 * (t0 + 1)], n1 = lr[4 * min(t0 + 2, upto)];
        int32_t t = t0 + 1;
        auto steps = [&](auto op) {
            auto two = [&](const float2 c0, const float2 c1) {
                hp.neg_step_size = c0.x;
                hp.inv_bc2_sqrt = c0.y;
#pragma unroll
                for (int j = 0; j < NP; ++j) op(P[j], M[j], Vv[j], hp);
                hp.neg_step_size = c1.x;
                hp.inv_bc2_sqrt = c1.y;
#pragma unroll
                for (int j = 0; j < NP; ++j) op(P[j], M[j], Vv[j], hp);
            };
            // steps t, t + 1 while the pair after them exists (t + 3 <= upto): its constants by a running pointer,
            // no clamp
            const float2* q = lr + 4 * (t0 + 3);
            for (; t + 3 <= upto; t += 2, q += 8) {
                const float2 c0 = n0, c1 = n1;
                n0 = q[0];
                n1 = q[4];
                __builtin_amdgcn_sched_barrier(0);  // (the loads first: their wait is the trip's end, after its work)
                two(c0, c1);
            }
            // one, two or three steps are left (t + 3 > upto); n0, n1 hold steps t and t + 1
            auto one = [&](const float2 c) {
                hp.neg_step_size = c.x;
                hp.inv_bc2_sqrt = c.y;
#pragma unroll
                for (int j = 0; j < NP; ++j) op(P[j], M[j], Vv[j], hp);
            };
            if (t < upto) {
                two(n0, n1);
                if (t + 2 == upto) one(lr[4 * upto]);
            } else if (t == upto) {
                one(n0);
            }
        };
        if (hp.wd != 0.f)
            steps([](float2v& p, float2v& m, float2v& v, const AdamHyper& h) { adam_elem2(p, float2v{0.f, 0.f}, m, v, h); });
        else
            steps([](float2v& p, float2v& m, float2v& v, const AdamHyper& h) { adam_decay2(p, m, v, h); });
        return;
    }
    for (int32_t t = t0 + 1; t <= upto; ++t) {
        const AdamHyper hp = hist[t];
#pragma unroll
        for (int j = 0; j < NP; ++j) {
            if (hp.wd != 0.f)
                adam_elem2(P[j], float2v{0.f, 0.f}, M[j], Vv[j], hp);
            else
                adam_decay2(P[j], M[j], Vv[j], hp);
        }
    }
}

template <int VPL>
__global__ __launch_bounds__(256) void lazy_catch_up_kernel(const int64_t* __restrict__ rows,
                                                            const int32_t* __restrict__ count, int64_t cap,
                                                            int32_t* __restrict__ last_step, float* __restrict__ p,
                                                            float* __restrict__ m, float* __restrict__ v, int D,
                                                            const AdamHyper* __restrict__ hist, int32_t upto) {
    const int lane = threadIdx.x & 63;
    const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t n = count ? (int64_t)*count : cap;
    if (s >= n || s >= cap) return;
    const int64_t r = rows ? rows[s] : s;
    const int32_t t0 = lazy_from(last_step[r], upto);
    if (t0 >= upto) return;
    float P[VPL], M[VPL], Vv[VPL];
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
        const int e = lane + 64 * j;
        if (e < D) {
            P[j] = p[r * D + e];
            M[j] = m[r * D + e];
            Vv[j] = v[r * D + e];
        }
    }
    for (int32_t t = t0 + 1; t <= upto; ++t) {
        const AdamHyper hp = hist[t];
#pragma unroll
        for (int j = 0; j < VPL; ++j)
            if (lane + 64 * j < D) adam_zero_grad_step(P[j], M[j], Vv[j], hp);
    }
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
        const int e = lane + 64 * j;
        if (e < D) {
            p[r * D + e] = P[j];
            m[r * D + e] = M[j];
            v[r * D + e] = Vv[j];
        }
    }
    if (lane == 0) last_step[r] = upto;
}

// float4 variant for D % 4 == 0, D <= 256: a row is D/4 lanes (16-B accesses), a wave holds 256/D rows,
// and each lane carries four independent replay chains (more ILP for the latency-bound recurrence).
template <int LPR>
__global__ __launch_bounds__(256) void lazy_catch_up_v4_kernel(const int64_t* __restrict__ rows,
                                                               const int32_t* __restrict__ count, int64_t cap,
                                                               int32_t* __restrict__ last_step,
                                                               float* __restrict__ p, float* __restrict__ m,
                                                               float* __restrict__ v,
                                                               const AdamHyper* __restrict__ hist, int32_t upto) {
    constexpr int D = LPR * 4;
    const int lane = threadIdx.x & 63;
    const int64_t s = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * (64 / LPR) + lane / LPR;
    const int64_t n = count ? (int64_t)*count : cap;
    const bool in_range = s < n && s < cap;
    const int64_t r = in_range ? (rows ? rows[s] : s) : 0;
    const int32_t t0 = in_range ? lazy_from(last_step[r], upto) : upto;
    // The rows of a wave have different last steps: replay over the wave's whole range with a uniform step
    // counter (hist[t] is then a scalar load, not a per-lane gather) and let each lane apply only its own
    // steps.  All lanes of a row agree, so the per-row result is exactly the per-row replay.
    int32_t t_lo = t0;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) t_lo = min(t_lo, __shfl_xor(t_lo, o, 64));
    t_lo = __builtin_amdgcn_readfirstlane(t_lo);
    if (t_lo >= upto) return;  // wave-uniform
    const bool live = t0 < upto;
    const int64_t off = r * D + (lane % LPR) * 4;
    float4 P = make_float4(0.f, 0.f, 0.f, 0.f), M = P, Vv = P;
    if (live) {
        P = *reinterpret_cast<const float4*>(p + off);
        M = *reinterpret_cast<const float4*>(m + off);
        Vv = *reinterpret_cast<const float4*>(v + off);
    }
    // lanes whose row starts later sit out the first steps under the exec mask (no per-element selects)
    // (the next step's constants are loaded one iteration ahead, off the recurrence's critical path)
    AdamHyper next = hist[t_lo + 1];
    for (int32_t t = t_lo + 1; t <= upto; ++t) {
        const AdamHyper hp = next;
        next = hist[min(t + 1, upto)];
        if (t > t0) adam_zero_grad_step4(P, M, Vv, hp);
    }
    if (!live) return;
    *reinterpret_cast<float4*>(p + off) = P;
    *reinterpret_cast<float4*>(m + off) = M;
    *reinterpret_cast<float4*>(v + off) = Vv;
    if (lane % LPR == 0) last_step[r] = upto;
}

template <int LPR>
__global__ __launch_bounds__(256) void lazy_apply_v4_kernel(const int64_t* __restrict__ rows,
                                                            const int32_t* __restrict__ count, int64_t cap,
                                                            const float* __restrict__ grad_rows,
                                                            int32_t* __restrict__ last_step, float* __restrict__ p,
                                                            float* __restrict__ m, float* __restrict__ v,
                                                            const AdamHyper* __restrict__ hist, int32_t step) {
    constexpr int D = LPR * 4;
    const int lane = threadIdx.x & 63;
    const int64_t s = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * (64 / LPR) + lane / LPR;
    if (s >= cap || s >= (int64_t)*count) return;
    const int64_t r = rows[s];
    const AdamHyper hp = hist[step];
    const int c = (lane % LPR) * 4;
    const int64_t off = r * D + c;
    float4 P = *reinterpret_cast<const float4*>(p + off);
    float4 M = *reinterpret_cast<const float4*>(m + off);
    float4 Vv = *reinterpret_cast<const float4*>(v + off);
    const float4 G = *reinterpret_cast<const float4*>(grad_rows + s * D + c);
    adam_elem4(P, G, M, Vv, hp);
    *reinterpret_cast<float4*>(p + off) = P;
    *reinterpret_cast<float4*>(m + off) = M;
    *reinterpret_cast<float4*>(v + off) = Vv;
    if (lane % LPR == 0) last_step[r] = step;
}

// One row per wave (D = 128 / 256: NP float2 per lane): the replay loop runs exactly the row's own steps.  The
// float4 kernels above put 256 / D rows in a wave and replay from the OLDEST of their last steps with the newer
// rows masked off, which wastes the difference -- with fresh ids each step and the end-of-run flush over every
// row, replay lengths are spread wide and that waste is most of the VALU time.  STAGE: write to the compact
// staged rows (slot order) instead of the table, leaving last_step alone (see lazy_stage_v4_kernel).
template <int NP, bool STAGE>
__global__ __launch_bounds__(256) void lazy_row_kernel(const int64_t* __restrict__ rows,
                                                       const int32_t* __restrict__ count, int64_t cap,
                                                       int32_t* __restrict__ last_step, float* __restrict__ p,
                                                       float* __restrict__ m, float* __restrict__ v,
                                                       const AdamHyper* __restrict__ hist, int32_t upto,
                                                       float* __restrict__ sp, float* __restrict__ sm,
                                                       float* __restrict__ sv) {
    constexpr int D = 128 * NP;
    const int lane = threadIdx.x & 63;
    const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t n = count ? (int64_t)*count : cap;
    if (s >= n || s >= cap) return;  // wave-uniform
    const int64_t r = rows ? rows[s] : s;
    float2v P[NP], M[NP], Vv[NP];
#pragma unroll
    for (int j = 0; j < NP; ++j) {
        const int64_t off = r * D + 2 * lane + 128 * j;
        const float2 a = *reinterpret_cast<const float2*>(p + off);
        const float2 b = *reinterpret_cast<const float2*>(m + off);
        const float2 c = *reinterpret_cast<const float2*>(v + off);
        P[j] = float2v{a.x, a.y};
        M[j] = float2v{b.x, b.y};
        Vv[j] = float2v{c.x, c.y};
    }
    const int32_t t0 = lazy_from(__builtin_amdgcn_readfirstlane(last_step[r]), upto);
    if (!STAGE && t0 >= upto) return;
    for (int32_t t = t0 + 1; t <= upto; ++t) {
        const AdamHyper hp = hist[t];
#pragma unroll
        for (int j = 0; j < NP; ++j) {
            if (hp.wd != 0.f)
                adam_elem2(P[j], float2v{0.f, 0.f}, M[j], Vv[j], hp);
            else
                adam_decay2(P[j], M[j], Vv[j], hp);
        }
    }
    float* op = STAGE ? sp + s * D : p + r * D;
    float* om = STAGE ? sm + s * D : m + r * D;
    float* ov = STAGE ? sv + s * D : v + r * D;
#pragma unroll
    for (int j = 0; j < NP; ++j) {
        const int c = 2 * lane + 128 * j;
        *reinterpret_cast<float2*>(op + c) = make_float2(P[j].x, P[j].y);
        *reinterpret_cast<float2*>(om + c) = make_float2(M[j].x, M[j].y);
        *reinterpret_cast<float2*>(ov + c) = make_float2(Vv[j].x, Vv[j].y);
    }
    if (!STAGE && lane == 0) last_step[r] = upto;
}

// Software-pipelined lazy replay: the full-table catch-up (flush(): every row brought to `upto`; rows == null) and
// the staging of the step's unique rows (STAGE: rows[s] -> the compact buffers at slot s).  In lazy_row_kernel a
// wave reads its slot's row id, waits, reads last_step, waits, reads the row, waits, replays and stores: at most one
// row's 1.5 KB in flight per wave and none while it replays, so the flush ran at ~3 TB/s with the VALU half idle.
// Here a wave owns RPW consecutive slots: one load brings all their row ids and one their last steps (lane i: slot
// base + i), and the p/m/v of slot i + PF - 1 are requested before slot i is replayed (a PF-deep register ring), so
// the row reads stream while the replay runs.  Same per-element operations (adam_elem2 / adam_decay2): same bits.
#ifndef ASME_FLUSH_PIPE
#define ASME_FLUSH_PIPE 1
#endif
#ifndef ASME_STAGE_PIPE
#define ASME_STAGE_PIPE 1
#endif
#ifndef ASME_FLUSH_RPW
#define ASME_FLUSH_RPW 16
#endif
#ifndef ASME_FLUSH_PF
#define ASME_FLUSH_PF 4
#endif
constexpr int kPipeRows = ASME_FLUSH_RPW;  // slots per wave
constexpr int kPipeDepth = ASME_FLUSH_PF;  // rows in the register ring (PF - 1 in flight during a replay)
#ifndef ASME_STAGE_P_NT
#define ASME_STAGE_P_NT 0
#endif
#ifndef ASME_STAGE_MV_NT
#define ASME_STAGE_MV_NT 1
#endif
template <int NP, int RPW, int PF, bool STAGE>
__global__ __launch_bounds__(256) void lazy_pipe_kernel(const int64_t* __restrict__ rows,
                                                        const int32_t* __restrict__ count, int64_t cap,
                                                        int32_t* __restrict__ last_step, float* __restrict__ p,
                                                        float* __restrict__ m, float* __restrict__ v,
                                                        const AdamHyper* __restrict__ hist, int32_t upto,
                                                        float* __restrict__ sp, float* __restrict__ sm,
                                                        float* __restrict__ sv) {
    static_assert(RPW <= 64 && PF >= 2 && PF <= RPW, "ring depth");
    constexpr int D = 128 * NP;
    const int lane = threadIdx.x & 63;
    const int64_t base = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW;
    int64_t n = count ? (int64_t)*count : cap;
    n = n < cap ? n : cap;
    if (base >= n) return;  // wave-uniform
    const int nr = (int)(n - base < RPW ? n - base : RPW);
    const int64_t my_r = lane < nr ? (rows ? rows[base + lane] : base + lane) : 0;
    const int32_t my_t = lane < nr ? lazy_from(last_step[my_r], upto) : upto;
    // the slots this wave works on, in slot order: every slot when staging (each is written to the staged rows),
    // else only the rows behind `upto` -- current rows and rows at rest are neither read nor written by the flush
    const uint64_t live = __ballot(lane < nr && (STAGE || my_t < upto));
    if (live == 0) return;  // wave-uniform
    const int nl = __popcll(live);
    const int32_t const_from = *reinterpret_cast<const int32_t*>(hist);
    int ln[RPW];  // lane (slot - base) of the i-th live slot; past the last one: the last one again (never stored)
    {
        uint64_t mm = live;
        const int last = 63 - __clzll(live);
#pragma unroll
        for (int i = 0; i < RPW; ++i) {
            ln[i] = mm ? __ffsll((unsigned long long)mm) - 1 : last;
            mm &= mm - 1;
        }
    }
    auto row_of = [&](int i) -> int64_t {
        const int k = ln[i];
        if (!rows) return base + k;
        const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)my_r, k);
        const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)((uint64_t)my_r >> 32), k);
        return (int64_t)(((uint64_t)hi << 32) | lo);
    };
    float2v P[PF][NP], M[PF][NP], Vv[PF][NP];
    auto load = [&](int i, int slot) {
        const int64_t r = row_of(i);
#pragma unroll
        for (int j = 0; j < NP; ++j) {
            const int64_t off = r * D + 2 * lane + 128 * j;
            const float2 a = *reinterpret_cast<const float2*>(p + off);
            const float2 b = *reinterpret_cast<const float2*>(m + off);
            const float2 c = *reinterpret_cast<const float2*>(v + off);
            P[slot][j] = float2v{a.x, a.y};
            M[slot][j] = float2v{b.x, b.y};
            Vv[slot][j] = float2v{c.x, c.y};
        }
    };
#pragma unroll
    for (int i = 0; i < PF - 1; ++i) load(i, i);
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
        if (i + PF - 1 < RPW) load(i + PF - 1, (i + PF - 1) % PF);
        const int sl = i % PF;
        const int32_t t0 = __builtin_amdgcn_readlane(my_t, ln[i]);
        if (i < nl) {
            replay_steps<NP>(P[sl], M[sl], Vv[sl], hist, t0, upto, const_from);
            const int64_t orow = STAGE ? base + ln[i] : row_of(i);
            float* op = STAGE ? sp : p;
            float* om = STAGE ? sm : m;
            float* ov = STAGE ? sv : v;
#pragma unroll
            for (int j = 0; j < NP; ++j) {
                const int64_t off = orow * D + 2 * lane + 128 * j;
                if (STAGE) {
                    // the staged parameters are read again right away by this step's gathers (the embedding
                    // forward follows this kernel); the staged moments only by the reduce-and-apply at the end of the
                    // step, ~6 ms and GBs of traffic later: streamed past the L2 / MALL, so their dirty lines do
                    // not drain into the next kernel's HBM time (an 0.9 GB cached write before the embedding forward
                    // cost it 55 -> 84 us, tools/emb_ln_bench.py)
#if ASME_STAGE_P_NT
                    table_store2(op + off, P[sl][j].x, P[sl][j].y);
#else
                    *reinterpret_cast<float2*>(op + off) = make_float2(P[sl][j].x, P[sl][j].y);
#endif
#if ASME_STAGE_MV_NT
                    table_store2(om + off, M[sl][j].x, M[sl][j].y);
                    table_store2(ov + off, Vv[sl][j].x, Vv[sl][j].y);
#else
                    *reinterpret_cast<float2*>(om + off) = make_float2(M[sl][j].x, M[sl][j].y);
                    *reinterpret_cast<float2*>(ov + off) = make_float2(Vv[sl][j].x, Vv[sl][j].y);
#endif
                } else {
                    table_store2(op + off, P[sl][j].x, P[sl][j].y);
                    table_store2(om + off, M[sl][j].x, M[sl][j].y);
                    table_store2(ov + off, Vv[sl][j].x, Vv[sl][j].y);
                }
            }
        }
    }
    if (!STAGE && lane < nr && my_t < upto) last_step[my_r] = upto;
}
template <int NP, bool STAGE>
void launch_pipe(const int64_t* rows, const int32_t* count, int64_t cap, int32_t* last_step, float* p, float* m,
                 float* v, const float* hist, int64_t upto, float* sp, float* sm, float* sv, hipStream_t s) {
    const int64_t per_block = 4 * kPipeRows;
    hipLaunchKernelGGL((lazy_pipe_kernel<NP, kPipeRows, kPipeDepth, STAGE>),
                       dim3((unsigned)((cap + per_block - 1) / per_block)), dim3(256), 0, s, rows, count, cap,
                       last_step, p, m, v, reinterpret_cast<const AdamHyper*>(hist), (int32_t)upto, sp, sm, sv);
}

#ifndef ASME_LAZY_ROW_WAVE
#define ASME_LAZY_ROW_WAVE 1
#endif
inline bool row_wave_ok(int64_t dim) { return ASME_LAZY_ROW_WAVE && (dim == 128 || dim == 256); }

// Staged variant (the step's unique rows read in slot order afterwards).  stage: slot s gets rows[s] brought up
// to `upto` into the compact buffers sp/sm/sv[s] -- the table and last_step are NOT written, so a step that
// never reaches the optimizer leaves the lazy state untouched; the row reads are random, the writes stream in
// slot order.  Every reader of the step's rows (embedding gather, sampled head, their backwards) then reads
// sp[inverse[t]], i.e. nearly in token order.  apply_staged: the real-gradient step from the staged values
// (streamed) into the table rows (random writes) and last_step = step.
template <int LPR>
__global__ __launch_bounds__(256) void lazy_stage_v4_kernel(const int64_t* __restrict__ rows,
                                                            const int32_t* __restrict__ count, int64_t cap,
                                                            const int32_t* __restrict__ last_step,
                                                            const float* __restrict__ p, const float* __restrict__ m,
                                                            const float* __restrict__ v,
                                                            const AdamHyper* __restrict__ hist, int32_t upto,
                                                            float* __restrict__ sp, float* __restrict__ sm,
                                                            float* __restrict__ sv) {
    constexpr int D = LPR * 4;
    const int lane = threadIdx.x & 63;
    const int64_t s = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * (64 / LPR) + lane / LPR;
    const int64_t n = (int64_t)*count;
    const bool in_range = s < n && s < cap;
    const int64_t r = in_range ? rows[s] : 0;
    const int64_t off = r * D + (lane % LPR) * 4;
    // the row loads do not wait for last_step
    float4 P = make_float4(0.f, 0.f, 0.f, 0.f), M = P, Vv = P;
    if (in_range) {
        P = *reinterpret_cast<const float4*>(p + off);
        M = *reinterpret_cast<const float4*>(m + off);
        Vv = *reinterpret_cast<const float4*>(v + off);
    }
    const int32_t t0 = in_range ? lazy_from(last_step[r], upto) : upto;
    int32_t t_lo = t0;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) t_lo = min(t_lo, __shfl_xor(t_lo, o, 64));
    t_lo = __builtin_amdgcn_readfirstlane(t_lo);
    if (t_lo < upto) {  // wave-uniform; same replay as lazy_catch_up_v4_kernel
        AdamHyper next = hist[t_lo + 1];
        for (int32_t t = t_lo + 1; t <= upto; ++t) {
            const AdamHyper hp = next;
            next = hist[min(t + 1, upto)];
            if (t > t0) adam_zero_grad_step4(P, M, Vv, hp);
        }
    }
    if (!in_range) return;
    const int64_t so = s * D + (lane % LPR) * 4;
    *reinterpret_cast<float4*>(sp + so) = P;
    *reinterpret_cast<float4*>(sm + so) = M;
    *reinterpret_cast<float4*>(sv + so) = Vv;
}

template <int LPR>
__global__ __launch_bounds__(256) void lazy_apply_staged_v4_kernel(
    const int64_t* __restrict__ rows, const int32_t* __restrict__ count, int64_t cap,
    const float* __restrict__ grad_rows, const float* __restrict__ sp, const float* __restrict__ sm,
    const float* __restrict__ sv, int32_t* __restrict__ last_step, float* __restrict__ p, float* __restrict__ m,
    float* __restrict__ v, const AdamHyper* __restrict__ hist, int32_t step) {
    constexpr int D = LPR * 4;
    const int lane = threadIdx.x & 63;
    const int64_t s = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * (64 / LPR) + lane / LPR;
    if (s >= cap || s >= (int64_t)*count) return;
    const int c = (lane % LPR) * 4;
    const int64_t so = s * D + c;
    float4 P = *reinterpret_cast<const float4*>(sp + so);
    float4 M = *reinterpret_cast<const float4*>(sm + so);
    float4 Vv = *reinterpret_cast<const float4*>(sv + so);
    const float4 G = *reinterpret_cast<const float4*>(grad_rows + so);
    const int64_t r = rows[s];
    const AdamHyper hp = hist[step];
    adam_elem4(P, G, M, Vv, hp);
    const int64_t off = r * D + c;
    table_store4(p + off, P);
    table_store4(m + off, M);
    table_store4(v + off, Vv);
    if (lane % LPR == 0) last_step[r] = step;
}

#define ASME_LPR_DISPATCH(DIM, ...)                                             \
    switch (DIM) {                                                              \
        case 32: { constexpr int LPR = 8; __VA_ARGS__; } break;                 \
        case 64: { constexpr int LPR = 16; __VA_ARGS__; } break;                \
        case 128: { constexpr int LPR = 32; __VA_ARGS__; } break;               \
        case 256: { constexpr int LPR = 64; __VA_ARGS__; } break;               \
        default: break;                                                         \
    }

inline bool v4_ok(int64_t dim, const void* a, const void* b, const void* c) {
    return (dim == 32 || dim == 64 || dim == 128 || dim == 256) &&
           ((((uintptr_t)a) | ((uintptr_t)b) | ((uintptr_t)c)) & 15) == 0;
}

// the real-gradient update of the step's unique rows (they were caught up to step-1 before the forward)
template <int VPL>
__global__ __launch_bounds__(256) void lazy_apply_kernel(const int64_t* __restrict__ rows,
                                                         const int32_t* __restrict__ count, int64_t cap,
                                                         const float* __restrict__ grad_rows,
                                                         int32_t* __restrict__ last_step, float* __restrict__ p,
                                                         float* __restrict__ m, float* __restrict__ v, int D,
                                                         const AdamHyper* __restrict__ hist, int32_t step) {
    const int lane = threadIdx.x & 63;
    const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (s >= cap || s >= (int64_t)*count) return;
    const int64_t r = rows[s];
    const AdamHyper hp = hist[step];
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
        const int e = lane + 64 * j;
        if (e < D) {
            float P = p[r * D + e], M = m[r * D + e], Vv = v[r * D + e];
            adam_elem(P, grad_rows[s * D + e], M, Vv, hp);
            p[r * D + e] = P;
            m[r * D + e] = M;
            v[r * D + e] = Vv;
        }
    }
    if (lane == 0) last_step[r] = step;
}

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

// hist[step] = the Adam constants of `step` (hist: (hist_rows, 8) floats on the device; step < hist_rows)
ASME_API int asme_lazy_adam_record_step(float* hist, int64_t hist_rows, int64_t step, float lr, float beta1,
                                        float beta2, float eps, float weight_decay, void* stream) {
    ASME_CHECK_ARG(hist && step >= 1, "asme_lazy_adam_record_step: bad argument");
    ASME_CHECK_ARG(step < hist_rows, "asme_lazy_adam_record_step: step beyond the history capacity");
    const AdamHyper hp = make_hyper(lr, beta1, beta2, eps, weight_decay, step);
    hipLaunchKernelGGL(record_step_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, hist, step, hp);
    ASME_LAUNCH_CHECK("asme_lazy_adam_record_step");
}

// bring rows[0..count) (rows == NULL: every row 0..cap) up to date through step `upto` with zero gradient
ASME_API int asme_lazy_adam_catch_up(const int64_t* rows, const int32_t* count, int64_t cap, int32_t* last_step,
                                     float* param, float* exp_avg, float* exp_avg_sq, int64_t dim, const float* hist,
                                     int64_t hist_rows, int64_t upto, void* stream) {
    ASME_CHECK_ARG(last_step && param && exp_avg && exp_avg_sq && hist, "asme_lazy_adam_catch_up: null pointer");
    ASME_CHECK_ARG(upto < hist_rows, "asme_lazy_adam_catch_up: step beyond the history capacity");
    ASME_CHECK_ARG(dim >= 1 && dim <= 512 && upto >= 0 && upto < (1LL << 31), "asme_lazy_adam_catch_up: bad shape");
    if (cap == 0 || upto == 0) return 0;
    if (ASME_FLUSH_PIPE && !rows && !count && row_wave_ok(dim) && v4_ok(dim, param, exp_avg, exp_avg_sq)) {
        if (dim == 128)
            launch_pipe<1, false>(rows, count, cap, last_step, param, exp_avg, exp_avg_sq, hist, upto, nullptr, nullptr,
                                  nullptr, (hipStream_t)stream);
        else
            launch_pipe<2, false>(rows, count, cap, last_step, param, exp_avg, exp_avg_sq, hist, upto, nullptr, nullptr,
                                  nullptr, (hipStream_t)stream);
        ASME_LAUNCH_CHECK("asme_lazy_adam_catch_up");
    }
    if (row_wave_ok(dim) && v4_ok(dim, param, exp_avg, exp_avg_sq)) {
        const dim3 g((unsigned)((cap + 3) / 4));
        if (dim == 128)
            hipLaunchKernelGGL((lazy_row_kernel<1, false>), g, dim3(256), 0, (hipStream_t)stream, rows, count, cap,
                               last_step, param, exp_avg, exp_avg_sq, reinterpret_cast<const AdamHyper*>(hist),
                               (int32_t)upto, nullptr, nullptr, nullptr);
        else
            hipLaunchKernelGGL((lazy_row_kernel<2, false>), g, dim3(256), 0, (hipStream_t)stream, rows, count, cap,
                               last_step, param, exp_avg, exp_avg_sq, reinterpret_cast<const AdamHyper*>(hist),
                               (int32_t)upto, nullptr, nullptr, nullptr);
        ASME_LAUNCH_CHECK("asme_lazy_adam_catch_up");
    }
    if (v4_ok(dim, param, exp_avg, exp_avg_sq)) {
        const int64_t rows_per_block = 4 * (256 / dim);
        const dim3 g4((unsigned)((cap + rows_per_block - 1) / rows_per_block));
        ASME_LPR_DISPATCH(dim, hipLaunchKernelGGL(lazy_catch_up_v4_kernel<LPR>, g4, dim3(256), 0,
                                                  (hipStream_t)stream, rows, count, cap, last_step, param, exp_avg,
                                                  exp_avg_sq, reinterpret_cast<const AdamHyper*>(hist),
                                                  (int32_t)upto));
        ASME_LAUNCH_CHECK("asme_lazy_adam_catch_up");
    }
    const dim3 grid((unsigned)((cap + 3) / 4));
    ASME_VPL_DISPATCH((int)((dim + 63) / 64),
                      hipLaunchKernelGGL(lazy_catch_up_kernel<VPL>, grid, dim3(256), 0, (hipStream_t)stream, rows,
                                         count, cap, last_step, param, exp_avg, exp_avg_sq, (int)dim,
                                         reinterpret_cast<const AdamHyper*>(hist), (int32_t)upto));
    ASME_LAUNCH_CHECK("asme_lazy_adam_catch_up");
}

ASME_API int asme_lazy_adam_stage_supported(int64_t dim) {
    return dim == 32 || dim == 64 || dim == 128 || dim == 256;
}

ASME_API int asme_lazy_adam_stage(const int64_t* rows, const int32_t* count, int64_t cap, const int32_t* last_step,
                                  const float* param, const float* exp_avg, const float* exp_avg_sq, int64_t dim,
                                  const float* hist, int64_t hist_rows, int64_t upto, float* staged_param,
                                  float* staged_exp_avg, float* staged_exp_avg_sq, void* stream) {
    ASME_CHECK_ARG(rows && count && last_step && param && exp_avg && exp_avg_sq && hist && staged_param &&
                       staged_exp_avg && staged_exp_avg_sq, "asme_lazy_adam_stage: null pointer");
    ASME_CHECK_ARG(upto >= 0 && upto < hist_rows && upto < (1LL << 31), "asme_lazy_adam_stage: step beyond the history");
    ASME_CHECK_ARG(asme_lazy_adam_stage_supported(dim) && v4_ok(dim, param, exp_avg, exp_avg_sq) &&
                       v4_ok(dim, staged_param, staged_exp_avg, staged_exp_avg_sq),
                   "asme_lazy_adam_stage: dim must be 32/64/128/256 and every row pointer 16-B aligned");
    if (cap == 0) return 0;
    if (ASME_STAGE_PIPE && row_wave_ok(dim)) {
        int32_t* ls = const_cast<int32_t*>(last_step);  // (not written in STAGE mode)
        float *pp = const_cast<float*>(param), *mm = const_cast<float*>(exp_avg), *vv = const_cast<float*>(exp_avg_sq);
        if (dim == 128)
            launch_pipe<1, true>(rows, count, cap, ls, pp, mm, vv, hist, upto, staged_param, staged_exp_avg,
                                 staged_exp_avg_sq, (hipStream_t)stream);
        else
            launch_pipe<2, true>(rows, count, cap, ls, pp, mm, vv, hist, upto, staged_param, staged_exp_avg,
                                 staged_exp_avg_sq, (hipStream_t)stream);
        ASME_LAUNCH_CHECK("asme_lazy_adam_stage");
    }
    if (row_wave_ok(dim)) {
        const dim3 g((unsigned)((cap + 3) / 4));
        int32_t* ls = const_cast<int32_t*>(last_step);  // (not written in STAGE mode)
        float *pp = const_cast<float*>(param), *mm = const_cast<float*>(exp_avg), *vv = const_cast<float*>(exp_avg_sq);
        if (dim == 128)
            hipLaunchKernelGGL((lazy_row_kernel<1, true>), g, dim3(256), 0, (hipStream_t)stream, rows, count, cap, ls,
                               pp, mm, vv, reinterpret_cast<const AdamHyper*>(hist), (int32_t)upto, staged_param,
                               staged_exp_avg, staged_exp_avg_sq);
        else
            hipLaunchKernelGGL((lazy_row_kernel<2, true>), g, dim3(256), 0, (hipStream_t)stream, rows, count, cap, ls,
                               pp, mm, vv, reinterpret_cast<const AdamHyper*>(hist), (int32_t)upto, staged_param,
                               staged_exp_avg, staged_exp_avg_sq);
        ASME_LAUNCH_CHECK("asme_lazy_adam_stage");
    }
    const int64_t rows_per_block = 4 * (256 / dim);
    const dim3 g4((unsigned)((cap + rows_per_block - 1) / rows_per_block));
    ASME_LPR_DISPATCH(dim, hipLaunchKernelGGL(lazy_stage_v4_kernel<LPR>, g4, dim3(256), 0, (hipStream_t)stream, rows,
                                              count, cap, last_step, param, exp_avg, exp_avg_sq,
                                              reinterpret_cast<const AdamHyper*>(hist), (int32_t)upto, staged_param,
                                              staged_exp_avg, staged_exp_avg_sq));
    ASME_LAUNCH_CHECK("asme_lazy_adam_stage");
}

ASME_API int asme_lazy_adam_apply_staged(const int64_t* rows, const int32_t* count, int64_t cap,
                                         const float* grad_rows, const float* staged_param,
                                         const float* staged_exp_avg, const float* staged_exp_avg_sq,
                                         int32_t* last_step, float* param, float* exp_avg, float* exp_avg_sq,
                                         int64_t dim, const float* hist, int64_t hist_rows, int64_t step,
                                         void* stream) {
    ASME_CHECK_ARG(rows && count && grad_rows && staged_param && staged_exp_avg && staged_exp_avg_sq && last_step &&
                       param && exp_avg && exp_avg_sq && hist, "asme_lazy_adam_apply_staged: null pointer");
    ASME_CHECK_ARG(step >= 1 && step < hist_rows, "asme_lazy_adam_apply_staged: step beyond the history");
    ASME_CHECK_ARG(asme_lazy_adam_stage_supported(dim) && v4_ok(dim, param, exp_avg, exp_avg_sq) &&
                       v4_ok(dim, staged_param, staged_exp_avg, staged_exp_avg_sq) && ((uintptr_t)grad_rows & 15) == 0,
                   "asme_lazy_adam_apply_staged: dim must be 32/64/128/256 and every row pointer 16-B aligned");
    if (cap == 0) return 0;
    const int64_t rows_per_block = 4 * (256 / dim);
    const dim3 g4((unsigned)((cap + rows_per_block - 1) / rows_per_block));
    ASME_LPR_DISPATCH(dim, hipLaunchKernelGGL(lazy_apply_staged_v4_kernel<LPR>, g4, dim3(256), 0, (hipStream_t)stream,
                                              rows, count, cap, grad_rows, staged_param, staged_exp_avg,
                                              staged_exp_avg_sq, last_step, param, exp_avg, exp_avg_sq,
                                              reinterpret_cast<const AdamHyper*>(hist), (int32_t)step));
    ASME_LAUNCH_CHECK("asme_lazy_adam_apply_staged");
}

ASME_API int asme_lazy_adam_apply(const int64_t* rows, const int32_t* count, int64_t cap, const float* grad_rows,
                                  int32_t* last_step, float* param, float* exp_avg, float* exp_avg_sq, int64_t dim,
                                  const float* hist, int64_t hist_rows, int64_t step, void* stream) {
    ASME_CHECK_ARG(rows && count && grad_rows && last_step && param && exp_avg && exp_avg_sq && hist,
                   "asme_lazy_adam_apply: null pointer");
    ASME_CHECK_ARG(step < hist_rows, "asme_lazy_adam_apply: step beyond the history capacity");
    ASME_CHECK_ARG(dim >= 1 && dim <= 512 && step >= 1, "asme_lazy_adam_apply: bad shape");
    if (cap == 0) return 0;
    if (v4_ok(dim, param, exp_avg, exp_avg_sq) && ((uintptr_t)grad_rows & 15) == 0) {
        const int64_t rows_per_block = 4 * (256 / dim);
        const dim3 g4((unsigned)((cap + rows_per_block - 1) / rows_per_block));
        ASME_LPR_DISPATCH(dim, hipLaunchKernelGGL(lazy_apply_v4_kernel<LPR>, g4, dim3(256), 0, (hipStream_t)stream,
                                                  rows, count, cap, grad_rows, last_step, param, exp_avg,
                                                  exp_avg_sq, reinterpret_cast<const AdamHyper*>(hist),
                                                  (int32_t)step));
        ASME_LAUNCH_CHECK("asme_lazy_adam_apply");
    }
    const dim3 grid((unsigned)((cap + 3) / 4));
    ASME_VPL_DISPATCH((int)((dim + 63) / 64),
                      hipLaunchKernelGGL(lazy_apply_kernel<VPL>, grid, dim3(256), 0, (hipStream_t)stream, rows, count,
                                         cap, grad_rows, last_step, param, exp_avg, exp_avg_sq, (int)dim,
                                         reinterpret_cast<const AdamHyper*>(hist), (int32_t)step));
    ASME_LAUNCH_CHECK("asme_lazy_adam_apply");
}
