// EXPERIMENT (round 5, not built into the product): asme_ws_linear on v_mfma_f32_32x32x16_bf16 with 32-token tiles.
// Correct (tests/test_gpu_wsgemm.py green when dispatched) but slower at every bench shape (tools/ws_ab.py, same
// process: 2.77 ms vs 1.25 ms for the nine products with NT stores, 1.83 ms with cached stores): the split VALU per
// token is unchanged (the X tile is re-split once per 64-feature block), scattered 32-B row stores, and the compiler
// waits vmcnt(3-4) at the top of the tile loop.  Kept as a record of the measurement.
// Weight-stationary streaming GEMM on v_mfma_f32_32x32x16_bf16 (bf16x6 split operands, common.h) for the
// token-major Linear layers, gfx950.  Same contract and epilogues as ws_gemm_kernel (wsgemm.hip), which it replaces
// for the shapes it takes (asme_ws_linear dispatches).
//
// Reference semantics (paths relative to /root/reference/src/asme):
//   nn.Linear projections         core/models/common/layers/transformer_layers.py:175-199 (Q,K,V,O)
//   PositionwiseFeedForward       transformer_layers.py:212-220  W2(dropout(GELU_erf(W1 x)))
//
// Why a second form.  The 16x16x32 kernel's tile (16 tokens x 16 features per MFMA) runs 192 MFMAs and ~260 vector
// instructions per 16-token x 128-feature tile at two waves per SIMD.  On gfx950 a 16x16x32 MFMA holds the SIMD's
// vector issue for 8 of its 16 cycles (MI355X_MICROARCH.md, cycle constants), so the MFMA holds plus the split /
// epilogue VALU of the two waves fill ~91 % of the matrix pipe's time and every memory stall lands on the critical
// path (measured: matrix work and streaming add instead of overlapping).  A 32x32x16 MFMA does twice the
// work of a 16x16x32 in 32 cycles and holds vector issue for 8 of them: per 32 tokens x 128 features the holds drop
// from 3,072 to 1,536 cycles against the same 6,144 cycles of matrix work, leaving the split, the epilogue and the
// memory instructions room to overlap.
//
// Layout.  C^T tile (32 features x 32 tokens) += W_blk (32 features x 16 k) . X^T (16 k x 32 tokens): lane
// (r = lane & 31, h = lane >> 5) supplies W row r, k 8h..8h+7 (three ds_read_b128 of the split W planes held in LDS
// for the workgroup's life) and X row (token) r, k 8h..8h+7 (two float4 buffer loads, split once in registers for
// all FT feature tiles); accumulator register i holds feature (i & 3) + 8 (i >> 2) + 4h of token r, so a lane stores
// four float4 of 4 consecutive features per feature tile (rows past M are dropped by the buffer range check).
// A wave streams 32-token tiles with the whole next tile's X in flight (K <= 128) or 8 k-steps ahead.
// Dropout of the GELU epilogue: the lane's chunk pair (features 8u + 4h and 8u + 4h + 16, u = 0, 1) is exactly one
// Philox block of asme_gelu_dropout_fwd's scheme (common.h gelu_keep_bits8), so the decisions are the row kernel's
// with one block per 8 elements and no lane exchange.
#include "common.h"

using namespace asme;

namespace {

typedef unsigned u32v4 __attribute__((ext_vector_type(4)));

constexpr int kWaves32 = 8;  // 512-thread workgroups, one per CU, two waves per SIMD
constexpr int kLdsMax32 = 160 * 1024;
constexpr uint32_t kDrop32 = 0x80000000u;  // >= every buffer's record count: the access is dropped / reads 0

enum { W32_STORE = 0, W32_GELU_DROP = 1, W32_GELU_BWD = 2, W32_ACCUM = 3 };
#ifndef ASME_W32_NT
#define ASME_W32_NT 1
#endif

struct Ws32Epi {
    const float* bias;
    float* pre_out;       // GELU forward: activation factor keep * GELU'(pre) out
    const float* pre_in;  // GELU backward: activation factor in
    float p;
    uint64_t seed;
    int64_t ldx, ldw;  // row strides of X and (non-trans) W
    int kofs;          // first k column (split-K halves of K = 512)
};

__device__ __forceinline__ int wslot32(int r, int s, int K8) { return r * K8 + (s ^ (r & 15)); }
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc32(const void* p, int64_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ float4 bload32(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    const u32v4 u = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
    return make_float4(__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z), __uint_as_float(u.w));
}
__device__ __forceinline__ void bstore32(float4 v, __amdgpu_buffer_rsrc_t r, uint32_t off, bool nt) {
    const u32v4 u = {__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)};
    if (nt)
        __builtin_amdgcn_raw_buffer_store_b128(u, r, off, 0, 2);
    else
        __builtin_amdgcn_raw_buffer_store_b128(u, r, off, 0, 0);
}

template <int K, int FT, bool TRANS, int EPI>
__global__ __launch_bounds__(kWaves32 * 64) __attribute__((amdgpu_waves_per_eu(2, 2))) void ws32_kernel(
    const float* __restrict__ X, int64_t M, const float* __restrict__ W, int N, float* __restrict__ Y, Ws32Epi ep) {
    constexpr int NB = 32 * FT;    // output features per workgroup
    constexpr int K8 = K / 8;      // 16-B slots (8 bf16) of a W image row
    constexpr int NKS = K / 16;    // 16-k steps
    constexpr int PL = NB * K8;    // slots of one bf16 plane
    constexpr int RD = NKS < 8 ? NKS : 8;  // k steps of X in flight
    static_assert(NKS % RD == 0, "the ring depth must divide the k steps");
    extern __shared__ __attribute__((aligned(16))) uint4 lds32[];
    const int nblk = N / NB;
    const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3, per_xcd = gridDim.x >> 3;
    const int wg_per_nb = per_xcd / nblk;
    if (slot >= wg_per_nb * nblk) return;
    const int nb = slot % nblk;
    const int n0 = nb * NB;
    // ---- the W block, once, split into its three bf16 planes
    for (int i = threadIdx.x; i < NB * K8; i += kWaves32 * 64) {
        const int r = TRANS ? i % NB : i / K8, s8 = TRANS ? i / NB : i % K8;
        float4 a, b;
        if (!TRANS) {
            const float* w = W + (int64_t)(n0 + r) * ep.ldw + ep.kofs + 8 * s8;
            a = *reinterpret_cast<const float4*>(w);
            b = *reinterpret_cast<const float4*>(w + 4);
        } else {
            const float* w = W + (int64_t)(ep.kofs + 8 * s8) * N + n0 + r;
            a = make_float4(w[0], w[N], w[2 * N], w[3 * N]);
            b = make_float4(w[4 * N], w[5 * N], w[6 * N], w[7 * N]);
        }
        const Bf3 pz = split_bf3(a, b);
        const int sl = wslot32(r, s8, K8);
        lds32[sl] = __builtin_bit_cast(uint4, pz.h);
        lds32[PL + sl] = __builtin_bit_cast(uint4, pz.m);
        lds32[2 * PL + sl] = __builtin_bit_cast(uint4, pz.l);
    }
    __syncthreads();
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
    // ---- 32-token tiles of this (XCD, feature block): contiguous per XCD, strided over its waves
    const int64_t ntile = (M + 31) / 32;
    const int64_t lo = ntile * xcd / 8, hi = ntile * (xcd + 1) / 8;
    const int wcount = wg_per_nb * kWaves32;
    const int widx = (slot / nblk) * kWaves32 + wave;
    const int64_t my_tiles = hi - lo > widx ? (hi - lo - widx + wcount - 1) / wcount : 0;
    if (my_tiles == 0) return;
    const int64_t t0 = lo + widx;
    const __amdgpu_buffer_rsrc_t xr = rsrc32(X, M * ep.ldx * 4);
    const __amdgpu_buffer_rsrc_t yr = rsrc32(Y, M * N * 4);
    const __amdgpu_buffer_rsrc_t pr = EPI == W32_ACCUM ? yr
                                    : rsrc32(EPI == W32_GELU_DROP ? (const void*)ep.pre_out : (const void*)ep.pre_in,
                                             EPI == W32_STORE ? 0 : M * N * 4);
    const bool nt_out = ASME_W32_NT && N >= 384;
    // this lane's X byte offset of k step ks in tile j (rows past M: dropped -> zeros)
    auto xoff = [&](int64_t j, int ks) -> uint32_t {
        const int64_t m = (t0 + (j < my_tiles ? j : my_tiles - 1) * wcount) * 32 + r;
        return m < M ? (uint32_t)((m * ep.ldx + ep.kofs + 16 * ks + 8 * h) * 4) : kDrop32;
    };
    // the lane's bias values: feature tile ft, float4 u = features 32 ft + 8u + 4h .. +3
    float4 bias4[FT][4];
#pragma unroll
    for (int ft = 0; ft < FT; ++ft)
#pragma unroll
        for (int u = 0; u < 4; ++u)
            bias4[ft][u] = ep.bias ? *reinterpret_cast<const float4*>(ep.bias + n0 + 32 * ft + 8 * u + 4 * h)
                                   : make_float4(0.f, 0.f, 0.f, 0.f);
    const float keep_k = ep.p > 0.f ? 1.f / (1.f - ep.p) : 1.f;
    const uint32_t thr = gelu_thresh(ep.p);
    // W operand of feature tile ft, k step ks: row 32 ft + r, slot 2 ks + h of the three planes
    auto wload = [&](int ft, int ks) -> Bf3 {
        const int sl = wslot32(32 * ft + r, 2 * ks + h, K8);
        Bf3 w;
        w.h = __builtin_bit_cast(bf16x8, lds32[sl]);
        w.m = __builtin_bit_cast(bf16x8, lds32[PL + sl]);
        w.l = __builtin_bit_cast(bf16x8, lds32[2 * PL + sl]);
        return w;
    };
    float4 ring[2 * RD];
#pragma unroll
    for (int d = 0; d < RD; ++d) {
        const uint32_t o = xoff(0, d);
        ring[2 * d] = bload32(xr, o);
        ring[2 * d + 1] = bload32(xr, o == kDrop32 ? kDrop32 : o + 16);
    }
    Bf3 wc = wload(0, 0);
    for (int64_t j = 0; j < my_tiles; ++j) {
        const int64_t m = (t0 + j * wcount) * 32 + r;
        // the epilogue's second operand (activation factor / the first K half's Y), in flight during the tile
        float4 pre[FT][4];
        if constexpr (EPI == W32_GELU_BWD || EPI == W32_ACCUM) {
#pragma unroll
            for (int ft = 0; ft < FT; ++ft)
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    pre[ft][u] = bload32(pr, m < M ? (uint32_t)((m * N + n0 + 32 * ft + 8 * u + 4 * h) * 4) : kDrop32);
        }
        floatx16 acc[FT];
#pragma unroll
        for (int ft = 0; ft < FT; ++ft)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[ft][i] = 0.f;
#pragma unroll 1
        for (int kq = 0; kq < NKS; kq += RD)
#pragma unroll
        for (int d = 0; d < RD; ++d) {
            const int ks = kq + d;
            const Bf3 xs = split_bf3(ring[2 * d], ring[2 * d + 1]);
            // refill the slot: k step ks + RD of this tile, or of the next one
            const int kn = ks + RD;
            const uint32_t o = kn < NKS ? xoff(j, kn) : xoff(j + 1, kn - NKS);
            ring[2 * d] = bload32(xr, o);
            ring[2 * d + 1] = bload32(xr, o == kDrop32 ? kDrop32 : o + 16);
#pragma unroll
            for (int ft = 0; ft < FT; ++ft) {
                const Bf3 w = wc;
                // next fragment: tile ft + 1 of this k step, or tile 0 of the next (wrapping to step 0)
                wc = ft + 1 < FT ? wload(ft + 1, ks) : wload(0, ks + 1 < NKS ? ks + 1 : 0);
                acc[ft] = mfma32_bf3(w, xs, acc[ft]);
                // (program order kept: the scheduler would otherwise hoist the whole tile's LDS reads and X splits
                // of the unrolled k loop and spill)
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        // epilogue: lane (r, h) holds features 32 ft + 8u + 4h + (0..3) of token m in acc[ft][4u .. 4u + 3]
#pragma unroll
        for (int ft = 0; ft < FT; ++ft) {
            uint32_t bits8[2] = {0xFFu, 0xFFu};
            if constexpr (EPI == W32_GELU_DROP) {
                if (ep.p > 0.f) {
#pragma unroll
                    for (int u = 0; u < 2; ++u) {
                        const uint64_t chunk = (uint64_t)((m * N + n0 + 32 * ft + 8 * u + 4 * h) >> 2);
                        bits8[u] = gelu_keep_bits8(ep.seed, chunk, thr);
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint32_t off = m < M ? (uint32_t)((m * N + n0 + 32 * ft + 8 * u + 4 * h) * 4) : kDrop32;
                const float4 b = bias4[ft][u];
                const float4 v = make_float4(acc[ft][4 * u] + b.x, acc[ft][4 * u + 1] + b.y, acc[ft][4 * u + 2] + b.z,
                                             acc[ft][4 * u + 3] + b.w);
                if constexpr (EPI == W32_STORE) {
                    bstore32(v, yr, off, nt_out);
                } else if constexpr (EPI == W32_ACCUM) {
                    const float4 q = pre[ft][u];
                    bstore32(make_float4(v.x + q.x, v.y + q.y, v.z + q.z, v.w + q.w), yr, off, nt_out);
                } else if constexpr (EPI == W32_GELU_BWD) {
                    const float4 q = pre[ft][u];
                    bstore32(make_float4(v.x * q.x, v.y * q.y, v.z * q.z, v.w * q.w), yr, off, nt_out);
                } else {
                    float fk[4] = {1.f, 1.f, 1.f, 1.f};
                    if (ep.p > 0.f) gelu_keep_factors((bits8[u & 1] >> (4 * (u >> 1))) & 0xFu, keep_k, fk);
                    float gl[4], gd[4];
                    gelu_erf_and_grad(v.x, gl[0], gd[0]);
                    gelu_erf_and_grad(v.y, gl[1], gd[1]);
                    gelu_erf_and_grad(v.z, gl[2], gd[2]);
                    gelu_erf_and_grad(v.w, gl[3], gd[3]);
                    bstore32(make_float4(fk[0] * gd[0], fk[1] * gd[1], fk[2] * gd[2], fk[3] * gd[3]), pr, off, nt_out);
                    bstore32(make_float4(gl[0] * fk[0], gl[1] * fk[1], gl[2] * fk[2], gl[3] * fk[3]), yr, off, nt_out);
                }
            }
        }
    }
}

template <int K, int FT, bool TRANS, int EPI>
int launch_ws32(const float* X, int64_t M, const float* W, int N, float* Y, const Ws32Epi& ep, hipStream_t s) {
    constexpr int NB = 32 * FT;
    constexpr size_t lds = (size_t)NB * K * 6;
    static_assert(lds <= (size_t)kLdsMax32, "W planes exceed the LDS");
    static const hipError_t attr = hipFuncSetAttribute((const void*)ws32_kernel<K, FT, TRANS, EPI>,
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (attr != hipSuccess) return hip_status(attr, "asme_ws_linear: LDS opt-in");
    int dev = 0, cus = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (N / NB > cus / 8) {
        set_error("asme_ws_linear: more feature blocks than workgroups per XCD");
        return -1;
    }
    hipLaunchKernelGGL((ws32_kernel<K, FT, TRANS, EPI>), dim3((cus / 8) * 8), dim3(kWaves32 * 64), lds, s, X, M, W, N,
                       Y, ep);
    return hip_status(hipGetLastError(), "asme_ws_linear");
}

template <int K, bool TRANS, int EPI>
int dispatch_ft32(int ft, const float* X, int64_t M, const float* W, int N, float* Y, const Ws32Epi& ep,
                  hipStream_t s) {
    if constexpr (64 * K * 6 <= kLdsMax32)
        if (ft == 2) return launch_ws32<K, 2, TRANS, EPI>(X, M, W, N, Y, ep, s);
    if constexpr (96 * K * 6 <= kLdsMax32)
        if (ft == 3) return launch_ws32<K, 3, TRANS, EPI>(X, M, W, N, Y, ep, s);
    if constexpr (128 * K * 6 <= kLdsMax32)
        if (ft == 4) return launch_ws32<K, 4, TRANS, EPI>(X, M, W, N, Y, ep, s);
    return launch_ws32<K, 1, TRANS, EPI>(X, M, W, N, Y, ep, s);
}

}  // namespace

namespace asme {
// feature tiles (of 32) per workgroup for the 32x32x16 form, 0 when it does not take (K, N): 64 features when
// N / 64 splits an XCD's 32 workgroups, else 96 or 128 (the W planes within the LDS), else 32
int ws32_pick_ft(int64_t N, int64_t K) {
    if (K != 128 && K != 256 && K != 384) return 0;
    if (N % 32 != 0 || N > 4096) return 0;
    auto fits = [&](int ft) { return N % (32 * ft) == 0 && 32 % (N / (32 * ft)) == 0 && 32 * ft * K * 6 <= kLdsMax32; };
    if (fits(2)) return 2;
    if (fits(3)) return 3;
    if (fits(4)) return 4;
    if (fits(1)) return 1;
    return 0;
}

// Y = X W^T (+ bias) with epilogue epi (0 store, 1 GELU + dropout, 2 through the activation factor, 3 accumulate
// into Y), X rows of stride ldx from column kofs; returns -1 (error set) when the shape is not taken
int ws32_linear(const float* X, int64_t M, int64_t K, const float* W, int64_t N, int trans, const float* bias, int epi,
                float* pre_out, const float* pre_in, float p, uint64_t seed, float* Y, int64_t ldx, int64_t ldw,
                int kofs, void* stream) {
    const int ft = ws32_pick_ft(N, K);
    if (ft == 0) {
        set_error("asme_ws_linear: shape not taken by the 32x32x16 form");
        return -1;
    }
    const Ws32Epi ep{bias, pre_out, pre_in, p, seed, ldx, ldw, kofs};
    hipStream_t s = (hipStream_t)stream;
    const int n = (int)N;
#define ASME_W32_K(KV)                                                                                              \
    if (K == KV) {                                                                                                  \
        if (trans) {                                                                                                \
            if (epi == 0) return dispatch_ft32<KV, true, W32_STORE>(ft, X, M, W, n, Y, ep, s);                      \
            if (epi == 1) return dispatch_ft32<KV, true, W32_GELU_DROP>(ft, X, M, W, n, Y, ep, s);                  \
            if (epi == 2) return dispatch_ft32<KV, true, W32_GELU_BWD>(ft, X, M, W, n, Y, ep, s);                   \
            return dispatch_ft32<KV, true, W32_ACCUM>(ft, X, M, W, n, Y, ep, s);                                    \
        }                                                                                                           \
        if (epi == 0) return dispatch_ft32<KV, false, W32_STORE>(ft, X, M, W, n, Y, ep, s);                         \
        if (epi == 1) return dispatch_ft32<KV, false, W32_GELU_DROP>(ft, X, M, W, n, Y, ep, s);                     \
        if (epi == 2) return dispatch_ft32<KV, false, W32_GELU_BWD>(ft, X, M, W, n, Y, ep, s);                      \
        return dispatch_ft32<KV, false, W32_ACCUM>(ft, X, M, W, n, Y, ep, s);                                       \
    }
    ASME_W32_K(128)
    ASME_W32_K(256)
    ASME_W32_K(384)
#undef ASME_W32_K
    set_error("asme_ws_linear: bad K");
    return -1;
}
}  // namespace asme
