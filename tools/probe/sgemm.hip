// Probe: weight-stationary streaming fp32 GEMM, Y = X W^T + b (X: M x K, W: N x K), C^T MFMA tiles.
// One 512-thread workgroup per CU holds an NB x K block of W (swizzled) in LDS for its whole life; each
// wave streams its own 16*RT-token tiles of X straight from HBM into registers (ring of D k16-blocks in
// flight), no barriers after the W load.  Build: hipcc -O3 --offload-arch=gfx950 -shared -fPIC.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {
typedef float floatx4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ floatx4 mfma16(float a, float b, floatx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void bstore(float4 v, __amdgpu_buffer_rsrc_t r, uint32_t off) {
    const u32x4 u = {__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)};
    __builtin_amdgcn_raw_buffer_store_b128(u, r, off, 0, 0);
}

// W image: row r (feature), 16-B slot s of the K-wide row stored at slot s ^ (r & 15)
__device__ __forceinline__ int wslot(int r, int s, int K4) { return r * K4 + (s ^ (r & 15)); }

template <int NB, int RT, int K, int D, bool TRANS, bool SB, int AB = 0, int WV = 8>
__global__ __launch_bounds__(WV * 64) __attribute__((amdgpu_waves_per_eu(2, 2))) void sgemm_kernel(
    const float* __restrict__ X, int64_t M, const float* __restrict__ W, const float* __restrict__ bias, int N,
    float* __restrict__ Y) {
    constexpr int K4 = K / 4;        // 16-B slots per W row
    constexpr int NKB = K / 16;      // k16 blocks per tile
    constexpr int CT = NB / 16;
    static_assert(NKB % D == 0, "ring depth must divide the k16 blocks of a tile");
    extern __shared__ __attribute__((aligned(16))) float4 lds4[];
    float* bs = reinterpret_cast<float*>(lds4 + NB * K4);
    const int nblk = N / NB;
    const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3, per_xcd = gridDim.x >> 3;
    const int wg_per_nb = per_xcd / nblk;
    if (slot >= wg_per_nb * nblk) return;
    const int nb = slot % nblk;
    const int n0 = nb * NB;
    // ---- W block -> LDS (once)
    if (!TRANS) {
        for (int i = threadIdx.x; i < NB * K4; i += WV * 64) {
            const int r = i / K4, s = i % K4;
            lds4[wslot(r, s, K4)] = *reinterpret_cast<const float4*>(W + (int64_t)(n0 + r) * K + 4 * s);
        }
    } else {  // W is K x N (dX = dY . W): block element (r, k) = W[k][n0 + r]
        float* l = reinterpret_cast<float*>(lds4);
        for (int i = threadIdx.x; i < NB * K; i += WV * 64) {
            const int r = i % NB, k = i / NB;
            l[wslot(r, k >> 2, K4) * 4 + (k & 3)] = W[(int64_t)k * N + n0 + r];
        }
    }
    for (int i = threadIdx.x; i < NB; i += WV * 64) bs[i] = bias ? bias[n0 + i] : 0.f;
    __syncthreads();
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c16 = lane & 15;
    // ---- token tiles of this (XCD, n-block) group of waves
    constexpr int TT = 16 * RT;
    const int64_t ntile = (M + TT - 1) / TT;
    const int64_t lo = ntile * xcd / 8, hi = ntile * (xcd + 1) / 8;
    const int wcount = wg_per_nb * WV;
    const int widx = (slot / nblk) * WV + wave;
    const int64_t my_tiles = hi - lo > widx ? (hi - lo - widx + wcount - 1) / wcount : 0;
    if (my_tiles == 0) return;
    const int64_t lo_tile0 = lo + widx;
    constexpr int GPT = NKB / D;  // ring groups per tile
    const int64_t groups = my_tiles * GPT;
    auto tile_row = [&](int64_t j, int rt) -> int64_t {  // clamped rows are computed and discarded
        const int64_t m = (lo + widx + j * wcount) * TT + rt * 16 + c16;
        return m < M ? m : M - 1;
    };
    // load cursor: the group after the one being computed; its row pointers change once per tile
    int64_t lj = 0;
    int lkb = 0;
    const float* lrow[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) lrow[rt] = X + tile_row(0, rt) * K + 4 * g;
    auto advance = [&]() {
        lkb += D;
        if (lkb == NKB) {
            lkb = 0;
            if (lj + 1 < my_tiles) {  // past the last tile the cursor keeps re-reading it (unconditional loads)
                ++lj;
#pragma unroll
                for (int rt = 0; rt < RT; ++rt) lrow[rt] = X + tile_row(lj, rt) * K + 4 * g;
            }
        }
    };
    float4 ring[D][RT];
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            ring[d][rt] = *reinterpret_cast<const float4*>(lrow[rt] + lkb * 16 + d * 16);
            __builtin_amdgcn_sched_barrier(0);  // issue in ring order: the loop's vmcnt waits assume it
        }
    advance();
    floatx4 acc[RT][CT];
    float4 wc[CT];  // W operands of the current k16 block; the next block's are read one block ahead
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) wc[ct] = lds4[wslot(ct * 16 + c16, g, K4)];
    int kb0 = 0;
    int64_t cj = 0;  // tile being computed
    float4 breg[(AB & 128) ? CT : 1];  // this lane's bias quads, held for the kernel's life
    if constexpr ((AB & 128) != 0) {
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) breg[ct] = *reinterpret_cast<const float4*>(bs + ct * 16 + 4 * g);
    }
    for (int64_t gi = 0; gi < groups; ++gi) {
        if (kb0 == 0) {
#pragma unroll
            for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                for (int ct = 0; ct < CT; ++ct) {
                    acc[rt][ct] = floatx4{0.f, 0.f, 0.f, 0.f};
                    if (AB & 4) asm volatile("" : "+a"(acc[rt][ct]));  // accumulators in AGPRs
                }
        }
        const float* lp[RT];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) lp[rt] = lrow[rt] + lkb * 16;
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const int kb = kb0 + d;
            const int kbn = kb + 1 == NKB ? 0 : kb + 1;
            float4 wn[CT];
#pragma unroll
            for (int ct = 0; ct < CT; ++ct)
                wn[ct] = (AB & 2) ? wc[ct] : lds4[wslot(ct * 16 + c16, kbn * 4 + g, K4)];
            if (SB) __builtin_amdgcn_sched_barrier(0);  // keep the next block's W reads ahead of this block's MFMAs
#pragma unroll
            for (int ct = 0; ct < CT; ++ct)
#pragma unroll
                for (int rt = 0; rt < RT; ++rt) acc[rt][ct] = mfma16(wc[ct].x, ring[d][rt].x, acc[rt][ct]);
#pragma unroll
            for (int ct = 0; ct < CT; ++ct)
#pragma unroll
                for (int rt = 0; rt < RT; ++rt) acc[rt][ct] = mfma16(wc[ct].y, ring[d][rt].y, acc[rt][ct]);
#pragma unroll
            for (int ct = 0; ct < CT; ++ct)
#pragma unroll
                for (int rt = 0; rt < RT; ++rt) acc[rt][ct] = mfma16(wc[ct].z, ring[d][rt].z, acc[rt][ct]);
#pragma unroll
            for (int ct = 0; ct < CT; ++ct)
#pragma unroll
                for (int rt = 0; rt < RT; ++rt) acc[rt][ct] = mfma16(wc[ct].w, ring[d][rt].w, acc[rt][ct]);
            // refill the slot just consumed (same registers every trip: no rotation copies at the back edge);
            // unconditional so the vmcnt tracking stays exact
#pragma unroll
            for (int rt = 0; rt < RT; ++rt)
                if (!(AB & 1)) ring[d][rt] = *reinterpret_cast<const float4*>(lp[rt] + d * 16);
#pragma unroll
            for (int ct = 0; ct < CT; ++ct) wc[ct] = wn[ct];
            if (SB) __builtin_amdgcn_sched_barrier(0);
        }
        advance();
        kb0 += D;
        if (kb0 == NKB) {  // tile done: epilogue
            kb0 = 0;
            if constexpr ((AB & 16) != 0) {
                // 128-B row segments per store: lanes c16 and c16^8 (DPP row_ror:8) trade the odd/even
                // 16-feature tiles so each instruction covers 8 rows x 128 contiguous bytes
                const bool lo = c16 < 8;
                const int col = (lo ? 0 : 16) + 4 * g;
#pragma unroll
                for (int rt = 0; rt < RT; ++rt) {
                    const int64_t mA = (lo_tile0 + cj * wcount) * TT + rt * 16 + (c16 & 7);
                    const int64_t mB = mA + 8;
                    float* yA = Y + mA * N + n0 + col;
                    float* yB = Y + mB * N + n0 + col;
#pragma unroll
                    for (int q = 0; q < CT / 2; ++q) {
                        const float4 be = *reinterpret_cast<const float4*>(bs + 32 * q + 4 * g);
                        const float4 bo = *reinterpret_cast<const float4*>(bs + 32 * q + 16 + 4 * g);
                        float e[4], o[4], give[4], got[4];
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            e[i] = acc[rt][2 * q][i] + (&be.x)[i];
                            o[i] = acc[rt][2 * q + 1][i] + (&bo.x)[i];
                            give[i] = lo ? o[i] : e[i];
                            got[i] = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(give[i]), 0x128, 0xF, 0xF, false));
                        }
                        const float4 va = lo ? make_float4(e[0], e[1], e[2], e[3]) : make_float4(got[0], got[1], got[2], got[3]);
                        const float4 vb = lo ? make_float4(got[0], got[1], got[2], got[3]) : make_float4(o[0], o[1], o[2], o[3]);
                        if (mA < M) *reinterpret_cast<float4*>(yA + 32 * q) = va;
                        if (mB < M) *reinterpret_cast<float4*>(yB + 32 * q) = vb;
                    }
                }
            } else {
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) {
                const int64_t m = (lo + widx + cj * wcount) * TT + rt * 16 + c16;
                if (m >= M) continue;
                float* yrow = Y + m * N + n0 + 4 * g;
#pragma unroll
                for (int ct = 0; ct < CT; ++ct) {
                    const float4 b = (AB & 128) ? breg[ct] : *reinterpret_cast<const float4*>(bs + ct * 16 + 4 * g);
                    const float4 o = make_float4(acc[rt][ct][0] + b.x, acc[rt][ct][1] + b.y, acc[rt][ct][2] + b.z,
                                    acc[rt][ct][3] + b.w);
                    float* dst = (AB & 64) ? Y + (m & 511) * N + n0 + 4 * g + ct * 16 : yrow + ct * 16;
                    if (AB & 32) {
                        __builtin_nontemporal_store(o.x, dst);
                        __builtin_nontemporal_store(o.y, dst + 1);
                        __builtin_nontemporal_store(o.z, dst + 2);
                        __builtin_nontemporal_store(o.w, dst + 3);
                    } else if (!(AB & 8) || o.x == 12345.f) {
                        *reinterpret_cast<float4*>(dst) = o;
                    }
                }
            }
            }
            ++cj;
        }
    }
}

// v2: one loop trip per token tile (all K/16 blocks unrolled); the finished tile's outputs (+bias) move to
// a stash and are written by buffer stores spread over the NEXT tile's first blocks, so no instruction
// overwrites a store's source registers until a whole tile later; rows past M are dropped by the buffer
// range check (Y < 2 GiB).
template <int NB, int RT, int K, int D, bool TRANS, int OCC>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(OCC, OCC))) void sgemm2_kernel(
    const float* __restrict__ X, int64_t M, const float* __restrict__ W, const float* __restrict__ bias, int N,
    float* __restrict__ Y) {
    constexpr int K4 = K / 4;
    constexpr int NKB = K / 16;
    constexpr int CT = NB / 16;
    static_assert(NKB % D == 0, "ring depth must divide the k16 blocks of a tile");
    extern __shared__ __attribute__((aligned(16))) float4 lds4[];
    float* bs = reinterpret_cast<float*>(lds4 + NB * K4);
    const int nblk = N / NB;
    const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3, per_xcd = gridDim.x >> 3;
    const int wg_per_nb = per_xcd / nblk;
    if (slot >= wg_per_nb * nblk) return;
    const int nb = slot % nblk;
    const int n0 = nb * NB;
    if (!TRANS) {
        for (int i = threadIdx.x; i < NB * K4; i += 512) {
            const int r = i / K4, s = i % K4;
            lds4[wslot(r, s, K4)] = *reinterpret_cast<const float4*>(W + (int64_t)(n0 + r) * K + 4 * s);
        }
    } else {
        float* l = reinterpret_cast<float*>(lds4);
        for (int i = threadIdx.x; i < NB * K; i += 512) {
            const int r = i % NB, k = i / NB;
            l[wslot(r, k >> 2, K4) * 4 + (k & 3)] = W[(int64_t)k * N + n0 + r];
        }
    }
    for (int i = threadIdx.x; i < NB; i += 512) bs[i] = bias ? bias[n0 + i] : 0.f;
    __syncthreads();
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c16 = lane & 15;
    constexpr int TT = 16 * RT;
    const int64_t ntile = (M + TT - 1) / TT;
    const int64_t lo = ntile * xcd / 8, hi = ntile * (xcd + 1) / 8;
    const int wcount = wg_per_nb * 8;
    const int widx = (slot / nblk) * 8 + wave;
    const int64_t my_tiles = hi - lo > widx ? (hi - lo - widx + wcount - 1) / wcount : 0;
    if (my_tiles == 0) return;
    const int64_t t0 = lo + widx;
    auto row_of = [&](int64_t j, int rt) -> int64_t { return (t0 + j * wcount) * TT + rt * 16 + c16; };
    auto xrow = [&](int64_t j, int rt) -> const float* {
        const int64_t m = row_of(j < my_tiles ? j : my_tiles - 1, rt);
        return X + (m < M ? m : M - 1) * K + 4 * g;
    };
    const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc(Y, 0, (int)(M * N * 4), 0x00020000);
    constexpr uint32_t kDrop = 0x80000000u;  // >= the record count: the store is dropped
    float4 breg[CT];
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) breg[ct] = *reinterpret_cast<const float4*>(bs + ct * 16 + 4 * g);
    const float* rc[RT];
    const float* rn[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
        rc[rt] = xrow(0, rt);
        rn[rt] = xrow(1, rt);
    }
    float4 ring[D][RT];
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            ring[d][rt] = *reinterpret_cast<const float4*>(rc[rt] + d * 16);
            __builtin_amdgcn_sched_barrier(0);
        }
    float4 stash[RT][CT];
    uint32_t soff[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) soff[rt] = kDrop;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) stash[rt][ct] = make_float4(0.f, 0.f, 0.f, 0.f);
    float4 wc[CT];
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) wc[ct] = lds4[wslot(ct * 16 + c16, g, K4)];
    floatx4 acc[RT][CT];
    for (int64_t j = 0; j < my_tiles; ++j) {
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
            for (int ct = 0; ct < CT; ++ct) acc[rt][ct] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb) {
            const int kbn = kb + 1 == NKB ? 0 : kb + 1;
            float4 wn[CT];
#pragma unroll
            for (int ct = 0; ct < CT; ++ct) wn[ct] = lds4[wslot(ct * 16 + c16, kbn * 4 + g, K4)];
            __builtin_amdgcn_sched_barrier(0);
            const int d = kb % D;
#pragma unroll
            for (int ct = 0; ct < CT; ++ct)
#pragma unroll
                for (int rt = 0; rt < RT; ++rt) acc[rt][ct] = mfma16(wc[ct].x, ring[d][rt].x, acc[rt][ct]);
#pragma unroll
            for (int ct = 0; ct < CT; ++ct)
#pragma unroll
                for (int rt = 0; rt < RT; ++rt) acc[rt][ct] = mfma16(wc[ct].y, ring[d][rt].y, acc[rt][ct]);
#pragma unroll
            for (int ct = 0; ct < CT; ++ct)
#pragma unroll
                for (int rt = 0; rt < RT; ++rt) acc[rt][ct] = mfma16(wc[ct].z, ring[d][rt].z, acc[rt][ct]);
#pragma unroll
            for (int ct = 0; ct < CT; ++ct)
#pragma unroll
                for (int rt = 0; rt < RT; ++rt) acc[rt][ct] = mfma16(wc[ct].w, ring[d][rt].w, acc[rt][ct]);
            // refill: block kb + D of this tile, or of the next one
#pragma unroll
            for (int rt = 0; rt < RT; ++rt)
                ring[d][rt] = *reinterpret_cast<const float4*>(
                    (kb + D < NKB ? rc[rt] : rn[rt]) + ((kb + D) % NKB) * 16);
            // the previous tile's outputs, one 16-feature tile at a time
#pragma unroll
            for (int ct = 0; ct < CT; ++ct)
                if (ct * NKB / CT == kb)
#pragma unroll
                    for (int rt = 0; rt < RT; ++rt)
                        bstore(stash[rt][ct], yr, soff[rt] + ct * 64);
#pragma unroll
            for (int ct = 0; ct < CT; ++ct) wc[ct] = wn[ct];
            __builtin_amdgcn_sched_barrier(0);
        }
        // tile done: outputs to the stash, stored during the next tile
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            const int64_t m = row_of(j, rt);
            soff[rt] = m < M ? (uint32_t)((m * N + n0 + 4 * g) * 4) : kDrop;
#pragma unroll
            for (int ct = 0; ct < CT; ++ct)
                stash[rt][ct] = make_float4(acc[rt][ct][0] + breg[ct].x, acc[rt][ct][1] + breg[ct].y,
                                            acc[rt][ct][2] + breg[ct].z, acc[rt][ct][3] + breg[ct].w);
        }
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            rc[rt] = rn[rt];
            rn[rt] = xrow(j + 2, rt);
        }
    }
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
            bstore(stash[rt][ct], yr, soff[rt] + ct * 64);
}

template <int NB, int RT, int K, int D, bool TRANS, int OCC = 2>
int launch2(const float* X, int64_t M, const float* W, const float* b, int N, float* Y, int grid, hipStream_t s) {
    if ((int64_t)M * N * 4 >= 0x80000000LL) return -2;
    const size_t lds = (size_t)NB * K * 4 + NB * 4;
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)sgemm2_kernel<NB, RT, K, D, TRANS, OCC>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        attr = true;
    }
    hipLaunchKernelGGL((sgemm2_kernel<NB, RT, K, D, TRANS, OCC>), dim3(grid * OCC / 2), dim3(512), lds, s, X, M, W, b, N, Y);
    return (int)hipGetLastError();
}

template <int NB, int RT, int K, int D, bool TRANS, bool SB = true, int AB = 0, int WV = 8>
int launch(const float* X, int64_t M, const float* W, const float* b, int N, float* Y, int grid, hipStream_t s) {
    const size_t lds = (size_t)NB * K * 4 + NB * 4;
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)sgemm_kernel<NB, RT, K, D, TRANS, SB, AB, WV>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        attr = true;
    }
    hipLaunchKernelGGL((sgemm_kernel<NB, RT, K, D, TRANS, SB, AB, WV>), dim3(grid * 8 / WV), dim3(WV * 64), lds, s, X, M, W, b, N, Y);
    return (int)hipGetLastError();
}
}  // namespace

extern "C" int run_sgemm(int variant, const float* X, int64_t M, int K, const float* W, const float* b, int N,
                         float* Y, int grid, void* stream) {
    hipStream_t s = (hipStream_t)stream;
    switch (variant) {
        // forward, K = 128
        case 0: return launch<128, 1, 128, 8, false>(X, M, W, b, N, Y, grid, s);
        case 1: return launch<128, 2, 128, 4, false>(X, M, W, b, N, Y, grid, s);
        case 2: return launch<64, 2, 128, 8, false>(X, M, W, b, N, Y, grid, s);
        case 3: return launch<256, 1, 128, 4, false>(X, M, W, b, N, Y, grid, s);
        // K = 512
        case 4: return launch<64, 1, 512, 8, false>(X, M, W, b, N, Y, grid, s);
        case 5: return launch<64, 2, 512, 8, false>(X, M, W, b, N, Y, grid, s);
        case 6: return launch<32, 4, 512, 8, false>(X, M, W, b, N, Y, grid, s);
        // dX forms (W: K x N)
        case 7: return launch<128, 1, 128, 8, true>(X, M, W, b, N, Y, grid, s);
        case 8: return launch<64, 2, 512, 8, true>(X, M, W, b, N, Y, grid, s);
        case 9: return launch<128, 2, 128, 4, false, false>(X, M, W, b, N, Y, grid, s);
        case 10: return launch<64, 2, 512, 8, false, false>(X, M, W, b, N, Y, grid, s);
        case 11: return launch<128, 1, 128, 8, false, true, 1>(X, M, W, b, N, Y, grid, s);
        case 12: return launch<128, 1, 128, 8, false, true, 2>(X, M, W, b, N, Y, grid, s);
        case 13: return launch<128, 1, 128, 8, false, true, 3>(X, M, W, b, N, Y, grid, s);
        case 14: return launch<128, 1, 128, 8, false, true, 4>(X, M, W, b, N, Y, grid, s);
        case 15: return launch<128, 2, 128, 4, false, true, 4>(X, M, W, b, N, Y, grid, s);
        case 16: return launch<64, 2, 512, 8, false, true, 4>(X, M, W, b, N, Y, grid, s);
        case 17: return launch<128, 1, 128, 8, false, true, 7>(X, M, W, b, N, Y, grid, s);
        case 18: return launch<128, 1, 128, 8, false, true, 11>(X, M, W, b, N, Y, grid, s);  // no mem at all
        case 19: return launch<128, 1, 128, 8, false, true, 0, 4>(X, M, W, b, N, Y, grid, s);   // 4-wave WGs
        case 20: return launch<128, 1, 128, 8, false, true, 3, 4>(X, M, W, b, N, Y, grid, s);
        case 21: return launch<128, 1, 128, 8, false, true, 11, 4>(X, M, W, b, N, Y, grid, s);
        case 22: return launch<128, 1, 128, 8, false, true, 16>(X, M, W, b, N, Y, grid, s);
        case 23: return launch<128, 2, 128, 4, false, true, 16>(X, M, W, b, N, Y, grid, s);
        case 24: return launch<64, 2, 512, 8, false, true, 16>(X, M, W, b, N, Y, grid, s);
        case 25: return launch<64, 1, 512, 8, false, true, 16>(X, M, W, b, N, Y, grid, s);
        case 26: return launch<128, 1, 128, 8, true, true, 16>(X, M, W, b, N, Y, grid, s);
        case 27: return launch<64, 2, 512, 8, true, true, 16>(X, M, W, b, N, Y, grid, s);
        case 28: return launch<128, 1, 128, 8, false, true, 32>(X, M, W, b, N, Y, grid, s);   // nontemporal
        case 29: return launch<128, 1, 128, 8, false, true, 64>(X, M, W, b, N, Y, grid, s);   // L2-resident dst
        case 30: return launch<128, 1, 128, 8, false, true, 3 | 64>(X, M, W, b, N, Y, grid, s);
        case 31: return launch<128, 1, 128, 8, false, true, 3 | 32>(X, M, W, b, N, Y, grid, s);
        case 32: return launch<128, 1, 128, 8, false, true, 128>(X, M, W, b, N, Y, grid, s);
        case 33: return launch<128, 1, 128, 8, false, true, 128 | 3>(X, M, W, b, N, Y, grid, s);
        case 34: return launch<128, 2, 128, 4, false, true, 128>(X, M, W, b, N, Y, grid, s);
        case 35: return launch<64, 2, 512, 8, false, true, 128>(X, M, W, b, N, Y, grid, s);
        case 36: return launch<64, 1, 512, 8, false, true, 128>(X, M, W, b, N, Y, grid, s);
        case 40: return launch2<128, 1, 128, 8, false>(X, M, W, b, N, Y, grid, s);
        case 41: return launch2<128, 2, 128, 4, false>(X, M, W, b, N, Y, grid, s);
        case 42: return launch2<64, 2, 512, 8, false>(X, M, W, b, N, Y, grid, s);
        case 43: return launch2<64, 1, 512, 8, false>(X, M, W, b, N, Y, grid, s);
        case 44: return launch2<128, 1, 128, 8, true>(X, M, W, b, N, Y, grid, s);
        case 45: return launch2<64, 2, 512, 8, true>(X, M, W, b, N, Y, grid, s);
        case 46: return launch2<64, 1, 128, 8, false>(X, M, W, b, N, Y, grid, s);
        case 47: return launch2<64, 1, 128, 8, false, 3>(X, M, W, b, N, Y, grid, s);
        case 48: return launch2<64, 1, 128, 8, false, 4>(X, M, W, b, N, Y, grid, s);
        case 49: return launch2<64, 1, 128, 4, false, 4>(X, M, W, b, N, Y, grid, s);
        case 50: return launch2<64, 1, 512, 4, false, 3>(X, M, W, b, N, Y, grid, s);
        case 51: return launch2<64, 1, 512, 8, false, 3>(X, M, W, b, N, Y, grid, s);
        case 52: return launch2<32, 1, 512, 8, false, 4>(X, M, W, b, N, Y, grid, s);
        case 53: return launch2<128, 1, 128, 8, false, 3>(X, M, W, b, N, Y, grid, s);
        default: return -1;
    }
}
