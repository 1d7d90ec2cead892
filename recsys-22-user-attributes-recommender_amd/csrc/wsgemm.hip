// Weight-stationary streaming GEMM for the token-major Linear layers: fp32 products on the bf16 matrix cores
// (bf16x6 split operands, common.h) on gfx950.
//
// Reference semantics (paths relative to /root/reference/src/asme):
//   nn.Linear projections         core/models/common/layers/transformer_layers.py:175-199 (Q,K,V,O)
//   PositionwiseFeedForward       transformer_layers.py:212-220  W2(dropout(GELU_erf(W1 x)))
// The shapes of the ASME transformer are tall and skinny: M = B*L tokens (2e5 at the bench shape) against
// K, N <= 512.  So the kernel keeps one NB x K block of the weight in LDS for the workgroup's whole life
// (split once into three bf16 planes h, m, l; the hot loop has no barrier) and every wave streams its own
// 16-token tiles of X from HBM straight into registers, kD k32 blocks in flight, while it multiplies the
// previous ones:
//   C^T tile (NB features x 16 tokens) += W_blk (NB x 32 k) . X_tile^T (32 k x 16 tokens)
// as six v_mfma_f32_16x16x32_bf16 per 16-feature tile (mm, hl, lh, hm, mh, hh).  Lane (c16, g) of an MFMA
// supplies k = 8g..8g+7 of one 32-k block for its feature / token, so the X rows are read as two float4 (4
// lanes = 128 contiguous bytes of a row) and split in registers once per block for all CT feature tiles, and
// the W planes as conflict-free ds_read_b128 (W image row r, 16-B slot s stored at slot s ^ (r & 15)).
// Each feature tile's next-block W read goes out right after its MFMAs consumed the registers.
// Epilogue: a finished tile's accumulators (+ bias) move to a stash and are written by buffer stores
// spread over the NEXT tile's k blocks, one 16-feature tile per block -- nothing overwrites a store's source
// registers until a tile later (an LDS read or MFMA landing on them right after the store stalls the
// wave until the store has left), and rows past M are dropped by the buffer range check.
// Epilogues: WS_STORE       Y = C (+ bias)
//            WS_GELU_DROP   pre = C + bias; Y = dropout(GELU(pre)); A = keep * GELU'(pre)   (FFN inner, forward)
//            WS_GELU_BWD    Y = C * A                                                   (through the activation)
//            WS_ACCUM       Y = C + Y                        (the second K = 256 half of a K = 512 product)
//            WS_RESID_LN    s = drop_b(res + drop_a(C + bias)) -> Y;  LN(s) -> ln_out, (mean, rstd) -> stats
//                           (the attention output projection fused with the SublayerConnection residual and the
//                           next pre-LN, transformer_layers.py:120-130 + 251-258: one 128-feature block is a whole
//                           row, so the row statistics are a 32-lane reduction in the epilogue -- the same
//                           rows.h sequence as asme_residual_ln_fwd, bit-identical to the unfused pair)
// A (the activation factor, written by the forward in place of the pre-activation, same bytes) makes the
// backward epilogue a single multiply: no Philox, erf or exp in the input-gradient GEMM.
// Dropout decisions are exactly those of asme_gelu_dropout_fwd/bwd (norm.hip): one Philox block per pair of
// 4-element chunks, 16-bit uniforms, salt 5 (common.h gelu_keep_bits8).
// Measured at M = 204800 (tools/probe/ab_ws.py; fp32-equivalent rate, bf16x6 ceiling 2516.6 / 6 = 419 TF/s):
// K=128 -> N=128 165 TF/s, K=384 -> N=128 (input gradient) 181, K=128 -> N=512 142 (row-staged stores),
// K=512 -> N=128 145 (as two K = 256 halves); the fp32-MFMA version of this kernel (157 TF/s ceiling): 113-126.
#include "common.h"
#include "rows.h"

using namespace asme;

namespace {

typedef unsigned u32v4 __attribute__((ext_vector_type(4)));

constexpr int kD = 4;               // k32 blocks of X in flight per wave
constexpr int kWaves = 8;           // 512-thread workgroups, one per CU, two waves per SIMD
constexpr int kLdsMax = 160 * 1024;
constexpr uint32_t kDrop = 0x80000000u;  // >= every buffer's record count: the access is dropped / reads 0

enum { WS_STORE = 0, WS_GELU_DROP = 1, WS_GELU_BWD = 2, WS_ACCUM = 3, WS_RESID_LN = 4 };

struct WsEpi {
    const float* bias;   // [N] or null
    float* pre_out;      // WS_GELU_DROP: activation factor keep * GELU'(pre) out
    const float* pre_in; // WS_GELU_BWD: activation factor in
    float p;             // dropout probability (0: none)
    uint64_t seed;
    // split-K over K = 512 (two K = 256 launches, the second WS_ACCUM): row strides of X and (non-trans) W and the
    // first k column
    int64_t ldx, ldw;
    int kofs;
    // WS_RESID_LN (pre_in = the residual, pre_out = the LayerNorm output; p / seed = drop_a): drop_b, the LayerNorm
    // parameters (null: no LayerNorm, s only) and its per-row (mean, rstd)
    float p2;
    uint64_t seed2;
    const float* ln_w;
    const float* ln_b;
    float eps;
    float* stats;
};

__device__ __forceinline__ int wslot(int r, int s, int K4) { return r * K4 + (s ^ (r & 15)); }
// Output stores of the wide launches (N >= kNtMinN: the QKV projection, the FFN's first GEMM and its GELU form) carry
// the non-temporal hint (aux bit 1, nt): measured alone (tools/probe/ab_ws.py, same process) N = 512 185 -> 148 us,
// GELU forward 318 -> 286 us, N = 384 120 -> 105 us; the N = 128 launches are unchanged or slower with it (K = 384
// input gradient 116 -> 121 us), so they keep the default policy.  (sc1 stores: no change.)
#ifndef ASME_WS_NT_MIN_N
#define ASME_WS_NT_MIN_N 384
#endif
constexpr int kNtMinN = ASME_WS_NT_MIN_N;
#ifndef ASME_WS_DIAG
#define ASME_WS_DIAG 0  // diagnostic builds (tools/ws_ab.py): 1 no MFMA, 2 no stores, 3 no W reads in the loop, 4 no X,
#endif                  // 5 no bf16 split of X (one plane reinterpreted: wrong products, timing only)
__device__ __forceinline__ void bstore(float4 v, __amdgpu_buffer_rsrc_t r, uint32_t off, bool nt) {
    if (ASME_WS_DIAG == 2) off = kDrop;
    const u32v4 u = {__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)};
    if (nt)  // (wave-uniform)
        __builtin_amdgcn_raw_buffer_store_b128(u, r, off, 0, 2);
    else
        __builtin_amdgcn_raw_buffer_store_b128(u, r, off, 0, 0);
}
__device__ __forceinline__ float4 bload(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    const u32v4 u = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
    return make_float4(__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z), __uint_as_float(u.w));
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, int64_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}

// X: M x K row-major.  TRANS = false: W is N x K (nn.Linear.weight), Y = X W^T.  TRANS = true: W is K x N
// (the input gradient dX = dY W of a layer whose weight is N_out x N_in = K x N).
// XP: X arrives already split into its three bf16 planes ([3][M][ldx] bf16, written by its producer): the ring holds
// the planes and the loop issues no split VALU (an experiment: asme_ws_linear_planes)
// (round 6, measured and removed -- git history before the commit that dropped them: four waves per SIMD on 16-wave
// workgroups, the W block register-resident at one wave per SIMD, K = 512 in one launch on 32-feature blocks, issue
// priority around the MFMA chains; all slower)
template <int K, int CT, bool TRANS, int EPI, bool XP = false>
__global__ __launch_bounds__(kWaves * 64) __attribute__((amdgpu_waves_per_eu(2, 2))) void ws_gemm_kernel(
    const float* __restrict__ X, int64_t M, const float* __restrict__ W, int N, float* __restrict__ Y, WsEpi ep) {
    constexpr int NB = 16 * CT;  // output features per workgroup
    // k32 blocks of X in flight: the whole 8-block tile for the first K = 256 half of the FFN-out forward (its waves
    // wait on X most; 256 VGPRs, no spill; tools/ws_ab.py same process 180 -> 173 us per product; the input-gradient
    // form and K = 384 measured flat or slower with a deeper ring)
    constexpr int RD = (K == 256 && EPI == WS_STORE && !TRANS) ? 8 : kD;
    constexpr int K8 = K / 8;    // 16-B slots (8 bf16) of a W image row
    constexpr int NKB = K / 32;
    constexpr int PL = NB * K8;  // slots of one bf16 plane
    static_assert(NKB % RD == 0, "the ring depth must divide the k32 blocks of a tile");
    static_assert(CT % 2 == 0, "GELU-dropout Philox blocks serve feature-tile pairs");
    // row-major staging of the finished tile (per wave, 16 rows x NB, 16-B row pad) so each store instruction
    // writes whole rows (16 lanes x 16 B = 256 B of one row at NB = 64) instead of 16 rows x 64 B (measured:
    // N = 384 / 512 launches 12-23 % faster); not where the W planes leave no room for it
    // CT = 8 (128-feature blocks, K = 128: the W planes take 96 KiB): the staging rows are not padded but their
    // 16-B chunks XOR-swizzled by the row (the 160 KiB hold planes + staging exactly), conflict-free both ways
    constexpr bool kSwz = CT == 8;
    constexpr int NB4 = NB / 4, SROW = kSwz ? NB : NB + 4;
    constexpr bool kStage = CT >= 4 && NB * K * 6 + kWaves * 16 * SROW * 4 <= kLdsMax;  // (CT = 2: no gain)
    // W fragments in flight: one k32 block ahead for every feature tile (CT <= 6), or a ring of four tiles ahead
    // (CT = 8: 48 instead of 96 registers; still 24 MFMAs between a fragment's read and its use)
    constexpr int WR = CT <= 6 ? CT : 4;
    extern __shared__ __attribute__((aligned(16))) uint4 lds16[];
    const int nblk = N / NB;
    const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3, per_xcd = gridDim.x >> 3;
    const int wg_per_nb = per_xcd / nblk;  // the workgroups of one XCD split over the feature blocks
    if (slot >= wg_per_nb * nblk) return;
    const int nb = slot % nblk;
    const int n0 = nb * NB;
    // ---- the W block, once, split into its three bf16 planes (h, m, l)
    for (int i = threadIdx.x; i < NB * K8; i += kWaves * 64) {
        // TRANS: block element (r, k) = W[k][n0 + r], lanes on consecutive r (coalesced column reads)
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
        const Bf3 p = split_bf3(a, b);
        const int sl = wslot(r, s8, K8);
        lds16[sl] = __builtin_bit_cast(uint4, p.h);
        lds16[PL + sl] = __builtin_bit_cast(uint4, p.m);
        lds16[2 * PL + sl] = __builtin_bit_cast(uint4, p.l);
    }
    __syncthreads();
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c16 = lane & 15;
    // ---- 16-token tiles of this (XCD, feature block): contiguous per XCD, strided over its waves
    const int64_t ntile = (M + 15) / 16;
    const int64_t lo = ntile * xcd / 8, hi = ntile * (xcd + 1) / 8;
    const int wcount = wg_per_nb * kWaves;
    const int widx = (slot / nblk) * kWaves + wave;
    const int64_t my_tiles = hi - lo > widx ? (hi - lo - widx + wcount - 1) / wcount : 0;
    if (my_tiles == 0) return;
    const int64_t t0 = lo + widx;
    auto xrow = [&](int64_t j) -> const float* {  // clamped rows are computed and dropped at the store
        int64_t m = (t0 + (j < my_tiles ? j : my_tiles - 1) * wcount) * 16 + c16;
        // (XP: the same element offset into the h plane, as a float pointer of half the distance)
        return XP ? reinterpret_cast<const float*>(reinterpret_cast<const __bf16*>(X) +
                                                   (m < M ? m : M - 1) * ep.ldx + ep.kofs + 8 * g)
                  : X + (m < M ? m : M - 1) * ep.ldx + ep.kofs + 8 * g;
    };
    const int64_t pl_bytes = M * ep.ldx * 2;  // XP: bytes between the planes
    // k32 block d of X at row pointer r: fp32 (two float4) or the three planes' 16 B
    auto xload = [&](const float* rp, int d, float4& a, float4& b, float4& c) {
        if constexpr (XP) {
            const char* pb = reinterpret_cast<const char*>(rp) + d * 64;
            a = *reinterpret_cast<const float4*>(pb);
            b = *reinterpret_cast<const float4*>(pb + pl_bytes);
            c = *reinterpret_cast<const float4*>(pb + 2 * pl_bytes);
        } else {
            a = *reinterpret_cast<const float4*>(rp + d * 32);
            b = *reinterpret_cast<const float4*>(rp + d * 32 + 4);
        }
    };
    auto xsplit = [&](const float4& a, const float4& b, const float4& c) -> Bf3 {
        if constexpr (XP) {
            Bf3 r;
            r.h = __builtin_bit_cast(bf16x8, a);
            r.m = __builtin_bit_cast(bf16x8, b);
            r.l = __builtin_bit_cast(bf16x8, c);
            return r;
        } else {
            (void)c;
            if (ASME_WS_DIAG == 5) {
                Bf3 r;
                r.h = __builtin_bit_cast(bf16x8, a);
                r.m = r.h;
                r.l = __builtin_bit_cast(bf16x8, b);
                return r;
            }
            return split_bf3(a, b);
        }
    };
    const __amdgpu_buffer_rsrc_t yr = rsrc(Y, M * N * 4);
    const bool nt_out = N >= kNtMinN;
    // the second operand stream of the epilogue: the activation factor (GELU forward writes / backward reads it) or,
    // for WS_ACCUM (second K half), Y itself -- read at the tile boundary like the factor, so the epilogue's
    // read-modify-write never drains the X ring (a load right before the store made the wave wait for vmcnt(0))
    const __amdgpu_buffer_rsrc_t pr = EPI == WS_ACCUM ? yr
                                    : rsrc(EPI == WS_GELU_DROP ? (const void*)ep.pre_out : (const void*)ep.pre_in,
                                           EPI == WS_STORE ? 0 : M * N * 4);
    static_assert(EPI != WS_RESID_LN || (kStage && CT == 8 && NB == 128),
                  "the residual + LayerNorm epilogue needs whole 128-feature rows in the staged tile");
    // WS_RESID_LN: the LayerNorm output stream and this lane's four LayerNorm weights / biases (its staged float4 is
    // always features 4 (lane % 32) .. +3), held in registers: no parameter load inside the epilogue
    const __amdgpu_buffer_rsrc_t lr = rsrc(ep.pre_out, EPI == WS_RESID_LN && ep.ln_w ? M * N * 4 : 0);
    float4 lnw = make_float4(0.f, 0.f, 0.f, 0.f), lnb = lnw;
    if (EPI == WS_RESID_LN && ep.ln_w) {
        lnw = *reinterpret_cast<const float4*>(ep.ln_w + 4 * (threadIdx.x & 31));
        lnb = *reinterpret_cast<const float4*>(ep.ln_b + 4 * (threadIdx.x & 31));
    }
    // the bias: added where the staged tile is read back when every read of a lane falls on the same float4 of
    // the feature block (64 % NB4 == 0: one register set instead of CT), else to the accumulators at the tile's end
    constexpr bool kBiasEpi = kStage && 64 % NB4 == 0;
    float4 breg[kBiasEpi ? 1 : CT];
#pragma unroll
    for (int ct = 0; ct < (kBiasEpi ? 1 : CT); ++ct)
        breg[ct] = !ep.bias ? make_float4(0.f, 0.f, 0.f, 0.f)
                 : kBiasEpi ? *reinterpret_cast<const float4*>(ep.bias + n0 + 4 * ((threadIdx.x & 63) % NB4))
                            : *reinterpret_cast<const float4*>(ep.bias + n0 + ct * 16 + 4 * g);
    const float keep_k = ep.p > 0.f ? 1.f / (1.f - ep.p) : 1.f;
    const uint32_t thr = gelu_thresh(ep.p);
    uint32_t pend = 0;  // GELU-dropout bits of the odd feature tile of the current pair
    const float* rc = xrow(0);
    const float* rn = xrow(1);
    float4 ring[2 * RD];  // k32 block d of X: ring[2d] (k 8g..8g+3), ring[2d + 1] (k 8g+4..8g+7)
    float4 ring3[XP ? RD : 1];  // XP: the l plane of block d (ring[2d] = h, ring[2d + 1] = m)
#pragma unroll
    for (int d = 0; d < RD; ++d) {
        xload(rc, d, ring[2 * d], ring[2 * d + 1], ring3[XP ? d : 0]);
        __builtin_amdgcn_sched_barrier(0);  // issue in ring order: the loop's vmcnt waits assume it
    }
    // GELU backward on 128-feature blocks: the activation factor of the stashed tile is read four feature tiles ahead
    // of its epilogue (a 4-slot ring) instead of all CT at the tile boundary, which would need CT x 4 more registers
    constexpr bool kLateA = EPI == WS_GELU_BWD && CT == 8;
    constexpr int NPRE = kLateA ? 4 : CT;
    float4 stash[CT], pre[NPRE];
    uint32_t soff = kDrop;  // byte offset of (row, n0 + 4g) of the stashed tile in Y
    int64_t srow0 = M;      // staged: first token of the stashed tile (M: none yet, every store dropped)
    float* stg = reinterpret_cast<float*>(lds16 + 3 * PL) + (threadIdx.x >> 6) * 16 * SROW;
    // staged store instruction ct: float4 64 ct + lane of the tile (row-major), its byte offset in Y
    auto staged_off = [&](int ct, int64_t r0) -> uint32_t {
        const int idx = 64 * ct + (threadIdx.x & 63), row = idx / NB4, c4 = idx % NB4;
        return r0 + row < M ? (uint32_t)(((r0 + row) * N + n0 + 4 * c4) * 4) : kDrop;
    };
    auto stg_at = [&](int row, int c4) -> float* {  // float4 chunk c4 of staging row `row` (row < 16)
        return stg + row * SROW + 4 * (kSwz ? (c4 ^ row) : c4);
    };
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) stash[ct] = pre[ct % NPRE] = make_float4(0.f, 0.f, 0.f, 0.f);
    // W operand of feature tile ct, k32 block kb: row ct*16 + c16, k 8g..8g+7 of the three planes
    auto wload = [&](int ct, int kb) -> Bf3 {
        const int sl = wslot(ct * 16 + c16, kb * 4 + g, K8);
        Bf3 w;
        w.h = __builtin_bit_cast(bf16x8, lds16[sl]);
        w.m = __builtin_bit_cast(bf16x8, lds16[PL + sl]);
        w.l = __builtin_bit_cast(bf16x8, lds16[2 * PL + sl]);
        return w;
    };
    Bf3 wc[WR];  // wc[ct % WR] holds tile ct's fragment of the current block when its MFMAs run
#pragma unroll
    for (int ct = 0; ct < WR; ++ct) wc[ct] = wload(ct, 0);
    Bf3 xs = xsplit(ring[0], ring[1], ring3[0]);
    // the stashed tile's epilogue for one 16-feature tile
    auto epilogue = [&](int ct) {
        if constexpr (kStage) {
            const int idx = 64 * ct + (threadIdx.x & 63);
            float4 v = *reinterpret_cast<const float4*>(stg_at(idx / NB4, idx % NB4));
            if constexpr (kBiasEpi) v = make_float4(v.x + breg[0].x, v.y + breg[0].y, v.z + breg[0].z, v.w + breg[0].w);
            const uint32_t off = staged_off(ct, srow0);
            if constexpr (EPI == WS_STORE) {
                bstore(v, yr, off, nt_out);
            } else if constexpr (EPI == WS_ACCUM) {
                const float4 o = pre[ct];
                bstore(make_float4(v.x + o.x, v.y + o.y, v.z + o.z, v.w + o.w), yr, off, nt_out);
            } else if constexpr (EPI == WS_GELU_DROP) {
                // A lane holds one 4-element chunk per feature tile; its partner lane ^ 4 holds the other chunk of
                // the same Philox block (chunk bit 2 == lane bit 2: N / 4 and n0 / 4 are multiples of 8).  So at
                // the even tile the bit-2-clear lane generates its tile-ct block, the bit-2-set lane the tile-ct+1
                // block, and one exchange gives both lanes both tiles' decisions: one Philox block per lane per
                // tile pair instead of one per tile (the second tile's half kept in `pend`).
                float u[4] = {1.f, 1.f, 1.f, 1.f};
                if (ep.p > 0.f) {
                    if ((ct & 1) == 0) {
                        const int sel = (threadIdx.x >> 2) & 1;
                        const int idx = 64 * (ct + sel) + (threadIdx.x & 63), row = idx / NB4, c4 = idx % NB4;
                        const uint64_t chunk = (uint64_t)(((srow0 + row) * N + n0 + 4 * c4) >> 2);
                        const uint32_t b8 = gelu_keep_bits8(ep.seed, chunk, thr);
                        const uint32_t x = (uint32_t)__shfl_xor((int)b8, 4, 64);
                        gelu_keep_factors(sel ? (x >> 4) : (b8 & 0xFu), keep_k, u);
                        pend = sel ? (b8 >> 4) : (x & 0xFu);
                    } else {
                        gelu_keep_factors(pend, keep_k, u);
                    }
                }
                float gl[4], gd[4];
                gelu_erf_and_grad(v.x, gl[0], gd[0]);
                gelu_erf_and_grad(v.y, gl[1], gd[1]);
                gelu_erf_and_grad(v.z, gl[2], gd[2]);
                gelu_erf_and_grad(v.w, gl[3], gd[3]);
                bstore(make_float4(u[0] * gd[0], u[1] * gd[1], u[2] * gd[2], u[3] * gd[3]), pr, off, nt_out);
                bstore(make_float4(gl[0] * u[0], gl[1] * u[1], gl[2] * u[2], gl[3] * u[3]), yr, off, nt_out);
            } else if constexpr (EPI == WS_RESID_LN) {
                // the asme_residual_ln_fwd sequence (norm.hip) on RowLayout<4, 32, 1>: lanes 0-31 hold row idx / 32 of
                // the tile, lanes 32-63 the next one, lane sub the features 4 sub .. 4 sub + 3
                using R = RowLayout<4, 32, 1>;
                const int sub = threadIdx.x & 31;
                const int64_t t = srow0 + idx / NB4;
                RowVals<R> a, h, f;
                a[0][0] = v.x, a[0][1] = v.y, a[0][2] = v.z, a[0][3] = v.w;
                h[0][0] = pre[ct].x, h[0][1] = pre[ct].y, h[0][2] = pre[ct].z, h[0][3] = pre[ct].w;
                if (ep.p > 0.f) {
                    row_keep<R>(ep.seed, 3u, (uint64_t)t * 128, sub, ep.p, f);
                    row_mul<R>(a, f);
                }
#pragma unroll
                for (int i = 0; i < 4; ++i) h[0][i] += a[0][i];
                if (ep.p2 > 0.f) {
                    row_keep<R>(ep.seed2, 4u, (uint64_t)t * 128, sub, ep.p2, f);
                    row_mul<R>(h, f);
                }
                bstore(make_float4(h[0][0], h[0][1], h[0][2], h[0][3]), yr, off, nt_out);
                if (ep.ln_w) {
                    float m, r;
                    row_ln_stats<R>(h, sub, 128, ep.eps, m, r);
                    row_normalise<R>(h, sub, 128, m, r, a);
                    bstore(make_float4(__builtin_fmaf(a[0][0], lnw.x, lnb.x), __builtin_fmaf(a[0][1], lnw.y, lnb.y),
                                       __builtin_fmaf(a[0][2], lnw.z, lnb.z), __builtin_fmaf(a[0][3], lnw.w, lnb.w)),
                           lr, off, nt_out);  // (row_affine's explicit fma)
                    if (sub == 0 && t < M) *reinterpret_cast<float2*>(ep.stats + 2 * t) = make_float2(m, r);
                }
            } else {
                const float4 f = pre[ct % NPRE];
                bstore(make_float4(v.x * f.x, v.y * f.y, v.z * f.z, v.w * f.w), yr, off, nt_out);
                if constexpr (kLateA)
                    if (ct + NPRE < CT) pre[ct % NPRE] = bload(pr, staged_off(ct + NPRE, srow0));
            }
            return;
        }
        const uint32_t off = soff + ct * 64;
        float4 v = stash[ct];
        if constexpr (EPI == WS_STORE) {
            bstore(v, yr, off, nt_out);
        } else if constexpr (EPI == WS_ACCUM) {
            const float4 o = pre[ct];
            bstore(make_float4(v.x + o.x, v.y + o.y, v.z + o.z, v.w + o.w), yr, off, nt_out);
        } else if constexpr (EPI == WS_GELU_DROP) {
            float u[4] = {1.f, 1.f, 1.f, 1.f};
            if (ep.p > 0.f) {
                // feature tiles ct and ct + 1 are the chunk pair (c, c | 4) of one Philox block: generated at the
                // even tile, the odd tile's half kept in `pend` (chunk = element index off / 4 over 4)
                if ((ct & 1) == 0) pend = gelu_keep_bits8(ep.seed, (uint64_t)(off >> 4), thr);
                gelu_keep_factors((ct & 1) ? (pend >> 4) : (pend & 0xFu), keep_k, u);
            }
            // the backward's whole activation factor keep * GELU'(pre), so its epilogue is one multiply
            float gl[4], gd[4];
            gelu_erf_and_grad(v.x, gl[0], gd[0]);
            gelu_erf_and_grad(v.y, gl[1], gd[1]);
            gelu_erf_and_grad(v.z, gl[2], gd[2]);
            gelu_erf_and_grad(v.w, gl[3], gd[3]);
            bstore(make_float4(u[0] * gd[0], u[1] * gd[1], u[2] * gd[2], u[3] * gd[3]), pr, off, nt_out);
            bstore(make_float4(gl[0] * u[0], gl[1] * u[1], gl[2] * u[2], gl[3] * u[3]), yr, off, nt_out);
        } else {
            const float4 f = pre[ct % NPRE];
            bstore(make_float4(v.x * f.x, v.y * f.y, v.z * f.z, v.w * f.w), yr, off, nt_out);
        }
    };
    floatx4 acc[CT];
    for (int64_t j = 0; j < my_tiles; ++j) {
#pragma unroll
        for (int ct = 0; ct < CT; ++ct) acc[ct] = floatx4{0.f, 0.f, 0.f, 0.f};
        // RD blocks per trip, unrolled; the trips themselves stay a loop (a fully unrolled K = 384 tile spills)
#pragma unroll 1
        for (int kq = 0; kq < NKB; kq += RD)
#pragma unroll
        for (int d = 0; d < RD; ++d) {
            const int kb = kq + d;
            const int kbn = kb + 1 == NKB ? 0 : kb + 1;
            // each feature tile's six MFMAs, then its next-block W read into the registers they consumed
#pragma unroll
            for (int ct = 0; ct < CT; ++ct) {
#if ASME_WS_DIAG != 1
                acc[ct] = mfma_bf3(wc[ct % WR], xs, acc[ct]);
#else
                acc[ct][0] += (float)xs.h[0] + (float)wc[ct % WR].h[0];
#endif
#if ASME_WS_DIAG != 3
                // the fragment WR tiles on: tile ct + WR of this block, or (past the last tile) of the next block
                wc[ct % WR] = ct + WR < CT ? wload(ct + WR, kb) : wload(ct + WR - CT, kbn);
#endif
                __builtin_amdgcn_sched_barrier(0);
            }
            // refill the slot just consumed: block kb + RD of this tile or of the next one (unconditional,
            // so the vmcnt bookkeeping stays exact; past the last tile it re-reads the last one)
            const float* src = kb + RD < NKB ? rc : rn;
#if ASME_WS_DIAG != 4
            xload(src, (kb + RD) % NKB, ring[2 * d], ring[2 * d + 1], ring3[XP ? d : 0]);
#else
            ring[2 * d].x += (float)(uintptr_t)src;
#endif
            // the next block's X terms
            const int dn = (kb + 1) % RD;
            xs = xsplit(ring[2 * dn], ring[2 * dn + 1], ring3[XP ? dn : 0]);
            // the previous tile's epilogue, spread over the blocks (late in the tile, so the pre-activation
            // loads WS_GELU_BWD issued at the tile boundary have landed)
#pragma unroll
            for (int ct = 0; ct < CT; ++ct)
                if (((ct + 1) * NKB + CT - 1) / CT - 1 == kb) epilogue(ct);  // every ct lands in [0, NKB)
            __builtin_amdgcn_sched_barrier(0);
        }
        // tile done: to the stash (written during the next tile)
        const int64_t m = (t0 + j * wcount) * 16 + c16;
        soff = m < M ? (uint32_t)((m * N + n0 + 4 * g) * 4) : kDrop;
        if constexpr (kStage) {
            srow0 = (t0 + j * wcount) * 16;
#pragma unroll
            for (int ct = 0; ct < CT; ++ct) {
                *reinterpret_cast<float4*>(stg_at(c16, ct * 4 + g)) =
                    kBiasEpi ? make_float4(acc[ct][0], acc[ct][1], acc[ct][2], acc[ct][3])
                             : make_float4(acc[ct][0] + breg[ct].x, acc[ct][1] + breg[ct].y, acc[ct][2] + breg[ct].z,
                                           acc[ct][3] + breg[ct].w);
                if constexpr (EPI == WS_GELU_BWD || EPI == WS_ACCUM || EPI == WS_RESID_LN)
                    if (ct < NPRE) pre[ct] = bload(pr, staged_off(ct, srow0));
            }
        } else {
#pragma unroll
            for (int ct = 0; ct < CT; ++ct) {
                stash[ct] = make_float4(acc[ct][0] + breg[kBiasEpi ? 0 : ct].x, acc[ct][1] + breg[kBiasEpi ? 0 : ct].y,
                                        acc[ct][2] + breg[kBiasEpi ? 0 : ct].z, acc[ct][3] + breg[kBiasEpi ? 0 : ct].w);
                if constexpr (EPI == WS_GELU_BWD || EPI == WS_ACCUM || EPI == WS_RESID_LN) pre[ct % NPRE] = bload(pr, soff + ct * 64);
            }
        }
        rc = rn;
        rn = xrow(j + 2);
    }
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) epilogue(ct);  // the last tile
}

template <int K, int CT, bool TRANS, int EPI, bool XP = false>
int launch_ws(const float* X, int64_t M, const float* W, int N, float* Y, const WsEpi& ep, hipStream_t s) {
    constexpr int NB = 16 * CT;
    const size_t planes = (size_t)NB * K * 6;  // three bf16 planes
    const size_t stage = (size_t)kWaves * 16 * (CT == 8 ? NB : NB + 4) * 4;  // (the kernel's SROW)
    const size_t lds = planes + (CT >= 4 && planes + stage <= (size_t)kLdsMax ? stage : 0);
    // opt in above 64 KiB of dynamic LDS once per instantiation (a function-local static: thread-safe initialisation)
    static const hipError_t attr = hipFuncSetAttribute((const void*)ws_gemm_kernel<K, CT, TRANS, EPI, XP>,
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (attr != hipSuccess) return hip_status(attr, "asme_ws_linear: LDS opt-in");
    int dev = 0, cus = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    // every feature block needs at least one workgroup of each XCD (the kernel's wg_per_nb = per_xcd / nblk): a
    // shape with more blocks than an XCD has workgroups would leave Y unwritten, so it is refused here
    if ((N + NB - 1) / NB > cus / 8) {
        set_error("asme_ws_linear: more feature blocks than workgroups per XCD for this epilogue");
        return -1;
    }
    hipLaunchKernelGGL((ws_gemm_kernel<K, CT, TRANS, EPI, XP>), dim3((cus / 8) * 8), dim3(kWaves * 64), lds, s, X, M,
                       W, N, Y, ep);
    return hip_status(hipGetLastError(), "asme_ws_linear");
}

// features per workgroup: 64; 96 when N / 64 does not divide the 32 workgroups of an XCD (N = 384, K = 128:
// wider tiles at larger K run out of registers); 32 when a 64-feature block of the three bf16 planes would
// not fit the LDS (K = 512); else 64 with the XCD's leftover workgroups idle
#ifndef ASME_WS_GBWD_CT8
#define ASME_WS_GBWD_CT8 1  // the GELU backward on 128-feature blocks, its factor read four tiles ahead (0: 64-feature
#endif                      // blocks, the whole tile's factor at the boundary; tools/ws_ab.py 211.3 -> 183.7 us)
#ifndef ASME_WS_CT8
#define ASME_WS_CT8 1
#endif
int pick_ct(int N, int K) {
    const bool fit4 = 64 * K * 6 <= kLdsMax;
    // K = 128 with whole 128-feature blocks that split an XCD's 32 workgroups: each X tile is split once per 128
    // features instead of once per 64 (the split's VALU does not overlap the MFMAs, §4)
    if (ASME_WS_CT8 && K == 128 && N % 128 == 0 && 32 % (N / 128) == 0) return 8;
    if (N % 64 == 0 && 32 % (N / 64) == 0 && fit4) return 4;
    if (K == 128 && N % 96 == 0 && 32 % (N / 96) == 0) return 6;
    if (N % 32 == 0 && 32 % (N / 32) == 0 && 32 * K * 6 <= kLdsMax) return 2;
    if (N % 64 == 0 && N / 64 <= 32 && fit4) return 4;
    return 0;
}

template <int K, bool TRANS, int EPI>
int dispatch_ct(int ct, const float* X, int64_t M, const float* W, int N, float* Y, const WsEpi& ep, hipStream_t s) {
    if constexpr (64 * K * 6 <= kLdsMax)
        if (ct == 4) return launch_ws<K, 4, TRANS, EPI>(X, M, W, N, Y, ep, s);
    if constexpr (K == 128)
        if (ct == 6) return launch_ws<K, 6, TRANS, EPI>(X, M, W, N, Y, ep, s);
    // (the activation-factor epilogue on 128-feature blocks reads its factor through a 4-slot ring, kLateA: CT = 8
    // factor registers at the tile boundary would spill)
    if constexpr (K == 128 && (EPI != WS_GELU_BWD || ASME_WS_GBWD_CT8))
        if (ct == 8) return launch_ws<K, 8, TRANS, EPI>(X, M, W, N, Y, ep, s);
    if constexpr (K == 128 && EPI == WS_GELU_BWD)
        if (ct == 8) return launch_ws<K, 4, TRANS, EPI>(X, M, W, N, Y, ep, s);
    return launch_ws<K, 2, TRANS, EPI>(X, M, W, N, Y, ep, s);
}

template <bool TRANS, int EPI>
int dispatch_k(int K, int ct, const float* X, int64_t M, const float* W, int N, float* Y, const WsEpi& ep,
               hipStream_t s) {
    switch (K) {
        case 128: return dispatch_ct<128, TRANS, EPI>(ct, X, M, W, N, Y, ep, s);
        case 256: return dispatch_ct<256, TRANS, EPI>(ct, X, M, W, N, Y, ep, s);
        case 384: return dispatch_ct<384, TRANS, EPI>(ct, X, M, W, N, Y, ep, s);
        default: return dispatch_ct<512, TRANS, EPI>(ct, X, M, W, N, Y, ep, s);
    }
}

}  // namespace

// 1 when (M, K, N) is a shape the weight-stationary kernel takes: K in {128, 256, 384, 512}, N a multiple of
// 32, 64 or 96 that splits the 32 workgroups of an XCD, the split W block within 160 KiB of LDS, Y < 2 GiB.
ASME_API int asme_ws_linear_supported(int64_t M, int64_t K, int64_t N) {
    if (M <= 0 || (K != 128 && K != 256 && K != 384 && K != 512)) return 0;
    if (N > 4096 || pick_ct((int)N, (int)K) == 0) return 0;
    // the activation-factor epilogue runs CT = 8 shapes on 64-feature blocks (dispatch_ct): those must fit an XCD's
    // 32 workgroups too, so the shape is supported for every epilogue (K = 128, N = 4096)
    // (with ASME_WS_GBWD_CT8 every epilogue runs CT = 8 shapes on 128-feature blocks: nothing to add)
    if (!ASME_WS_GBWD_CT8 && pick_ct((int)N, (int)K) == 8 && !(N % 64 == 0 && 32 % (N / 64) == 0)) return 0;
    if (M * N * 4 >= (int64_t)kDrop || M * K * 4 >= ((int64_t)1 << 40)) return 0;
    return 1;
}

// Y (M x N) = X (M x K) . W^T (+ bias) with epilogue `epi` (0 store, 1 GELU + dropout with the
// pre-activation in pre_out, 2 GELU backward with the pre-activation pre_in); trans = 1: W is K x N and
// Y = X . W (the input gradient of a Linear with weight W).  Rows of X, Y, pre: contiguous, 16-B aligned.
ASME_API int asme_ws_linear(const float* X, int64_t M, int64_t K, const float* W, int64_t N, int trans,
                            const float* bias, int epi, float* pre_out, const float* pre_in, float p, uint64_t seed,
                            float* Y, void* stream) {
    ASME_CHECK_ARG(X && W && Y, "asme_ws_linear: null pointer");
    ASME_CHECK_ARG(asme_ws_linear_supported(M, K, N), "asme_ws_linear: unsupported shape");
    ASME_CHECK_ARG(epi >= 0 && epi <= 2, "asme_ws_linear: bad epilogue");
    ASME_CHECK_ARG(epi != 1 || pre_out, "asme_ws_linear: GELU forward needs pre_out");
    ASME_CHECK_ARG(epi != 2 || pre_in, "asme_ws_linear: GELU backward needs pre_in");
    ASME_CHECK_ARG(((uintptr_t)X & 15) == 0 && ((uintptr_t)Y & 15) == 0 && ((uintptr_t)W & 15) == 0,
                   "asme_ws_linear: 16-B alignment");
    ASME_CHECK_ARG(p >= 0.f && p < 1.f, "asme_ws_linear: dropout probability in [0, 1)");
    const WsEpi ep{bias, pre_out, pre_in, p, seed, K, K, 0};
    const int ct = pick_ct((int)N, (int)K);
    hipStream_t s = (hipStream_t)stream;
    // K = 512 plain stores: two K = 256 halves with 64-feature blocks (the 512-deep split W block only fits 32
    // features, which splits and re-reads X four times); the second half accumulates into Y
    if (K == 512 && epi == 0 && pick_ct((int)N, 256) == 4) {
        const WsEpi e1{bias, nullptr, nullptr, 0.f, 0, 512, 512, 0};
        const WsEpi e2{nullptr, nullptr, nullptr, 0.f, 0, 512, 512, 256};
        const int rc = trans ? launch_ws<256, 4, true, WS_STORE>(X, M, W, (int)N, Y, e1, s)
                             : launch_ws<256, 4, false, WS_STORE>(X, M, W, (int)N, Y, e1, s);
        if (rc != 0) return rc;
        return trans ? launch_ws<256, 4, true, WS_ACCUM>(X, M, W, (int)N, Y, e2, s)
                     : launch_ws<256, 4, false, WS_ACCUM>(X, M, W, (int)N, Y, e2, s);
    }
    if (trans) {
        if (epi == 0) return dispatch_k<true, WS_STORE>((int)K, ct, X, M, W, (int)N, Y, ep, s);
        if (epi == 1) return dispatch_k<true, WS_GELU_DROP>((int)K, ct, X, M, W, (int)N, Y, ep, s);
        return dispatch_k<true, WS_GELU_BWD>((int)K, ct, X, M, W, (int)N, Y, ep, s);
    }
    if (epi == 0) return dispatch_k<false, WS_STORE>((int)K, ct, X, M, W, (int)N, Y, ep, s);
    if (epi == 1) return dispatch_k<false, WS_GELU_DROP>((int)K, ct, X, M, W, (int)N, Y, ep, s);
    return dispatch_k<false, WS_GELU_BWD>((int)K, ct, X, M, W, (int)N, Y, ep, s);
}

// 1 when asme_ws_linear_residual_ln takes the shape: K = N = 128 (one 128-feature block is a whole row) and the
// plain kernel's limits
ASME_API int asme_ws_linear_residual_ln_supported(int64_t M, int64_t K, int64_t N) {
    return K == 128 && N == 128 && asme_ws_linear_supported(M, K, N) && pick_ct(128, 128) == 8 ? 1 : 0;
}

// The attention output projection with the SublayerConnection residual and the next pre-LayerNorm in its epilogue:
//   s_out = drop_b(res + drop_a(X W^T + bias));  ln_out = LN(s_out; ln_w, ln_b, eps);  stats = (mean, rstd) per row
// bit-identical to asme_ws_linear (epi 0) followed by asme_residual_ln_fwd with the same seeds (same products, same
// dropout streams, same row-statistics sequence), without the Y round trip.  ln_w null: s_out only (ln_b, ln_out,
// stats unused).  X, res, s_out, ln_out: M x 128 contiguous rows, 16-B aligned; W: 128 x 128 (nn.Linear.weight).
ASME_API int asme_ws_linear_residual_ln(const float* X, int64_t M, int64_t K, const float* W, int64_t N,
                                        const float* bias, const float* res, float p_a, uint64_t seed_a, float p_b,
                                        uint64_t seed_b, const float* ln_w, const float* ln_b, float eps,
                                        float* s_out, float* ln_out, float* stats, void* stream) {
    ASME_CHECK_ARG(X && W && res && s_out, "asme_ws_linear_residual_ln: null pointer");
    ASME_CHECK_ARG(!ln_w || (ln_b && ln_out && stats), "asme_ws_linear_residual_ln: LayerNorm outputs missing");
    ASME_CHECK_ARG(asme_ws_linear_residual_ln_supported(M, K, N), "asme_ws_linear_residual_ln: unsupported shape");
    ASME_CHECK_ARG(p_a >= 0.f && p_a < 1.f && p_b >= 0.f && p_b < 1.f, "asme_ws_linear_residual_ln: bad dropout p");
    ASME_CHECK_ARG(((uintptr_t)X & 15) == 0 && ((uintptr_t)W & 15) == 0 && ((uintptr_t)res & 15) == 0 &&
                       ((uintptr_t)s_out & 15) == 0 && (!ln_w || (((uintptr_t)ln_out & 15) == 0 &&
                                                                   ((uintptr_t)ln_w & 15) == 0 &&
                                                                   ((uintptr_t)ln_b & 15) == 0 &&
                                                                   ((uintptr_t)stats & 7) == 0)),
                   "asme_ws_linear_residual_ln: alignment");
    WsEpi ep{bias, ln_w ? ln_out : nullptr, res, p_a, seed_a, 128, 128, 0};
    ep.p2 = p_b;
    ep.seed2 = seed_b;
    ep.ln_w = ln_w;
    ep.ln_b = ln_b;
    ep.eps = eps;
    ep.stats = stats;
    return launch_ws<128, 8, false, WS_RESID_LN>(X, M, W, 128, s_out, ep, (hipStream_t)stream);
}

// ---- experiment: X pre-split into its bf16 planes by its producer
namespace {
__global__ __launch_bounds__(256) void split_rows_kernel(const float* __restrict__ X, int64_t n8, int64_t plane,
                                                         __bf16* __restrict__ P) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // one thread per 8 elements
    if (t >= n8) return;
    const Bf3 b = split_bf3(*reinterpret_cast<const float4*>(X + 8 * t), *reinterpret_cast<const float4*>(X + 8 * t + 4));
    *reinterpret_cast<bf16x8*>(P + 8 * t) = b.h;
    *reinterpret_cast<bf16x8*>(P + plane + 8 * t) = b.m;
    *reinterpret_cast<bf16x8*>(P + 2 * plane + 8 * t) = b.l;
}
}  // namespace

// planes [3][M][K] bf16 = the exact split of X (M x K, contiguous); the standalone form of what a producer's epilogue
// would write
ASME_API int asme_ws_split_planes(const float* X, int64_t M, int64_t K, void* planes, void* stream) {
    ASME_CHECK_ARG(X && planes && K % 8 == 0, "asme_ws_split_planes: bad arguments");
    const int64_t n8 = M * K / 8;
    hipLaunchKernelGGL(split_rows_kernel, dim3((unsigned)((n8 + 255) / 256)), dim3(256), 0, (hipStream_t)stream, X, n8,
                       M * K, reinterpret_cast<__bf16*>(planes));
    ASME_LAUNCH_CHECK("asme_ws_split_planes");
}

// asme_ws_linear (trans = 0, K = 128, epilogue 0 or 1) reading X as its three bf16 planes ([3][M][128])
ASME_API int asme_ws_linear_planes(const void* Xp, int64_t M, int64_t K, const float* W, int64_t N, const float* bias,
                                   int epi, float* pre_out, float p, uint64_t seed, float* Y, void* stream) {
    ASME_CHECK_ARG(Xp && W && Y && K == 128 && (epi == 0 || epi == 1) && asme_ws_linear_supported(M, K, N),
                   "asme_ws_linear_planes: unsupported");
    const WsEpi ep{bias, pre_out, nullptr, p, seed, K, K, 0};
    const int ct = pick_ct((int)N, (int)K);
    hipStream_t s = (hipStream_t)stream;
    const float* X = reinterpret_cast<const float*>(Xp);
    if (epi == 1) {
        if (ct == 8) return launch_ws<128, 8, false, WS_GELU_DROP, true>(X, M, W, (int)N, Y, ep, s);
        if (ct == 6) return launch_ws<128, 6, false, WS_GELU_DROP, true>(X, M, W, (int)N, Y, ep, s);
        return launch_ws<128, 4, false, WS_GELU_DROP, true>(X, M, W, (int)N, Y, ep, s);
    }
    if (ct == 8) return launch_ws<128, 8, false, WS_STORE, true>(X, M, W, (int)N, Y, ep, s);
    if (ct == 6) return launch_ws<128, 6, false, WS_STORE, true>(X, M, W, (int)N, Y, ep, s);
    return launch_ws<128, 4, false, WS_STORE, true>(X, M, W, (int)N, Y, ep, s);
}
