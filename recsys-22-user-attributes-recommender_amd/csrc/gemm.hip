// Weight/bias gradient of the transformer's Linear layers on gfx950: dW = dY^T X, db = sum_t dY.
//
// Reference: every nn.Linear of the block (transformer_layers.py:175-199 projections, :212-220 FFN)
// gets dW = grad_out^T @ input from autograd.  Here T = B*L = 204,800 tokens and N, K <= 512, so the
// product is a small output with a huge reduction: library GEMMs run it at 14-38 TFLOP/s (measured,
// DESIGN.md §4).  This kernel splits the token dimension over many workgroups (split-T), each owning a
// 128x128 output tile for one token chunk and writing an fp32 partial slab; a fixed-order column reduction
// then sums the slabs (deterministic, no atomics).  The bias gradient is summed from the same dY registers.
//
// Products run on the bf16 matrix cores with split operands (bf16x6, common.h: error at or below fp32
// MFMA's): a 32-token block of dY and X is split in registers into three bf16 planes and stored transposed
// in LDS -- per column, the 32 tokens as four 16-B slots of 8 -- so the MFMA operand (8 consecutive tokens
// of one column, v_mfma_f32_16x16x32_bf16) is one ds_read_b128 per plane.  The slot layout (tslot) is
// conflict-free for both the ds_read_b128 lane groups and the ds_write_b128 8-lane groups.
//
// Layout: A = dY (T x N, row stride lda), B = X (T x K, row stride ldb), both row-major fp32.
// Workgroup = 8 waves (two per SIMD, one workgroup per CU) over a super-tile of one 128x128 tile or two paired
// ones (WgShape): 2x4 waves of 4x2 MFMA tiles, or 4x2 / 2x4 waves of 4x4.  The LDS holds two token blocks (double
// buffer, 96 or 144 KiB): while the waves multiply block n, they split and store block n+1 (loaded into registers
// two blocks earlier) into the other buffer and issue the loads of block n+3 -- one barrier per block.  Each loader
// unit is 8 tokens x 2 columns of one operand (rows of 512 contiguous bytes per wave); a thread holds one unit, or
// two in a paired super-tile's first four waves.
#include "common.h"

#include <cstdlib>
#include <type_traits>

using namespace asme;

namespace {

constexpr int kTile = 128;         // output tile (N and K)
constexpr int kTT = 32;            // token rows per LDS block
constexpr int kWgThreads = 512;

// 16-B slot of (column c, token slot s): column position c ^ ((c >> 1) & 1), slot ((c >> 2) ^ 3s) mod 4.
// ds_read_b128 (lanes {0-3,12-15,20-27}, ...: 16 consecutive columns, s = lane / 16) and ds_write_b128
// (8 contiguous lanes: columns 2i + jj, one s) both land on distinct 16-B bank slots.
__device__ __forceinline__ int tslot(int c, int s) {
    return (c ^ ((c >> 1) & 1)) * 4 + ((((c >> 2) & 3) ^ (3 * s)) & 3);
}

typedef unsigned u32v2 __attribute__((ext_vector_type(2)));
#ifndef ASME_WG_LOAD_AUX
#define ASME_WG_LOAD_AUX 2  // operand loads with the non-temporal policy (same-box A/B: the kernel 1.5 % faster)
#endif
constexpr uint32_t kDrop = 0x80000000u;  // >= every chunk's record count: the load returns 0

// rows 8 rg .. + 7 of a token block of this thread's column pair, by buffer loads against the chunk's record range:
// voff[q] = the thread's constant byte offset of row 8 rg + q (kDrop for a column pair past the operand), soff =
// the block's first row within the chunk (scalar).  Rows past the chunk read 0 with no branch, so every block issues
// the same loads and the compiler's vmcnt waits stay exact (a branchy tail made it wait for vmcnt(0): one block of
// loads in flight instead of two), and no per-load vector address arithmetic is left in the loop.
__device__ __forceinline__ void load_cols(__amdgpu_buffer_rsrc_t rs, const uint32_t (&voff)[8], uint32_t soff,
                                          float2 (&r)[8]) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const u32v2 v = __builtin_amdgcn_raw_buffer_load_b64(rs, voff[q], soff, ASME_WG_LOAD_AUX);
        r[q] = make_float2(__uint_as_float(v.x), __uint_as_float(v.y));
    }
}

// the thread's 2 columns x 8 tokens, split, into token slot rg of those columns of the three planes (pstride
// slots apart)
__device__ __forceinline__ void store_cols(uint4* __restrict__ planes, int pstride, int rg, int cg,
                                           const float2 (&r)[8]) {
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
        const float4 a = jj == 0 ? make_float4(r[0].x, r[1].x, r[2].x, r[3].x)
                                 : make_float4(r[0].y, r[1].y, r[2].y, r[3].y);
        const float4 b = jj == 0 ? make_float4(r[4].x, r[5].x, r[6].x, r[7].x)
                                 : make_float4(r[4].y, r[5].y, r[6].y, r[7].y);
        const Bf3 p = split_bf3(a, b);
        const int sl = tslot(2 * cg + jj, rg);
        planes[sl] = __builtin_bit_cast(uint4, p.h);
        planes[pstride + sl] = __builtin_bit_cast(uint4, p.m);
        planes[2 * pstride + sl] = __builtin_bit_cast(uint4, p.l);
    }
}

// A workgroup's output super-tile: TNX x TKX tiles of 128 x 128 (dY columns x X columns).  Pairing two tiles
// (256 x 128 or 128 x 256) shares one operand's loads and bf16 split between them: per token block the workgroup
// loads and splits 384 columns for two tiles' products instead of 256 for one (0.75x the load / split / LDS-write
// work per MFMA).  The buffer is then 72 KiB (144 KiB double-buffered).
template <int TNX, int TKX>
struct WgShape {
    static constexpr int NA = kTile * TNX, NB = kTile * TKX;  // dY / X columns
    static constexpr int PA = NA * 4, PB = NB * 4;            // 16-B slots of one bf16 plane
    static constexpr int BUF = 3 * (PA + PB);                 // one token block: dY planes h, m, l then X's
    static constexpr int UA = 2 * NA, U = 2 * (NA + NB);      // loader units (column pair x 8-token row group)
    static constexpr int WR = NA / 64, WC = 8 / WR;           // wave grid: 64 dY columns x NB / WC X columns
    static constexpr int MJ = NB / WC / 16;                   // MFMA tiles per wave along X (4 along dY)
    static constexpr int LDS = 2 * BUF * 16;
    static_assert(UA % 64 == 0 && UA <= kWgThreads && U <= 2 * kWgThreads, "loader units");
};

// one loader unit: a column pair of one operand over the 8-token row group rg of every block
struct WgUnit {
    __amdgpu_buffer_rsrc_t rs;
    uint32_t voff[8];
    uint32_t ld_bytes;
    int planes, pstride, rg, cg;
};

template <int TNX, int TKX>
__global__ __launch_bounds__(kWgThreads) __attribute__((amdgpu_waves_per_eu(2, 2))) void weight_grad_kernel(
    const float* __restrict__ A, int64_t lda, const float* __restrict__ B, int64_t ldb, int64_t T, int N, int K,
    int64_t chunk_rows, float* __restrict__ part, float* __restrict__ bias_part) {
    using S = WgShape<TNX, TKX>;
    extern __shared__ uint4 lds[];  // two token blocks of S::BUF slots
    // XCD-aware order: the output super-tiles of one token chunk are consecutive workgroups of ONE XCD (ids
    // xcd, xcd + 8, ...), resident together, so the dY / X rows they share come from that XCD's L2 once
    const int nsn = (N + S::NA - 1) / S::NA, ntiles = nsn * ((K + S::NB - 1) / S::NB);
    const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
    const int tile = slot % ntiles;
    const int64_t chunk = (int64_t)(slot / ntiles) * 8 + xcd;
    if (chunk * chunk_rows >= T) return;
    const int tn = tile % nsn, tk = tile / nsn;
    const int n0 = tn * S::NA, k0 = tk * S::NB;
    const int64_t t_begin = chunk * chunk_rows;
    const int64_t t_end = min(T, t_begin + chunk_rows);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c16 = lane & 15;
    const int wr = wave / S::WC, wc = wave % S::WC;
    // loader units: thread t takes unit t and, when the super-tile has more than 512, unit t + 512.  Units
    // [0, UA) are dY, the rest X; the operand is wave-uniform (UA is a multiple of 64 and the unit index is read
    // from the first lane), so each unit's buffer resource lives in scalar registers
    const int wave_u = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) * 64;
    auto make_unit = [&](int first, int u) {
        const bool a = first < S::UA;
        const int v = a ? u : u - S::UA, pairs = a ? S::NA / 2 : S::NB / 2;
        WgUnit un;
        un.cg = v % pairs;
        un.rg = v / pairs;
        const int64_t ld = a ? lda : ldb;
        un.rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>((a ? A : B) + t_begin * ld), 0,
                                                  (int)((t_end - t_begin) * ld * 4), 0x00020000);
        un.ld_bytes = (uint32_t)(ld * 4);
        un.planes = a ? 0 : 3 * S::PA;
        un.pstride = a ? S::PA : S::PB;
        const int col = (a ? n0 : k0) + 2 * un.cg;
        const bool col_ok = col < (a ? N : K);
#pragma unroll
        for (int q = 0; q < 8; ++q)
            un.voff[q] = col_ok ? (uint32_t)(8 * un.rg + q) * un.ld_bytes + (uint32_t)(col * 4) : kDrop;
        return un;
    };
    const WgUnit u0 = make_unit(wave_u, (int)threadIdx.x);
    const bool do_bias = bias_part != nullptr && tk == 0 && wave_u < S::UA;  // (units past 512 are never dY)
    float2 bsum = make_float2(0.f, 0.f);  // dY columns n0 + 2 cg, + 1 over this thread's rows

    floatx4 acc[4][S::MJ];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < S::MJ; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

    // (loads past the chunk are issued too and read zeros: unconditional, see load_cols)
    auto load = [&](const WgUnit& un, int64_t t0, float2 (&r)[8]) {
        load_cols(un.rs, un.voff, __builtin_amdgcn_readfirstlane((uint32_t)(t0 - t_begin) * un.ld_bytes), r);
    };
    auto compute = [&](int buf) {
        const uint4* L = lds + buf * S::BUF;
        Bf3 b[S::MJ];
#pragma unroll
        for (int j = 0; j < S::MJ; ++j) {
            const int sl = tslot(wc * (S::NB / S::WC) + j * 16 + c16, g);
            b[j].h = __builtin_bit_cast(bf16x8, L[3 * S::PA + sl]);
            b[j].m = __builtin_bit_cast(bf16x8, L[3 * S::PA + S::PB + sl]);
            b[j].l = __builtin_bit_cast(bf16x8, L[3 * S::PA + 2 * S::PB + sl]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int sl = tslot(wr * 64 + i * 16 + c16, g);
            Bf3 a;
            a.h = __builtin_bit_cast(bf16x8, L[sl]);
            a.m = __builtin_bit_cast(bf16x8, L[S::PA + sl]);
            a.l = __builtin_bit_cast(bf16x8, L[2 * S::PA + sl]);
#pragma unroll
            for (int j = 0; j < S::MJ; ++j) acc[i][j] = mfma_bf3(a, b[j], acc[i][j]);
        }
    };
    const int64_t nblk = (t_end - t_begin + kTT - 1) / kTT;
    // The block loop, compiled once per loader role (one unit or two): the role is wave-uniform and chosen outside
    // the loop, so the loop body has no branch -- any control flow around the loads made the compiler copy the
    // in-flight registers and wait for every load (vmcnt(0)).
    auto run = [&](auto two) {
        constexpr bool kTwo = decltype(two)::value;
        const WgUnit u1 = kTwo ? make_unit(wave_u + kWgThreads, (int)threadIdx.x + kWgThreads) : u0;
        // the block at t0 (in r) into LDS buffer buf; r then takes the block two ahead.  A block past the chunk
        // holds zeros (its loads read nothing) and lands in the buffer nobody multiplies any more.
        auto stage = [&](int64_t t0, float2 (&r)[8], float2 (&q)[8], int buf) {
            store_cols(lds + buf * S::BUF + u0.planes, u0.pstride, u0.rg, u0.cg, r);
            if constexpr (kTwo) store_cols(lds + buf * S::BUF + u1.planes, u1.pstride, u1.rg, u1.cg, q);
            if (do_bias) {
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    bsum.x += r[j].x;
                    bsum.y += r[j].y;
                }
            }
            load(u0, t0 + 2 * kTT, r);
            if constexpr (kTwo) load(u1, t0 + 2 * kTT, q);
        };
        float2 r0[8], r1[8], q0r[8], q1r[8];  // two blocks in flight per unit (q: the second unit, if any)
        load(u0, t_begin, r0);
        if constexpr (kTwo) load(u1, t_begin, q0r);
        load(u0, t_begin + kTT, r1);
        if constexpr (kTwo) load(u1, t_begin + kTT, q1r);
        stage(t_begin, r0, q0r, 0);
        __syncthreads();
        // pairs of blocks with no exit in between (buf 0 holds block i, r1 block i + 1, r0 block i + 2 at the top
        // of a trip); an odd last block is multiplied after the loop
        int64_t i = 0;
        for (; i + 2 <= nblk; i += 2) {
            const int64_t t0 = t_begin + i * kTT;
            stage(t0 + kTT, r1, q1r, 1);
            compute(0);
            __syncthreads();
            stage(t0 + 2 * kTT, r0, q0r, 0);
            compute(1);
            __syncthreads();
        }
        if (i < nblk) compute(0);
    };
    if constexpr (S::U > kWgThreads) {
        if (wave_u + kWgThreads < S::U) run(std::true_type{});
        else run(std::false_type{});
    } else {
        run(std::false_type{});
    }
    // partial slab: part[chunk][n][k]; lane holds rows n = ... + 4g + q, column k = ... + c16
    // chunk slab: [N x K dW partial | N db partial (when db is requested)]
    const int64_t slab = (int64_t)N * K + (bias_part != nullptr ? N : 0);
    float* P = part + chunk * slab;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < S::MJ; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int n = n0 + wr * 64 + i * 16 + 4 * g + q;
                const int k = k0 + wc * (S::NB / S::WC) + j * 16 + c16;
                if (n < N && k < K) P[(int64_t)n * K + k] = acc[i][j][q];
            }
    if (bias_part != nullptr && tk == 0) {  // the 4 row groups' column sums, in row-group order
        constexpr int kPairs = S::NA / 2;
        float2* red = reinterpret_cast<float2*>(lds);  // (the loop's last barrier retired every LDS read)
        if (wave_u < S::UA) red[u0.rg * kPairs + u0.cg] = bsum;
        __syncthreads();
        if (threadIdx.x < kPairs && n0 + 2 * (int)threadIdx.x < N) {
            float2 s = red[threadIdx.x];
#pragma unroll
            for (int q = 1; q < 4; ++q) {
                const float2 v = red[q * kPairs + threadIdx.x];
                s.x += v.x;
                s.y += v.y;
            }
            *reinterpret_cast<float2*>(P + (int64_t)N * K + n0 + 2 * threadIdx.x) = s;
        }
    }
}

// column sums with a fixed order (see reduce_rows_kernel in embedding.hip)
constexpr int kRedCols = 64, kRedGroups = 16;
// Column c of the slabs (row stride width_w + width_b) goes to out_w[c] (c < width_w) or out_b[c - width_w]:
// the dW and db partials of one weight gradient reduced by one launch.
__global__ __launch_bounds__(1024) void sum_slabs_kernel(const float* __restrict__ part, int64_t nrows,
                                                         int64_t width_w, float* __restrict__ out_w, int64_t width_b,
                                                         float* __restrict__ out_b, int accumulate) {
    const int64_t width = width_w + width_b;
    __shared__ float red[kRedGroups][kRedCols];
    const int col = threadIdx.x % kRedCols, grp = threadIdx.x / kRedCols;
    const int64_t c = (int64_t)blockIdx.x * kRedCols + col;
    // four independent chains per thread (rows grp + 16 (4i + j), chain j), added in a fixed order: 4x the
    // loads in flight of a single chain (a few column blocks of a narrow matrix are otherwise latency-bound)
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    if (c < width) {
        int64_t r = grp;
        for (; r + 3 * kRedGroups < nrows; r += 4 * kRedGroups) {
            s0 += part[r * width + c];
            s1 += part[(r + kRedGroups) * width + c];
            s2 += part[(r + 2 * kRedGroups) * width + c];
            s3 += part[(r + 3 * kRedGroups) * width + c];
        }
        for (; r < nrows; r += kRedGroups) s0 += part[r * width + c];
    }
    red[grp][col] = (s0 + s1) + (s2 + s3);
    __syncthreads();
    for (int h = kRedGroups / 2; h > 0; h >>= 1) {
        if (grp < h) red[grp][col] += red[grp + h][col];
        __syncthreads();
    }
    if (grp == 0 && c < width) {
        float* o = c < width_w ? out_w + c : out_b + (c - width_w);
        *o = accumulate ? *o + red[0][col] : red[0][col];
    }
}

// Few slabs (the split-T chunks of one weight gradient: 8-64): one thread per column, its rows in flight 8 at a time
// and added in row order -- no LDS tree, no barrier (the 64-column form above spends its time in the tree and the
// round trips of 2-4 loads per thread at these row counts)
__global__ __launch_bounds__(256) void sum_slabs_cols_kernel(const float* __restrict__ part, int64_t nrows,
                                                             int64_t width_w, float* __restrict__ out_w,
                                                             int64_t width_b, float* __restrict__ out_b,
                                                             int accumulate) {
    const int64_t width = width_w + width_b;
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= width) return;
    float s = 0.f;
    int64_t r = 0;
    for (; r + 8 <= nrows; r += 8) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = part[(r + u) * width + c];
#pragma unroll
        for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; r < nrows; ++r) s += part[r * width + c];
    float* o = c < width_w ? out_w + c : out_b + (c - width_w);
    *o = accumulate ? *o + s : s;
}

struct Plan {
    int64_t nchunks, chunk_rows;
};

// super-tile shape for an N x K gradient: pair two 128-column tiles along whichever side has an even count of them
// (the FFN's 512 x 128 and 128 x 512), else one tile per workgroup.  (Unpaired A/B builds: -DASME_WG_PAIR=0.)
#ifndef ASME_WG_PAIR
#define ASME_WG_PAIR 1
#endif
struct Pairing {
    int tnx, tkx;
};

Pairing pick_pairing(int64_t N, int64_t K) {
    const int64_t ntn = (N + kTile - 1) / kTile, ntk = (K + kTile - 1) / kTile;
    if (ASME_WG_PAIR && ntn % 2 == 0) return {2, 1};
    if (ASME_WG_PAIR && ntk % 2 == 0) return {1, 2};
    return {1, 1};
}

int64_t super_tiles(int64_t N, int64_t K) {
    const Pairing pr = pick_pairing(N, K);
    return ((N + kTile * pr.tnx - 1) / (kTile * pr.tnx)) * ((K + kTile * pr.tkx - 1) / (kTile * pr.tkx));
}

Plan make_plan(int64_t T, int64_t N, int64_t K) {
    if (T <= 0 || N <= 0 || K <= 0) return {0, kTT};  // (no chunk; the entry points reject the shape)
    const int64_t tiles = super_tiles(N, K);
    // one workgroup per CU (96 or 144 KiB of LDS each): chunks a multiple of 8 (one per XCD lane), tiles x chunks
    // <= 256
    const int64_t want = std::max<int64_t>(8, (256 / tiles) / 8 * 8);
    int64_t rows = (T + want - 1) / want;
    rows = std::max<int64_t>(kTT, ((rows + kTT - 1) / kTT) * kTT);
    // a chunk's rows (plus the two blocks read past it) must stay within a buffer resource's 2 GiB offsets
    const int64_t max_rows = (((int64_t)1 << 31) / (4 * std::max<int64_t>(std::max<int64_t>(N, K), 1)) - 2 * kTT) /
                             kTT * kTT;
    rows = std::min<int64_t>(rows, std::max<int64_t>(kTT, max_rows));
    return {(T + rows - 1) / rows, rows};  // chunks holding tokens; the grid rounds them up to a multiple of 8
}

template <int TNX, int TKX>
hipError_t launch_weight_grad(dim3 grid, hipStream_t s, const float* dy, int64_t ld_dy, const float* x,
                              int64_t ld_x, int64_t T, int N, int K, int64_t chunk_rows, float* part, float* bpart) {
    // 96 / 144 KiB of dynamic LDS: opt in once per shape (a function-local static: thread-safe initialisation)
    static const hipError_t attr = hipFuncSetAttribute((const void*)weight_grad_kernel<TNX, TKX>,
                                                       hipFuncAttributeMaxDynamicSharedMemorySize,
                                                       WgShape<TNX, TKX>::LDS);
    if (attr != hipSuccess) return attr;
    constexpr int kLds = WgShape<TNX, TKX>::LDS;
    weight_grad_kernel<TNX, TKX><<<grid, dim3(kWgThreads), kLds, s>>>(dy, ld_dy, x, ld_x, T, N, K, chunk_rows, part,
                                                                      bpart);
    return hipSuccess;
}

}  // namespace

ASME_API int64_t asme_linear_weight_grad_workspace(int64_t n_tokens, int64_t out_features, int64_t in_features) {
    if (n_tokens < 0 || out_features <= 0 || in_features <= 0 || out_features > (1 << 20) || in_features > (1 << 20))
        return 0;
    const Plan p = make_plan(n_tokens, out_features, in_features);
    return p.nchunks * (out_features * in_features + out_features) * (int64_t)sizeof(float);
}

// dW (out_features x in_features) (+)= dY^T X ; db (out_features) (+)= sum_t dY  (db nullable)
ASME_API int asme_linear_weight_grad(const float* dy, int64_t ld_dy, const float* x, int64_t ld_x, int64_t n_tokens,
                                     int64_t out_features, int64_t in_features, float* workspace,
                                     int64_t workspace_bytes, float* dw, float* db, int accumulate, void* stream) {
    ASME_CHECK_ARG(dy && x && workspace && dw, "asme_linear_weight_grad: null pointer");
    ASME_CHECK_ARG(n_tokens >= 0 && out_features > 0 && in_features > 0 && out_features <= (1 << 20) &&
                       in_features <= (1 << 20) && ld_dy >= out_features && ld_x >= in_features,
                   "asme_linear_weight_grad: bad sizes");
    ASME_CHECK_ARG(out_features % 4 == 0 && in_features % 4 == 0 && ld_dy % 4 == 0 && ld_x % 4 == 0 &&
                       ((uintptr_t)dy & 15) == 0 && ((uintptr_t)x & 15) == 0,
                   "asme_linear_weight_grad: features / strides must be multiples of 4 floats, 16-B aligned");
    ASME_CHECK_ARG(workspace_bytes >= asme_linear_weight_grad_workspace(n_tokens, out_features, in_features),
                   "asme_linear_weight_grad: workspace too small");
    if (n_tokens == 0) return 0;
    const Plan p = make_plan(n_tokens, out_features, in_features);
    ASME_CHECK_ARG((p.chunk_rows + 2 * kTT) * std::max(ld_dy, ld_x) * 4 < ((int64_t)1 << 31),
                   "asme_linear_weight_grad: row stride too large for the chunk's buffer range");
    hipStream_t s = (hipStream_t)stream;
    float* part = workspace;
    float* bpart = db ? workspace : nullptr;  // (a flag: the bias partials sit in each chunk's slab)
    const dim3 grid((unsigned)(super_tiles(out_features, in_features) * ((p.nchunks + 7) / 8) * 8));
    const Pairing pr = pick_pairing(out_features, in_features);
    const int N = (int)out_features, K = (int)in_features;
    const hipError_t e =
        pr.tnx == 2 ? launch_weight_grad<2, 1>(grid, s, dy, ld_dy, x, ld_x, n_tokens, N, K, p.chunk_rows, part, bpart)
        : pr.tkx == 2
            ? launch_weight_grad<1, 2>(grid, s, dy, ld_dy, x, ld_x, n_tokens, N, K, p.chunk_rows, part, bpart)
            : launch_weight_grad<1, 1>(grid, s, dy, ld_dy, x, ld_x, n_tokens, N, K, p.chunk_rows, part, bpart);
    if (e != hipSuccess) return hip_status(e, "asme_linear_weight_grad: LDS opt-in");
    const int64_t width_w = out_features * in_features, width_b = db ? out_features : 0;
    if (p.nchunks <= 64)
        hipLaunchKernelGGL(sum_slabs_cols_kernel, dim3((unsigned)((width_w + width_b + 255) / 256)), dim3(256), 0, s,
                           part, p.nchunks, width_w, dw, width_b, db, accumulate);
    else
        hipLaunchKernelGGL(sum_slabs_kernel, dim3((unsigned)((width_w + width_b + kRedCols - 1) / kRedCols)),
                           dim3(1024), 0, s, part, p.nchunks, width_w, dw, width_b, db, accumulate);
    ASME_LAUNCH_CHECK("asme_linear_weight_grad");
}
