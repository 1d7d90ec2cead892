// Weight/bias gradient of the transformer's Linear layers on gfx950: dW = dY^T X, db = sum_t dY.
//
// Reference: every nn.Linear of the block (transformer_layers.py:175-199 projections, :212-220 FFN)
// gets dW = grad_out^T @ input from autograd.  Here T = B*L = 204,800 tokens and N, K <= 512, so the
// product is a small output with a huge reduction: library GEMMs run it at 14-38 TFLOP/s (measured,
// DESIGN.md §4).  This kernel splits the token dimension over many workgroups (split-T), each owning a
// 128x128 output tile for one token chunk, accumulating with fp32 MFMA (v_mfma_f32_16x16x4f32, exact
// f32 FMA chain) and writing an fp32 partial slab; a fixed-order column reduction then sums the slabs
// (deterministic, no atomics).  The bias gradient is summed from the same LDS-staged dY tiles.
//
// Layout: A = dY (T x N, row stride lda), B = X (T x K, row stride ldb), both row-major fp32.
// Workgroup = 4 waves in a 2x2 grid over the 128x128 tile; each wave owns 64x64 = 4x4 MFMA tiles
// (16 accumulators).  Token rows stream through LDS 32 at a time (register-prefetched one block ahead);
// the LDS row stride of 144 floats puts the two 16-lane halves of a b32 read on disjoint banks.
#include "common.h"

using namespace asme;

namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int kTile = 128;   // output tile (N and K)
constexpr int kTT = 32;      // token rows per LDS block
constexpr int kLds = 144;    // LDS row stride (floats)

__device__ __forceinline__ floatx4 mfma16(float a, float b, floatx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// thread i of 256 loads 4 float4 of a kTT x 128 block: row = (i / 32) + 8*q, col4 = i % 32
__device__ __forceinline__ void load_block(const float* __restrict__ base, int64_t ld, int64_t t0, int64_t T,
                                           int col0, int ncols, float4 (&r)[4]) {
    const int c4 = (threadIdx.x & 31) * 4;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int64_t t = t0 + (threadIdx.x >> 5) + 8 * q;
        if (t < T && col0 + c4 < ncols)
            r[q] = *reinterpret_cast<const float4*>(base + t * ld + col0 + c4);
        else
            r[q] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
}

__device__ __forceinline__ void store_block(float* __restrict__ s, const float4 (&r)[4]) {
    const int c4 = (threadIdx.x & 31) * 4;
#pragma unroll
    for (int q = 0; q < 4; ++q) *reinterpret_cast<float4*>(s + ((threadIdx.x >> 5) + 8 * q) * kLds + c4) = r[q];
}

__global__ __launch_bounds__(256) void weight_grad_kernel(const float* __restrict__ A, int64_t lda,
                                                          const float* __restrict__ B, int64_t ldb, int64_t T,
                                                          int N, int K, int64_t chunk_rows,
                                                          float* __restrict__ part, float* __restrict__ bias_part) {
    __shared__ __attribute__((aligned(16))) float As[kTT * kLds];
    __shared__ __attribute__((aligned(16))) float Bs[kTT * kLds];
    const int n0 = blockIdx.x * kTile, k0 = blockIdx.y * kTile;
    const int64_t chunk = blockIdx.z;
    const int64_t t_begin = chunk * chunk_rows;
    const int64_t t_end = min(T, t_begin + chunk_rows);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c16 = lane & 15;
    const int wr = wave >> 1, wc = wave & 1;
    const bool do_bias = bias_part != nullptr && blockIdx.y == 0;

    floatx4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    float bsum = 0.f;  // threads 0..127: column n0 + tid of the bias gradient

    float4 ra[4], rb[4];
    load_block(A, lda, t_begin, t_end, n0, N, ra);
    load_block(B, ldb, t_begin, t_end, k0, K, rb);
    for (int64_t t0 = t_begin; t0 < t_end; t0 += kTT) {
        __syncthreads();
        store_block(As, ra);
        store_block(Bs, rb);
        __syncthreads();
        if (t0 + kTT < t_end) {  // prefetch the next block while this one is consumed
            load_block(A, lda, t0 + kTT, t_end, n0, N, ra);
            load_block(B, ldb, t0 + kTT, t_end, k0, K, rb);
        }
        if (do_bias && threadIdx.x < kTile) {
#pragma unroll 8
            for (int r = 0; r < kTT; ++r) bsum += As[r * kLds + threadIdx.x];
        }
#pragma unroll
        for (int kk = 0; kk < kTT / 4; ++kk) {
            const int trow = (kk * 4 + g) * kLds;
            float a[4], b[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) a[i] = As[trow + wr * 64 + i * 16 + c16];
#pragma unroll
            for (int j = 0; j < 4; ++j) b[j] = Bs[trow + wc * 64 + j * 16 + c16];
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(a[i], b[j], acc[i][j]);
        }
    }
    // partial slab: part[chunk][n][k]; lane holds rows n = ... + 4g + r, column k = ... + c16
    float* P = part + chunk * (int64_t)N * K;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int n = n0 + wr * 64 + i * 16 + 4 * g + r;
                const int k = k0 + wc * 64 + j * 16 + c16;
                if (n < N && k < K) P[(int64_t)n * K + k] = acc[i][j][r];
            }
    if (do_bias && threadIdx.x < kTile && n0 + (int)threadIdx.x < N)
        bias_part[chunk * (int64_t)N + n0 + threadIdx.x] = bsum;
}

// column sums with a fixed order (see reduce_rows_kernel in embedding.hip)
constexpr int kRedCols = 64, kRedGroups = 16;
__global__ __launch_bounds__(1024) void sum_slabs_kernel(const float* __restrict__ part, int64_t nrows, int64_t width,
                                                         float* __restrict__ out, int accumulate) {
    __shared__ float red[kRedGroups][kRedCols];
    const int col = threadIdx.x % kRedCols, grp = threadIdx.x / kRedCols;
    const int64_t c = (int64_t)blockIdx.x * kRedCols + col;
    float s = 0.f;
    if (c < width)
        for (int64_t r = grp; r < nrows; r += kRedGroups) s += part[r * width + c];
    red[grp][col] = s;
    __syncthreads();
    for (int h = kRedGroups / 2; h > 0; h >>= 1) {
        if (grp < h) red[grp][col] += red[grp + h][col];
        __syncthreads();
    }
    if (grp == 0 && c < width) out[c] = accumulate ? out[c] + red[0][col] : red[0][col];
}

struct Plan {
    int64_t nchunks, chunk_rows;
};

Plan make_plan(int64_t T, int64_t N, int64_t K) {
    const int64_t tiles = ((N + kTile - 1) / kTile) * ((K + kTile - 1) / kTile);
    int64_t want = std::max<int64_t>(1, 512 / tiles);  // ~2 workgroups per CU
    int64_t rows = (T + want - 1) / want;
    rows = std::max<int64_t>(kTT, ((rows + kTT - 1) / kTT) * kTT);
    return {(T + rows - 1) / rows, rows};
}

}  // namespace

ASME_API int64_t asme_linear_weight_grad_workspace(int64_t n_tokens, int64_t out_features, int64_t in_features) {
    const Plan p = make_plan(n_tokens, out_features, in_features);
    return p.nchunks * (out_features * in_features + out_features) * (int64_t)sizeof(float);
}

// dW (out_features x in_features) (+)= dY^T X ; db (out_features) (+)= sum_t dY  (db nullable)
ASME_API int asme_linear_weight_grad(const float* dy, int64_t ld_dy, const float* x, int64_t ld_x, int64_t n_tokens,
                                     int64_t out_features, int64_t in_features, float* workspace,
                                     int64_t workspace_bytes, float* dw, float* db, int accumulate, void* stream) {
    ASME_CHECK_ARG(dy && x && workspace && dw, "asme_linear_weight_grad: null pointer");
    ASME_CHECK_ARG(out_features % 4 == 0 && in_features % 4 == 0 && ld_dy % 4 == 0 && ld_x % 4 == 0 &&
                       ((uintptr_t)dy & 15) == 0 && ((uintptr_t)x & 15) == 0,
                   "asme_linear_weight_grad: features / strides must be multiples of 4 floats, 16-B aligned");
    ASME_CHECK_ARG(workspace_bytes >= asme_linear_weight_grad_workspace(n_tokens, out_features, in_features),
                   "asme_linear_weight_grad: workspace too small");
    if (n_tokens == 0) return 0;
    const Plan p = make_plan(n_tokens, out_features, in_features);
    hipStream_t s = (hipStream_t)stream;
    float* part = workspace;
    float* bpart = db ? workspace + p.nchunks * out_features * in_features : nullptr;
    const dim3 grid((unsigned)((out_features + kTile - 1) / kTile), (unsigned)((in_features + kTile - 1) / kTile),
                    (unsigned)p.nchunks);
    hipLaunchKernelGGL(weight_grad_kernel, grid, dim3(256), 0, s, dy, ld_dy, x, ld_x, n_tokens, (int)out_features,
                       (int)in_features, p.chunk_rows, part, bpart);
    const int64_t width = out_features * in_features;
    hipLaunchKernelGGL(sum_slabs_kernel, dim3((unsigned)((width + kRedCols - 1) / kRedCols)), dim3(1024), 0, s, part,
                       p.nchunks, width, dw, accumulate);
    if (db)
        hipLaunchKernelGGL(sum_slabs_kernel, dim3((unsigned)((out_features + kRedCols - 1) / kRedCols)), dim3(1024),
                           0, s, bpart, p.nchunks, out_features, db, accumulate);
    ASME_LAUNCH_CHECK("asme_linear_weight_grad");
}
