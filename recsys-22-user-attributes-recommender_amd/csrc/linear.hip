// General fp32-MFMA Linear GEMM on gfx950 for the shapes the weight-stationary bf16x6 kernel (wsgemm.hip) does not
// take (hidden sizes other than 128..512, e.g. the reference's d = 32 / 64 configurations, and the FFN modifier /
// post-fusion Linear at those widths).
//
// Reference semantics (paths relative to /root/reference/src/asme):
//   nn.Linear                     core/models/common/layers/transformer_layers.py:175-199, :212-220
//   FFN modifier Linear           core/models/common/components/representation_modifier/ffn_modifier.py:24-26
// Forward  Y = X W^T + b (X: M x K row-major, W: N x K row-major = nn.Linear.weight)
// Backward dX (+)= dY W  (dY: M x N, W: N x K row-major; the output width is the layer's in_features)
//
// Kernel shape: C^T tiles are computed (MFMA rows = output features, columns = tokens) so each lane ends with 4
// consecutive output features of one token (float4 stores).  Workgroup = 4 waves = 128 tokens x 128 features;
// wave w owns tokens 32w..32w+31 (2 x 8 MFMA 16x16 tiles).  The reduction dimension streams through LDS in
// 32-wide slabs (register-prefetched one slab ahead); within a slab lane group g supplies k = 8g .. 8g+7
// (ds_read_b128 operand reads).  Persistent XCD-aware tile schedule: the feature blocks of one token block run
// on the same XCD (shared L2).
#include "common.h"
#include "rows.h"
#include <algorithm>

using namespace asme;

namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int kBM = 128;  // tokens per workgroup
constexpr int kBN = 128;  // output features per workgroup
constexpr int kBK = 32;   // reduction slab (double-buffered in LDS)
constexpr int kLd = 36;   // LDS row stride (floats)
constexpr int kThreads = 256;


__device__ __forceinline__ floatx4 mfma16(float a, float b, floatx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Row slab: 128 rows x 32 floats of a row-major matrix; thread t holds float4 (row (t>>3) + 32q, col (t&7)*4)
__device__ __forceinline__ void load_rows_slab(const float* __restrict__ base, int64_t ld, int64_t row0,
                                               int64_t nrows, int k0, int K, float4 (&r)[4]) {
    const int c4 = (threadIdx.x & 7) * 4;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int64_t row = row0 + (threadIdx.x >> 3) + 32 * q;
        r[q] = (row < nrows && k0 + c4 < K) ? *reinterpret_cast<const float4*>(base + row * ld + k0 + c4)
                                             : make_float4(0.f, 0.f, 0.f, 0.f);
    }
}
__device__ __forceinline__ void store_rows_slab(float* __restrict__ s, const float4 (&r)[4]) {
    const int c4 = (threadIdx.x & 7) * 4;
#pragma unroll
    for (int q = 0; q < 4; ++q) *reinterpret_cast<float4*>(s + ((threadIdx.x >> 3) + 32 * q) * kLd + c4) = r[q];
}
// Column slab for the backward: W is (K x N) row-major and the slab needs [n][k], k in [k0, k0+32):
// thread t gathers 4 consecutive k of column n = t & 127 (lanes read consecutive n: coalesced).
__device__ __forceinline__ void load_cols_slab(const float* __restrict__ w, int64_t ldw, int k0, int K, int n0,
                                               int N, float4 (&r)[4]) {
    const int n = n0 + (threadIdx.x & 127);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int k = k0 + 4 * ((threadIdx.x >> 7) + 2 * q);
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = (n < N && k + i < K) ? w[(int64_t)(k + i) * ldw + n] : 0.f;
        r[q] = make_float4(v[0], v[1], v[2], v[3]);
    }
}
__device__ __forceinline__ void store_cols_slab(float* __restrict__ s, const float4 (&r)[4]) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
        *reinterpret_cast<float4*>(s + (threadIdx.x & 127) * kLd + 4 * ((threadIdx.x >> 7) + 2 * q)) = r[q];
}

template <bool TRANS_W>
__device__ __forceinline__ void load_slab(const float* __restrict__ X, int64_t ldx, int64_t M, int K,
                                          const float* __restrict__ W, int64_t ldw, int N, int64_t m0, int n0, int k0,
                                          float4 (&rx)[4], float4 (&rw)[4]) {
    load_rows_slab(X, ldx, m0, M, k0, K, rx);
    if (TRANS_W)
        load_cols_slab(W, ldw, k0, K, n0, N, rw);
    else
        load_rows_slab(W, ldw, n0, N, k0, K, rw);
}
template <bool TRANS_W>
__device__ __forceinline__ void store_slab(float* __restrict__ buf, const float4 (&rx)[4], const float4 (&rw)[4]) {
    store_rows_slab(buf, rx);
    if (TRANS_W)
        store_cols_slab(buf + kBM * kLd, rw);
    else
        store_rows_slab(buf + kBM * kLd, rw);
}

// acc[rt][ct] += C^T tile (features ct*16.., tokens rt*16..) of this wave for one 32-wide slab in LDS;
// in half h lane group g supplies k = 16h + 4g .. +3 (one ds_read_b128 per operand and half).
__device__ __forceinline__ void slab_mfma(const float* __restrict__ buf, int wave, int g, int c16,
                                          floatx4 (&acc)[2][8]) {
    const float* Xs = buf;
    const float* Ws = buf + kBM * kLd;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        float4 xb[2], wa[8];
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
            xb[rt] = *reinterpret_cast<const float4*>(Xs + (wave * 32 + rt * 16 + c16) * kLd + 16 * h + 4 * g);
#pragma unroll
        for (int ct = 0; ct < 8; ++ct)
            wa[ct] = *reinterpret_cast<const float4*>(Ws + (ct * 16 + c16) * kLd + 16 * h + 4 * g);
#pragma unroll
        for (int ct = 0; ct < 8; ++ct)
#pragma unroll
            for (int rt = 0; rt < 2; ++rt) acc[rt][ct] = mfma16(wa[ct].x, xb[rt].x, acc[rt][ct]);
#pragma unroll
        for (int ct = 0; ct < 8; ++ct)
#pragma unroll
            for (int rt = 0; rt < 2; ++rt) acc[rt][ct] = mfma16(wa[ct].y, xb[rt].y, acc[rt][ct]);
#pragma unroll
        for (int ct = 0; ct < 8; ++ct)
#pragma unroll
            for (int rt = 0; rt < 2; ++rt) acc[rt][ct] = mfma16(wa[ct].z, xb[rt].z, acc[rt][ct]);
#pragma unroll
        for (int ct = 0; ct < 8; ++ct)
#pragma unroll
            for (int rt = 0; rt < 2; ++rt) acc[rt][ct] = mfma16(wa[ct].w, xb[rt].w, acc[rt][ct]);
    }
}

// Persistent tile schedule: the tile list [m-block][n-block] is split into 8 contiguous ranges, one
// per XCD (hardware workgroup ids go round-robin over the XCDs), so the n-blocks of one m-block -- which
// stream the same X slabs -- run side by side on one XCD and share its L2.
struct TileSched {
    int64_t first, stride, count;
    __device__ explicit TileSched(int64_t nt) {
        const int xcd = blockIdx.x % 8, slot = blockIdx.x / 8;
        const int64_t per_xcd = (nt + 7) / 8;
        first = (int64_t)xcd * per_xcd + slot;
        stride = gridDim.x / 8;  // the launch uses a multiple of 8 workgroups
        const int64_t end = min(nt, (int64_t)(xcd + 1) * per_xcd);
        count = first < end ? (end - first + stride - 1) / stride : 0;
    }
    __device__ int64_t tile(int64_t j) const { return first + j * stride; }
};

struct EpiArgs {
    const float* bias;  // [N] (forward)
    int accumulate;     // backward: dX += C
};

template <bool TRANS_W>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(2, 2))) void linear_kernel(const float* __restrict__ X, int64_t ldx, int64_t M, int K,
                                                          const float* __restrict__ W, int64_t ldw, int N,
                                                          float* __restrict__ Y, int64_t ldy, EpiArgs ep) {
    __shared__ __attribute__((aligned(16))) float lds[2][(kBM + kBN) * kLd];
    const int nblk_n = (N + kBN - 1) / kBN;
    const int nslab = (K + kBK - 1) / kBK;
    const TileSched ts(((M + kBM - 1) / kBM) * nblk_n);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, g = lane >> 4, c16 = lane & 15;
    const int64_t steps = ts.count * nslab;
    // flattened (tile, slab) pipeline over a double-buffered LDS slab: slab it+1 is stored while slab it
    // is multiplied, slab it+2 is in flight in registers, and a finished tile's epilogue overlaps both
    auto coords = [&](int64_t it, int64_t& m0, int& n0, int& k0) {
        const int j = (int)it / nslab;  // steps < 2^31
        const int t = (int)ts.tile(j);  // tiles < 2^31
        m0 = (int64_t)(t / nblk_n) * kBM;
        n0 = (t % nblk_n) * kBN;
        k0 = ((int)it - j * nslab) * kBK;
    };
    float4 rx[4], rw[4];
    if (steps > 0) {
        int64_t m0;
        int n0, k0;
        coords(0, m0, n0, k0);
        load_slab<TRANS_W>(X, ldx, M, K, W, ldw, N, m0, n0, k0, rx, rw);
        store_slab<TRANS_W>(lds[0], rx, rw);
        if (steps > 1) {
            coords(1, m0, n0, k0);
            load_slab<TRANS_W>(X, ldx, M, K, W, ldw, N, m0, n0, k0, rx, rw);
        }
        __syncthreads();
    }
    floatx4 acc[2][8];
    for (int64_t it = 0; it < steps; ++it) {
        const int slab = (int)it % nslab;
        int64_t m0;
        int n0, k0;
        coords(it, m0, n0, k0);
        if (slab == 0) {
#pragma unroll
            for (int rt = 0; rt < 2; ++rt)
#pragma unroll
                for (int ct = 0; ct < 8; ++ct) acc[rt][ct] = floatx4{0.f, 0.f, 0.f, 0.f};
        }
        slab_mfma(lds[it & 1], wave, g, c16, acc);
        if (it + 1 < steps) store_slab<TRANS_W>(lds[(it + 1) & 1], rx, rw);
        // the prefetch registers are free from here until the next slab's loads are issued below, which
        // keeps the epilogue's register budget; those loads still have a whole slab of MFMA work to land
        if (slab == nslab - 1) {
#pragma unroll
            for (int rt = 0; rt < 2; ++rt) {
                const int64_t m = m0 + wave * 32 + rt * 16 + c16;
                if (m >= M) continue;
#pragma unroll
                for (int ct = 0; ct < 8; ++ct) {
                    const int n = n0 + ct * 16 + 4 * g;
                    if (n >= N) continue;
                    float4 v = make_float4(acc[rt][ct][0], acc[rt][ct][1], acc[rt][ct][2], acc[rt][ct][3]);
                    if (ep.bias) {
                        const float4 bv = *reinterpret_cast<const float4*>(ep.bias + n);
                        v.x += bv.x;
                        v.y += bv.y;
                        v.z += bv.z;
                        v.w += bv.w;
                    }
                    float* dst = Y + m * ldy + n;
                    if (ep.accumulate) {
                        const float4 o = *reinterpret_cast<const float4*>(dst);
                        v.x += o.x;
                        v.y += o.y;
                        v.z += o.z;
                        v.w += o.w;
                    }
                    *reinterpret_cast<float4*>(dst) = v;
                }
            }
        }
        if (it + 2 < steps) {
            int64_t m2;
            int n2, k2;
            coords(it + 2, m2, n2, k2);
            load_slab<TRANS_W>(X, ldx, M, K, W, ldw, N, m2, n2, k2, rx, rw);
        }
        __syncthreads();
    }
}

// persistent grid: 2 resident workgroups per CU (VGPR-bound), a multiple of 8 for the XCD split
int64_t linear_grid(int64_t M, int64_t N) {
    static const int n_cu = [] {  // (thread-safe initialisation)
        int dev = 0;
        hipDeviceProp_t prop;
        return (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
                   ? prop.multiProcessorCount
                   : 256;
    }();
    const int64_t ntiles = ((M + kBM - 1) / kBM) * ((N + kBN - 1) / kBN);
    const int64_t grid = std::min<int64_t>((int64_t)n_cu * 2, (ntiles + 7) / 8 * 8);
    return std::max<int64_t>(8, grid / 8 * 8);
}

template <bool TRANS_W>
int launch_linear(const float* X, int64_t ldx, int64_t M, int K, const float* W, int64_t ldw, int N, float* Y,
                  int64_t ldy, const EpiArgs& ep, hipStream_t s) {
    const int64_t grid = linear_grid(M, N);
    hipLaunchKernelGGL((linear_kernel<TRANS_W>), dim3((unsigned)grid), dim3(kThreads), 0, s, X, ldx, M, K, W,
                       ldw, N, Y, ldy, ep);
    return hip_status(hipGetLastError(), "linear");
}

bool shapes_ok(const void* a, int64_t lda, const void* b, int64_t ldb, int K, int N) {
    return K % 4 == 0 && N % 4 == 0 && lda % 4 == 0 && ldb % 4 == 0 && ((uintptr_t)a & 15) == 0 &&
           ((uintptr_t)b & 15) == 0;
}

}  // namespace

// y (n_rows x out_f, row stride ld_y) = x (n_rows x in_f, stride ld_x) . w^T + b      (w: out_f x in_f)
ASME_API int asme_linear_fwd(const float* x, int64_t ld_x, int64_t n_rows, int64_t in_f, const float* w,
                             const float* b, int64_t out_f, float* y, int64_t ld_y, void* stream) {
    ASME_CHECK_ARG(x && w && y, "asme_linear_fwd: null pointer");
    ASME_CHECK_ARG(shapes_ok(x, ld_x, w, in_f, (int)in_f, (int)out_f) && ld_y % 4 == 0 && ((uintptr_t)y & 15) == 0,
                   "asme_linear_fwd: features / strides must be multiples of 4 floats, 16-B aligned");
    if (n_rows == 0) return 0;
    EpiArgs ep{};
    ep.bias = b;
    return launch_linear<false>(x, ld_x, n_rows, (int)in_f, w, in_f, (int)out_f, y, ld_y, ep,
                                           (hipStream_t)stream);
}

// dx (n_rows x in_f) (+)= dy (n_rows x out_f) . w      (w: out_f x in_f)
ASME_API int asme_linear_dx(const float* dy, int64_t ld_dy, int64_t n_rows, int64_t out_f, const float* w,
                            int64_t in_f, float* dx, int64_t ld_dx, int accumulate, void* stream) {
    ASME_CHECK_ARG(dy && w && dx, "asme_linear_dx: null pointer");
    ASME_CHECK_ARG(shapes_ok(dy, ld_dy, w, in_f, (int)out_f, (int)in_f) && ld_dx % 4 == 0 &&
                       ((uintptr_t)dx & 15) == 0,
                   "asme_linear_dx: features / strides must be multiples of 4 floats, 16-B aligned");
    if (n_rows == 0) return 0;
    EpiArgs ep{};
    ep.accumulate = accumulate;
    return launch_linear<true>(dy, ld_dy, n_rows, (int)out_f, w, in_f, (int)in_f, dx, ld_dx, ep,
                                          (hipStream_t)stream);
}
