// Full-catalogue logits head on gfx950's bf16 matrix cores with fp32-level products (bf16x6, common.h):
// fused logits + CrossEntropyLoss(ignore_index) for training (the (n x |V|) logits never reach HBM) and the
// materialised (n x |V|) scores for evaluation / predict.
//
// Reference semantics (paths relative to /root/reference/src/asme):
//   LinearProjectionLayer / ItemEmbeddingProjectionLayer (tied h E^T + b)   core/models/common/layers/layers.py:105-109,138-143
//   MaskedTrainingModule._calc_loss, CrossEntropyLoss(ignore_index=pad)      core/modules/masked_training_module.py:93-111
//   SingleTargetCrossEntropyLoss / SASRecFullSequenceCrossEntropyLoss       core/losses/losses.py:77-115
//   SASRecProjectionComponent inference (last position . E^T)               core/models/sasrec/components.py:46-61
//
//   s[q][i] = H[q] . W[i] + b[i],  lse[q] = log sum_i exp s[q][i],  loss = mean_{valid q} (lse[q] - s[q][t_q])
//   dS = (softmax(s) - onehot(t)) * dloss / count;  dH = dS W;  dW = dS^T H;  db = colsum(dS)
//
// Operands.  H (n x d) and W (|V| x d) are split once per call into three bf16 planes each (x = h + m + l exactly,
// rows zero-padded to 128 features and to a multiple of 128 rows): the hot loops then run only MFMAs and LDS
// reads -- no VALU split of a reused operand.  Every pass is one kernel template over a (stationary, streamed)
// pair of those planes:
//   stationary rows: 16 per wave, their three planes held as MFMA B fragments in registers for the whole kernel
//   streamed rows:   64-row tiles of the three planes through a double-buffered LDS image (one barrier per tile)
//                    in the T10 swizzle (plain 256-B rows, chunk ^ ((r&3)<<2 | (r>>2)&3)): ds_read_b128 row
//                    reads for the score product, ds_read_b64_tr_b16 transposed reads for the gradient product
//   X = A_streamed . B_stationary^T (v_mfma_f32_16x16x32_bf16 x 6): lane (stationary row c, group g) holds
//   streamed rows 4g..4g+3 of each 16-row sub-tile, so a pair of sub-tiles gives the 8 values the lane supplies
//   as the B fragment of the NEXT product, which sums over the streamed rows with no lane movement:
//   Y^T[f][c] += (streamed^T)[f][rows] . P[rows][c]   (the streamed operand read back transposed)
// Passes (n queries, V items; the streamed operand is split into 8k chunks, chunk = workgroup % nchunks, so the
// workgroups of one XCD share one chunk in their L2):
//   stats   stationary = queries, streamed = items: online (max, sum exp) per query per chunk + target logit
//   dH      stationary = queries, streamed = items: P = exp(s + b - lse) - onehot; dH^T += W^T P^T
//   dW, db  stationary = items, streamed = queries: P^T the same way;            dW^T += H^T P
//   logits  stationary = queries, streamed = items: out = s + b
//   fdh     stationary = queries, streamed = items: the training forward with dH folded in -- online (max, sum exp)
//           per query per chunk and U^T += W^T exp(s + b - reference max), rescaled when a tile's max passes the
//           reference by more than 8 (the flash-attention forward with the item table as V); a finish pass merges
//           the chunks into lse, the loss and dH_raw = softmax(s) W - W[t] (0 for ignored rows), and the backward
//           only scales it (x dloss / count)
// Work: training runs fdh (4 n|V|d FLOP) + dW (4) = 8 n|V|d executed for the 6 of a materialised head (stats + dH +
// dW: 10); HBM bytes O((n+V)d).  Partial slabs of the chunks are summed in a fixed order: deterministic.
#include "common.h"
#include <algorithm>

#ifndef ASME_LOGITS_PIPE
#define ASME_LOGITS_PIPE 0
#endif
#ifndef ASME_LOGITS_DIAG
#define ASME_LOGITS_DIAG 0  // diagnostic builds of the fdh pass: 1 no gradient product, 2 no score product, 3 no exp,
                            // 4 no next-tile DMA (the current tile re-used)
#endif

using namespace asme;

namespace {

typedef short short4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) short4v lds_short4;

constexpr int kDP = 128;                 // padded feature width of a plane row (256 B)
constexpr int kRowB = kDP * 2;           // bytes per plane row
constexpr int kTS = 64;                  // streamed rows per LDS tile
// workgroup = W waves x 32 stationary rows: W = 8 (two waves per SIMD, 256 registers each: the partner wave's
// MFMAs fill this wave's softmax VALU) where the pass fits that budget (stats, logits); W = 4 (one wave per SIMD,
// 512 registers) for the gradient passes, whose stationary fragments + 128-feature accumulators need more
constexpr int kRowPad = 256;             // plane rows are padded to a multiple of this (>= 32 W, kTS)
template <int MODE> struct EngineWaves { static constexpr int W = (MODE == 1 || MODE == 2 || MODE == 4) ? 4 : 8; };
// M_RANK / M_TSCORE (modes 5 / 6): the full-catalogue evaluation's target ranks on the same score product
constexpr int kPlaneTile = kTS * kRowB;  // 16 KiB: one plane of one tile
constexpr int kTile = 3 * kPlaneTile;    // 48 KiB

enum { M_STATS = 0, M_DH = 1, M_DW = 2, M_LOGITS = 3, M_FDH = 4, M_RANK = 5, M_TSCORE = 6 };

__host__ __device__ constexpr int64_t pad_rows(int64_t r) { return (r + kRowPad - 1) / kRowPad * kRowPad; }

// byte offset of 16-B chunk ch of row r in a plane image of 256-B rows (cdna_hip_programming.md T10, image (b)):
// conflict-free ds_read_b64_tr_b16 reads, 2-way ds_read_b128 row reads of the 16x16x32 operand
__device__ __forceinline__ int swz(int r, int ch) { return r * kRowB + 16 * (ch ^ (((r & 3) << 2) | ((r >> 2) & 3))); }

__device__ __forceinline__ bf16x8 lds_b128(const char* base, int off) {
    return *reinterpret_cast<const bf16x8*>(base + off);
}
__device__ __forceinline__ short4v lds_tr(const char* base, int off) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4*)(base + off));
}
__device__ __forceinline__ bf16x8 cat8(short4v lo, short4v hi) {
    typedef short short8v __attribute__((ext_vector_type(8)));
    const short8v v = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    return __builtin_bit_cast(bf16x8, v);
}

// ------------------------------------------------------------------------------------------------ split
// planes[p][r][0..127] (bf16) = plane p of X[r][0..d) (zero beyond d and for r >= rows), r < rows_pad
__global__ __launch_bounds__(256) void split_planes_kernel(const float* __restrict__ X, int64_t ld, int64_t rows,
                                                           int d, int64_t rows_pad, __bf16* __restrict__ planes) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // one thread per 8 features
    if (t >= rows_pad * (kDP / 8)) return;
    const int64_t r = t / (kDP / 8);
    const int c = (int)(t % (kDP / 8)) * 8;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
    if (r < rows) {
        const float* x = X + r * ld;
        if (c + 8 <= d) {
            a = *reinterpret_cast<const float4*>(x + c);
            b = *reinterpret_cast<const float4*>(x + c + 4);
        } else if (c < d) {
            float v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = c + j < d ? x[c + j] : 0.f;
            a = make_float4(v[0], v[1], v[2], v[3]);
            b = make_float4(v[4], v[5], v[6], v[7]);
        }
    }
    const Bf3 s = split_bf3(a, b);
    const int64_t o = r * kDP + c, P = rows_pad * kDP;
    *reinterpret_cast<bf16x8*>(planes + o) = s.h;
    *reinterpret_cast<bf16x8*>(planes + P + o) = s.m;
    *reinterpret_cast<bf16x8*>(planes + 2 * P + o) = s.l;
}

// ------------------------------------------------------------------------------------------------ engine
struct LogitsArgs {
    const __bf16* stat;     // stationary planes (3 x stat_pad x 128)
    const __bf16* strm;     // streamed planes (3 x strm_pad x 128)
    int64_t stat_pad, strm_pad;
    int64_t n_stat, n_strm;  // real rows
    int64_t chunk;           // streamed rows per chunk (multiple of kTS)
    int nchunks;
    int d;
    const float* bias;       // [V] or null
    const int64_t* targets;  // [n]
    int64_t ignore;
    int64_t V;               // = the item count (n_strm in stats / dH / logits, n_stat in dW)
    const float* lse;        // [n] (dH, dW)
    const float* dloss;      // dH, dW: scale = dloss[0] / stats[1]
    const float* stats;
    float* part;             // stats: (nchunks, n, 2); dH: (nchunks, n, d) or dH; dW: (nchunks, V, d) or dW
    float* part2;            // stats: target logits [n]; dW: db partials (nchunks, V) or db (nullable)
    float* out;              // logits: (n, ld_out)
    int64_t ld_out;
    float* upart;            // fdh: (nchunks, n, d) unnormalised softmax-weighted item rows per chunk
    // full-catalogue ranking (rank: stationary = queries, streamed = items; tscore: streamed = the queries' gathered
    // target rows, row q = the target of query q): global item id of streamed row j = j * id_stride + id_offset
    const float* tscore;     // rank: the target's score per query (from the tscore pass: the same products)
    int32_t* counts;         // rank: per query, items ranked above the target (atomically summed over chunks)
    int64_t id_stride, id_offset;
    int64_t tclamp;          // rank: > 0: a target outside [0, tclamp) counts as item 0 (as gather_targets_kernel reads it)
    int64_t sblocks, per_xcd;  // set by launch_engine: the grid's work items and work items per XCD slot group
};

// workgroup -> (chunk, stationary block), chunk-major within an XCD.  Workgroups b, b + 8, b + 16, ... share an XCD
// (the dispatcher deals them round-robin; a speed assumption only -- any placement gives the same results), so slot
// group b % 8 takes the contiguous run [(b % 8) per_xcd, (b % 8 + 1) per_xcd) of the chunk-major work list: the CUs
// of one XCD stream the same chunk's tiles at about the same time and keep one copy of them in that XCD's L2 (with
// chunk = b % nchunks every XCD streamed every chunk whenever nchunks was not a multiple of 8).  The grid's few
// padding workgroups (w >= sblocks x nchunks) return before touching anything.
#ifndef ASME_LOGITS_XCD
#define ASME_LOGITS_XCD 1  // 0: chunk = b % nchunks (the round-4 mapping, for A/B)
#endif
__device__ __forceinline__ bool work_item(const LogitsArgs& a, int& chunk_id, int64_t& sblock) {
    if (!ASME_LOGITS_XCD) {
        if (blockIdx.x >= a.sblocks * a.nchunks) return false;
        chunk_id = (int)(blockIdx.x % (unsigned)a.nchunks);
        sblock = blockIdx.x / (unsigned)a.nchunks;
        return true;
    }
    const int64_t w = (int64_t)(blockIdx.x & 7u) * a.per_xcd + (blockIdx.x >> 3);
    if (w >= a.sblocks * a.nchunks) return false;
    chunk_id = (int)(w / a.sblocks);
    sblock = w - (int64_t)chunk_id * a.sblocks;
    return true;
}

__device__ __forceinline__ bool valid_target(int64_t t, int64_t ignore, int64_t V) {
    return t != ignore && t >= 0 && t < V;
}

// One streamed tile (3 planes x kTS rows x 256 B) straight from HBM/L2 into an LDS buffer by LDS-DMA
// (global_load_lds_dwordx4: 1 KiB = 4 image rows per wave-instruction, lane L -> bytes 16L..16L+15): each lane
// fetches the source chunk that the swizzle puts at its destination slot, so the image is written in place
// without registers or ds_write.  Completion: the issuing wave's vmcnt, then the workgroup barrier.
template <int W>
__device__ __forceinline__ void dma_tile(const __bf16* __restrict__ planes, int64_t pad, int64_t row0, char* buf) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int i = 0; i < kTile / 1024 / W; ++i) {
        const int w = wave + W * i;                     // wave-instruction: plane w / 16, image rows 4 (w % 16) ..
        const int p = w / (kTS / 4), R = 4 * (w % (kTS / 4));
        const int row = R + (lane >> 4);
        const int ch = (lane & 15) ^ (((row & 3) << 2) | ((row >> 2) & 3));  // swz(): slot lane & 15 holds chunk ch
        const __bf16* src = planes + (int64_t)p * pad * kDP + (row0 + row) * kDP + ch * 8;
        __builtin_amdgcn_global_load_lds((const void*)src,
                                         (__attribute__((address_space(3))) void*)(buf + p * kPlaneTile + R * kRowB),
                                         16, 0, 0);
    }
}
__device__ __forceinline__ void wait_dma() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// per-streamed-row metadata staged next to the tile: M_STATS / M_DH / M_LOGITS: item bias (-inf beyond V);
// M_DW: query lse (+inf for ignored / padding queries) and target (-1 for them)
struct TileMeta {
    float f;
    int t;
    __device__ __forceinline__ void load(int mode, const LogitsArgs& a, int64_t row) {
        if (mode == M_DW) {
            const int64_t tg = row < a.n_strm ? a.targets[row] : -1;
            const bool ok = row < a.n_strm && valid_target(tg, a.ignore, a.V);
            f = ok ? a.lse[row] : INFINITY;
            t = ok ? (int)tg : -1;
        } else {
            f = row < a.n_strm ? (a.bias ? a.bias[row] : 0.f) : -INFINITY;
            t = 0;
        }
    }
};

// 32x32x16 fragment maps (cdna_hip_programming.md §3): lane l (r = l & 31, h = l >> 5) supplies A[row r][k 8h..8h+7]
// and B[k 8h..8h+7][col r]; accumulator register i holds C[row (i & 3) + 8 (i >> 2) + 4h][col r].
__device__ __forceinline__ int acc_row(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

template <int MODE, int KB, int W>
__global__ __launch_bounds__(W * 64) void logits_engine_kernel(LogitsArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* bufs = smem;                                                  // 2 x kTile
    float* mf = reinterpret_cast<float*>(smem + 2 * kTile);            // 2 x kTS
    int* mt = reinterpret_cast<int*>(smem + 2 * kTile + 2 * kTS * 4);  // 2 x kTS
    constexpr int KS = 2 * KB;  // 16-k steps of the score product
    constexpr int NFT = KB;     // 32-feature tiles of the gradient product
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, h = lane >> 5, r32 = lane & 31;
    int chunk_id;
    int64_t sblock;
    if (!work_item(a, chunk_id, sblock)) return;  // grid padding (whole workgroup)
    const int64_t srow = sblock * (32 * W) + wave * 32 + r32;  // this lane's stationary row (MFMA column)
    // (M_TSCORE: the streamed rows are the stationary block's own gathered target rows)
    const int64_t s_begin = MODE == M_TSCORE ? sblock * (32 * W) : (int64_t)chunk_id * a.chunk;
    const int64_t s_end = std::min(a.strm_pad, s_begin + (MODE == M_TSCORE ? 32 * W : a.chunk));  // past n_strm: zero planes

    // stationary fragments (B operand): row srow, k = 16 ks + 8 h .. +7, three planes
    Bf3 st[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
        const int64_t o = srow * kDP + 16 * ks + 8 * h;
        st[ks].h = *reinterpret_cast<const bf16x8*>(a.stat + o);
        st[ks].m = *reinterpret_cast<const bf16x8*>(a.stat + a.stat_pad * kDP + o);
        st[ks].l = *reinterpret_cast<const bf16x8*>(a.stat + 2 * a.stat_pad * kDP + o);
    }
    // stationary-row metadata
    float s_lse = 0.f, s_bias = 0.f;
    int s_tgt = -1;
    if (MODE == M_DH || MODE == M_STATS || MODE == M_FDH) {
        const int64_t tg = srow < a.n_stat ? a.targets[srow] : -1;
        const bool ok = srow < a.n_stat && valid_target(tg, a.ignore, a.V);
        s_tgt = ok ? (int)tg : -1;
        if (MODE == M_DH) s_lse = ok ? a.lse[srow] : INFINITY;  // ignored / padding queries: P = 0
    } else if (MODE == M_DW) {
        s_bias = srow < a.n_stat ? (a.bias ? a.bias[srow] : 0.f) : -INFINITY;
        s_tgt = (int)srow;  // compare the streamed query's target against this item
    }
    float run_max = -INFINITY, run_sum = 0.f, t_logit = 0.f;
    bool have_t = false;
    // M_RANK: this query's target score and, in local row numbers j of the streamed table (item j * id_stride +
    // id_offset), the target's own row (j_eq, -1 when another shard holds it) and the rows of lower item ids
    // (j < j_lt): every per-element test below is 32-bit
    float r_ts = 0.f;
    int r_jeq = -1, r_jlt = 0, r_cnt = 0;
    if (MODE == M_RANK && srow < a.n_stat) {
        r_ts = a.tscore[srow];
        int64_t tg = a.targets[srow];
        if (a.tclamp > 0 && (tg < 0 || tg >= a.tclamp)) tg = 0;  // the id whose score tscore holds
        // (64-bit until clamped to this shard's rows: any target id, valid or not, gives 32-bit row numbers)
        const int64_t rel = tg - a.id_offset;
        const int64_t jq = rel >= 0 ? rel / a.id_stride : -1;
        r_jeq = (rel >= 0 && rel % a.id_stride == 0 && jq < a.n_strm) ? (int)jq : -1;
        const int64_t jl = rel > 0 ? (rel + a.id_stride - 1) / a.id_stride : 0;
        r_jlt = (int)(jl < a.n_strm ? jl : a.n_strm);
    }
    floatx16 y[NFT];  // gradient product: Y^T[feature 32 ft + acc_row(i, h)][stationary row r32]
#pragma unroll
    for (int f = 0; f < NFT; ++f)
#pragma unroll
        for (int i = 0; i < 16; ++i) y[f][i] = 0.f;
    float db = 0.f;

    TileMeta tm;
    if (s_begin < s_end) {
        dma_tile<W>(a.strm, a.strm_pad, s_begin, bufs);
        if (threadIdx.x < kTS) {
            tm.load(MODE, a, s_begin + threadIdx.x);
            mf[threadIdx.x] = tm.f;
            mt[threadIdx.x] = tm.t;
        }
        wait_dma();
    }
    __syncthreads();
    int it = 0;
    for (int64_t r0 = s_begin; r0 < s_end; r0 += kTS, ++it) {
        const int cur = it & 1;
        const bool more = r0 + kTS < s_end;
        if (more) {  // the next tile flies into the other buffer during this tile's MFMAs
            if (ASME_LOGITS_DIAG != 4 || MODE != M_FDH) dma_tile<W>(a.strm, a.strm_pad, r0 + kTS, bufs + (cur ^ 1) * kTile);
            if (threadIdx.x < kTS) tm.load(MODE, a, r0 + kTS + threadIdx.x);
        }
        const char* buf = bufs + cur * kTile;
        const float* tf = mf + cur * kTS;
        const int* tt = mt + cur * kTS;
        // X = streamed rows 32 sub .. +31 (MFMA rows) x stationary rows (columns): row reads of the tile
        auto score_a = [&](int sub, int ks) {
            const int off = swz(32 * sub + r32, 2 * ks + h);
            Bf3 A;
            A.h = lds_b128(buf, off);
            A.m = lds_b128(buf + kPlaneTile, off);
            A.l = lds_b128(buf + 2 * kPlaneTile, off);
            return A;
        };
        auto score = [&](int sub) {
            floatx16 x;
#pragma unroll
            for (int i = 0; i < 16; ++i) x[i] = 0.f;
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) x = mfma32_bf3(score_a(sub, ks), st[ks], x);
            return x;
        };
        // P (unscaled) as the split B fragments of the two 16-row k steps:
        //   dH: streamed = items (bias tf, id r0 + lr), stationary = query (s_lse, s_tgt)
        //   dW: streamed = queries (lse tf, target tt), stationary = item (s_bias, id srow)
        auto probs = [&](floatx16 x, int sub, Bf3 (&P)[2]) {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int lr = 32 * sub + acc_row(i, h);
                if (MODE == M_DH) {
                    x[i] = __expf(x[i] + tf[lr] - s_lse) - ((int64_t)s_tgt == r0 + lr ? 1.f : 0.f);
                } else {
                    x[i] = __expf(x[i] + s_bias - tf[lr]) - (tt[lr] == s_tgt ? 1.f : 0.f);
                    db += x[i];
                }
            }
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2)
                P[s2] = split_bf3(make_float4(x[8 * s2], x[8 * s2 + 1], x[8 * s2 + 2], x[8 * s2 + 3]),
                                  make_float4(x[8 * s2 + 4], x[8 * s2 + 5], x[8 * s2 + 6], x[8 * s2 + 7]));
        };
        // Y^T[f][r32] += streamed^T[f][rows] . P[rows][r32], k step s2 = rows 16 s2 .. +15 of the sub-tile: the
        // B fragment is P registers 8 s2 .. 8 s2 + 7 (element j = row 16 s2 + 8 (j >> 2) + 4 h + (j & 3)); the A
        // fragment comes from two transposed reads: 16-lane group (h, fh) reads rows 16 s2 + 4 h + q (+8) x
        // features 32 ft + 16 fh + 4 p4 .. +3 (lane 4q + p4 addresses one row), lane receives its feature
        auto grad_a = [&](int sub, int s2, int ft) {
            const int fh = (lane >> 4) & 1, q = (lane & 15) >> 2, p4 = lane & 3;
            const int rlo = 32 * sub + 16 * s2 + 4 * h + q, rhi = rlo + 8;
            const int ch = 4 * ft + 2 * fh + (p4 >> 1);
            const int olo = swz(rlo, ch) + 8 * (p4 & 1), ohi = swz(rhi, ch) + 8 * (p4 & 1);
            Bf3 A;
            A.h = cat8(lds_tr(buf, olo), lds_tr(buf, ohi));
            A.m = cat8(lds_tr(buf + kPlaneTile, olo), lds_tr(buf + kPlaneTile, ohi));
            A.l = cat8(lds_tr(buf + 2 * kPlaneTile, olo), lds_tr(buf + 2 * kPlaneTile, ohi));
            return A;
        };
        auto grad = [&](int sub, const Bf3 (&P)[2]) {
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
                for (int ft = 0; ft < NFT; ++ft) y[ft] = mfma32_bf3(grad_a(sub, s2, ft), P[s2], y[ft]);
        };
        if constexpr (MODE == M_FDH) {
#if ASME_LOGITS_DIAG == 2
            floatx16 xs[2];
#pragma unroll
            for (int i = 0; i < 16; ++i) xs[0][i] = xs[1][i] = tf[i] * (float)(i + 1);
#else
            floatx16 xs[2] = {score(0), score(1)};
#endif
            float tmax = -INFINITY;
#pragma unroll
            for (int sub = 0; sub < 2; ++sub) {
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    xs[sub][i] += tf[32 * sub + acc_row(i, h)];
                    tmax = fmaxf(tmax, xs[sub][i]);
                }
                const int rel = s_tgt - (int)(r0 + 32 * sub);  // target in this sub-tile and lane half?
                if ((unsigned)rel < 32u && ((rel >> 2) & 1) == h) {
                    const int ri = (rel & 3) + 4 * (rel >> 3);
#pragma unroll
                    for (int i = 0; i < 16; ++i)
                        if (i == ri) t_logit = xs[sub][i];
                    have_t = true;
                }
            }
            // one running max per query over both lane halves: both halves' P feed the same accumulators
            tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
            // lazy rescale: the reference max moves (and the 64 accumulators are rescaled) only when some query's
            // tile max exceeds it by more than 8 -- P = exp(s - ref) then stays <= e^8, exact in the bf16x6 split
            // and far from fp32 overflow; the (ref, sum, U) triple it leaves is the same softmax state.  The rescale
            // had run every tile (64 multiplies on accumulators held in AGPRs, moved through VGPRs): fwd_dh
            // 2.71 -> 2.61 ms at the C3 shape (tools/xent_bench.py, same box)
            if (__ballot(!(tmax <= run_max + 8.f)) != 0ull) {
                const float nm = fmaxf(run_max, tmax);
                const float alpha = run_max == -INFINITY ? 0.f : __expf(run_max - nm);
#pragma unroll
                for (int f = 0; f < NFT; ++f)
#pragma unroll
                    for (int i = 0; i < 16; ++i) y[f][i] *= alpha;
                run_sum *= alpha;
                run_max = nm;
            }
            const float base = run_max == -INFINITY ? 0.f : run_max;  // nothing finite yet: P = 0, no NaN
#pragma unroll
            for (int sub = 0; sub < 2; ++sub) {
#pragma unroll
                for (int i = 0; i < 16; ++i) {
#if ASME_LOGITS_DIAG == 3
                    xs[sub][i] = xs[sub][i] - base;
#else
                    xs[sub][i] = __expf(xs[sub][i] - base);
#endif
                    run_sum += xs[sub][i];
                }
                Bf3 P[2];
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2)
                    P[s2] = split_bf3(
                        make_float4(xs[sub][8 * s2], xs[sub][8 * s2 + 1], xs[sub][8 * s2 + 2], xs[sub][8 * s2 + 3]),
                        make_float4(xs[sub][8 * s2 + 4], xs[sub][8 * s2 + 5], xs[sub][8 * s2 + 6],
                                    xs[sub][8 * s2 + 7]));
#if ASME_LOGITS_DIAG == 1
                asm volatile("" ::"v"(P[0].h), "v"(P[0].m), "v"(P[0].l), "v"(P[1].h), "v"(P[1].m), "v"(P[1].l));
#else
                grad(sub, P);
#endif
            }
        } else if constexpr (MODE == M_DH || MODE == M_DW) {
#if ASME_LOGITS_PIPE
            // one wave per SIMD: software-pipeline the tile's two sub-tiles so the softmax VALU of one runs in the
            // MFMA shadow of the other's products: [S0] [P0 | S1] [G0 | P1] [G1], interleaved by the scheduler
            // directives (per MFMA: at most one LDS read and five vector instructions, MI355X guide T19)
            const floatx16 x0 = score(0);
            __builtin_amdgcn_sched_barrier(0);
            Bf3 P0[2], P1[2];
            probs(x0, 0, P0);
            const floatx16 x1 = score(1);
#pragma unroll
            for (int i = 0; i < 6 * KS / 2; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, 5, 0);
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, 5, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
            grad(0, P0);
            probs(x1, 1, P1);
#pragma unroll
            for (int i = 0; i < 12 * NFT; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 1);
                __builtin_amdgcn_sched_group_barrier(0x002, 5, 1);
            }
            __builtin_amdgcn_sched_barrier(0);
            grad(1, P1);
#else
#pragma unroll
            for (int sub = 0; sub < kTS / 32; ++sub) {
                Bf3 P[2];
                probs(score(sub), sub, P);
                grad(sub, P);
            }
#endif
        } else {
#pragma unroll
            for (int sub = 0; sub < kTS / 32; ++sub) {
                floatx16 x = score(sub);
                if (MODE == M_RANK) {
                    // item i is ranked above the target t iff s_i > s_t, or s_i == s_t and i < t (ties to the lower
                    // id, the reference argsort's order on tie-free data); s = products + bias exactly as M_TSCORE and
                    // M_LOGITS form it, so the target compares bit-identically with itself
                    // (row j = j0 + c, c = acc_row(i, h) in [0, 32); tests without short-circuit branches)
                    const int j0 = (int)r0 + 32 * sub;
                    const int t_lt = r_jlt - j0, t_eq = r_jeq - j0, t_n = (int)a.n_strm - j0;
                    // the common case: for every lane of the wave the sub-tile holds neither its target's row nor its
                    // lower-id boundary and every row exists; then "above" is sc > r_ts (no row below the target's
                    // id) or sc >= r_ts (all rows below it) = sc > the float just below r_ts -- one compare per element
                    // (r_ts finite and non-zero, so the float below is a normal number or the largest negative one)
                    const bool clean = t_n >= 32 && (t_eq < 0 || t_eq >= 32) && (t_lt <= 0 || t_lt >= 32) &&
                                       __builtin_isfinite(r_ts) && r_ts != 0.f;
                    if (__ballot(!clean) == 0ull) {
                        const float thr = t_lt >= 32 ? __int_as_float(__float_as_int(r_ts) + (r_ts > 0.f ? -1 : 1))
                                                     : r_ts;
                        if (!a.bias) {  // (no bias: every row of a clean sub-tile adds +0, which no comparison sees)
#pragma unroll
                            for (int i = 0; i < 16; ++i) r_cnt += x[i] > thr ? 1 : 0;
                        } else {
#pragma unroll
                            for (int i = 0; i < 16; ++i) r_cnt += (x[i] + tf[32 * sub + acc_row(i, h)]) > thr ? 1 : 0;
                        }
                    } else {
#pragma unroll
                        for (int i = 0; i < 16; ++i) {
                            const int c = acc_row(i, h);
                            const float sc = x[i] + tf[32 * sub + c];
                            const bool above = ((sc > r_ts) | ((sc == r_ts) & (c < t_lt))) & (c < t_n) & (c != t_eq);
                            r_cnt += above ? 1 : 0;
                        }
                    }
                    continue;
                }
                if (MODE == M_TSCORE) {
                    // the diagonal: streamed row == stationary row (query q's gathered target row)
#pragma unroll
                    for (int i = 0; i < 16; ++i) {
                        const int lr = 32 * sub + acc_row(i, h);
                        if (r0 + lr == srow && srow < a.n_stat) a.part2[srow] = x[i] + tf[lr];
                    }
                    continue;
                }
                if (MODE == M_LOGITS) {
#pragma unroll
                    for (int i = 0; i < 16; ++i) {
                        const int lr = 32 * sub + acc_row(i, h);
                        const int64_t item = r0 + lr;
                        if (item < a.n_strm && srow < a.n_stat) a.out[srow * a.ld_out + item] = x[i] + tf[lr];
                    }
                    continue;
                }
                // M_STATS: online (max, sum exp) over the lane's streamed rows + the target logit
                float tmax = -INFINITY;
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    x[i] += tf[32 * sub + acc_row(i, h)];
                    tmax = fmaxf(tmax, x[i]);
                }
                const int rel = s_tgt - (int)(r0 + 32 * sub);  // target in this sub-tile and lane half?
                if ((unsigned)rel < 32u && ((rel >> 2) & 1) == h) {
                    const int ri = (rel & 3) + 4 * (rel >> 3);
#pragma unroll
                    for (int i = 0; i < 16; ++i)
                        if (i == ri) t_logit = x[i];
                    have_t = true;
                }
                const float nm = fmaxf(run_max, tmax);
                if (nm != -INFINITY) {
                    float sum = 0.f;
#pragma unroll
                    for (int i = 0; i < 16; ++i) sum += __expf(x[i] - nm);
                    run_sum = run_sum * __expf(run_max - nm) + sum;
                    run_max = nm;
                }
            }
        }
        if (more) {
            if (threadIdx.x < kTS) {
                mf[(cur ^ 1) * kTS + threadIdx.x] = tm.f;
                mt[(cur ^ 1) * kTS + threadIdx.x] = tm.t;
            }
            wait_dma();
        }
        __syncthreads();
    }

    if (MODE == M_LOGITS || MODE == M_TSCORE) return;
    if (MODE == M_RANK) {
        r_cnt += __shfl_xor(r_cnt, 32, 64);  // the two lane halves hold different streamed rows of one query
        if (h == 0 && srow < a.n_stat && r_cnt) atomicAdd(a.counts + srow, r_cnt);
        return;
    }
    if (MODE == M_FDH) {
        run_sum += __shfl_xor(run_sum, 32, 64);  // (the halves share the running max)
        if (srow < a.n_stat) {
            if (h == 0) {
                a.part[((int64_t)chunk_id * a.n_stat + srow) * 2] = run_max;
                a.part[((int64_t)chunk_id * a.n_stat + srow) * 2 + 1] = run_sum;
            }
            if (have_t) a.part2[srow] = t_logit;
            float* dst = a.upart + ((int64_t)chunk_id * a.n_stat + srow) * a.d;
#pragma unroll
            for (int ft = 0; ft < NFT; ++ft)
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int f = 32 * ft + 8 * u + 4 * h;
                    if (f < a.d)
                        *reinterpret_cast<float4*>(dst + f) =
                            make_float4(y[ft][4 * u], y[ft][4 * u + 1], y[ft][4 * u + 2], y[ft][4 * u + 3]);
                }
        }
        return;
    }
    if (MODE == M_STATS) {
        // merge the two lane halves of each query (each holds its own streamed rows)
        const float m2 = __shfl_xor(run_max, 32, 64), s2 = __shfl_xor(run_sum, 32, 64);
        const float nm = fmaxf(run_max, m2);
        if (nm != -INFINITY) {
            run_sum = run_sum * __expf(run_max - nm) + s2 * __expf(m2 - nm);
            run_max = nm;
        }
        if (srow < a.n_stat) {
            if (h == 0) {
                a.part[((int64_t)chunk_id * a.n_stat + srow) * 2] = run_max;
                a.part[((int64_t)chunk_id * a.n_stat + srow) * 2 + 1] = run_sum;
            }
            if (have_t) a.part2[srow] = t_logit;
        }
        return;
    }
    const float scale = a.dloss[0] / a.stats[1];
    // lane (r32, h) holds Y^T[32 ft + 8 u + 4 h + (0..3)][r32] = gradient[srow][that feature], u = reg >> 2
    if (srow < a.n_stat) {
        float* dst = a.part + ((a.nchunks > 1 ? (int64_t)chunk_id * a.n_stat : 0) + srow) * a.d;
#pragma unroll
        for (int ft = 0; ft < NFT; ++ft)
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int f = 32 * ft + 8 * u + 4 * h;
                if (f < a.d)
                    *reinterpret_cast<float4*>(dst + f) =
                        make_float4(y[ft][4 * u] * scale, y[ft][4 * u + 1] * scale, y[ft][4 * u + 2] * scale,
                                    y[ft][4 * u + 3] * scale);
            }
    }
    if (MODE == M_DW && a.part2) {
        db += __shfl_xor(db, 32, 64);
        if (h == 0 && srow < a.n_stat) a.part2[(a.nchunks > 1 ? (int64_t)chunk_id * a.n_stat : 0) + srow] = db * scale;
    }
}

// ------------------------------------------------------------------------------------------------ gradient passes
// The gradient passes (dH, dW, fdh) as a two-stage software pipeline over the streamed tiles, three LDS buffers
// (144 KiB + metadata; one workgroup of 4 waves per CU):
//   iteration t:  DMA of tile t + 2 (issued first, waited for at the end of the iteration)
//                 [A] score product of tile t + 1 (16 steps of 6 MFMAs, row reads one step ahead)
//                     || P of tile t: exp, one-hot, the exact three-way bf16 split (a value pair per step)
//                 [B] gradient product of tile t (16 steps of 6 MFMAs, transposed reads one step ahead)
//                     || tile t + 1's scores prepared: + bias / - lse, one-hot bits, running max (a pair per step)
// Each step is its own scheduling region (sched_barrier) in which a dependent chain of six MFMAs takes the step's
// vector work and next step's reads into its shadow (at one wave per SIMD up to ~5 single-issue instructions per
// 32x32x16 MFMA hide, MI355X_MICROARCH.md).  The engine above ran the softmax VALU between the products and read
// its LDS operands just before use.
// The tile DMA is issued by inline assembly: with the compiler's LDS-DMA builtin in flight, every
// ds_read_b64_tr_b16 is preceded by s_waitcnt vmcnt(0) (the compiler cannot tell the buffers apart), which put the
// next tile's fetch on the critical path once per tile.  Completion is explicit: s_waitcnt vmcnt(0) in every
// issuing wave, then the workgroup barrier, before a buffer is read.  Products, sums and their order are those of
// the engine: results are bit-identical to it.
constexpr int kGradW = 4;
constexpr size_t kSmemGrad = 3 * kTile + 3 * kTS * 8;

// The tile's 12 wave-instructions of this wave in one asm block: wave-instruction i = plane / image-row group
// w = wave + 4 i lands at LDS byte w * 1 KiB of the buffer (plane w / 16 at 16 KiB, rows 4 (w % 16) at 1 KiB), so
// M0 starts at buf + 1 KiB * wave and steps by 4 KiB; it is saved and restored around the block.
static_assert(kTile / 1024 / kGradW == 12 && kPlaneTile == 16 * 1024, "dma_tile_asm: 12 x 1 KiB per wave");
__device__ __forceinline__ void dma_tile_asm(const __bf16* __restrict__ planes, int64_t pad, int64_t row0, char* buf) {
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const uint32_t base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)buf + 1024u * (uint32_t)wave;
    const __bf16* src[12];
#pragma unroll
    for (int i = 0; i < 12; ++i) {
        const int w = wave + kGradW * i;
        const int p = w / (kTS / 4), R = 4 * (w % (kTS / 4));
        const int row = R + (lane >> 4);
        const int ch = (lane & 15) ^ (((row & 3) << 2) | ((row >> 2) & 3));  // swz(): slot lane & 15 holds chunk ch
        src[i] = planes + (int64_t)p * pad * kDP + (row0 + row) * kDP + ch * 8;
    }
    uint32_t saved;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %13\n\t"
        "global_load_lds_dwordx4 %1, off\n\ts_add_u32 m0, m0, 4096\n\t"
        "global_load_lds_dwordx4 %2, off\n\ts_add_u32 m0, m0, 4096\n\t"
        "global_load_lds_dwordx4 %3, off\n\ts_add_u32 m0, m0, 4096\n\t"
        "global_load_lds_dwordx4 %4, off\n\ts_add_u32 m0, m0, 4096\n\t"
        "global_load_lds_dwordx4 %5, off\n\ts_add_u32 m0, m0, 4096\n\t"
        "global_load_lds_dwordx4 %6, off\n\ts_add_u32 m0, m0, 4096\n\t"
        "global_load_lds_dwordx4 %7, off\n\ts_add_u32 m0, m0, 4096\n\t"
        "global_load_lds_dwordx4 %8, off\n\ts_add_u32 m0, m0, 4096\n\t"
        "global_load_lds_dwordx4 %9, off\n\ts_add_u32 m0, m0, 4096\n\t"
        "global_load_lds_dwordx4 %10, off\n\ts_add_u32 m0, m0, 4096\n\t"
        "global_load_lds_dwordx4 %11, off\n\ts_add_u32 m0, m0, 4096\n\t"
        "global_load_lds_dwordx4 %12, off\n\ts_mov_b32 m0, %0"
        : "=&s"(saved)
        : "v"(src[0]), "v"(src[1]), "v"(src[2]), "v"(src[3]), "v"(src[4]), "v"(src[5]), "v"(src[6]), "v"(src[7]),
          "v"(src[8]), "v"(src[9]), "v"(src[10]), "v"(src[11]), "s"(__builtin_amdgcn_readfirstlane(base))
        : "memory", "scc");
}

typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
struct Bf3u {  // a Bf3 viewed as packed bf16 pairs
    u32x4v h, m, l;
};
// the exact three-way split (split_bf3) of one value pair into bf16 pair k of each plane
__device__ __forceinline__ void split_pair(float a, float b, Bf3u& P, int k) {
    typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
    const bf16x2 h = {(__bf16)a, (__bf16)b};
    const float ra = a - (float)h[0], rb = b - (float)h[1];
    const bf16x2 m = {(__bf16)ra, (__bf16)rb};
    const bf16x2 l = {(__bf16)(ra - (float)m[0]), (__bf16)(rb - (float)m[1])};
    P.h[k] = __builtin_bit_cast(uint32_t, h);
    P.m[k] = __builtin_bit_cast(uint32_t, m);
    P.l[k] = __builtin_bit_cast(uint32_t, l);
}
__device__ __forceinline__ Bf3 as_bf3(const Bf3u& u) {
    Bf3 b;
    b.h = __builtin_bit_cast(bf16x8, u.h);
    b.m = __builtin_bit_cast(bf16x8, u.m);
    b.l = __builtin_bit_cast(bf16x8, u.l);
    return b;
}

#ifndef ASME_LOGITS_SCHED
#define ASME_LOGITS_SCHED 0  // per-step sched_group_barrier pattern (MFMA, read, vector work)
#endif
// the step boundary: the next step's operand reads (issued above it) are not sunk below it (a compiler-level
// memory fence), and this step's MFMAs do not rise above it (their operand passes through the fence)
__device__ __forceinline__ void step_fence(Bf3& A) {
    asm volatile("" ::: "memory");
    asm volatile("" : "+v"(A.h), "+v"(A.m), "+v"(A.l));
}
// one MFMA, then up to R LDS reads and V vector instructions, six times: the step's schedule
template <int R, int V>
__device__ __forceinline__ void step_pattern() {
#if ASME_LOGITS_SCHED
#pragma unroll
    for (int m = 0; m < 6; ++m) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        if (R > 0) __builtin_amdgcn_sched_group_barrier(0x100, R, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, V, 0);
    }
#endif
}

template <int MODE, int KB>
__global__ __launch_bounds__(kGradW * 64) void logits_grad_kernel(LogitsArgs a) {
    constexpr int W = kGradW;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* bufs = smem;                                                  // 3 x kTile
    float* mf = reinterpret_cast<float*>(smem + 3 * kTile);            // 3 x kTS
    int* mt = reinterpret_cast<int*>(smem + 3 * kTile + 3 * kTS * 4);  // 3 x kTS
    constexpr int KS = 2 * KB;   // 16-k steps of the score product (per 32-row sub-tile)
    constexpr int NFT = KB;      // 32-feature tiles of the gradient product
    constexpr int NA = 2 * KS;   // stage-A steps (sub-tile, k step)
    constexpr int NB = 4 * NFT;  // stage-B steps (sub-tile, 16-row half, feature tile)
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, h = lane >> 5, r32 = lane & 31;
    int chunk_id;
    int64_t sblock;
    if (!work_item(a, chunk_id, sblock)) return;  // grid padding (whole workgroup)
    const int64_t srow = sblock * (32 * W) + wave * 32 + r32;  // this lane's stationary row (MFMA column)
    // (M_TSCORE: the streamed rows are the stationary block's own gathered target rows)
    const int64_t s_begin = MODE == M_TSCORE ? sblock * (32 * W) : (int64_t)chunk_id * a.chunk;
    const int64_t s_end = std::min(a.strm_pad, s_begin + (MODE == M_TSCORE ? 32 * W : a.chunk));  // past n_strm: zero planes
    const int ntiles = (int)((s_end - s_begin) / kTS);

    // stationary fragments, loaded straight into AGPRs (the MFMAs read their B operand there): the 256
    // architectural VGPRs are left to the scores, P, the prefetched operands and the addresses
    Bf3 st[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
        const __bf16* o = a.stat + srow * kDP + 16 * ks + 8 * h;
        asm volatile("global_load_dwordx4 %0, %1, off" : "=a"(st[ks].h) : "v"(o) : "memory");
        asm volatile("global_load_dwordx4 %0, %1, off" : "=a"(st[ks].m) : "v"(o + a.stat_pad * kDP) : "memory");
        asm volatile("global_load_dwordx4 %0, %1, off" : "=a"(st[ks].l) : "v"(o + 2 * a.stat_pad * kDP) : "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    float s_lse = 0.f, s_bias = 0.f;
    int s_tgt = -1;
    if (MODE == M_DH || MODE == M_FDH) {
        const int64_t tg = srow < a.n_stat ? a.targets[srow] : -1;
        const bool ok = srow < a.n_stat && valid_target(tg, a.ignore, a.V);
        s_tgt = ok ? (int)tg : -1;
        if (MODE == M_DH) s_lse = ok ? a.lse[srow] : INFINITY;  // ignored / padding queries: P = 0
    } else {
        s_bias = srow < a.n_stat ? (a.bias ? a.bias[srow] : 0.f) : -INFINITY;
        s_tgt = (int)srow;  // compare the streamed query's target against this item
    }
    float run_max = -INFINITY, run_sum = 0.f, t_logit = 0.f, base = 0.f;
    bool have_t = false;
    floatx16 y[NFT];
#pragma unroll
    for (int f = 0; f < NFT; ++f)
#pragma unroll
        for (int i = 0; i < 16; ++i) y[f][i] = 0.f;
    float db = 0.f;

    auto score_a = [&](const char* buf, int sub, int ks) {
        const int off = swz(32 * sub + r32, 2 * ks + h);
        Bf3 A;
        A.h = lds_b128(buf, off);
        A.m = lds_b128(buf + kPlaneTile, off);
        A.l = lds_b128(buf + 2 * kPlaneTile, off);
        return A;
    };
    auto grad_a = [&](const char* buf, int sub, int s2, int ft) {
        const int fh = (lane >> 4) & 1, q = (lane & 15) >> 2, p4 = lane & 3;
        const int rlo = 32 * sub + 16 * s2 + 4 * h + q, rhi = rlo + 8;
        const int ch = 4 * ft + 2 * fh + (p4 >> 1);
        const int olo = swz(rlo, ch) + 8 * (p4 & 1), ohi = swz(rhi, ch) + 8 * (p4 & 1);
        Bf3 A;
        A.h = cat8(lds_tr(buf, olo), lds_tr(buf, ohi));
        A.m = cat8(lds_tr(buf + kPlaneTile, olo), lds_tr(buf + kPlaneTile, ohi));
        A.l = cat8(lds_tr(buf + 2 * kPlaneTile, olo), lds_tr(buf + 2 * kPlaneTile, ohi));
        return A;
    };

    TileMeta tm;
    auto stage = [&](int slot, int64_t r0) {  // tile at streamed row r0 into buffer slot: metadata load + DMA
        if (threadIdx.x < kTS) tm.load(MODE, a, r0 + threadIdx.x);
        dma_tile_asm(a.strm, a.strm_pad, r0, bufs + slot * kTile);
    };
    auto stage_meta = [&](int slot) {
        if (threadIdx.x < kTS) {
            mf[slot * kTS + threadIdx.x] = tm.f;
            mt[slot * kTS + threadIdx.x] = tm.t;
        }
    };

    // scores of the current tile (xs) and of the next (xn); value v = 16 sub + i is streamed row
    // 32 sub + acc_row(i, h); oh / ohn: the one-hot bits (dH, dW)
    floatx16 xs[2], xn[2];
#pragma unroll
    for (int i = 0; i < 16; ++i) xs[0][i] = xs[1][i] = xn[0][i] = xn[1][i] = 0.f;
    uint32_t oh = 0u, ohn = 0u;
    float tmax = -INFINITY;
    // prepare value pair p (values 2p, 2p + 1) of the scores x of the tile at streamed row r0 from the pair's
    // metadata (read one step ahead of its use: a read just before its use would wait for the step's prefetched
    // transposed reads too)
    struct PairMeta {
        float2 f;
        int2 t;
    };
    auto load_meta = [&](int slot, int p) {
        const int lr = 32 * (p >> 3) + acc_row(2 * (p & 7), h);  // rows lr, lr + 1
        PairMeta m;
        m.f = *reinterpret_cast<const float2*>(mf + slot * kTS + lr);
        if (MODE == M_DW) m.t = *reinterpret_cast<const int2*>(mt + slot * kTS + lr);
        return m;
    };
    auto prep_pair = [&](floatx16 (&x)[2], uint32_t& bits, const PairMeta& m, int64_t r0, int p) {
        const int sub = p >> 3, i0 = 2 * (p & 7);
        const int lr = 32 * sub + acc_row(i0, h);
        if constexpr (MODE == M_FDH) {
            x[sub][i0] += m.f.x;
            x[sub][i0 + 1] += m.f.y;
            tmax = fmaxf(tmax, fmaxf(x[sub][i0], x[sub][i0 + 1]));
        } else if constexpr (MODE == M_DH) {
            x[sub][i0] = x[sub][i0] + m.f.x - s_lse;
            x[sub][i0 + 1] = x[sub][i0 + 1] + m.f.y - s_lse;
            bits |= ((int64_t)s_tgt == r0 + lr ? 1u : 0u) << (2 * p);
            bits |= ((int64_t)s_tgt == r0 + lr + 1 ? 1u : 0u) << (2 * p + 1);
        } else {
            x[sub][i0] = x[sub][i0] + s_bias - m.f.x;
            x[sub][i0 + 1] = x[sub][i0 + 1] + s_bias - m.f.y;
            bits |= (m.t.x == s_tgt ? 1u : 0u) << (2 * p);
            bits |= (m.t.y == s_tgt ? 1u : 0u) << (2 * p + 1);
        }
    };
    // fdh, after a tile's scores are prepared: the target logit, the running max (lazy rescale: the reference max
    // moves only when a tile's max passes it by more than 8, so P = exp(s - ref) <= e^8), the exp base
    auto fdh_post = [&](const floatx16 (&x)[2], int64_t r0) {
#pragma unroll
        for (int sub = 0; sub < 2; ++sub) {
            const int rel = s_tgt - (int)(r0 + 32 * sub);  // target in this sub-tile and lane half?
            if ((unsigned)rel < 32u && ((rel >> 2) & 1) == h) {
                const int ri = (rel & 3) + 4 * (rel >> 3);
#pragma unroll
                for (int i = 0; i < 16; ++i)
                    if (i == ri) t_logit = x[sub][i];
                have_t = true;
            }
        }
        const float tm2 = fmaxf(tmax, __shfl_xor(tmax, 32, 64));  // one running max per query over both halves
        tmax = -INFINITY;
        if (__ballot(!(tm2 <= run_max + 8.f)) != 0ull) {
            const float nm = fmaxf(run_max, tm2);
            const float alpha = run_max == -INFINITY ? 0.f : __expf(run_max - nm);
#pragma unroll
            for (int f = 0; f < NFT; ++f)
#pragma unroll
                for (int i = 0; i < 16; ++i) y[f][i] *= alpha;
            run_sum *= alpha;
            run_max = nm;
        }
        base = run_max == -INFINITY ? 0.f : run_max;  // nothing finite yet: P = 0, no NaN
    };
    // P value pair p of the current tile into the split B fragments
    Bf3u P[2][2];
    auto p_pair = [&](int p) {
        const int sub = p >> 3, i0 = 2 * (p & 7), s2 = i0 >> 3, k = (i0 & 7) >> 1;
        float v0 = xs[sub][i0], v1 = xs[sub][i0 + 1];
        if constexpr (MODE == M_FDH) {
            v0 = __expf(v0 - base);
            v1 = __expf(v1 - base);
            run_sum += v0;
            run_sum += v1;
        } else {
            v0 = __expf(v0) - (float)((oh >> (2 * p)) & 1u);
            v1 = __expf(v1) - (float)((oh >> (2 * p + 1)) & 1u);
            if (MODE == M_DW) {
                db += v0;
                db += v1;
            }
        }
        split_pair(v0, v1, P[sub][s2], k);
    };

    if (ntiles > 0) {
        stage(0, s_begin);
        stage_meta(0);
        if (ntiles > 1) {
            stage(1, s_begin + kTS);
            stage_meta(1);
        }
        wait_dma();
        __syncthreads();
#pragma unroll
        for (int sub = 0; sub < 2; ++sub)
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) xs[sub] = mfma32_bf3(score_a(bufs, sub, ks), st[ks], xs[sub]);
#pragma unroll
        for (int p = 0; p < 16; ++p) prep_pair(xs, oh, load_meta(0, p), s_begin, p);
        if constexpr (MODE == M_FDH) fdh_post(xs, s_begin);
    }
    int cur = 0;
    for (int it = 0; it < ntiles; ++it) {
        const int nxt = cur == 2 ? 0 : cur + 1, nn = nxt == 2 ? 0 : nxt + 1;
        const bool has_next = it + 1 < ntiles, has_nn = it + 2 < ntiles;
        const int64_t r0 = s_begin + (int64_t)it * kTS;
        if (has_nn) stage(nn, r0 + 2 * kTS);
        const char* buf = bufs + cur * kTile;
        __builtin_amdgcn_sched_barrier(0);
        // stage A
#pragma unroll
        for (int i = 0; i < 16; ++i) xn[0][i] = xn[1][i] = 0.f;
        ohn = 0u;
        if (has_next) {
            const char* nbuf = bufs + nxt * kTile;
            Bf3 A = score_a(nbuf, 0, 0);
#pragma unroll
            for (int s = 0; s < NA; ++s) {
                const int sub = s / KS, ks = s % KS;
                Bf3 An = A;
                if (s + 1 < NA) An = score_a(nbuf, (s + 1) / KS, (s + 1) % KS);
                step_fence(A);
                xn[sub] = mfma32_bf3(A, st[ks], xn[sub]);
#pragma unroll
                for (int p = s * 16 / NA; p < (s + 1) * 16 / NA; ++p) p_pair(p);
                step_pattern<1, 4>();
                A = An;
            }
        } else {
#pragma unroll
            for (int p = 0; p < 16; ++p) p_pair(p);
        }
        // stage B
        {
            Bf3 A = grad_a(buf, 0, 0, 0);
            const int64_t r1 = r0 + kTS;
            constexpr int MP = (16 + NB - 1) / NB;  // most pairs per step
            PairMeta cm[MP], nm[MP];
#pragma unroll
            for (int p = 0; p < 16 / NB; ++p) cm[p] = load_meta(nxt, p);
#pragma unroll
            for (int s = 0; s < NB; ++s) {
                const int sub = s / (2 * NFT), s2 = (s / NFT) % 2, ft = s % NFT;
                const int plo = s * 16 / NB, phi = (s + 1) * 16 / NB, nhi = (s + 2) * 16 / NB;
#pragma unroll
                for (int p = phi; p < nhi && s + 1 < NB; ++p) nm[p - phi] = load_meta(nxt, p);
                Bf3 An = A;
                if (s + 1 < NB) An = grad_a(buf, (s + 1) / (2 * NFT), ((s + 1) / NFT) % 2, (s + 1) % NFT);
                step_fence(A);
                y[ft] = mfma32_bf3(A, as_bf3(P[sub][s2]), y[ft]);
                // (on the last tile this prepares stale values that are never used: no branch in the chain)
#pragma unroll
                for (int p = plo; p < phi; ++p) prep_pair(xn, ohn, cm[p - plo], r1, p);
#pragma unroll
                for (int p = 0; p < MP; ++p) cm[p] = nm[p];
                step_pattern<1, 3>();
                A = An;
            }
        }
        if constexpr (MODE == M_FDH) {
            if (has_next) fdh_post(xn, r0 + kTS);
        }
        xs[0] = xn[0];
        xs[1] = xn[1];
        oh = ohn;
        if (has_nn) stage_meta(nn);
        wait_dma();
        __syncthreads();
        cur = nxt;
    }

    if (MODE == M_FDH) {
        run_sum += __shfl_xor(run_sum, 32, 64);  // (the halves share the running max)
        if (srow < a.n_stat) {
            if (h == 0) {
                a.part[((int64_t)chunk_id * a.n_stat + srow) * 2] = run_max;
                a.part[((int64_t)chunk_id * a.n_stat + srow) * 2 + 1] = run_sum;
            }
            if (have_t) a.part2[srow] = t_logit;
            float* dst = a.upart + ((int64_t)chunk_id * a.n_stat + srow) * a.d;
#pragma unroll
            for (int ft = 0; ft < NFT; ++ft)
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int f = 32 * ft + 8 * u + 4 * h;
                    if (f < a.d)
                        *reinterpret_cast<float4*>(dst + f) =
                            make_float4(y[ft][4 * u], y[ft][4 * u + 1], y[ft][4 * u + 2], y[ft][4 * u + 3]);
                }
        }
        return;
    }
    const float scale = a.dloss[0] / a.stats[1];
    if (srow < a.n_stat) {
        float* dst = a.part + ((a.nchunks > 1 ? (int64_t)chunk_id * a.n_stat : 0) + srow) * a.d;
#pragma unroll
        for (int ft = 0; ft < NFT; ++ft)
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int f = 32 * ft + 8 * u + 4 * h;
                if (f < a.d)
                    *reinterpret_cast<float4*>(dst + f) =
                        make_float4(y[ft][4 * u] * scale, y[ft][4 * u + 1] * scale, y[ft][4 * u + 2] * scale,
                                    y[ft][4 * u + 3] * scale);
            }
    }
    if (MODE == M_DW && a.part2) {
        db += __shfl_xor(db, 32, 64);
        if (h == 0 && srow < a.n_stat) a.part2[(a.nchunks > 1 ? (int64_t)chunk_id * a.n_stat : 0) + srow] = db * scale;
    }
}

// one block: lse[q] = merge of the chunks; out[0] = mean over valid rows of lse - s_t (NaN if none), out[1] = count
// The forward's finish, in two launches (one 1,024-thread block had merged every row's chunk partials alone:
// 0.19 ms per C3 step for 37k rows x 53 chunks): lce_rows_kernel merges each row's partials into its lse and sums
// its block's (loss, count) in a fixed tree; lce_finish_kernel adds the block sums in a fixed order.
constexpr int kLceRows = 256;
__global__ __launch_bounds__(kLceRows) void lce_rows_kernel(const float* __restrict__ part, int64_t n, int nchunks,
                                                            const int64_t* __restrict__ targets, int64_t ignore,
                                                            int64_t V, const float* __restrict__ tlogit,
                                                            float* __restrict__ lse, float* __restrict__ bsum) {
    __shared__ float sa[kLceRows], sc[kLceRows];
    const int64_t q = (int64_t)blockIdx.x * kLceRows + threadIdx.x;
    float acc = 0.f, cnt = 0.f;
    if (q < n) {
        float m = -INFINITY, s = 0.f;
        for (int k = 0; k < nchunks; ++k) {
            const float m2 = part[((int64_t)k * n + q) * 2], s2 = part[((int64_t)k * n + q) * 2 + 1];
            const float nm = fmaxf(m, m2);
            if (nm == -INFINITY) continue;
            s = s * __expf(m - nm) + s2 * __expf(m2 - nm);
            m = nm;
        }
        const float l = m + logf(s);
        lse[q] = l;
        if (valid_target(targets[q], ignore, V)) {
            acc = l - tlogit[q];
            cnt = 1.f;
        }
    }
    sa[threadIdx.x] = acc;
    sc[threadIdx.x] = cnt;
    __syncthreads();
    for (int h = kLceRows / 2; h > 0; h >>= 1) {
        if (threadIdx.x < h) {
            sa[threadIdx.x] += sa[threadIdx.x + h];
            sc[threadIdx.x] += sc[threadIdx.x + h];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        bsum[2 * blockIdx.x] = sa[0];
        bsum[2 * blockIdx.x + 1] = sc[0];
    }
}
__global__ __launch_bounds__(1024) void lce_finish_kernel(const float* __restrict__ bsum, int64_t nblocks,
                                                          float* __restrict__ out) {
    __shared__ float sa[1024], sc[1024];
    float acc = 0.f, cnt = 0.f;
    for (int64_t q = threadIdx.x; q < nblocks; q += blockDim.x) {
        acc += bsum[2 * q];
        cnt += bsum[2 * q + 1];
    }
    sa[threadIdx.x] = acc;
    sc[threadIdx.x] = cnt;
    __syncthreads();
    for (int h = blockDim.x / 2; h > 0; h >>= 1) {
        if (threadIdx.x < h) {
            sa[threadIdx.x] += sa[threadIdx.x + h];
            sc[threadIdx.x] += sc[threadIdx.x + h];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        out[0] = sa[0] / sc[0];
        out[1] = sc[0];
    }
}

// out[i] = sum_{c < nparts} part[c * stride + i] (fixed order)
__global__ __launch_bounds__(256) void sum_parts_kernel(const float* __restrict__ part, int64_t stride, int nparts,
                                                        int64_t count, float* __restrict__ out) {
    const int64_t i4 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
    if (i4 >= count) return;
    if (i4 + 4 <= count) {
        float4 s = *reinterpret_cast<const float4*>(part + i4);
        for (int c = 1; c < nparts; ++c) {
            const float4 v = *reinterpret_cast<const float4*>(part + c * stride + i4);
            s.x += v.x;
            s.y += v.y;
            s.z += v.z;
            s.w += v.w;
        }
        *reinterpret_cast<float4*>(out + i4) = s;
    } else {
        for (int64_t i = i4; i < count; ++i) {
            float s = part[i];
            for (int c = 1; c < nparts; ++c) s += part[c * stride + i];
            out[i] = s;
        }
    }
}

// fdh finish: one wave per query (lane c holds chunk c's (max, sum); chunks <= 64): lse, the query's loss term into
// its block's (loss, count) pair (fixed-order tree, then lce_finish_kernel), and
// dH_raw[q] = sum_c e^(m_c - M) U_c[q] / S - W[t_q]  (0 for an ignored or padding row)
constexpr int kFdhWaves = 4;
__global__ __launch_bounds__(kFdhWaves * 64) void fdh_finish_kernel(
    const float* __restrict__ part, const float* __restrict__ upart, int64_t n, int nchunks, int d,
    const int64_t* __restrict__ targets, int64_t ignore, int64_t V, const float* __restrict__ tlogit,
    const float* __restrict__ W, int64_t ld_w, float* __restrict__ lse, float* __restrict__ dh_raw, int64_t ld_dh,
    float* __restrict__ bsum) {
    __shared__ float sa[kFdhWaves], sc[kFdhWaves];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t q = (int64_t)blockIdx.x * kFdhWaves + wave;
    float acc_loss = 0.f, cnt = 0.f;
    if (q < n) {
        const float mc = lane < nchunks ? part[((int64_t)lane * n + q) * 2] : -INFINITY;
        const float scv = lane < nchunks ? part[((int64_t)lane * n + q) * 2 + 1] : 0.f;
        float M = mc;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) M = fmaxf(M, __shfl_xor(M, o, 64));
        const float w = (mc == -INFINITY || M == -INFINITY) ? 0.f : __expf(mc - M);
        float S = scv * w;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) S += __shfl_xor(S, o, 64);
        const float l = M + logf(S);
        const int64_t tg = targets[q];
        const bool ok = valid_target(tg, ignore, V);
        if (lane == 0) {
            lse[q] = l;
            if (ok) {
                acc_loss = l - tlogit[q];
                cnt = 1.f;
            }
        }
        const float inv = 1.f / S;
        for (int f = 2 * lane; f < d; f += 128) {
            float2 u = make_float2(0.f, 0.f);
            for (int c = 0; c < nchunks; ++c) {
                const float wc = __shfl(w, c, 64);
                const float2 v = *reinterpret_cast<const float2*>(upart + ((int64_t)c * n + q) * d + f);
                u.x += wc * v.x;
                u.y += wc * v.y;
            }
            float2 r = make_float2(0.f, 0.f);
            if (ok) {
                const float2 wt = *reinterpret_cast<const float2*>(W + tg * ld_w + f);
                r = make_float2(u.x * inv - wt.x, u.y * inv - wt.y);
            }
            *reinterpret_cast<float2*>(dh_raw + q * ld_dh + f) = r;
        }
    }
    if (lane == 0) {
        sa[wave] = acc_loss;
        sc[wave] = cnt;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float a0 = 0.f, c0 = 0.f;
#pragma unroll
        for (int k = 0; k < kFdhWaves; ++k) {
            a0 += sa[k];
            c0 += sc[k];
        }
        bsum[2 * blockIdx.x] = a0;
        bsum[2 * blockIdx.x + 1] = c0;
    }
}

// dH = dH_raw * dloss[0] / stats[1] (the mean's upstream gradient over the valid-row count)
__global__ __launch_bounds__(256) void scale_rows_kernel(const float* __restrict__ src, int64_t count,
                                                         const float* __restrict__ dloss, const float* __restrict__ stats,
                                                         float* __restrict__ dst) {
    const int64_t i4 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
    if (i4 >= count) return;
    const float sc = dloss[0] / stats[1];
    const float4 v = *reinterpret_cast<const float4*>(src + i4);
    *reinterpret_cast<float4*>(dst + i4) = make_float4(v.x * sc, v.y * sc, v.z * sc, v.w * sc);
}

// ------------------------------------------------------------------------------------------------ host
constexpr size_t kSmem = 2 * kTile + 2 * kTS * 8;

// chunks of the streamed operand: a multiple of 8 (one set per XCD) when there is enough work, each a whole
// number of tiles; the stationary blocks times the chunks give the grid
struct Plan {
    int64_t stat_pad, strm_pad, sblocks, chunk;
    int nchunks;
};
template <int MODE>
Plan make_plan(int64_t n_stat, int64_t n_strm, int cus, int64_t chunk_cap = 64) {
    Plan p;
    p.stat_pad = pad_rows(std::max<int64_t>(n_stat, 1));
    p.strm_pad = pad_rows(std::max<int64_t>(n_strm, 1));
    p.sblocks = p.stat_pad / (32 * EngineWaves<MODE>::W);
    const int64_t tiles = p.strm_pad / kTS;
    // one workgroup per CU at a time (96 KiB of LDS): pick the chunk count whose grid fills its last round best
    // (the workgroups of a round take about equally long), preferring multiples of 8 (a chunk per XCD, its tiles
    // shared in that XCD's L2) at equal fill; chunks of at least 4 tiles
    const int64_t max_chunks = std::max<int64_t>(1, std::min<int64_t>(tiles / 4, chunk_cap));
    double best = -1.0;
    p.chunk = tiles * kTS;
    for (int64_t want = 1; want <= max_chunks; ++want) {
        const int64_t chunk = (tiles + want - 1) / want;
        const int64_t nch = (tiles + chunk - 1) / chunk;
        const int64_t wgs = p.sblocks * nch;
        if (wgs < cus && want < max_chunks) continue;  // fewer workgroups than CUs: keep splitting
        const int64_t rounds = (wgs + cus - 1) / cus;
        // fill of the CU-rounds, minus a small cost per round (per-workgroup prologue / epilogue, partial slabs)
        const double score = (double)wgs / (double)(rounds * cus) + (nch % 8 == 0 ? 0.02 : 0.0) - 0.002 * rounds;
        if (score > best) {
            best = score;
            p.chunk = chunk * kTS;
        }
    }
    p.nchunks = (int)((p.strm_pad + p.chunk - 1) / p.chunk);
    return p;
}

int device_cus() {
    int dev = 0, cus = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    return cus;
}

int64_t planes_bytes(int64_t rows) { return 3 * pad_rows(std::max<int64_t>(rows, 1)) * kDP * 2; }

int split(const float* X, int64_t ld, int64_t rows, int d, __bf16* planes, hipStream_t s) {
    const int64_t pad = pad_rows(std::max<int64_t>(rows, 1));
    const int64_t threads = pad * (kDP / 8);
    hipLaunchKernelGGL(split_planes_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, X, ld, rows, d,
                       pad, planes);
    return hip_status(hipGetLastError(), "logits: split");
}

#ifndef ASME_LOGITS_XTILE
#define ASME_LOGITS_XTILE 1  // gradient passes on logits_grad_kernel (0: the single-stage engine, for A/B)
#endif
template <int MODE>
constexpr bool kGradKernel = ASME_LOGITS_XTILE && ASME_LOGITS_DIAG == 0 && (MODE == M_DH || MODE == M_DW || MODE == M_FDH);

template <int MODE, int KB>
int launch_engine(const LogitsArgs& a, int64_t sblocks, hipStream_t s) {
    LogitsArgs g = a;
    g.sblocks = sblocks;
    g.per_xcd = (sblocks * a.nchunks + 7) / 8;  // grid = 8 per_xcd workgroups (work_item)
    if constexpr (kGradKernel<MODE>) {
        static const hipError_t attr = hipFuncSetAttribute((const void*)logits_grad_kernel<MODE, KB>,
                                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)kSmemGrad);
        if (attr != hipSuccess) return hip_status(attr, "logits: LDS opt-in");
        static_assert(EngineWaves<MODE>::W == kGradW, "the plan's stationary blocks are kGradW waves");
        hipLaunchKernelGGL((logits_grad_kernel<MODE, KB>), dim3((unsigned)(8 * g.per_xcd)), dim3(kGradW * 64),
                           kSmemGrad, s, g);
        return hip_status(hipGetLastError(), "logits: gradient pass");
    }
    // LDS opt-in once per instantiation (a function-local static: thread-safe initialisation)
    static const hipError_t attr = hipFuncSetAttribute(
        (const void*)logits_engine_kernel<MODE, KB, EngineWaves<MODE>::W>, hipFuncAttributeMaxDynamicSharedMemorySize,
        (int)kSmem);
    if (attr != hipSuccess) return hip_status(attr, "logits: LDS opt-in");
    constexpr int W = EngineWaves<MODE>::W;
    hipLaunchKernelGGL((logits_engine_kernel<MODE, KB, W>), dim3((unsigned)(8 * g.per_xcd)), dim3(W * 64), kSmem, s,
                       g);
    return hip_status(hipGetLastError(), "logits: engine");
}

template <int MODE>
int launch_kb(const LogitsArgs& a, int64_t sblocks, hipStream_t s) {
    switch ((a.d + 31) / 32) {
        case 1: return launch_engine<MODE, 1>(a, sblocks, s);
        case 2: return launch_engine<MODE, 2>(a, sblocks, s);
        case 3: return launch_engine<MODE, 3>(a, sblocks, s);
        default: return launch_engine<MODE, 4>(a, sblocks, s);
    }
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

int64_t align256(int64_t b) { return (b + 255) / 256 * 256; }

}  // namespace

// ---------------------------------------------------------------------------------------- fused CE, forward
ASME_API int64_t asme_linear_xent_fwd_workspace(int64_t n, int64_t V, int64_t dim) {
    (void)dim;
    const Plan p = make_plan<M_STATS>(n, V, device_cus());
    return align256(planes_bytes(n)) + align256(planes_bytes(V)) + align256(p.nchunks * n * 2 * 4) + align256(n * 4) +
           align256(((n + kLceRows - 1) / kLceRows) * 2 * 4 + 8);
}

// lse[q] (n) and out = {mean loss over the valid rows, their count}; H (n x dim), W (V x dim), dim <= 128
ASME_API int asme_linear_xent_fwd(const float* H, int64_t ld_h, int64_t n, int64_t dim, const float* W, int64_t ld_w,
                                  int64_t V, const float* bias, const int64_t* targets, int64_t ignore_index,
                                  float* lse, float* workspace, int64_t ws_bytes, float* out, void* stream) {
    ASME_CHECK_ARG(H && W && targets && lse && workspace && out, "asme_linear_xent_fwd: null pointer");
    ASME_CHECK_ARG(dim >= 4 && dim <= kDP && dim % 4 == 0 && ld_h % 4 == 0 && ld_w % 4 == 0 && aligned16(H) &&
                       aligned16(W),
                   "asme_linear_xent_fwd: dim must be a multiple of 4 in [4, 128], rows 16-B aligned");
    ASME_CHECK_ARG(n >= 0 && V >= 1 && V < (1LL << 31), "asme_linear_xent_fwd: bad shape");
    ASME_CHECK_ARG(ws_bytes >= asme_linear_xent_fwd_workspace(n, V, dim), "asme_linear_xent_fwd: workspace too small");
    hipStream_t s = (hipStream_t)stream;
    const Plan p = make_plan<M_STATS>(n, V, device_cus());
    char* w = reinterpret_cast<char*>(workspace);
    __bf16* hp = reinterpret_cast<__bf16*>(w);
    __bf16* wp = reinterpret_cast<__bf16*>(w + align256(planes_bytes(n)));
    float* part = reinterpret_cast<float*>(w + align256(planes_bytes(n)) + align256(planes_bytes(V)));
    float* tlogit = part + align256(p.nchunks * n * 2 * 4) / 4;
    if (n > 0) {
        int rc = split(H, ld_h, n, (int)dim, hp, s);
        if (rc == 0) rc = split(W, ld_w, V, (int)dim, wp, s);
        if (rc != 0) return rc;
        LogitsArgs a{};
        a.stat = hp;
        a.strm = wp;
        a.stat_pad = p.stat_pad;
        a.strm_pad = p.strm_pad;
        a.n_stat = n;
        a.n_strm = V;
        a.chunk = p.chunk;
        a.nchunks = p.nchunks;
        a.d = (int)dim;
        a.bias = bias;
        a.targets = targets;
        a.ignore = ignore_index;
        a.V = V;
        a.part = part;
        a.part2 = tlogit;
        rc = launch_kb<M_STATS>(a, p.sblocks, s);
        if (rc != 0) return rc;
    }
    float* bsum = tlogit + align256(n * 4) / 4;
    const int64_t nb = (n + kLceRows - 1) / kLceRows;
    if (nb > 0)
        hipLaunchKernelGGL(lce_rows_kernel, dim3((unsigned)nb), dim3(kLceRows), 0, s, part, n, p.nchunks, targets,
                           ignore_index, V, tlogit, lse, bsum);
    hipLaunchKernelGGL(lce_finish_kernel, dim3(1), dim3(1024), 0, s, bsum, nb, out);
    ASME_LAUNCH_CHECK("asme_linear_xent_fwd");
}

// --------------------------------------------------------------------------------------- fused CE, backward
ASME_API int64_t asme_linear_xent_bwd_workspace(int64_t n, int64_t V, int64_t dim) {
    const int cus = device_cus();
    const Plan ph = make_plan<M_DH>(n, V, cus), pw = make_plan<M_DW>(V, n, cus);
    const int64_t dh = ph.nchunks > 1 ? ph.nchunks * n * dim : 0;
    const int64_t dw = pw.nchunks > 1 ? pw.nchunks * V * (dim + 1) : 0;
    return align256(planes_bytes(n)) + align256(planes_bytes(V)) + align256(dh * 4) + align256(dw * 4);
}

// dH (n x dim), dW (V x dim), db (V, nullable) are overwritten (not accumulated)
ASME_API int asme_linear_xent_bwd(const float* H, int64_t ld_h, int64_t n, int64_t dim, const float* W, int64_t ld_w,
                                  int64_t V, const float* bias, const int64_t* targets, int64_t ignore_index,
                                  const float* lse, const float* stats, const float* dloss, float* dH, float* dW,
                                  float* db, float* workspace, int64_t ws_bytes, void* stream) {
    ASME_CHECK_ARG(H && W && targets && lse && stats && dloss && dH && dW, "asme_linear_xent_bwd: null pointer");
    ASME_CHECK_ARG(dim >= 4 && dim <= kDP && dim % 4 == 0 && ld_h % 4 == 0 && ld_w % 4 == 0 && aligned16(H) &&
                       aligned16(W) && aligned16(dH) && aligned16(dW),
                   "asme_linear_xent_bwd: dim must be a multiple of 4 in [4, 128], rows 16-B aligned");
    ASME_CHECK_ARG(V >= 1 && V < (1LL << 31), "asme_linear_xent_bwd: bad shape");
    ASME_CHECK_ARG(ws_bytes >= asme_linear_xent_bwd_workspace(n, V, dim), "asme_linear_xent_bwd: workspace too small");
    hipStream_t s = (hipStream_t)stream;
    if (n == 0) {
        if (hipMemsetAsync(dW, 0, V * dim * sizeof(float), s) != hipSuccess ||
            (db && hipMemsetAsync(db, 0, V * sizeof(float), s) != hipSuccess))
            return hip_status(hipGetLastError(), "asme_linear_xent_bwd");
        return 0;
    }
    const int cus = device_cus();
    const Plan ph = make_plan<M_DH>(n, V, cus), pw = make_plan<M_DW>(V, n, cus);
    char* w = reinterpret_cast<char*>(workspace);
    __bf16* hp = reinterpret_cast<__bf16*>(w);
    __bf16* wp = reinterpret_cast<__bf16*>(w + align256(planes_bytes(n)));
    float* dh_part = reinterpret_cast<float*>(w + align256(planes_bytes(n)) + align256(planes_bytes(V)));
    const int64_t dh_elems = ph.nchunks > 1 ? ph.nchunks * n * dim : 0;
    float* dw_part = dh_part + align256(dh_elems * 4) / 4;
    float* db_part = dw_part + (pw.nchunks > 1 ? pw.nchunks * V * dim : 0);
    int rc = split(H, ld_h, n, (int)dim, hp, s);
    if (rc == 0) rc = split(W, ld_w, V, (int)dim, wp, s);
    if (rc != 0) return rc;
    LogitsArgs a{};
    a.d = (int)dim;
    a.bias = bias;
    a.targets = targets;
    a.ignore = ignore_index;
    a.V = V;
    a.lse = lse;
    a.dloss = dloss;
    a.stats = stats;
    // dH: queries stationary, items streamed
    a.stat = hp;
    a.strm = wp;
    a.stat_pad = ph.stat_pad;
    a.strm_pad = ph.strm_pad;
    a.n_stat = n;
    a.n_strm = V;
    a.chunk = ph.chunk;
    a.nchunks = ph.nchunks;
    a.part = ph.nchunks > 1 ? dh_part : dH;
    a.part2 = nullptr;
    rc = launch_kb<M_DH>(a, ph.sblocks, s);
    if (rc != 0) return rc;
    // dW, db: items stationary, queries streamed
    a.stat = wp;
    a.strm = hp;
    a.stat_pad = pw.stat_pad;
    a.strm_pad = pw.strm_pad;
    a.n_stat = V;
    a.n_strm = n;
    a.chunk = pw.chunk;
    a.nchunks = pw.nchunks;
    a.part = pw.nchunks > 1 ? dw_part : dW;
    a.part2 = pw.nchunks > 1 ? (db ? db_part : nullptr) : db;
    rc = launch_kb<M_DW>(a, pw.sblocks, s);
    if (rc != 0) return rc;
    auto sum = [&](const float* part, int64_t stride, int64_t nparts, int64_t count, float* out) {
        const int64_t thr = (count + 3) / 4;
        hipLaunchKernelGGL(sum_parts_kernel, dim3((unsigned)((thr + 255) / 256)), dim3(256), 0, s, part, stride,
                           (int)nparts, count, out);
    };
    if (ph.nchunks > 1) sum(dh_part, n * dim, ph.nchunks, n * dim, dH);
    if (pw.nchunks > 1) {
        sum(dw_part, V * dim, pw.nchunks, V * dim, dW);
        if (db) sum(db_part, V, pw.nchunks, V, db);
    }
    ASME_LAUNCH_CHECK("asme_linear_xent_bwd");
}

// ------------------------------------------------- fused CE with dH in the forward (training), dW in the backward
// fdh's per-chunk U slabs cost 2 n d 4 B each (written, then merged): at most kFdhChunks chunks
constexpr int64_t kFdhChunks = 8;

ASME_API int64_t asme_linear_xent_fwd_dh_workspace(int64_t n, int64_t V, int64_t dim) {
    const Plan p = make_plan<M_FDH>(n, V, device_cus(), kFdhChunks);
    const int64_t nb = (n + kFdhWaves - 1) / kFdhWaves;
    return align256(planes_bytes(n)) + align256(planes_bytes(V)) + align256(p.nchunks * n * 2 * 4) + align256(n * 4) +
           align256(p.nchunks * n * dim * 4) + align256(nb * 2 * 4 + 8);
}

// The training forward: lse (n), out = {mean loss over the valid rows, their count}, and dh_raw (n x dim,
// contiguous: ld_dh must equal dim, the layout asme_linear_xent_bwd_dw reads) = softmax(H W^T + b) W - W[t] per valid row (0 for ignored rows): dH before the upstream scale,
// which asme_linear_xent_bwd_dw applies.  H (n x dim), W (V x dim), dim <= 128.
ASME_API int asme_linear_xent_fwd_dh(const float* H, int64_t ld_h, int64_t n, int64_t dim, const float* W, int64_t ld_w,
                                     int64_t V, const float* bias, const int64_t* targets, int64_t ignore_index,
                                     float* lse, float* dh_raw, int64_t ld_dh, float* workspace, int64_t ws_bytes,
                                     float* out, void* stream) {
    ASME_CHECK_ARG(H && W && targets && lse && dh_raw && workspace && out, "asme_linear_xent_fwd_dh: null pointer");
    ASME_CHECK_ARG(dim >= 4 && dim <= kDP && dim % 4 == 0 && ld_h % 4 == 0 && ld_w % 4 == 0 && aligned16(H) &&
                       aligned16(W),
                   "asme_linear_xent_fwd_dh: dim must be a multiple of 4 in [4, 128], rows 16-B aligned");
    // dh_raw is consumed by asme_linear_xent_bwd_dw as a contiguous n x dim buffer: no other row stride
    ASME_CHECK_ARG(ld_dh == dim, "asme_linear_xent_fwd_dh: dh_raw must be contiguous (ld_dh == dim)");
    ASME_CHECK_ARG(n >= 0 && V >= 1 && V < (1LL << 31), "asme_linear_xent_fwd_dh: bad shape");
    ASME_CHECK_ARG(ws_bytes >= asme_linear_xent_fwd_dh_workspace(n, V, dim),
                   "asme_linear_xent_fwd_dh: workspace too small");
    hipStream_t s = (hipStream_t)stream;
    const Plan p = make_plan<M_FDH>(n, V, device_cus(), kFdhChunks);
    char* w = reinterpret_cast<char*>(workspace);
    __bf16* hp = reinterpret_cast<__bf16*>(w);
    __bf16* wp = reinterpret_cast<__bf16*>(w + align256(planes_bytes(n)));
    float* part = reinterpret_cast<float*>(w + align256(planes_bytes(n)) + align256(planes_bytes(V)));
    float* tlogit = part + align256(p.nchunks * n * 2 * 4) / 4;
    float* upart = tlogit + align256(n * 4) / 4;
    float* bsum = upart + align256(p.nchunks * n * dim * 4) / 4;
    const int64_t nb = (n + kFdhWaves - 1) / kFdhWaves;
    if (n > 0) {
        int rc = split(H, ld_h, n, (int)dim, hp, s);
        if (rc == 0) rc = split(W, ld_w, V, (int)dim, wp, s);
        if (rc != 0) return rc;
        LogitsArgs a{};
        a.stat = hp;
        a.strm = wp;
        a.stat_pad = p.stat_pad;
        a.strm_pad = p.strm_pad;
        a.n_stat = n;
        a.n_strm = V;
        a.chunk = p.chunk;
        a.nchunks = p.nchunks;
        a.d = (int)dim;
        a.bias = bias;
        a.targets = targets;
        a.ignore = ignore_index;
        a.V = V;
        a.part = part;
        a.part2 = tlogit;
        a.upart = upart;
        rc = launch_kb<M_FDH>(a, p.sblocks, s);
        if (rc != 0) return rc;
        hipLaunchKernelGGL(fdh_finish_kernel, dim3((unsigned)nb), dim3(kFdhWaves * 64), 0, s, part, upart, n,
                           p.nchunks, (int)dim, targets, ignore_index, V, tlogit, W, ld_w, lse, dh_raw, ld_dh, bsum);
    }
    hipLaunchKernelGGL(lce_finish_kernel, dim3(1), dim3(1024), 0, s, bsum, nb, out);
    ASME_LAUNCH_CHECK("asme_linear_xent_fwd_dh");
}

ASME_API int64_t asme_linear_xent_bwd_dw_workspace(int64_t n, int64_t V, int64_t dim) {
    const Plan pw = make_plan<M_DW>(V, n, device_cus());
    const int64_t dw = pw.nchunks > 1 ? pw.nchunks * V * (dim + 1) : 0;
    return align256(planes_bytes(n)) + align256(planes_bytes(V)) + align256(dw * 4);
}

// The backward of asme_linear_xent_fwd_dh: dH (n x dim, contiguous) = dh_raw * dloss[0] / stats[1]; dW (V x dim),
// db (V, nullable) from the dW pass (the logits recomputed once).  dH, dW, db are overwritten.
ASME_API int asme_linear_xent_bwd_dw(const float* H, int64_t ld_h, int64_t n, int64_t dim, const float* W,
                                     int64_t ld_w, int64_t V, const float* bias, const int64_t* targets,
                                     int64_t ignore_index, const float* lse, const float* stats, const float* dloss,
                                     const float* dh_raw, float* dH, float* dW, float* db, float* workspace,
                                     int64_t ws_bytes, void* stream) {
    ASME_CHECK_ARG(H && W && targets && lse && stats && dloss && dh_raw && dH && dW,
                   "asme_linear_xent_bwd_dw: null pointer");
    ASME_CHECK_ARG(dim >= 4 && dim <= kDP && dim % 4 == 0 && ld_h % 4 == 0 && ld_w % 4 == 0 && aligned16(H) &&
                       aligned16(W) && aligned16(dH) && aligned16(dW) && aligned16(dh_raw),
                   "asme_linear_xent_bwd_dw: dim must be a multiple of 4 in [4, 128], rows 16-B aligned");
    ASME_CHECK_ARG(V >= 1 && V < (1LL << 31), "asme_linear_xent_bwd_dw: bad shape");
    ASME_CHECK_ARG(ws_bytes >= asme_linear_xent_bwd_dw_workspace(n, V, dim),
                   "asme_linear_xent_bwd_dw: workspace too small");
    hipStream_t s = (hipStream_t)stream;
    if (n == 0) {
        if (hipMemsetAsync(dW, 0, V * dim * sizeof(float), s) != hipSuccess ||
            (db && hipMemsetAsync(db, 0, V * sizeof(float), s) != hipSuccess))
            return hip_status(hipGetLastError(), "asme_linear_xent_bwd_dw");
        return 0;
    }
    const int64_t cnt = n * dim;
    hipLaunchKernelGGL(scale_rows_kernel, dim3((unsigned)((cnt / 4 + 255) / 256)), dim3(256), 0, s, dh_raw, cnt, dloss,
                       stats, dH);
    const Plan pw = make_plan<M_DW>(V, n, device_cus());
    char* w = reinterpret_cast<char*>(workspace);
    __bf16* hp = reinterpret_cast<__bf16*>(w);
    __bf16* wp = reinterpret_cast<__bf16*>(w + align256(planes_bytes(n)));
    float* dw_part = reinterpret_cast<float*>(w + align256(planes_bytes(n)) + align256(planes_bytes(V)));
    float* db_part = dw_part + (pw.nchunks > 1 ? pw.nchunks * V * dim : 0);
    int rc = split(H, ld_h, n, (int)dim, hp, s);
    if (rc == 0) rc = split(W, ld_w, V, (int)dim, wp, s);
    if (rc != 0) return rc;
    LogitsArgs a{};
    a.d = (int)dim;
    a.bias = bias;
    a.targets = targets;
    a.ignore = ignore_index;
    a.V = V;
    a.lse = lse;
    a.dloss = dloss;
    a.stats = stats;
    a.stat = wp;
    a.strm = hp;
    a.stat_pad = pw.stat_pad;
    a.strm_pad = pw.strm_pad;
    a.n_stat = V;
    a.n_strm = n;
    a.chunk = pw.chunk;
    a.nchunks = pw.nchunks;
    a.part = pw.nchunks > 1 ? dw_part : dW;
    a.part2 = pw.nchunks > 1 ? (db ? db_part : nullptr) : db;
    rc = launch_kb<M_DW>(a, pw.sblocks, s);
    if (rc != 0) return rc;
    if (pw.nchunks > 1) {
        auto sum = [&](const float* part, int64_t stride, int64_t nparts, int64_t count, float* out) {
            const int64_t thr = (count + 3) / 4;
            hipLaunchKernelGGL(sum_parts_kernel, dim3((unsigned)((thr + 255) / 256)), dim3(256), 0, s, part, stride,
                               (int)nparts, count, out);
        };
        sum(dw_part, V * dim, pw.nchunks, V * dim, dW);
        if (db) sum(db_part, V, pw.nchunks, V, db);
    }
    ASME_LAUNCH_CHECK("asme_linear_xent_bwd_dw");
}

// ------------------------------------------------------------------------------------ materialised scores
ASME_API int64_t asme_logits_workspace(int64_t n, int64_t V, int64_t dim) {
    (void)dim;
    return align256(planes_bytes(n)) + align256(planes_bytes(V));
}

// out (n x V, row stride ld_out) = H (n x dim) . W^T (V x dim) + bias (nullable), fp32-level products (bf16x6)
ASME_API int asme_logits(const float* H, int64_t ld_h, int64_t n, int64_t dim, const float* W, int64_t ld_w,
                         int64_t V, const float* bias, float* out, int64_t ld_out, float* workspace, int64_t ws_bytes,
                         void* stream) {
    ASME_CHECK_ARG(H && W && out && workspace, "asme_logits: null pointer");
    ASME_CHECK_ARG(dim >= 4 && dim <= kDP && dim % 4 == 0 && ld_h % 4 == 0 && ld_w % 4 == 0 && aligned16(H) &&
                       aligned16(W) && ld_out >= V,
                   "asme_logits: dim must be a multiple of 4 in [4, 128], rows 16-B aligned");
    ASME_CHECK_ARG(n >= 0 && V >= 1 && V < (1LL << 31), "asme_logits: bad shape");
    ASME_CHECK_ARG(ws_bytes >= asme_logits_workspace(n, V, dim), "asme_logits: workspace too small");
    if (n == 0) return 0;
    hipStream_t s = (hipStream_t)stream;
    const Plan p = make_plan<M_LOGITS>(n, V, device_cus());
    char* w = reinterpret_cast<char*>(workspace);
    __bf16* hp = reinterpret_cast<__bf16*>(w);
    __bf16* wp = reinterpret_cast<__bf16*>(w + align256(planes_bytes(n)));
    int rc = split(H, ld_h, n, (int)dim, hp, s);
    if (rc == 0) rc = split(W, ld_w, V, (int)dim, wp, s);
    if (rc != 0) return rc;
    LogitsArgs a{};
    a.stat = hp;
    a.strm = wp;
    a.stat_pad = p.stat_pad;
    a.strm_pad = p.strm_pad;
    a.n_stat = n;
    a.n_strm = V;
    a.chunk = p.chunk;
    a.nchunks = p.nchunks;
    a.d = (int)dim;
    a.bias = bias;
    a.V = V;
    a.out = out;
    a.ld_out = ld_out;
    return launch_kb<M_LOGITS>(a, p.sblocks, s);
}

// ------------------------------------------------------------------------------ full-catalogue ranking (bf16x6)
// The evaluation's target ranks (SASRecProjectionComponent inference, sasrec/components.py:46-61; AllItemsSampler +
// argsort + get_true_positives, metrics_sampler.py:51-72 and metrics/common.py:4-27) on this engine: the scores are
// the products asme_logits materialises (bf16x6, 0.53 of the bf16 peak / 6 in the stats pass at the C3 shape, vs
// 0.49 of the 4x smaller fp32 MFMA peak for csrc/catalog.hip's kernel), never stored.  Two passes: M_TSCORE scores
// each query against its own gathered target row (the same products, so the target compares bit-identically with
// itself), then M_RANK streams the catalogue's planes and counts the items ranked above the target.
namespace {
__global__ __launch_bounds__(256) void gather_targets_kernel(const float* __restrict__ E, int64_t ld_e, int64_t V,
                                                             const float* __restrict__ bias,
                                                             const int64_t* __restrict__ targets, int64_t nq, int d,
                                                             float* __restrict__ rows, float* __restrict__ tbias) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // one thread per 4 features
    const int c4 = (d + 3) / 4;
    if (t >= nq * c4) return;
    const int64_t q = t / c4;
    const int c = (int)(t % c4) * 4;
    int64_t it = targets[q];
    it = (it < 0 || it >= V) ? 0 : it;
    *reinterpret_cast<float4*>(rows + q * d + c) = *reinterpret_cast<const float4*>(E + it * ld_e + c);
    if (c == 0 && tbias) tbias[q] = bias ? bias[it] : 0.f;
}

__global__ void rank_from_counts_kernel(const int32_t* __restrict__ counts, int64_t n, int64_t* __restrict__ ranks) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) ranks[i] = (int64_t)counts[i] + 1;
}

bool catalog_shape_ok(int64_t dim, int64_t ld_h, const void* H) {
    return dim >= 4 && dim <= kDP && dim % 4 == 0 && ld_h % 4 == 0 && aligned16(H);
}
}  // namespace

// bytes of the three bf16 planes of a (rows x dim <= 128) operand (asme_catalog_split)
ASME_API int64_t asme_catalog_planes_bytes(int64_t rows) { return planes_bytes(rows); }

// planes = the exact three-way bf16 split of X (rows x dim), rows zero-padded: split a catalogue once, rank many
// query batches against it
ASME_API int asme_catalog_split(const float* X, int64_t ld, int64_t rows, int64_t dim, void* planes, void* stream) {
    ASME_CHECK_ARG(X && planes, "asme_catalog_split: null pointer");
    ASME_CHECK_ARG(catalog_shape_ok(dim, ld, X) && rows >= 1 && rows < (1LL << 31),
                   "asme_catalog_split: dim must be a multiple of 4 in [4, 128], rows 16-B aligned");
    return split(X, ld, rows, (int)dim, reinterpret_cast<__bf16*>(planes), (hipStream_t)stream);
}

// workspace of asme_catalog_target_scores_x6 / asme_catalog_count_above_x6 / asme_catalog_rank_x6 for nq queries
ASME_API int64_t asme_catalog_x6_workspace(int64_t nq, int64_t dim) {
    (void)dim;
    return 2 * align256(planes_bytes(nq)) + align256(nq * kDP * 4) + 2 * align256(nq * 4) + 256;
}

namespace {
int target_scores_x6(const float* H, int64_t ld_h, int64_t nq, int64_t dim, const float* rows, int64_t ld_rows,
                     const float* row_bias, float* tscore, char* w, hipStream_t s) {
    __bf16* hp = reinterpret_cast<__bf16*>(w);
    __bf16* tp = reinterpret_cast<__bf16*>(w + align256(planes_bytes(nq)));
    int rc = split(H, ld_h, nq, (int)dim, hp, s);
    if (rc == 0) rc = split(rows, ld_rows, nq, (int)dim, tp, s);
    if (rc != 0) return rc;
    const Plan p = make_plan<M_TSCORE>(nq, nq, device_cus());
    LogitsArgs a{};
    a.stat = hp;
    a.strm = tp;
    a.stat_pad = p.stat_pad;
    a.strm_pad = p.stat_pad;  // (the same padding: stationary block b reads streamed rows of block b)
    a.n_stat = nq;
    a.n_strm = nq;
    a.chunk = p.stat_pad;
    a.nchunks = 1;
    a.d = (int)dim;
    a.bias = row_bias;
    a.part2 = tscore;
    return launch_kb<M_TSCORE>(a, p.sblocks, s);
}

int count_above_x6(const float* H, int64_t ld_h, int64_t nq, int64_t dim, const void* E_planes, int64_t V,
                   const float* bias, const int64_t* targets, const float* tscore, int64_t id_stride,
                   int64_t id_offset, int64_t tclamp, int32_t* counts, char* w, hipStream_t s) {
    __bf16* hp = reinterpret_cast<__bf16*>(w);
    int rc = split(H, ld_h, nq, (int)dim, hp, s);
    if (rc != 0) return rc;
    if (hipMemsetAsync(counts, 0, nq * sizeof(int32_t), s) != hipSuccess) return hip_status(hipGetLastError(), "memset");
    const Plan p = make_plan<M_RANK>(nq, V, device_cus());
    LogitsArgs a{};
    a.stat = hp;
    a.strm = reinterpret_cast<const __bf16*>(E_planes);
    a.stat_pad = p.stat_pad;
    a.strm_pad = p.strm_pad;
    a.n_stat = nq;
    a.n_strm = V;
    a.chunk = p.chunk;
    a.nchunks = p.nchunks;
    a.d = (int)dim;
    a.bias = bias;
    a.targets = targets;
    a.V = V;
    a.tscore = tscore;
    a.counts = counts;
    a.id_stride = id_stride;
    a.id_offset = id_offset;
    a.tclamp = tclamp;
    return launch_kb<M_RANK>(a, p.sblocks, s);
}
}  // namespace

// tscore[q] = H[q] . rows[q] (+ row_bias[q]) by the products the ranking pass forms (the sharded evaluation's
// target scores from the rows their owners sent)
ASME_API int asme_catalog_target_scores_x6(const float* H, int64_t ld_h, int64_t nq, int64_t dim, const float* rows,
                                           int64_t ld_rows, const float* row_bias, float* tscore, void* workspace,
                                           int64_t ws_bytes, void* stream) {
    ASME_CHECK_ARG(H && rows && tscore && workspace, "asme_catalog_target_scores_x6: null pointer");
    ASME_CHECK_ARG(catalog_shape_ok(dim, ld_h, H) && ld_rows % 4 == 0 && aligned16(rows) && nq < (1LL << 31),
                   "asme_catalog_target_scores_x6: dim must be a multiple of 4 in [4, 128], rows 16-B aligned");
    ASME_CHECK_ARG(ws_bytes >= asme_catalog_x6_workspace(nq, dim), "asme_catalog_target_scores_x6: workspace too small");
    if (nq == 0) return 0;
    const int rc = target_scores_x6(H, ld_h, nq, dim, rows, ld_rows, row_bias, tscore,
                                    reinterpret_cast<char*>(workspace), (hipStream_t)stream);
    if (rc != 0) return rc;
    ASME_LAUNCH_CHECK("asme_catalog_target_scores_x6");
}

// counts[q] = #{local rows j of E_planes (V rows, asme_catalog_split) ranked above query q's target}: item id
// j * id_stride + id_offset, ranked above iff its score is higher, or equal with a lower id (overwrites counts)
ASME_API int asme_catalog_count_above_x6(const float* H, int64_t ld_h, int64_t nq, int64_t dim, const void* E_planes,
                                         int64_t V, const float* bias, const int64_t* targets, const float* tscore,
                                         int64_t id_stride, int64_t id_offset, int32_t* counts, void* workspace,
                                         int64_t ws_bytes, void* stream) {
    ASME_CHECK_ARG(H && E_planes && targets && tscore && counts && workspace, "asme_catalog_count_above_x6: null pointer");
    ASME_CHECK_ARG(catalog_shape_ok(dim, ld_h, H) && V >= 1 && V < (1LL << 31) && nq < (1LL << 31),
                   "asme_catalog_count_above_x6: bad shape");
    ASME_CHECK_ARG(ws_bytes >= asme_catalog_x6_workspace(nq, dim), "asme_catalog_count_above_x6: workspace too small");
    if (nq == 0) return 0;
    const int rc = count_above_x6(H, ld_h, nq, dim, E_planes, V, bias, targets, tscore, id_stride, id_offset, 0, counts,
                                  reinterpret_cast<char*>(workspace), (hipStream_t)stream);
    if (rc != 0) return rc;
    ASME_LAUNCH_CHECK("asme_catalog_count_above_x6");
}

// ranks[q] = 1 + #{items scoring above query q's target, or equal with a lower id} over the whole catalogue E
// (V x dim); E_planes = asme_catalog_split(E) (a catalogue split once for many batches); counts_ws nq int32
ASME_API int asme_catalog_rank_x6(const float* H, int64_t ld_h, int64_t nq, int64_t dim, const float* E, int64_t ld_e,
                                  const void* E_planes, int64_t V, const float* bias, const int64_t* targets,
                                  int32_t* counts_ws, int64_t* ranks, void* workspace, int64_t ws_bytes, void* stream) {
    ASME_CHECK_ARG(H && E && E_planes && targets && counts_ws && ranks && workspace, "asme_catalog_rank_x6: null pointer");
    ASME_CHECK_ARG(catalog_shape_ok(dim, ld_h, H) && ld_e % 4 == 0 && aligned16(E) && V >= 1 && V < (1LL << 31) &&
                       nq < (1LL << 31),
                   "asme_catalog_rank_x6: dim must be a multiple of 4 in [4, 128], rows 16-B aligned");
    ASME_CHECK_ARG(ws_bytes >= asme_catalog_x6_workspace(nq, dim), "asme_catalog_rank_x6: workspace too small");
    if (nq == 0) return 0;
    hipStream_t s = (hipStream_t)stream;
    char* w = reinterpret_cast<char*>(workspace);
    float* rows = reinterpret_cast<float*>(w + 2 * align256(planes_bytes(nq)));
    float* tbias = reinterpret_cast<float*>(reinterpret_cast<char*>(rows) + align256(nq * kDP * 4));
    float* tscore = tbias + align256(nq * 4) / 4;
    const int64_t nt = nq * ((dim + 3) / 4);
    hipLaunchKernelGGL(gather_targets_kernel, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, s, E, ld_e, V, bias,
                       targets, nq, (int)dim, rows, tbias);
    int rc = target_scores_x6(H, ld_h, nq, dim, rows, dim, bias ? tbias : nullptr, tscore, w, s);
    if (rc == 0)
        rc = count_above_x6(H, ld_h, nq, dim, E_planes, V, bias, targets, tscore, 1, 0, V, counts_ws, w, s);
    if (rc != 0) return rc;
    hipLaunchKernelGGL(rank_from_counts_kernel, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, s, counts_ws, nq,
                       ranks);
    ASME_LAUNCH_CHECK("asme_catalog_rank_x6");
}
