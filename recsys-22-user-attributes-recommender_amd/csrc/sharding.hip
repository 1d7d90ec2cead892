// Item-id deduplication and row-shard bucketing on gfx950.
//
// Used by (a) the sparse-gradient dense-Adam path of the item table (row_slot map) and (b) the
// row-sharded item table (cyclic shard: global row g -> owner g % W, local row g / W), whose
// lookups/gradients cross ranks with RCCL all-to-all.  The reference has no such code:
// it runs nn.Embedding with a dense gradient under Lightning DDP.
//
// Dedup is deterministic: a |V|-sized int32 map (all -1 at rest) gets atomicMin(i) per occurrence,
// so each distinct id's representative is its FIRST occurrence; ranking the representatives (wave ballots per
// block, the block counts scanned by the last block to finish) assigns compact slots in first-occurrence order.
// The map keeps the first occurrences and must be reset with asme_dedup_reset.
#include "adam_math.h"
#include "common.h"

using namespace asme;

namespace {

// Block-level aggregation of the per-key global atomics (claim, CSR count and scatter).  A key on a large share of
// the batch (PAD of short sessions, the cloze MASK token, a small attribute vocabulary) made every occurrence an
// atomic on ONE address -- 0.34 ms per kernel for the 37k MASK occurrences of a KeBERT4Rec batch, against ~10 us
// for uniform ids.  Each 256-thread block first combines its occurrences per key in an LDS hash table (512 slots,
// linear probing, at most 256 keys: every insert terminates) and then issues one global atomic per distinct key.
// kOcc occurrences per thread (4: 1,024 per block, 2,048 slots): a key on every block -- the head of a Zipf(1.07)
// id distribution at |I| = 10M, ~160 keys on > 256 occurrences of a 614k-occurrence batch -- costs a quarter of
// the same-address atomics (they serialise at the L2: the claim took 0.17-0.24 ms per call on Zipf ids).
#ifndef ASME_HASH_OCC
#define ASME_HASH_OCC 4
#endif
constexpr int kOcc = ASME_HASH_OCC;
constexpr int kHashSlots = 512 * kOcc;
constexpr int kHashBits = kOcc == 1 ? 9 : kOcc == 2 ? 10 : kOcc == 4 ? 11 : 12;
static_assert((1 << kHashBits) == kHashSlots, "hash slots: a power of two");
struct BlockHash {
    int32_t key[kHashSlots];
    int32_t val[kHashSlots];
    int32_t aux[kHashSlots];
};
__device__ __forceinline__ void hash_init(BlockHash& t, int32_t v0) {
    for (int j = threadIdx.x; j < kHashSlots; j += blockDim.x) {
        t.key[j] = -1;
        t.val[j] = v0;
    }
    __syncthreads();
}
__device__ __forceinline__ int hash_insert(BlockHash& t, int32_t key) {  // key >= 0
    uint32_t h = ((uint32_t)key * 2654435761u) >> (32 - kHashBits);
    for (;;) {
        const int32_t prev = atomicCAS(&t.key[h], -1, key);
        if (prev == -1 || prev == key) return (int)h;
        h = (h + 1) & (kHashSlots - 1);
    }
}

// Cross-workgroup hand-off inside one launch without an L2 writeback: the published values are stored with
// device-coherent (agent-scope atomic) stores, the storing wave waits for them (vmcnt(0)) before it takes the ticket,
// and the last workgroup reads them with device-coherent loads.  (__threadfence() here wrote back every dirty L2 line
// of the XCD once per workgroup: 76 us for the 600 blocks of a 614k-id dedup.)
__device__ __forceinline__ void publish_i32(int32_t* p, int32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int32_t coherent_i32(const int32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool last_arrival(int32_t* ticket, int64_t arrivals) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's published stores have completed
    return __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (int32_t)(arrivals - 1);
}

// The id list of one dedup: up to kMaxSegs segments read in place (the step's input, positive and negative id
// tensors: no concatenated copy), occurrence i = flat position over the segments.
constexpr int kMaxSegs = 4;
struct IdSegs {
    const int64_t* p[kMaxSegs];
    int64_t start[kMaxSegs + 1];
    int n;
};
__device__ __forceinline__ int64_t seg_id(const IdSegs& S, int64_t i) {
    const int64_t* p = S.p[0];
    int64_t o = i;
#pragma unroll
    for (int q = 1; q < kMaxSegs; ++q)  // constant indices: the table stays in SGPRs
        if (q < S.n && i >= S.start[q]) {
            p = S.p[q];
            o = i - S.start[q];
        }
    return p[o];
}

// (1) map[id] = min occurrence index (its first occurrence); block 0 also zeroes the slot-scan ticket of (2)
__global__ __launch_bounds__(256) void claim_kernel(IdSegs S, int64_t n, int64_t V, int32_t* __restrict__ map,
                                                    int32_t* __restrict__ ticket) {
    __shared__ BlockHash t;
    hash_init(t, INT32_MAX);
#pragma unroll
    for (int q = 0; q < kOcc; ++q) {
        const int64_t i = ((int64_t)blockIdx.x * kOcc + q) * blockDim.x + threadIdx.x;
        const int64_t id = i < n ? seg_id(S, i) : -1;
        if (id >= 0 && id < V) atomicMin(&t.val[hash_insert(t, (int32_t)id)], (int32_t)i);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) *ticket = 0;
    __syncthreads();
    for (int j = threadIdx.x; j < kHashSlots; j += blockDim.x)
        if (t.key[j] >= 0) atomicMin(reinterpret_cast<unsigned int*>(map + t.key[j]), (unsigned int)t.val[j]);
}

// (2) slots in first-occurrence order without a library scan: a block of kDedupBk occurrences ranks its
// representatives (map[id] == i) by wave ballots -> lpre[i] (rank within the block) and bcnt[b]; the last block to
// finish (ticket, no waiting) scans bcnt in place into block offsets and writes the count.  slot(r) = bcnt[r / kDedupBk]
// + lpre[r] for a representative r.
constexpr int kDedupBk = 1024;
__global__ __launch_bounds__(256) void dedup_rank_kernel(IdSegs S, int64_t n, int64_t V,
                                                         const int32_t* __restrict__ map, int32_t* __restrict__ lpre,
                                                         int32_t* __restrict__ bcnt, int32_t* __restrict__ ticket,
                                                         int32_t* __restrict__ count) {
    __shared__ int32_t wsum[4];
    __shared__ int last;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    const int64_t b0 = (int64_t)blockIdx.x * kDedupBk;
    int32_t base = 0;
    for (int r = 0; r < kDedupBk / 256; ++r) {
        const int64_t i = b0 + r * 256 + threadIdx.x;
        bool rep = false;
        if (i < n) {
            const int64_t id = seg_id(S, i);
            rep = id >= 0 && id < V && map[id] == (int32_t)i;
        }
        const uint64_t m = __ballot(rep);
        if (lane == 0) wsum[wave] = __popcll(m);
        __syncthreads();
        int32_t pre = base;
        for (int w = 0; w < wave; ++w) pre += wsum[w];
        if (rep) lpre[i] = pre + __popcll(m & lt);
        base += wsum[0] + wsum[1] + wsum[2] + wsum[3];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        publish_i32(bcnt + blockIdx.x, base);
        last = last_arrival(ticket, gridDim.x);
    }
    __syncthreads();
    if (!last) return;
    // exclusive scan of bcnt[0, nb) by this block: 256-entry rounds, one wave-scan per wave + the wave carries
    const int64_t nb = gridDim.x;
    __shared__ int32_t wtot[4];
    int32_t carry = 0;
    for (int64_t c0 = 0; c0 < nb; c0 += 256) {
        const int64_t b = c0 + threadIdx.x;
        const int32_t v = b < nb ? coherent_i32(bcnt + b) : 0;
        int32_t x = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int32_t y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) wtot[wave] = x;
        __syncthreads();
        int32_t wpre = carry;
        for (int w = 0; w < wave; ++w) wpre += wtot[w];
        if (b < nb) bcnt[b] = wpre + x - v;
        carry += wtot[0] + wtot[1] + wtot[2] + wtot[3];
        __syncthreads();
    }
    if (threadIdx.x == 0) *count = carry;
}

// (3) every occurrence's slot (inverse) through its representative r = map[id]; the representative writes unique
__global__ __launch_bounds__(256) void dedup_slot_kernel(IdSegs S, int64_t n, int64_t V,
                                                         const int32_t* __restrict__ map,
                                                         const int32_t* __restrict__ lpre,
                                                         const int32_t* __restrict__ boff, int64_t* __restrict__ unique,
                                                         int64_t* __restrict__ inverse) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t id = seg_id(S, i);
    int64_t slot = -1;
    if (id >= 0 && id < V) {
        const int32_t r = map[id];
        slot = (int64_t)boff[r / kDedupBk] + lpre[r];
        if (r == (int32_t)i) unique[slot] = id;
    }
    if (inverse) inverse[i] = slot;
}

__global__ void map_slots_kernel(const int64_t* __restrict__ unique, const int32_t* __restrict__ count,
                                 int32_t* __restrict__ map, int64_t cap) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= cap || s >= *count) return;
    map[unique[s]] = (int32_t)s;
}

__global__ void reset_kernel(const int64_t* __restrict__ unique, const int32_t* __restrict__ count,
                             int32_t* __restrict__ map, int64_t cap) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= cap || s >= *count) return;
    map[unique[s]] = -1;
}

// owner = id % W, local = id / W; counts[w] = #ids owned by w (ids already unique)
__global__ void owner_hist_kernel(const int64_t* __restrict__ ids, const int32_t* __restrict__ count, int64_t cap,
                                  int W, int32_t* __restrict__ owner, int32_t* __restrict__ counts) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= cap || i >= *count) return;
    const int w = (int)(ids[i] % W);
    owner[i] = w;
    atomicAdd(counts + w, 1);
}

inline unsigned nblk(int64_t n) { return (unsigned)((n + 255) / 256); }
inline unsigned nblk_occ(int64_t n) { return (unsigned)((n + 256 * kOcc - 1) / (256 * kOcc)); }  // hashed kernels

// ---- stable bucketing of the requester's unique ids by owner (counting sort over W <= 64 buckets):
// block b of kBk ids -> bcount[w * nb + b]; one block scans (w-major) into offsets; the scatter pass ranks
// each id among the same-owner ids of its block (wave ballots + LDS wave prefixes, four rounds in order),
// so positions are stable: bucket w holds its ids in increasing unique-index order.
constexpr int kBk = 1024, kBkThreads = 256, kMaxW = 64;

// n_dev (nullable): the number of ids is *n_dev <= n (a dedup count that never visits the host)
__device__ __forceinline__ int64_t live_n(int64_t n, const int32_t* n_dev) { return n_dev ? min(n, (int64_t)*n_dev) : n; }
// bucket of id i: its owner id % Wo, or -- with a class split (split non-null: the slots >= *split, the requester's
// negative-only rows, travel in a second exchange) -- owner + Wo for the second class: 2 Wo buckets, class-major
__device__ __forceinline__ int bucket_key(int64_t id, int64_t i, int Wo, int32_t split) {
    return (int)(id % Wo) + (i >= split ? Wo : 0);
}

__global__ __launch_bounds__(kBkThreads) void bucket_count_kernel(const int64_t* __restrict__ ids, int64_t n,
                                                                  const int32_t* __restrict__ n_dev, int W,
                                                                  int32_t* __restrict__ bcount, int64_t nb, int Wo,
                                                                  const int32_t* __restrict__ split) {
    __shared__ int32_t h[kMaxW];
    n = live_n(n, n_dev);
    const int32_t sp = split ? *split : 0x7FFFFFFF;
    for (int w = threadIdx.x; w < W; w += blockDim.x) h[w] = 0;
    __syncthreads();
    const int64_t b0 = (int64_t)blockIdx.x * kBk;
    for (int r = 0; r < kBk / kBkThreads; ++r) {
        const int64_t i = b0 + r * kBkThreads + threadIdx.x;
        if (i < n) atomicAdd(h + bucket_key(ids[i], i, Wo, sp), 1);
    }
    __syncthreads();
    for (int w = threadIdx.x; w < W; w += blockDim.x) bcount[(int64_t)w * nb + blockIdx.x] = h[w];
}

// exclusive scan of bcount (W * nb, w-major) in place; counts[w] = ids owned by w
__global__ __launch_bounds__(1024) void bucket_scan_kernel(int32_t* __restrict__ bcount, int64_t nb, int W, int64_t n,
                                                           const int32_t* __restrict__ n_dev,
                                                           int64_t* __restrict__ counts) {
    __shared__ int32_t part[1024];
    n = live_n(n, n_dev);
    const int64_t total = nb * W;
    const int64_t per = (total + blockDim.x - 1) / blockDim.x;
    const int64_t lo = min(total, (int64_t)threadIdx.x * per), hi = min(total, lo + per);
    int32_t s = 0;
    for (int64_t i = lo; i < hi; ++i) s += bcount[i];
    part[threadIdx.x] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        int32_t run = 0;
        for (int t = 0; t < (int)blockDim.x; ++t) {
            const int32_t v = part[t];
            part[t] = run;
            run += v;
        }
    }
    __syncthreads();
    int32_t run = part[threadIdx.x];
    for (int64_t i = lo; i < hi; ++i) {
        const int32_t v = bcount[i];
        bcount[i] = run;
        run += v;
    }
    __syncthreads();
    for (int w = threadIdx.x; w < W; w += blockDim.x) {
        const int64_t beg = bcount[(int64_t)w * nb];
        const int64_t end = w + 1 < W ? (int64_t)bcount[(int64_t)(w + 1) * nb] : n;
        counts[w] = end - beg;
    }
}

__global__ __launch_bounds__(kBkThreads) void bucket_scatter_kernel(const int64_t* __restrict__ ids, int64_t n,
                                                                    const int32_t* __restrict__ n_dev, int W,
                                                                    const int32_t* __restrict__ boff, int64_t nb,
                                                                    int64_t* __restrict__ order,
                                                                    int32_t* __restrict__ send_local, int Wo,
                                                                    const int32_t* __restrict__ split) {
    constexpr int kWv = kBkThreads / 64;
    n = live_n(n, n_dev);
    const int32_t sp = split ? *split : 0x7FFFFFFF;
    __shared__ int32_t base[kMaxW];
    __shared__ int32_t wcnt[kWv][kMaxW];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int w = threadIdx.x; w < W; w += blockDim.x) base[w] = boff[(int64_t)w * nb + blockIdx.x];
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    const int64_t b0 = (int64_t)blockIdx.x * kBk;
    for (int r = 0; r < kBk / kBkThreads; ++r) {
        const int64_t i = b0 + r * kBkThreads + threadIdx.x;
        const bool live = i < n;
        const int64_t id = live ? ids[i] : 0;
        const int mine = live ? bucket_key(id, i, Wo, sp) : -1;
        int rank = 0;
        for (int w = 0; w < W; ++w) {
            const uint64_t m = __ballot(mine == w);
            if (mine == w) rank = __popcll(m & lt);
            if (lane == 0) wcnt[wave][w] = __popcll(m);
        }
        __syncthreads();
        if (live) {
            int pre = 0;
            for (int v = 0; v < wave; ++v) pre += wcnt[v][mine];
            const int64_t pos = (int64_t)base[mine] + pre + rank;
            order[pos] = i;
            send_local[pos] = (int32_t)(id / Wo);
        }
        __syncthreads();
        for (int w = threadIdx.x; w < W; w += blockDim.x) {
            int t = 0;
            for (int v = 0; v < kWv; ++v) t += wcnt[v][w];
            base[w] += t;
        }
        __syncthreads();
    }
}

__global__ void invert_perm_kernel(const int64_t* __restrict__ order, int64_t n, const int32_t* __restrict__ n_dev,
                                   int64_t* __restrict__ pos) {
    n = live_n(n, n_dev);
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < n) pos[order[j]] = j;
}

}  // namespace

namespace {
size_t ws_up(size_t x) { return (x + 255) & ~(size_t)255; }
}  // namespace

ASME_API int64_t asme_dedup_workspace_bytes(int64_t n) {
    // per-occurrence rank within its block (int32), per-block counts / offsets, the scan ticket
    const int64_t nb = (n + kDedupBk - 1) / kDedupBk;
    return (int64_t)(ws_up((size_t)n * 4) + ws_up((size_t)(nb + 1) * 4));
}

// ids: nseg (1..4) segments seg_ids[q] of seg_n[q] ids (host arrays), occurrence i = flat position over them.
// -> unique (cap >= n) in first-occurrence order, inverse (n, nullable) slot per occurrence (-1 for an id outside
// [0, vocab)), count (1 int32 on the device).  map: |V| int32, all -1 on entry; on exit map[unique[s]] = the first
// occurrence of unique[s] (call asme_dedup_reset afterwards).  Three launches, no library scan.
ASME_API int asme_dedup_ids_segments(int nseg, const int64_t* const* seg_ids, const int64_t* seg_n, int64_t vocab,
                                     int32_t* map, void* workspace, int64_t workspace_bytes, int64_t* unique,
                                     int64_t* inverse, int32_t* count, void* stream) {
    ASME_CHECK_ARG(nseg >= 1 && nseg <= kMaxSegs && seg_ids && seg_n, "asme_dedup_ids: 1..4 id segments");
    IdSegs S{};
    S.n = nseg;
    int64_t n = 0;
    for (int q = 0; q < nseg; ++q) {
        ASME_CHECK_ARG(seg_n[q] >= 0 && (seg_ids[q] || seg_n[q] == 0), "asme_dedup_ids: bad segment");
        S.p[q] = seg_ids[q];
        S.start[q] = n;
        n += seg_n[q];
    }
    for (int q = nseg; q <= kMaxSegs; ++q) S.start[q] = n;
    ASME_CHECK_ARG(map && workspace && unique && count, "asme_dedup_ids: null pointer");
    ASME_CHECK_ARG(n >= 1 && n < (int64_t)1 << 31, "asme_dedup_ids: n must be in [1, 2^31)");
    ASME_CHECK_ARG(vocab >= 1 && vocab < (int64_t)1 << 31, "asme_dedup_ids: vocab must be in [1, 2^31)");
    ASME_CHECK_ARG(workspace_bytes >= asme_dedup_workspace_bytes(n), "asme_dedup_ids: workspace too small");
    hipStream_t s = (hipStream_t)stream;
    const int64_t nb = (n + kDedupBk - 1) / kDedupBk;
    char* ws = (char*)workspace;
    int32_t* lpre = (int32_t*)ws;
    int32_t* bcnt = (int32_t*)(ws + ws_up((size_t)n * 4));
    int32_t* ticket = bcnt + nb;
    hipLaunchKernelGGL(claim_kernel, dim3(nblk_occ(n)), dim3(256), 0, s, S, n, vocab, map, ticket);
    hipLaunchKernelGGL(dedup_rank_kernel, dim3((unsigned)nb), dim3(256), 0, s, S, n, vocab, map, lpre, bcnt, ticket,
                       count);
    hipLaunchKernelGGL(dedup_slot_kernel, dim3(nblk(n)), dim3(256), 0, s, S, n, vocab, map, lpre, bcnt, unique,
                       inverse);
    ASME_LAUNCH_CHECK("asme_dedup_ids");
}

ASME_API int asme_dedup_ids(const int64_t* ids, int64_t n, int64_t vocab, int32_t* map, void* workspace,
                            int64_t workspace_bytes, int64_t* unique, int64_t* inverse, int32_t* count,
                            void* stream) {
    ASME_CHECK_ARG(ids, "asme_dedup_ids: null pointer");
    const int64_t* segs[1] = {ids};
    const int64_t ns[1] = {n};
    return asme_dedup_ids_segments(1, segs, ns, vocab, map, workspace, workspace_bytes, unique, inverse, count,
                                   stream);
}

// map[unique[s]] = s for s < *count: the dedup's map as a row -> slot table (asme_adam_rows_step's row_slot)
ASME_API int asme_dedup_map_slots(const int64_t* unique, const int32_t* count, int64_t cap, int32_t* map,
                                  void* stream) {
    ASME_CHECK_ARG(unique && count && map, "asme_dedup_map_slots: null pointer");
    if (cap == 0) return 0;
    hipLaunchKernelGGL(map_slots_kernel, dim3(nblk(cap)), dim3(256), 0, (hipStream_t)stream, unique, count, map, cap);
    ASME_LAUNCH_CHECK("asme_dedup_map_slots");
}

ASME_API int asme_dedup_reset(const int64_t* unique, const int32_t* count, int64_t cap, int32_t* map, void* stream) {
    ASME_CHECK_ARG(unique && count && map, "asme_dedup_reset: null pointer");
    if (cap == 0) return 0;
    hipLaunchKernelGGL(reset_kernel, dim3(nblk(cap)), dim3(256), 0, (hipStream_t)stream, unique, count, map, cap);
    ASME_LAUNCH_CHECK("asme_dedup_reset");
}

// counts (W int32, zeroed by caller) += per-owner counts of unique ids; owner[i] = unique[i] % W
ASME_API int asme_owner_histogram(const int64_t* unique, const int32_t* count, int64_t cap, int world,
                                  int32_t* owner, int32_t* counts, void* stream) {
    ASME_CHECK_ARG(unique && count && owner && counts && world >= 1, "asme_owner_histogram: bad argument");
    if (cap == 0) return 0;
    hipLaunchKernelGGL(owner_hist_kernel, dim3(nblk(cap)), dim3(256), 0, (hipStream_t)stream, unique, count, cap,
                       world, owner, counts);
    ASME_LAUNCH_CHECK("asme_owner_histogram");
}

ASME_API int64_t asme_bucket_by_owner_workspace(int64_t n, int world) {
    const int64_t nb = (n + kBk - 1) / kBk;
    return (nb * world + 1) * (int64_t)sizeof(int32_t);
}

// Row-shard request routing: the n unique ids, grouped by owner (id % world) in a stable order.
// order[j] = index into ids of the j-th id sent; send_local[j] = ids[order[j]] / world (the owner's row, int32: what
// crosses the fabric; a shard holds < 2^31 rows);
// counts[w] = ids sent to rank w (int64, world entries); pos[order[j]] = j (nullable: the inverse permutation).
// n_dev (nullable): only the first *n_dev <= n ids are live (the dedup count on the device: no host sync).
namespace {
int bucket_by_owner(const int64_t* ids, int64_t n, const int32_t* n_dev, int world, const int32_t* split,
                    void* workspace, int64_t ws_bytes, int64_t* order, int32_t* send_local, int64_t* counts,
                    int64_t* pos, void* stream) {
    const int nbk = split ? 2 * world : world;  // buckets
    ASME_CHECK_ARG(ids && workspace && order && send_local && counts, "asme_bucket_by_owner: null pointer");
    ASME_CHECK_ARG(world >= 1 && nbk <= kMaxW, "asme_bucket_by_owner: world must be in [1, 64] (split: [1, 32])");
    ASME_CHECK_ARG(n >= 0 && n < ((int64_t)1 << 31), "asme_bucket_by_owner: bad n");
    ASME_CHECK_ARG(ws_bytes >= asme_bucket_by_owner_workspace(n, nbk), "asme_bucket_by_owner: workspace too small");
    hipStream_t s = (hipStream_t)stream;
    if (n == 0) {
        if (hipMemsetAsync(counts, 0, nbk * sizeof(int64_t), s) != hipSuccess)
            return hip_status(hipGetLastError(), "asme_bucket_by_owner");
        return 0;
    }
    const int64_t nb = (n + kBk - 1) / kBk;
    int32_t* bcount = (int32_t*)workspace;
    hipLaunchKernelGGL(bucket_count_kernel, dim3((unsigned)nb), dim3(kBkThreads), 0, s, ids, n, n_dev, nbk, bcount,
                       nb, world, split);
    hipLaunchKernelGGL(bucket_scan_kernel, dim3(1), dim3(1024), 0, s, bcount, nb, nbk, n, n_dev, counts);
    hipLaunchKernelGGL(bucket_scatter_kernel, dim3((unsigned)nb), dim3(kBkThreads), 0, s, ids, n, n_dev, nbk, bcount,
                       nb, order, send_local, world, split);
    if (pos) hipLaunchKernelGGL(invert_perm_kernel, dim3(nblk(n)), dim3(256), 0, s, order, n, n_dev, pos);
    ASME_LAUNCH_CHECK("asme_bucket_by_owner");
}
}  // namespace

ASME_API int asme_bucket_by_owner(const int64_t* ids, int64_t n, const int32_t* n_dev, int world, void* workspace,
                                  int64_t ws_bytes, int64_t* order, int32_t* send_local, int64_t* counts, int64_t* pos,
                                  void* stream) {
    return bucket_by_owner(ids, n, n_dev, world, nullptr, workspace, ws_bytes, order, send_local, counts, pos, stream);
}

// asme_bucket_by_owner with the ids split in two classes at the device slot *split: ids[i] with i < *split first, by
// owner, then the rest, by owner -- 2 * world buckets (counts: 2 * world entries, class-major; workspace:
// asme_bucket_by_owner_workspace(n, 2 * world)).  The row-sharded step sends its sequence / positive rows and its
// negative-only rows in two exchanges, the second overlapping the transformer (sharded.py overlap_negatives).
ASME_API int asme_bucket_by_owner_split(const int64_t* ids, int64_t n, const int32_t* n_dev, int world,
                                        const int32_t* split, void* workspace, int64_t ws_bytes, int64_t* order,
                                        int32_t* send_local, int64_t* counts, int64_t* pos, void* stream) {
    ASME_CHECK_ARG(split, "asme_bucket_by_owner_split: null split");
    return bucket_by_owner(ids, n, n_dev, world, split, workspace, ws_bytes, order, send_local, counts, pos, stream);
}

// ---------------------------------------------------------------------------------------------------
// Deterministic table gradient (SURVEY §8b `embedding_scatter_add_bwd(..., mode=deterministic)`, A19).
// Reference: autograd's embedding_dense_backward sums every occurrence's gradient row into the table
// row.  Here the step's occurrences (the dedup inverse, slot per occurrence) are grouped by slot with a
// counting sort -> per-slot lists in increasing occurrence order; each unique row's gradient is then the
// ordered sum over its list (no float atomics: bit-reproducible run to run, and the compact gradient buffer
// needs no zero fill).
namespace {

// Counting sort of the occurrences by slot.  Key of occurrence i: its slot, or cap for an occurrence without one
// (inverse -1: an id outside the table), which sorts last.  (1) per-key counts (integer atomics), (2) exclusive
// scan -> seg_off, (3) scatter: each occurrence takes a position of its key's range by an atomic count-down (any
// order), (4) each range is then put in increasing occurrence order -- the same arrays a stable sort gives, so the
// sums are bit-reproducible.  Ranges of up to kShortSeg by their own thread (a sorting network), up to kLongSeg = 256
// (popular items) by a workgroup that ranks every element against the range (listed by (4), done by (5)), longer
// ones -- a key on a large share of the batch: PAD of short sessions, the cloze MASK token, a small attribute
// vocabulary; the quadratic ranking took 0.15 s for the 37k MASK occurrences of a KeBERT4Rec batch -- by a segmented
// radix sort over at most n / kLongSeg segments (their list and bounds written by (4)).
constexpr int kShortSeg = 16;
#ifndef ASME_LONG_SEG
#define ASME_LONG_SEG 256
#endif
constexpr int kLongSeg = ASME_LONG_SEG;  // (a 2,048-long range took ~100 us in one workgroup)
inline int64_t max_huge(int64_t n) { return n / (kLongSeg + 1) + 1; }
constexpr int kHugeFast = 256;  // huge ranges placed by the stable ballot scatter (below); the rest are long ranges

__device__ __forceinline__ int32_t occ_key(const int64_t* __restrict__ inverse, int64_t i, int64_t cap) {
    const int64_t k = inverse[i];
    return (int32_t)(k >= 0 && k < cap ? k : cap);
}

__global__ __launch_bounds__(256) void csr_count_kernel(const int64_t* __restrict__ inverse, int64_t n, int64_t cap,
                                                        int32_t* __restrict__ cnt) {
    __shared__ BlockHash t;
    hash_init(t, 0);
#pragma unroll
    for (int q = 0; q < kOcc; ++q) {
        const int64_t i = ((int64_t)blockIdx.x * kOcc + q) * blockDim.x + threadIdx.x;
        if (i < n) atomicAdd(&t.val[hash_insert(t, occ_key(inverse, i, cap))], 1);
    }
    __syncthreads();
    for (int j = threadIdx.x; j < kHashSlots; j += blockDim.x)
        if (t.key[j] >= 0) atomicAdd(cnt + t.key[j], t.val[j]);
}

// each block reserves one run of positions per key of its own (count-down from the key's count), its occurrences
// take the places of that run in any order (put in occurrence order per range afterwards)
__global__ __launch_bounds__(256) void csr_scatter_kernel(const int64_t* __restrict__ inverse, int64_t n,
                                                          int64_t cap, const int32_t* __restrict__ seg_off,
                                                          int32_t* __restrict__ cnt, int32_t* __restrict__ order,
                                                          int32_t* __restrict__ sorted_slot) {
    __shared__ BlockHash t;
    hash_init(t, 0);
    int32_t k[kOcc];
    int h[kOcc], r[kOcc];
#pragma unroll
    for (int q = 0; q < kOcc; ++q) {
        const int64_t i = ((int64_t)blockIdx.x * kOcc + q) * blockDim.x + threadIdx.x;
        k[q] = 0;
        h[q] = r[q] = 0;
        if (i < n) {
            k[q] = occ_key(inverse, i, cap);
            h[q] = hash_insert(t, k[q]);
            r[q] = atomicAdd(&t.val[h[q]], 1);
        }
    }
    __syncthreads();
    for (int j = threadIdx.x; j < kHashSlots; j += blockDim.x)
        if (t.key[j] >= 0) t.aux[j] = atomicSub(cnt + t.key[j], t.val[j]) - t.val[j];
    __syncthreads();
#pragma unroll
    for (int q = 0; q < kOcc; ++q) {
        const int64_t i = ((int64_t)blockIdx.x * kOcc + q) * blockDim.x + threadIdx.x;
        if (i >= n) break;
        const int32_t pos = seg_off[k[q]] + t.aux[h[q]] + r[q];
        order[pos] = (int32_t)i;
        sorted_slot[pos] = k[q];
    }
}

// one thread per key: ranges of 2..kShortSeg sorted in registers (an odd-even transposition network over a padded
// array: static indices only), longer ones appended to longs[1..] (longs[0] = their count)
__global__ void csr_order_kernel(const int32_t* __restrict__ seg_off, int64_t n, int64_t cap,
                                 int32_t* __restrict__ order, int32_t* __restrict__ longs, int32_t* __restrict__ huge,
                                 int32_t* __restrict__ hbeg, int32_t* __restrict__ hend, int32_t* __restrict__ hidx) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k > cap) return;
    const int32_t b = seg_off[k];
    const int len = (k < cap ? seg_off[k + 1] : (int32_t)n) - b;
    int32_t hi = -1;  // the key's huge-range index (every key written: no fill)
    if (len > kLongSeg) {
        hi = atomicAdd(huge, 1);
        if (hi < kHugeFast) {
            hbeg[hi] = b;
            hend[hi] = b + len;
        } else {  // past the stable placement's capacity: ranked by a workgroup like the long ranges
            longs[1 + atomicAdd(longs, 1)] = (int32_t)k;
            hi = -1;
        }
    }
    hidx[k] = hi;
    if (len < 2 || hi >= 0 || len > kLongSeg) return;
    if (len == 2) {
        const int32_t x = order[b], y = order[b + 1];
        if (x > y) {
            order[b] = y;
            order[b + 1] = x;
        }
        return;
    }
    if (len > kShortSeg) {
        longs[1 + atomicAdd(longs, 1)] = (int32_t)k;
        return;
    }
    int32_t v[kShortSeg];
#pragma unroll
    for (int j = 0; j < kShortSeg; ++j) v[j] = j < len ? order[b + j] : INT32_MAX;
#pragma unroll
    for (int r = 0; r < kShortSeg; ++r)
#pragma unroll
        for (int j = r & 1; j + 1 < kShortSeg; j += 2) {
            const int32_t lo = min(v[j], v[j + 1]), hi = max(v[j], v[j + 1]);
            v[j] = lo;
            v[j + 1] = hi;
        }
#pragma unroll
    for (int j = 0; j < kShortSeg; ++j)
        if (j < len) order[b + j] = v[j];
}

// long ranges: one workgroup each; an element's place is the number of smaller occurrence indices in its range
__device__ __forceinline__ void csr_long(const int32_t* __restrict__ seg_off, int64_t n, int64_t cap,
                                         const int32_t* __restrict__ longs, int32_t* __restrict__ order,
                                         int32_t* __restrict__ tmp, int blk, int nblocks) {
    const int nl = longs[0];
    for (int t = blk; t < nl; t += nblocks) {
        const int64_t k = longs[1 + t];
        const int32_t b = seg_off[k];
        const int len = (k < cap ? seg_off[k + 1] : (int32_t)n) - b;
        for (int e = threadIdx.x; e < len; e += blockDim.x) {
            const int32_t x = order[b + e];
            int r = 0;
            for (int j = 0; j < len; ++j) r += order[b + j] < x ? 1 : 0;
            tmp[b + r] = x;
        }
        __syncthreads();
        for (int e = threadIdx.x; e < len; e += blockDim.x) order[b + e] = tmp[b + e];
        __syncthreads();
    }
}

// Huge ranges without a sort (the first kHugeFast of them; a hot key's list is long but the keys are few): a
// stable placement over the occurrence array.  (6) per block of kHugeOcc occurrences, the count of each huge key,
// (7) per huge key an exclusive scan of those counts over the blocks (+ the range start), (8) each block walks its
// occurrences in index order -- four rounds of 256, every wave groups its lanes by key with ballots -- and an
// occurrence of huge key j goes to base[j][block] + (earlier occurrences of j in the block).  The range then lists
// its occurrences in increasing order, the arrays the segmented radix sort gave (a single block sorting the 37k
// MASK occurrences of a cloze batch took 0.25 ms).  Huge keys past kHugeFast (a batch with more than 256 keys
// on > 256 occurrences each) are ranked by the long-range workgroups instead (correct at any length, quadratic).
constexpr int kHugeOcc = 1024;  // occurrences per placement block (256 threads x 4 rounds)
inline int64_t huge_blocks(int64_t n) { return (n + kHugeOcc - 1) / kHugeOcc; }

__device__ __forceinline__ void csr_huge_count(const int64_t* __restrict__ inverse, int64_t n, int64_t cap,
                                               const int32_t* __restrict__ hidx, const int32_t* __restrict__ huge,
                                               const int32_t* __restrict__ hbeg, int32_t* __restrict__ cntm,
                                               int64_t nblk_h, int blk) {
    const int nh = min(*huge, kHugeFast);
    if (nh == 0) return;
    __shared__ int32_t c[kHugeFast];
    if (threadIdx.x < kHugeFast) c[threadIdx.x] = 0;
    __syncthreads();
    const int64_t b0 = (int64_t)blk * kHugeOcc;
    for (int r = 0; r < kHugeOcc / 256; ++r) {
        const int64_t i = b0 + r * 256 + threadIdx.x;
        const int j = i < n ? hidx[occ_key(inverse, i, cap)] : -1;
        if (j >= 0 && j < kHugeFast) atomicAdd(&c[j], 1);  // (counts only: order does not matter here)
    }
    __syncthreads();
    if ((int)threadIdx.x < nh) cntm[(int64_t)threadIdx.x * nblk_h + blk] = c[threadIdx.x];
}

// (7) per huge key j (one wave each, its own launch): base[j][b] = hbeg[j] + its counts over the blocks < b, in place.
// (This scan had run in the last block of (6) to finish, one wave per key over every key: ~160 keys of a Zipf(1.07)
// batch at |I| = 10M, each a chain of dependent device-coherent loads; the occurrence CSR of the Zipf bench leg
// 0.45 -> 0.39 ms per call with this launch, same box.)
__global__ __launch_bounds__(64) void csr_huge_scan_kernel(const int32_t* __restrict__ huge,
                                                           const int32_t* __restrict__ hbeg, int32_t* __restrict__ cntm,
                                                           int64_t nblk_h) {
    const int j = blockIdx.x, lane = threadIdx.x;
    if (j >= min(*huge, kHugeFast)) return;
    int32_t* row = cntm + (int64_t)j * nblk_h;
    int32_t carry = hbeg[j];
    for (int64_t c0 = 0; c0 < nblk_h; c0 += 64) {
        const int64_t b = c0 + lane;
        const int32_t v = b < nblk_h ? row[b] : 0;
        int32_t x = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int32_t y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (b < nblk_h) row[b] = carry + x - v;
        carry += __shfl(x, 63, 64);
    }
}

// (5) and (6) in one launch: blocks [0, kLongBlocks) rank the long ranges, the rest count the huge keys
constexpr int kLongBlocks = 64;
__global__ __launch_bounds__(256) void csr_long_huge_kernel(const int64_t* __restrict__ inverse,
                                                            const int32_t* __restrict__ seg_off, int64_t n,
                                                            int64_t cap, const int32_t* __restrict__ longs,
                                                            int32_t* __restrict__ order, int32_t* __restrict__ tmp,
                                                            const int32_t* __restrict__ hidx,
                                                            const int32_t* __restrict__ huge,
                                                            const int32_t* __restrict__ hbeg,
                                                            int32_t* __restrict__ cntm, int64_t nblk_h) {
    if (blockIdx.x < kLongBlocks)
        csr_long(seg_off, n, cap, longs, order, tmp, blockIdx.x, kLongBlocks);
    else
        csr_huge_count(inverse, n, cap, hidx, huge, hbeg, cntm, nblk_h, blockIdx.x - kLongBlocks);
}

__global__ __launch_bounds__(256) void csr_huge_place_kernel(const int64_t* __restrict__ inverse, int64_t n,
                                                             int64_t cap, const int32_t* __restrict__ hidx,
                                                             const int32_t* __restrict__ huge,
                                                             const int32_t* __restrict__ cntm, int64_t nblk_h,
                                                             int32_t* __restrict__ order) {
    const int nh = min(*huge, kHugeFast);
    if (nh == 0) return;
    __shared__ int32_t run[kHugeFast];      // this block's occurrences of key j placed so far (+ its base)
    __shared__ int32_t wc[4][kHugeFast];    // per wave of the current round: occurrences of key j
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if ((int)threadIdx.x < nh) run[threadIdx.x] = cntm[(int64_t)threadIdx.x * nblk_h + blockIdx.x];
    const uint64_t below = (1ull << lane) - 1;
    const int64_t b0 = (int64_t)blockIdx.x * kHugeOcc;
    for (int r = 0; r < kHugeOcc / 256; ++r) {
        for (int t = threadIdx.x; t < 4 * kHugeFast; t += 256) (&wc[0][0])[t] = 0;
        __syncthreads();
        const int64_t i = b0 + r * 256 + threadIdx.x;
        int j = i < n ? hidx[occ_key(inverse, i, cap)] : -1;
        if (j >= kHugeFast) j = -1;
        int rank = 0;
        uint64_t todo = __ballot(j >= 0);
        while (todo) {  // lanes grouped by key, lowest lane's key first
            const int jj = __shfl(j, __ffsll((unsigned long long)todo) - 1);
            const uint64_t m = __ballot(j == jj);
            if (j == jj) rank = __popcll(m & below);
            if (lane == __ffsll((unsigned long long)m) - 1) wc[wave][jj] = __popcll(m);
            todo &= ~m;
        }
        __syncthreads();
        if (j >= 0) {
            int p = run[j] + rank;
            for (int w = 0; w < wave; ++w) p += wc[w][j];
            order[p] = (int32_t)i;
        }
        __syncthreads();
        if ((int)threadIdx.x < nh) run[threadIdx.x] += wc[0][threadIdx.x] + wc[1][threadIdx.x] + wc[2][threadIdx.x] +
                                                        wc[3][threadIdx.x];
        __syncthreads();
    }
}

// Exclusive scan of in[0, n) -> out (single pass, decoupled look-back): a block takes the next tile index from a
// counter (tiles start in index order, so every predecessor is resident or done), scans its kScanTile values, publishes
// its total (status 1) and, once its predecessors' prefix is known from their published words, its inclusive prefix
// (status 2).  Word of tile t = status << 32 | value, in `state` (1 + tiles 64-bit words, zeroed by the caller).
constexpr int kScanTile = 1024;
__global__ __launch_bounds__(256) void chained_scan_kernel(const int32_t* __restrict__ in, int64_t n,
                                                           int32_t* __restrict__ out,
                                                           unsigned long long* __restrict__ state) {
    __shared__ int tile_s;
    __shared__ int32_t wtot[4];
    __shared__ int32_t prefix_s;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (threadIdx.x == 0) tile_s = (int)atomicAdd(state, 1ull);
    __syncthreads();
    const int64_t tile = tile_s;
    const int64_t i0 = tile * kScanTile + 4 * threadIdx.x;  // 4 consecutive values per thread
    int32_t v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = i0 + j < n ? in[i0 + j] : 0;
    const int32_t tsum = v[0] + v[1] + v[2] + v[3];
    int32_t x = tsum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) wtot[wave] = x;
    __syncthreads();
    int32_t wpre = 0;
    for (int w = 0; w < wave; ++w) wpre += wtot[w];
    const int32_t total = wtot[0] + wtot[1] + wtot[2] + wtot[3];
    if (wave == 0) {
        // the word carries its own value: relaxed device-coherent atomics, no fence.  Look-back 64 predecessors at a
        // time (lane l: tile j - l), summing up to the nearest one with an inclusive prefix; a window with an
        // unpublished tile before that one is read again.
        unsigned long long* word = state + 1;
        if (lane == 0 && tile > 0)
            __hip_atomic_store(word + tile, (1ull << 32) | (uint32_t)total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int32_t prefix = 0;
        for (int64_t j = tile - 1; j >= 0;) {
            const int64_t k = j - lane;
            const unsigned long long w =
                k >= 0 ? __hip_atomic_load(word + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : (2ull << 32);
            const unsigned st = (unsigned)(w >> 32);
            const uint64_t inc = __ballot(st == 2), zero = __ballot(st == 0);
            const int first = inc ? __ffsll((unsigned long long)inc) - 1 : 64;  // nearest inclusive predecessor
            const uint64_t upto = first == 64 ? ~0ull : (first == 63 ? ~0ull : ((2ull << first) - 1));
            if (zero & upto) continue;  // a tile before it has not published yet
            int32_t v = lane <= first ? (int32_t)(uint32_t)w : 0;
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
            prefix += v;
            if (first < 64) break;
            j -= 64;
        }
        if (lane == 0) {
            __hip_atomic_store(word + tile, (2ull << 32) | (uint32_t)(prefix + total), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
            prefix_s = prefix;
        }
    }
    __syncthreads();
    int32_t run = prefix_s + wpre + x - tsum;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        if (i0 + j < n) out[i0 + j] = run;
        run += v[j];
    }
}
inline int64_t scan_tiles(int64_t n) { return (n + kScanTile - 1) / kScanTile; }

constexpr int kMaxContrib = 4;
constexpr int kChunk = 32;  // occurrences per reduction group: bounds the serial work of any group

struct Contribs {
    int64_t off[kMaxContrib];       // first flat occurrence index of the contribution
    int64_t n[kMaxContrib];         // occurrences covered
    const float* rows[kMaxContrib]; // (n, dim): the rows themselves, or h for scaled contributions
    const float* scale[kMaxContrib];// nullable: contribution t = scale[t] * rows[t]
    int count;
};

__device__ __forceinline__ void add4(float4& a, const float4& b) {
    a.x += b.x;
    a.y += b.y;
    a.z += b.z;
    a.w += b.w;
}

__device__ __forceinline__ float4 scale4(const float4& a, float s) {
    return make_float4(a.x * s, a.y * s, a.z * s, a.w * s);
}

// Fused optimizer step (asme_table_grad_reduce_apply): a finished gradient row of slot s is not stored but
// applied at once -- the lazy table Adam's real-gradient step from the staged row values (slot order) into the
// table row rows[s] -- exactly asme_lazy_adam_apply_staged's arithmetic on the same gradient values.
struct TableApply {
    const int64_t* rows;
    const float* sp;
    const float* sm;
    const float* sv;
    int32_t* last_step;
    float* p;
    float* m;
    float* v;
    const AdamHyper* hist;
    int32_t step;
};

__device__ __forceinline__ void apply_grad4(const TableApply& A, int64_t s, int dim, int c0, const float4& G) {
    const AdamHyper hp = A.hist[A.step];
    const int64_t so = s * dim + c0;
    // the staged rows are read once, here: non-temporal loads (same-box A/B: the pass 0.350 -> 0.316 ms)
    typedef float f4v __attribute__((ext_vector_type(4)));
    const f4v p4 = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(A.sp + so));
    const f4v m4 = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(A.sm + so));
    const f4v v4 = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(A.sv + so));
    float4 P = make_float4(p4.x, p4.y, p4.z, p4.w);
    float4 M = make_float4(m4.x, m4.y, m4.z, m4.w);
    float4 V = make_float4(v4.x, v4.y, v4.z, v4.w);
    adam_elem4(P, G, M, V, hp);
    const int64_t r = A.rows[s];
    const int64_t off = r * dim + c0;
    table_store4(A.p + off, P);
    table_store4(A.m + off, M);
    table_store4(A.v + off, V);
    if (c0 == 0) A.last_step[r] = A.step;
}

// Pass 1: one 32-lane group per chunk of kChunk consecutive sorted occurrences (float4 per lane).  A slot
// whose occurrence list lies inside the chunk gets its final row; the list cut by the chunk's start is
// left in head[chunk], the list cut by its end in tail[chunk] (a chunk inside one list: head).  Each lane
// first resolves one occurrence (slot, source row, scale: coalesced loads) into LDS; the group then walks
// the chunk with eight row gathers in flight.
constexpr int kChunkGroups = 8;  // 32-lane groups per 256-thread block
template <bool APPLY>
__global__ __launch_bounds__(256) void grad_chunk_kernel(const int32_t* __restrict__ order,
                                                         const int32_t* __restrict__ slot,
                                                         const int32_t* __restrict__ seg_off, int64_t n,
                                                         int64_t cap, int dim, Contribs C, float out_scale,
                                                         float* __restrict__ grad_rows, float* __restrict__ head,
                                                         float* __restrict__ tail, TableApply A) {
    __shared__ int32_t s_slot[kChunkGroups][kChunk];
    __shared__ const float* s_src[kChunkGroups][kChunk];
    __shared__ float s_sc[kChunkGroups][kChunk];
    const int lane = threadIdx.x & 31, g = threadIdx.x >> 5;
    const int64_t c = (int64_t)blockIdx.x * kChunkGroups + g;
    const int64_t i0 = c * kChunk;
    const int64_t i1 = i0 + kChunk < n ? i0 + kChunk : n;
    {
        const int64_t i = i0 + lane;
        int32_t sl = -1;
        const float* src = nullptr;
        float sc = 1.f;
        if (i < i1) {
            const int32_t k = slot[i];
            if (k < cap) {
                sl = k;
                const int64_t o = order[i];
                const float* sp = nullptr;
                int64_t t = 0;
#pragma unroll
                for (int q = 0; q < kMaxContrib; ++q)  // constant indices: the table stays in SGPRs
                    if (q < C.count && o >= C.off[q] && o < C.off[q] + C.n[q]) {
                        t = o - C.off[q];
                        src = C.rows[q] + t * dim;
                        sp = C.scale[q];
                    }
                if (sp) sc = sp[t];
            }
        }
        s_slot[g][lane] = sl;
        s_src[g][lane] = src;
        s_sc[g][lane] = sc;
    }
    __syncthreads();
    if (i0 >= n) return;
    const int32_t first = s_slot[g][0];
    if (first < 0) return;  // only slot-less occurrences from here on
    const int cnt = (int)(i1 - i0);
    for (int c0 = 4 * lane; c0 < dim; c0 += 128) {
        int32_t cur = first;
        bool started = seg_off[cur] == i0;
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        auto flush = [&](bool ended) {
            if (started && ended) {
                if constexpr (APPLY)
                    apply_grad4(A, cur, dim, c0, scale4(acc, out_scale));
                else
                    *reinterpret_cast<float4*>(grad_rows + (int64_t)cur * dim + c0) = scale4(acc, out_scale);
            } else
                *reinterpret_cast<float4*>((started ? tail : head) + c * dim + c0) = acc;
        };
        for (int j0 = 0; j0 < cnt; j0 += 8) {
            int32_t sl[8];
            float4 v[8];
            float sc[8];
            bool ok[8];
            // eight gathers before the dependent adds: unconditional global loads (an occurrence without a source row
            // reads the chunk's own head row instead, discarded below), scaled only once all eight are in flight --
            // a load inside the `ok` branch, scaled right after, was a flat load waited on before the next was issued
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int j = j0 + q;
                sl[q] = j < cnt ? s_slot[g][j] : -1;
                const float* src = j < cnt ? s_src[g][j] : nullptr;
                sc[q] = j < cnt ? s_sc[g][j] : 0.f;
                ok[q] = sl[q] >= 0 && src;
                const float* a = ok[q] ? src + c0 : head + c0;
                const floatx4 x = *(const __attribute__((address_space(1))) floatx4*)a;
                v[q] = make_float4(x[0], x[1], x[2], x[3]);
            }
#pragma unroll
            for (int q = 0; q < 8; ++q) v[q] = ok[q] ? scale4(v[q], sc[q]) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                if (sl[q] < 0) break;
                if (sl[q] != cur) {
                    flush(true);
                    cur = sl[q];
                    started = true;
                    acc = make_float4(0.f, 0.f, 0.f, 0.f);
                }
                add4(acc, v[q]);
            }
        }
        flush(seg_off[cur + 1] <= i1);
    }
}

// Pass 2: slots whose list spans chunks: tail of the first chunk + heads of the following ones, in order.
// One 32-lane group per chunk boundary k (sorted position k * kChunk): the slot there spans chunks iff its list
// started in chunk k - 1; that boundary is the slot's first, so each spanning slot is summed exactly once (a grid
// over the boundaries, not over every slot: the spanning ones are few).
template <bool APPLY>
__global__ __launch_bounds__(256) void grad_span_kernel(const int32_t* __restrict__ slot,
                                                        const int32_t* __restrict__ seg_off,
                                                        const int32_t* __restrict__ count, int64_t n, int64_t cap,
                                                        int dim, float out_scale, const float* __restrict__ head,
                                                        const float* __restrict__ tail,
                                                        float* __restrict__ grad_rows, TableApply A) {
    const int lane = threadIdx.x & 31;
    const int64_t k = (((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 5) + 1;
    if (k * kChunk >= n) return;
    const int32_t s = slot[k * kChunk];
    if (s >= cap || s >= *count) return;
    const int64_t cf = seg_off[s] / kChunk;
    if (cf != k - 1) return;
    const int64_t cl = (seg_off[s + 1] - 1) / kChunk;
    for (int c0 = 4 * lane; c0 < dim; c0 += 128) {
        float4 acc = *reinterpret_cast<const float4*>(tail + cf * dim + c0);
        if (cl - cf <= 8) {
            for (int64_t q = cf + 1; q <= cl; ++q) add4(acc, *reinterpret_cast<const float4*>(head + q * dim + c0));
        } else {
            // a hot slot (PAD, MASK: tens of thousands of occurrences, > 1,000 chunk partials): kHotWays interleaved
            // partial sums (as many loads in flight), combined in a fixed tree -- still one fixed order
            // (deterministic).  8 ways left the 1,150 partials of a C3 batch's MASK row at 62 us (latency-bound).
            constexpr int kHotWays = 16;
            float4 pr[kHotWays];
#pragma unroll
            for (int u = 0; u < kHotWays; ++u) pr[u] = make_float4(0.f, 0.f, 0.f, 0.f);
            int64_t q = cf + 1;
            for (; q + kHotWays - 1 <= cl; q += kHotWays)
#pragma unroll
                for (int u = 0; u < kHotWays; ++u)
                    add4(pr[u], *reinterpret_cast<const float4*>(head + (q + u) * dim + c0));
            for (; q + 7 <= cl; q += 8)  // the tail: fewer than kHotWays partials, eight in flight
#pragma unroll
                for (int u = 0; u < 8; ++u) add4(pr[u], *reinterpret_cast<const float4*>(head + (q + u) * dim + c0));
            for (; q <= cl; ++q) add4(pr[0], *reinterpret_cast<const float4*>(head + q * dim + c0));
#pragma unroll
            for (int w = 1; w < kHotWays; w *= 2)
#pragma unroll
                for (int u = 0; u < kHotWays; u += 2 * w) add4(pr[u], pr[u + w]);
            add4(acc, pr[0]);
        }
        if constexpr (APPLY)
            apply_grad4(A, s, dim, c0, scale4(acc, out_scale));
        else
            *reinterpret_cast<float4*>(grad_rows + (int64_t)s * dim + c0) = scale4(acc, out_scale);
    }
}

}  // namespace

namespace {
size_t csr_up(size_t x) { return (x + 255) & ~(size_t)255; }
}  // namespace

ASME_API int64_t asme_occurrence_csr_workspace(int64_t n) {
    // per-key counts (n + 1), huge-range count + bounds + huge ticket (2 + 2 max_huge), the scan's tile counter and
    // tile words (1 + tiles, 64-bit), long-range list (n + 2), rank / sort scratch (n), key -> huge index (n + 1),
    // huge-key counts per placement block
    return (int64_t)(csr_up((size_t)(n + 1) * 4) + csr_up((size_t)(2 + 2 * max_huge(n)) * 4) +
                     csr_up((size_t)(1 + scan_tiles(n + 1)) * 8) + csr_up((size_t)(n + 2) * 4) +
                     csr_up((size_t)n * 4) + csr_up((size_t)(n + 1) * 4) + csr_up((size_t)kHugeFast * huge_blocks(n) * 4));
}

// inverse (n int64 slots < cap <= n) -> order (n int32 occurrence indices grouped by slot, increasing within a
// slot; occurrences without a slot last), sorted_slot (n int32: the slot of order[i], cap for none) and seg_off
// (cap + 1 int32: first sorted position of each slot, slots past the last one at the end of the slotted ones)
ASME_API int asme_occurrence_csr(const int64_t* inverse, int64_t n, int64_t cap, void* workspace,
                                 int64_t workspace_bytes, int32_t* order, int32_t* sorted_slot, int32_t* seg_off,
                                 void* stream) {
    ASME_CHECK_ARG(inverse && workspace && order && sorted_slot && seg_off, "asme_occurrence_csr: null pointer");
    ASME_CHECK_ARG(n >= 1 && n < (int64_t)1 << 31 && cap >= 0 && cap <= n, "asme_occurrence_csr: bad size");
    ASME_CHECK_ARG(workspace_bytes >= asme_occurrence_csr_workspace(n), "asme_occurrence_csr: workspace too small");
    hipStream_t s = (hipStream_t)stream;
    const int64_t nh = max_huge(n);
    char* ws = (char*)workspace;
    int32_t* cnt = (int32_t*)ws;
    int32_t* huge = (int32_t*)(ws + csr_up((size_t)(n + 1) * 4));
    int32_t* hbeg = huge + 1;
    int32_t* hend = hbeg + nh;
    unsigned long long* scan_state = (unsigned long long*)((char*)huge + csr_up((size_t)(2 + 2 * nh) * 4));
    int32_t* longs = (int32_t*)((char*)scan_state + csr_up((size_t)(1 + scan_tiles(cap + 1)) * 8));
    int32_t* tmp = (int32_t*)((char*)longs + csr_up((size_t)(n + 2) * 4));
    int32_t* hidx = (int32_t*)((char*)tmp + csr_up((size_t)n * 4));
    int32_t* cntm = (int32_t*)((char*)hidx + csr_up((size_t)(n + 1) * 4));
    const int64_t nblk_h = huge_blocks(n);
    // counts of keys 0..cap, the huge-range count and bounds, the scan's tile words, the long-range counter: zeroed
    // together (contiguous)
    if (hipMemsetAsync(cnt, 0, (char*)longs - ws + 4, s) != hipSuccess)
        return hip_status(hipGetLastError(), "asme_occurrence_csr: zero");
    hipLaunchKernelGGL(csr_count_kernel, dim3(nblk_occ(n)), dim3(256), 0, s, inverse, n, cap, cnt);
    hipLaunchKernelGGL(chained_scan_kernel, dim3((unsigned)scan_tiles(cap + 1)), dim3(256), 0, s, cnt, cap + 1, seg_off,
                       scan_state);
    hipLaunchKernelGGL(csr_scatter_kernel, dim3(nblk_occ(n)), dim3(256), 0, s, inverse, n, cap, seg_off, cnt, order,
                       sorted_slot);
    hipLaunchKernelGGL(csr_order_kernel, dim3(nblk(cap + 1)), dim3(256), 0, s, seg_off, n, cap, order, longs, huge,
                       hbeg, hend, hidx);
    // long ranges ranked and (a huge range is possible) huge keys counted in one launch, then the stable placement
    const int64_t hblocks = n > kLongSeg ? nblk_h : 0;
    hipLaunchKernelGGL(csr_long_huge_kernel, dim3((unsigned)(kLongBlocks + hblocks)), dim3(256), 0, s, inverse, seg_off,
                       n, cap, longs, order, tmp, hidx, huge, hbeg, cntm, nblk_h);
    if (n > kLongSeg) {
        hipLaunchKernelGGL(csr_huge_scan_kernel, dim3(kHugeFast), dim3(64), 0, s, huge, hbeg, cntm, nblk_h);
        hipLaunchKernelGGL(csr_huge_place_kernel, dim3((unsigned)nblk_h), dim3(256), 0, s, inverse, n, cap, hidx, huge,
                           cntm, nblk_h, order);
    }
    ASME_LAUNCH_CHECK("asme_occurrence_csr");
}

ASME_API int64_t asme_table_grad_workspace(int64_t n, int64_t dim) {
    return 2 * ((n + kChunk - 1) / kChunk) * dim * (int64_t)sizeof(float);
}

namespace {

int table_grad_launch(const int32_t* order, const int32_t* sorted_slot, const int32_t* seg_off, const int32_t* count,
                      int64_t n, int64_t cap, int64_t dim, int n_contrib, const int64_t* c_off, const int64_t* c_n,
                      const float* const* c_rows, const float* const* c_scale, float out_scale, void* workspace,
                      int64_t workspace_bytes, float* grad_rows, const TableApply* apply, void* stream) {
    ASME_CHECK_ARG(order && sorted_slot && seg_off && count && (grad_rows || apply) && c_off && c_n && c_rows,
                   "asme_table_grad_reduce: null");
    ASME_CHECK_ARG(n_contrib >= 1 && n_contrib <= kMaxContrib, "asme_table_grad_reduce: 1..4 contributions");
    ASME_CHECK_ARG(dim > 0 && dim % 4 == 0 && ((uintptr_t)grad_rows & 15) == 0,
                   "asme_table_grad_reduce: dim % 4 == 0, 16-B aligned rows");
    ASME_CHECK_ARG(workspace_bytes >= asme_table_grad_workspace(n, dim) && (workspace || n == 0),
                   "asme_table_grad_reduce: workspace too small");
    Contribs C{};
    C.count = n_contrib;
    for (int k = 0; k < n_contrib; ++k) {
        C.off[k] = c_off[k];
        C.n[k] = c_n[k];
        C.rows[k] = c_rows[k];
        C.scale[k] = c_scale ? c_scale[k] : nullptr;
        ASME_CHECK_ARG(c_rows[k] && ((uintptr_t)c_rows[k] & 15) == 0, "asme_table_grad_reduce: rows 16-B aligned");
        ASME_CHECK_ARG(k == 0 || c_off[k] >= c_off[k - 1] + c_n[k - 1], "asme_table_grad_reduce: sorted, disjoint");
    }
    if (n == 0 || cap == 0) return 0;
    hipStream_t s = (hipStream_t)stream;
    const int64_t nchunks = (n + kChunk - 1) / kChunk;
    float* head = (float*)workspace;
    float* tail = head + nchunks * dim;
    const TableApply A = apply ? *apply : TableApply{};
    const dim3 gc((unsigned)((nchunks + kChunkGroups - 1) / kChunkGroups));
    const dim3 gs((unsigned)(((nchunks > 1 ? nchunks - 1 : 1) * 32 + 255) / 256));
    if (apply) {
        hipLaunchKernelGGL(grad_chunk_kernel<true>, gc, dim3(256), 0, s, order, sorted_slot, seg_off, n, cap, (int)dim,
                           C, out_scale, grad_rows, head, tail, A);
        if (nchunks > 1)
            hipLaunchKernelGGL(grad_span_kernel<true>, gs, dim3(256), 0, s, sorted_slot, seg_off, count, n, cap,
                               (int)dim, out_scale, head, tail, grad_rows, A);
    } else {
        hipLaunchKernelGGL(grad_chunk_kernel<false>, gc, dim3(256), 0, s, order, sorted_slot, seg_off, n, cap,
                           (int)dim, C, out_scale, grad_rows, head, tail, A);
        if (nchunks > 1)
            hipLaunchKernelGGL(grad_span_kernel<false>, gs, dim3(256), 0, s, sorted_slot, seg_off, count, n, cap,
                               (int)dim, out_scale, head, tail, grad_rows, A);
    }
    ASME_LAUNCH_CHECK("asme_table_grad_reduce");
}

}  // namespace

// grad_rows[s] = out_scale * sum over slot s's occurrences of their contribution rows, in a fixed order
// (chunks of 32 sorted occurrences, then chunk partials in order: bit-reproducible).  Contribution k covers
// flat occurrences [c_off[k], c_off[k] + c_n[k]): row t = c_rows[k][t] (* c_scale[k][t]).  Host arrays of at
// most 4 contributions, sorted by c_off and disjoint; dim % 4 == 0.  Rows of slots >= *count are untouched.
ASME_API int asme_table_grad_reduce(const int32_t* order, const int32_t* sorted_slot, const int32_t* seg_off,
                                    const int32_t* count, int64_t n, int64_t cap, int64_t dim, int n_contrib,
                                    const int64_t* c_off, const int64_t* c_n, const float* const* c_rows,
                                    const float* const* c_scale, float out_scale, void* workspace,
                                    int64_t workspace_bytes, float* grad_rows, void* stream) {
    return table_grad_launch(order, sorted_slot, seg_off, count, n, cap, dim, n_contrib, c_off, c_n, c_rows, c_scale,
                             out_scale, workspace, workspace_bytes, grad_rows, nullptr, stream);
}

// The same sums, each finished row applied at once as the lazy table Adam's real-gradient step instead of being
// stored: from the staged values sp/sm/sv[s] into param/exp_avg/exp_avg_sq[rows[s]], last_step[rows[s]] = step --
// bit-identical to asme_table_grad_reduce followed by asme_lazy_adam_apply_staged, without the gradient rows'
// round trip through HBM.  dim % 4 == 0; every pointer 16-B aligned.
ASME_API int asme_table_grad_reduce_apply(const int32_t* order, const int32_t* sorted_slot, const int32_t* seg_off,
                                          const int32_t* count, int64_t n, int64_t cap, int64_t dim, int n_contrib,
                                          const int64_t* c_off, const int64_t* c_n, const float* const* c_rows,
                                          const float* const* c_scale, float out_scale, void* workspace,
                                          int64_t workspace_bytes, const int64_t* rows, const float* sp,
                                          const float* sm, const float* sv, int32_t* last_step, float* param,
                                          float* exp_avg, float* exp_avg_sq, const float* hist, int64_t hist_cap,
                                          int64_t step, void* stream) {
    ASME_CHECK_ARG(rows && sp && sm && sv && last_step && param && exp_avg && exp_avg_sq && hist,
                   "asme_table_grad_reduce_apply: null pointer");
    ASME_CHECK_ARG(step >= 1 && step < hist_cap, "asme_table_grad_reduce_apply: step outside the history");
    ASME_CHECK_ARG(((((uintptr_t)sp) | ((uintptr_t)sm) | ((uintptr_t)sv) | ((uintptr_t)param) | ((uintptr_t)exp_avg) |
                     ((uintptr_t)exp_avg_sq)) & 15) == 0,
                   "asme_table_grad_reduce_apply: 16-B aligned rows");
    const TableApply A{rows, sp, sm, sv, last_step, param, exp_avg, exp_avg_sq,
                       reinterpret_cast<const AdamHyper*>(hist), (int32_t)step};
    return table_grad_launch(order, sorted_slot, seg_off, count, n, cap, dim, n_contrib, c_off, c_n, c_rows, c_scale,
                             out_scale, workspace, workspace_bytes, nullptr, &A, stream);
}
