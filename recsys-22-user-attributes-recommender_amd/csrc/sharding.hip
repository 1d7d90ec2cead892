// Item-id deduplication and row-shard bucketing on gfx950.
//
// Used by (a) the sparse-gradient dense-Adam path of the item table (row_slot map) and (b) the
// row-sharded item table (cyclic shard: global row g -> owner g % W, local row g / W), whose
// lookups/gradients cross ranks with RCCL all-to-all.  The reference has no such code:
// it runs nn.Embedding with a dense gradient under Lightning DDP.
//
// Dedup is deterministic: a |V|-sized int32 map (all -1 at rest) gets atomicMin(i) per occurrence,
// so each distinct id's representative is its FIRST occurrence; a device exclusive scan over the
// representative flags assigns compact slots in first-occurrence order.  The map is then rewritten
// to hold the slot (row_slot for the Adam kernel) and must be reset with asme_dedup_reset.
#include <hipcub/hipcub.hpp>

#include "common.h"

using namespace asme;

namespace {

__global__ void claim_kernel(const int64_t* __restrict__ ids, int64_t n, int64_t V, int32_t* __restrict__ map) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t id = ids[i];
    if (id < 0 || id >= V) return;
    atomicMin(reinterpret_cast<unsigned int*>(map + id), (unsigned int)i);
}

__global__ void flag_kernel(const int64_t* __restrict__ ids, int64_t n, int64_t V, const int32_t* __restrict__ map,
                            int32_t* __restrict__ flags) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t id = ids[i];
    flags[i] = (id >= 0 && id < V && map[id] == (int32_t)i) ? 1 : 0;
}

__global__ void compact_kernel(const int64_t* __restrict__ ids, int64_t n, const int32_t* __restrict__ flags,
                               const int32_t* __restrict__ scan, int64_t* __restrict__ unique,
                               int32_t* __restrict__ count) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (flags[i]) unique[scan[i]] = ids[i];
    if (i == n - 1) *count = scan[i] + flags[i];
}

// after compaction: map[unique[s]] = s
__global__ void slot_kernel(const int64_t* __restrict__ unique, const int32_t* __restrict__ count,
                            int32_t* __restrict__ map, int64_t cap) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= cap || s >= *count) return;
    map[unique[s]] = (int32_t)s;
}

__global__ void inverse_kernel(const int64_t* __restrict__ ids, int64_t n, int64_t V, const int32_t* __restrict__ map,
                               int64_t* __restrict__ inverse) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t id = ids[i];
    inverse[i] = (id >= 0 && id < V) ? (int64_t)map[id] : -1;
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

}  // namespace

ASME_API int64_t asme_dedup_workspace_bytes(int64_t n) {
    size_t temp = 0;
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, temp, (int32_t*)nullptr, (int32_t*)nullptr, (int)n);
    // flags + scan (int32 each) + cub temp, 256-B aligned pieces
    auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
    return (int64_t)(2 * up((size_t)n * sizeof(int32_t)) + up(temp));
}

// ids (n) -> unique (cap >= n) in first-occurrence order, inverse (n) slot per occurrence, count (1 int32 on device).
// map: |V| int32, all -1 on entry; on exit map[unique[s]] = s (call asme_dedup_reset afterwards).
ASME_API int asme_dedup_ids(const int64_t* ids, int64_t n, int64_t vocab, int32_t* map, void* workspace,
                            int64_t workspace_bytes, int64_t* unique, int64_t* inverse, int32_t* count,
                            void* stream) {
    ASME_CHECK_ARG(ids && map && workspace && unique && count, "asme_dedup_ids: null pointer");
    ASME_CHECK_ARG(n >= 1 && n < (int64_t)1 << 31, "asme_dedup_ids: n must be in [1, 2^31)");
    ASME_CHECK_ARG(workspace_bytes >= asme_dedup_workspace_bytes(n), "asme_dedup_ids: workspace too small");
    hipStream_t s = (hipStream_t)stream;
    auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
    char* ws = (char*)workspace;
    int32_t* flags = (int32_t*)ws;
    int32_t* scan = (int32_t*)(ws + up((size_t)n * 4));
    void* temp = ws + 2 * up((size_t)n * 4);
    size_t temp_bytes = (size_t)workspace_bytes - 2 * up((size_t)n * 4);
    hipLaunchKernelGGL(claim_kernel, dim3(nblk(n)), dim3(256), 0, s, ids, n, vocab, map);
    hipLaunchKernelGGL(flag_kernel, dim3(nblk(n)), dim3(256), 0, s, ids, n, vocab, map, flags);
    if (hipcub::DeviceScan::ExclusiveSum(temp, temp_bytes, flags, scan, (int)n, s) != hipSuccess)
        return hip_status(hipErrorUnknown, "asme_dedup_ids: scan");
    hipLaunchKernelGGL(compact_kernel, dim3(nblk(n)), dim3(256), 0, s, ids, n, flags, scan, unique, count);
    hipLaunchKernelGGL(slot_kernel, dim3(nblk(n)), dim3(256), 0, s, unique, count, map, n);
    if (inverse) hipLaunchKernelGGL(inverse_kernel, dim3(nblk(n)), dim3(256), 0, s, ids, n, vocab, map, inverse);
    ASME_LAUNCH_CHECK("asme_dedup_ids");
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
