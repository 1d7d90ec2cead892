// GPU-side input producers for ASME's training batches.  The reference builds every
// sample in CPU DataLoader workers, one Python processor call per session; at |I| = 10M its negative sampler
// alone is O(|V|) per session (a dense multinomial weight vector, 46 ms/session).  Here sessions live in HBM
// (flat item ids + offsets) and one kernel per processor builds the padded (B, L) batch.
//
// Reference semantics (paths relative to /root/reference/src/asme):
//   collate (left-truncate to max_seq_length, right-pad with PAD)       data/collate.py:42-111
//   PositiveNegativeSamplerProcessor.process / _sample_negative_target  data/datasets/processors/pos_neg_sampler.py:41-63,89-106
//       x = s[:-1], pos = s[1:], neg ~ uniform over ids that are neither special nor anywhere in the session,
//       with replacement (torch.multinomial over 0/1 weights)
//   ClozeMaskProcessor.process                                         data/datasets/processors/cloze_mask.py:50-92
//       u0 <= p_last: mask only the last item, targets PAD elsewhere; else per position u < p: u/p < 0.8 MASK,
//       < 0.9 a random id in [0, |V|-1) (random_(0, len-1), utils.py:41-50), else keep; target = item; u >= p:
//       target PAD.  The comparisons are made in double, as Python does on the .item() of a float32 draw.
// Randomness: counter-based Philox4x32-10 (seed, sequence, position), so a batch is reproducible from its
// seed; the cloze kernel can instead take the draws (u per position, the random ids) from the caller, which
// is how the tests replay the reference's own torch CPU generator stream bit-exactly.
#include "common.h"

using namespace asme;

namespace {

constexpr int kWavesPerBlock = 4;
constexpr int kMaxSpecial = 8;
constexpr int kSessLds = 2048;  // session items staged in LDS per workgroup (16 KiB)

__device__ __forceinline__ float u01(uint32_t x) { return (float)(x >> 8) * 5.9604644775390625e-08f; }

// ---------------------------------------------------------------------------------------------- collate
// out (B, L): the last min(len, L) items of session batch_idx[b] (left truncation), PAD after; out_len = that count
__global__ __launch_bounds__(256) void session_batch_kernel(const int64_t* __restrict__ flat,
                                                            const int64_t* __restrict__ offsets, int64_t n_sessions,
                                                            const int64_t* __restrict__ batch_idx, int64_t B,
                                                            int64_t L, int64_t drop_last, int64_t pad,
                                                            int64_t* __restrict__ out, int64_t* __restrict__ out_len) {
    const int64_t b = blockIdx.x;
    if (b >= B) return;
    const int64_t s = batch_idx[b];
    const bool ok = s >= 0 && s < n_sessions;
    const int64_t beg = ok ? offsets[s] : 0, end = ok ? offsets[s + 1] - drop_last : 0;
    const int64_t m = end > beg ? end - beg : 0;
    const int64_t n = m < L ? m : L;
    const int64_t first = end - n;
    for (int64_t i = threadIdx.x; i < L; i += blockDim.x) out[b * L + i] = i < n ? flat[first + i] : pad;
    if (threadIdx.x == 0 && out_len) out_len[b] = n;
}

// (session, target position) pairs of ASME's position indices (data/datasets/index.py; LOO / next-item splits):
// SequencePositionDataset truncates the session to [:pos + 1] (sequence_position.py:50-58) and the target extractor
// splits off the last item (target_extractor.py:41-70): out = the last min(pos, L) items before pos, target = s[pos]
__global__ __launch_bounds__(256) void position_batch_kernel(const int64_t* __restrict__ flat,
                                                             const int64_t* __restrict__ offsets, int64_t n_sessions,
                                                             const int64_t* __restrict__ pairs, int64_t B, int64_t L,
                                                             int64_t pad, int64_t* __restrict__ out,
                                                             int64_t* __restrict__ out_len,
                                                             int64_t* __restrict__ target, int* __restrict__ err) {
    const int64_t b = blockIdx.x;
    if (b >= B) return;
    const int64_t s = pairs[2 * b], p = pairs[2 * b + 1];
    const bool ok = s >= 0 && s < n_sessions && p >= 0 && p < offsets[s + 1] - offsets[s];
    if (!ok && threadIdx.x == 0 && err) atomicOr(err, 1);
    const int64_t beg = ok ? offsets[s] : 0;
    const int64_t n = ok ? (p < L ? p : L) : 0;
    const int64_t first = beg + p - n;
    for (int64_t i = threadIdx.x; i < L; i += blockDim.x) out[b * L + i] = i < n ? flat[first + i] : pad;
    if (threadIdx.x == 0) {
        if (out_len) out_len[b] = n;
        if (target) target[b] = ok ? flat[beg + p] : pad;
    }
}

// LastItemMaskProcessor (data/datasets/processors/last_item_mask.py:35-44) ahead of the collate: the session gets
// the MASK token appended, then the collate keeps the last L_out entries, right-padded.  On an already collated
// row (the last min(len, L_in) items, L_in >= L_out - 1) that is: the last min(len, L_out - 1) items, MASK, PAD.
__global__ __launch_bounds__(256) void last_item_mask_kernel(const int64_t* __restrict__ items,
                                                             const int64_t* __restrict__ lengths, int64_t B,
                                                             int64_t L_in, int64_t L_out, int64_t mask_id, int64_t pad,
                                                             int64_t* __restrict__ out, int64_t* __restrict__ out_len) {
    const int64_t b = blockIdx.x;
    if (b >= B) return;
    int64_t len = lengths[b];
    len = len < 0 ? 0 : (len > L_in ? L_in : len);
    const int64_t keep = len < L_out - 1 ? len : L_out - 1;  // items kept before the MASK
    const int64_t first = len - keep;
    for (int64_t i = threadIdx.x; i < L_out; i += blockDim.x)
        out[b * L_out + i] = i < keep ? items[b * L_in + first + i] : (i == keep ? mask_id : pad);
    if (threadIdx.x == 0 && out_len) out_len[b] = keep + 1;
}

// ------------------------------------------------------------------------------------- pos / neg sampler
// One workgroup per session.  x, pos: the collated s[:-1], s[1:]; neg: for each kept position one id drawn uniformly
// from [0, V) and redrawn (next Philox counter) while it is special or occurs ANYWHERE in the full session (the
// exclusion set of the reference is the whole session, not the truncated window).  err bit 0: a session with
// no admissible id (the reference's multinomial raises), bit 1: a session shorter than 2 (AssertionError).
__global__ __launch_bounds__(256) void posneg_kernel(const int64_t* __restrict__ flat,
                                                     const int64_t* __restrict__ offsets, int64_t n_sessions,
                                                     const int64_t* __restrict__ batch_idx, int64_t B, int64_t L,
                                                     int64_t V, const int64_t* __restrict__ special, int n_special,
                                                     int64_t pad, uint64_t seed, int64_t* __restrict__ x,
                                                     int64_t* __restrict__ pos, int64_t* __restrict__ neg,
                                                     int64_t* __restrict__ out_len, int* __restrict__ err) {
    // one workgroup per session; its waves take the 64-position chunks in turn (one wave per session left a
    // 1,024-session batch with one wave per SIMD and every latency exposed)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t b = blockIdx.x;
    if (b >= B) return;  // (workgroup-uniform)
    const int64_t s = batch_idx[b];
    const bool ok = s >= 0 && s < n_sessions;
    const int64_t beg = ok ? offsets[s] : 0, end = ok ? offsets[s + 1] : 0;
    const int64_t m = end - beg;  // session length (x, pos, neg have m - 1 entries before truncation)
    if (m < 2) {
        if (threadIdx.x == 0 && err) atomicOr(err, 2);
        for (int64_t i = threadIdx.x; i < L; i += blockDim.x) x[b * L + i] = pos[b * L + i] = neg[b * L + i] = pad;
        if (threadIdx.x == 0 && out_len) out_len[b] = 0;
        return;
    }
    const int64_t n = (m - 1) < L ? (m - 1) : L;  // kept positions: the last n of the m - 1
    const int64_t first = m - 1 - n;              // index (into x) of the first kept position
    // the session (the exclusion set) staged in LDS when it fits (else scanned in place)
    __shared__ int64_t sl[kSessLds];
    const bool in_lds = m <= kSessLds;
    if (in_lds)
        for (int64_t j = threadIdx.x; j < m; j += blockDim.x) sl[j] = flat[beg + j];
    __syncthreads();
    int64_t sp[kMaxSpecial];
#pragma unroll
    for (int k = 0; k < kMaxSpecial; ++k) sp[k] = k < n_special ? special[k] : -1;
    bool any_fail = false;
    for (int64_t i0 = 64 * wave; i0 < L; i0 += 64 * kWavesPerBlock) {
        const int64_t i = i0 + lane;
        const bool live = i < n;
        int64_t cand = pad;
        bool need = live;
        uint32_t attempt = 0;
        // wave-uniform retry loop: every lane tests its candidate against the whole session
        while (__ballot(need) != 0ull) {
            if (need) {
                u32x4 c{(uint32_t)b, (uint32_t)(first + i), attempt, 0x9E3779B9u};
                const u32x4 r = philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
                const uint64_t wide = ((uint64_t)r.x << 32) | r.y;
                cand = (int64_t)(wide % (uint64_t)V);  // bias < V / 2^64
                bool bad = false;
#pragma unroll
                for (int k = 0; k < kMaxSpecial; ++k) bad = bad || cand == sp[k];
                // eight independent reads per trip (indices clamped to the session, no short circuit), from the LDS
                // copy by LDS instructions: with one wave per SIMD every dependent round trip of the one-at-a-time
                // scan through a generic pointer was exposed (66 us per 1,024-session batch)
                auto scan8 = [&](const int64_t* src) {
                    for (int64_t j = 0; j < m && !bad; j += 8) {
                        int64_t v8[8];
#pragma unroll
                        for (int u = 0; u < 8; ++u) v8[u] = src[j + u < m ? j + u : m - 1];
                        __builtin_amdgcn_sched_barrier(0);  // all eight reads issued before the first compare
                        bool hit = false;
#pragma unroll
                        for (int u = 0; u < 8; ++u) hit |= v8[u] == cand;
                        bad = hit;
                    }
                };
                if (!bad) {
                    if (in_lds)
                        scan8(sl);
                    else
                        scan8(flat + beg);
                }
                need = bad && ++attempt < 4096u;
                if (bad && !need) {
                    any_fail = true;
                    cand = pad;
                }
            }
        }
        if (i < L) {
            x[b * L + i] = live ? flat[beg + first + i] : pad;
            pos[b * L + i] = live ? flat[beg + first + i + 1] : pad;
            neg[b * L + i] = live ? cand : pad;
        }
    }
    if (__ballot(any_fail) && lane == 0 && err) atomicOr(err, 1);
    if (threadIdx.x == 0 && out_len) out_len[b] = n;
}

// ------------------------------------------------------------------------------------------------ cloze
// items / lengths: the collated (B, L) batch.  draws_u (B, L + 1) and draws_r (B, L) optional (replay).
__global__ __launch_bounds__(256) void cloze_kernel(const int64_t* __restrict__ items,
                                                    const int64_t* __restrict__ lengths, int64_t B, int64_t L,
                                                    int64_t V, int64_t pad, int64_t mask_id, double mask_prob,
                                                    double last_prob, const float* __restrict__ draws_u,
                                                    const int64_t* __restrict__ draws_r, uint64_t seed,
                                                    int64_t* __restrict__ out, int64_t* __restrict__ target) {
    const int64_t b = blockIdx.x;
    if (b >= B) return;
    const int64_t n = lengths[b] < L ? lengths[b] : L;
    auto uniform = [&](int64_t k) -> float {  // k = 0: the last-item decision, 1 + i: position i
        if (draws_u) return draws_u[b * (L + 1) + k];
        u32x4 c{(uint32_t)b, (uint32_t)k, 0x243F6A88u, 0x85A308D3u};
        return u01(philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32)).x);
    };
    auto random_id = [&](int64_t i) -> int64_t {  // random_(0, V - 1): uniform in [0, V - 1)
        if (draws_r) return draws_r[b * L + i];
        u32x4 c{(uint32_t)b, (uint32_t)i, 0x13198A2Eu, 0x03707344u};
        const u32x4 r = philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
        return (int64_t)((((uint64_t)r.x << 32) | r.y) % (uint64_t)(V - 1));
    };
    const bool last_only = n > 0 && (double)uniform(0) <= last_prob;
    for (int64_t i = threadIdx.x; i < L; i += blockDim.x) {
        const int64_t it = items[b * L + i];
        int64_t o = it, t = pad;
        if (i < n) {
            if (last_only) {
                if (i == n - 1) {
                    o = mask_id;
                    t = it;
                }
            } else {
                const double u = (double)uniform(1 + i);
                if (u < mask_prob) {
                    const double q = u / mask_prob;
                    if (q < 0.8) o = mask_id;
                    else if (q < 0.9) o = random_id(i);
                    t = it;
                }
            }
        }
        out[b * L + i] = i < n ? o : pad;
        target[b * L + i] = t;
    }
}

// ------------------------------------------------------------------------------------------ padding mask
// out[i] = seq[i] != pad (modules.get_padding_mask, the reference's input.ne(pad_token_id)); four ids per thread,
// one 4-byte store of their four flags
__global__ __launch_bounds__(256) void padding_mask_kernel(const int64_t* __restrict__ seq, int64_t n, int64_t pad,
                                                           uint8_t* __restrict__ out) {
    const int64_t i0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
    if (i0 + 3 < n) {
        const longlong2 a = *reinterpret_cast<const longlong2*>(seq + i0);
        const longlong2 b = *reinterpret_cast<const longlong2*>(seq + i0 + 2);
        const uint32_t w = (uint32_t)(a.x != pad) | (uint32_t)(a.y != pad) << 8 | (uint32_t)(b.x != pad) << 16 |
                           (uint32_t)(b.y != pad) << 24;
        *reinterpret_cast<uint32_t*>(out + i0) = w;
    } else {
        for (int64_t i = i0; i < n; ++i) out[i] = seq[i] != pad;
    }
}

}  // namespace

ASME_API int asme_session_batch(const int64_t* flat, const int64_t* offsets, int64_t n_sessions,
                                const int64_t* batch_idx, int64_t batch, int64_t seq_len, int64_t drop_last,
                                int64_t pad, int64_t* out, int64_t* out_len, void* stream) {
    ASME_CHECK_ARG(flat && offsets && batch_idx && out, "asme_session_batch: null pointer");
    ASME_CHECK_ARG(seq_len >= 1 && batch >= 0 && drop_last >= 0, "asme_session_batch: bad shape");
    if (batch == 0) return 0;
    hipLaunchKernelGGL(session_batch_kernel, dim3((unsigned)batch), dim3(256), 0, (hipStream_t)stream, flat, offsets,
                       n_sessions, batch_idx, batch, seq_len, drop_last, pad, out, out_len);
    ASME_LAUNCH_CHECK("asme_session_batch");
}

ASME_API int asme_position_batch(const int64_t* flat, const int64_t* offsets, int64_t n_sessions,
                                 const int64_t* pairs, int64_t batch, int64_t seq_len, int64_t pad, int64_t* out,
                                 int64_t* out_len, int64_t* target, int* err_flag, void* stream) {
    ASME_CHECK_ARG(flat && offsets && pairs && out, "asme_position_batch: null pointer");
    ASME_CHECK_ARG(seq_len >= 1 && batch >= 0, "asme_position_batch: bad shape");
    if (batch == 0) return 0;
    hipLaunchKernelGGL(position_batch_kernel, dim3((unsigned)batch), dim3(256), 0, (hipStream_t)stream, flat, offsets,
                       n_sessions, pairs, batch, seq_len, pad, out, out_len, target, err_flag);
    ASME_LAUNCH_CHECK("asme_position_batch");
}

// items (B, L_in) right-padded sessions with lengths (B,) -> out (B, L_out): MASK appended after the last item,
// left-truncated to L_out, right-padded; out_len = the new lengths (nullable)
ASME_API int asme_last_item_mask(const int64_t* items, const int64_t* lengths, int64_t batch, int64_t in_len,
                                 int64_t out_len_max, int64_t mask_id, int64_t pad, int64_t* out, int64_t* out_len,
                                 void* stream) {
    ASME_CHECK_ARG(items && lengths && out, "asme_last_item_mask: null pointer");
    ASME_CHECK_ARG(batch >= 0 && out_len_max >= 1 && in_len >= out_len_max - 1 && in_len >= 0,
                   "asme_last_item_mask: bad shape (needs in_len >= out_len - 1)");
    if (batch == 0) return 0;
    hipLaunchKernelGGL(last_item_mask_kernel, dim3((unsigned)batch), dim3(256), 0, (hipStream_t)stream, items, lengths,
                       batch, in_len, out_len_max, mask_id, pad, out, out_len);
    ASME_LAUNCH_CHECK("asme_last_item_mask");
}

ASME_API int asme_posneg_sample(const int64_t* flat, const int64_t* offsets, int64_t n_sessions,
                                const int64_t* batch_idx, int64_t batch, int64_t seq_len, int64_t vocab,
                                const int64_t* special_ids, int n_special, int64_t pad, uint64_t seed, int64_t* x,
                                int64_t* pos, int64_t* neg, int64_t* out_len, int* err_flag, void* stream) {
    ASME_CHECK_ARG(flat && offsets && batch_idx && x && pos && neg, "asme_posneg_sample: null pointer");
    ASME_CHECK_ARG(seq_len >= 1 && batch >= 0 && vocab >= 1, "asme_posneg_sample: bad shape");
    ASME_CHECK_ARG(n_special >= 0 && n_special <= kMaxSpecial && (n_special == 0 || special_ids),
                   "asme_posneg_sample: at most 8 special ids");
    if (batch == 0) return 0;
    hipLaunchKernelGGL(posneg_kernel, dim3((unsigned)batch), dim3(64 * kWavesPerBlock), 0, (hipStream_t)stream, flat, offsets,
                       n_sessions, batch_idx, batch, seq_len, vocab, special_ids, n_special, pad, seed, x, pos, neg,
                       out_len, err_flag);
    ASME_LAUNCH_CHECK("asme_posneg_sample");
}

ASME_API int asme_cloze_mask(const int64_t* items, const int64_t* lengths, int64_t batch, int64_t seq_len,
                             int64_t vocab, int64_t pad, int64_t mask_id, double mask_prob, double last_prob,
                             const float* draws_u, const int64_t* draws_r, uint64_t seed, int64_t* out,
                             int64_t* target, void* stream) {
    ASME_CHECK_ARG(items && lengths && out && target, "asme_cloze_mask: null pointer");
    ASME_CHECK_ARG(seq_len >= 1 && batch >= 0 && vocab >= 2, "asme_cloze_mask: bad shape");
    ASME_CHECK_ARG(mask_prob > 0.0 && mask_prob <= 1.0 && last_prob >= 0.0 && last_prob <= 1.0,
                   "asme_cloze_mask: probabilities out of range");
    if (batch == 0) return 0;
    hipLaunchKernelGGL(cloze_kernel, dim3((unsigned)batch), dim3(256), 0, (hipStream_t)stream, items, lengths, batch,
                       seq_len, vocab, pad, mask_id, mask_prob, last_prob, draws_u, draws_r, seed, out, target);
    ASME_LAUNCH_CHECK("asme_cloze_mask");
}

// flags[i] = seq[i] != pad for n int64 ids (16-B aligned): the model's padding mask (modules.get_padding_mask)
ASME_API int asme_padding_mask(const int64_t* seq, int64_t n, int64_t pad, uint8_t* flags, void* stream) {
    ASME_CHECK_ARG(seq && flags, "asme_padding_mask: null pointer");
    ASME_CHECK_ARG(((uintptr_t)seq & 15) == 0 && ((uintptr_t)flags & 3) == 0, "asme_padding_mask: alignment");
    if (n <= 0) return 0;
    hipLaunchKernelGGL(padding_mask_kernel, dim3((unsigned)((n + 1023) / 1024)), dim3(256), 0, (hipStream_t)stream, seq,
                       n, pad, flags);
    ASME_LAUNCH_CHECK("asme_padding_mask");
}
