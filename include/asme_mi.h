/*
 * asme_mi.h — C ABI of libasme_mi.so: hand-written gfx950 (MI355X / CDNA4) HIP kernels for the
 * ASME sequential-recommender training/eval hot path.
 *
 * The reference (LSX-UniWue/recsys-22-user-attributes-recommender, "ASME") is pure Python on
 * PyTorch; it has no native FFI.  Each entry point below replaces the stock PyTorch op chain that
 * the cited reference function executes (paths relative to /root/reference/src/asme).  The Python
 * host package (recsys-22-user-attributes-recommender_amd/) binds them with ctypes and mirrors the
 * reference's model/module classes, so ASME's `imports:` plugin mechanism can swap them in
 * (see INTEGRATION.md).
 *
 * Conventions
 *   - All pointers are DEVICE pointers (caller-owned; kernels never allocate or free), except the
 *     pointer ARRAYS of asme_adam_step, which are host arrays of device pointers.
 *   - fp32 storage and fp32 arithmetic; ids are int64; masks are uint8 (0 / 1).  The Linear GEMMs
 *     (asme_ws_linear, asme_linear_weight_grad) form their fp32 products on the bf16 matrix cores from
 *     operands split exactly into three bf16 terms (six MFMAs per product tile, fp32 accumulation): error vs
 *     float64 at or below the fp32 MFMA's (DESIGN.md §4 "bf16x6").
 *   - `stream` is a hipStream_t (NULL = default stream).  Every call is asynchronous and
 *     stream-ordered; no call synchronises the device.
 *   - Return value: 0 = OK, -1 = invalid argument, -2 = HIP launch error.  The message of the last
 *     failure on the calling thread is returned by asme_mi_last_error().
 *   - Dropout uses a counter-based Philox4x32-10 keyed by (seed, element index), so forward and
 *     backward regenerate identical masks; p = 0 disables it.
 */
#ifndef ASME_MI_H
#define ASME_MI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status ------------------------------------------------------------------------------ */
const char* asme_mi_last_error(void);
int asme_mi_abi_version(void);

/* ---- embedding (core/models/common/layers/transformer_layers.py:55-80 TransformerEmbedding.forward,
 *      core/models/kebert4rec/components.py:54-63 PreFusion...forward) ------------------------------
 * out[t] = drop2( LN2( drop1( LN1( table[ids[t]] + pos_table[t % seq_len] ) ) + extra[t] ) )
 * Any of pos_table / LN1 (ln1_w,ln1_b) / extra / LN2 may be NULL (identity).  stats: (n_tokens, 4)
 * = mean1, rstd1, mean2, rstd2 for the backward.  err_flag (nullable) gets bit 0 set on an
 * out-of-range id (nn.Embedding would raise IndexError).  keep_mask (nullable; dim % 4 == 0 only):
 * (n_tokens, dim/4) bytes, byte c of token t = the dropout decisions of elements 4c..4c+3 (bit i: drop1
 * keeps element 4c+i, bit 4+i: drop2), written when p1 > 0 or p2 > 0 and read back by the backward. */
int asme_embedding_fwd(const int64_t* ids, int64_t n_tokens, int64_t seq_len, const float* table, int64_t vocab,
                       int64_t dim, const float* pos_table, const float* ln1_w, const float* ln1_b, float ln1_eps,
                       float p1, uint64_t seed1, const float* extra, const float* ln2_w, const float* ln2_b,
                       float ln2_eps, float p2, uint64_t seed2, float* out, float* stats, uint8_t* keep_mask,
                       int* err_flag, void* stream);
/* Backward of asme_embedding_fwd: d_rows (n_tokens, dim) = grad wrt (table row + pos row);
 * d_extra (nullable) = grad wrt extra; partials (n_partials, 4*dim) = per-block sums of
 * dLN1.w, dLN1.b, dLN2.w, dLN2.b (reduce with asme_reduce_rows). */
int asme_embedding_bwd(const int64_t* ids, int64_t n_tokens, int64_t seq_len, const float* table, int64_t vocab,
                       int64_t dim, const float* pos_table, const float* ln1_w, const float* ln1_b, float p1,
                       uint64_t seed1, const float* extra, const float* ln2_w, float p2, uint64_t seed2,
                       const uint8_t* keep_mask, const float* dout, const float* stats, float* d_rows,
                       float* d_extra, float* partials, int64_t n_partials, void* stream);
int asme_embedding_bwd_partials_count(void);
/* asme_embedding_fwd + the first transformer block's input LayerNorm (transformer_layers.py:251-258, the
 * SublayerConnection norm of block 0, which TransformerLayer applies to the embedding output) on the same rows:
 * out = the embedding output (the residual stream), ln3_out = LN3(out), ln3_stats (T, 2) = (mean, rstd).
 * Replaces asme_embedding_fwd followed by asme_layernorm_fwd on its output.  dim % 4 == 0. */
int asme_embedding_ln_fwd(const int64_t* ids, int64_t n_tokens, int64_t seq_len, const float* table, int64_t vocab,
                          int64_t dim, const float* pos_table, const float* ln1_w, const float* ln1_b, float ln1_eps,
                          float p1, uint64_t seed1, const float* extra, const float* ln2_w, const float* ln2_b,
                          float ln2_eps, float p2, uint64_t seed2, const float* ln3_w, const float* ln3_b,
                          float ln3_eps, float* out, float* stats, float* ln3_out, float* ln3_stats,
                          uint8_t* keep_mask, int* err_flag, void* stream);
/* Backward of asme_embedding_ln_fwd (replaces asme_layernorm_bwd_add + asme_embedding_bwd): dout = gradient of
 * `out` through the residual stream, dln = gradient of ln3_out; partials (n_partials, 6 * dim) = column partials
 * of LN1 w / b, LN2 w / b, LN3 w / b.  ln2_b is required with ln2_w. */
int asme_embedding_ln_bwd(const int64_t* ids, int64_t n_tokens, int64_t seq_len, const float* table, int64_t vocab,
                          int64_t dim, const float* pos_table, const float* ln1_w, const float* ln1_b, float p1,
                          uint64_t seed1, const float* extra, const float* ln2_w, const float* ln2_b, float p2,
                          uint64_t seed2, const float* ln3_w, const float* ln3_stats, const uint8_t* keep_mask,
                          const float* dout, const float* dln, const float* stats, float* d_rows, float* d_extra,
                          float* partials, int64_t n_partials, void* stream);
/* nn.Embedding dense backward (autograd embedding_dense_backward): grad[ids[r]] += scale * rows[r]
 * (hardware fp32 atomics; ids outside [0, vocab) are skipped). */
int asme_scatter_add_rows(const float* rows, const int64_t* ids, int64_t n_rows, int64_t dim, float* grad,
                          int64_t vocab, float scale, void* stream);
/* dest[ids[s]] = rows[s] for s < min(*count, cap) (device count; distinct ids): the dense nn.Embedding gradient
 * written from the deduplicated, occurrence-ordered row sums (replaces embedding_dense_backward's scatter-add,
 * core/models/common/layers/transformer_layers.py:55-80 item_embedding, without float atomics). */
int asme_scatter_rows(const float* rows, const int64_t* ids, const int32_t* count, int64_t cap, int64_t dim,
                      float* dest, int64_t vocab, void* stream);
/* position-embedding gradient: grad_pos[p] (+)= sum_b rows[b*seq_len + p]; workspace n_chunks*seq_len*dim */
int asme_position_grad(const float* rows, int64_t batch, int64_t seq_len, int64_t dim, float* workspace,
                       int64_t n_chunks, float* grad_pos, int accumulate, void* stream);
/* column sums of a (n_rows, width) matrix: out (+)= sum_r part[r] */
int asme_reduce_rows(const float* part, int64_t n_rows, int64_t width, float* out, int accumulate, void* stream);
/* attribute embeddings (core/models/kebert4rec/components.py:15-24; layers.py:15-27 LinearUpscaler):
 * out[t] (+)= bias + sum_k table[ids[t,k]] (ids == 0 skipped when skip_zero: the pad category) */
int asme_gather_sum_fwd(const int64_t* ids, int64_t n, int64_t k, int skip_zero, const float* table, int64_t vocab,
                        int64_t dim, const float* bias, float* out, int accumulate, void* stream);
int asme_gather_sum_bwd(const float* dout, const int64_t* ids, int64_t n, int64_t k, int skip_zero, float* grad,
                        int64_t vocab, int64_t dim, void* stream);

/* ---- transformer block pointwise (transformer_layers.py:120-130 SublayerConnection, :251-258
 *      TransformerBlock, :217-220 PositionwiseFeedForward; ffn_modifier.py:24-26) ---------------- */
int asme_layernorm_fwd(const float* x, int64_t n_rows, int64_t dim, const float* w, const float* b, float eps,
                       float* y, float* stats, void* stream);
int asme_layernorm_bwd(const float* x, int64_t n_rows, int64_t dim, const float* w, const float* stats,
                       const float* dy, float* dx, int accumulate, float* partials, int64_t n_partials, void* stream);
/* dx = LN backward of dy + dadd (nullable): the first block input feeds both its pre-LN and the residual, so its
 * two gradients are summed in the same pass (autograd's separate add, transformer_layers.py:120-130) */
int asme_layernorm_bwd_add(const float* x, int64_t n_rows, int64_t dim, const float* w, const float* stats,
                           const float* dy, const float* dadd, float* dx, float* partials, int64_t n_partials,
                           void* stream);
/* s = drop_b(res + drop_a(y)); ln_out = LN(s) (LN optional: w == NULL) */
int asme_residual_ln_fwd(const float* res, const float* y, int64_t n_rows, int64_t dim, float p_a, uint64_t seed_a,
                         float p_b, uint64_t seed_b, const float* w, const float* b, float eps, float* s_out,
                         float* ln_out, float* stats, void* stream);
/* d_res = drop_b'(d_s + LN'(d_ln)); d_y = drop_a'(d_res); partials (n_partials, 2*dim): dLN.w, dLN.b */
int asme_residual_ln_bwd(const float* s, int64_t n_rows, int64_t dim, float p_a, uint64_t seed_a, float p_b,
                         uint64_t seed_b, const float* w, const float* stats, const float* d_s, const float* d_ln,
                         float* d_res, float* d_y, float* partials, int64_t n_partials, void* stream);
/* y = drop(GELU_erf(x)) elementwise (16-B aligned buffers) */
int asme_gelu_dropout_fwd(const float* x, int64_t n, float p, uint64_t seed, float* y, void* stream);
int asme_gelu_dropout_bwd(const float* x, const float* dy, int64_t n, float p, uint64_t seed, float* dx,
                          void* stream);

/* ---- attention (transformer_layers.py:138-155 Attention.forward, :181-199 MultiHeadedAttention;
 *      core/models/transformer/sequence_representation.py:34-48 mask) -------------------------------
 * Q/K/V: token-major rows with row strides ld_*; head h = columns [h*head_dim, (h+1)*head_dim).
 * key_valid (batch, seq_len) uint8 (NULL = all valid); causal = tril mask (SASRec).
 * Masked scores are exactly -1e9 (reference masked_fill); out (n_tokens, heads*head_dim) with
 * stride ld_out; lse (batch*heads, seq_len, 2) = (row max, 1/row sum of exp) of the scaled, masked
 * scores (kept separate so a row with no admissible key keeps its exact 1/L weights).
 * head_dim in {16, 32, 64, 128}; seq_len <= 1024.  drop_mask (nullable; asme_attention_dropout_mask_bytes()
 * bytes): the forward records the dropout decisions (key-major 16-bit words, and query-major nibbles when the
 * backward's dQ pass will read them -- not when the resident backward stores dS) which the backward then reads instead
 * of regenerating them: an opaque record for the backward of the same shape and kernel family. */
int asme_attention_fwd(const float* q, const float* k, const float* v, int64_t ld_q, int64_t ld_k, int64_t ld_v,
                       const uint8_t* key_valid, int64_t batch, int64_t heads, int64_t seq_len, int64_t head_dim,
                       int causal, float scale, float p_drop, uint64_t seed, float* out, int64_t ld_out, float* lse,
                       uint8_t* drop_mask, void* stream);
/* workspace: asme_attention_bwd_workspace() bytes (row sums D_i = dO_i . O_i, then the dS image the resident
 * path's dK/dV pass stores for its dQ pass: (batch*heads) x Lp x Lp floats, Lp = seq_len rounded up to 16).
 * dq/dk/dv may be column blocks of one buffer. */
int64_t asme_attention_bwd_workspace(int64_t batch, int64_t heads, int64_t seq_len, int64_t head_dim);
int asme_attention_bwd(const float* q, const float* k, const float* v, int64_t ld_q, int64_t ld_k, int64_t ld_v,
                       const float* out, int64_t ld_out, const float* dout, int64_t ld_dout, const float* lse,
                       const uint8_t* key_valid, int64_t batch, int64_t heads, int64_t seq_len, int64_t head_dim,
                       int causal, float scale, float p_drop, uint64_t seed, const uint8_t* drop_mask, float* workspace,
                       float* dq, int64_t ld_dq, float* dk, int64_t ld_dk, float* dv, int64_t ld_dv, void* stream);
/* The same two calls with the kernel family chosen per call (kernel tests and same-process A/B timing; the product
 * entry points above always run family 0): 0 = automatic (one workgroup per (batch, head) with the head's operands
 * resident in LDS whenever 2*ceil(L/16)*16*(dk+4)*4 B fits 160 KiB, else the 64-row streaming kernels; the resident
 * backward runs dK/dV first, storing dS, then dQ = dS K), 1 = streaming kernels only, 2 = resident kernels with a
 * dQ pass that recomputes S and dP.  No process-wide state.  A drop_mask is read only by the backward of the family
 * whose forward wrote it. */
int asme_attention_fwd_kernels(int kernels, const float* q, const float* k, const float* v, int64_t ld_q,
                               int64_t ld_k, int64_t ld_v, const uint8_t* key_valid, int64_t batch, int64_t heads,
                               int64_t seq_len, int64_t head_dim, int causal, float scale, float p_drop, uint64_t seed,
                               float* out, int64_t ld_out, float* lse, uint8_t* drop_mask, void* stream);
int asme_attention_bwd_kernels(int kernels, const float* q, const float* k, const float* v, int64_t ld_q,
                               int64_t ld_k, int64_t ld_v, const float* out, int64_t ld_out, const float* dout,
                               int64_t ld_dout, const float* lse, const uint8_t* key_valid, int64_t batch,
                               int64_t heads, int64_t seq_len, int64_t head_dim, int causal, float scale, float p_drop,
                               uint64_t seed, const uint8_t* drop_mask, float* workspace, float* dq, int64_t ld_dq,
                               float* dk, int64_t ld_dk, float* dv, int64_t ld_dv, void* stream);
/* Size of the drop_mask buffer for asme_attention_fwd/bwd (p_drop > 0). */
int64_t asme_attention_dropout_mask_bytes(int64_t batch, int64_t heads, int64_t seq_len);

/* ---- Linear weight/bias gradient (autograd of nn.Linear in transformer_layers.py:175-220):
 * dW (out x in) (+)= dY^T X, db (out) (+)= sum_t dY, split over the token dimension into fp32 partial
 * slabs (workspace) summed in a fixed order.  Features and strides multiples of 4 floats. */
int64_t asme_linear_weight_grad_workspace(int64_t n_tokens, int64_t out_features, int64_t in_features);
int asme_linear_weight_grad(const float* dy, int64_t ld_dy, const float* x, int64_t ld_x, int64_t n_tokens,
                            int64_t out_features, int64_t in_features, float* workspace, int64_t workspace_bytes,
                            float* dw, float* db, int accumulate, void* stream);

/* ---- heads & losses -----------------------------------------------------------------------
 * sampled head (core/models/sasrec/components.py:34-44): pos_out[t] = <hidden[t], table[pos_ids[t]]> */
int asme_sampled_logits_fwd(const float* hidden, const float* table, const int64_t* pos_ids, const int64_t* neg_ids,
                            int64_t n_tokens, int64_t dim, int64_t vocab, float* pos_out, float* neg_out,
                            void* stream);
/* d_hidden[t] = g_pos[t] table[pos] + g_neg[t] table[neg]; d_table[pos] += g_pos[t] hidden[t] (atomics) */
int asme_sampled_logits_bwd(const float* hidden, const float* table, const int64_t* pos_ids, const int64_t* neg_ids,
                            int64_t n_tokens, int64_t dim, int64_t vocab, const float* g_pos, const float* g_neg,
                            float* d_hidden, float* d_table, void* stream);
/* SASRec BCE (core/losses/sasrec/sas_rec_losses.py:47-75); out[0] = loss, out[1] = sum(mask);
 * workspace: 2*n_parts floats */
int asme_sasrec_bce_fwd(const float* pos_logits, const float* neg_logits, const uint8_t* mask, int64_t n_tokens,
                        float* workspace, int64_t n_parts, float* out, void* stream);
int asme_sasrec_bce_bwd(const float* pos_logits, const float* neg_logits, const uint8_t* mask, int64_t n_tokens,
                        const float* dloss, const float* stats, float* g_pos, float* g_neg, void* stream);
/* nn.CrossEntropyLoss(ignore_index) mean reduction (masked_training_module.py:93-111,
 * sas_rec_losses.py:15-32, losses.py:77-115): lse/row_loss (n_rows); out[0] = loss, out[1] = count */
int asme_cross_entropy_fwd(const float* logits, int64_t ld, const int64_t* targets, int64_t ignore_index,
                           int64_t n_rows, int64_t n_classes, float* lse, float* row_loss, float* out, void* stream);
/* dlogits may alias logits (in-place) */
int asme_cross_entropy_bwd(const float* logits, int64_t ld, const float* lse, const int64_t* targets,
                           int64_t ignore_index, int64_t n_rows, int64_t n_classes, const float* dloss,
                           const float* stats, float* dlogits, int64_t ld_dlogits, void* stream);
/* Full-catalogue logits head fused with CrossEntropyLoss(ignore_index), logits never materialised
 * (layers.py:105-109,138-143 + masked_training_module.py:93-111 / losses.py:77-115; SURVEY A14+A17).
 * s = H W^T + bias (H: n x dim, W: V x dim, dim a multiple of 4 in [4, 128], rows 16-B aligned); lse (n);
 * products at fp32 level on the bf16 matrix cores (bf16x6 split operands, csrc/logits.hip);
 * out[0] = mean over rows with a valid target of lse - s[t] (NaN if none), out[1] = that count.
 * The backward overwrites dH (n x dim), dW (V x dim) and db (V, nullable) with the gradients of
 * dloss[0] * out[0].  Workspaces are caller-owned, sized by the *_workspace functions (bytes). */
int64_t asme_linear_xent_fwd_workspace(int64_t n, int64_t V, int64_t dim);
int asme_linear_xent_fwd(const float* H, int64_t ld_h, int64_t n, int64_t dim, const float* W, int64_t ld_w, int64_t V,
                         const float* bias, const int64_t* targets, int64_t ignore_index, float* lse, float* workspace,
                         int64_t ws_bytes, float* out, void* stream);
int64_t asme_linear_xent_bwd_workspace(int64_t n, int64_t V, int64_t dim);
int asme_linear_xent_bwd(const float* H, int64_t ld_h, int64_t n, int64_t dim, const float* W, int64_t ld_w, int64_t V,
                         const float* bias, const int64_t* targets, int64_t ignore_index, const float* lse,
                         const float* stats, const float* dloss, float* dH, float* dW, float* db, float* workspace,
                         int64_t ws_bytes, void* stream);
/* Training form of the fused CE head (the logits recomputed once instead of twice): the forward also returns
 * dh_raw (n x dim, contiguous: ld_dh must equal dim) = softmax(H W^T + b) W - W[t] per valid row, 0 for ignored
 * rows -- dH before the upstream scale; the backward scales it (dH = dh_raw * dloss[0] / out[1]) and runs the dW / db pass. */
int64_t asme_linear_xent_fwd_dh_workspace(int64_t n, int64_t V, int64_t dim);
int asme_linear_xent_fwd_dh(const float* H, int64_t ld_h, int64_t n, int64_t dim, const float* W, int64_t ld_w,
                            int64_t V, const float* bias, const int64_t* targets, int64_t ignore_index, float* lse,
                            float* dh_raw, int64_t ld_dh, float* workspace, int64_t ws_bytes, float* out, void* stream);
int64_t asme_linear_xent_bwd_dw_workspace(int64_t n, int64_t V, int64_t dim);
int asme_linear_xent_bwd_dw(const float* H, int64_t ld_h, int64_t n, int64_t dim, const float* W, int64_t ld_w,
                            int64_t V, const float* bias, const int64_t* targets, int64_t ignore_index,
                            const float* lse, const float* stats, const float* dloss, const float* dh_raw, float* dH,
                            float* dW, float* db, float* workspace, int64_t ws_bytes, void* stream);
/* Materialised full-catalogue scores (evaluation / predict_step: layers.py:105-109,138-143,
 * sasrec/components.py:46-61): out (n x V, row stride ld_out) = H (n x dim) W^T (V x dim) + bias (nullable),
 * same products as the fused head.  Workspace (bytes) from asme_logits_workspace. */
int64_t asme_logits_workspace(int64_t n, int64_t V, int64_t dim);
int asme_logits(const float* H, int64_t ld_h, int64_t n, int64_t dim, const float* W, int64_t ld_w, int64_t V,
                const float* bias, float* out, int64_t ld_out, float* workspace, int64_t ws_bytes, void* stream);
/* ranking (core/metrics/common.py:4-27 get_true_positives): 1-based rank of targets[r] in row r of
 * scores, descending, ties broken by lower item id */
int asme_target_rank(const float* scores, int64_t ld, const int64_t* targets, int64_t n_rows, int64_t n_items,
                     int64_t* ranks, void* stream);

/* ---- optimizer (torch.optim.Adam as configured in core/modules/*_training_module.py) ---------- */
int asme_adam_step(int n_tensors, float* const* params, const float* const* grads, float* const* exp_avg,
                   float* const* exp_avg_sq, const int64_t* numels, float lr, float beta1, float beta2, float eps,
                   float weight_decay, int64_t step, void* stream);
/* dense Adam over a (rows, dim) table whose gradient is row-sparse: row r's gradient is
 * grad_rows[row_slot[r]] when row_slot[r] >= 0, else 0 (still decayed / L2-coupled like torch) */
int asme_adam_rows_step(float* param, float* exp_avg, float* exp_avg_sq, int64_t rows, int64_t dim,
                        const int32_t* row_slot, const float* grad_rows, float lr, float beta1, float beta2,
                        float eps, float weight_decay, int64_t step, void* stream);

/* Lazy dense Adam ("exact catch-up"): bit-identical to asme_adam_rows_step every step, but a row with a
 * zero gradient is only rewritten when it is next read.  last_step (rows int32) = step each row is up to
 * date with; hist (hist_rows, 8) float = per-step constants written by asme_lazy_adam_record_step (allocate it
 * zero-filled and write it only through that call: row 0 is no step, it holds the first step of the current run of
 * identical beta1 / beta2 / eps / weight_decay, which lets the replay keep those in registers); every
 * step named (step / upto) must be < hist_rows, else the call fails with ASME_ERR_ARG. */
int asme_lazy_adam_record_step(float* hist, int64_t hist_rows, int64_t step, float lr, float beta1, float beta2,
                               float eps, float weight_decay, void* stream);
/* replay zero-gradient steps (last_step[r], upto] for rows[0..*count) (rows == NULL: all rows 0..cap) */
int asme_lazy_adam_catch_up(const int64_t* rows, const int32_t* count, int64_t cap, int32_t* last_step,
                            float* param, float* exp_avg, float* exp_avg_sq, int64_t dim, const float* hist,
                            int64_t hist_rows, int64_t upto, void* stream);
/* step `step` with the real gradient grad_rows[s] for rows[s], s < *count (rows already at step-1) */
int asme_lazy_adam_apply(const int64_t* rows, const int32_t* count, int64_t cap, const float* grad_rows,
                         int32_t* last_step, float* param, float* exp_avg, float* exp_avg_sq, int64_t dim,
                         const float* hist, int64_t hist_rows, int64_t step, void* stream);
/* Staged form of catch-up + apply (dim 32/64/128/256, 16-B aligned rows): asme_lazy_adam_stage writes rows[s]
 * brought up to `upto` into staged_*[s] (slot order) WITHOUT touching the table or last_step -- the step's
 * readers gather staged_param[inverse[t]] (near-sequential) instead of random table rows;
 * asme_lazy_adam_apply_staged then steps `step` from staged_*[s] with grad_rows[s] into the table rows and
 * sets last_step.  Same per-element operations as catch_up + apply, so the same bits
 * (replaces the per-step torch.optim.Adam update of nn.Embedding.weight). */
int asme_lazy_adam_stage_supported(int64_t dim);
int asme_lazy_adam_stage(const int64_t* rows, const int32_t* count, int64_t cap, const int32_t* last_step,
                         const float* param, const float* exp_avg, const float* exp_avg_sq, int64_t dim,
                         const float* hist, int64_t hist_rows, int64_t upto, float* staged_param,
                         float* staged_exp_avg, float* staged_exp_avg_sq, void* stream);
int asme_lazy_adam_apply_staged(const int64_t* rows, const int32_t* count, int64_t cap, const float* grad_rows,
                                const float* staged_param, const float* staged_exp_avg,
                                const float* staged_exp_avg_sq, int32_t* last_step, float* param, float* exp_avg,
                                float* exp_avg_sq, int64_t dim, const float* hist, int64_t hist_rows, int64_t step,
                                void* stream);

/* ---- input producers: sessions in HBM as flat item ids + offsets (n_sessions + 1) ---------
 * asme_session_batch: collate (data/collate.py:42-111): out (batch, seq_len) = the last min(len - drop_last,
 *   seq_len) items of session batch_idx[b] (left truncation), pad after; out_len (nullable) = that count.
 * asme_posneg_sample: PositiveNegativeSamplerProcessor (pos_neg_sampler.py:41-63,89-106) + collate: x = s[:-1],
 *   pos = s[1:], neg uniform over ids in [0, vocab) that are neither special (<= 8 ids) nor in the session,
 *   with replacement (Philox, seed); err_flag bit 0: no admissible id, bit 1: a session shorter than 2.
 * asme_cloze_mask: ClozeMaskProcessor (cloze_mask.py:50-92) on a collated batch (items, lengths); draws_u
 *   (batch, seq_len + 1) / draws_r (batch, seq_len) replay given draws (nullable: Philox, seed). */
int asme_session_batch(const int64_t* flat, const int64_t* offsets, int64_t n_sessions, const int64_t* batch_idx,
                       int64_t batch, int64_t seq_len, int64_t drop_last, int64_t pad, int64_t* out, int64_t* out_len,
                       void* stream);
/* asme_position_batch: (session, target_pos) pairs of a position index (data/datasets/index.py): out = the last
 *   min(pos, seq_len) items before pos (right-padded), target = s[pos]; err_flag bit 0: a pair outside its session */
int asme_position_batch(const int64_t* flat, const int64_t* offsets, int64_t n_sessions, const int64_t* pairs,
                        int64_t batch, int64_t seq_len, int64_t pad, int64_t* out, int64_t* out_len, int64_t* target,
                        int* err_flag, void* stream);
int asme_posneg_sample(const int64_t* flat, const int64_t* offsets, int64_t n_sessions, const int64_t* batch_idx,
                       int64_t batch, int64_t seq_len, int64_t vocab, const int64_t* special_ids, int n_special,
                       int64_t pad, uint64_t seed, int64_t* x, int64_t* pos, int64_t* neg, int64_t* out_len,
                       int* err_flag, void* stream);
int asme_cloze_mask(const int64_t* items, const int64_t* lengths, int64_t batch, int64_t seq_len, int64_t vocab,
                    int64_t pad, int64_t mask_id, double mask_prob, double last_prob, const float* draws_u,
                    const int64_t* draws_r, uint64_t seed, int64_t* out, int64_t* target, void* stream);
/* asme_padding_mask: flags[i] = seq[i] != pad over n ids (core/modules/util/module_util.py:13-30 get_padding_mask,
 *   sequence.ne(pad_token_id)); flags are bytes (a torch.bool tensor), seq 16-B and flags 4-B aligned. */
int asme_padding_mask(const int64_t* seq, int64_t n, int64_t pad, uint8_t* flags, void* stream);
/* asme_last_item_mask: LastItemMaskProcessor (last_item_mask.py:35-44) + collate on a collated batch (items
 *   (batch, in_len), lengths): out (batch, out_len_max) = the last min(len, out_len_max - 1) items, MASK, PAD;
 *   out_len (nullable) = the new lengths; requires in_len >= out_len_max - 1 */
int asme_last_item_mask(const int64_t* items, const int64_t* lengths, int64_t batch, int64_t in_len,
                        int64_t out_len_max, int64_t mask_id, int64_t pad, int64_t* out, int64_t* out_len,
                        void* stream);

/* ---- id dedup & shard bucketing (row-sharded item table) ------------------------ */
/* ids (n) -> unique (capacity n) in first-occurrence order, inverse (n, nullable: slot per occurrence, -1 for an id
 * outside [0, vocab)), count (1 int32 on the device; no host sync).  map: vocab int32, all -1 at rest; the call
 * leaves map[unique[s]] = first occurrence of unique[s] -- asme_dedup_reset restores it.  Three launches.
 * _segments: the occurrences are nseg (1..4) id arrays read in place (host arrays of pointers / lengths). */
int64_t asme_dedup_workspace_bytes(int64_t n);
int asme_dedup_ids(const int64_t* ids, int64_t n, int64_t vocab, int32_t* map, void* workspace,
                   int64_t workspace_bytes, int64_t* unique, int64_t* inverse, int32_t* count, void* stream);
int asme_dedup_ids_segments(int nseg, const int64_t* const* seg_ids, const int64_t* seg_n, int64_t vocab, int32_t* map,
                            void* workspace, int64_t workspace_bytes, int64_t* unique, int64_t* inverse,
                            int32_t* count, void* stream);
int asme_dedup_reset(const int64_t* unique, const int32_t* count, int64_t cap, int32_t* map, void* stream);
/* rewrite the dedup's map to map[unique[s]] = s (a row -> slot table for asme_adam_rows_step) */
int asme_dedup_map_slots(const int64_t* unique, const int32_t* count, int64_t cap, int32_t* map, void* stream);
int asme_owner_histogram(const int64_t* unique, const int32_t* count, int64_t cap, int world, int32_t* owner,
                         int32_t* counts, void* stream);
/* stable grouping of n unique ids by owner (id % world, world <= 64): order[j] = index of the j-th id sent,
 * send_local[j] (int32) = ids[order[j]] / world, counts[w] (int64) = ids sent to rank w, pos (nullable) = the inverse
 * permutation (pos[order[j]] = j).  n_dev (nullable): only the first min(n, *n_dev) ids take part -- the dedup
 * count stays on the device (no host sync before the exchange).  Workspace: asme_bucket_by_owner_workspace
 * bytes. */
int64_t asme_bucket_by_owner_workspace(int64_t n, int world);
int asme_bucket_by_owner(const int64_t* ids, int64_t n, const int32_t* n_dev, int world, void* workspace,
                         int64_t ws_bytes, int64_t* order, int32_t* send_local, int64_t* counts, int64_t* pos,
                         void* stream);
/* the same with two classes of ids (world <= 32): ids[i] with i < *split (a device int32: the requester's sequence /
 * positive rows, first in the dedup's slot order) grouped by owner, then the rest (negative-only rows) by owner --
 * counts has 2 * world entries, class-major, and the workspace is asme_bucket_by_owner_workspace(n, 2 * world).  The
 * row-sharded SASRec step sends the two classes in two exchanges, the second overlapping the transformer
 * (replaces the reference's replicated nn.Embedding lookup under DDP, sasrec_config.jsonnet:77-79). */
int asme_bucket_by_owner_split(const int64_t* ids, int64_t n, const int32_t* n_dev, int world, const int32_t* split,
                               void* workspace, int64_t ws_bytes, int64_t* order, int32_t* send_local,
                               int64_t* counts, int64_t* pos, void* stream);
/* out[r] = table[ids[r]] (zero row for ids outside [0, vocab)): the owner side of the sharded lookup */
int asme_gather_rows(const int64_t* ids, int64_t n, const float* table, int64_t vocab, int64_t dim, float* out,
                     void* stream);


/* nn.Dropout (training): y = x * keep / (1 - p), keep iff a Philox4x32-10 uniform (seed, salt 6, element index / 4)
 * >= p; the gradient is the same call on dy with the same seed (x may alias y).  Reference: the embedding dropout of
 * UBERT4Rec (ubert4rec/components.py:157-160). */
int asme_dropout(const float* x, int64_t n, float p, uint64_t seed, float* y, void* stream);
/* nn.Dropout2d on (N, C, L) (training): rows of row_len values kept (scaled) or zeroed together, one Philox draw per
 * row (salt 7, row index / 4); the gradient is the same call on dy.  Reference: NARM's embedding dropout
 * (core/models/common/layers/sequence_embedding.py:72-73, :92 on (N, S, E) = one draw per position). */
int asme_dropout_rows(const float* x, int64_t n, int64_t row_len, float p, uint64_t seed, float* y, void* stream);

/* ---- General Linear GEMMs (csrc/linear.hip), fp32 MFMA: the widths asme_ws_linear does not tile (e.g. the
 * reference's d = 32 / 64 configurations; in_f, out_f multiples of 4, rows 16-B aligned).  w is nn.Linear.weight
 * (out_f x in_f, row-major).  Reference: transformer_layers.py:175-199 (projections), 212-220
 * (PositionwiseFeedForward), ffn_modifier.py:24-26. */
/* y = x . w^T + b */
int asme_linear_fwd(const float* x, int64_t ld_x, int64_t n_rows, int64_t in_f, const float* w, const float* b,
                    int64_t out_f, float* y, int64_t ld_y, void* stream);
/* dx (+)= dy . w */
int asme_linear_dx(const float* dy, int64_t ld_dy, int64_t n_rows, int64_t out_f, const float* w, int64_t in_f,
                   float* dx, int64_t ld_dx, int accumulate, void* stream);


/* ---- Full-catalogue evaluation (csrc/catalog.hip), no (queries x |V|) logits.  Reference:
 * SASRecProjectionComponent inference (sasrec/components.py:46-61), ItemEmbeddingProjectionLayer
 * (layers.py:138-143), AllItemsSampler + argsort + get_true_positives (metrics_sampler.py:51-72,
 * metrics/common.py:4-27).  score(q, i) = H[q] . E[i] (+ bias[i]); dim in {32, 64, 128}. */
/* ranks[q] = 1 + #{i : score > score(target), or equal with i < target}; counts_ws: nq int32 */
int asme_catalog_rank(const float* H, int64_t ld_h, int64_t nq, int64_t dim, const float* E, int64_t ld_e, int64_t V,
                      const float* bias, const int64_t* targets, int32_t* counts_ws, int64_t* ranks, void* stream);
int64_t asme_catalog_topk_workspace(int64_t nq, int64_t V, int64_t dim);
/* k <= 16 best (score, item) per query, descending, ties to the lower id; row j of E is item
 * j * id_stride + id_offset (1, 0 for a whole table; W, rank for a cyclic row shard) */
int asme_catalog_topk(const float* H, int64_t ld_h, int64_t nq, int64_t dim, const float* E, int64_t ld_e, int64_t V,
                      const float* bias, int64_t id_stride, int64_t id_offset, int64_t k, void* ws, int64_t ws_bytes,
                      float* out_val, int64_t* out_idx, void* stream);
/* sharded ranks: target scores from the gathered target rows (same MFMA sequence as the shard scans), then
 * per-shard counts of items above the target (global ids); rank = 1 + all-reduced sum of the counts */
int asme_catalog_target_scores(const float* H, int64_t ld_h, int64_t nq, int64_t dim, const float* rows,
                               int64_t ld_rows, const float* row_bias, float* tscore, void* stream);
int asme_catalog_count_above(const float* H, int64_t ld_h, int64_t nq, int64_t dim, const float* E, int64_t ld_e,
                             int64_t V_local, const float* bias, const int64_t* targets, const float* tscore,
                             int64_t id_stride, int64_t id_offset, int32_t* counts, void* stream);
/* The same ranking on the bf16x6 logits engine (csrc/logits.hip, round 5): scores are the fp32-level products
 * asme_logits materialises, never stored; dim a multiple of 4 up to 128.  The catalogue is split once into three
 * bf16 planes (asme_catalog_split, asme_catalog_planes_bytes(V) bytes) and ranked against many query batches;
 * workspace: asme_catalog_x6_workspace(nq, dim) bytes. */
int64_t asme_catalog_planes_bytes(int64_t rows);
int asme_catalog_split(const float* X, int64_t ld, int64_t rows, int64_t dim, void* planes, void* stream);
int64_t asme_catalog_x6_workspace(int64_t nq, int64_t dim);
int asme_catalog_rank_x6(const float* H, int64_t ld_h, int64_t nq, int64_t dim, const float* E, int64_t ld_e,
                         const void* E_planes, int64_t V, const float* bias, const int64_t* targets, int32_t* counts_ws,
                         int64_t* ranks, void* workspace, int64_t ws_bytes, void* stream);
int asme_catalog_target_scores_x6(const float* H, int64_t ld_h, int64_t nq, int64_t dim, const float* rows,
                                  int64_t ld_rows, const float* row_bias, float* tscore, void* workspace,
                                  int64_t ws_bytes, void* stream);
int asme_catalog_count_above_x6(const float* H, int64_t ld_h, int64_t nq, int64_t dim, const void* E_planes,
                                int64_t V_local, const float* bias, const int64_t* targets, const float* tscore,
                                int64_t id_stride, int64_t id_offset, int32_t* counts, void* workspace,
                                int64_t ws_bytes, void* stream);


/* ---- Deterministic table gradient (csrc/sharding.hip; SURVEY §8b embedding_scatter_add_bwd
 * mode=deterministic; reference: autograd embedding_dense_backward).  Occurrences grouped per unique row
 * by a counting sort (each slot's list then put in occurrence order: the arrays of a stable sort), then
 * ordered sums: bit-reproducible, no float atomics, no zero fill. */
int64_t asme_occurrence_csr_workspace(int64_t n);
/* inverse (n int64 slots < cap <= n) -> order (n int32 occurrences grouped by slot, increasing within a slot;
 * slot-less occurrences last), sorted_slot (n int32, slot of order[i], cap for none), seg_off (cap + 1 int32) */
int asme_occurrence_csr(const int64_t* inverse, int64_t n, int64_t cap, void* workspace, int64_t workspace_bytes,
                        int32_t* order, int32_t* sorted_slot, int32_t* seg_off, void* stream);
int64_t asme_table_grad_workspace(int64_t n, int64_t dim);
/* grad_rows[s] = out_scale * sum over slot s's occurrences of contribution rows, fixed summation order
 * (32-occurrence chunks, then chunk partials in order); contribution k covers flat occurrences
 * [c_off[k], c_off[k]+c_n[k]) with row t = c_rows[k][t] (* c_scale[k][t]); <= 4, host arrays */
int asme_table_grad_reduce(const int32_t* order, const int32_t* sorted_slot, const int32_t* seg_off,
                           const int32_t* count, int64_t n, int64_t cap, int64_t dim, int n_contrib,
                           const int64_t* c_off, const int64_t* c_n, const float* const* c_rows,
                           const float* const* c_scale, float out_scale, void* workspace, int64_t workspace_bytes,
                           float* grad_rows, void* stream);
/* The same sums with each finished row applied at once as the lazy table Adam's real-gradient step (from the
 * staged rows sp/sm/sv[s] into param/exp_avg/exp_avg_sq[rows[s]], last_step[rows[s]] = step) instead of being
 * stored: bit-identical to asme_table_grad_reduce + asme_lazy_adam_apply_staged, no gradient-row round trip. */
int asme_table_grad_reduce_apply(const int32_t* order, const int32_t* sorted_slot, const int32_t* seg_off,
                                 const int32_t* count, int64_t n, int64_t cap, int64_t dim, int n_contrib,
                                 const int64_t* c_off, const int64_t* c_n, const float* const* c_rows,
                                 const float* const* c_scale, float out_scale, void* workspace,
                                 int64_t workspace_bytes, const int64_t* rows, const float* sp, const float* sm,
                                 const float* sv, int32_t* last_step, float* param, float* exp_avg,
                                 float* exp_avg_sq, const float* hist, int64_t hist_cap, int64_t step, void* stream);


/* ---- Weight-stationary Linear GEMM (csrc/wsgemm.hip; transformer_layers.py:175-199, 212-220 nn.Linear and
 * PositionwiseFeedForward).  One NB x K weight block resident in LDS per workgroup, X streamed from HBM into
 * registers, deferred buffer-store epilogue.  epi: 0 store (+bias), 1 pre = C + bias, Y = dropout(GELU(pre))
 * and the activation factor keep * GELU'(pre) -> pre_out, 2 Y = C * pre_in (pre_in = that factor); trans = 1:
 * W is K x N (Y = X W).  Dropout as asme_gelu_dropout_fwd (salt 5, element m*N + n). */
int asme_ws_linear_supported(int64_t M, int64_t K, int64_t N);
int asme_ws_linear(const float* X, int64_t M, int64_t K, const float* W, int64_t N, int trans, const float* bias,
                   int epi, float* pre_out, const float* pre_in, float p, uint64_t seed, float* Y, void* stream);
/* The attention output projection fused with the SublayerConnection residual and the next pre-LayerNorm
 * (transformer_layers.py:120-130 + 251-258): s_out = drop_b(res + drop_a(X W^T + bias)), ln_out = LN(s_out),
 * stats = (mean, rstd) per row -- bit-identical to asme_ws_linear (epi 0) + asme_residual_ln_fwd with the same seeds.
 * K = N = 128 only (asme_ws_linear_residual_ln_supported); ln_w null: s_out only. */
int asme_ws_linear_residual_ln_supported(int64_t M, int64_t K, int64_t N);
int asme_ws_linear_residual_ln(const float* X, int64_t M, int64_t K, const float* W, int64_t N, const float* bias,
                               const float* res, float p_a, uint64_t seed_a, float p_b, uint64_t seed_b,
                               const float* ln_w, const float* ln_b, float eps, float* s_out, float* ln_out,
                               float* stats, void* stream);

/* ---- NARM encoders (csrc/narm.hip).  Global encoder: one nn.GRU layer, batch_first, h_0 = 0
 * (core/models/narm/components.py:32-56; the reference packs the padded batch, the recurrence is causal so the
 * valid positions are identical).  Hidden size padded to hp (multiple of 16, <= 128; padded gate rows/columns and
 * biases zero).  gx (B, L, 3hp) = x W_ih^T + b_ih (a Linear GEMM); gates (B, L, 4, hp) = r, z, n, W_hn h + b_hn.
 * h0/dhT/dh0 nullable.  Backward: dgx (B, L, 3hp) = dL/d(input-side pre-activations) -> dX, dW_ih, db_ih;
 * dgh (B, L, 3hp) = dL/d(W_h* h_{t-1} + b_h*) -> dW_hh = dgh^T H_{t-1}, db_hh. */
int asme_gru_fwd(const float* gx, const float* whh, const float* bhh, const float* h0, int64_t batch,
                 int64_t seq_len, int64_t hp, float* hout, float* gates, void* stream);
int asme_gru_bwd(const float* dhout, const float* dhT, const float* whh, const float* h0, const float* hout,
                 const float* gates, int64_t batch, int64_t seq_len, int64_t hp, float* dgx, float* dgh, float* dh0,
                 void* stream);
/* Local encoder (core/models/narm/layers.py:32-66): alpha = v . sigmoid(p1 + p2_s), c_l = sum_s mask_s alpha_s hs_s;
 * p1 = A1 c_g (n, h), p2 = A2 h_i (n, s, h), mask (n, s) bytes.  Backward writes dp1, dp2, dhs and the per-row
 * partials dv_part (n, h) of dL/dv. */
int asme_narm_attend_fwd(const float* p1, const float* p2, const float* v, const float* hs, const uint8_t* mask,
                         int64_t n, int64_t s, int64_t h, float* out, float* alpha, void* stream);
int asme_narm_attend_bwd(const float* dc, const float* p1, const float* p2, const float* v, const float* hs,
                         const uint8_t* mask, const float* alpha, int64_t n, int64_t s, int64_t h, float* dp1,
                         float* dp2, float* dhs, float* dv_part, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* ASME_MI_H */
