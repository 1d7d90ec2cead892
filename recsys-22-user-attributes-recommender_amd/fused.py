"""The pre-LN transformer stack as ONE autograd function with a hand-written backward, so every
elementwise/normalisation pass rides in a GEMM epilogue (csrc/linear.hip) and nothing is materialised
that the backward does not need.

Reference semantics (paths relative to /root/reference/src/asme):
  TransformerBlock.forward       core/models/common/layers/transformer_layers.py:251-258
  SublayerConnection.forward     transformer_layers.py:120-130   x + dropout(sublayer(LN(x)))   (pre-LN)
  MultiHeadedAttention.forward   transformer_layers.py:181-199
  PositionwiseFeedForward        transformer_layers.py:212-220   W2(dropout(GELU_erf(W1 x)))
No final LayerNorm after the last block.

Forward of block j (x_j = block input, ln_j = LN1_j(x_j) -- for j > 0 produced by block j-1's last GEMM):
  qkv     = ln_j Wqkv^T + bqkv                          library GEMM
  o       = attention(qkv)                              asme_attention_fwd
  h1, ln2 = x_j + drop(o Wo^T + bo), LN2(h1)            asme_linear_residual_ln_fwd   (Wo GEMM + epilogue)
  pre, g  = ln2 W1^T + b1, drop(GELU(pre))              asme_linear_gelu_dropout_fwd  (W1 GEMM + epilogue)
  x_j+1, ln_j+1 = drop(h1 + drop(g W2^T + b2)), LN1_j+1 asme_linear_residual_ln_fwd   (W2 GEMM + epilogue)
Backward of block j (d_h1 and d_f2 = dL/d(g W2^T + b2) arrive from the GEMM that closed block j+1):
  d_pre   = (d_f2 W2) * keep * GELU'(pre)               asme_linear_dx_gelu_bwd
  d_s1    = d_h1 + LN2_bwd(d_pre W1); d_a = drop'(d_s1) asme_linear_dx_residual_ln_bwd
  d_o     = d_a Wo                                      library GEMM
  d_qkv   = attention_bwd                               asme_attention_bwd
  (block j-1's d_h1, d_f2) or d_x0 = drop'(d_s1 + LN1_bwd(d_qkv Wqkv))  asme_linear_dx_residual_ln_bwd
and every dW/db on asme_linear_weight_grad.  Dropout decisions equal those of the unfused kernels.
"""
from __future__ import annotations

import math
from typing import List, Sequence

import torch
import torch.nn.functional as F

from . import _lib
from ._lib import call, ptr, stream
from .ops import _mask_bytes, _reduce_partials, new_seed

_PER_BLOCK = 12  # ln1_w, ln1_b, wqkv, bqkv, wo, bo, ln2_w, ln2_b, w1, b1, w2, b2


def fusable(hidden: int, ffn: int, heads: int, x: torch.Tensor) -> bool:
    """Shapes the fused kernels cover: hidden 128 (whole rows in one GEMM tile), features % 4 == 0."""
    return (x.is_cuda and x.dtype == torch.float32 and hidden == 128 and ffn % 4 == 0 and hidden % heads == 0
            and (hidden // heads) in (16, 32, 64, 128))


def _weight_grad(dy: torch.Tensor, x: torch.Tensor):
    """(dW, db) = (dy^T x, sum_rows dy) on the split-token MFMA kernel."""
    T, N = dy.shape
    K = x.shape[1]
    nbytes = int(_lib.load().asme_linear_weight_grad_workspace(T, N, K))
    ws = torch.empty(max(4, nbytes // 4), device=dy.device, dtype=torch.float32)
    dw = torch.empty(N, K, device=dy.device, dtype=torch.float32)
    db = torch.empty(N, device=dy.device, dtype=torch.float32)
    call("asme_linear_weight_grad", ptr(dy), dy.stride(0), ptr(x), x.stride(0), T, N, K, ptr(ws), nbytes, ptr(dw),
         ptr(db), 0, stream())
    return dw, db


class _StackFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, key_valid, cfg, *params):
        nb, heads, causal, probs, eps1, eps2 = cfg
        shape = x.shape
        D = shape[-1]
        B, L = shape[0], shape[1]
        T = B * L
        dev = x.device
        dk = D // heads
        scale = 1.0 / math.sqrt(dk)
        xi = x.reshape(T, D).contiguous()
        ln = torch.empty_like(xi)
        st = torch.empty(T, 2, device=dev, dtype=torch.float32)
        call("asme_layernorm_fwd", ptr(xi), T, D, ptr(params[0]), ptr(params[1]), eps1[0], ptr(ln), ptr(st),
             stream())
        saved: List[torch.Tensor] = [key_valid]
        seeds = []
        for j in range(nb):
            (ln1_w, ln1_b, wqkv, bqkv, wo, bo, ln2_w, ln2_b, w1, b1, w2, b2) = params[_PER_BLOCK * j:
                                                                                     _PER_BLOCK * (j + 1)]
            p_att, p_a1, p_ffn, p_a2, p_b2 = probs[j]
            Fd = w1.shape[0]
            qkv = F.linear(ln, wqkv, bqkv)
            o = torch.empty(T, D, device=dev, dtype=torch.float32)
            lse = torch.empty(B * heads, L, 2, device=dev, dtype=torch.float32)
            mask = torch.empty(_mask_bytes(B, heads, L), device=dev, dtype=torch.uint8) if p_att > 0 else None
            s_att = new_seed(p_att)
            base = qkv.data_ptr()
            call("asme_attention_fwd", base, base + 4 * D, base + 8 * D, 3 * D, 3 * D, 3 * D, ptr(key_valid), B,
                 heads, L, dk, int(causal), scale, p_att, s_att, ptr(o), D, ptr(lse), ptr(mask), stream())
            h1 = torch.empty(T, D, device=dev, dtype=torch.float32)
            ln2 = torch.empty_like(h1)
            st2 = torch.empty(T, 2, device=dev, dtype=torch.float32)
            s_a1 = new_seed(p_a1)
            call("asme_linear_residual_ln_fwd", ptr(o), D, T, D, ptr(wo), ptr(bo), D, ptr(xi), p_a1, s_a1, 0.0, 0,
                 ptr(ln2_w), ptr(ln2_b), eps2[j], ptr(h1), ptr(ln2), ptr(st2), stream())
            pre = torch.empty(T, Fd, device=dev, dtype=torch.float32)
            g = torch.empty_like(pre)
            s_ffn = new_seed(p_ffn)
            call("asme_linear_gelu_dropout_fwd", ptr(ln2), D, T, D, ptr(w1), ptr(b1), Fd, p_ffn, s_ffn, ptr(pre),
                 ptr(g), Fd, stream())
            last = j == nb - 1
            x_next = torch.empty(T, D, device=dev, dtype=torch.float32)
            ln_next = None if last else torch.empty_like(x_next)
            st_next = None if last else torch.empty(T, 2, device=dev, dtype=torch.float32)
            nw = None if last else params[_PER_BLOCK * (j + 1)]
            nbias = None if last else params[_PER_BLOCK * (j + 1) + 1]
            s_a2, s_b2 = new_seed(p_a2), new_seed(p_b2)
            call("asme_linear_residual_ln_fwd", ptr(g), Fd, T, Fd, ptr(w2), ptr(b2), D, ptr(h1), p_a2, s_a2, p_b2,
                 s_b2, ptr(nw), ptr(nbias), 0.0 if last else eps1[j + 1], ptr(x_next), ptr(ln_next), ptr(st_next),
                 stream())
            saved += [xi, ln, st, qkv, o, lse, mask if mask is not None else lse.new_empty(0), h1, ln2, st2, pre, g]
            seeds.append((s_att, s_a1, s_ffn, s_a2, s_b2))
            xi, ln, st = x_next, ln_next, st_next
        ctx.save_for_backward(*saved, *params)
        ctx.cfg = cfg
        ctx.seeds = seeds
        ctx.shape = shape
        return xi.view(shape)

    @staticmethod
    def backward(ctx, d_out):
        nb, heads, causal, probs, eps1, eps2 = ctx.cfg
        shape = ctx.shape
        D = shape[-1]
        B, L = shape[0], shape[1]
        T = B * L
        dk = D // heads
        scale = 1.0 / math.sqrt(dk)
        saved = ctx.saved_tensors
        key_valid = saved[0]
        per = 12
        acts = [saved[1 + per * j: 1 + per * (j + 1)] for j in range(nb)]
        params = saved[1 + per * nb:]
        dev = d_out.device
        grads: List[torch.Tensor] = [None] * len(params)
        rows = int(_lib.load().asme_linear_partials_rows(T))

        # last block's closing residual has no LayerNorm after it
        j = nb - 1
        p_att, p_a1, p_ffn, p_a2, p_b2 = probs[j]
        s_att, s_a1, s_ffn, s_a2, s_b2 = ctx.seeds[j]
        d = d_out.reshape(T, D).contiguous()
        d_h1 = torch.empty(T, D, device=dev, dtype=torch.float32)
        d_f2 = torch.empty_like(d_h1) if p_a2 > 0 else None
        call("asme_residual_ln_bwd", None, T, D, p_a2, s_a2, p_b2, s_b2, None, None, ptr(d), None, ptr(d_h1),
             ptr(d_f2), None, 1, stream())
        if d_f2 is None:
            d_f2 = d_h1
        d_x0 = None
        for j in range(nb - 1, -1, -1):
            xi, ln, st, qkv, o, lse, mask, h1, ln2, st2, pre, g = acts[j]
            (ln1_w, ln1_b, wqkv, bqkv, wo, bo, ln2_w, ln2_b, w1, b1, w2, b2) = params[per * j: per * (j + 1)]
            p_att, p_a1, p_ffn, p_a2, p_b2 = probs[j]
            s_att, s_a1, s_ffn, s_a2, s_b2 = ctx.seeds[j]
            Fd = w1.shape[0]
            # FFN output projection: input grad through GELU + dropout, weight grads
            d_pre = torch.empty(T, Fd, device=dev, dtype=torch.float32)
            call("asme_linear_dx_gelu_bwd", ptr(d_f2), D, T, D, ptr(w2), Fd, ptr(pre), p_ffn, s_ffn, ptr(d_pre), Fd,
                 stream())
            grads[per * j + 10], grads[per * j + 11] = _weight_grad(d_f2, g)
            # FFN input projection: input grad + LN2 backward + first residual
            d_s1 = torch.empty(T, D, device=dev, dtype=torch.float32)
            d_a = torch.empty_like(d_s1) if p_a1 > 0 else None
            part = torch.empty(rows, 2 * D, device=dev, dtype=torch.float32)
            call("asme_linear_dx_residual_ln_bwd", ptr(d_pre), Fd, T, Fd, ptr(w1), D, ptr(h1), ptr(st2), ptr(ln2_w),
                 ptr(d_h1), p_a1, s_a1, 0.0, 0, ptr(d_s1), ptr(d_a), ptr(part), stream())
            red = _reduce_partials(part, 2 * D)
            grads[per * j + 6], grads[per * j + 7] = red[:D], red[D:]
            grads[per * j + 8], grads[per * j + 9] = _weight_grad(d_pre, ln2)
            if d_a is None:
                d_a = d_s1
            # attention output projection
            d_o = d_a @ wo
            grads[per * j + 4], grads[per * j + 5] = _weight_grad(d_a, o)
            # attention
            d_qkv = torch.empty(T, 3 * D, device=dev, dtype=torch.float32)
            dsum = torch.empty(B * heads * L, device=dev, dtype=torch.float32)
            base, gb = qkv.data_ptr(), d_qkv.data_ptr()
            call("asme_attention_bwd", base, base + 4 * D, base + 8 * D, 3 * D, 3 * D, 3 * D, ptr(o), D, ptr(d_o), D,
                 ptr(lse), ptr(key_valid), B, heads, L, dk, int(causal), scale, p_att, s_att,
                 ptr(mask) if mask.numel() else None, ptr(dsum), gb, 3 * D, gb + 4 * D, 3 * D, gb + 8 * D, 3 * D,
                 stream())
            grads[per * j + 2], grads[per * j + 3] = _weight_grad(d_qkv, ln)
            # QKV input grad + LN1_j backward + the residual that produced x_j
            part = torch.empty(rows, 2 * D, device=dev, dtype=torch.float32)
            d_res = torch.empty(T, D, device=dev, dtype=torch.float32)
            if j > 0:
                pp_a2, pp_b2 = probs[j - 1][3], probs[j - 1][4]
                ps_a2, ps_b2 = ctx.seeds[j - 1][3], ctx.seeds[j - 1][4]
                d_y = torch.empty_like(d_res) if pp_a2 > 0 else None
            else:
                pp_a2 = pp_b2 = 0.0
                ps_a2 = ps_b2 = 0
                d_y = None
            call("asme_linear_dx_residual_ln_bwd", ptr(d_qkv), 3 * D, T, 3 * D, ptr(wqkv), D, ptr(xi), ptr(st),
                 ptr(ln1_w), ptr(d_s1), pp_a2, ps_a2, pp_b2, ps_b2, ptr(d_res), ptr(d_y), ptr(part), stream())
            red = _reduce_partials(part, 2 * D)
            grads[per * j + 0], grads[per * j + 1] = red[:D], red[D:]
            if j > 0:
                d_h1 = d_res
                d_f2 = d_y if d_y is not None else d_res
            else:
                d_x0 = d_res
        return (d_x0.view(shape), None, None, *grads)


def transformer_stack(x: torch.Tensor, key_valid: torch.Tensor, blocks: Sequence, causal: bool,
                      training: bool) -> torch.Tensor:
    """Run `blocks` (layers.TransformerBlock) as one fused autograd function."""
    from .layers import _p  # local import: layers imports this module

    params: List[torch.Tensor] = []
    probs, eps1, eps2 = [], [], []
    for blk in blocks:
        att, ff = blk.attention, blk.feed_forward
        wqkv, bqkv = att.qkv_weights()
        n1, n2 = blk.input_sublayer.norm, blk.output_sublayer.norm
        params += [n1.weight, n1.bias, wqkv, bqkv, att.output_linear.weight, att.output_linear.bias, n2.weight,
                   n2.bias, ff.w_1.weight, ff.w_1.bias, ff.w_2.weight, ff.w_2.bias]
        probs.append((_p(att.dropout, training), _p(blk.input_sublayer.dropout, training), _p(ff.dropout, training),
                      _p(blk.output_sublayer.dropout, training), _p(blk.dropout, training)))
        eps1.append(n1.eps)
        eps2.append(n2.eps)
    cfg = (len(blocks), blocks[0].attention.heads, bool(causal), tuple(probs), tuple(eps1), tuple(eps2))
    return _StackFn.apply(x, key_valid, cfg, *params)
