"""Transformer-recommender building blocks with the reference's module hierarchy and fused forwards.

Attribute names mirror the reference so `state_dict` keys (and therefore checkpoints and the golden
fixtures) are interchangeable, e.g.
  _sequence_embedding_layer.item_embedding_layer.item_embedding.embedding.weight
  _sequence_representation_layer.transformer_layer.transformer_blocks.0.attention.linear_layers.0.weight
The forward passes do not call the sub-modules one by one: they hand the parameters to the fused
gfx950 kernels in `ops` (embedding+LN+dropout, attention, residual+dropout+LN, the weight-stationary
bf16x6 Linear GEMMs with the FFN's GELU+dropout epilogues, the full-catalogue logits head).

Reference classes (paths relative to /root/reference/src/asme):
  SequenceElementsEmbeddingLayer    core/models/common/layers/sequence_embedding.py:47-93
  TransformerEmbedding              core/models/common/layers/transformer_layers.py:15-80
  TransformerLayer / Block / ...    transformer_layers.py:83-258
  TransformerSequenceRepresentationComponent  core/models/transformer/sequence_representation.py:10-51
  LinearProjectionLayer / ItemEmbeddingProjectionLayer / build_projection_layer
                                    core/models/common/layers/layers.py:92-157
  FFNSequenceRepresentationModifierComponent  core/models/common/components/representation_modifier/ffn_modifier.py
  PreFusion / PostFusion components, LinearUpscaler  core/models/kebert4rec/{components,layers}.py
  PostFusionIdentitySequenceRepresentationModifierLayer  core/models/sasrec/components.py:63-106
"""
from __future__ import annotations

import math
from typing import Any, Dict, Optional

import torch
import torch.nn.functional as F
from torch import nn

from . import ops
from .sequence import get_attribute




def _p(module: nn.Module, training: bool) -> float:
    """dropout probability of an nn.Dropout (0 in eval mode / for Identity)."""
    if not training or not isinstance(module, (nn.Dropout, nn.Dropout2d)):
        return 0.0
    return float(module.p)


def has_forward_hooks(module: nn.Module) -> bool:
    """forward hooks or pre-hooks on `module`, or global module hooks: such a module must run as a module call"""
    from torch.nn.modules import module as _m
    return bool(module._forward_hooks or module._forward_pre_hooks or _m._global_forward_hooks
                or _m._global_forward_pre_hooks)


def key_valid_mask(padding_mask: Optional[torch.Tensor], shape) -> Optional[torch.Tensor]:
    if padding_mask is None:
        return None
    return ops.as_u8(padding_mask.reshape(shape[0], shape[1]))


# ------------------------------------------------------------------------------------ embeddings
class SequenceElementsEmbeddingLayer(nn.Module):
    def __init__(self, item_voc_size: int, embedding_size: int, embedding_pooling_type: Optional[str] = None,
                 dropout: Optional[float] = None):
        super().__init__()
        if embedding_pooling_type:
            raise NotImplementedError("basket pooling (embedding_pooling_type) is outside the MI355X hot path")
        self.item_voc_size = item_voc_size
        self.embedding_size = embedding_size
        self.embedding_mode = embedding_pooling_type
        self.dropout = dropout
        self.pooling = nn.Identity()
        # NARM's Dropout2d on (N, S, E) drops whole (n, s) positions; applied by _dropout
        self.dropout_layer = nn.Dropout2d(p=dropout) if dropout and dropout > 0.0 else nn.Identity()
        self.embedding = nn.Embedding(num_embeddings=item_voc_size, embedding_dim=embedding_size)
        self.embedding.weight._asme_table_grad = ops.TableGrad()

    def get_weight(self) -> torch.Tensor:
        return self.embedding.weight

    def _dropout(self, emb: torch.Tensor) -> torch.Tensor:
        """Dropout2d (training): on (N, S, E) one draw per (n, s) position, on a 2-D (NI, E) matrix one per element
        (torch's feature dropout with no spatial dims), sequence_embedding.py:72-73, :92"""
        p = _p(self.dropout_layer, self.training)
        if p <= 0.0:
            return emb
        return ops.dropout_rows(emb, p) if emb.dim() == 3 else ops.dropout(emb, p)

    def forward(self, items: torch.Tensor, flatten: bool = True) -> torch.Tensor:
        spec = ops.EmbeddingSpec(seq_len=items.shape[-1] if items.dim() > 1 else max(1, items.numel()),
                                 table_grad=self.embedding.weight._asme_table_grad)
        return self._dropout(ops.embedding(items, self.embedding.weight, spec=spec))

    def item_matrix(self) -> torch.Tensor:
        """forward(arange(|V|), flatten=False) without the identity gather: the whole table through the dropout"""
        return self._dropout(self.embedding.weight)


class TransformerEmbedding(nn.Module):
    def __init__(self, item_voc_size: int, max_seq_len: int, embedding_size: int, dropout: float,
                 positional_embedding: bool = True, embedding_pooling_type: str = None, norm_embedding: bool = True):
        super().__init__()
        self.embedding_size = embedding_size
        self.positional_embedding_active = positional_embedding
        self.item_embedding = SequenceElementsEmbeddingLayer(item_voc_size=item_voc_size,
                                                             embedding_size=embedding_size,
                                                             embedding_pooling_type=embedding_pooling_type)
        if self.positional_embedding_active:
            self.position_embedding = nn.Embedding(max_seq_len, self.embedding_size)
        self.embedding_norm = nn.LayerNorm(self.embedding_size) if norm_embedding else nn.Identity()
        self.dropout = nn.Dropout(p=dropout)

    def get_item_embedding_weight(self) -> torch.Tensor:
        override = getattr(self, "_table_override", None)
        return override if override is not None else self.item_embedding.embedding.weight

    def fused_args(self):
        pos = self.position_embedding.weight if self.positional_embedding_active else None
        ln1 = (self.embedding_norm.weight, self.embedding_norm.bias) if isinstance(self.embedding_norm,
                                                                                   nn.LayerNorm) else None
        eps1 = self.embedding_norm.eps if ln1 is not None else 1e-5
        return pos, ln1, eps1

    def embed(self, ids: torch.Tensor, extra=None, ln2: Optional[nn.LayerNorm] = None, p2: float = 0.0):
        """Fused: drop2(LN2(drop1(LN1(E[ids] + P)) + extra)) — transformer_layers.py:55-80
        (+ kebert4rec/components.py:54-63 when ln2/extra are given)."""
        pos, ln1, eps1 = self.fused_args()
        if pos is not None and ids.shape[1] > pos.shape[0]:
            raise IndexError(f"sequence length {ids.shape[1]} exceeds max_seq_len {pos.shape[0]}")
        w = self.get_item_embedding_weight()
        spec = ops.EmbeddingSpec(seq_len=ids.shape[1], ln1_eps=eps1, p1=_p(self.dropout, self.training),
                                 ln2_eps=ln2.eps if ln2 is not None else 1e-5, p2=p2,
                                 table_grad=w._asme_table_grad)
        ln2_t = (ln2.weight, ln2.bias) if ln2 is not None else None
        # the first transformer block's input LayerNorm, when the model feeds this output straight into it
        # (TransformerEncoderModel.fuse_embedding_norm sets it): computed by the same kernel, handed over on the output
        # tensor.  Not while that norm carries forward hooks: then block 0 calls it as a module (TransformerLayer)
        ln3 = self.__dict__.get("_asme_next_norm")
        if ln3 is None or has_forward_hooks(ln3):
            return ops.embedding(ids, w, pos, ln1, extra, ln2_t, spec)
        x, ln = ops.embedding(ids, w, pos, ln1, extra, ln2_t, spec, ln3=ln3)
        x._asme_ln = (ln3, ln)
        return x

    def forward(self, sequence) -> torch.Tensor:
        return self.embed(sequence.sequence)


class LinearUpscaler(nn.Module):
    """multi-hot(ids) -> Linear(vocab -> d); pad category 0 ignored (kebert4rec/layers.py:15-27)."""

    def __init__(self, vocab_size: int, embed_size: int):
        super().__init__()
        self.linear = nn.Linear(vocab_size, embed_size)
        self.vocab_size = vocab_size

    def forward(self, content_input: torch.Tensor) -> torch.Tensor:
        table = self.linear.weight.t().contiguous()  # (vocab, d): column gather == row gather
        return ops.gather_sum(content_input, table, self.linear.bias, skip_zero=True)


class _ContentEmbedding(nn.Embedding):
    """nn.Embedding whose lookup runs on the gather kernel (kebert4rec/components.py:15-24)."""

    def forward(self, ids: torch.Tensor) -> torch.Tensor:
        return ops.gather_sum(ids, self.weight, None, skip_zero=False)


def build_embedding_type(embedding_type: str, vocab_size: int, hidden_size: int) -> nn.Module:
    if embedding_type == "content_embedding":
        return _ContentEmbedding(num_embeddings=vocab_size, embedding_dim=hidden_size)
    if embedding_type == "linear_upscale":
        return LinearUpscaler(vocab_size=vocab_size, embed_size=hidden_size)
    raise KeyError(embedding_type)


def _attribute_sum(modules: nn.ModuleDict, sequence) -> Optional[torch.Tensor]:
    total = None
    for key, module in modules.items():
        meta = get_attribute(sequence, key)
        if meta is None:
            raise Exception(f"The batch does not contain the following additional metadata: {key}.")
        e = module(meta)
        total = e if total is None else total + e
    return total


class PreFusionContextSequenceElementsRepresentationComponent(nn.Module):
    def __init__(self, item_embedding_layer: TransformerEmbedding, embedding_size: int,
                 prefusion_attributes: Optional[Dict[str, Dict[str, Any]]],
                 additional_attributes_tokenizer: Optional[Dict[str, Any]], dropout: float = 0.0):
        super().__init__()
        self.item_embedding_layer = item_embedding_layer
        pre = {}
        for name, info in (prefusion_attributes or {}).items():
            vocab = len(additional_attributes_tokenizer["tokenizers." + name])
            pre[name] = build_embedding_type(info["embedding_type"], vocab, embedding_size)
        self.prefusion_attribute_embeddings = nn.ModuleDict(pre)
        self.dropout_embedding = nn.Dropout(dropout)
        self.norm_embedding = nn.LayerNorm(embedding_size)

    def forward(self, sequence) -> torch.Tensor:
        extra = _attribute_sum(self.prefusion_attribute_embeddings, sequence)
        return self.item_embedding_layer.embed(sequence.sequence, extra=extra, ln2=self.norm_embedding,
                                               p2=_p(self.dropout_embedding, self.training))


# ------------------------------------------------------------------------------------ transformer
class LayerNorm(nn.LayerNorm):
    """nn.LayerNorm (same parameters and state_dict keys) whose module call runs the LayerNorm kernel.  The
    transformer blocks read the parameters directly into their fused kernels; any of their norms with forward hooks
    or pre-hooks registered (or global module hooks) is called as a module instead, so the hooks run and may replace
    its input or output (TransformerLayer.forward, _residual_norm)."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return ops.layer_norm(x, self)


class SublayerConnection(nn.Module):
    def __init__(self, size, dropout):
        super().__init__()
        self.norm = LayerNorm(size)
        self.dropout = nn.Dropout(dropout)


class Attention(nn.Module):
    """parameter-free marker (the computation is ops.attention)"""


class MultiHeadedAttention(nn.Module):
    def __init__(self, heads: int, d_model: int, dropout: float = 0.1):
        super().__init__()
        assert d_model % heads == 0
        self.d_k = d_model // heads
        self.heads = heads
        self.linear_layers = nn.ModuleList([nn.Linear(d_model, d_model) for _ in range(3)])
        self.output_linear = nn.Linear(d_model, d_model)
        self.attention = Attention()
        self.dropout = nn.Dropout(p=dropout)

    def qkv_weights(self):
        w = torch.cat([l.weight for l in self.linear_layers], 0)
        b = torch.cat([l.bias for l in self.linear_layers], 0)
        return w, b

    def qkv(self, x):
        """the fused Q/K/V projection (transformer_layers.py:191-194) as one GEMM: the three weights (and biases) are
        kept as consecutive row blocks of one buffer, re-homed there on first use, so no per-forward concatenation"""
        ws = [l.weight for l in self.linear_layers]
        bs = [l.bias for l in self.linear_layers]
        if ops.adjacent_rows(ws) is None or ops.adjacent_rows(bs) is None:
            ops.fuse_rows_(ws)
            ops.fuse_rows_(bs)
        return ops.linear_row_parts(x, ws, bs)


class PositionwiseFeedForward(nn.Module):
    def __init__(self, d_model: int, d_ff: int, dropout: float = 0.1):
        super().__init__()
        self.w_1 = nn.Linear(d_model, d_ff)
        self.w_2 = nn.Linear(d_ff, d_model)
        self.dropout = nn.Dropout(dropout)
        self.activation = nn.GELU()


class TransformerBlock(nn.Module):
    def __init__(self, hidden: int, attn_heads: int, feed_forward_hidden: int, dropout: float,
                 attention_dropout: float = None):
        super().__init__()
        if attention_dropout is None:
            attention_dropout = dropout
        self.attention = MultiHeadedAttention(heads=attn_heads, d_model=hidden, dropout=attention_dropout)
        self.feed_forward = PositionwiseFeedForward(d_model=hidden, d_ff=feed_forward_hidden, dropout=dropout)
        self.input_sublayer = SublayerConnection(size=hidden, dropout=dropout)
        self.output_sublayer = SublayerConnection(size=hidden, dropout=dropout)
        self.dropout = nn.Dropout(p=dropout)


class TransformerLayer(nn.Module):
    def __init__(self, hidden_size: int, num_heads: int, num_layers: int, dim_feedforward: int, dropout: float,
                 attention_dropout: float = None):
        super().__init__()
        self.transformer_blocks = nn.ModuleList(
            [TransformerBlock(hidden_size, num_heads, dim_feedforward, dropout, attention_dropout=attention_dropout)
             for _ in range(num_layers)])

    def forward(self, x: torch.Tensor, key_valid: Optional[torch.Tensor], causal: bool) -> torch.Tensor:
        """N pre-LN blocks (transformer_layers.py:100-106, 120-130, 251-258) on the fused kernels:
           h1 = x + drop(O(attn(LN_in(x))));  x' = drop(h1 + drop(W2 drop(GELU(W1 LN_out(h1)))))
        No final LayerNorm after the last block."""
        blocks = self.transformer_blocks
        if len(blocks) == 0:
            return x
        tr = self.training
        norm0 = blocks[0].input_sublayer.norm
        pre = getattr(x, "_asme_ln", None)  # LN_in(x) of block 0, computed by the embedding kernel
        if has_forward_hooks(norm0):
            ln = norm0(x)  # a module call, so the hooks run (and may replace its input or output)
        elif pre is not None and pre[0] is norm0:
            ln = pre[1]
        else:  # no hand-off (fuse_embedding_norm off, or an op between the embedding and block 0 made x anew)
            x, ln = ops.layer_norm_pass(x, norm0)
        for i, blk in enumerate(blocks):
            att, ff = blk.attention, blk.feed_forward
            qkv = att.qkv(ln)
            o = ops.attention(qkv, key_valid, att.heads, causal, _p(att.dropout, tr))
            h1, ln2 = self._projection_residual_norm(o, att.output_linear, x, blk.output_sublayer.norm,
                                                     _p(blk.input_sublayer.dropout, tr))
            f2 = ops.ffn(ln2, ff.w_1.weight, ff.w_1.bias, ff.w_2.weight, ff.w_2.bias, _p(ff.dropout, tr))
            nxt = blocks[i + 1].input_sublayer.norm if i + 1 < len(blocks) else None
            x, ln = _residual_norm(h1, f2, nxt, _p(blk.output_sublayer.dropout, tr), _p(blk.dropout, tr))
        return x

    # True: the attention output projection, its residual and the next pre-LN in one kernel where it tiles (d = 128:
    # asme_ws_linear_residual_ln, bit-identical to the separate Linear + residual-LN kernels).  Off: measured slower in
    # the step (128 us per call vs 48 + 65 us for the two kernels, -0.6 % per step, tools/rln_step_ab.py): at two
    # waves per SIMD the epilogue's row reductions and dropout do not hide under the GEMM's streaming
    fuse_output_projection = False

    def _projection_residual_norm(self, o, lin: nn.Linear, res, norm, p_a: float):
        """(h1, LN(h1)) with h1 = res + drop_a(lin(o)) (transformer_layers.py:120-130 around :181-199)"""
        if (self.fuse_output_projection and (norm is None or not has_forward_hooks(norm))
                and ops.linear_residual_ln_ok(o, lin.weight, res)):
            return ops.linear_residual_ln(o, lin.weight, lin.bias, res, norm, p_a, 0.0)
        a = ops.linear(o, lin.weight, lin.bias)
        return _residual_norm(res, a, norm, p_a, 0.0)


def _residual_norm(res, y, norm, p_a: float, p_b: float):
    """(s, norm(s)) with s = drop_b(res + drop_a(y)): the norm fused into the residual kernel, or -- when it has
    forward hooks -- called as a module on s, so its hooks see the reference's call"""
    if norm is not None and has_forward_hooks(norm):
        s, _ = ops.residual_ln(res, y, None, p_a, p_b)
        return s, norm(s)
    return ops.residual_ln(res, y, norm, p_a, p_b)


class TransformerSequenceRepresentationComponent(nn.Module):
    def __init__(self, transformer_layer: TransformerLayer, bidirectional: bool):
        super().__init__()
        self.transformer_layer = transformer_layer
        self.bidirectional = bidirectional

    def forward(self, embedded: torch.Tensor, padding_mask: Optional[torch.Tensor]) -> torch.Tensor:
        kv = key_valid_mask(padding_mask, embedded.shape)
        return self.transformer_layer(embedded, kv, causal=not self.bidirectional)


# ------------------------------------------------------------------------------------ modifiers
class IdentitySequenceRepresentationModifierLayer(nn.Module):
    def forward(self, encoded: torch.Tensor, sequence=None) -> torch.Tensor:
        return encoded

    def forward_rows(self, encoded_rows: torch.Tensor, sequence=None, rows=None, inverse=None) -> torch.Tensor:
        """the modifier on the selected flattened positions only (models.TransformerEncoderModel.encode_rows)"""
        return encoded_rows


class FFNSequenceRepresentationModifierComponent(nn.Module):
    """LN(GELU(Linear(x))) (ffn_modifier.py:24-26)"""

    def __init__(self, feature_size: int):
        super().__init__()
        self.transform = nn.Sequential(nn.Linear(feature_size, feature_size), nn.GELU(), nn.LayerNorm(feature_size))

    def forward(self, encoded: torch.Tensor, sequence=None) -> torch.Tensor:
        lin, _, norm = self.transform
        return ops.layer_norm(ops.gelu_dropout(ops.linear(encoded, lin.weight, lin.bias), 0.0), norm)

    def forward_rows(self, encoded_rows: torch.Tensor, sequence=None, rows=None, inverse=None) -> torch.Tensor:
        """position-wise: the same transform on the selected rows (M, d) alone"""
        return self.forward(encoded_rows)


def _rows_of(x: Optional[torch.Tensor], rows: torch.Tensor, inverse=None) -> Optional[torch.Tensor]:
    """the flattened positions `rows` of a (B, L, d) per-position tensor"""
    return None if x is None else ops.select_rows(x.reshape(-1, x.shape[-1]), rows, inverse)


def _merge(x: torch.Tensor, ctx: torch.Tensor, fn: str) -> torch.Tensor:
    if fn == "add":
        return x + ctx
    if fn == "multiply":
        return x * ctx
    return x


class PostFusionContextSequenceRepresentationModifierComponent(nn.Module):
    """x (+|*)= sum attr-emb, then Linear -> GELU -> LN (kebert4rec/components.py:65-115)"""

    def __init__(self, feature_size: int, postfusion_attributes, additional_attributes_tokenizer,
                 merge_function: str = "add"):
        super().__init__()
        self.merge_function = merge_function
        post = {}
        for name, info in postfusion_attributes.items():
            vocab = len(additional_attributes_tokenizer["tokenizers." + name])
            post[name] = build_embedding_type(info["embedding_type"], vocab, feature_size)
        self.postfusion_attribute_embeddings = nn.ModuleDict(post)
        self.transform = nn.Sequential(nn.Linear(feature_size, feature_size), nn.GELU(), nn.LayerNorm(feature_size))

    def forward(self, encoded: torch.Tensor, sequence=None) -> torch.Tensor:
        x = _merge(encoded, _attribute_sum(self.postfusion_attribute_embeddings, sequence), self.merge_function)
        lin, _, norm = self.transform
        return ops.layer_norm(ops.gelu_dropout(ops.linear(x, lin.weight, lin.bias), 0.0), norm)

    def forward_rows(self, encoded_rows: torch.Tensor, sequence=None, rows=None, inverse=None) -> torch.Tensor:
        """position-wise: the selected rows merged with their positions' attribute sums, then the transform"""
        x = _merge(encoded_rows, _rows_of(_attribute_sum(self.postfusion_attribute_embeddings, sequence), rows,
                                          inverse), self.merge_function)
        lin, _, norm = self.transform
        return ops.layer_norm(ops.gelu_dropout(ops.linear(x, lin.weight, lin.bias), 0.0), norm)


class PostFusionIdentitySequenceRepresentationModifierLayer(nn.Module):
    """x (+|*)= sum attr-emb, no transform (sasrec/components.py:63-106)"""

    def __init__(self, feature_size: int, postfusion_attributes, additional_attributes_tokenizer,
                 merge_function: str = "add"):
        super().__init__()
        self.merge_function = merge_function
        post = {}
        for name, info in postfusion_attributes.items():
            vocab = len(additional_attributes_tokenizer["tokenizers." + name])
            post[name] = build_embedding_type(info["embedding_type"], vocab, feature_size)
        self.postfusion_attribute_embeddings = nn.ModuleDict(post)

    def forward(self, encoded: torch.Tensor, sequence=None) -> torch.Tensor:
        return _merge(encoded, _attribute_sum(self.postfusion_attribute_embeddings, sequence), self.merge_function)

    def forward_rows(self, encoded_rows: torch.Tensor, sequence=None, rows=None, inverse=None) -> torch.Tensor:
        return _merge(encoded_rows, _rows_of(_attribute_sum(self.postfusion_attribute_embeddings, sequence), rows,
                                             inverse), self.merge_function)


# ------------------------------------------------------------------------------------ projections
PROJECT_TYPE_LINEAR = "linear"


class LinearProjectionLayer(nn.Module):
    def __init__(self, hidden_size: int, item_vocab_size: int):
        super().__init__()
        self.linear = nn.Linear(hidden_size, item_vocab_size)

    def weight_bias(self):
        return self.linear.weight, self.linear.bias

    def forward(self, representation: torch.Tensor, sequence=None) -> torch.Tensor:
        return ops.logits(representation, self.linear.weight, self.linear.bias)


class ItemEmbeddingProjectionLayer(nn.Module):
    """tied head h E^T + b (layers.py:112-143)"""

    def __init__(self, item_vocab_size: int, embedding: nn.Embedding):
        super().__init__()
        self.item_vocab_size = item_vocab_size
        self.embedding = embedding
        self.output_bias = nn.Parameter(torch.empty(item_vocab_size))
        bound = 1 / math.sqrt(item_vocab_size)
        nn.init.uniform_(self.output_bias, -bound, bound)

    def weight_bias(self):
        return self.embedding.weight, self.output_bias

    def forward(self, representation: torch.Tensor, sequence=None) -> torch.Tensor:
        return ops.logits(representation, self.embedding.weight, self.output_bias)


def build_projection_layer(project_type: str, transformer_hidden_size: int, item_voc_size: int,
                           embedding: nn.Embedding) -> nn.Module:
    if project_type == PROJECT_TYPE_LINEAR:
        return LinearProjectionLayer(transformer_hidden_size, item_voc_size)
    if project_type == "transpose_embedding":
        return ItemEmbeddingProjectionLayer(item_voc_size, embedding)
    raise KeyError(f"{project_type} invalid projection layer")


class SASRecProjectionComponent(nn.Module):
    """sasrec/components.py:14-61: sampled pos/neg dot products (train) or full-catalogue scores of
    the last valid position (inference)."""

    def __init__(self, embedding: TransformerEmbedding):
        super().__init__()
        self.embedding = embedding

    def forward(self, representation: torch.Tensor, sequence) -> Any:
        pos = get_attribute(sequence, "positive_samples")
        neg = get_attribute(sequence, "negative_samples")
        table = self.embedding.get_item_embedding_weight()
        if neg is not None:
            return ops.sampled_logits(representation, table, pos, neg, table._asme_table_grad)
        # inference: H[b, len_b - 1] . E[items]^T
        mask = sequence.padding_mask
        idx = mask.sum(-1) - 1
        last = representation[torch.arange(representation.shape[0], device=representation.device), idx]
        if getattr(pos, "_asme_all_items", False) and pos.dim() == 2 and pos.shape[1] == table.shape[0]:
            return ops.logits(last, table)  # all items, in id order (predict_step's items_to_rank)
        rows = F.embedding(pos, table)  # (N, I, d)
        return torch.bmm(rows, last.unsqueeze(-1)).squeeze(-1)
