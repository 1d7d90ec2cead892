"""SASRec / BERT4Rec / KeBERT4Rec / NARM with the reference constructors and forward contract.

Constructor parameter names and defaults equal the reference's, because ASME's GenericModelFactory
builds models by introspecting `__init__` (core/init/factories/modules/modules.py:116-127):
  SASRecModel      core/models/sasrec/sasrec_model.py:29-116
  BERT4RecModel    core/models/bert4rec/bert4rec_model.py:24-68
  KeBERT4RecModel  core/models/kebert4rec/kebert4rec_model.py:24-89
  NarmModel        core/models/narm/narm_model.py:25-68 (+ components.py, layers.py)
`forward(InputSequence) -> Tensor | (Tensor, Tensor)` follows SequenceRecommenderModel.forward
(core/models/sequence_recommendation_model.py:35-53): embed -> represent -> modify -> project.
"""
from __future__ import annotations

import functools
from typing import Any, Dict, List, Optional

import torch
import torch.nn.functional as F
from torch import nn

from . import layers as Ly
from . import ops
from .sequence import get_attribute


class SequenceRecommenderModel(nn.Module):
    def __init__(self, sequence_embedding_layer, sequence_representation_layer,
                 sequence_representation_modifier_layer, projection_layer):
        super().__init__()
        self._sequence_embedding_layer = sequence_embedding_layer
        self._sequence_representation_layer = sequence_representation_layer
        self._sequence_representation_modifier_layer = sequence_representation_modifier_layer
        self._projection_layer = projection_layer
        self.register_state_dict_pre_hook(lambda module, prefix, keep_vars: module.flush_table())
        # before a load: bring the table and its Adam moments current, so the loaded rows are not later
        # "caught up" with zero-gradient steps they never missed
        self.register_load_state_dict_pre_hook(lambda module, *args: module.flush_table())

    def flush_table(self):
        """Apply pending lazy-Adam updates of the item table (see ops.LazyTableState)."""
        table = self.item_table()
        tg = getattr(table, "_asme_table_grad", None) if table is not None else None
        if tg is not None and tg.lazy is not None:
            tg.lazy.flush()

    def encode(self, sequence) -> torch.Tensor:
        """embed -> represent -> modify; returns the representation fed to the projection."""
        emb = self._sequence_embedding_layer(sequence)
        rep = self._sequence_representation_layer(emb, sequence.padding_mask)
        return self._sequence_representation_modifier_layer(rep, sequence)

    def forward(self, sequence):
        return self._projection_layer(self.encode(sequence), sequence)

    def catalog_query(self, sequence):
        """(queries (N, d), item table (|V|, d), bias or None) such that the full-catalogue scores the
        inference forward would produce are queries . table^T (+ bias) -- for the fused evaluation
        (ops.catalog_rank) that never builds them.  None when the projection is not of that form."""
        return None

    def required_metadata_keys(self) -> List[str]:
        return []

    def optional_metadata_keys(self) -> List[str]:
        return []

    def item_table(self) -> Optional[nn.Parameter]:
        return None

    def table_grad_sparse_ok(self) -> bool:
        """True when every read of the item table goes through the gather kernels (no tied/bilinear
        full-catalogue head), so its gradient is row-sparse."""
        return False


class TransformerEncoderModel(SequenceRecommenderModel):
    """core/models/transformer/transformer_encoder_model.py:12-73"""

    def __init__(self, transformer_hidden_size: int, num_transformer_heads: int, num_transformer_layers: int,
                 transformer_dropout: float, embedding_layer, sequence_representation_modifier_layer,
                 projection_layer, bidirectional: bool = False, transformer_intermediate_size: int = None,
                 transformer_attention_dropout: float = None):
        if transformer_intermediate_size is None:
            transformer_intermediate_size = 4 * transformer_hidden_size
        transformer_layer = Ly.TransformerLayer(transformer_hidden_size, num_transformer_heads,
                                                num_transformer_layers, transformer_intermediate_size,
                                                transformer_dropout, attention_dropout=transformer_attention_dropout)
        rep = Ly.TransformerSequenceRepresentationComponent(transformer_layer, bidirectional=bidirectional)
        super().__init__(embedding_layer, rep, sequence_representation_modifier_layer, projection_layer)
        self.apply(self._init_weights)
        self.fuse_embedding_norm = True

    # The embedding output goes straight into block 0, whose first op is its input LayerNorm: with
    # fuse_embedding_norm (the default) the embedding kernel computes that LayerNorm too (ops.embedding ln3,
    # asme_embedding_ln_fwd) and hands LN(x) to block 0 on its output tensor.  The embedding holds the norm as a plain
    # attribute (`_asme_next_norm`, not a registered submodule: state_dict, parameters() and named_modules() are
    # unchanged).  Fallbacks, same results: any op between the embedding and block 0 makes a new tensor without the
    # hand-off, and block 0 normalises it itself; forward hooks on block 0's input norm (or global module hooks) make
    # block 0 call the norm as a module so the hooks run (layers.TransformerLayer.forward).
    @property
    def fuse_embedding_norm(self) -> bool:
        return self._embedding_norm_target() is not None and \
            "_asme_next_norm" in self._embedding_norm_target().__dict__

    @fuse_embedding_norm.setter
    def fuse_embedding_norm(self, on: bool):
        target = self._embedding_norm_target()
        if target is None:
            return  # this composition does not feed the embedding straight into block 0 (UBERT4Rec's user column)
        if on:
            norm = self._sequence_representation_layer.transformer_layer.transformer_blocks[0].input_sublayer.norm
            object.__setattr__(target, "_asme_next_norm", norm)
        else:
            target.__dict__.pop("_asme_next_norm", None)

    def _embedding_norm_target(self):
        emb = self._sequence_embedding_layer
        pre = type(emb) is Ly.PreFusionContextSequenceElementsRepresentationComponent
        target = emb.item_embedding_layer if pre else emb
        if len(self._sequence_representation_layer.transformer_layer.transformer_blocks) and \
                type(target) is Ly.TransformerEmbedding and (pre or type(emb) is Ly.TransformerEmbedding):
            return target
        return None

    @staticmethod
    def _init_weights(module):
        is_linear, is_emb = isinstance(module, nn.Linear), isinstance(module, nn.Embedding)
        if is_linear or is_emb:
            nn.init.xavier_normal_(module.weight.data)
        elif isinstance(module, nn.LayerNorm):
            module.bias.data.zero_()
            module.weight.data.fill_(1.0)
        if is_linear and module.bias is not None:
            module.bias.data.zero_()

    def encode_rows(self, sequence, rows: torch.Tensor, inverse: Optional[torch.Tensor] = None) -> torch.Tensor:
        """representations of the flattened positions `rows` only, (M, d) == encode(sequence).view(-1, d)[rows].
        The transformer runs on every position; the representation modifier is position-wise (Linear -> GELU -> LN,
        optionally after merging the position's attribute embeddings), so it runs on the selected rows alone
        (`forward_rows` of the modifier layers) -- a masked batch selects ~18 % of the positions.  `inverse`: the
        rows' inverse map (ops.row_inverse), if built ahead."""
        emb = self._sequence_embedding_layer(sequence)
        rep = self._sequence_representation_layer(emb, sequence.padding_mask)
        modifier = self._sequence_representation_modifier_layer
        rows_fn = getattr(modifier, "forward_rows", None)
        if rows_fn is None:
            rep = modifier(rep, sequence)
        picked = ops.select_rows(rep.reshape(-1, rep.shape[-1]), rows, inverse)
        return picked if rows_fn is None else rows_fn(picked, sequence, rows, inverse)

    def forward_rows(self, sequence, rows: torch.Tensor, inverse: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Full-catalogue logits for the flattened positions `rows` only, (M, |V|).  Identical to
        forward(sequence).view(-1, |V|)[rows] without the (B, L, |V|) tensor."""
        return self._projection_layer(self.encode_rows(sequence, rows, inverse), sequence)

    def head_weight_bias(self):
        """(W (|V|, d), b or None) when the projection is the linear / tied full-catalogue head h W^T + b
        (layers.py:105-109,138-143) -- the fused logits + cross-entropy kernels then apply; else None."""
        wb = getattr(self._projection_layer, "weight_bias", None)
        return wb() if wb is not None else None


def normal_initialize_weights(module: nn.Module, initializer_range: float = 0.2) -> None:
    """core/models/bert4rec/bert4rec_model.py:59-68"""
    is_linear, is_emb = isinstance(module, nn.Linear), isinstance(module, nn.Embedding)
    if is_linear or is_emb:
        module.weight.data.normal_(mean=0.0, std=initializer_range)
    elif isinstance(module, nn.LayerNorm):
        module.bias.data.zero_()
        module.weight.data.fill_(1.0)
    if is_linear and module.bias is not None:
        module.bias.data.zero_()


class SASRecModel(TransformerEncoderModel):
    def __init__(self, transformer_hidden_size: int, num_transformer_heads: int, num_transformer_layers: int,
                 item_vocab_size: int, max_seq_length: int, transformer_dropout: float,
                 prefusion_attributes: Dict[str, Dict[str, Any]] = None,
                 postfusion_attributes: Dict[str, Dict[str, Any]] = None,
                 additional_attributes_tokenizer: Dict[str, Any] = None, postfusion_merge_function: str = "add",
                 embedding_pooling_type: str = None, transformer_intermediate_size: int = None,
                 transformer_attention_dropout: float = None, mode: str = "neg_sampling"):
        self.additional_metadata_keys = list(prefusion_attributes or {}) + list(postfusion_attributes or {})
        emb = Ly.TransformerEmbedding(item_voc_size=item_vocab_size, max_seq_len=max_seq_length,
                                      embedding_size=transformer_hidden_size, dropout=transformer_dropout,
                                      embedding_pooling_type=embedding_pooling_type, positional_embedding=True)
        element_rep = Ly.PreFusionContextSequenceElementsRepresentationComponent(
            emb, transformer_hidden_size, prefusion_attributes, additional_attributes_tokenizer,
            dropout=transformer_dropout)
        self.mode = mode
        if mode == "neg_sampling":
            projection = Ly.SASRecProjectionComponent(emb)
        elif mode == "full":
            projection = Ly.LinearProjectionLayer(transformer_hidden_size, item_vocab_size)
        else:
            raise Exception(f"{mode} is an unknown projection mode. Choose either <full> or <neg_sampling>.")
        if postfusion_attributes is not None:
            modifier = Ly.PostFusionIdentitySequenceRepresentationModifierLayer(
                transformer_hidden_size, postfusion_attributes, additional_attributes_tokenizer,
                postfusion_merge_function)
        else:
            modifier = Ly.IdentitySequenceRepresentationModifierLayer()
        super().__init__(transformer_hidden_size=transformer_hidden_size, num_transformer_heads=num_transformer_heads,
                         num_transformer_layers=num_transformer_layers, transformer_dropout=transformer_dropout,
                         bidirectional=False, embedding_layer=element_rep,
                         sequence_representation_modifier_layer=modifier, projection_layer=projection,
                         transformer_intermediate_size=transformer_intermediate_size,
                         transformer_attention_dropout=transformer_attention_dropout)
        self.apply(self._init_weights)  # the reference initialises twice

    def required_metadata_keys(self):
        return self.additional_metadata_keys

    def catalog_query(self, sequence):
        """last valid position's representation vs the item table (SASRecProjectionComponent inference,
        sasrec/components.py:46-61); the 'full' mode's Linear head is weight + bias over |V| outputs."""
        rep = self.encode(sequence)
        idx = sequence.padding_mask.sum(-1) - 1
        last = rep[torch.arange(rep.shape[0], device=rep.device), idx]
        proj = self._projection_layer
        if isinstance(proj, Ly.SASRecProjectionComponent):
            return last, proj.embedding.get_item_embedding_weight(), None
        lin = getattr(proj, "linear", None)
        if isinstance(lin, nn.Linear):
            return last, lin.weight, lin.bias
        return None

    def item_table(self):
        return self._sequence_embedding_layer.item_embedding_layer.get_item_embedding_weight()

    def table_grad_sparse_ok(self) -> bool:
        return True


class BERT4RecModel(TransformerEncoderModel):
    def __init__(self, transformer_hidden_size: int, num_transformer_heads: int, num_transformer_layers: int,
                 item_vocab_size: int, max_seq_length: int, transformer_dropout: float,
                 project_layer_type: str = "transpose_embedding", embedding_pooling_type: str = None,
                 initializer_range: float = 0.02, transformer_intermediate_size: int = None,
                 transformer_attention_dropout: float = None):
        modifier = Ly.FFNSequenceRepresentationModifierComponent(transformer_hidden_size)
        # The reference passes embedding_pooling_type POSITIONALLY into TransformerEmbedding's 5th
        # parameter, `positional_embedding` (bert4rec_model.py:40-41 vs transformer_layers.py:21-28): with
        # the default None, BERT4Rec runs WITHOUT a position embedding.  Reproduced on purpose.
        emb = Ly.TransformerEmbedding(item_vocab_size, max_seq_length, transformer_hidden_size, transformer_dropout,
                                      embedding_pooling_type)
        projection = Ly.build_projection_layer(project_layer_type, transformer_hidden_size, item_vocab_size,
                                               emb.item_embedding.embedding)
        super().__init__(transformer_hidden_size=transformer_hidden_size, num_transformer_heads=num_transformer_heads,
                         num_transformer_layers=num_transformer_layers, transformer_dropout=transformer_dropout,
                         bidirectional=True, embedding_layer=emb,
                         projection_layer=projection, sequence_representation_modifier_layer=modifier,
                         transformer_intermediate_size=transformer_intermediate_size,
                         transformer_attention_dropout=transformer_attention_dropout)
        self.apply(functools.partial(normal_initialize_weights, initializer_range=initializer_range))

    def item_table(self):
        return self._sequence_embedding_layer.get_item_embedding_weight()

    def table_grad_sparse_ok(self) -> bool:
        return isinstance(self._projection_layer, Ly.LinearProjectionLayer)


class KeBERT4RecModel(TransformerEncoderModel):
    def __init__(self, transformer_hidden_size: int, num_transformer_heads: int, num_transformer_layers: int,
                 item_vocab_size: int, max_seq_length: int, transformer_dropout: float,
                 prefusion_attributes: Dict[str, Dict[str, Any]] = None,
                 postfusion_attributes: Dict[str, Dict[str, Any]] = None,
                 additional_attributes_tokenizer: Dict[str, Any] = None, postfusion_merge_function: str = "add",
                 positional_embedding: bool = True, embedding_pooling_type: str = None,
                 initializer_range: float = 0.02, transformer_intermediate_size: Optional[int] = None,
                 transformer_attention_dropout: Optional[float] = None):
        self.additional_metadata_keys = list(prefusion_attributes or {}) + list(postfusion_attributes or {})
        emb = Ly.TransformerEmbedding(item_vocab_size, max_seq_length, transformer_hidden_size, 0.0,
                                      positional_embedding=positional_embedding,
                                      embedding_pooling_type=embedding_pooling_type, norm_embedding=False)
        element_rep = Ly.PreFusionContextSequenceElementsRepresentationComponent(
            emb, transformer_hidden_size, prefusion_attributes, additional_attributes_tokenizer,
            dropout=transformer_dropout)
        if postfusion_attributes is not None:
            modifier = Ly.PostFusionContextSequenceRepresentationModifierComponent(
                transformer_hidden_size, postfusion_attributes, additional_attributes_tokenizer,
                postfusion_merge_function)
        else:
            modifier = Ly.FFNSequenceRepresentationModifierComponent(transformer_hidden_size)
        projection = Ly.build_projection_layer(Ly.PROJECT_TYPE_LINEAR, transformer_hidden_size, item_vocab_size,
                                               emb.item_embedding.embedding)
        super().__init__(transformer_hidden_size=transformer_hidden_size, num_transformer_heads=num_transformer_heads,
                         num_transformer_layers=num_transformer_layers, transformer_dropout=transformer_dropout,
                         embedding_layer=element_rep, sequence_representation_modifier_layer=modifier,
                         projection_layer=projection, bidirectional=True,
                         transformer_intermediate_size=transformer_intermediate_size,
                         transformer_attention_dropout=transformer_attention_dropout)
        self.apply(functools.partial(normal_initialize_weights, initializer_range=initializer_range))

    def required_metadata_keys(self):
        return self.additional_metadata_keys

    def item_table(self):
        return self._sequence_embedding_layer.item_embedding_layer.get_item_embedding_weight()

    def table_grad_sparse_ok(self) -> bool:
        return True


# ------------------------------------------------------------------------------------ UBERT4Rec
class _UserLinearUpscaler(nn.Module):
    """multi-hot(ids) -> Linear(vocab -> d) WITHOUT dropping the pad category (ubert4rec/components.py:13-31)"""

    def __init__(self, vocab_size: int, embed_size: int):
        super().__init__()
        self.linear = nn.Linear(vocab_size, embed_size)
        self.vocab_size = vocab_size

    def forward(self, content_input: torch.Tensor) -> torch.Tensor:
        table = self.linear.weight.t().contiguous()  # (vocab, d): column gather == row gather
        return ops.gather_sum(content_input, table, self.linear.bias, skip_zero=False, multi_hot=True)


def _build_user_embedding_type(embedding_type: str, vocab_size: int, hidden_size: int) -> nn.Module:
    """ubert4rec/components.py:33-46"""
    if embedding_type in ("user_embedding", "content_embedding"):
        return Ly._ContentEmbedding(num_embeddings=vocab_size, embedding_dim=hidden_size)
    if embedding_type == "linear_upscale":
        return Ly.LinearUpscaler(vocab_size=vocab_size, embed_size=hidden_size)
    if embedding_type == "user_linear_upscale":
        return _UserLinearUpscaler(vocab_size=vocab_size, embed_size=hidden_size)
    raise KeyError(embedding_type)


class UBERT4RecSequenceElementsRepresentationComponent(nn.Module):
    """ubert4rec/components.py:49-160: item + position rows (+ the additional attributes) on the embedding kernel,
    the user-attribute token prepended, + segment rows, LayerNorm, dropout -- every gather and the LN / dropout on
    the gfx950 kernels"""

    def __init__(self, item_embedding_layer: Ly.TransformerEmbedding, embedding_size: int,
                 additional_attributes: Optional[Dict[str, Dict[str, Any]]],
                 user_attributes: Optional[Dict[str, Dict[str, Any]]], additional_tokenizers: Dict[str, Any],
                 segment_embedding: bool = True, dropout: float = 0.0, replace_first_item: bool = False):
        super().__init__()
        if replace_first_item:
            raise NotImplementedError("replace_first_item (unused by UBERT4RecModel) is outside the hot path")
        self.segment_embedding = None
        self.item_embedding_layer = item_embedding_layer
        self.segment_embedding_active = segment_embedding
        self.attribute_types = 0
        self.replace_first_item = replace_first_item
        add = {}
        if additional_attributes is not None:
            for name, info in additional_attributes.items():
                vocab = len(additional_tokenizers["tokenizers." + name])
                add[name] = _build_user_embedding_type(info["embedding_type"], vocab, embedding_size)
            self.attribute_types += 1  # once for all additional attributes, as the reference counts
        self.additional_attribute_embeddings = nn.ModuleDict(add)
        users = {}
        if user_attributes is not None:
            for name, info in user_attributes.items():
                vocab = len(additional_tokenizers["tokenizers." + name])
                users[name] = _build_user_embedding_type(info["embedding_type"], vocab, embedding_size)
                self.attribute_types += 1
        self.user_attribute_embeddings = nn.ModuleDict(users)
        if self.segment_embedding_active:
            self.segment_embedding = Ly._ContentEmbedding(self.attribute_types, embedding_size)
        self.dropout_embedding = nn.Dropout(dropout)
        self.norm_embedding = nn.LayerNorm(embedding_size)

    def forward(self, sequence) -> torch.Tensor:
        extra = Ly._attribute_sum(self.additional_attribute_embeddings, sequence)
        emb = self.item_embedding_layer.embed(sequence.sequence, extra=extra)  # E[id] + P[pos] + attributes
        user = None
        for key, module in self.user_attribute_embeddings.items():
            meta = get_attribute(sequence, key)[:, 0:1]
            e = module(meta)
            user = e if user is None else user + e
        if user is not None:
            emb = torch.cat([user, emb], dim=1)
        if self.segment_embedding_active:
            B, T = emb.shape[0], emb.shape[1]
            segs = torch.ones(B, T, dtype=torch.int64, device=emb.device)
            if user is not None:
                segs[:, 0] = 0
            emb = emb + self.segment_embedding(segs)
        return ops.dropout(ops.layer_norm(emb, self.norm_embedding), Ly._p(self.dropout_embedding, self.training))


class UserTransformerSequenceRepresentationComponent(nn.Module):
    """ubert4rec/components.py:162-203: the transformer over [user token, items]; the key mask gains a valid user
    position; causal when bidirectional=False (as UBERT4RecModel builds it)"""

    def __init__(self, transformer_hidden_size: int, num_transformer_heads: int, num_transformer_layers: int,
                 transformer_dropout: float, user_attributes: Optional[Dict[str, Dict[str, Any]]], bidirectional: bool,
                 transformer_attention_dropout: Optional[float] = None,
                 transformer_intermediate_size: Optional[int] = None, replace_first_item: bool = False):
        super().__init__()
        self.user_attributes = user_attributes
        self.bidirectional = bidirectional
        self.replace_first_item = replace_first_item
        if transformer_intermediate_size is None:
            transformer_intermediate_size = 4 * transformer_hidden_size
        self.transformer_encoder = Ly.TransformerLayer(transformer_hidden_size, num_transformer_heads,
                                                       num_transformer_layers, transformer_intermediate_size,
                                                       transformer_dropout,
                                                       attention_dropout=transformer_attention_dropout)

    def forward(self, embedded: torch.Tensor, padding_mask: Optional[torch.Tensor]) -> torch.Tensor:
        if padding_mask is not None and self.user_attributes and not self.replace_first_item:
            padding_mask = torch.cat([torch.ones(padding_mask.shape[0], 1, dtype=padding_mask.dtype,
                                                 device=padding_mask.device), padding_mask], dim=1)
        kv = Ly.key_valid_mask(padding_mask, embedded.shape)
        return self.transformer_encoder(embedded, kv, causal=not self.bidirectional)


class UBERT4RecModel(TransformerEncoderModel):
    """core/models/ubert4rec/ubert4rec_model.py:16-92 -- the user-attribute BERT4Rec variant (the reference builds
    its transformer with bidirectional=False).  Output (B, L + 1, |V|) when user attributes are configured."""

    def __init__(self, transformer_hidden_size: int, num_transformer_heads: int, num_transformer_layers: int,
                 item_vocab_size: int, max_seq_length: int, transformer_dropout: float,
                 additional_attributes: Dict[str, Dict[str, Any]], additional_tokenizers: Dict[str, Any],
                 user_attributes: Dict[str, Dict[str, Any]], positional_embedding: bool, segment_embedding: bool,
                 embedding_pooling_type: str = None, initializer_range: float = 0.02,
                 transformer_intermediate_size: Optional[int] = None,
                 transformer_attention_dropout: Optional[float] = None):
        self.additional_userdata_keys = []
        self.additional_metadata_keys = []
        if user_attributes is not None:
            self.additional_metadata_keys = list(user_attributes.keys())
            self.additional_userdata_keys = list(user_attributes.keys())
            max_seq_length += 1
        if additional_attributes is not None:
            self.additional_metadata_keys = self.additional_metadata_keys + list(additional_attributes.keys())
        emb = Ly.TransformerEmbedding(item_vocab_size, max_seq_length, transformer_hidden_size, 0.0,
                                      embedding_pooling_type=embedding_pooling_type, norm_embedding=False,
                                      positional_embedding=positional_embedding)
        element_rep = UBERT4RecSequenceElementsRepresentationComponent(
            emb, transformer_hidden_size, additional_attributes, user_attributes, additional_tokenizers,
            segment_embedding, dropout=transformer_dropout, replace_first_item=False)
        modifier = Ly.FFNSequenceRepresentationModifierComponent(transformer_hidden_size)
        projection = Ly.build_projection_layer(Ly.PROJECT_TYPE_LINEAR, transformer_hidden_size, item_vocab_size,
                                               emb.item_embedding.embedding)
        super().__init__(transformer_hidden_size=transformer_hidden_size, num_transformer_heads=num_transformer_heads,
                         num_transformer_layers=num_transformer_layers, transformer_dropout=transformer_dropout,
                         embedding_layer=element_rep, sequence_representation_modifier_layer=modifier,
                         projection_layer=projection, bidirectional=False,
                         transformer_intermediate_size=transformer_intermediate_size,
                         transformer_attention_dropout=transformer_attention_dropout)
        self._sequence_representation_layer = UserTransformerSequenceRepresentationComponent(
            transformer_hidden_size, num_transformer_heads, num_transformer_layers, transformer_dropout,
            user_attributes, bidirectional=False, transformer_attention_dropout=transformer_attention_dropout,
            transformer_intermediate_size=transformer_intermediate_size)
        self.apply(functools.partial(normal_initialize_weights, initializer_range=initializer_range))

    def required_metadata_keys(self):
        return self.additional_metadata_keys

    def optional_metadata_keys(self):
        return self.additional_userdata_keys

    def item_table(self):
        return self._sequence_embedding_layer.item_embedding_layer.get_item_embedding_weight()

    def table_grad_sparse_ok(self) -> bool:
        return True


# ------------------------------------------------------------------------------------ NARM
class SequenceElementsEmbeddingComponent(nn.Module):
    """core/models/common/components/representations/sequence_embedding.py:12-35"""

    def __init__(self, vocabulary_size: int, embedding_size: int, pooling_type: Optional[str] = None,
                 dropout: Optional[float] = None):
        super().__init__()
        self.elements_embedding = Ly.SequenceElementsEmbeddingLayer(vocabulary_size, embedding_size, pooling_type,
                                                                    dropout)

    def forward(self, sequence) -> torch.Tensor:
        return self.elements_embedding(sequence.sequence)


class LocalEncoderLayer(nn.Module):
    """v . sigmoid(A1 c_g + A2 h_i), masked weighted sum (core/models/narm/layers.py:8-66): the projections on the
    Linear kernels, the attention and weighted sum on asme_narm_attend_fwd/_bwd"""

    def __init__(self, hidden_size: int, latent_size: int):
        super().__init__()
        self.A1 = nn.Linear(hidden_size, latent_size, bias=False)
        self.A2 = nn.Linear(hidden_size, latent_size, bias=False)
        self.v = nn.Parameter(torch.empty(latent_size))
        self.projection_activation = nn.Sigmoid()
        torch.nn.init.uniform_(self.v, -1.0, 1.0)

    def forward(self, s1, s2, mask):
        return ops.narm_attend(ops.linear(s1, self.A1.weight), ops.linear(s2, self.A2.weight), self.v, s2, mask)


class NARMSequenceRepresentationComponent(nn.Module):
    """GRU global encoder + attentive local encoder (core/models/narm/components.py:14-56).
    The reference packs the padded batch (lengths.cpu(): a host sync); the GRU is causal,
    so running it on the padded batch (ops.gru: the recurrence kernel) and reading the output at len-1 gives
    the same c_g and the same masked local context without leaving the device.  nn.GRU is kept for its
    parameters, initialisation and state_dict keys only; its forward (MIOpen) is never called."""

    def __init__(self, item_embedding_size: int, global_encoder_size: int, global_encoder_num_layers: int,
                 context_dropout: float, batch_first: bool = True):
        super().__init__()
        self.batch_first = batch_first
        self.global_encoder = nn.GRU(item_embedding_size, global_encoder_size, num_layers=global_encoder_num_layers,
                                     batch_first=batch_first)
        self.local_encoder = LocalEncoderLayer(global_encoder_size, global_encoder_size)
        self.context_dropout = nn.Dropout(context_dropout)

    def forward(self, embedded: torch.Tensor, padding_mask: torch.Tensor) -> torch.Tensor:
        h_i = ops.gru(embedded, self.global_encoder)
        last = padding_mask.sum(-1) - 1
        c_g = h_i[torch.arange(h_i.shape[0], device=h_i.device), last]
        c_l = self.local_encoder(c_g, h_i, padding_mask)
        return ops.dropout(torch.cat([c_g, c_l], dim=1), Ly._p(self.context_dropout, self.training))


class BilinearDecoderLayer(nn.Module):
    """scores = context . (B E_items)^T over all items (core/models/narm/layers.py:69-120).  The item matrix
    goes through the embedding layer as in the reference, i.e. with its dropout in training (Dropout2d on the 2-D
    (|V|, E) matrix = independent elements, layers.py:113-117); W_eff = B(E_items) is a Linear kernel and the
    scores are the logits kernel (or, in training, never materialised: NarmModel.context_and_head)."""

    def __init__(self, embedding_layer: Ly.SequenceElementsEmbeddingLayer, encoded_representation_size: int,
                 apply_softmax: bool = False):
        super().__init__()
        self.embedding_layer = embedding_layer
        self.B = nn.Linear(embedding_layer.embedding.weight.size()[1], encoded_representation_size, bias=False)
        self.activation = nn.Softmax() if apply_softmax else nn.Identity()

    def item_weight(self, items: torch.Tensor = None) -> torch.Tensor:
        """B(embedding_layer(items)) (NI, 2H); all items when items is None"""
        emb = self.embedding_layer.item_matrix() if items is None else self.embedding_layer(items, flatten=False)
        return ops.linear(emb, self.B.weight)

    def forward(self, context: torch.Tensor, items: torch.Tensor = None):
        return self.activation(ops.logits(context, self.item_weight(items)))


class BilinearProjectionComponent(nn.Module):
    def __init__(self, embedding_layer, encoded_representation_size: int, apply_softmax: bool = False):
        super().__init__()
        self.decoder = BilinearDecoderLayer(embedding_layer, encoded_representation_size, apply_softmax)

    def forward(self, representation: torch.Tensor, sequence=None):
        return self.decoder(representation)


class NarmModel(SequenceRecommenderModel):
    def __init__(self, item_vocab_size: int, item_embedding_size: int, global_encoder_size: int,
                 global_encoder_num_layers: int, embedding_dropout: float, context_dropout: float,
                 batch_first: bool = True, embedding_pooling_type: str = None):
        emb = SequenceElementsEmbeddingComponent(item_vocab_size, item_embedding_size, embedding_pooling_type,
                                                 embedding_dropout)
        rep = NARMSequenceRepresentationComponent(item_embedding_size, global_encoder_size,
                                                  global_encoder_num_layers, context_dropout, batch_first)
        modifier = Ly.IdentitySequenceRepresentationModifierLayer()
        projection = BilinearProjectionComponent(emb.elements_embedding, 2 * global_encoder_size)
        super().__init__(emb, rep, modifier, projection)

    def item_table(self):
        return self._sequence_embedding_layer.elements_embedding.embedding.weight

    def context_and_head(self, sequence):
        """(context (N, 2H), W_eff (|V|, 2H)) with forward(sequence) == context . W_eff^T (no softmax head): the
        single-target cross-entropy then runs on the fused logits kernels without the (N, |V|) scores"""
        decoder = self._projection_layer.decoder
        if not isinstance(decoder.activation, nn.Identity):
            return None
        return self.encode(sequence), decoder.item_weight()

    def catalog_query(self, sequence):
        cw = self.context_and_head(sequence)
        return None if cw is None else (cw[0], cw[1], None)
