"""Training modules: the boundary the ASME trainer calls (training_step / validation_step /
predict_step / configure_optimizers), re-provided with the reference's constructor signatures.

  SequenceNextItemPredictionTrainingModule  core/modules/sequence_next_item_prediction_training_module.py:22-185
  NextItemPredictionTrainingModule          core/modules/next_item_prediction_training_module.py:24-256
  MaskedTrainingModule                      core/modules/masked_training_module.py:20-189
  get_padding_mask / build_model_input      core/modules/util/module_util.py:13-30,106-151

Differences that do not change results:
  * full-catalogue losses are computed on the non-ignored rows only (identical loss, the
    (B, L, |V|) logits tensor is never built);
  * validation of sasrec-neg uses predict_step (the reference calls an undefined self.predict, Q13);
  * `table_grad="sparse"` keeps the item-table gradient row-sparse and lets FusedAdam apply the exact
    dense Adam update (Q7) without a dense (|V|, d) gradient.  It is the default (table_grad=None) for
    every model whose item table is only read through the gather kernels (table_grad_sparse_ok());
    tied / full-catalogue heads that read the whole table keep the dense gradient.
Batch keys: item, item.target, positive_samples, negative_samples (data/datasets/__init__.py:5-14).
"""
from __future__ import annotations

import inspect
from typing import Dict, Optional, Tuple

import torch
import torch.nn.functional as F
from torch import nn
from torch.optim.lr_scheduler import LambdaLR

from . import ops
from .losses import SASRecBinaryCrossEntropyLoss, SASRecFullSequenceCrossEntropyLoss, SingleTargetCrossEntropyLoss
from .optim import FusedAdam
from .sequence import InputSequence

ITEM_SEQ_ENTRY_NAME = "item"
TARGET_ENTRY_NAME = "item.target"
POSITIVE_SAMPLES_ENTRY_NAME = "positive_samples"
NEGATIVE_SAMPLES_ENTRY_NAME = "negative_samples"
LOG_KEY_TRAINING_LOSS = "train_loss"
LOG_KEY_VALIDATION_LOSS = "val_loss"
LOG_KEY_TEST_LOSS = "test_loss"

try:  # use Lightning when it is installed (the reference's trainer); otherwise a plain nn.Module
    import pytorch_lightning as _pl  # type: ignore

    _Base = _pl.LightningModule
except Exception:  # pragma: no cover - Lightning is not part of this image
    class _Base(nn.Module):
        def log(self, *args, **kwargs):
            pass

        def save_hyperparameters(self, *args, **kwargs):
            pass


# catalogue size from which validation ranks targets with the fused kernel (asme_catalog_rank) by default: every
# size -- the ranks (and so NDCG / recall / MRR) are those of the materialised scores, without the (B, |V|)
# prediction tensor (4 GiB at B = 1024, |V| = 2^20) or its sort; fused_eval=False materialises them
FUSED_EVAL_MIN_ITEMS = 0


def get_padding_mask(sequence: torch.Tensor, tokenizer) -> torch.Tensor:
    """sequence != pad (core/modules/util/module_util.py:13-30); a device int64 batch on asme_padding_mask"""
    if sequence.dim() > 2:
        sequence = sequence.max(dim=2).values
    if sequence.is_cuda and sequence.dtype == torch.int64:
        return ops.padding_mask(sequence, tokenizer.pad_token_id)
    return sequence.ne(tokenizer.pad_token_id)


def get_additional_meta_data(model, batch: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    metadata = {}
    for key in model.required_metadata_keys():
        if key not in batch:
            raise Exception(f"The batch does not contain the following additional metadata: {key}. "
                            f"Found the following batch entries: {', '.join(batch.keys())}")
        metadata[key] = batch[key]
    for key in model.optional_metadata_keys():
        if key in batch:
            metadata[key] = batch[key]
    return metadata


def build_model_input(model, item_tokenizer, batch) -> InputSequence:
    seq = batch[ITEM_SEQ_ENTRY_NAME]
    return InputSequence(seq, get_padding_mask(seq, item_tokenizer), get_additional_meta_data(model, batch))


def build_eval_step_return_dict(input_sequence, predictions, targets, mask=None) -> Dict[str, torch.Tensor]:
    d = {"sequence": input_sequence, "predictions": predictions, "targets": targets}
    if mask is not None:
        d["mask"] = mask
    return d


class _TableGradMixin:
    """Row-sparse item-table gradients (see ops.SparseTablePlan / optim.FusedAdam)."""

    def _init_table_grad(self, mode: Optional[str]):
        if mode is None:
            mode = "sparse" if self.model.table_grad_sparse_ok() else "dense"
        if mode not in ("dense", "sparse"):
            raise ValueError("table_grad must be 'dense' or 'sparse'")
        if mode == "sparse" and not self.model.table_grad_sparse_ok():
            raise ValueError(f"{type(self.model).__name__} reads the whole item table in its head; "
                             "use table_grad='dense'")
        self.table_grad = mode
        self._slot_map = None
        self._spare_map = None   # the second slot map of the ids-ahead path (prefetch_table_ids)
        self._ids_ahead = None   # ops.TableIdsAhead of the next training step's ids
        self.ids_ahead_hits = 0  # training steps that took a dedup made ahead (tests assert the overlap ran)
        # the catalogue's bf16 planes for fused evaluation, split once per validation pass (ops.CatalogPlanes)
        self._catalog_planes = ops.CatalogPlanes()


    def _plan_table(self, id_sets):
        self._catalog_planes.clear()  # training again: the evaluation's catalogue planes are stale (and 6 B / element)
        if self.table_grad != "sparse" or not self.training:
            return
        table = self.model.item_table()
        if table is None or not table.requires_grad:
            return
        if self._slot_map is None or self._slot_map.device != table.device:
            self._slot_map = ops.new_slot_map(table.shape[0], table.device)
            self._spare_map = None
        ahead, self._ids_ahead = self._ids_ahead, None
        if ahead is not None and not ahead.matches(id_sets):
            ahead.discard()  # prefetched for other tensors: its map entries reset, the dedup runs inline below
            ahead = None
        if ahead is not None:  # its dedup used the spare map: that becomes this plan's map
            self._slot_map, self._spare_map = self._spare_map, self._slot_map
            self.ids_ahead_hits += 1
        tg = table._asme_table_grad
        if tg.plan is not None and not tg.plan.consumed:
            if tg.plan.has_gradient():
                # a backward's table gradient that neither optimizer.step() applied nor optimizer.zero_grad() dropped
                # (FusedAdam.zero_grad is the skip signal: GradScaler / a trainer skipping the step call it, gradient
                # accumulation -- the trainer's accumulate_grad_batches, trainer_builder.py:25 -- does not): the
                # per-step row-sparse plan cannot merge two backward passes, so this fails instead of dropping it
                raise RuntimeError("table_grad='sparse' takes one backward per optimizer step (the previous "
                                   "backward's item-table gradient was neither applied by optimizer.step() nor "
                                   "dropped by optimizer.zero_grad()); use table_grad='dense' for gradient "
                                   "accumulation")
            tg.plan.release()  # a forward without a backward: nothing to lose
        tg.plan = ops.SparseTablePlan(table, id_sets, self._slot_map, ahead=ahead)

    def _prefetch_table_ids(self, id_sets):
        """the next training step's table-id dedup + occurrence CSR, enqueued now on the CURRENT stream (a producer's
        side stream) over the spare slot map -- see ops.TableIdsAhead.  The next training_step must receive the
        very same id tensors (else the prefetch is discarded and the dedup runs inline); it makes the training
        stream wait for this stream's work itself."""
        if self.table_grad != "sparse" or not self.training:
            return
        table = self.model.item_table()
        if table is None or not table.requires_grad or not table.is_cuda:
            return
        if self._ids_ahead is not None:
            self._ids_ahead.discard()
            self._ids_ahead = None
        if self._slot_map is None or self._slot_map.device != table.device:
            self._slot_map = ops.new_slot_map(table.shape[0], table.device)
            self._spare_map = None
        if self._spare_map is None:
            self._spare_map = ops.new_slot_map(table.shape[0], table.device)
        self._ids_ahead = ops.TableIdsAhead(table.shape[0], table.shape[1], id_sets, self._spare_map)

    @staticmethod
    def _ids_i64(batch, keys):
        """the id tensors the sparse plan registers must be the very tensors the model later reads: normalise
        int32 / non-contiguous dataloader ids to int64 contiguous once, up front"""
        out = dict(batch)
        for k in keys:
            t = out.get(k)
            if t is not None and (t.dtype != torch.int64 or not t.is_contiguous()):
                out[k] = t.to(torch.int64).contiguous()
        return out

    def _flush_table(self):
        self.model.flush_table()

    def _update_metrics(self, targets: torch.Tensor, predictions: torch.Tensor):
        if self.metrics is not None and targets.dim() == 1:
            self.metrics.update(None, targets, predictions)


class SequenceNextItemPredictionTrainingModule(_TableGradMixin, _Base):
    def __init__(self, model, item_tokenizer, metrics, learning_rate: float = 0.001, beta_1: float = 0.99,
                 beta_2: float = 0.998, weight_decay: float = 1e-3,
                 loss_function=None, table_grad: Optional[str] = None, fused_eval: Optional[bool] = None):
        super().__init__()
        self.model = model
        self.learning_rate, self.beta_1, self.beta_2, self.weight_decay = learning_rate, beta_1, beta_2, weight_decay
        self.item_tokenizer = item_tokenizer
        self.metrics = metrics
        self.loss_function = loss_function if loss_function is not None else SASRecBinaryCrossEntropyLoss()
        self._init_table_grad(table_grad)
        # fused_eval: rank the targets with asme_catalog_rank instead of materialising (B, |V|) predictions
        # (None = automatically from |V| >= FUSED_EVAL_MIN_ITEMS); validation then returns predictions=None
        self.fused_eval = fused_eval

    def training_step(self, batch, batch_idx):
        batch = self._ids_i64(batch, (ITEM_SEQ_ENTRY_NAME, POSITIVE_SAMPLES_ENTRY_NAME, NEGATIVE_SAMPLES_ENTRY_NAME))
        input_seq = batch[ITEM_SEQ_ENTRY_NAME]
        padding_mask = get_padding_mask(input_seq, self.item_tokenizer)
        pos, neg = batch[POSITIVE_SAMPLES_ENTRY_NAME], batch[NEGATIVE_SAMPLES_ENTRY_NAME]
        meta = get_additional_meta_data(self.model, batch)
        meta["positive_samples"], meta["negative_samples"] = pos, neg
        self._plan_table([input_seq, pos, neg])
        pos_logits, neg_logits = self.model(InputSequence(input_seq, padding_mask, meta))
        # the loss mask is the padding mask of the (B, L) input (the reference recomputes input_seq != pad)
        item_mask = padding_mask if input_seq.dim() == 2 else input_seq.ne(self.item_tokenizer.pad_token_id)
        loss = self.loss_function(pos_logits, neg_logits, mask=item_mask)
        self.log(LOG_KEY_TRAINING_LOSS, loss)
        return {"loss": loss}

    _ID_KEYS = (ITEM_SEQ_ENTRY_NAME, POSITIVE_SAMPLES_ENTRY_NAME, NEGATIVE_SAMPLES_ENTRY_NAME)

    def prefetch(self, batch):
        """Dedup the NEXT training step's table ids (sequence, positives, negatives) and build their occurrence CSR
        now, on the current stream -- the stream that produced `batch`, one step ahead (the reference's DataLoader
        workers run a batch ahead the same way).  The next training_step must receive this batch's very id
        tensors (int64, contiguous: as the GPU producer writes them); it waits for this stream's work itself."""
        ids = [batch[k] for k in self._ID_KEYS]
        if any(t.dtype != torch.int64 or not t.is_contiguous() for t in ids):
            return  # (training_step would normalise them into other tensors: nothing to match)
        self._prefetch_table_ids(ids)

    def predict_step(self, batch, batch_idx, dataloader_idx: Optional[int] = None) -> torch.Tensor:
        self._flush_table()
        input_seq = batch[ITEM_SEQ_ENTRY_NAME]
        meta = get_additional_meta_data(self.model, batch)
        padding_mask = get_padding_mask(input_seq, self.item_tokenizer)
        n = len(self.item_tokenizer.get_vocabulary())
        # the reference's items_to_rank (B, |V|) as a stride-0 view, tagged so the projection scores the whole
        # catalogue on the logits kernel without inspecting it (no (B, |V|) int64 buffer, no host sync)
        items = torch.arange(n, dtype=torch.long, device=input_seq.device).expand(input_seq.shape[0], n)
        items._asme_all_items = True
        meta["positive_samples"] = items
        return self.model(InputSequence(input_seq, padding_mask, meta))

    def _use_fused_eval(self, targets) -> bool:
        if targets.dim() != 1 or self.metrics is None or not hasattr(self.metrics, "update_ranks"):
            return False
        if self.fused_eval is not None:
            return bool(self.fused_eval)
        return self.model.item_table().shape[0] >= FUSED_EVAL_MIN_ITEMS

    def catalog_ranks(self, batch) -> torch.Tensor:
        """1-based full-catalogue rank of each sequence's target (ties to the lower id) with the scores
        streamed through asme_catalog_rank -- no (B, |V|) predictions."""
        self._flush_table()
        input_seq, targets = batch[ITEM_SEQ_ENTRY_NAME], batch[TARGET_ENTRY_NAME]
        meta = get_additional_meta_data(self.model, batch)
        padding_mask = get_padding_mask(input_seq, self.item_tokenizer)
        q = self.model.catalog_query(InputSequence(input_seq, padding_mask, meta))
        if q is None:
            raise NotImplementedError("model projection is not a dot product with an item table")
        h, table, bias = q
        return ops.catalog_rank(h, table, targets, bias, planes=self._catalog_planes.get(table))

    def validation_step(self, batch, batch_idx):
        input_seq, targets = batch[ITEM_SEQ_ENTRY_NAME], batch[TARGET_ENTRY_NAME]
        if self._use_fused_eval(targets):
            with torch.no_grad():
                self.metrics.update_ranks(self.catalog_ranks(batch))
            return build_eval_step_return_dict(input_seq, None, targets)
        prediction = self.predict_step(batch, batch_idx)
        self._update_metrics(targets, prediction)
        mask = None if targets.dim() == 1 else ~targets.eq(self.item_tokenizer.pad_token_id)
        return build_eval_step_return_dict(input_seq, prediction, targets, mask=mask)

    def test_step(self, batch, batch_idx):
        return self.validation_step(batch, batch_idx)

    def configure_optimizers(self):
        return FusedAdam(self.parameters(), lr=self.learning_rate, betas=(self.beta_1, self.beta_2),
                         weight_decay=self.weight_decay)


def _instantiate_loss(loss_function, item_tokenizer):
    if loss_function is None:
        return SingleTargetCrossEntropyLoss(item_tokenizer)
    if inspect.isclass(loss_function):
        if "item_tokenizer" in inspect.signature(loss_function).parameters:
            return loss_function(item_tokenizer=item_tokenizer)
        return loss_function()
    return loss_function


# Full-catalogue CE heads (linear / tied): True (default) = asme_linear_xent_* (csrc/logits.hip: bf16x6 MFMA logits +
# online LSE + dH/dW passes, the (n, |V|) logits never stored; at BERT4Rec C3, 37k x 27k, 7.2 ms against 10.0 ms for
# library-GEMM logits + CE, tools/xent_bench.py); False = materialised logits on asme_logits + the CE kernels.
FUSED_XENT: bool = True


def _rows_cross_entropy(model, sequence, rows, targets, pad: int, inverse=None) -> torch.Tensor:
    """CrossEntropyLoss(ignore_index=pad) of the full-catalogue logits at the flattened positions `rows`
    (masked_training_module.py:93-111 / losses.py:77-115).  With a linear or tied head the logits are never
    materialised (ops.linear_cross_entropy); otherwise they are, for the selected rows only.  `inverse`: the rows'
    inverse map (ops.row_inverse) when built ahead."""
    wb = model.head_weight_bias() if hasattr(model, "head_weight_bias") else None
    if wb is not None:
        h = model.encode_rows(sequence, rows, inverse)
        if FUSED_XENT and ops.linear_xent_ok(h, wb[0], wb[1]):
            return ops.linear_cross_entropy(h, wb[0], wb[1], targets, pad)
        return ops.cross_entropy(ops.logits(h, wb[0], wb[1]), targets, pad)
    return ops.cross_entropy(model.forward_rows(sequence, rows, inverse), targets, pad)


def _single_target_cross_entropy(model, sequence, targets, pad: int) -> torch.Tensor:
    """SingleTargetCrossEntropyLoss(context . W^T) for a bilinear head (NARM, losses.py:77-115 + narm/layers.py:
    93-120): the fused logits + cross-entropy kernels where the width fits them, else logits on the Linear kernel
    followed by the cross-entropy kernel."""
    cw = model.context_and_head(sequence)
    if cw is None:
        return ops.cross_entropy(model(sequence), targets, pad)
    context, weight = cw
    if FUSED_XENT and ops.linear_xent_ok(context, weight):
        return ops.linear_cross_entropy(context, weight, None, targets, pad)
    return ops.cross_entropy(ops.logits(context, weight), targets, pad)


class NextItemPredictionTrainingModule(_TableGradMixin, _Base):
    def __init__(self, model, item_tokenizer, metrics, learning_rate: float = 0.001, beta_1: float = 0.99,
                 beta_2: float = 0.998, weight_decay: float = 0, loss_function=None, table_grad: Optional[str] = None):
        super().__init__()
        self.model = model
        self.learning_rate, self.beta_1, self.beta_2, self.weight_decay = learning_rate, beta_1, beta_2, weight_decay
        self.item_tokenizer = item_tokenizer
        self.metrics = metrics
        self.loss_function = _instantiate_loss(loss_function, item_tokenizer)
        self._init_table_grad(table_grad)

    def forward(self, batch, batch_idx: Optional[int] = None) -> torch.Tensor:
        return self.model(build_model_input(self.model, self.item_tokenizer, batch))

    def training_step(self, batch, batch_idx):
        batch = self._ids_i64(batch, (ITEM_SEQ_ENTRY_NAME,))
        target = batch[TARGET_ENTRY_NAME]
        pad = self.item_tokenizer.pad_token_id
        ce_loss = isinstance(self.loss_function, (SASRecFullSequenceCrossEntropyLoss, SingleTargetCrossEntropyLoss))
        self._plan_table([batch[ITEM_SEQ_ENTRY_NAME]])
        if ce_loss and target.dim() == 2 and hasattr(self.model, "forward_rows"):
            # per-step targets: only the non-pad positions contribute to the CE
            rows = torch.nonzero(target.reshape(-1) != pad).squeeze(1)
            loss = _rows_cross_entropy(self.model, build_model_input(self.model, self.item_tokenizer, batch), rows,
                                       target.reshape(-1).index_select(0, rows), pad)
        elif ce_loss and target.dim() == 1 and hasattr(self.model, "context_and_head"):
            loss = _single_target_cross_entropy(self.model, build_model_input(self.model, self.item_tokenizer, batch),
                                                target, pad)
        else:
            loss = self.loss_function(target, self(batch, batch_idx))
        self.log(LOG_KEY_TRAINING_LOSS, loss)
        return {"loss": loss}

    def _extract_target_logits(self, input_seq, logits):
        seq_length = get_padding_mask(input_seq, self.item_tokenizer).sum(dim=-1) - 1
        return logits[torch.arange(input_seq.shape[0], device=logits.device), seq_length]

    def _last_position_logits(self, batch):
        self._flush_table()
        input_seq = batch[ITEM_SEQ_ENTRY_NAME]
        if hasattr(self.model, "forward_rows"):
            L = input_seq.shape[1]
            last = get_padding_mask(input_seq, self.item_tokenizer).sum(dim=-1) - 1
            rows = torch.arange(input_seq.shape[0], device=input_seq.device) * L + last
            return self.model.forward_rows(build_model_input(self.model, self.item_tokenizer, batch), rows)
        logits = self(batch)
        return self._extract_target_logits(input_seq, logits) if logits.dim() == 3 else logits

    def validation_step(self, batch, batch_idx):
        input_seq, target = batch[ITEM_SEQ_ENTRY_NAME], batch[TARGET_ENTRY_NAME]
        target_logits = self._last_position_logits(batch)
        loss = self.loss_function(target, target_logits)
        self.log(LOG_KEY_VALIDATION_LOSS, loss, prog_bar=True)
        self._update_metrics(target, target_logits)
        mask = None if target.dim() == 1 else ~target.eq(self.item_tokenizer.pad_token_id)
        return build_eval_step_return_dict(input_seq, target_logits, target, mask=mask)

    def test_step(self, batch, batch_idx):
        return self.validation_step(batch, batch_idx)

    def predict_step(self, batch, batch_idx, dataloader_idx: Optional[int] = None):
        return self._last_position_logits(batch)

    def configure_optimizers(self):
        return FusedAdam(self.parameters(), lr=self.learning_rate, betas=(self.beta_1, self.beta_2),
                         weight_decay=self.weight_decay)


class MaskedTrainingModule(_TableGradMixin, _Base):
    def __init__(self, model, item_tokenizer, metrics, learning_rate: float = 0.001, beta_1: float = 0.99,
                 beta_2: float = 0.998, weight_decay: float = 0.001, num_warmup_steps: int = 10000,
                 table_grad: Optional[str] = None, fused_eval: Optional[bool] = None):
        super().__init__()
        self.model = model
        self.learning_rate, self.beta_1, self.beta_2 = learning_rate, beta_1, beta_2
        self.weight_decay = weight_decay  # accepted but unused by the optimizer, as in the reference (Q7)
        self.num_warmup_steps = num_warmup_steps
        self.item_tokenizer = item_tokenizer
        self.metrics = metrics
        # fused_eval: rank each masked position's target with asme_catalog_rank from its hidden state and the head
        # (no (n, |V|) predictions; needs a linear / tied head, one target per sequence and a rank-based metrics
        # container); None = whenever that holds.  Validation then returns predictions=None.
        self.fused_eval = fused_eval
        self._init_table_grad(table_grad)

    def forward(self, batch, batch_idx: Optional[int] = None) -> torch.Tensor:
        return self.model(build_model_input(self.model, self.item_tokenizer, batch))

    def training_step(self, batch, batch_idx):
        batch = self._ids_i64(batch, (ITEM_SEQ_ENTRY_NAME,))
        target = batch[TARGET_ENTRY_NAME]
        if target.dim() > 2:
            raise NotImplementedError("basket (multi-target) masked training is outside the MI355X hot path")
        pad = self.item_tokenizer.pad_token_id
        self._plan_table([batch[ITEM_SEQ_ENTRY_NAME]])
        ahead, self._rows_ahead = self._rows_ahead, None
        if ahead is not None and ahead[0] is target:
            rows, row_targets, inverse = ahead[1], ahead[2], ahead[3]
            if rows.is_cuda:
                # allocated on the prefetch's side stream, read on this one: keep the caching allocator from
                # handing their blocks back to the side stream before this stream's reads are done
                cur = torch.cuda.current_stream(rows.device)
                for t in (rows, row_targets, inverse):
                    t.record_stream(cur)
        else:
            rows = torch.nonzero(target.reshape(-1) != pad).squeeze(1)  # (reads the row count on the host)
            row_targets, inverse = target.reshape(-1).index_select(0, rows), None
        loss = _rows_cross_entropy(self.model, build_model_input(self.model, self.item_tokenizer, batch), rows,
                                   row_targets, pad, inverse)
        self.log(LOG_KEY_TRAINING_LOSS, loss, prog_bar=False)
        return {"loss": loss}

    _rows_ahead = None

    def prefetch(self, batch):
        """Select the NEXT training step's masked rows now (torch.nonzero: the host reads their count).  Called on
        the stream that produced `batch` (a side stream) once the current step is enqueued, the host waits only
        for that stream's work -- the cloze producer -- never for the main stream's queue, which a nonzero at the
        start of the step drains.  The next training_step must receive the very same target tensor; the caller
        makes the main stream wait for the side stream before that step (training_step itself records the
        prefetched tensors on its stream, so the caller need not record_stream them)."""
        target = batch[TARGET_ENTRY_NAME]
        if target.dim() != 2:
            return
        rows = torch.nonzero(target.reshape(-1) != self.item_tokenizer.pad_token_id).squeeze(1)
        # (with the rows' inverse map for the selection's backward, so the main stream never builds it)
        self._rows_ahead = (target, rows, target.reshape(-1).index_select(0, rows),
                            ops.row_inverse(rows, target.numel()))

    def _get_prediction_for_masked_item(self, batch, batch_idx=None) -> torch.Tensor:
        self._flush_table()
        rows = self._masked_rows(batch)
        return self.model.forward_rows(build_model_input(self.model, self.item_tokenizer, batch), rows)

    def _masked_rows(self, batch) -> torch.Tensor:
        target_mask = batch[ITEM_SEQ_ENTRY_NAME].eq(self.item_tokenizer.mask_token_id)
        if target_mask.dim() == 3:
            target_mask = target_mask.max(dim=-1).values
        return torch.nonzero(target_mask.reshape(-1)).squeeze(1)

    def catalog_ranks(self, batch) -> torch.Tensor:
        """1-based full-catalogue rank (ties to the lower id) of the target of each sequence's masked position
        (the last-item mask of evaluation, last_item_mask.py:35-44): the masked positions' hidden states against the
        head through asme_catalog_rank, no (n, |V|) predictions.  masked_training_module.py:80-91 + AllItemsSampler
        + NDCG's argsort (metrics/common.py:4-27)."""
        return self._fused_eval(batch, with_loss=False)[0]

    def _fused_eval(self, batch, with_loss: bool):
        """(ranks, loss or None) of the masked positions' targets from one encoder pass: the ranks streamed
        through asme_catalog_rank and, with_loss, the CrossEntropyLoss(ignore_index=pad) of the same hidden states
        on the fused logits + CE kernels (masked_training_module.py:145-147 logs it) -- no (n, |V|) predictions"""
        self._flush_table()
        sequence = build_model_input(self.model, self.item_tokenizer, batch)
        rows = self._masked_rows(batch)
        targets = batch[TARGET_ENTRY_NAME]
        if rows.numel() != targets.numel():
            raise ValueError("fused masked evaluation needs exactly one masked position per sequence")
        w, b = self.model.head_weight_bias()
        h = self.model.encode_rows(sequence, rows)
        ranks = ops.catalog_rank(h, w, targets, b, planes=self._catalog_planes.get(w))
        loss = None
        if with_loss:
            pad = self.item_tokenizer.pad_token_id
            loss = (ops.linear_cross_entropy(h, w, b, targets, pad) if ops.linear_xent_ok(h, w, b)
                    else ops.cross_entropy(ops.logits(h, w, b), targets, pad))
        return ranks, loss

    def _use_fused_eval(self, targets) -> bool:
        if targets.dim() != 1 or self.metrics is None or not hasattr(self.metrics, "update_ranks"):
            return False
        if not hasattr(self.model, "head_weight_bias") or self.model.head_weight_bias() is None:
            return False
        return True if self.fused_eval is None else bool(self.fused_eval)

    def _eval_step(self, batch, batch_idx, is_test: bool = False):
        input_seq, targets = batch[ITEM_SEQ_ENTRY_NAME], batch[TARGET_ENTRY_NAME]
        if self._use_fused_eval(targets) and self._masked_rows(batch).numel() == targets.numel():
            with torch.no_grad():
                ranks, loss = self._fused_eval(batch, with_loss=True)
                self.metrics.update_ranks(ranks)
            self.log(LOG_KEY_TEST_LOSS if is_test else LOG_KEY_VALIDATION_LOSS, loss, prog_bar=True)
            return build_eval_step_return_dict(input_seq, None, targets)
        prediction = self._get_prediction_for_masked_item(batch, batch_idx)
        loss = ops.cross_entropy(prediction, targets, self.item_tokenizer.pad_token_id)
        self.log(LOG_KEY_TEST_LOSS if is_test else LOG_KEY_VALIDATION_LOSS, loss, prog_bar=True)
        self._update_metrics(targets, prediction)
        mask = None if targets.dim() == 1 else ~targets.eq(self.item_tokenizer.pad_token_id)
        return build_eval_step_return_dict(input_seq, prediction, targets, mask=mask)

    def validation_step(self, batch, batch_idx):
        return self._eval_step(batch, batch_idx)

    def test_step(self, batch, batch_idx):
        return self._eval_step(batch, batch_idx, is_test=True)

    def predict_step(self, batch, batch_idx, dataloader_idx: Optional[int] = None):
        return self._get_prediction_for_masked_item(batch, batch_idx)

    def configure_optimizers(self):
        optimizer = FusedAdam(self.parameters(), lr=self.learning_rate, betas=(self.beta_1, self.beta_2))
        if self.num_warmup_steps > 0:
            warm = self.num_warmup_steps
            scheduler = LambdaLR(optimizer, lambda step: min(1.0, step / warm))
            return [optimizer], [{"scheduler": scheduler, "interval": "step", "strict": True}]
        return [optimizer]


class UBERTMaskedTrainingModule(MaskedTrainingModule):
    """core/modules/ubert_masked_training_module.py:20-208: masked-item training of UBERT4Rec, whose output has one
    more position (the user token) in front when user attributes are configured: the targets and the eval mask
    get a leading pad / False column.  Same loss (CrossEntropyLoss(ignore_index=pad), on the fused logits head),
    optimizer (Adam without weight decay) and warm-up as MaskedTrainingModule."""

    def __init__(self, model, item_tokenizer, metrics, learning_rate: float = 0.001, beta_1: float = 0.99,
                 beta_2: float = 0.998, weight_decay: float = 0.001, num_warmup_steps: int = 10000,
                 table_grad: Optional[str] = None):
        super().__init__(model, item_tokenizer, metrics, learning_rate, beta_1, beta_2, weight_decay,
                         num_warmup_steps, table_grad)
        self.user_key_len = len(model.optional_metadata_keys())

    def _use_fused_eval(self, targets) -> bool:
        return False  # the output carries the user column: predictions come from the overridden row extraction

    def _with_user_column(self, x: torch.Tensor, fill) -> torch.Tensor:
        if self.user_key_len == 0:
            return x
        return torch.cat([torch.full((x.shape[0], 1), fill, dtype=x.dtype, device=x.device), x], dim=1)

    def training_step(self, batch, batch_idx):
        batch = dict(batch)
        target = batch[TARGET_ENTRY_NAME]
        if target.dim() > 2:
            raise NotImplementedError("basket (multi-target) masked training is outside the MI355X hot path")
        batch[TARGET_ENTRY_NAME] = self._with_user_column(target, self.item_tokenizer.pad_token_id)
        return super().training_step(batch, batch_idx)

    def _get_prediction_for_masked_item(self, batch, batch_idx=None) -> torch.Tensor:
        self._flush_table()
        input_seq = batch[ITEM_SEQ_ENTRY_NAME]
        target_mask = input_seq.eq(self.item_tokenizer.mask_token_id)
        if target_mask.dim() == 3:
            target_mask = target_mask.max(dim=-1).values
        target_mask = self._with_user_column(target_mask, False)
        rows = torch.nonzero(target_mask.reshape(-1)).squeeze(1)
        return self.model.forward_rows(build_model_input(self.model, self.item_tokenizer, batch), rows)


def split_optimizers(configured):
    """Normalise configure_optimizers() output -> (optimizer, scheduler or None)."""
    if isinstance(configured, torch.optim.Optimizer):
        return configured, None
    if isinstance(configured, (list, tuple)) and len(configured) == 2 and isinstance(configured[0], list):
        opts, scheds = configured
        s = scheds[0]["scheduler"] if scheds and isinstance(scheds[0], dict) else (scheds[0] if scheds else None)
        return opts[0], s
    if isinstance(configured, (list, tuple)):
        return configured[0], None
    raise TypeError(f"unsupported optimizer configuration {type(configured)}")


_ONES: Dict[Tuple[torch.device, torch.dtype], torch.Tensor] = {}


def backward(loss: torch.Tensor):
    """loss.backward() with a cached scalar 1 as the seed gradient (autograd's implicit torch.ones_like is a fill
    launch per step)"""
    key = (loss.device, loss.dtype)
    one = _ONES.get(key)
    if one is None:
        one = _ONES[key] = torch.ones((), device=loss.device, dtype=loss.dtype)
    loss.backward(one if loss.dim() == 0 else None)


def train_step(module, optimizer, scheduler, batch, batch_idx: int = 0) -> torch.Tensor:
    """One optimisation step as Lightning's automatic optimisation runs it."""
    out = module.training_step(batch, batch_idx)
    loss = out["loss"]
    backward(loss)
    optimizer.step()
    if scheduler is not None:
        scheduler.step()
    optimizer.zero_grad(set_to_none=True)
    return loss
