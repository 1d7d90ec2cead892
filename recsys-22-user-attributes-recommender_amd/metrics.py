"""Ranking metrics (NDCG@k / recall@k / MRR@k) for full-catalogue evaluation on the device.

Reference: core/metrics/common.py:4-27,118-175 (get_true_positives / calc_ndcg / calc_dcg),
core/metrics/metric.py:18-108 (sum / count state, compute = sum / count, dist_reduce_fx='sum'),
core/metrics/mrr.py, recall.py, ndcg.py, core/metrics/container/metrics_sampler.py:45-72 (AllItemsSampler).

Single-target rows (next-item / cloze evaluation) never sort: the `asme_target_rank` kernel counts the
items that outrank the target (ties broken by lower id), which is exactly the target's position in a
descending order, so NDCG@k = 1/log2(rank+1) for rank <= k.  The reference argsorts the whole (B, |V|)
matrix (unstable for ties); on tie-free scores both agree exactly.
Rows with several positives (basket targets) use a top-k path in PyTorch (outside the hot path).
"""
from __future__ import annotations

from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from . import ops


def _dcg_weights(k: int, device) -> torch.Tensor:
    return 1.0 / torch.log2(torch.arange(2, k + 2, device=device, dtype=torch.float32))


def ndcg_from_ranks(ranks: torch.Tensor, k: int) -> torch.Tensor:
    r = ranks.to(torch.float32)
    val = 1.0 / torch.log2(r + 1.0)
    return torch.where(ranks <= k, val, torch.zeros_like(val))


def recall_from_ranks(ranks: torch.Tensor, k: int) -> torch.Tensor:
    return (ranks <= k).to(torch.float32)


def mrr_from_ranks(ranks: torch.Tensor, k: int) -> torch.Tensor:
    r = ranks.to(torch.float32)
    return torch.where(ranks <= k, 1.0 / r, torch.zeros_like(r))


def _multi_positive(prediction, positive_item_mask, k, metric_mask, kind):
    pred = prediction
    if metric_mask is not None:
        pred = pred.masked_fill(metric_mask == 0, torch.finfo(torch.float).min)
    kk = min(k, pred.shape[1])
    top = torch.topk(pred, kk, dim=1).indices
    tp = positive_item_mask.gather(1, top).to(torch.float32)
    n_rel = positive_item_mask.sum(1)
    if kind == "ndcg":
        w = _dcg_weights(kk, pred.device)
        dcg = (tp * w).sum(1)
        idcg_w = _dcg_weights(k, pred.device)
        rel = torch.clamp(n_rel.to(torch.int64), max=k)
        idcg = (idcg_w.unsqueeze(0) * (torch.arange(k, device=pred.device).unsqueeze(0) < rel.unsqueeze(1))).sum(1)
        out = dcg / idcg
        out[torch.isnan(out)] = 0
        return out
    if kind == "recall":
        out = tp.sum(1) / n_rel
        out[torch.isnan(out)] = 0
        return out
    ranks = torch.arange(1, kk + 1, device=pred.device).unsqueeze(0)
    rank = (ranks * tp).max(dim=-1).values
    out = 1 / rank
    out[out == float("inf")] = 0
    return out


class RankingMetric(torch.nn.Module):
    kind = ""
    label = ""

    def __init__(self, k: int, dist_sync_on_step: bool = False, storage_mode=None):
        super().__init__()
        self._k = k
        self.reset()

    def reset(self):
        self.value_sum = torch.zeros((), dtype=torch.float32)
        self.count = torch.zeros((), dtype=torch.int64)

    def _accumulate(self, per_row: torch.Tensor):
        if self.value_sum.device != per_row.device:
            self.value_sum = self.value_sum.to(per_row.device)
            self.count = self.count.to(per_row.device)
        self.value_sum = self.value_sum + per_row.sum()
        self.count = self.count + per_row.shape[0]

    def from_ranks(self, ranks: torch.Tensor) -> torch.Tensor:
        return {"ndcg": ndcg_from_ranks, "recall": recall_from_ranks, "mrr": mrr_from_ranks}[self.kind](ranks,
                                                                                                    self._k)

    def update_ranks(self, ranks: torch.Tensor):
        self._accumulate(self.from_ranks(ranks))

    def update(self, predictions: torch.Tensor, positive_item_mask: torch.Tensor,
               metric_mask: Optional[torch.Tensor] = None):
        single = metric_mask is None and bool((positive_item_mask.sum(1) == 1).all())
        if single and predictions.is_cuda:
            targets = positive_item_mask.argmax(1)
            self.update_ranks(ops.target_rank(predictions.float(), targets))
        else:
            self._accumulate(_multi_positive(predictions.float(), positive_item_mask, self._k, metric_mask,
                                             self.kind))

    def forward(self, *args):
        return self.update(*args)

    def compute(self) -> torch.Tensor:
        s, c = self.value_sum, self.count
        if dist.is_available() and dist.is_initialized():
            t = torch.stack([s.to(torch.float64), c.to(torch.float64)])
            dist.all_reduce(t)
            return (t[0] / t[1]).to(torch.float32)
        return s / c

    def name(self) -> str:
        return f"{self.label}@{self._k}"


class NormalizedDiscountedCumulativeGainMetric(RankingMetric):
    kind, label = "ndcg", "NDCG"


class RecallMetric(RankingMetric):
    kind, label = "recall", "recall"


class MRRMetric(RankingMetric):
    kind, label = "mrr", "MRR"


class RankingMetricsContainer(torch.nn.Module):
    """AllItemsSampler container (metrics_container.py:68-127): every item is ranked."""

    def __init__(self, metrics: List[RankingMetric]):
        super().__init__()
        self.metrics = torch.nn.ModuleList(metrics)

    def update(self, input_seq, targets: torch.Tensor, predictions: torch.Tensor, mask=None) -> Dict[str, torch.Tensor]:
        if targets.dim() != 1:
            raise NotImplementedError("multi-target (basket) evaluation is outside the MI355X hot path")
        return self.update_ranks(ops.target_rank(predictions.float(), targets))

    def update_ranks(self, ranks: torch.Tensor) -> Dict[str, torch.Tensor]:
        """Accumulate from the targets' 1-based ranks directly (the fused full-catalogue path,
        ops.catalog_rank / sharded.catalog_ranks, never materialises the predictions)."""
        out = {}
        for m in self.metrics:
            per_row = m.from_ranks(ranks)
            m._accumulate(per_row)
            out[m.name()] = per_row.mean()
        return out

    def compute(self) -> Dict[str, torch.Tensor]:
        return {m.name(): m.compute() for m in self.metrics}

    def reset(self):
        for m in self.metrics:
            m.reset()

    def get_metric_names(self) -> List[str]:
        return [m.name() for m in self.metrics]
