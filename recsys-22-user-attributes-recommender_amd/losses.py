"""Losses of the hot path on the fused HIP kernels (same class names / call signatures as the reference).

  SASRecBinaryCrossEntropyLoss       core/losses/sasrec/sas_rec_losses.py:35-75
  SASRecFullSequenceCrossEntropyLoss core/losses/sasrec/sas_rec_losses.py:9-32
  SingleTargetCrossEntropyLoss       core/losses/losses.py:65-115
"""
from __future__ import annotations

import torch
from torch import nn

from . import ops


class SASRecBinaryCrossEntropyLoss(nn.Module):
    def __init__(self, reduction: str = "elementwise_mean"):
        super().__init__()
        self.reduction = reduction

    def forward(self, pos_input: torch.Tensor, neg_input: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
        # torchmetrics reduce(scalar, 'elementwise_mean') is the identity on the scalar mean
        return ops.sasrec_bce(pos_input, neg_input, mask)


class SASRecFullSequenceCrossEntropyLoss(nn.Module):
    def __init__(self, item_tokenizer):
        super().__init__()
        self.item_tokenizer = item_tokenizer

    def forward(self, target: torch.Tensor, logit: torch.Tensor) -> torch.Tensor:
        return ops.cross_entropy(logit.reshape(-1, logit.shape[-1]), target.reshape(-1),
                                 self.item_tokenizer.pad_token_id)


class SingleTargetCrossEntropyLoss(nn.Module):
    def __init__(self, item_tokenizer):
        super().__init__()
        self.item_tokenizer = item_tokenizer

    def forward(self, target: torch.Tensor, logits: torch.Tensor) -> torch.Tensor:
        td, ld = target.dim(), logits.dim()
        pad = self.item_tokenizer.pad_token_id
        if td == 1 and ld == 2:
            return ops.cross_entropy(logits, target, pad)
        if td == 2 and ld == 3:
            if logits.shape[1] != target.shape[1]:
                raise Exception(f"Number of sequence elements must be equal for logits and targets. "
                                f"logits: {tuple(logits.shape)}, targets: {tuple(target.shape)}")
            return ops.cross_entropy(logits.reshape(-1, logits.shape[2]), target.reshape(-1), pad)
        raise Exception(f"This loss can not be applied to logits and targets with these dimensions: "
                        f"logits: {tuple(logits.shape)}, target: {tuple(target.shape)}")
