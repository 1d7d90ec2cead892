"""GPU-side training-batch producers behind the reference's processor names.

The reference builds each sample in CPU DataLoader workers: a chain of per-session processors
(data/datasets/processors/*) followed by `_padded_session_collate` (data/collate.py:42-111).  Its negative
sampler builds a dense |V| weight vector per session (pos_neg_sampler.py:41-63), which at |I| = 10M caps the
input pipeline at ~22 sessions/s per core.  Here the sessions stay in HBM (`SessionStore`, flat item
ids + offsets) and each processor is one kernel over the whole batch (csrc/batch.hip):

  PositiveNegativeSamplerProcessor.process_batch  -> item / positive_samples / negative_samples (B, L)
  ClozeMaskProcessor.process_batch                -> item (masked) / item.target (B, L)
  padded_session_batch                            -> collated (B, L) items + lengths

Same semantics as the reference (left truncation to max_seq_length, right padding with PAD; negatives uniform
over the non-special ids absent from the whole session, with replacement; the cloze 80/10/10 rule with the
last-item-only branch).  Randomness is counter-based Philox keyed by a seed, so batches are reproducible; the
cloze kernel can also replay given draws (tests replay the reference's torch CPU generator bit-exactly).
"""
from __future__ import annotations

from typing import Dict, Optional, Sequence, Tuple

import torch

from . import _lib
from ._lib import call, ptr, stream
from .ops import new_seed

ITEM_SEQ_ENTRY_NAME = "item"
TARGET_ENTRY_NAME = "item.target"
POSITIVE_SAMPLES_ENTRY_NAME = "positive_samples"
NEGATIVE_SAMPLES_ENTRY_NAME = "negative_samples"


def _item_tokenizer(tokenizers):
    if isinstance(tokenizers, dict):
        for key in ("tokenizers.item", "item"):
            if key in tokenizers:
                return tokenizers[key]
        raise KeyError("no item tokenizer ('tokenizers.item') in the tokenizers")
    return tokenizers


class SessionStore:
    """Sessions in device memory: flat int64 item ids and int64 offsets (n + 1)."""

    def __init__(self, flat: torch.Tensor, offsets: torch.Tensor):
        if not flat.is_cuda or not offsets.is_cuda:
            raise _lib.ASMEKernelError("SessionStore lives on the GPU")
        self.flat = flat.to(torch.int64).contiguous()
        self.offsets = offsets.to(torch.int64).contiguous()
        self.n_sessions = self.offsets.numel() - 1

    @classmethod
    def from_lists(cls, sessions: Sequence[Sequence[int]], device) -> "SessionStore":
        lengths = torch.tensor([len(s) for s in sessions], dtype=torch.int64)
        offsets = torch.zeros(len(sessions) + 1, dtype=torch.int64)
        offsets[1:] = torch.cumsum(lengths, 0)
        flat = torch.tensor([v for s in sessions for v in s], dtype=torch.int64)
        return cls(flat.to(device), offsets.to(device))


def padded_session_batch(store: SessionStore, batch_idx: torch.Tensor, max_seq_length: int, pad_token_id: int = 0,
                         drop_last: int = 0):
    """collate (data/collate.py:42-111, RIGHT padding): the last max_seq_length items of each selected session
    (minus `drop_last` trailing items) and the kept lengths"""
    idx = batch_idx.to(torch.int64).contiguous()
    B = idx.numel()
    out = torch.empty(B, max_seq_length, device=idx.device, dtype=torch.int64)
    lengths = torch.empty(B, device=idx.device, dtype=torch.int64)
    call("asme_session_batch", ptr(store.flat), ptr(store.offsets), store.n_sessions, ptr(idx), B, max_seq_length,
         drop_last, pad_token_id, ptr(out), ptr(lengths), stream())
    return out, lengths


class PositiveNegativeSamplerProcessor:
    """data/datasets/processors/pos_neg_sampler.py:29-106 (single-item sessions) + collate, batched on the GPU."""

    def __init__(self, tokenizers, features=None):
        self.tokenizer = _item_tokenizer(tokenizers)
        self.features = features
        specials = sorted(set(int(t) for t in self.tokenizer.get_special_token_ids()))
        if len(specials) > 8:
            raise ValueError("at most 8 special token ids")
        self._specials = specials
        self._special_dev: Dict[torch.device, torch.Tensor] = {}
        self._err_dev: Dict[torch.device, torch.Tensor] = {}

    def process_batch(self, store: SessionStore, batch_idx: torch.Tensor, max_seq_length: int,
                      seed: Optional[int] = None) -> Dict[str, torch.Tensor]:
        dev = store.flat.device
        if dev not in self._special_dev:
            self._special_dev[dev] = torch.tensor(self._specials or [0], dtype=torch.int64, device=dev)
        idx = batch_idx.to(device=dev, dtype=torch.int64).contiguous()
        B, L = idx.numel(), max_seq_length
        x = torch.empty(B, L, device=dev, dtype=torch.int64)
        pos = torch.empty_like(x)
        neg = torch.empty_like(x)
        lengths = torch.empty(B, device=dev, dtype=torch.int64)
        # error bits are sticky (a set bit is an error check_errors raises on): one zeroed flag per device, no
        # zero-fill launch per batch
        err = self._err_dev.get(dev)
        if err is None:
            err = self._err_dev[dev] = torch.zeros(1, device=dev, dtype=torch.int32)
        seed = new_seed(1.0) if seed is None else int(seed)
        call("asme_posneg_sample", ptr(store.flat), ptr(store.offsets), store.n_sessions, ptr(idx), B, L,
             len(self.tokenizer), ptr(self._special_dev[dev]), len(self._specials), self.tokenizer.pad_token_id,
             seed, ptr(x), ptr(pos), ptr(neg), ptr(lengths), ptr(err), stream())
        self._err = err  # checked lazily (check_errors) so the producer never forces a host sync
        return {ITEM_SEQ_ENTRY_NAME: x, POSITIVE_SAMPLES_ENTRY_NAME: pos, NEGATIVE_SAMPLES_ENTRY_NAME: neg,
                "length": lengths}

    def check_errors(self):
        """raise like the reference would (AssertionError for a 1-item session, multinomial failure when no
        id is admissible); syncs the device"""
        e = int(self._err.item()) if getattr(self, "_err", None) is not None else 0
        if e:
            self._err.zero_()  # reported once (the flag is shared by the batches of this device)
        if e & 2:
            raise AssertionError("a session of length 1 reached the positive/negative sampler")
        if e & 1:
            raise RuntimeError("invalid multinomial distribution (a session covers every admissible id)")


class ClozeMaskProcessor:
    """data/datasets/processors/cloze_mask.py:22-92 (item sequence target), batched on the GPU."""

    def __init__(self, tokenizers, mask_prob: float, only_last_item_mask_prob: float, masking_targets=None):
        if masking_targets not in (None, [ITEM_SEQ_ENTRY_NAME]):
            raise NotImplementedError("masking of attribute sequences is outside the MI355X hot path")
        self.tokenizer = _item_tokenizer(tokenizers)
        self.mask_prob = float(mask_prob)
        self.only_last_item_mask_prob = float(only_last_item_mask_prob)

    def process_batch(self, items: torch.Tensor, lengths: torch.Tensor, seed: Optional[int] = None,
                      draws: Optional[tuple] = None) -> Dict[str, torch.Tensor]:
        """items (B, L) collated (right-padded) sessions, lengths (B,).  draws = (u (B, L+1) float32, r (B, L)
        int64) replays given random draws instead of Philox(seed)."""
        items = items.to(torch.int64).contiguous()
        B, L = items.shape
        lengths = lengths.to(device=items.device, dtype=torch.int64).contiguous()
        out = torch.empty_like(items)
        target = torch.empty_like(items)
        du = dr = None
        if draws is not None:
            du = draws[0].to(device=items.device, dtype=torch.float32).contiguous()
            dr = draws[1].to(device=items.device, dtype=torch.int64).contiguous()
            if du.shape != (B, L + 1) or dr.shape != (B, L):
                raise ValueError("draws must be (B, L + 1) uniforms and (B, L) random ids")
        seed = new_seed(1.0) if seed is None else int(seed)
        call("asme_cloze_mask", ptr(items), ptr(lengths), B, L, len(self.tokenizer), self.tokenizer.pad_token_id,
             self.tokenizer.mask_token_id, self.mask_prob, self.only_last_item_mask_prob, ptr(du), ptr(dr), seed,
             ptr(out), ptr(target), stream())
        return {ITEM_SEQ_ENTRY_NAME: out, TARGET_ENTRY_NAME: target}


class LastItemMaskProcessor:
    """data/datasets/processors/last_item_mask.py:9-44 (item sequence target) + the collate, batched on the GPU:
    the MASK token appended after each session's last item (BERT4Rec evaluation input), left-truncated to
    max_seq_length, right-padded."""

    def __init__(self, tokenizers, masking_targets=None):
        if masking_targets not in (None, [ITEM_SEQ_ENTRY_NAME]):
            raise NotImplementedError("masking of attribute sequences is outside the MI355X hot path")
        self.tokenizer = _item_tokenizer(tokenizers)

    def process_batch(self, items: torch.Tensor, lengths: torch.Tensor, max_seq_length: Optional[int] = None
                      ) -> Tuple[torch.Tensor, torch.Tensor]:
        """items (B, L) collated (right-padded) sessions, lengths (B,) -> (items (B, max_seq_length), lengths)"""
        items = items.to(torch.int64).contiguous()
        B, L = items.shape
        Lo = L if max_seq_length is None else int(max_seq_length)
        lengths = lengths.to(device=items.device, dtype=torch.int64).contiguous()
        out = torch.empty(B, Lo, device=items.device, dtype=torch.int64)
        out_len = torch.empty(B, device=items.device, dtype=torch.int64)
        call("asme_last_item_mask", ptr(items), ptr(lengths), B, L, Lo, self.tokenizer.mask_token_id,
             self.tokenizer.pad_token_id, ptr(out), ptr(out_len), stream())
        return out, out_len
