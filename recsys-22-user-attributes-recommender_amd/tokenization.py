"""Minimal item vocabulary/tokenizer: the hot path only needs the special-token ids and len(vocab).

Mirrors the parts of core/tokenization/{tokenizer,vocabulary}.py the models/modules use:
pad_token_id / mask_token_id / unk_token_id, get_special_token_ids(), len(), get_vocabulary().ids().
ASME's own Tokenizer objects can be passed anywhere these are accepted (duck typing)."""
from __future__ import annotations

from typing import List


class Vocabulary:
    def __init__(self, size: int):
        self._size = int(size)

    def ids(self) -> List[int]:
        return list(range(self._size))

    def __len__(self):
        return self._size


class Tokenizer:
    """Synthetic vocabulary: <PAD>=0, <MASK>=1, <UNK>=2 followed by `n_items` item ids (the ASME
    vocabulary convention, data/datamodule/preprocessing/vocabulary.py)."""

    def __init__(self, n_items: int, pad_token_id: int = 0, mask_token_id: int = 1, unk_token_id: int = 2):
        self.pad_token_id = pad_token_id
        self.mask_token_id = mask_token_id
        self.unk_token_id = unk_token_id
        self._vocab = Vocabulary(n_items + 3)

    def get_special_token_ids(self) -> List[int]:
        return [self.pad_token_id, self.mask_token_id, self.unk_token_id]

    def get_vocabulary(self) -> Vocabulary:
        return self._vocab

    def __len__(self):
        return len(self._vocab)
