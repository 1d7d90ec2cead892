"""ASME's on-disk dataset format -> sessions in HBM.

Reads what ASME's preprocessing writes (so an ml-1m / ml-20m / steam split produced by the reference can be
trained and evaluated here):
  <name>.csv                      tab-separated rows, one per interaction, grouped by session, header first
  <name>.session.idx              uint64 (start, end) byte ranges of each session in the csv + trailing count
                                  (data/base/csv_index_builder.py:139-156; read by data/base/reader.py:18-73)
  <name>.<split>.loo.idx / .nextitem.idx
                                  uint64 (session, target_pos) pairs + trailing count (data/datasets/index.py:9-59,
                                  data/datasets/index_builder.py:24-44)
  <name>.vocabulary.<col>.txt     `token\\tid` lines (core/tokenization/vocabulary.py:72-90)
Parsing is host work done once per split (csv module on each session's byte range, like ItemSessionParser,
data/datasets/sequence.py:93-133); the tokenized sessions go to the GPU as a `batches.SessionStore`, and position
indices become (session, pos) pairs for `position_batch` (asme_position_batch: SequencePositionDataset's
truncation + the target extractor in one kernel).
"""
from __future__ import annotations

import csv
import io
import sys
from pathlib import Path
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from ._lib import call, ptr, stream
from .batches import SessionStore


def read_vocabulary(path) -> Dict[str, int]:
    """`token\\tid` per line (CSVVocabularyReaderWriter.read)"""
    vocab: Dict[str, int] = {}
    with open(path, encoding="utf-8") as f:
        for line in f:
            line = line.rstrip("\n")
            if not line:
                continue
            token, idx = line.rsplit("\t", 1)
            vocab[token] = int(idx)
    return vocab


def _read_uint64_pairs(path) -> np.ndarray:
    raw = np.fromfile(path, dtype=np.dtype("uint64").newbyteorder("=" if sys.byteorder == "little" else ">"))
    if raw.size == 0:
        raise ValueError(f"empty index file {path}")
    n = int(raw[-1])
    if raw.size != 2 * n + 1:
        raise ValueError(f"{path}: {raw.size - 1} entries for {n} pairs")
    return raw[:-1].reshape(n, 2).astype(np.int64)


def read_session_index(path) -> np.ndarray:
    """(n, 2) int64 byte ranges [start, end) of each session in the csv (CsvDatasetIndex)"""
    return _read_uint64_pairs(path)


def read_position_index(path) -> np.ndarray:
    """(n, 2) int64 (session, target_pos) pairs (SequencePositionIndex)"""
    return _read_uint64_pairs(path)


def read_sessions(csv_path, session_index_path, vocabulary, item_column: str = "item_id", delimiter: str = "\t",
                  unk_token: str = "<UNK>") -> List[List[int]]:
    """every session of the csv, its `item_column` tokenized with `vocabulary` (a path or a token->id dict;
    unknown tokens map to the unk id, as Tokenizer.convert_tokens_to_ids does)"""
    vocab = read_vocabulary(vocabulary) if not isinstance(vocabulary, dict) else vocabulary
    unk = vocab.get(unk_token)
    data = Path(csv_path).read_bytes()
    header = next(csv.reader(io.StringIO(data[:data.index(b"\n")].decode("utf-8")), delimiter=delimiter))
    col = header.index(item_column)
    out = []
    for start, end in read_session_index(session_index_path):
        rows = csv.reader(io.StringIO(data[start:end].decode("utf-8")), delimiter=delimiter)
        out.append([vocab.get(r[col], unk) for r in rows if r])
    return out


def load_session_store(csv_path, session_index_path, vocabulary, device, item_column: str = "item_id",
                       delimiter: str = "\t") -> SessionStore:
    """the tokenized sessions of an ASME split as a SessionStore on `device`"""
    return SessionStore.from_lists(read_sessions(csv_path, session_index_path, vocabulary, item_column, delimiter),
                                   device)


def position_batch(store: SessionStore, pairs: torch.Tensor, max_seq_length: int, pad_token_id: int = 0
                   ) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """(items (B, L), lengths (B,), targets (B,)) for (session, target_pos) pairs: the last max_seq_length items
    before pos, right-padded, and the item at pos (SequencePositionDataset + TargetExtractorProcessor)"""
    pr = pairs.to(device=store.flat.device, dtype=torch.int64).contiguous()
    B = pr.shape[0]
    dev = store.flat.device
    out = torch.empty(B, max_seq_length, device=dev, dtype=torch.int64)
    lengths = torch.empty(B, device=dev, dtype=torch.int64)
    target = torch.empty(B, device=dev, dtype=torch.int64)
    err = torch.zeros(1, device=dev, dtype=torch.int32)
    call("asme_position_batch", ptr(store.flat), ptr(store.offsets), store.n_sessions, ptr(pr), B, max_seq_length,
         pad_token_id, ptr(out), ptr(lengths), ptr(target), ptr(err), stream())
    position_batch.last_error = err
    return out, lengths, target


position_batch.last_error: Optional[torch.Tensor] = None
