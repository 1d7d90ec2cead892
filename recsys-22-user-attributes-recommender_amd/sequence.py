"""Batch containers of the model contract (mirror of core/models/common/layers/data/sequence.py:8-113).

Models accept any object exposing `.sequence`, `.padding_mask` and `.attributes`, so ASME's own
InputSequence instances work unchanged when the models are plugged into an ASME run."""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

import torch


@dataclass
class InputSequence:
    sequence: torch.Tensor                       # (N, S) int64 item ids
    padding_mask: Optional[torch.Tensor]         # (N, S) bool, True = real item
    attributes: Dict[str, Any] = field(default_factory=dict)

    def get_attributes(self) -> List[str]:
        return list(self.attributes.keys())

    def has_attribute(self, name: str) -> bool:
        return name in self.attributes

    def get_attribute(self, name: str) -> Optional[Any]:
        return self.attributes.get(name)

    def set_attribute(self, name: str, value: Any, overwrite: bool = False):
        if name in self.attributes and not overwrite:
            raise Exception(f"attribute {name} already set")
        self.attributes[name] = value


def get_attribute(seq, name: str):
    attrs = getattr(seq, "attributes", None) or {}
    return attrs.get(name)
