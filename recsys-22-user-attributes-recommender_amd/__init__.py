"""ASME on MI355X: the sequential-recommender training/eval hot path on hand-written gfx950 kernels.

Import name: `asme_amd` (the directory name is not a Python identifier; `__graft_entry__.load_package()`
registers it).  Public surface mirrors the reference (LSX-UniWue/recsys-22-user-attributes-recommender):
models (SASRecModel, BERT4RecModel, KeBERT4RecModel, UBERT4RecModel, NarmModel), training modules, losses, metrics,
and `registry.register()` for ASME's `imports:` plugin mechanism.
"""
from . import _lib, batches, dataparallel, datasets, layers, losses, metrics, models, modules, ops, optim, registry, sequence, sharded, tokenization  # noqa
from .models import BERT4RecModel, KeBERT4RecModel, NarmModel, SASRecModel, UBERT4RecModel  # noqa
from .modules import (MaskedTrainingModule, NextItemPredictionTrainingModule,  # noqa
                      SequenceNextItemPredictionTrainingModule, UBERTMaskedTrainingModule)
from .optim import FusedAdam  # noqa
from .sequence import InputSequence  # noqa

__version__ = "0.1.0"
