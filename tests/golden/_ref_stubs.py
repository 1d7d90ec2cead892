"""Import harness for the READ-ONLY reference (golden-vector generation only).

Runs only in the build container (never on the GPU box, never shipped as product):
the reference needs pytorch_lightning / torchmetrics / loguru / dataclasses_json /
flatten_dict, none of which are installed, so we register permissive stand-in
modules in ``sys.modules`` before importing ``asme``.  This follows SURVEY.md
Appendix A.  Nothing here is reference source; it only makes the reference's own
files importable so we can record their outputs as fixtures.
"""
from __future__ import annotations

import importlib.abc
import importlib.machinery
import random
import sys
import types

REF_SRC = "/root/reference/src"


class _Dummy:
    def __init__(self, *a, **k):
        pass

    def __call__(self, *a, **k):
        return self

    def __getattr__(self, item):
        return _Dummy()


def _seed_everything(seed: int):
    import numpy as np
    import torch
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    return seed


class _AutoModule(types.ModuleType):
    def __getattr__(self, item):
        if item.startswith("__"):
            raise AttributeError(item)
        return type(item, (_Dummy,), {})


class _AutoFinder(importlib.abc.MetaPathFinder, importlib.abc.Loader):
    roots = ("pytorch_lightning", "aim", "mlflow", "wandb", "optuna", "redis", "_jsonnet")

    def find_spec(self, fullname, path, target=None):
        if fullname.split(".")[0] in self.roots:
            return importlib.machinery.ModuleSpec(fullname, self, is_package=True)
        return None

    def create_module(self, spec):
        m = _AutoModule(spec.name)
        m.__path__ = []
        return m

    def exec_module(self, module):
        if module.__name__ == "pytorch_lightning":
            import torch.nn as nn

            class LightningModule(nn.Module):
                def save_hyperparameters(self, *a, **k):
                    pass

                def log(self, *a, **k):
                    pass

                @property
                def device(self):  # LightningModule.device (ubert_masked_training_module.py:72)
                    import torch
                    p = next(self.parameters(), None)
                    return p.device if p is not None else torch.device("cpu")

            module.LightningModule = LightningModule
            core = types.ModuleType("pytorch_lightning.core")  # `from pytorch_lightning import core as pl`
            core.LightningModule = LightningModule
            module.core = core
            sys.modules["pytorch_lightning.core"] = core
            module.seed_everything = _seed_everything
            module.Trainer = _Dummy
            module.Callback = type("Callback", (), {})


def install():
    if getattr(install, "_done", False):
        return
    import torch
    import torch.nn as nn

    sys.meta_path.insert(0, _AutoFinder())

    # torchmetrics: Metric as nn.Module with add_state/reset; reduce()
    tm = types.ModuleType("torchmetrics")
    tm_metric = types.ModuleType("torchmetrics.metric")
    tm_util = types.ModuleType("torchmetrics.utilities")

    class Metric(nn.Module):
        def __init__(self, *a, **k):
            super().__init__()
            self._defaults = {}

        def add_state(self, name, default, dist_reduce_fx=None, persistent=False):
            self._defaults[name] = default
            setattr(self, name, default.clone() if isinstance(default, torch.Tensor) else list(default))

        def reset(self):
            for n, d in self._defaults.items():
                setattr(self, n, d.clone() if isinstance(d, torch.Tensor) else list(d))

        def forward(self, *a, **k):
            return self.update(*a, **k)

    def reduce(x, reduction):
        if reduction == "elementwise_mean":
            return torch.mean(x)
        if reduction == "sum":
            return torch.sum(x)
        return x

    tm_metric.Metric = Metric
    tm.Metric = Metric
    tm.metric = tm_metric
    tm_util.reduce = reduce
    tm.utilities = tm_util
    sys.modules.update({"torchmetrics": tm, "torchmetrics.metric": tm_metric,
                        "torchmetrics.utilities": tm_util})

    lg = types.ModuleType("loguru")
    lg.logger = _Dummy()
    sys.modules["loguru"] = lg

    dj = types.ModuleType("dataclasses_json")
    dj.dataclass_json = lambda cls=None, **k: (cls if cls is not None else (lambda c: c))
    sys.modules["dataclasses_json"] = dj

    fd = types.ModuleType("flatten_dict")
    fd.flatten = lambda d, *a, **k: d
    fd.unflatten = lambda d, *a, **k: d
    fdr = types.ModuleType("flatten_dict.reducers")
    fdr.make_reducer = lambda *a, **k: None
    fds = types.ModuleType("flatten_dict.splitters")
    fds.make_splitter = lambda *a, **k: None
    fd.reducers, fd.splitters = fdr, fds
    sys.modules.update({"flatten_dict": fd, "flatten_dict.reducers": fdr,
                        "flatten_dict.splitters": fds})

    if REF_SRC not in sys.path:
        sys.path.insert(0, REF_SRC)
    install._done = True


def make_tokenizer(n_items: int, prefix: str = "Item"):
    """Reference Tokenizer over a synthetic vocabulary: <PAD>=0, <MASK>=1, <UNK>=2, items 3..."""
    from asme.core.tokenization.tokenizer import Tokenizer
    from asme.core.tokenization.vocabulary import Vocabulary
    from collections import OrderedDict
    tok2id = OrderedDict()
    for i, t in enumerate(["<PAD>", "<MASK>", "<UNK>"] + [f"{prefix} {j}" for j in range(n_items)]):
        tok2id[t] = i
    vocab = Vocabulary(tok2id)
    return Tokenizer(vocab, pad_token="<PAD>", mask_token="<MASK>", unk_token="<UNK>")


def set_context(tokenizers: dict):
    """Set the global injection context BEFORE the first model import."""
    install()
    import asme.core.init.factories as fac
    from asme.core.init.config import Config
    from asme.core.init.context import Context
    from asme.core.init.factories import BuildContext
    ctx = Context()
    for k, v in tokenizers.items():
        ctx.set(f"tokenizers.{k}", v)
    fac.GLOBAL_ASME_INJECTION_CONTEXT = BuildContext(Config({}), ctx)
    # inject.py binds the context by value at import time: refresh it if already imported
    if "asme.core.utils.inject" in sys.modules:
        sys.modules["asme.core.utils.inject"].GLOBAL_ASME_INJECTION_CONTEXT = fac.GLOBAL_ASME_INJECTION_CONTEXT
    return ctx
