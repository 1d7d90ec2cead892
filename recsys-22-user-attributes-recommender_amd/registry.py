"""Drop-in registration under ASME's module registry (the `imports:` plugin boundary).

ASME loads a plugin listed in a config's `imports:` section (core/init/factories/include/
import_factory.py:33-79) after its default registries; the plugin calls
`register_module(key, ModuleConfig(GenericModuleFactory, ModuleCls, {"model_cls": ...}), overwrite=True)`
(core/modules/registry.py:19-24).  `register()` does exactly that for the six hot-path keys
(core/modules/config.py:27-55), wrapping the classes with ASME's own @inject so `item_vocab_size`,
`item_tokenizer` and `additional_attributes_tokenizer` are injected as for the reference classes.
"""
from __future__ import annotations

from . import losses, models, modules

KEYS = {
    "sasrec-neg": (modules.SequenceNextItemPredictionTrainingModule, models.SASRecModel,
                   {"loss_function": losses.SASRecBinaryCrossEntropyLoss()}),
    "sasrec-cross": (modules.NextItemPredictionTrainingModule, models.SASRecModel,
                     {"loss_function": losses.SASRecFullSequenceCrossEntropyLoss}),
    "bert4rec": (modules.MaskedTrainingModule, models.BERT4RecModel, {}),
    "kebert4rec": (modules.MaskedTrainingModule, models.KeBERT4RecModel, {}),
    "ubert4rec": (modules.UBERTMaskedTrainingModule, models.UBERT4RecModel, {}),
    "narm": (modules.NextItemPredictionTrainingModule, models.NarmModel, {}),
}


def _with_asme_injection(cls, **injects):
    from asme.core.utils.inject import inject  # noqa: WPS433 (only inside an ASME process)
    wrapped = type(cls.__name__, (cls,), {})
    wrapped.__init__ = inject(**injects)(cls.__init__)
    return wrapped


def register(overwrite: bool = True):
    """Register the MI355X modules/models in a running ASME process (requires the `asme` package)."""
    from asme.core.init.factories.modules.modules import GenericModuleFactory
    from asme.core.modules.registry import ModuleConfig, register_module
    from asme.core.utils.inject import InjectTokenizer, InjectTokenizers, InjectVocabularySize

    for key, (module_cls, model_cls, extra) in KEYS.items():
        model_injects = {"item_vocab_size": InjectVocabularySize("item")}
        for name in ("additional_attributes_tokenizer", "additional_tokenizers"):
            if name in model_cls.__init__.__code__.co_varnames:
                model_injects[name] = InjectTokenizers()
        m_cls = _with_asme_injection(module_cls, item_tokenizer=InjectTokenizer("item"))
        md_cls = _with_asme_injection(model_cls, **model_injects)
        register_module(key, ModuleConfig(GenericModuleFactory, m_cls, {"model_cls": md_cls, **extra}),
                        overwrite=overwrite)
    return sorted(KEYS)
