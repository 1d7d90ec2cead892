"""Drop-in check against ASME itself (build container only; needs the read-only /root/reference).

Runs `registry.register()` inside an importable ASME (the _ref_stubs harness), then builds every registered
key exactly as `asme train cfg.yaml` would: ASME's registry lookup -> ModuleConfig -> GenericModuleFactory
-> GenericModelFactory, from a yaml `module:` section (core/init/factories/modules/modules.py:55-127), with
the item tokenizer injected through ASME's @inject (core/utils/inject.py).  Records, per key, the class
that came out, its module, the constructor parameters the factory introspected and the state_dict keys,
as tests/golden/registry_build.json -- data, checked on CPU by tests/test_boundary.py.

    python tests/golden/make_registry_fixture.py
"""
from __future__ import annotations

import inspect
import json
import os
import sys

import yaml

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
import _ref_stubs as S  # noqa: E402

S.install()
import torch  # noqa: E402

MODULE_YAML = {
    "sasrec-neg": """
type: sasrec-neg
metrics: {full: {metrics: {ndcg: [1, 5, 10], recall: [1, 5, 10]}}}
model: {max_seq_length: 200, num_transformer_heads: 2, num_transformer_layers: 2, transformer_hidden_size: 128,
        transformer_dropout: 0.2}
learning_rate: 0.001
""",
    "bert4rec": """
type: bert4rec
metrics: {full: {metrics: {ndcg: [10]}}}
model: {max_seq_length: 200, num_transformer_heads: 2, num_transformer_layers: 2, transformer_hidden_size: 128,
        transformer_dropout: 0.2, project_layer_type: linear}
num_warmup_steps: 100
""",
    "kebert4rec": """
type: kebert4rec
metrics: {full: {metrics: {ndcg: [10]}}}
model: {max_seq_length: 200, num_transformer_heads: 2, num_transformer_layers: 2, transformer_hidden_size: 128,
        transformer_dropout: 0.2, prefusion_attributes: {genre: {embedding_type: content_embedding}}}
""",
}


def main():
    tok = S.make_tokenizer(1000)
    genre = S.make_tokenizer(20, "Genre")
    ctx = S.set_context({"item": tok, "genre": genre})
    sys.path.insert(0, ROOT)
    import __graft_entry__
    asme_amd = __graft_entry__.load_package()
    import asme.core.modules.config  # noqa: F401  (ASME's own registrations first, as in a real run)
    from asme.core.init.config import Config
    from asme.core.init.factories import BuildContext
    from asme.core.modules.registry import REGISTERED_MODULES

    keys = asme_amd.registry.register()
    out = {"registered": keys, "builds": {}}
    for key, text in MODULE_YAML.items():
        section = yaml.safe_load(text)
        factory = REGISTERED_MODULES[key]  # register_module stores the built factory (core/modules/registry.py:19-22)
        bc = BuildContext(Config({"module": section}), ctx)
        bc.enter_section("module")
        module = factory.build(bc)
        model = module.model
        out["builds"][key] = {
            "module_class": type(module).__mro__[1].__qualname__,
            "module_defined_in": type(module).__mro__[1].__module__,
            "model_class": type(model).__mro__[1].__qualname__,
            "model_defined_in": type(model).__mro__[1].__module__,
            "module_init_params": [p for p in inspect.signature(type(module).__mro__[1].__init__).parameters
                                   if p != "self"],
            "item_vocab_size": int(model.item_table().shape[0]),
            "table_grad": getattr(module, "table_grad", None),
            "state_dict_keys": sorted(model.state_dict().keys()),
        }
        print(key, "->", out["builds"][key]["module_class"], out["builds"][key]["model_class"],
              out["builds"][key]["item_vocab_size"])
    with open(os.path.join(HERE, "registry_build.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    torch.set_num_threads(1)
    main()
