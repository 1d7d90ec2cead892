"""Host-side plumbing that needs no GPU: which models hand block 0's input LayerNorm to their embedding kernel
(ops.embedding ln3, asme_embedding_ln_fwd), and that the hand-over is invisible to state_dict / module traversal /
deepcopy; the lazy table's start state (rows at rest only for fresh moments without weight decay)."""
import copy
import os

import numpy as np
import pytest
import torch

from helpers import MODEL_FIXTURES, build_model

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _target(m):
    emb = m._sequence_embedding_layer
    return getattr(emb, "item_embedding_layer", emb)


@pytest.mark.parametrize("name", [n for n in MODEL_FIXTURES if n != "narm"])
def test_next_norm_handed_to_the_embedding(asme, name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"))
    m = build_model(asme, name, z)
    norm = _target(m).__dict__.get("_asme_next_norm")
    if name.startswith("ubert4rec"):
        # the user token is concatenated after the embedding: the embedding output is not block 0's input
        assert norm is None
        return
    blocks = m._sequence_representation_layer.transformer_layer.transformer_blocks
    assert norm is blocks[0].input_sublayer.norm
    keys = set(m.state_dict())
    assert not any("_asme_next_norm" in k for k in keys)
    assert len(list(m.parameters())) == len({id(p) for p in m.parameters()})
    assert not any(n.endswith("_asme_next_norm") for n, _ in m.named_modules())
    c = copy.deepcopy(m)  # the copy's embedding points at the copy's own norm
    cb = c._sequence_representation_layer.transformer_layer.transformer_blocks
    assert _target(c).__dict__["_asme_next_norm"] is cb[0].input_sublayer.norm
    assert set(c.state_dict()) == keys


@pytest.mark.parametrize("fresh,wd,rest", [(True, 0.0, True), (True, 1e-3, False), (False, 0.0, False)])
def test_lazy_table_start(asme, fresh, wd, rest):
    p = torch.zeros(7, 4)
    st = asme.ops.LazyTableState(p, torch.zeros_like(p), torch.zeros_like(p))
    st.start(5, fresh, wd)
    assert st.rest is rest and st.step == 5
    assert bool((st.last_step == (asme.ops.REST_STEP if rest else 5)).all())
