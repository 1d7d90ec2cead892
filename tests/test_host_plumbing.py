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


def test_fuse_embedding_norm_flag_and_hook_fallback(asme, monkeypatch):
    """fuse_embedding_norm is an explicit model flag: off, the embedding kernel gets no block-0 norm; on, it does --
    except while that norm carries a forward hook (or pre-hook), when the embedding leaves it to block 0, which then
    calls the norm as a module so the hook runs (layers.TransformerLayer.forward).  The embedding kernel call is
    recorded instead of run (no GPU here)."""
    z = np.load(os.path.join(GOLDEN, "sasrec_neg.npz"))
    m = build_model(asme, "sasrec_neg", z)
    norm = m._sequence_representation_layer.transformer_layer.transformer_blocks[0].input_sublayer.norm
    assert isinstance(norm, torch.nn.LayerNorm) and m.fuse_embedding_norm
    seen = []

    def fake_embedding(ids, w, pos, ln1, extra, ln2, spec, ln3=None):
        seen.append(ln3)
        x = torch.zeros(*ids.shape, w.shape[1])
        return (x, x.clone()) if ln3 is not None else x

    monkeypatch.setattr(asme.ops, "embedding", fake_embedding)
    ids = torch.randint(3, int(z["cfg"][5]), (2, 5))
    emb = _target(m)
    x = emb.embed(ids)
    assert seen[-1] is norm and x._asme_ln[0] is norm
    h = norm.register_forward_hook(lambda mod, inp, out: None)
    assert not hasattr(emb.embed(ids), "_asme_ln") and seen[-1] is None  # hooked: not fused
    assert asme.layers.has_forward_hooks(norm)
    h.remove()
    h = norm.register_forward_pre_hook(lambda mod, inp: None)
    emb.embed(ids)
    assert seen[-1] is None
    h.remove()
    m.fuse_embedding_norm = False
    assert not m.fuse_embedding_norm and "_asme_next_norm" not in emb.__dict__
    emb.embed(ids)
    assert seen[-1] is None
    m.fuse_embedding_norm = True
    emb.embed(ids)
    assert seen[-1] is norm
    assert set(m.state_dict()) == set(build_model(asme, "sasrec_neg", z).state_dict())


@pytest.mark.parametrize("fresh,wd,rest", [(True, 0.0, True), (True, 1e-3, False), (False, 0.0, False)])
def test_lazy_table_start(asme, fresh, wd, rest):
    p = torch.zeros(7, 4)
    st = asme.ops.LazyTableState(p, torch.zeros_like(p), torch.zeros_like(p))
    st.start(5, fresh, wd)
    assert st.rest is rest and st.step == 5
    assert bool((st.last_step == (asme.ops.REST_STEP if rest else 5)).all())
