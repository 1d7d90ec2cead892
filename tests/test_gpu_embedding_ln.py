"""The embedding kernel with the first transformer block's input LayerNorm fused (asme_embedding_ln_fwd / _bwd,
ops.embedding(..., ln3=norm)) against the unfused composition it replaces -- asme_embedding_fwd followed by
ops.layer_norm_pass -- and against a PyTorch fp32 reference of the whole chain (transformer_layers.py:55-80, 251-258;
kebert4rec/components.py:54-63).  Same seeds, so the dropout decisions are the same in both kernels."""
import pytest
import torch

pytestmark = pytest.mark.gpu

CASES = {  # name: (pos, ln1, extra, ln2, p1, p2)
    "bert4rec": (True, True, False, False, 0.2, 0.0),
    "sasrec": (True, True, False, True, 0.2, 0.2),
    "kebert4rec_pre": (True, True, True, True, 0.1, 0.3),
    "no_ln1": (True, False, False, False, 0.0, 0.0),
}


def _ref(ids, table, pos, ln1, extra, ln2, ln3, L):
    """fp32 reference with p = 0"""
    F = torch.nn.functional
    x = table[ids]
    if pos is not None:
        x = x + pos[torch.arange(ids.shape[1], device=ids.device) % L]
    if ln1 is not None:
        x = F.layer_norm(x, (x.shape[-1],), ln1[0], ln1[1], 1e-5)
    if extra is not None:
        x = x + extra
    if ln2 is not None:
        x = F.layer_norm(x, (x.shape[-1],), ln2[0], ln2[1], 1e-5)
    return x, F.layer_norm(x, (x.shape[-1],), ln3.weight, ln3.bias, ln3.eps)


@pytest.mark.parametrize("D", [32, 128])
@pytest.mark.parametrize("case", list(CASES))
def test_embedding_ln_fused_equals_unfused(asme, dev, case, D):
    has_pos, has_ln1, has_extra, has_ln2, p1, p2 = CASES[case]
    torch.manual_seed(3)
    B, L, V = 6, 37, 501
    ids = torch.randint(0, V, (B, L), device=dev)
    ids[0, :5] = 0  # padding rows
    leaf = lambda *s, scale=1.0: (torch.randn(*s, device=dev) * scale).requires_grad_(True)  # noqa: E731
    table = leaf(V, D)
    pos = leaf(L, D) if has_pos else None
    ln1 = (leaf(D, scale=0.3) + 1.0, leaf(D, scale=0.1)) if has_ln1 else None
    ln1 = tuple(t.detach().requires_grad_(True) for t in ln1) if ln1 else None
    ln2 = tuple(t.detach().requires_grad_(True) for t in (leaf(D, scale=0.3) + 1.0, leaf(D, scale=0.1))) \
        if has_ln2 else None
    extra = leaf(B, L, D) if has_extra else None
    ln3 = torch.nn.LayerNorm(D).to(dev)
    with torch.no_grad():
        ln3.weight.add_(torch.randn(D, device=dev) * 0.3)
        ln3.bias.add_(torch.randn(D, device=dev) * 0.1)
    gx, gl = torch.randn(B, L, D, device=dev), torch.randn(B, L, D, device=dev)
    leaves = [t for t in (table, pos, *(ln1 or ()), extra, *(ln2 or ()), ln3.weight, ln3.bias) if t is not None]

    def run(fused: bool):
        spec = asme.ops.EmbeddingSpec(seq_len=L, p1=p1, p2=p2)
        torch.manual_seed(11)  # same dropout seeds for both forms
        if fused:
            x, ln = asme.ops.embedding(ids, table, pos, ln1, extra, ln2, spec, ln3=ln3)
        else:
            x = asme.ops.embedding(ids, table, pos, ln1, extra, ln2, spec)
            x, ln = asme.ops.layer_norm_pass(x, ln3)
        grads = torch.autograd.grad((x * gx).sum() + (ln * gl).sum(), leaves)
        return x.detach(), ln.detach(), grads

    xf, lf, gf = run(True)
    xu, lu, gu = run(False)
    # (the two kernel instantiations may contract the affine steps differently: ulp-level differences)
    torch.testing.assert_close(xf, xu, rtol=2e-6, atol=1e-6)
    torch.testing.assert_close(lf, lu, rtol=1e-5, atol=1e-5)
    for a, b in zip(gf, gu):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-4 * float(b.abs().max()) + 1e-6)
    if p1 == 0.0 and p2 == 0.0:
        xr, lr = _ref(ids, table, pos, ln1, extra, ln2, ln3, L)
        torch.testing.assert_close(xf, xr.detach(), rtol=1e-4, atol=1e-5)
        torch.testing.assert_close(lf, lr.detach(), rtol=1e-4, atol=1e-4)
        gr = torch.autograd.grad((xr * gx).sum() + (lr * gl).sum(), leaves)
        for a, b in zip(gf, gr):
            torch.testing.assert_close(a, b, rtol=1e-3, atol=1e-3 * float(b.abs().max()) + 1e-6)


def test_models_take_the_fused_embedding_ln(asme, dev):
    """SASRec / BERT4Rec route block 0's input LayerNorm through the embedding kernel (no separate LayerNorm launch in
    the forward); UBERT4Rec (user token concatenated after the embedding) keeps the unfused path"""
    calls = []
    orig = asme.ops.call

    def spy(name, *a):
        calls.append(name)
        return orig(name, *a)

    m = asme.SASRecModel(transformer_hidden_size=32, num_transformer_heads=2, num_transformer_layers=2,
                         item_vocab_size=100, max_seq_length=12, transformer_dropout=0.1).to(dev)
    seq = torch.randint(1, 100, (3, 12), device=dev)
    asme.ops.call = spy
    try:
        rep = m.encode(asme.InputSequence(seq, seq.ne(0)))
    finally:
        asme.ops.call = orig
    assert "asme_embedding_ln_fwd" in calls and "asme_layernorm_fwd" not in calls
    rep.sum().backward()
    assert m._sequence_embedding_layer.item_embedding_layer.embedding_norm.weight.grad is not None
    blk0 = m._sequence_representation_layer.transformer_layer.transformer_blocks[0]
    assert blk0.input_sublayer.norm.weight.grad is not None
    assert "_asme_next_norm" not in dict(m.named_modules()) and not any(
        "_asme_next_norm" in k for k in m.state_dict())


@pytest.mark.parametrize("mode", ["hook", "flag_off"])
def test_block0_norm_fallbacks_match_the_fused_path(asme, dev, mode):
    """A forward hook on block 0's input norm runs (the norm becomes a module call on the LayerNorm kernel), and
    fuse_embedding_norm = False drops the hand-off; both give the fused path's output and gradients"""
    torch.manual_seed(3)
    res = []
    for variant in ("fused", mode):
        torch.manual_seed(0)
        m = asme.SASRecModel(transformer_hidden_size=32, num_transformer_heads=2, num_transformer_layers=2,
                             item_vocab_size=100, max_seq_length=12, transformer_dropout=0.0).to(dev)
        norm = m._sequence_representation_layer.transformer_layer.transformer_blocks[0].input_sublayer.norm
        fired = []
        if variant == "hook":
            norm.register_forward_hook(lambda mod, inp, out: fired.append(out.shape))
        elif variant == "flag_off":
            m.fuse_embedding_norm = False
        seq = torch.randint(1, 100, (3, 12), generator=torch.Generator().manual_seed(1)).to(dev)
        rep = m.encode(asme.InputSequence(seq, seq.ne(0)))
        rep.square().sum().backward()
        assert len(fired) == (1 if variant == "hook" else 0)
        res.append((rep.detach(), {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None}))
    torch.testing.assert_close(res[1][0], res[0][0], rtol=1e-5, atol=1e-5)
    assert set(res[0][1]) == set(res[1][1])
    for n, g in res[0][1].items():
        torch.testing.assert_close(res[1][1][n], g, rtol=1e-4, atol=1e-4 * float(g.abs().max()) + 1e-7)


@pytest.mark.parametrize("B,L,D", [(1024, 200, 128), (37, 13, 32), (5, 7, 6)])
def test_position_grad_equals_batch_sum(asme, dev, B, L, D):
    """asme_position_grad (the position embedding's gradient: the token rows summed over the batch per position) vs
    torch's sum in fp64 (32 batch chunks, then the column sums)"""
    torch.manual_seed(5)
    rows = torch.randn(B * L, D, device=dev)
    nch = max(1, min(32, B))
    ws = torch.empty(nch, L, D, device=dev)
    out = torch.empty(L, D, device=dev)
    asme._lib.call("asme_position_grad", rows.data_ptr(), B, L, D, ws.data_ptr(), nch, out.data_ptr(), 0,
                   asme._lib.stream())
    want = rows.double().view(B, L, D).sum(0)
    torch.testing.assert_close(out.double(), want, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("rows,width", [(1024, 256), (2048, 768), (1024, 1024), (300, 256), (32, 25600), (1, 5)])
def test_reduce_rows_column_sums(asme, dev, rows, width):
    """asme_reduce_rows (fixed-order column sums of the per-block partials; narrow matrices on the 16-column kernel)
    vs fp64, plain and accumulating"""
    torch.manual_seed(9)
    part = torch.randn(rows, width, device=dev)
    out = torch.randn(width, device=dev)
    base = out.clone()
    asme._lib.call("asme_reduce_rows", part.data_ptr(), rows, width, out.data_ptr(), 1, asme._lib.stream())
    want = part.double().sum(0) + base.double()
    torch.testing.assert_close(out.double(), want, rtol=1e-5, atol=1e-4)
    asme._lib.call("asme_reduce_rows", part.data_ptr(), rows, width, out.data_ptr(), 0, asme._lib.stream())
    torch.testing.assert_close(out.double(), part.double().sum(0), rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("which", ["blk0_output", "blk1_input", "blk1_output"])
def test_hooks_on_every_block_norm_run(asme, dev, which):
    """A forward hook on any block's input / output norm runs (that norm becomes a module call after the residual
    kernel) and the outputs and gradients equal the fused path's; a hook that rescales the norm's output changes
    the result exactly as in nn.LayerNorm semantics"""
    res = []
    for variant in ("fused", "hook", "scale"):
        torch.manual_seed(0)
        m = asme.SASRecModel(transformer_hidden_size=32, num_transformer_heads=2, num_transformer_layers=2,
                             item_vocab_size=100, max_seq_length=12, transformer_dropout=0.0).to(dev)
        blocks = m._sequence_representation_layer.transformer_layer.transformer_blocks
        norm = {"blk0_output": blocks[0].output_sublayer.norm, "blk1_input": blocks[1].input_sublayer.norm,
                "blk1_output": blocks[1].output_sublayer.norm}[which]
        fired = []
        if variant == "hook":
            norm.register_forward_hook(lambda mod, inp, out: fired.append(out.shape))
        elif variant == "scale":
            norm.register_forward_hook(lambda mod, inp, out: out * 2.0)
        seq = torch.randint(1, 100, (3, 12), generator=torch.Generator().manual_seed(1)).to(dev)
        rep = m.encode(asme.InputSequence(seq, seq.ne(0)))
        rep.square().sum().backward()
        assert len(fired) == (1 if variant == "hook" else 0)
        res.append((rep.detach(), {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None}))
    torch.testing.assert_close(res[1][0], res[0][0], rtol=1e-5, atol=1e-5)
    # (the key projection's bias has an analytically zero gradient: rounding noise, held to the global scale)
    gmax = max(float(g.abs().max()) for g in res[0][1].values())
    for n, g in res[0][1].items():
        torch.testing.assert_close(res[1][1][n], g, rtol=1e-4, atol=1e-4 * max(float(g.abs().max()), 1e-2 * gmax))
    assert not torch.allclose(res[2][0], res[0][0])  # the hook's returned output was used
