"""NARM's encoders on the hand kernels (csrc/narm.hip, ops.gru / ops.narm_attend / ops.dropout_rows) against
plain PyTorch fp64 on the CPU: nn.GRU itself (core/models/narm/components.py:32-56 builds one) for the recurrence,
the LocalEncoderLayer expression (core/models/narm/layers.py:32-66) for the attention, and the oracle's NARM
restatement (oracle/asme_oracle.py narm_scores, pinned to the reference's narm fixture by
tests/test_oracle_golden.py) for a full training step at the ml-1m configuration's widths
(configs-new/narm/ml-1m.yaml: E = 64, H = 128, batch 128, L = 200).  fp32 tolerances are stated per check."""
import math

import pytest
import torch
import torch.nn.functional as F

from oracle import asme_oracle as O

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / (b.abs().max() + 1e-30))


@pytest.mark.parametrize("E,H,layers", [(16, 24, 1), (64, 128, 1), (180, 30, 1), (32, 64, 2), (20, 16, 3),
                                        (64, 100, 2)])
@pytest.mark.parametrize("B,L", [(1, 1), (5, 9), (37, 50)])
def test_gru_matches_torch(asme, dev, E, H, layers, B, L):
    """outputs of every step and every gradient (input, all weights and biases) of a stacked batch_first GRU;
    fp32 kernels vs fp64: rel 2e-5 on outputs, 1e-4 on gradients (50-step recurrences)"""
    torch.manual_seed(E * 1000 + H * 10 + layers + B + L)
    ref = torch.nn.GRU(E, H, num_layers=layers, batch_first=True).double()
    x = torch.randn(B, L, E, dtype=torch.float64)
    dy = torch.randn(B, L, H, dtype=torch.float64)
    xr = x.clone().requires_grad_(True)
    yr, _ = ref(xr)
    (yr * dy).sum().backward()

    mod = torch.nn.GRU(E, H, num_layers=layers, batch_first=True)
    mod.load_state_dict({k: v.float() for k, v in ref.state_dict().items()})
    mod.to(dev)
    xd = x.float().to(dev).requires_grad_(True)
    yd = asme.ops.gru(xd, mod)
    (yd * dy.float().to(dev)).sum().backward()
    torch.cuda.synchronize()
    assert yd.shape == (B, L, H)
    assert _rel(yd, yr) < 2e-5
    assert _rel(xd.grad, xr.grad) < 1e-4
    rp = dict(ref.named_parameters())
    for k, p in mod.named_parameters():
        assert _rel(p.grad, rp[k].grad) < 1e-4, k


def test_gru_rejects_unsupported(asme, dev):
    for kw in ({"bidirectional": True}, {"batch_first": False}):
        mod = torch.nn.GRU(8, 16, **{"batch_first": True, **kw}).to(dev)
        with pytest.raises(NotImplementedError):
            asme.ops.gru(torch.randn(2, 3, 8, device=dev), mod)
    # wider than the register-resident kernel: the library GRU on the device (the reference's own nn.GRU)
    mod = torch.nn.GRU(8, 144, batch_first=True).to(dev)
    x = torch.randn(2, 3, 8, device=dev)
    assert torch.equal(asme.ops.gru(x, mod), mod(x)[0])
    with pytest.raises(asme._lib.ASMEKernelError):
        asme.ops.gru(x.cpu(), mod.cpu())


@pytest.mark.parametrize("N,S,H", [(1, 1, 8), (7, 9, 24), (33, 200, 128), (4, 300, 130)])
def test_local_encoder_matches_torch(asme, dev, N, S, H):
    """alpha = v . sigmoid(P1 + P2), c_l = sum mask * alpha * h and its gradients wrt P1, P2, v, h: rel 1e-5"""
    torch.manual_seed(N + S + H)
    p1 = torch.randn(N, H, dtype=torch.float64)
    p2 = torch.randn(N, S, H, dtype=torch.float64)
    v = torch.rand(H, dtype=torch.float64) * 2 - 1
    hs = torch.randn(N, S, H, dtype=torch.float64)
    lengths = torch.randint(1, S + 1, (N,))
    mask = torch.arange(S).unsqueeze(0) < lengths.unsqueeze(1)
    dc = torch.randn(N, H, dtype=torch.float64)
    ts = [t.clone().requires_grad_(True) for t in (p1, p2, v, hs)]
    alphas = torch.matmul(torch.sigmoid(ts[0].unsqueeze(1) + ts[1]), ts[2]).unsqueeze(2)
    ref = (mask.unsqueeze(-1).double() * (alphas * ts[3])).sum(1)
    (ref * dc).sum().backward()
    ds = [t.float().to(dev).requires_grad_(True) for t in (p1, p2, v, hs)]
    out = asme.ops.narm_attend(*ds, mask.to(dev))
    (out * dc.float().to(dev)).sum().backward()
    torch.cuda.synchronize()
    assert _rel(out, ref) < 1e-5
    for got, want in zip(ds, ts):
        assert _rel(got.grad, want.grad) < 1e-5


def test_dropout_rows_semantics(asme, dev):
    """Dropout2d on (N, S, E): every (n, s) row kept (scaled by 1/(1-p)) or zeroed as a whole, drop rate ~ p,
    the backward replays the same rows"""
    torch.manual_seed(3)
    p = 0.3
    x = (torch.rand(64, 200, 36, device=dev) + 0.5).requires_grad_(True)
    y = asme.ops.dropout_rows(x, p)
    y.backward(torch.ones_like(y))
    kept = (y != 0)
    rows_all = kept.all(-1)
    rows_none = (~kept).all(-1)
    assert bool((rows_all | rows_none).all())
    assert torch.allclose(y[rows_all], x[rows_all] / (1 - p), rtol=1e-6)
    rate = float(rows_none.float().mean())
    assert abs(rate - p) < 0.02, rate
    assert torch.equal(x.grad != 0, kept)
    assert torch.allclose(x.grad[rows_all], torch.full_like(x.grad[rows_all], 1 / (1 - p)))


def test_decoder_item_matrix_dropout(asme, dev):
    """training: the decoder's (|V|, E) item matrix goes through the embedding dropout element-wise (Dropout2d on
    2-D input, narm/layers.py:113-117), the sequence embedding drops whole positions; eval: the raw table"""
    torch.manual_seed(4)
    model = asme.NarmModel(item_vocab_size=500, item_embedding_size=64, global_encoder_size=32,
                           global_encoder_num_layers=1, embedding_dropout=0.25, context_dropout=0.1).to(dev)
    layer = model._sequence_embedding_layer.elements_embedding
    table = layer.embedding.weight
    model.train()
    m = layer.item_matrix()
    zero = m == 0
    assert 0.2 < float(zero.float().mean()) < 0.3
    assert not bool(zero.all(-1).any())  # element-wise, not whole rows
    assert torch.allclose(m[~zero], table[~zero] / 0.75, rtol=1e-6)
    seq = torch.randint(3, 500, (16, 40), device=dev)
    emb = layer(seq)
    ez = emb == 0
    assert bool((ez.all(-1) | (~ez).all(-1)).all())  # whole positions
    model.eval()
    assert layer.item_matrix() is table


def _narm_sd(asme, dev, B, L, E, H, V, layers, seed):
    torch.manual_seed(seed)
    model = asme.NarmModel(item_vocab_size=V, item_embedding_size=E, global_encoder_size=H,
                           global_encoder_num_layers=layers, embedding_dropout=0.0, context_dropout=0.0)
    g = torch.Generator().manual_seed(seed + 1)
    lengths = torch.randint(1, L + 1, (B,), generator=g)
    lengths[0] = L
    seq = torch.randint(3, V, (B, L), generator=g)
    seq[torch.arange(L).unsqueeze(0) >= lengths.unsqueeze(1)] = 0
    tgt = torch.randint(3, V, (B,), generator=g)
    return model, seq, tgt


@pytest.mark.parametrize("fused_xent", [True, False])
@pytest.mark.parametrize("B,L,E,H,V,layers", [(128, 200, 64, 128, 3706, 1), (40, 30, 48, 32, 1001, 2)])
def test_narm_training_step_vs_oracle(asme, dev, monkeypatch, fused_xent, B, L, E, H, V, layers):
    """one NextItemPredictionTrainingModule step (loss + every gradient) at the ml-1m widths against the oracle's
    NARM restatement differentiated in fp64 (2H = 256 runs the Linear-kernel logits + CE kernel path, 2H = 64 the
    fused bf16x6 head): loss rel 1e-5, gradients rel 2e-4"""
    monkeypatch.setattr(asme.modules, "FUSED_XENT", fused_xent)
    model, seq, tgt = _narm_sd(asme, dev, B, L, E, H, V, layers, seed=B + L + H)
    sd = {k: v.detach().double().clone().requires_grad_(True) for k, v in model.state_dict().items()}
    logits = O.narm_scores(sd, seq)
    ref = F.cross_entropy(logits, tgt)
    ref.backward()

    model.to(dev)
    tok = asme.tokenization.Tokenizer(V - 3)
    module = asme.NextItemPredictionTrainingModule(model=model, item_tokenizer=tok, metrics=None)
    loss = module.training_step({"item": seq.to(dev), "item.target": tgt.to(dev)}, 0)["loss"]
    loss.backward()
    torch.cuda.synchronize()
    assert abs(loss.item() - ref.item()) / abs(ref.item()) < 1e-5, (loss.item(), ref.item())
    for k, p in model.named_parameters():
        assert p.grad is not None, k
        assert _rel(p.grad, sd[k].grad) < 2e-4, (k, _rel(p.grad, sd[k].grad))
    with torch.no_grad():
        module.eval()
        scores = module.predict_step({"item": seq.to(dev)}, 0)
    assert _rel(scores, logits) < 1e-5
    assert not math.isnan(loss.item())
