"""Fused full-catalogue logits head + CrossEntropyLoss (csrc/logits.hip, ops.linear_cross_entropy) against the
plain PyTorch fp64 CPU computation F.cross_entropy(F.linear(h, W, b), t, ignore_index) (layers.py:105-109,
138-143; losses.py:77-115): loss, dH, dW, db; ignored rows, out-of-range targets, all rows ignored (NaN,
like torch), ragged n / |V| (not multiples of the 64-row tiles), every supported width."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / (b.abs().max() + 1e-30))


@pytest.mark.parametrize("d", [32, 36, 64, 100, 128])
@pytest.mark.parametrize("n,V", [(1, 5), (37, 67), (300, 1000), (2051, 4099), (513, 27003)])
@pytest.mark.parametrize("with_bias", [True, False])
def test_linear_xent_matches_reference(asme, dev, d, n, V, with_bias):
    torch.manual_seed(n + V + d)
    h = torch.randn(n, d) * 0.5
    W = torch.randn(V, d) * 0.5
    b = torch.randn(V) * 0.3 if with_bias else None
    t = torch.randint(0, V, (n,))
    t[::5] = 0  # ignore_index = pad = 0 rows
    hc, Wc = h.double().requires_grad_(True), W.double().requires_grad_(True)
    bc = b.double().requires_grad_(True) if with_bias else None
    ref = F.cross_entropy(F.linear(hc, Wc, bc), t, ignore_index=0)
    ref.backward()
    hd, Wd = h.to(dev).requires_grad_(True), W.to(dev).requires_grad_(True)
    bd = b.to(dev).requires_grad_(True) if with_bias else None
    loss = asme.ops.linear_cross_entropy(hd, Wd, bd, t.to(dev), 0)
    loss.backward()
    if bool((t == 0).all()):
        assert math.isnan(loss.item()) and math.isnan(ref.item())
        return
    assert abs(loss.item() - ref.item()) / abs(ref.item()) < 1e-5
    assert _rel(hd.grad, hc.grad) < 1e-4
    assert _rel(Wd.grad, Wc.grad) < 1e-4
    if with_bias:
        assert _rel(bd.grad, bc.grad) < 1e-4


def test_linear_xent_all_ignored_and_out_of_range(asme, dev):
    torch.manual_seed(0)
    n, V, d = 70, 130, 64
    h, W, b = torch.randn(n, d, device=dev), torch.randn(V, d, device=dev), torch.randn(V, device=dev)
    t = torch.zeros(n, dtype=torch.int64, device=dev)
    hd, Wd = h.clone().requires_grad_(True), W.clone().requires_grad_(True)
    loss = asme.ops.linear_cross_entropy(hd, Wd, b, t, 0)
    assert math.isnan(loss.item())
    # out-of-range targets are skipped like ignored ones (torch would raise; the kernel must not fault)
    t2 = torch.randint(1, V, (n,), device=dev)
    t2[3] = V + 5
    t2[7] = -3
    keep = (t2 >= 0) & (t2 < V)
    loss2 = asme.ops.linear_cross_entropy(h, W, b, t2, 0)
    ref = F.cross_entropy(F.linear(h[keep].double(), W.double(), b.double()), t2[keep])
    assert abs(loss2.item() - ref.item()) / abs(ref.item()) < 1e-5


@pytest.mark.parametrize("d", [32, 64, 128])
@pytest.mark.parametrize("n,V", [(1, 3), (129, 257), (700, 27003)])
def test_logits_exact_on_integer_data(asme, dev, d, n, V):
    """asme_logits on integer-valued operands (every product and sum exact in fp32 and in the split bf16 terms):
    bit-exact against float64, which pins the operand / fragment layouts of the engine"""
    g = torch.Generator().manual_seed(d + n + V)
    h = torch.randint(-4, 5, (n, d), generator=g).float()
    W = torch.randint(-4, 5, (V, d), generator=g).float()
    b = torch.randint(-9, 10, (V,), generator=g).float()
    want = h.double() @ W.double().t() + b.double()
    got = asme.ops.logits(h.to(dev), W.to(dev), b.to(dev))
    assert torch.equal(got.cpu().double(), want)


@pytest.mark.parametrize("d", [64, 128])
def test_logits_random_vs_fp64(asme, dev, d):
    """fp32-level accuracy of the split-bf16 products: error vs float64 within fp32 GEMM rounding"""
    torch.manual_seed(d)
    n, V = 333, 5001
    h, W, b = torch.randn(n, d), torch.randn(V, d), torch.randn(V)
    want = h.double() @ W.double().t() + b.double()
    got = asme.ops.logits(h.to(dev), W.to(dev), b.to(dev)).cpu().double()
    scale = h.double().abs() @ W.double().abs().t() + b.double().abs()
    assert ((got - want).abs() / scale).max().item() < 2e-6


def test_linear_xent_vs_materialised_kernels(asme, dev):
    """fused kernels == library GEMM logits + the CE kernel (the unfused GPU path) at a BERT4Rec-like shape"""
    torch.manual_seed(3)
    n, V, d = 3000, 27003, 128
    h = torch.randn(n, d, device=dev) * 0.3
    W = torch.randn(V, d, device=dev) * 0.3
    b = torch.randn(V, device=dev) * 0.1
    t = torch.randint(0, V, (n,), device=dev)
    p1 = [x.clone().requires_grad_(True) for x in (h, W, b)]
    p2 = [x.clone().requires_grad_(True) for x in (h, W, b)]
    l1 = asme.ops.linear_cross_entropy(p1[0], p1[1], p1[2], t, 0)
    l1.backward()
    l2 = asme.ops.cross_entropy(F.linear(p2[0], p2[1], p2[2]), t, 0)
    l2.backward()
    assert abs(l1.item() - l2.item()) / abs(l2.item()) < 1e-5
    for a, c in zip(p1, p2):
        assert _rel(a.grad, c.grad) < 1e-4


@pytest.mark.parametrize("h_grad", [True, False])
def test_linear_xent_training_and_weight_only_paths(asme, dev, h_grad):
    """hidden requiring grad takes the training form (dH folded into the forward, asme_linear_xent_fwd_dh +
    asme_linear_xent_bwd_dw); a frozen hidden takes the two-pass backward (asme_linear_xent_bwd): both match fp64,
    with a dloss other than 1 (the upstream scale is applied in the backward)"""
    torch.manual_seed(5)
    n, V, d = 1500, 9001, 128
    h, W, b = torch.randn(n, d) * 0.4, torch.randn(V, d) * 0.4, torch.randn(V) * 0.2
    t = torch.randint(0, V, (n,))
    t[::7] = 0
    hc, Wc, bc = h.double().requires_grad_(h_grad), W.double().requires_grad_(True), b.double().requires_grad_(True)
    (3.5 * F.cross_entropy(F.linear(hc, Wc, bc), t, ignore_index=0)).backward()
    hd, Wd, bd = h.to(dev).requires_grad_(h_grad), W.to(dev).requires_grad_(True), b.to(dev).requires_grad_(True)
    (3.5 * asme.ops.linear_cross_entropy(hd, Wd, bd, t.to(dev), 0)).backward()
    if h_grad:
        assert _rel(hd.grad, hc.grad) < 1e-4
    else:
        assert hd.grad is None
    assert _rel(Wd.grad, Wc.grad) < 1e-4
    assert _rel(bd.grad, bc.grad) < 1e-4


@pytest.mark.parametrize("order", ["rising", "falling", "wide"])
def test_linear_xent_running_max_moves(asme, dev, order):
    """the training form's online softmax (running max per query over the item tiles, the accumulators rescaled
    only when a tile's max exceeds the reference by more than e^8): item biases rising along the catalogue move the
    maximum at nearly every tile, falling ones never after the first, wide-range logits (|s| up to ~60) mix both --
    loss, dH, dW, db against fp64"""
    torch.manual_seed(11)
    n, V, d = 600, 5003, 128
    h, W = torch.randn(n, d) * 0.4, torch.randn(V, d) * 0.4
    if order == "rising":
        b = torch.linspace(-40.0, 40.0, V)
    elif order == "falling":
        b = torch.linspace(40.0, -40.0, V)
    else:
        h, b = h * 6.0, torch.randn(V) * 8.0
    t = torch.randint(0, V, (n,))
    t[::9] = 0
    hc, Wc, bc = (x.double().requires_grad_(True) for x in (h, W, b))
    ref = F.cross_entropy(F.linear(hc, Wc, bc), t, ignore_index=0)
    ref.backward()
    hd, Wd, bd = (x.to(dev).requires_grad_(True) for x in (h, W, b))
    loss = asme.ops.linear_cross_entropy(hd, Wd, bd, t.to(dev), 0)
    loss.backward()
    assert abs(loss.item() - ref.item()) / abs(ref.item()) < 1e-5
    assert _rel(hd.grad, hc.grad) < 1e-4
    assert _rel(Wd.grad, Wc.grad) < 1e-4
    assert _rel(bd.grad, bc.grad) < 1e-4
