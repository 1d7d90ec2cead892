"""The fused transformer stack (fused.py: GEMM epilogues + hand-written backward) against the per-op
path it replaces (itself checked against the oracle in test_gpu_models.py), same seeds, same dropout
decisions: outputs and every parameter gradient must agree to fp32 rounding."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-12)).item()


def _run(asme, layer, x, valid, causal, fused_on, seed):
    asme.layers.FUSED_STACK = fused_on
    try:
        layer.zero_grad(set_to_none=True)
        xx = x.clone().requires_grad_(True)
        torch.manual_seed(seed)
        y = layer(xx, valid, causal)
        g = torch.randn_like(y, generator=torch.Generator(device=y.device).manual_seed(7))
        (y * g).sum().backward()
        grads = {n: p.grad.clone() for n, p in layer.named_parameters() if p.grad is not None}
        return y.detach(), xx.grad.clone(), grads
    finally:
        asme.layers.FUSED_STACK = False


@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("dropout", [0.0, 0.2])
@pytest.mark.parametrize("n_layers", [1, 2, 3])
def test_fused_stack_matches_per_op_path(asme, dev, causal, dropout, n_layers):
    torch.manual_seed(n_layers * 10 + int(causal))
    B, L, D, H, Fd = 3, 57, 128, 2, 512
    layer = asme.layers.TransformerLayer(D, H, n_layers, Fd, dropout).to(dev).train()
    with torch.no_grad():  # non-trivial LayerNorm parameters
        for n, p in layer.named_parameters():
            if "norm" in n:
                p.add_(0.1 * torch.randn_like(p))
    x = torch.randn(B, L, D, device=dev)
    lengths = torch.tensor([L, 31, 1])
    valid = (torch.arange(L).unsqueeze(0) < lengths.unsqueeze(1)).to(torch.uint8).to(dev)
    assert asme.fused.fusable(D, Fd, H, x)
    y0, dx0, g0 = _run(asme, layer, x, valid, causal, False, 123)
    y1, dx1, g1 = _run(asme, layer, x, valid, causal, True, 123)
    assert _rel(y1, y0) < 1e-5
    assert _rel(dx1, dx0) < 1e-4
    assert g0.keys() == g1.keys()
    for n in g0:
        if n.endswith("linear_layers.1.bias"):  # dL/d(key bias) is analytically 0: pure rounding noise
            assert g1[n].abs().max() < 1e-3
            continue
        assert _rel(g1[n], g0[n]) < 1e-4, n


def test_fused_stack_long_rows(asme, dev):
    """L = 200 (the bench length) exercises the resident attention kernels and partial GEMM tiles."""
    torch.manual_seed(5)
    B, L, D, H, Fd = 2, 200, 128, 2, 512
    layer = asme.layers.TransformerLayer(D, H, 2, Fd, 0.1).to(dev).train()
    x = torch.randn(B, L, D, device=dev)
    valid = (torch.arange(L).unsqueeze(0) < torch.tensor([200, 137]).unsqueeze(1)).to(torch.uint8).to(dev)
    y0, dx0, g0 = _run(asme, layer, x, valid, True, False, 9)
    y1, dx1, g1 = _run(asme, layer, x, valid, True, True, 9)
    assert _rel(y1, y0) < 1e-5
    assert _rel(dx1, dx0) < 1e-4
    for n in g0:
        if not n.endswith("linear_layers.1.bias"):
            assert _rel(g1[n], g0[n]) < 1e-4, n
