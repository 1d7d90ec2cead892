"""Weight-stationary Linear GEMM (csrc/wsgemm.hip) against fp64 references, its fused GELU/dropout
epilogues against the standalone row kernels (bitwise), and the fused FFN autograd function against the
per-op composition (transformer_layers.py:212-220)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _call(asme, x, w, N, trans, bias=None, epi=0, pre_out=None, pre_in=None, p=0.0, seed=0):
    M, K = x.shape
    y = torch.full((M, N), float("nan"), device=x.device)
    L = asme._lib
    L.call("asme_ws_linear", L.ptr(x), M, K, L.ptr(w), N, trans, L.ptr(bias), epi, L.ptr(pre_out), L.ptr(pre_in),
           p, seed, L.ptr(y), L.stream())
    return y


@pytest.mark.parametrize("M", [1, 17, 1000, 4099, 65536 + 48])
@pytest.mark.parametrize("K,N", [(128, 128), (128, 256), (128, 384), (128, 512), (512, 128), (384, 128), (256, 64)])
def test_ws_linear_matches_fp64(asme, dev, M, K, N):
    torch.manual_seed(M + K + N)
    assert asme._lib.load().asme_ws_linear_supported(M, K, N) == 1
    x = torch.randn(M, K, device=dev)
    w = torch.randn(N, K, device=dev) / K ** 0.5
    b = torch.randn(N, device=dev)
    y = _call(asme, x, w, N, 0, bias=b)
    ref = x.double() @ w.double().t() + b.double()
    assert torch.isfinite(y).all()
    assert (y.double() - ref).abs().max().item() < 2e-5 * max(1.0, ref.abs().max().item())
    # trans: W is K x N (the input gradient of a Linear with weight W)
    wt = torch.randn(K, N, device=dev) / K ** 0.5
    y = _call(asme, x, wt, N, 1)
    ref = x.double() @ wt.double()
    assert torch.isfinite(y).all()
    assert (y.double() - ref).abs().max().item() < 2e-5 * max(1.0, ref.abs().max().item())


@pytest.mark.parametrize("K,N", [(128, 512), (512, 128), (384, 128)])
@pytest.mark.parametrize("dist", ["normal", "positive", "wide"])
def test_ws_linear_bf16x6_error_at_fp32_level(asme, dev, K, N, dist):
    """the fp32 products on split-bf16 MFMAs (csrc/common.h bf16x6) are as accurate as fp32 arithmetic: error vs
    float64, relative to sum |x * w|, no worse than 1.25x torch's own fp32 GEMM on the same inputs"""
    torch.manual_seed(K + N)
    M = 8192
    gen = {"normal": lambda *s: torch.randn(*s, device=dev),
           "positive": lambda *s: torch.rand(*s, device=dev),
           "wide": lambda *s: torch.randn(*s, device=dev) * torch.exp(3 * torch.randn(*s, device=dev))}[dist]
    x, w = gen(M, K), gen(N, K)
    ref = x.double() @ w.double().t()
    scale = x.double().abs() @ w.double().abs().t()
    ours = ((_call(asme, x, w, N, 0).double() - ref).abs() / scale).max().item()
    theirs = (((x @ w.t()).double() - ref).abs() / scale).max().item()
    assert ours <= 1.25 * theirs + 1e-9, (ours, theirs)
    assert ours < 2e-6


def test_ws_linear_rejects_unsupported(asme):
    lib = asme._lib.load()
    assert lib.asme_ws_linear_supported(100, 100, 128) == 0      # K not tiled
    assert lib.asme_ws_linear_supported(100, 128, 100) == 0      # N not a multiple of 64 / 96
    assert lib.asme_ws_linear_supported(100, 512, 384) == 0      # split W block over 160 KiB of LDS
    assert lib.asme_ws_linear_supported(1 << 22, 128, 512) == 0  # Y over 2 GiB
    # K = 128, N = 4096: 32 128-feature blocks fill an XCD's 32 workgroups -- every epilogue runs on 128-feature
    # blocks (the activation-factor one since round 6), so it is taken; 4224 (33 blocks) is not
    assert lib.asme_ws_linear_supported(100, 128, 4096) == 1
    assert lib.asme_ws_linear_supported(100, 128, 2048) == 1
    assert lib.asme_ws_linear_supported(100, 128, 4224) == 0


@pytest.mark.parametrize("Fd", [2048, 4096])
def test_ws_gelu_bwd_wide_feature_blocks(asme, dev, Fd):
    """the activation-factor epilogue at K = 128, N = 2048 / 4096 (CT = 8 shapes: 128-feature blocks, the factor read
    through the 4-slot ring; 4096 = one block per workgroup of an XCD): every output element written, equal to
    (dY W2) * factor"""
    torch.manual_seed(9)
    M, D = 3000, 128
    w2 = torch.randn(D, Fd, device=dev) / Fd ** 0.5
    dy = torch.randn(M, D, device=dev)
    fac = torch.rand(M, Fd, device=dev)
    d_pre = _call(asme, dy, w2, Fd, 1, epi=2, pre_in=fac, p=0.0, seed=1)
    ref = (dy.double() @ w2.double()) * fac.double()
    assert torch.isfinite(d_pre).all()
    assert (d_pre.double() - ref).abs().max().item() < 2e-5 * max(1.0, ref.abs().max().item())


@pytest.mark.parametrize("p", [0.0, 0.2])
@pytest.mark.parametrize("M", [333, 20000])
def test_ws_gelu_epilogues_match_row_kernels(asme, dev, p, M):
    torch.manual_seed(3)
    D, Fd = 128, 512
    L = asme._lib
    x = torch.randn(M, D, device=dev)
    w1 = torch.randn(Fd, D, device=dev) / D ** 0.5
    b1 = torch.randn(Fd, device=dev)
    seed = 987654321
    fac = torch.empty(M, Fd, device=dev)
    act = _call(asme, x, w1, Fd, 0, bias=b1, epi=1, pre_out=fac, p=p, seed=seed)
    pre = _call(asme, x, w1, Fd, 0, bias=b1)
    act_ref = torch.empty_like(pre)
    L.call("asme_gelu_dropout_fwd", L.ptr(pre), pre.numel(), p, seed, L.ptr(act_ref), L.stream())
    assert torch.equal(act, act_ref)
    # the stored activation factor keep * GELU'(pre) == the row kernel's backward of a unit gradient (bitwise)
    ones = torch.ones_like(pre)
    fac_ref = torch.empty_like(pre)
    L.call("asme_gelu_dropout_bwd", L.ptr(pre), L.ptr(ones), pre.numel(), p, seed, L.ptr(fac_ref), L.stream())
    assert torch.equal(fac, fac_ref)
    # backward through the activation: (dY W2) * factor; the row kernel rounds (g * keep) * GELU' instead
    w2 = torch.randn(D, Fd, device=dev) / Fd ** 0.5
    dy = torch.randn(M, D, device=dev)
    d_pre = _call(asme, dy, w2, Fd, 1, epi=2, pre_in=fac, p=p, seed=seed)
    dg = _call(asme, dy, w2, Fd, 1)
    d_ref = torch.empty_like(pre)
    L.call("asme_gelu_dropout_bwd", L.ptr(pre), L.ptr(dg), pre.numel(), p, seed, L.ptr(d_ref), L.stream())
    assert torch.allclose(d_pre, d_ref, rtol=1e-6, atol=1e-30)
    assert torch.equal(d_pre == 0, d_ref == 0)


@pytest.mark.parametrize("p", [0.0, 0.3])
def test_fused_ffn_matches_composition(asme, dev, p):
    torch.manual_seed(4)
    B, L_, D, Fd = 3, 50, 128, 512
    ff = torch.nn.ModuleDict({"w_1": torch.nn.Linear(D, Fd), "w_2": torch.nn.Linear(Fd, D)}).to(dev)
    x = torch.randn(B, L_, D, device=dev)
    outs = []
    for fused in (True, False):
        ff.zero_grad(set_to_none=True)
        xx = x.clone().requires_grad_(True)
        torch.manual_seed(11)  # same dropout seed draw
        if fused:
            y = asme.ops.ffn(xx, ff["w_1"].weight, ff["w_1"].bias, ff["w_2"].weight, ff["w_2"].bias, p)
        else:
            h = asme.ops.gelu_dropout(asme.ops.linear(xx, ff["w_1"].weight, ff["w_1"].bias), p)
            y = asme.ops.linear(h, ff["w_2"].weight, ff["w_2"].bias)
        gy = torch.randn_like(y, generator=torch.Generator(device=dev).manual_seed(5))
        (y * gy).sum().backward()
        outs.append((y.detach(), xx.grad.clone(), [q.grad.clone() for q in ff.parameters()]))
    (y1, dx1, g1), (y0, dx0, g0) = outs
    assert torch.allclose(y1, y0, rtol=1e-5, atol=1e-5)
    assert torch.allclose(dx1, dx0, rtol=1e-5, atol=1e-5)
    for a, b in zip(g1, g0):
        assert torch.allclose(a, b, rtol=1e-4, atol=1e-4)
    if p == 0.0:  # against plain PyTorch fp32
        ff.zero_grad(set_to_none=True)
        xx = x.clone().requires_grad_(True)
        y = ff["w_2"](F.gelu(ff["w_1"](xx)))
        assert torch.allclose(y1, y.detach(), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("p_a,p_b,with_ln", [(0.0, 0.0, True), (0.2, 0.0, True), (0.2, 0.3, True), (0.1, 0.0, False)])
def test_linear_residual_ln_fused_is_bit_identical(asme, dev, p_a, p_b, with_ln):
    """asme_ws_linear_residual_ln (output projection + residual + dropouts + next pre-LN in one epilogue) equals
    asme_ws_linear followed by asme_residual_ln_fwd bit for bit -- outputs, statistics and every gradient"""
    ops = asme.ops
    torch.manual_seed(11)
    M, d = 3 * 4096 + 77, 128  # ragged tail rows
    x = torch.randn(M, d, device=dev)
    w = torch.randn(d, d, device=dev) / d ** 0.5
    b = torch.randn(d, device=dev)
    res = torch.randn(M, d, device=dev)
    norm = torch.nn.LayerNorm(d).to(dev) if with_ln else None
    if norm is not None:
        with torch.no_grad():
            norm.weight.add_(torch.randn(d, device=dev) * 0.1)
            norm.bias.add_(torch.randn(d, device=dev) * 0.1)
    ds, dl = torch.randn(M, d, device=dev), torch.randn(M, d, device=dev)
    assert ops.linear_residual_ln_ok(x, w, res)
    outs = []
    for fused in (False, True):
        xs, ws, bs, rs = (t.clone().requires_grad_(True) for t in (x, w, b, res))
        if norm is not None:
            norm.weight.grad = norm.bias.grad = None
        torch.manual_seed(5)  # the dropout seeds
        if fused:
            s, ln = ops.linear_residual_ln(xs, ws, bs, rs, norm, p_a, p_b)
        else:
            s, ln = ops.residual_ln(rs, ops.linear(xs, ws, bs), norm, p_a, p_b)
        loss = (s * ds).sum() + ((ln * dl).sum() if ln is not None else 0.0)
        loss.backward()
        grads = [xs.grad, ws.grad, bs.grad, rs.grad]
        if norm is not None:
            grads += [norm.weight.grad.clone(), norm.bias.grad.clone()]
        outs.append((s.detach(), None if ln is None else ln.detach(), grads))
    (s0, l0, g0), (s1, l1, g1) = outs
    assert torch.equal(s0, s1)
    assert (l0 is None) == (l1 is None) and (l0 is None or torch.equal(l0, l1))
    for a, c in zip(g0, g1):
        assert torch.equal(a, c)


def test_linear_residual_ln_refuses_other_widths(asme, dev):
    ops = asme.ops
    x, w, res = (torch.randn(256, 64, device=dev), torch.randn(64, 64, device=dev), torch.randn(256, 64, device=dev))
    assert not ops.linear_residual_ln_ok(x, w, res)
    assert asme._lib.load().asme_ws_linear_residual_ln_supported(256, 256, 128) == 0
